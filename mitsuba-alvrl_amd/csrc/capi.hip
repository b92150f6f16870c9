// capi.hip -- implementation of the C ABI declared in include/alvrl.h.
//
// Owns the device state a vrlIntegrator instance holds between prepass and
// render (vrlIntegrator.cpp:1088-1121: m_vrls, m_ci) and launches the kernels
// of gather.hip / refine.hip.  Device state is immutable while gathers run, so
// concurrent gathers from several host threads (the reference calls Li from
// every LocalWorker, renderproc.cpp:52-86) only need their own streams.
#include "../../include/alvrl.h"
#include "vrl_device.hpp"
#include "host/scene.hpp"

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace alvrl {
namespace host {
MediumParams medium_of(const alvrl_medium_desc& d);   // host_capi.cpp
}  // namespace host
hipError_t launch_prepare_vrls(const float* soa, uint32_t n, VrlPrep* out, hipStream_t s);
hipError_t launch_gather_brute(const Rec* recs, const uint32_t* ids, uint32_t nrec,
                               const VrlPrep* vp, uint32_t nvrl, const DevParams& P,
                               float normalization, float* out, unsigned long long* counter,
                               hipStream_t s);
struct WorkItem { uint32_t slice, begin, count, pad; };
hipError_t launch_gather_clustered(const Rec* recs, const uint32_t* ids, const WorkItem* items,
                                   uint32_t nitems, const VrlPrep* vp, const uint32_t* slice_off,
                                   const uint32_t* reps, const float* weights,
                                   const uint32_t* fb_reps, const float* fb_w, uint32_t n_fb,
                                   const DevParams& P, float inv_pc, float* out,
                                   unsigned long long* counter, hipStream_t s);
struct SplitUnit { uint32_t item, first; };
hipError_t launch_gather_clustered_split(const Rec* recs, const uint32_t* ids, const WorkItem* items,
                                         uint32_t nitems, const SplitUnit* units, uint32_t nunits, uint32_t chunk,
                                         const uint64_t* base, float* cbuf, const VrlPrep* vp,
                                         const uint32_t* slice_off, const uint32_t* reps, const float* weights,
                                         const uint32_t* fb_reps, const float* fb_w, uint32_t n_fb,
                                         const DevParams& P, float inv_pc, float* out,
                                         unsigned long long* counter, hipStream_t s);
hipError_t launch_build_R(const Rec* recs, const uint32_t* ids, uint32_t nrows, const VrlPrep* vp,
                          uint32_t nvrl, const DevParams& P, float normalization, float2* Rt,
                          uint64_t ld, uint64_t row0, unsigned long long* counter, hipStream_t s);
hipError_t launch_build_R_blocks(const Rec* recs, const uint32_t* ids, uint32_t nrows, const VrlPrep* vp,
                                 uint32_t nvrl, const DevParams& P, float normalization, float2* Rt,
                                 const uint64_t* roff, const uint32_t* rstride, uint8_t* nonzero,
                                 unsigned long long* counter, hipStream_t s);
hipError_t launch_build_R_strict(const Rec* recs, const uint32_t* ids, uint32_t nrows, const void* svrl,
                                 uint32_t nvrl, const DevParams& P, float normalization, float2* Rt, uint64_t ld,
                                 uint64_t row0, const uint64_t* roff, const uint32_t* rstride, uint8_t* nonzero,
                                 unsigned long long* counter, hipStream_t s);
hipError_t launch_detmath(int fn, const float* in, float* out, uint32_t n, hipStream_t s);
hipError_t launch_detmath_exhaustive(int fn, uint64_t begin, uint64_t end, unsigned long long* out,
                                     uint32_t* first, hipStream_t s);
size_t strict_vrl_bytes();
hipError_t launch_div_check(uint64_t n, uint64_t seed, unsigned long long* out, uint32_t* first, hipStream_t s);
hipError_t launch_prepare_strict(const float* soa, uint32_t n, void* out, hipStream_t s);
hipError_t launch_false_color(const Rec* recs, const WorkItem* items, uint32_t n, int mode,
                              const uint32_t* slice_off, uint32_t n_fb, uint32_t nvrl, float* out,
                              unsigned long long* counter, hipStream_t s);
hipError_t launch_nonzero_columns(const float2* Rt, uint64_t ld, uint32_t nrows, uint32_t nvrl,
                                  uint8_t* mask, hipStream_t s);
hipError_t launch_accumulate_rgb(const float* rgb, const uint32_t* pix, uint32_t n, float* fb,
                                 hipStream_t s);
struct HostJob {
    const uint32_t* rows;
    const double* locw;
    uint32_t nrows;
    float pixel_under, undersampling, depth_correction;
    int do_refine;
    uint32_t stage_refine, stage_sample;
    const uint64_t* row_off;
    const uint32_t* row_stride;
    uint32_t* members;
    uint32_t* moff;
    uint32_t* nclusters;
};
int refine_jobs(hipStream_t s, const float* d_Rt, uint64_t ld, uint32_t nvrl, uint32_t seed,
                uint32_t pass, uint32_t njobs, const HostJob* jobs, const uint32_t* init_vrls,
                const uint32_t* init_off, uint32_t ninit, uint32_t* out_off, uint32_t* out_reps,
                float* out_w, int* out_refined, float* ms, unsigned long long* entries, std::string* err,
                RefineArenas* cache);
}  // namespace alvrl

using namespace alvrl;

static_assert(sizeof(alvrl_gather_rec) == sizeof(Rec), "record layout");
static_assert(sizeof(alvrl_work_item) == sizeof(WorkItem), "work item layout");

// Per calling thread of one context: the stream and grow-only device scratch
// of the host-pointer gathers, and the HIP events that time the thread's last
// launch.  Mitsuba calls renderBlock from every LocalWorker at once
// (renderproc.cpp:52-86), each block a separate call: one stream per thread
// keeps the calls concurrent, and nothing is allocated or freed per call.
struct ThreadSlot {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    char* scratch = nullptr;
    size_t cap = 0;
    hipError_t init(int dev)
    {
        device = dev;
        hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreate(&ev0);
        if (e == hipSuccess) e = hipEventCreate(&ev1);
        return e;
    }
    // scratch of at least n bytes; a grown buffer replaces the old one after
    // this thread's earlier calls (the only users of it) have finished
    hipError_t need(size_t n)
    {
        if (n <= cap) return hipSuccess;
        hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return e;
        if (scratch) (void)hipFree(scratch);
        scratch = nullptr;
        cap = 0;
        const size_t want = n + n / 2;
        e = hipMalloc(&scratch, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    ~ThreadSlot()
    {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        if (scratch) (void)hipFree(scratch);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// Host-pointer gathers (alvrl_gather_*_host) called concurrently are merged:
// the first caller leads one launch over every request queued by then and
// hands the lead to a waiting caller, so renderBlock-sized calls from many
// worker threads (renderproc.cpp:52-86) fill the device instead of queueing
// small launches behind the process's few hardware queues.
struct HostReq {
    const alvrl_gather_rec* recs;
    const uint32_t* ids;      // nullptr: the record's index in its own call
    const uint32_t* sl;       // clustered: slice per record
    uint32_t n;
    float* out;
    int rc = ALVRL_OK;
    std::string err;
    bool done = false;
};
// Work items below which a host batch takes the split gather (2,048 waves:
// half the chip's wave slots at two waves per SIMD); ALVRL_HOST_SPLIT=0 turns
// it off (developer A/B), =1 forces it for every batch.
constexpr uint32_t kSplitItems = 2048;
static bool split_enabled()
{
    const char* e = std::getenv("ALVRL_HOST_SPLIT");
    return !e || std::atoi(e) != 0;
}
static bool split_forced()
{
    const char* e = std::getenv("ALVRL_HOST_SPLIT");
    return e && std::atoi(e) == 1;
}
struct HostBatcher {
    unsigned long long split_batches = 0;   // batches that took the split gather
    std::mutex mu;
    std::condition_variable cv;
    std::vector<HostReq*> pending[2];   // [0] brute, [1] clustered
    bool leading[2] = {false, false};
    char* pin[2] = {nullptr, nullptr};  // the leader's pinned staging, per kind
    size_t pin_cap[2] = {0, 0};
    unsigned long long batches[2] = {0, 0}, requests[2] = {0, 0};
};

struct alvrl_ctx {
    alvrl_config cfg;
    DevParams P;
    bool medium_set = false;
    hipStream_t stream = nullptr;
    float* d_soa = nullptr;
    VrlPrep* d_vrl = nullptr;
    void* d_svrl = nullptr;   // the strict R build's per-VRL values (rbuild_strict.hip StrictVrl)
    uint32_t nvrl = 0, cap_vrl = 0;
    uint64_t particle_count = 0;
    unsigned long long* d_counter = nullptr;   // [0] preprocess, [1] render
    // clusters
    uint32_t nslices = 0, n_fb = 0;
    std::vector<uint32_t> h_slice_off;   // the lists' sizes on the host (the host gathers' split form)
    uint32_t* d_slice_off = nullptr;
    uint32_t* d_reps = nullptr;
    float* d_weights = nullptr;
    uint32_t* d_fb_reps = nullptr;
    float* d_fb_w = nullptr;
    uint32_t cap_slices = 0, cap_rep = 0, cap_fb = 0;   // grow-only: a prepass re-sets them every pass
    bool clusters_set = false;
    bool strict_rb = false;   // alvrl_set_strict_rbuild: the R build in the oracle's arithmetic
    float refine_ms = 0.0f;
    unsigned long long refine_entries[2] = {0, 0};   // refine_jobs: all entries, the splits' share
    // occluder BVH (alvrl_set_occluders); P.occ views it
    BvhNode* d_bvh_nodes = nullptr;
    float* d_bvh_tris = nullptr;
    uint32_t* d_bvh_ids = nullptr;
    RefineArenas refine_arenas;   // alvrl_refine's device scratch, reused across passes
    std::mutex mu;
    // launches that read the context's device state (VRLs, cluster lists,
    // occluders) hold it shared from their checks to their enqueue; calls
    // that overwrite that state hold it exclusively and then wait for the
    // device, so no launch is enqueued between that wait and the overwrite
    std::shared_mutex state_mu;
    std::mutex slots_mu;
    std::unordered_map<std::thread::id, std::unique_ptr<ThreadSlot>> slots;
    HostBatcher hb;
};

// the calling thread's slot (created on first use)
static ThreadSlot* slot_of(alvrl_ctx* c, hipError_t* e)
{
    std::lock_guard<std::mutex> g(c->slots_mu);
    auto& p = c->slots[std::this_thread::get_id()];
    *e = hipSuccess;
    if (!p) {
        std::unique_ptr<ThreadSlot> t(new ThreadSlot());
        *e = t->init(c->cfg.device);
        if (*e != hipSuccess) return nullptr;
        p = std::move(t);
    }
    return p.get();
}

#define STATE_SHARED(c)                                                                         \
    std::shared_lock<std::shared_mutex> state_;                                                 \
    if (c) state_ = std::shared_lock<std::shared_mutex>((c)->state_mu)
#define STATE_EXCLUSIVE(c)                                                                      \
    std::unique_lock<std::shared_mutex> state_;                                                 \
    if (c) state_ = std::unique_lock<std::shared_mutex>((c)->state_mu)
#define SLOT(c, t)                                                                              \
    ThreadSlot* t = nullptr;                                                                    \
    do {                                                                                        \
        hipError_t es_;                                                                         \
        t = slot_of(c, &es_);                                                                   \
        if (!t) return fail(ALVRL_ERR_HIP, std::string("per-thread stream: ") + hipGetErrorString(es_)); \
    } while (0)

static void free_occluders(alvrl_ctx* c)
{
    hipFree(c->d_bvh_nodes); hipFree(c->d_bvh_tris); hipFree(c->d_bvh_ids);
    c->d_bvh_nodes = nullptr; c->d_bvh_tris = nullptr; c->d_bvh_ids = nullptr;
    c->P.occ = bvh::View{nullptr, nullptr, nullptr, 0u};
}

static thread_local std::string g_err = "";

static int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                  \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail(ALVRL_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// NULL stream argument: the calling thread's (non-blocking) stream of this
// context, ordered after the work already queued on the null stream -- a
// caller's zero fill or copy of the buffers it passes, which the non-blocking
// stream would otherwise race
static hipStream_t pick(alvrl_ctx* c, void* s)
{
    if (s) return (hipStream_t)s;
    hipError_t e;
    ThreadSlot* t = slot_of(c, &e);
    hipStream_t st = t ? t->stream : c->stream;
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
        if (hipEventRecord(ev, nullptr) == hipSuccess) (void)hipStreamWaitEvent(st, ev, 0);
        (void)hipEventDestroy(ev);
    }
    return st;
}

extern "C" {

ALVRL_API int alvrl_abi_version(void) { return ALVRL_ABI_VERSION; }

#ifndef ALVRL_SRC_HASH
#define ALVRL_SRC_HASH "unknown"
#endif
ALVRL_API const char* alvrl_build_id(void) { return "src " ALVRL_SRC_HASH " gfx950 hipcc -O3"; }

ALVRL_API const char* alvrl_last_error(const alvrl_ctx*) { return g_err.c_str(); }

ALVRL_API int alvrl_ctx_create(const alvrl_config* cfg, alvrl_ctx** out)
{
    if (!cfg || !out) return fail(ALVRL_ERR_INVALID, "alvrl_ctx_create: null argument");
    // vrlIntegrator.cpp:148-156
    if (cfg->vol_vol_samples != 0 && cfg->vol_vol_samples < 2)
        return fail(ALVRL_ERR_INVALID, "Need at least 2 volVolSamples for variance estimate, but received: " +
                                           std::to_string(cfg->vol_vol_samples));
    if (cfg->vol_surf_samples != 0 && cfg->vol_surf_samples < 2)
        return fail(ALVRL_ERR_INVALID, "Need at least 2 volSurfSamples for variance estimate, but received: " +
                                           std::to_string(cfg->vol_surf_samples));
    if (cfg->vol_vol_samples > 64 || cfg->vol_surf_samples > 64)
        return fail(ALVRL_ERR_INVALID, "at most 64 volVol/volSurf samples are supported");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (cfg->device < 0 || cfg->device >= ndev)
        return fail(ALVRL_ERR_INVALID, "alvrl_ctx_create: no HIP device " + std::to_string(cfg->device));
    HIPCHK(hipSetDevice(cfg->device));
    alvrl_ctx* c = new alvrl_ctx();
    c->cfg = *cfg;
    std::memset(&c->P, 0, sizeof(c->P));
    c->P.nvv = cfg->vol_vol_samples;
    c->P.nvs = cfg->vol_surf_samples;
    c->P.short_vrls = cfg->short_vrls ? 1 : 0;
    c->P.seed = cfg->seed;
    c->P.pass = 0;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&c->d_counter, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(c->d_counter, 0, 2 * sizeof(unsigned long long));
    if (e != hipSuccess) {
        alvrl_ctx_destroy(c);
        return fail(ALVRL_ERR_HIP, std::string("alvrl_ctx_create: ") + hipGetErrorString(e));
    }
    *out = c;
    return ALVRL_OK;
}

static void free_clusters(alvrl_ctx* c)
{
    hipFree(c->d_slice_off); hipFree(c->d_reps); hipFree(c->d_weights);
    hipFree(c->d_fb_reps); hipFree(c->d_fb_w);
    c->d_slice_off = nullptr; c->d_reps = nullptr; c->d_weights = nullptr;
    c->d_fb_reps = nullptr; c->d_fb_w = nullptr;
    c->cap_slices = c->cap_rep = c->cap_fb = 0;
    c->clusters_set = false;
}

ALVRL_API void alvrl_ctx_destroy(alvrl_ctx* c)
{
    if (!c) return;
    hipSetDevice(c->cfg.device);
    if (c->stream) hipStreamSynchronize(c->stream);
    hipFree(c->d_soa); hipFree(c->d_vrl); hipFree(c->d_svrl); hipFree(c->d_counter);
    free_clusters(c);
    free_occluders(c);
    c->refine_arenas.release();
    for (int k = 0; k < 2; k++)
        if (c->hb.pin[k]) (void)hipHostFree(c->hb.pin[k]);
    c->slots.clear();
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

ALVRL_API int alvrl_set_medium(alvrl_ctx* c, const alvrl_medium_desc* m)
{
    if (!c || !m) return fail(ALVRL_ERR_INVALID, "alvrl_set_medium: null argument");
    if (m->phase_type != 0 && m->phase_type != 1)
        return fail(ALVRL_ERR_INVALID, "alvrl_set_medium: phase_type must be 0 (isotropic) or 1 (hg)");
    // HomogeneousMedium(props): sigma_t, the auto sampling weight
    // (homogeneous.cpp:168-184) and the strategy's terms, as the host tracer has them
    alvrl::host::MediumParams mp = alvrl::host::medium_of(*m);
    if (const char* e = mp.problem()) return fail(ALVRL_ERR_INVALID, std::string("alvrl_set_medium: ") + e);
    mp.resolve();
    for (int i = 0; i < 3; i++) { c->P.sigma_s[i] = mp.sigma_s[i]; c->P.sigma_t[i] = mp.sigma_t[i]; }
    c->P.w = mp.sampling_weight;
    c->P.strategy = mp.strategy;
    c->P.density = mp.density;
    for (int i = 0; i < 3; i++) {
        c->P.mx_sigma[i] = mp.mx_sigma[i]; c->P.mx_start[i] = mp.mx_start[i]; c->P.mx_lower[i] = mp.mx_lower[i];
    }
    for (int i = 0; i < 4; i++) c->P.mx_cdf[i] = mp.mx_cdf[i];
    c->P.mx_inv_norm = mp.mx_inv_norm;
    c->P.phase_type = m->phase_type;
    c->P.g = m->phase_g;
    c->medium_set = true;
    return ALVRL_OK;
}

ALVRL_API int alvrl_set_occluders(alvrl_ctx* c, const float* tris, uint32_t ntri, const uint32_t* material)
{
    STATE_EXCLUSIVE(c);
    if (!c || (!tris && ntri)) return fail(ALVRL_ERR_INVALID, "alvrl_set_occluders: null argument");
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipDeviceSynchronize());   // no gather on any stream still reads the old BVH
    free_occluders(c);
    if (ntri == 0) return ALVRL_OK;
    for (size_t i = 0; i < 9 * (size_t)ntri; i++)
        if (!std::isfinite(tris[i])) return fail(ALVRL_ERR_INVALID, "alvrl_set_occluders: non-finite vertex");
    BvhHost b;
    try {
        b = build_bvh(tris, ntri, material);
    } catch (const std::exception& ex) {
        return fail(ALVRL_ERR_INVALID, std::string("alvrl_set_occluders: ") + ex.what());
    }
    HIPCHK(hipMalloc(&c->d_bvh_nodes, b.nodes.size() * sizeof(BvhNode)));
    HIPCHK(hipMalloc(&c->d_bvh_tris, b.tris.size() * 4));
    HIPCHK(hipMalloc(&c->d_bvh_ids, b.ids.size() * 4));
    HIPCHK(hipMemcpy(c->d_bvh_nodes, b.nodes.data(), b.nodes.size() * sizeof(BvhNode), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_bvh_tris, b.tris.data(), b.tris.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_bvh_ids, b.ids.data(), b.ids.size() * 4, hipMemcpyHostToDevice));
    c->P.occ = bvh::View{c->d_bvh_nodes, c->d_bvh_tris, c->d_bvh_ids, ntri};
    return ALVRL_OK;
}

ALVRL_API int alvrl_set_pass(alvrl_ctx* c, uint32_t pass)
{
    if (!c) return fail(ALVRL_ERR_INVALID, "alvrl_set_pass: null ctx");
    c->P.pass = pass;
    return ALVRL_OK;
}

ALVRL_API uint32_t alvrl_num_vrls(const alvrl_ctx* c) { return c ? c->nvrl : 0; }

ALVRL_API int alvrl_upload_vrls(alvrl_ctx* c, const float* soa, uint32_t n, uint64_t pc, int on_dev)
{
    STATE_EXCLUSIVE(c);
    if (!c || (!soa && n)) return fail(ALVRL_ERR_INVALID, "alvrl_upload_vrls: null argument");
    if (n > 0 && pc == 0) return fail(ALVRL_ERR_INVALID, "alvrl_upload_vrls: particle_count must be > 0");
    HIPCHK(hipSetDevice(c->cfg.device));
    // the records are overwritten in place: no launch on any stream (the
    // caller's included) may still read the previous pass's
    HIPCHK(hipDeviceSynchronize());
    if (n > c->cap_vrl) {
        hipFree(c->d_soa); hipFree(c->d_vrl); hipFree(c->d_svrl);
        c->d_soa = nullptr; c->d_vrl = nullptr; c->d_svrl = nullptr; c->cap_vrl = 0;
        HIPCHK(hipMalloc(&c->d_soa, sizeof(float) * 9 * (size_t)n));
        HIPCHK(hipMalloc(&c->d_vrl, sizeof(VrlPrep) * (size_t)n));
        HIPCHK(hipMalloc(&c->d_svrl, strict_vrl_bytes() * (size_t)n));
        c->cap_vrl = n;
    }
    if (n) {
        // SoA planes are compacted to stride n on the device.
        HIPCHK(hipMemcpyAsync(c->d_soa, soa, sizeof(float) * 9 * (size_t)n,
                              on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
        HIPCHK(launch_prepare_vrls(c->d_soa, n, c->d_vrl, c->stream));
        HIPCHK(launch_prepare_strict(c->d_soa, n, c->d_svrl, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    c->nvrl = n;
    c->particle_count = pc;
    return ALVRL_OK;
}

ALVRL_API int alvrl_set_clusters(alvrl_ctx* c, uint32_t nslices, const uint32_t* slice_off,
                                 const uint32_t* reps, const float* weights,
                                 const uint32_t* fb_reps, const float* fb_w, uint32_t n_fb)
{
    STATE_EXCLUSIVE(c);
    if (!c || (!slice_off && nslices)) return fail(ALVRL_ERR_INVALID, "alvrl_set_clusters: null argument");
    HIPCHK(hipSetDevice(c->cfg.device));
    // the lists' device buffers are reused: every gather or false-colour
    // launch still reading them -- on any stream, the caller's included --
    // finishes first (the contract in alvrl.h)
    HIPCHK(hipDeviceSynchronize());
    const uint32_t nrep = nslices ? slice_off[nslices] : 0;
    for (uint32_t i = 0; i < nrep; i++)
        if (reps[i] >= c->nvrl) return fail(ALVRL_ERR_INVALID, "alvrl_set_clusters: representative out of range");
    for (uint32_t i = 0; i < n_fb; i++)
        if (fb_reps[i] >= c->nvrl) return fail(ALVRL_ERR_INVALID, "alvrl_set_clusters: fall-back representative out of range");
    c->clusters_set = false;
    if (nslices + 1 > c->cap_slices) {
        hipFree(c->d_slice_off); c->d_slice_off = nullptr; c->cap_slices = 0;
        HIPCHK(hipMalloc(&c->d_slice_off, sizeof(uint32_t) * (nslices + 1)));
        c->cap_slices = nslices + 1;
    }
    if (std::max(nrep, 1u) > c->cap_rep) {
        hipFree(c->d_reps); hipFree(c->d_weights); c->d_reps = nullptr; c->d_weights = nullptr; c->cap_rep = 0;
        const uint32_t cap = std::max(nrep, 1u) + std::max(nrep, 1u) / 4;
        HIPCHK(hipMalloc(&c->d_reps, sizeof(uint32_t) * cap));
        HIPCHK(hipMalloc(&c->d_weights, sizeof(float) * cap));
        c->cap_rep = cap;
    }
    if (std::max(n_fb, 1u) > c->cap_fb) {
        hipFree(c->d_fb_reps); hipFree(c->d_fb_w); c->d_fb_reps = nullptr; c->d_fb_w = nullptr; c->cap_fb = 0;
        HIPCHK(hipMalloc(&c->d_fb_reps, sizeof(uint32_t) * std::max(n_fb, 1u)));
        HIPCHK(hipMalloc(&c->d_fb_w, sizeof(float) * std::max(n_fb, 1u)));
        c->cap_fb = std::max(n_fb, 1u);
    }
    if (nslices)
        HIPCHK(hipMemcpyAsync(c->d_slice_off, slice_off, sizeof(uint32_t) * (nslices + 1), hipMemcpyHostToDevice, c->stream));
    if (nrep) {
        HIPCHK(hipMemcpyAsync(c->d_reps, reps, sizeof(uint32_t) * nrep, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->d_weights, weights, sizeof(float) * nrep, hipMemcpyHostToDevice, c->stream));
    }
    if (n_fb) {
        HIPCHK(hipMemcpyAsync(c->d_fb_reps, fb_reps, sizeof(uint32_t) * n_fb, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->d_fb_w, fb_w, sizeof(float) * n_fb, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));   // the host buffers are the caller's
    c->nslices = nslices;
    c->n_fb = n_fb;
    c->h_slice_off.assign(slice_off, slice_off + (nslices ? nslices + 1 : 0));
    c->clusters_set = true;
    return ALVRL_OK;
}

static int check_ready(alvrl_ctx* c, const char* fn)
{
    if (!c) return fail(ALVRL_ERR_INVALID, std::string(fn) + ": null ctx");
    if (!c->medium_set) return fail(ALVRL_ERR_STATE, std::string(fn) + ": alvrl_set_medium not called");
    if (!c->d_vrl && c->nvrl) return fail(ALVRL_ERR_STATE, std::string(fn) + ": no VRLs uploaded");
    if (c->particle_count == 0) return fail(ALVRL_ERR_STATE, std::string(fn) + ": alvrl_upload_vrls not called");
    return ALVRL_OK;
}

ALVRL_API int alvrl_gather_brute(alvrl_ctx* c, const alvrl_gather_rec* d_recs, const uint32_t* d_ids,
                                 uint32_t nrec, float* d_out, void* stream)
{
    STATE_SHARED(c);
    int rc = check_ready(c, "alvrl_gather_brute");
    if (rc) return rc;
    if (nrec && (!d_recs || !d_out)) return fail(ALVRL_ERR_INVALID, "alvrl_gather_brute: null buffer");
    HIPCHK(hipSetDevice(c->cfg.device));
    hipStream_t s = pick(c, stream);
    // Float normalization = 1.0 / m_vrls->getParticleCount()  (:805)
    const float norm = (float)(1.0 / (double)c->particle_count);
    SLOT(c, ts);
    HIPCHK(hipEventRecord(ts->ev0, s));
    HIPCHK(launch_gather_brute(reinterpret_cast<const Rec*>(d_recs), d_ids, nrec, c->d_vrl, c->nvrl,
                               c->P, norm, d_out, c->d_counter + 1, s));
    HIPCHK(hipEventRecord(ts->ev1, s));
    ts->timed = true;
    return ALVRL_OK;
}

ALVRL_API int alvrl_gather_clustered(alvrl_ctx* c, const alvrl_gather_rec* d_recs, const uint32_t* d_ids,
                                     const alvrl_work_item* d_items, uint32_t nitems, float* d_out,
                                     void* stream)
{
    STATE_SHARED(c);
    int rc = check_ready(c, "alvrl_gather_clustered");
    if (rc) return rc;
    if (!c->clusters_set) return fail(ALVRL_ERR_STATE, "alvrl_gather_clustered: alvrl_set_clusters not called");
    if (nitems && (!d_recs || !d_out || !d_items)) return fail(ALVRL_ERR_INVALID, "alvrl_gather_clustered: null buffer");
    HIPCHK(hipSetDevice(c->cfg.device));
    hipStream_t s = pick(c, stream);
    const float inv_pc = 1.0f / (float)c->particle_count;   // Li /= getParticleCount() (:590)
    SLOT(c, ts);
    HIPCHK(hipEventRecord(ts->ev0, s));
    HIPCHK(launch_gather_clustered(reinterpret_cast<const Rec*>(d_recs), d_ids,
                                   reinterpret_cast<const WorkItem*>(d_items), nitems, c->d_vrl,
                                   c->d_slice_off, c->d_reps, c->d_weights, c->d_fb_reps, c->d_fb_w,
                                   c->n_fb, c->P, inv_pc, d_out, c->d_counter + 1, s));
    HIPCHK(hipEventRecord(ts->ev1, s));
    ts->timed = true;
    return ALVRL_OK;
}

ALVRL_API int alvrl_gather_false_color(alvrl_ctx* c, int mode, const alvrl_gather_rec* d_recs,
                                       const alvrl_work_item* d_items, uint32_t n, float* d_out_rgb,
                                       void* stream)
{
    STATE_SHARED(c);
    int rc = check_ready(c, "alvrl_gather_false_color");
    if (rc) return rc;
    if (mode != ALVRL_FALSE_COLOR_NUM_VRLS && mode != ALVRL_FALSE_COLOR_SLICES)
        return fail(ALVRL_ERR_INVALID, "alvrl_gather_false_color: bad mode");
    if (mode == ALVRL_FALSE_COLOR_SLICES && !d_items)
        return fail(ALVRL_ERR_INVALID, "requested slices false color image without clustering!");
    if (d_items && !c->clusters_set) return fail(ALVRL_ERR_STATE, "alvrl_gather_false_color: no clusters set");
    if (n && (!d_recs || !d_out_rgb)) return fail(ALVRL_ERR_INVALID, "alvrl_gather_false_color: null buffer");
    HIPCHK(hipSetDevice(c->cfg.device));
    hipStream_t s = pick(c, stream);
    HIPCHK(launch_false_color(reinterpret_cast<const Rec*>(d_recs), reinterpret_cast<const WorkItem*>(d_items), n,
                              mode, c->d_slice_off, c->n_fb, c->nvrl, d_out_rgb, c->d_counter + 1, s));
    return ALVRL_OK;
}

ALVRL_API uint32_t alvrl_make_work_items(const uint32_t* sl, uint32_t nrec, alvrl_work_item* items,
                                         uint32_t cap)
{
    uint32_t n = 0, i = 0;
    while (i < nrec) {
        uint32_t j = i + 1;
        while (j < nrec && j - i < 64 && sl[j] == sl[i]) j++;
        if (n < cap) items[n] = alvrl_work_item{sl[i], i, j - i, 0u};
        n++;
        i = j;
    }
    return std::min(n, cap);
}

ALVRL_API int alvrl_build_R(alvrl_ctx* c, const alvrl_gather_rec* d_recs, const uint32_t* d_ids,
                            uint32_t nrows, float* d_Rt, uint64_t ld, uint64_t row0, void* stream)
{
    STATE_SHARED(c);
    int rc = check_ready(c, "alvrl_build_R");
    if (rc) return rc;
    if (nrows && (!d_recs || !d_Rt)) return fail(ALVRL_ERR_INVALID, "alvrl_build_R: null buffer");
    if (row0 + nrows > ld) return fail(ALVRL_ERR_INVALID, "alvrl_build_R: rows exceed ld");
    HIPCHK(hipSetDevice(c->cfg.device));
    hipStream_t s = pick(c, stream);
    const float norm = (float)(1.0 / (double)c->particle_count);
    SLOT(c, ts);
    HIPCHK(hipEventRecord(ts->ev0, s));
    if (c->strict_rb)
        HIPCHK(launch_build_R_strict(reinterpret_cast<const Rec*>(d_recs), d_ids, nrows, c->d_svrl, c->nvrl, c->P,
                                     norm, reinterpret_cast<float2*>(d_Rt), ld, row0, nullptr, nullptr, nullptr,
                                     c->d_counter + 0, s));
    else
        HIPCHK(launch_build_R(reinterpret_cast<const Rec*>(d_recs), d_ids, nrows, c->d_vrl, c->nvrl, c->P,
                              norm, reinterpret_cast<float2*>(d_Rt), ld, row0, c->d_counter + 0, s));
    HIPCHK(hipEventRecord(ts->ev1, s));
    ts->timed = true;
    return ALVRL_OK;
}

ALVRL_API int alvrl_set_rsamples(alvrl_ctx* c, int rsamples)
{
    if (!c) return fail(ALVRL_ERR_INVALID, "alvrl_set_rsamples: null ctx");
    if (rsamples < 1 || rsamples > 0xFFFF) return fail(ALVRL_ERR_INVALID, "Rsamples must be in [1, 2^16)");
    std::lock_guard<std::mutex> g(c->mu);
    c->P.rsamples = rsamples;
    return ALVRL_OK;
}

ALVRL_API int alvrl_set_strict_rbuild(alvrl_ctx* c, int on)
{
    if (!c) return fail(ALVRL_ERR_INVALID, "alvrl_set_strict_rbuild: null ctx");
    std::lock_guard<std::mutex> g(c->mu);
    c->strict_rb = on != 0;
    return ALVRL_OK;
}

ALVRL_API int alvrl_detmath_eval(int fn, const float* d_in, float* d_out, uint32_t n, void* stream)
{
    if (fn < 0 || fn > 13 || (fn > 5 && fn < 8) || fn == 9)
        return fail(ALVRL_ERR_INVALID, "alvrl_detmath_eval: fn must be in [0, 5] or 8, 10-13");
    if (n && (!d_in || !d_out)) return fail(ALVRL_ERR_INVALID, "alvrl_detmath_eval: null buffer");
    HIPCHK(launch_detmath(fn, d_in, d_out, n, (hipStream_t)stream));
    return ALVRL_OK;
}

ALVRL_API int alvrl_detmath_div_check(uint64_t n, uint64_t seed, uint64_t* mismatches, uint32_t* first,
                                      uint32_t nfirst)
{
    if (!mismatches) return fail(ALVRL_ERR_INVALID, "alvrl_detmath_div_check: null output");
    unsigned long long* d_out = nullptr;
    uint32_t* d_first = nullptr;
    HIPCHK(hipMalloc(&d_out, 2 * sizeof(unsigned long long)));
    hipError_t e = hipMalloc(&d_first, 16 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(d_out, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(d_first, 0xFF, 16 * sizeof(uint32_t));
    if (e == hipSuccess) e = launch_div_check(n, seed, d_out, d_first, nullptr);
    unsigned long long h[2] = {0, 0};
    uint32_t hf[16];
    if (e == hipSuccess) e = hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(hf, d_first, sizeof(hf), hipMemcpyDeviceToHost);
    hipFree(d_out);
    hipFree(d_first);
    HIPCHK(e);
    *mismatches = h[0];
    if (first)
        for (uint32_t i = 0; i < nfirst && i < 16; i++) first[i] = hf[i];
    return ALVRL_OK;
}

ALVRL_API int alvrl_detmath_exhaustive(int fn, uint64_t begin, uint64_t end, uint64_t* mismatches,
                                       uint32_t* first, uint32_t nfirst)
{
    if (fn != 0 && (fn < 2 || fn > 7))
        return fail(ALVRL_ERR_INVALID, "alvrl_detmath_exhaustive: fn must be 0 or in [2, 7]");
    if (end > (1ull << 32) || begin > end) return fail(ALVRL_ERR_INVALID, "alvrl_detmath_exhaustive: bad range");
    if (!mismatches) return fail(ALVRL_ERR_INVALID, "alvrl_detmath_exhaustive: null output");
    unsigned long long* d_out = nullptr;
    uint32_t* d_first = nullptr;
    HIPCHK(hipMalloc(&d_out, 2 * sizeof(unsigned long long)));
    hipError_t e = hipMalloc(&d_first, 16 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(d_out, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(d_first, 0xFF, 16 * sizeof(uint32_t));
    if (e == hipSuccess) e = launch_detmath_exhaustive(fn, begin, end, d_out, d_first, nullptr);
    unsigned long long h[2] = {0, 0};
    uint32_t hf[16];
    if (e == hipSuccess) e = hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(hf, d_first, sizeof(hf), hipMemcpyDeviceToHost);
    hipFree(d_out);
    hipFree(d_first);
    HIPCHK(e);
    *mismatches = h[0];
    if (first)
        for (uint32_t i = 0; i < nfirst && i < 16; i++) first[i] = hf[i];
    return ALVRL_OK;
}

ALVRL_API int alvrl_build_R_blocks(alvrl_ctx* c, const alvrl_gather_rec* d_recs, const uint32_t* d_ids,
                                   uint32_t nrows, float* d_Rt, const uint64_t* d_row_off,
                                   const uint32_t* d_row_stride, uint8_t* d_nonzero, void* stream)
{
    STATE_SHARED(c);
    int rc = check_ready(c, "alvrl_build_R_blocks");
    if (rc) return rc;
    if (nrows && (!d_recs || !d_Rt || !d_row_off || !d_row_stride))
        return fail(ALVRL_ERR_INVALID, "alvrl_build_R_blocks: null buffer");
    HIPCHK(hipSetDevice(c->cfg.device));
    hipStream_t s = pick(c, stream);
    const float norm = (float)(1.0 / (double)c->particle_count);
    SLOT(c, ts);
    HIPCHK(hipEventRecord(ts->ev0, s));
    if (c->strict_rb)
        HIPCHK(launch_build_R_strict(reinterpret_cast<const Rec*>(d_recs), d_ids, nrows, c->d_svrl, c->nvrl, c->P,
                                     norm, reinterpret_cast<float2*>(d_Rt), 0, 0, d_row_off, d_row_stride,
                                     d_nonzero, c->d_counter + 0, s));
    else
        HIPCHK(launch_build_R_blocks(reinterpret_cast<const Rec*>(d_recs), d_ids, nrows, c->d_vrl, c->nvrl, c->P,
                                     norm, reinterpret_cast<float2*>(d_Rt), d_row_off, d_row_stride, d_nonzero,
                                     c->d_counter + 0, s));
    HIPCHK(hipEventRecord(ts->ev1, s));
    ts->timed = true;
    return ALVRL_OK;
}

ALVRL_API int alvrl_refine(alvrl_ctx* c, const float* d_Rt, uint64_t ld, uint32_t njobs,
                           const alvrl_cluster_job* jobs, const uint32_t* init_vrls,
                           const uint32_t* init_off, uint32_t ninit, uint32_t* out_off,
                           uint32_t* out_reps, float* out_weights, int* out_refined, void* stream)
{
    if (!c) return fail(ALVRL_ERR_INVALID, "alvrl_refine: null ctx");
    if (njobs && (!d_Rt || !jobs || !init_off || !out_off || !out_reps || !out_weights || !out_refined))
        return fail(ALVRL_ERR_INVALID, "alvrl_refine: null argument");
    if (c->nvrl == 0) return fail(ALVRL_ERR_STATE, "alvrl_refine: no VRLs uploaded");
    if (c->nvrl < 2) return fail(ALVRL_ERR_NUMERIC, "Need at least 2 VRLs to estimate variance");
    std::vector<HostJob> hj(njobs);
    for (uint32_t j = 0; j < njobs; j++) {
        const alvrl_cluster_job& J = jobs[j];
        if ((!J.rows && !J.row_off) || !J.locw || (J.row_off && !J.row_stride))
            return fail(ALVRL_ERR_INVALID, "alvrl_refine: job without rows");
        // Clustering ctor checks (Preprocessor.cpp:307-313)
        double n1 = 0.0;
        for (uint32_t r = 0; r < J.nrows; r++) n1 += std::fabs(J.locw[r]);
        if (std::fabs((float)n1 - 1) > 1e-3)
            return fail(ALVRL_ERR_NUMERIC, "Incorrect normalization in localityWeights: " + std::to_string(n1));
        if (J.pixel_undersampling <= 0 || J.pixel_undersampling > 1)
            return fail(ALVRL_ERR_NUMERIC, "Invalid pixel undersampling: " + std::to_string(J.pixel_undersampling));
        hj[j] = HostJob{J.rows, J.locw, J.nrows, J.pixel_undersampling, J.undersampling,
                        J.depth_correction, J.do_refine, J.stage_refine, J.stage_sample,
                        J.row_off, J.row_stride, nullptr, nullptr, nullptr};
    }
    HIPCHK(hipSetDevice(c->cfg.device));
    std::string err;
    float ms = 0.0f;
    std::lock_guard<std::mutex> g(c->mu);   // the context's refine scratch
    int rc = refine_jobs(pick(c, stream), d_Rt, ld, c->nvrl, c->P.seed, c->P.pass, njobs, hj.data(),
                         init_vrls, init_off, ninit, out_off, out_reps, out_weights, out_refined,
                         &ms, c->refine_entries, &err, &c->refine_arenas);
    c->refine_ms = ms;
    if (rc) return fail(rc, err);
    return ALVRL_OK;
}

ALVRL_API int alvrl_refine_members(alvrl_ctx* c, const float* d_Rt, uint64_t ld, const alvrl_cluster_job* job,
                                   const uint32_t* init_vrls, const uint32_t* init_off, uint32_t ninit,
                                   uint32_t* out_vrls, uint32_t* out_off, uint32_t* n_clusters,
                                   int* out_refined, void* stream)
{
    if (!c) return fail(ALVRL_ERR_INVALID, "alvrl_refine_members: null ctx");
    if (!d_Rt || !job || !init_off || !out_vrls || !out_off || !n_clusters || !out_refined)
        return fail(ALVRL_ERR_INVALID, "alvrl_refine_members: null argument");
    if (c->nvrl == 0) return fail(ALVRL_ERR_STATE, "alvrl_refine_members: no VRLs uploaded");
    if (c->nvrl < 2) return fail(ALVRL_ERR_NUMERIC, "Need at least 2 VRLs to estimate variance");
    const alvrl_cluster_job& J = *job;
    if ((!J.rows && !J.row_off) || !J.locw || (J.row_off && !J.row_stride))
        return fail(ALVRL_ERR_INVALID, "alvrl_refine_members: job without rows");
    double n1 = 0.0;
    for (uint32_t r = 0; r < J.nrows; r++) n1 += std::fabs(J.locw[r]);
    if (std::fabs((float)n1 - 1) > 1e-3)
        return fail(ALVRL_ERR_NUMERIC, "Incorrect normalization in localityWeights: " + std::to_string(n1));
    if (J.pixel_undersampling <= 0 || J.pixel_undersampling > 1)
        return fail(ALVRL_ERR_NUMERIC, "Invalid pixel undersampling: " + std::to_string(J.pixel_undersampling));
    HostJob hj{J.rows, J.locw, J.nrows, J.pixel_undersampling, J.undersampling, 1.0f, 1,
               J.stage_refine, J.stage_sample, J.row_off, J.row_stride, out_vrls, out_off, n_clusters};
    const uint32_t nv = init_off[ninit];
    std::vector<uint32_t> off(2), reps(c->nvrl + 1);
    std::vector<float> w(c->nvrl + 1);
    HIPCHK(hipSetDevice(c->cfg.device));
    std::string err;
    float ms = 0.0f;
    *n_clusters = 0;
    std::lock_guard<std::mutex> g(c->mu);   // the context's refine scratch
    int rc = refine_jobs(pick(c, stream), d_Rt, ld, c->nvrl, c->P.seed, c->P.pass, 1, &hj, init_vrls,
                         init_off, ninit, off.data(), reps.data(), w.data(), out_refined, &ms,
                         c->refine_entries, &err, &c->refine_arenas);
    c->refine_ms = ms;
    if (rc) return fail(rc, err);
    (void)nv;
    return ALVRL_OK;
}

ALVRL_API int alvrl_last_refine_ms(alvrl_ctx* c, float* ms)
{
    if (!c || !ms) return fail(ALVRL_ERR_INVALID, "alvrl_last_refine_ms: null argument");
    *ms = c->refine_ms;
    return ALVRL_OK;
}

ALVRL_API int alvrl_last_refine_entries(alvrl_ctx* c, uint64_t* entries)
{
    if (!c || !entries) return fail(ALVRL_ERR_INVALID, "alvrl_last_refine_entries: null argument");
    *entries = c->refine_entries[0];
    return ALVRL_OK;
}

ALVRL_API int alvrl_last_refine_split_entries(alvrl_ctx* c, uint64_t* entries)
{
    if (!c || !entries) return fail(ALVRL_ERR_INVALID, "alvrl_last_refine_split_entries: null argument");
    *entries = c->refine_entries[1];
    return ALVRL_OK;
}

ALVRL_API int alvrl_nonzero_columns(alvrl_ctx* c, const float* d_Rt, uint64_t ld, uint32_t nrows,
                                    uint8_t* out_mask, void* stream)
{
    if (!c || !out_mask || (!d_Rt && c->nvrl)) return fail(ALVRL_ERR_INVALID, "alvrl_nonzero_columns: null argument");
    if (nrows > ld) return fail(ALVRL_ERR_INVALID, "alvrl_nonzero_columns: nrows > ld");
    if (c->nvrl == 0) return ALVRL_OK;
    HIPCHK(hipSetDevice(c->cfg.device));
    SLOT(c, ts);
    HIPCHK(ts->need(c->nvrl));   // the thread's scratch: free, its earlier calls synchronised
    hipStream_t s = stream ? (hipStream_t)stream : ts->stream;
    if (!stream) {   // after the caller's work on the null stream
        hipEvent_t ev = nullptr;
        HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        hipError_t ew = hipEventRecord(ev, nullptr);
        if (ew == hipSuccess) ew = hipStreamWaitEvent(s, ev, 0);
        (void)hipEventDestroy(ev);
        HIPCHK(ew);
    }
    uint8_t* d_mask = reinterpret_cast<uint8_t*>(ts->scratch);
    hipError_t e = launch_nonzero_columns(reinterpret_cast<const float2*>(d_Rt), ld, nrows, c->nvrl, d_mask, s);
    if (e == hipSuccess) e = hipMemcpyAsync(out_mask, d_mask, c->nvrl, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(ALVRL_ERR_HIP, std::string("alvrl_nonzero_columns: ") + hipGetErrorString(e));
    return ALVRL_OK;
}

ALVRL_API int alvrl_accumulate_rgb(alvrl_ctx* c, const float* d_rgb, const uint32_t* d_pixel, uint32_t n,
                                   float* d_fb, void* stream)
{
    if (!c || (n && (!d_rgb || !d_pixel || !d_fb))) return fail(ALVRL_ERR_INVALID, "alvrl_accumulate_rgb: null argument");
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(launch_accumulate_rgb(d_rgb, d_pixel, n, d_fb, pick(c, stream)));
    return ALVRL_OK;
}

ALVRL_API int alvrl_get_stats(alvrl_ctx* c, uint64_t* pre, uint64_t* ren)
{
    if (!c) return fail(ALVRL_ERR_INVALID, "alvrl_get_stats: null ctx");
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    unsigned long long h[2];
    HIPCHK(hipMemcpy(h, c->d_counter, sizeof(h), hipMemcpyDeviceToHost));
    if (pre) *pre = h[0];
    if (ren) *ren = h[1];
    return ALVRL_OK;
}

ALVRL_API int alvrl_reset_stats(alvrl_ctx* c)
{
    if (!c) return fail(ALVRL_ERR_INVALID, "alvrl_reset_stats: null ctx");
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemset(c->d_counter, 0, 2 * sizeof(unsigned long long)));
    return ALVRL_OK;
}

ALVRL_API int alvrl_last_kernel_ms(alvrl_ctx* c, float* ms)
{
    if (!c || !ms) return fail(ALVRL_ERR_INVALID, "alvrl_last_kernel_ms: null argument");
    HIPCHK(hipSetDevice(c->cfg.device));
    SLOT(c, ts);
    if (!ts->timed) return fail(ALVRL_ERR_STATE, "alvrl_last_kernel_ms: nothing launched yet on this thread");
    HIPCHK(hipEventSynchronize(ts->ev1));
    HIPCHK(hipEventElapsedTime(ms, ts->ev0, ts->ev1));
    return ALVRL_OK;
}

// carve the slot's scratch into 256-byte aligned pieces
static size_t carve(size_t* at, size_t bytes)
{
    const size_t o = *at;
    *at += (bytes + 255) & ~(size_t)255;
    return o;
}

// One launch over a batch of host-pointer requests (kind 0 brute, 1
// clustered): records staged in pinned memory, for the clustered gather
// bucketed by slice (stable) into wave work items, results scattered back.
// A record's result depends on its own record, stream id and list only, so a
// batch gives every request the bits it would get alone.
static int run_host_batch(alvrl_ctx* c, int kind, const std::vector<HostReq*>& batch, std::string* err)
{
    size_t n = 0;
    for (const HostReq* r : batch) n += r->n;
    if (n > 0xFFFFFFFFull) { *err = "host gather batch: more than 2^32 records"; return ALVRL_ERR_INVALID; }
    const uint32_t nrec = (uint32_t)n;
    HostBatcher& B = c->hb;
    size_t at = 0;
    const size_t h_r = carve(&at, sizeof(alvrl_gather_rec) * nrec);
    const size_t h_i = carve(&at, sizeof(uint32_t) * nrec);
    const size_t h_t = carve(&at, kind ? sizeof(alvrl_work_item) * nrec : 0);
    const size_t h_o = carve(&at, sizeof(float) * 3 * nrec);
    if (at > B.pin_cap[kind]) {
        if (B.pin[kind]) (void)hipHostFree(B.pin[kind]);
        B.pin[kind] = nullptr;
        B.pin_cap[kind] = 0;
        const size_t want = at + at / 2;
        if (hipHostMalloc(&B.pin[kind], want, hipHostMallocDefault) != hipSuccess) {
            *err = "host gather: pinned staging";
            return ALVRL_ERR_NOMEM;
        }
        B.pin_cap[kind] = want;
    }
    auto* r2 = reinterpret_cast<alvrl_gather_rec*>(B.pin[kind] + h_r);
    auto* id2 = reinterpret_cast<uint32_t*>(B.pin[kind] + h_i);
    auto* items = reinterpret_cast<alvrl_work_item*>(B.pin[kind] + h_t);
    auto* o2 = reinterpret_cast<float*>(B.pin[kind] + h_o);
    // (request, index) of every staged record
    std::vector<std::pair<uint32_t, uint32_t>> src(nrec);
    {
        uint32_t g = 0;
        for (uint32_t q = 0; q < (uint32_t)batch.size(); q++)
            for (uint32_t i = 0; i < batch[q]->n; i++) src[g++] = {q, i};
    }
    if (kind) {
        std::stable_sort(src.begin(), src.end(), [&](const std::pair<uint32_t, uint32_t>& a,
                                                     const std::pair<uint32_t, uint32_t>& b) {
            return batch[a.first]->sl[a.second] < batch[b.first]->sl[b.second];
        });
    }
    std::vector<uint32_t> sl2(kind ? nrec : 0);
    for (uint32_t g = 0; g < nrec; g++) {
        const HostReq* q = batch[src[g].first];
        const uint32_t i = src[g].second;
        r2[g] = q->recs[i];
        id2[g] = q->ids ? q->ids[i] : i;
        if (kind) sl2[g] = q->sl[i];
    }
    const uint32_t nit = kind ? alvrl_make_work_items(sl2.data(), nrec, items, nrec) : 0;
    // a batch too small to fill the chip takes the split form: one wave per
    // chunk of a work item's representative list (gather.hip, same bits)
    std::vector<SplitUnit> units;
    std::vector<uint64_t> base;
    uint64_t cfloats = 0;
    uint32_t chunk = 0;
    if (kind && (nit < kSplitItems || split_forced()) && split_enabled()) {
        base.resize(nit);
        uint64_t pairs = 0;
        for (uint32_t j = 0; j < nit; j++) {
            const uint32_t sj = items[j].slice;
            const uint32_t k = sj == 0xFFFFFFFFu ? c->n_fb : c->h_slice_off[sj + 1] - c->h_slice_off[sj];
            base[j] = cfloats;
            cfloats += (uint64_t)k * 3 * 64;
            pairs += k;
        }
        // about 8 waves per SIMD slot of the chip, chunks of 16..256 pairs
        chunk = (uint32_t)std::min<uint64_t>(256, std::max<uint64_t>(16, pairs / 8192 + 1));
        for (uint32_t j = 0; j < nit; j++) {
            const uint32_t sj = items[j].slice;
            const uint32_t k = sj == 0xFFFFFFFFu ? c->n_fb : c->h_slice_off[sj + 1] - c->h_slice_off[sj];
            for (uint32_t f = 0; f < k; f += chunk) units.push_back({j, f});
        }
    }
    const bool split = !base.empty();
    hipError_t e = hipSetDevice(c->cfg.device);
    ThreadSlot* ts = e == hipSuccess ? slot_of(c, &e) : nullptr;
    if (!ts) { *err = std::string("per-thread stream: ") + hipGetErrorString(e); return ALVRL_ERR_HIP; }
    at = 0;
    const size_t o_r = carve(&at, sizeof(alvrl_gather_rec) * nrec);
    const size_t o_i = carve(&at, sizeof(uint32_t) * nrec);
    const size_t o_o = carve(&at, sizeof(float) * 3 * nrec);
    const size_t o_t = carve(&at, sizeof(alvrl_work_item) * nit);
    const size_t o_u = carve(&at, sizeof(SplitUnit) * units.size());
    const size_t o_b = carve(&at, sizeof(uint64_t) * base.size());
    const size_t o_c = carve(&at, sizeof(float) * cfloats);
    e = ts->need(at);
    hipStream_t s = ts->stream;
    auto* dr = reinterpret_cast<alvrl_gather_rec*>(ts->scratch + o_r);
    auto* di = reinterpret_cast<uint32_t*>(ts->scratch + o_i);
    auto* dout = reinterpret_cast<float*>(ts->scratch + o_o);
    auto* dit = reinterpret_cast<alvrl_work_item*>(ts->scratch + o_t);
    auto* du = reinterpret_cast<SplitUnit*>(ts->scratch + o_u);
    auto* db = reinterpret_cast<uint64_t*>(ts->scratch + o_b);
    auto* dcb = reinterpret_cast<float*>(ts->scratch + o_c);
    if (e == hipSuccess) e = hipMemcpyAsync(dr, r2, sizeof(alvrl_gather_rec) * nrec, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(di, id2, sizeof(uint32_t) * nrec, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && kind)
        e = hipMemcpyAsync(dit, items, sizeof(alvrl_work_item) * nit, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && split && !units.empty())
        e = hipMemcpyAsync(du, units.data(), sizeof(SplitUnit) * units.size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess && split)
        e = hipMemcpyAsync(db, base.data(), sizeof(uint64_t) * base.size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipEventRecord(ts->ev0, s);
    if (e == hipSuccess) {
        if (kind && split) {
            const float inv_pc = 1.0f / (float)c->particle_count;   // Li /= getParticleCount() (:590)
            e = launch_gather_clustered_split(reinterpret_cast<const Rec*>(dr), di,
                                              reinterpret_cast<const WorkItem*>(dit), nit, du,
                                              (uint32_t)units.size(), chunk, db, dcb, c->d_vrl, c->d_slice_off,
                                              c->d_reps, c->d_weights, c->d_fb_reps, c->d_fb_w, c->n_fb, c->P,
                                              inv_pc, dout, c->d_counter + 1, s);
            B.split_batches++;
        } else if (kind) {
            const float inv_pc = 1.0f / (float)c->particle_count;   // Li /= getParticleCount() (:590)
            e = launch_gather_clustered(reinterpret_cast<const Rec*>(dr), di, reinterpret_cast<const WorkItem*>(dit),
                                        nit, c->d_vrl, c->d_slice_off, c->d_reps, c->d_weights, c->d_fb_reps,
                                        c->d_fb_w, c->n_fb, c->P, inv_pc, dout, c->d_counter + 1, s);
        } else {
            const float norm = (float)(1.0 / (double)c->particle_count);   // :805
            e = launch_gather_brute(reinterpret_cast<const Rec*>(dr), di, nrec, c->d_vrl, c->nvrl, c->P, norm, dout,
                                    c->d_counter + 1, s);
        }
    }
    if (e == hipSuccess) e = hipEventRecord(ts->ev1, s);
    if (e == hipSuccess) ts->timed = true;
    if (e == hipSuccess) e = hipMemcpyAsync(o2, dout, sizeof(float) * 3 * nrec, hipMemcpyDeviceToHost, s);
    const hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
    if (e != hipSuccess) {
        *err = std::string(kind ? "alvrl_gather_clustered_host: " : "alvrl_gather_brute_host: ") + hipGetErrorString(e);
        return ALVRL_ERR_HIP;
    }
    for (uint32_t g = 0; g < nrec; g++) {
        float* o = batch[src[g].first]->out + 3 * (size_t)src[g].second;
        o[0] = o2[3 * (size_t)g]; o[1] = o2[3 * (size_t)g + 1]; o[2] = o2[3 * (size_t)g + 2];
    }
    B.batches[kind]++;
    B.requests[kind] += batch.size();
    return ALVRL_OK;
}

// Queue the request; the caller that finds no leader leads one batch (every
// request queued by then, its own included) and, with its own result in
// hand, hands the lead on to a waiting caller.
static int host_gather(alvrl_ctx* c, int kind, HostReq* req)
{
    HostBatcher& B = c->hb;
    std::unique_lock<std::mutex> lk(B.mu);
    B.pending[kind].push_back(req);
    while (!req->done) {
        if (B.leading[kind]) {
            B.cv.wait(lk, [&] { return req->done || !B.leading[kind]; });
            continue;
        }
        B.leading[kind] = true;
        std::vector<HostReq*> batch;
        batch.swap(B.pending[kind]);
        lk.unlock();
        std::string err;
        const int rc = run_host_batch(c, kind, batch, &err);
        lk.lock();
        for (HostReq* r : batch) { r->rc = rc; r->err = err; r->done = true; }
        B.leading[kind] = false;
        B.cv.notify_all();
    }
    if (req->rc != ALVRL_OK) return fail(req->rc, req->err);
    return ALVRL_OK;
}

ALVRL_API int alvrl_gather_brute_host(alvrl_ctx* c, const alvrl_gather_rec* recs, const uint32_t* ids,
                                      uint32_t nrec, float* out)
{
    STATE_SHARED(c);
    int rc = check_ready(c, "alvrl_gather_brute_host");
    if (rc) return rc;
    if (nrec == 0) return ALVRL_OK;
    if (!recs || !out) return fail(ALVRL_ERR_INVALID, "alvrl_gather_brute_host: null buffer");
    HostReq req{recs, ids, nullptr, nrec, out};
    return host_gather(c, 0, &req);
}

ALVRL_API int alvrl_gather_clustered_host(alvrl_ctx* c, const alvrl_gather_rec* recs,
                                          const uint32_t* ids, const uint32_t* slice_of_rec,
                                          uint32_t nrec, float* out)
{
    STATE_SHARED(c);
    int rc = check_ready(c, "alvrl_gather_clustered_host");
    if (rc) return rc;
    if (!c->clusters_set) return fail(ALVRL_ERR_STATE, "alvrl_gather_clustered_host: alvrl_set_clusters not called");
    if (nrec == 0) return ALVRL_OK;
    if (!recs || !out || !slice_of_rec) return fail(ALVRL_ERR_INVALID, "alvrl_gather_clustered_host: null buffer");
    for (uint32_t i = 0; i < nrec; i++)
        if (slice_of_rec[i] != 0xFFFFFFFFu && slice_of_rec[i] >= c->nslices)
            return fail(ALVRL_ERR_INVALID, "alvrl_gather_clustered_host: slice out of range");
    HostReq req{recs, ids, slice_of_rec, nrec, out};
    return host_gather(c, 1, &req);
}

/* diagnostic: host-pointer gather launches and the requests they carried */
ALVRL_API int alvrl_host_batch_stats(alvrl_ctx* c, uint64_t* batches, uint64_t* requests)
{
    if (!c || !batches || !requests) return fail(ALVRL_ERR_INVALID, "alvrl_host_batch_stats: null argument");
    std::lock_guard<std::mutex> g(c->hb.mu);
    batches[0] = c->hb.batches[0]; batches[1] = c->hb.batches[1];
    requests[0] = c->hb.requests[0]; requests[1] = c->hb.requests[1];
    return ALVRL_OK;
}

}  // extern "C"
