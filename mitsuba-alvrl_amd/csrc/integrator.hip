// integrator.hip -- the vrl integrator pipeline on top of include/alvrl.h.
//
// Mirrors class vrlIntegrator (src/integrators/vrl/vrlIntegrator.cpp): the
// same property names and defaults (:128-208), preprocess (:237-267: optional
// vrlFile, buildSlices), prepass (:270-356: VRLs, representative pixels, R,
// buildClusters) and rendering (Li -> getClusteredVrlContributions /
// getVRLContributions for every pixel of the owned tiles).  All per-pair work
// runs in the HIP kernels behind the C ABI; this file is orchestration.
#include "../../include/alvrl.h"
#include "../../include/alvrl_host.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "host/exchange.hpp"
#include "host/preprocessor.hpp"
#include "host/scene.hpp"

namespace alvrl {
namespace host {
extern thread_local std::string g_host_err;
SmokeBox to_box(const alvrl_scene_desc& s);
MediumParams medium_of(const alvrl_medium_desc& d);
const char* scene_problem(const alvrl_scene_desc& s);
}  // namespace host
}  // namespace alvrl

using namespace alvrl::host;

namespace {
// Clustering stream ids (oracle/alvrl_preproc.h).
constexpr uint32_t kStageFallbackRefine = 1u, kStageFallbackSample = 2u, kStageGlobalRefine = 0xFFFFFFFEu;
inline uint32_t stage_slice_refine(uint32_t s) { return 3u + 2u * s; }
inline uint32_t stage_slice_sample(uint32_t s) { return 4u + 2u * s; }

struct IntegError : std::runtime_error {
    int code;
    IntegError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void chk(int rc, const char* what)
{
    if (rc != ALVRL_OK) throw IntegError(rc, std::string(what) + ": " + alvrl_last_error(nullptr));
}
void chk_host(int rc)
{
    if (rc != ALVRL_OK) throw IntegError(rc, alvrl_host_last_error());
}
void hchk(hipError_t e, const char* what)
{
    if (e != hipSuccess) throw IntegError(ALVRL_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    void ensure(size_t cnt)
    {
        if (cnt <= n && p) return;
        if (p) hipFree(p);
        p = nullptr;
        n = 0;
        hchk(hipMalloc(&p, std::max<size_t>(cnt, 1) * sizeof(T)), "hipMalloc");
        n = cnt;
    }
    ~DevBuf() { if (p) hipFree(p); }
};
}  // namespace

__global__ void __launch_bounds__(256) k_scale_f32(float* __restrict__ v, uint32_t n, float f)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] *= f;
}

struct alvrl_integrator {
    // ---- properties (vrlIntegrator.cpp:128-208; integrator.cpp:272-277, 348-349)
    bool shortVrls = true;
    int vrlTargetNum = 500;
    int maxParticleDepth = -1;
    int specRRdepth = 100;
    float initialSpecularThroughput = 20;
    int volVolSamples = 2, volSurfSamples = 2;
    int sampleCount = 1;      // the sampler's sampleCount: sensor samples per pixel and pass (integrator.cpp:240-264)
    bool globalCluster = false;
    float globalUndersampling = -1;
    bool localRefinement = true;
    float localUndersampling = -1;
    float fallBackUndersampling = 5;
    int targetNumSlices = 100;
    float targetPixelUndersampling = 64;
    float sliceCurvatureFactor = 0.5f;
    int neighbourCount = 0;
    float neighbourWeight = 0;
    int Rsamples = 1;
    float depthCorrection = 1;
    bool numVrlFalseColor = false, slicesFalseColor = false, convergenceFalseColor = false;
    std::string vrlFile;
    int maxPasses = 1;
    bool dumpPasses = false;
    int rrDepth = 5, maxDepth = -1;
    uint32_t seed = 0xA1B2C3D4u, vrlSeed = 0x5EED0001u;
    // trace the pass's VRLs on the device (csrc/tracer.hip, bit-identical to
    // the host tracer) wherever the scene fits it -- no mirror / null /
    // dielectric triangles, whose particles the host traces; false: always the host
    bool gpuTracer = true;
    bool strictRbuild = true;
    // slices to ranks with world > 1: "cost" (longest processing time first on
    // each slice's local rows, the default) or "roundrobin" (s % world)
    bool sliceRoundRobin = false;    // the R build in the oracle's arithmetic (alvrl_set_strict_rbuild); false: the gathers' fast maths
    // ---- state
    int device = 0;
    alvrl_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    // the last render's gather, timed on the stream it ran on by the
    // integrator's own events (get_stats may run on any thread)
    hipEvent_t ev_r0 = nullptr, ev_r1 = nullptr;
    bool render_timed = false;
    SmokeBox scene;
    alvrl_scene_desc scene_desc{};
    bool have_scene = false;
    // host-cast scene: the VRL tracer's scene (alvrl_scene_ext::tracer), owned copy
    bool have_tracer = false;
    SmokeBox tracer_box;
    alvrl_scene_desc tracer_desc{};
    std::unique_ptr<Preprocessor> prep;
    std::vector<uint32_t> pixel_to_slice;   // y + H*x
    VrlSet vrls;
    bool vrls_from_file = false;
    std::vector<uint32_t> local_slices;     // the slices the last prepass refined here (alvrl_integrator_local_slices)
    uint32_t uploaded_pass = 0xFFFFFFFFu;
    bool clustered = false;
    // R
    DevBuf<float> Rt;                       // R in per-slice [vrl][row] blocks
    std::vector<uint64_t> row_base;         // float2 index of (vrl 0, global row g); UINT64_MAX if not built
    std::vector<uint32_t> row_stride;       // rows of g's slice
    DevBuf<alvrl_gather_rec> rep_recs;
    DevBuf<uint32_t> rep_ids;
    DevBuf<uint64_t> rb_off;                // per built row: float2 index of (vrl 0, row)
    DevBuf<uint32_t> rb_stride;
    DevBuf<uint8_t> nz_dev;
    uint32_t rows_built = 0;                // rows of R held (all of them at world 1)
    // the last prepass's clustering inputs (alvrl_integrator_slice_job):
    // initial clusters, and per local slice its rows and locality weights
    std::vector<uint32_t> job_init, job_init_off, job_slices;
    std::vector<std::vector<uint32_t>> job_rows;
    std::vector<std::vector<double>> job_locw;
    // cluster info (vrlClusterInfo)
    std::vector<uint32_t> slice_off, reps, fb_reps;
    std::vector<uint32_t> rep_buf;          // alvrl_refine's output buffers, reused across passes
    std::vector<float> w_buf;
    std::vector<float> weights, fb_w;
    // render cache per (rank, world)
    uint32_t cache_rank = 0xFFFFFFFFu, cache_world = 0, cache_mode = 0, cache_pass = 0xFFFFFFFFu;
    uint32_t cur_pass = 0;
    // the eye paths' delta-BSDF chains (scene.has_delta()): records of depth
    // d >= 1 follow the primary records, level by level
    bool chains = false;
    DevBuf<alvrl_gather_rec> ch_recs;
    DevBuf<uint32_t> ch_ids, ch_stride;
    DevBuf<uint64_t> ch_off;
    std::vector<uint32_t> level_rec;        // render: first record of each depth level (+ end)
    std::vector<uint32_t> level_item;       // render: first work item of each level (+ end)
    DevBuf<alvrl_gather_rec> rec_buf;
    DevBuf<uint32_t> pix_buf;
    DevBuf<alvrl_work_item> item_buf;
    DevBuf<float> out_buf;
    uint32_t nrec = 0, nitems = 0;
    alvrl_integrator_stats st{};
    // host-cast scene (alvrl_integrator_preprocess_ext): no descriptor; the
    // slicing records, the R rows' records and the VRLs come from the caller.
    // ext_recs / ext_row / ext_n: the records of the running
    // alvrl_integrator_prepass_records call
    bool ext = false, ext_active = false;
    const alvrl_gather_rec* ext_recs = nullptr;
    const uint32_t* ext_row = nullptr;
    uint32_t ext_n = 0;

    ~alvrl_integrator()
    {
        if (ctx) alvrl_ctx_destroy(ctx);
        if (ev_r0) hipEventDestroy(ev_r0);
        if (ev_r1) hipEventDestroy(ev_r1);
        if (stream) hipStreamDestroy(stream);
    }

    void set(const std::string& k, const std::string& v)
    {
        auto b = [&](const std::string& x) {
            if (x == "true" || x == "1" || x == "yes") return true;
            if (x == "false" || x == "0" || x == "no") return false;
            throw IntegError(ALVRL_ERR_INVALID, "bad boolean for " + k + ": " + x);
        };
        auto i = [&](const std::string& x) { return (int)std::stol(x, nullptr, 0); };
        auto f = [&](const std::string& x) { return std::stof(x); };
        if (k == "nc") throw IntegError(ALVRL_ERR_INVALID, "Neighbourcount is now called 'neighbourCount' instead of 'nc'!");
        else if (k == "shortVrls") shortVrls = b(v);
        else if (k == "gpuTracer") gpuTracer = b(v);
        else if (k == "strictRbuild") strictRbuild = b(v);
        else if (k == "sliceSharding") {
            if (v != "cost" && v != "roundrobin") throw IntegError(ALVRL_ERR_INVALID, "sliceSharding must be cost or roundrobin");
            sliceRoundRobin = v == "roundrobin";
        }
        else if (k == "vrlTargetNum") vrlTargetNum = i(v);
        else if (k == "maxParticleDepth") maxParticleDepth = i(v);
        else if (k == "specularForcedRRdepth") specRRdepth = i(v);
        else if (k == "initialSpecularThroughput") initialSpecularThroughput = f(v);
        else if (k == "volVolSamples") volVolSamples = i(v);
        else if (k == "volSurfSamples") volSurfSamples = i(v);
        else if (k == "sampleCount") {
            sampleCount = i(v);
            if (sampleCount < 1 || sampleCount > 65535) throw IntegError(ALVRL_ERR_INVALID, "sampleCount must be in [1, 65535]");
        }
        else if (k == "globalCluster") globalCluster = b(v);
        else if (k == "globalUndersampling") globalUndersampling = f(v);
        else if (k == "localRefinement") localRefinement = b(v);
        else if (k == "localUndersampling") localUndersampling = f(v);
        else if (k == "fallBackUndersampling") fallBackUndersampling = f(v);
        else if (k == "targetNumSlices") targetNumSlices = i(v);
        else if (k == "targetPixelUndersampling") targetPixelUndersampling = f(v);
        else if (k == "sliceCurvatureFactor") sliceCurvatureFactor = f(v);
        else if (k == "neighbourCount") neighbourCount = i(v);
        else if (k == "neighbourWeight") neighbourWeight = f(v);
        else if (k == "Rsamples") Rsamples = i(v);
        else if (k == "depthCorrection") depthCorrection = f(v);
        else if (k == "numVrlFalseColor") numVrlFalseColor = b(v);
        else if (k == "slicesFalseColor") slicesFalseColor = b(v);
        else if (k == "convergenceFalseColor") convergenceFalseColor = b(v);
        else if (k == "vrlFile") vrlFile = v;
        else if (k == "maxPasses") maxPasses = i(v);
        else if (k == "dumpPasses") dumpPasses = b(v);
        else if (k == "rrDepth") rrDepth = i(v);
        else if (k == "maxDepth") maxDepth = i(v);
        else if (k == "seed") seed = (uint32_t)std::stoul(v, nullptr, 0);
        else if (k == "vrlSeed") vrlSeed = (uint32_t)std::stoul(v, nullptr, 0);
        else throw IntegError(ALVRL_ERR_INVALID, "unknown vrl integrator property '" + k + "'");
    }

    void validate()
    {
        if (volVolSamples != 0 && volVolSamples < 2)
            throw IntegError(ALVRL_ERR_INVALID, "Need at least 2 volVolSamples for variance estimate, but received: " + std::to_string(volVolSamples));
        if (volSurfSamples != 0 && volSurfSamples < 2)
            throw IntegError(ALVRL_ERR_INVALID, "Need at least 2 volSurfSamples for variance estimate, but received: " + std::to_string(volSurfSamples));
        if (targetNumSlices < 1) throw IntegError(ALVRL_ERR_INVALID, "Invalid target number of slices!");
        if (Rsamples < 1) throw IntegError(ALVRL_ERR_INVALID, "Rsamples must be >= 1");
        clustered = globalCluster || localRefinement;
    }

    void preprocess(const alvrl_scene_desc& s)
    {
        ext = false;
        have_tracer = false;
        scene = to_box(s);
        scene_desc = s;
        scene_desc.occluders = scene.occ.empty() ? nullptr : scene.occ.data();   // the owned copy
        scene_desc.n_occluders = scene.n_occ();
        have_scene = true;
        alvrl_medium_desc md = s.medium;
        chk(alvrl_set_medium(ctx, &md), "alvrl_set_medium");
        scene_desc.occluder_material = scene.occ_mat.empty() ? nullptr : scene.occ_mat.data();
        scene_desc.occluder_albedos = scene.occ_alb.empty() ? nullptr : scene.occ_alb.data();
        scene_desc.emitter_tris = scene.emit.empty() ? nullptr : scene.emit.data();   // the owned copy
        scene_desc.n_emitter_tris = (uint32_t)(scene.emit.size() / 9);
        chains = scene.has_delta();
        if (chains && convergenceFalseColor)
            throw IntegError(ALVRL_ERR_INVALID, "convergenceFalseColor is not supported with delta-BSDF occluders");
        chk(alvrl_set_occluders(ctx, scene_desc.occluders, scene_desc.n_occluders, scene_desc.occluder_material),
            "alvrl_set_occluders");
        load_vrl_file();
        if (clustered) {          // :254-265
            PrepParams pp;
            pp.target_num_slices = (uint32_t)targetNumSlices;
            pp.neighbour_count = (uint32_t)neighbourCount;
            pp.neighbour_weight = neighbourWeight;
            pp.slice_curvature_factor = sliceCurvatureFactor;
            pp.seed = seed;
            pp.pass = 0;
            prep.reset(new Preprocessor(pp));
            const double t0 = now_ms();
            // the eye-ray first hit of every pixel on the device (Preprocessor.cpp:1140-1170)
            const uint32_t npix = (uint32_t)scene.width * (uint32_t)scene.height;
            std::vector<alvrl_gather_rec> h_all;
            if (npix && !chains) {
                DevBuf<alvrl_gather_rec> d_all;
                d_all.ensure(npix);
                h_all.resize(npix);
                chk_host(alvrl_scene_records_gpu(&scene_desc, 1, nullptr, npix, d_all.p, stream));
                hchk(hipMemcpy(h_all.data(), d_all.p, sizeof(alvrl_gather_rec) * npix, hipMemcpyDeviceToHost), "copy records");
            }
            // with null surfaces the slicing ray passes them (:1157-1169): host records
            pixel_to_slice = prep->build_slices(scene, h_all.empty() ? nullptr : reinterpret_cast<const float*>(h_all.data()));
            st.ms_slices = now_ms() - t0;
            st.slices = prep->num_slices();
        }
        cache_rank = 0xFFFFFFFFu;
    }

    void load_vrl_file()
    {
        if (!vrlFile.empty()) {   // :243-252
            std::string err;
            if (!read_vrl_file(vrlFile.c_str(), scene.medium, &vrls, &err)) throw IntegError(ALVRL_ERR_INVALID, err);
            vrls_from_file = true;
            uploaded_pass = 0xFFFFFFFFu;
        }
    }

    // preprocess (:237-267) of a host-cast scene: the medium, the scene's
    // triangles for the gathers' occluder test, buildSlices over the host's
    // gather points (Preprocessor.cpp:1130-1193)
    void preprocess_ext(const alvrl_scene_ext& e)
    {
        if (e.width <= 0 || e.height <= 0) throw IntegError(ALVRL_ERR_INVALID, "alvrl_scene_ext: width and height must be > 0");
        if (e.n_triangles && !e.triangles) throw IntegError(ALVRL_ERR_INVALID, "alvrl_scene_ext: n_triangles > 0 without triangles");
        MediumParams m = medium_of(e.medium);
        if (const char* p = m.problem()) throw IntegError(ALVRL_ERR_INVALID, p);
        m.resolve();
        SmokeBox b;
        b.width = e.width;
        b.height = e.height;
        for (int i = 0; i < 3; i++) { b.box_min[i] = e.scene_min[i]; b.box_max[i] = e.scene_max[i]; }
        b.medium = m;
        if (e.n_triangles) b.occ.assign(e.triangles, e.triangles + 9 * (size_t)e.n_triangles);
        if (e.n_triangles && e.triangle_material) {
            b.occ_mat.assign(e.triangle_material, e.triangle_material + e.n_triangles);
            for (uint32_t x : b.occ_mat)
                if (x > ALVRL_MAT_DIELECTRIC) throw IntegError(ALVRL_ERR_INVALID, "alvrl_scene_ext: unknown triangle material");
        }
        have_tracer = false;
        if (e.tracer) {   // the VRL tracer's view of the scene, traced every pass
            if (const char* p = scene_problem(*e.tracer)) throw IntegError(ALVRL_ERR_INVALID, std::string("alvrl_scene_ext::tracer: ") + p);
            tracer_box = to_box(*e.tracer);
            tracer_desc = *e.tracer;
            tracer_desc.occluders = tracer_box.occ.empty() ? nullptr : tracer_box.occ.data();
            tracer_desc.n_occluders = tracer_box.n_occ();
            tracer_desc.occluder_material = tracer_box.occ_mat.empty() ? nullptr : tracer_box.occ_mat.data();
            tracer_desc.occluder_albedos = tracer_box.occ_alb.empty() ? nullptr : tracer_box.occ_alb.data();
            tracer_desc.emitter_tris = tracer_box.emit.empty() ? nullptr : tracer_box.emit.data();
            tracer_desc.n_emitter_tris = (uint32_t)(tracer_box.emit.size() / 9);
            have_tracer = true;
        }
        scene = b;
        std::memset(&scene_desc, 0, sizeof(scene_desc));
        ext = true;
        have_scene = true;
        chains = false;
        alvrl_medium_desc md = e.medium;
        chk(alvrl_set_medium(ctx, &md), "alvrl_set_medium");
        chk(alvrl_set_occluders(ctx, scene.occ.empty() ? nullptr : scene.occ.data(), scene.n_occ(),
                                scene.occ_mat.empty() ? nullptr : scene.occ_mat.data()), "alvrl_set_occluders");
        load_vrl_file();
        prep.reset();
        pixel_to_slice.clear();
        st.slices = 0;
        // no gather points: a render worker whose slices and cluster lists
        // arrive through alvrl_integrator_set_cluster_info (the reference's
        // wakeup, vrlIntegrator.cpp:378-384) and that never runs a prepass
        if (clustered && e.slice_recs) {
            PrepParams pp;
            pp.target_num_slices = (uint32_t)targetNumSlices;
            pp.neighbour_count = (uint32_t)neighbourCount;
            pp.neighbour_weight = neighbourWeight;
            pp.slice_curvature_factor = sliceCurvatureFactor;
            pp.seed = seed;
            pp.pass = 0;
            prep.reset(new Preprocessor(pp));
            const double t0 = now_ms();
            pixel_to_slice = prep->build_slices(scene, reinterpret_cast<const float*>(e.slice_recs));
            st.ms_slices = now_ms() - t0;
            st.slices = prep->num_slices();
        }
        cache_rank = 0xFFFFFFFFu;
    }

    // sampleSliceMapping of the pass (:293-296): representative pixels,
    // row-major ids in R-row order
    std::vector<uint32_t> rep_pixels(uint32_t pass)
    {
        if (!have_scene) throw IntegError(ALVRL_ERR_STATE, "rep_pixels before preprocess");
        if (!clustered || !prep) throw IntegError(ALVRL_ERR_STATE, "no slices: the integrator does not cluster");
        prep->set_pass(pass);
        prep->sample_slice_mapping(targetPixelUndersampling);
        const auto& rp = prep->rep_pix();
        const uint32_t W = (uint32_t)scene.width, H = (uint32_t)scene.height;
        std::vector<uint32_t> out(rp.size());
        for (size_t i = 0; i < rp.size(); i++) out[i] = (rp[i] % H) * W + rp[i] / H;   // x*H + y -> y*W + x
        return out;
    }

    void prepass_records(uint32_t pass, const alvrl_gather_rec* recs, const uint32_t* rows, uint32_t n,
                         uint32_t rank, uint32_t world, const alvrl_exchange* ex)
    {
        if (!ext) throw IntegError(ALVRL_ERR_STATE, "alvrl_integrator_prepass_records needs a host-cast scene (alvrl_integrator_preprocess_ext)");
        if (n && (!recs || !rows)) throw IntegError(ALVRL_ERR_INVALID, "alvrl_integrator_prepass_records: null records");
        struct Done {
            alvrl_integrator* it;
            ~Done() { it->ext_active = false; it->ext_recs = nullptr; it->ext_row = nullptr; it->ext_n = 0; }
        } done{this};
        ext_recs = recs; ext_row = rows; ext_n = n; ext_active = true;
        prepass(pass, rank, world, ex);
    }

    void prepass(uint32_t pass, uint32_t rank = 0, uint32_t world = 1, const alvrl_exchange* ex = nullptr)
    {
        if (ext && clustered && !ext_active)
            throw IntegError(ALVRL_ERR_STATE, "host-cast scene: run the prepass with alvrl_integrator_prepass_records");
        if (world == 0 || rank >= world) throw IntegError(ALVRL_ERR_INVALID, "bad rank/world");
        if (world > 1 && (!ex || !ex->allgather)) throw IntegError(ALVRL_ERR_INVALID, "world > 1 needs an alvrl_exchange");
        if (!have_scene) throw IntegError(ALVRL_ERR_STATE, "prepass before preprocess");
        const double tw = now_ms();
        pass_vrls(pass);
        st.slices_failed = 0;
        st.fallback_built = 0;
        st.ms_rbuild = st.ms_refine = st.ms_exchange = st.ms_refine_kernel = st.ms_alloc = 0;
        st.refine_entries = 0;
        st.refine_split_entries = 0;
        st.global_clusters = 0;
        st.slices_local = 0;
        st.rows_built = 0;
        if (clustered) build_clusters(pass, rank, world, ex);
        st.ms_prepass_wall = now_ms() - tw;
    }

    // the pass's VRLs on the device (:276-287): traced per pass unless preloaded
    void pass_vrls(uint32_t pass)
    {
        if (ext && !vrls_from_file && !have_tracer)
            throw IntegError(ALVRL_ERR_STATE, "host-cast scene without a tracer scene: set the pass's VRLs with "
                             "alvrl_integrator_set_vrls first");
        chk(alvrl_set_pass(ctx, pass), "alvrl_set_pass");
        cur_pass = pass;
        // VRLs (:276-287): traced per pass unless preloaded from a file, over
        // the descriptor scene or a host-cast scene's tracer scene
        if (!vrls_from_file) {
            const double t0 = now_ms();
            const alvrl_scene_desc& td = ext ? tracer_desc : scene_desc;
            const SmokeBox& tb = ext ? tracer_box : scene;
            if (gpuTracer && !tb.has_delta()) {
                const uint32_t target = (uint32_t)std::max(vrlTargetNum, 0);
                uint32_t n = 0;
                uint64_t pc = 0;
                chk_host(alvrl_trace_vrls_gpu(&td, vrlSeed, pass, target, shortVrls ? 1 : 0, maxParticleDepth,
                                              rrDepth, nullptr, 0, &n, &pc));
                vrls.n = n;
                vrls.particle_count = pc;
                vrls.soa.assign(9 * (size_t)n, 0.0f);
                if (n)
                    chk_host(alvrl_trace_vrls_gpu(&td, vrlSeed, pass, target, shortVrls ? 1 : 0,
                                                  maxParticleDepth, rrDepth, vrls.soa.data(), n, &n, &pc));
            } else {
                vrls = trace_vrls(tb, vrlSeed, pass, (uint32_t)std::max(vrlTargetNum, 0), shortVrls,
                                  maxParticleDepth, rrDepth);
            }
            st.ms_trace = now_ms() - t0;
            uploaded_pass = 0xFFFFFFFFu;
        }
        if (!vrls_from_file || uploaded_pass == 0xFFFFFFFFu) {
            chk(alvrl_upload_vrls(ctx, vrls.soa.data(), vrls.n, std::max<uint64_t>(vrls.particle_count, 1), 0),
                "alvrl_upload_vrls");
            uploaded_pass = pass;
        }
        st.vrls = vrls.n;
        st.particles = vrls.particle_count;
    }

    // vrlClusterInfo out / in (vrlIntegrator.cpp:29-101): the state a remote
    // worker receives instead of running the prepass (:353-354)
    void save_cluster_info(const char* path) const
    {
        if (!clustered || slice_off.empty())
            throw IntegError(ALVRL_ERR_STATE, "no cluster info: run a clustered prepass first");
        chk_host(alvrl_cluster_info_write(path, (uint32_t)pixel_to_slice.size(), pixel_to_slice.data(),
                                          (uint32_t)slice_off.size() - 1, slice_off.data(), reps.data(),
                                          weights.data(), 0, nullptr, nullptr, (uint32_t)fb_reps.size(),
                                          fb_reps.data(), fb_w.data()));
    }

    void load_cluster_info(const char* path, uint32_t pass)
    {
        if (!have_scene) throw IntegError(ALVRL_ERR_STATE, "load_cluster_info before preprocess");
        alvrl_cluster_info* ci = nullptr;
        chk_host(alvrl_cluster_info_read(path, &ci));
        std::unique_ptr<alvrl_cluster_info, void (*)(alvrl_cluster_info*)> guard(ci, alvrl_cluster_info_free);
        uint32_t npix = 0, ns = 0, nr = 0, ng = 0, nfb = 0;
        chk_host(alvrl_cluster_info_sizes(ci, &npix, &ns, &nr, &ng, &nfb));
        if (npix != (uint32_t)scene.width * (uint32_t)scene.height)
            throw IntegError(ALVRL_ERR_INVALID, "cluster info: pixel count does not match the scene");
        std::vector<uint32_t> p2s(npix), so(ns + 1), rp(nr), fr(nfb);
        std::vector<float> w(nr), fw(nfb);
        chk_host(alvrl_cluster_info_get(ci, p2s.data(), so.data(), rp.data(), w.data(), nullptr, nullptr,
                                        fr.data(), fw.data()));
        install_cluster_info(pass, p2s, so, rp, w, fr, fw);
    }

    // the vrlClusterInfo of a pass received instead of computed (wakeup, :378-384)
    void install_cluster_info(uint32_t pass, std::vector<uint32_t>& p2s, std::vector<uint32_t>& so,
                              std::vector<uint32_t>& rp, std::vector<float>& w, std::vector<uint32_t>& fr,
                              std::vector<float>& fw)
    {
        if (!have_scene) throw IntegError(ALVRL_ERR_STATE, "cluster info before preprocess");
        if (p2s.size() != (size_t)scene.width * (size_t)scene.height)
            throw IntegError(ALVRL_ERR_INVALID, "cluster info: pixel count does not match the scene");
        if (so.empty() || so[0] != 0 || so.back() != rp.size() || w.size() != rp.size() || fw.size() != fr.size())
            throw IntegError(ALVRL_ERR_INVALID, "cluster info: inconsistent list sizes");
        for (size_t s = 0; s + 1 < so.size(); s++)
            if (so[s] > so[s + 1]) throw IntegError(ALVRL_ERR_INVALID, "cluster info: slice offsets decrease");
        const uint32_t ns = (uint32_t)so.size() - 1;
        for (uint32_t s : p2s)
            if (s != 0xFFFFFFFFu && s >= ns) throw IntegError(ALVRL_ERR_INVALID, "cluster info: slice id out of range");
        pass_vrls(pass);
        for (uint32_t v : rp)
            if (v >= vrls.n) throw IntegError(ALVRL_ERR_INVALID, "cluster info: VRL id out of range");
        for (uint32_t v : fr)
            if (v >= vrls.n) throw IntegError(ALVRL_ERR_INVALID, "cluster info: VRL id out of range");
        chk(alvrl_set_clusters(ctx, ns, so.data(), rp.data(), w.data(), fr.data(), fw.data(), (uint32_t)fr.size()),
            "alvrl_set_clusters");
        pixel_to_slice.swap(p2s);
        slice_off.swap(so); reps.swap(rp); weights.swap(w); fb_reps.swap(fr); fb_w.swap(fw);
        clustered = true;
        cache_rank = 0xFFFFFFFFu;
        st.slices = ns;
        st.clusters_total = reps.size();
    }

    // LiInternal's specular chains (:445-511) of the given row-major pixels,
    // traced on the host (SmokeBox::make_chain, the occluders are few):
    // recs[d - 1] = the records of depth d >= 1 (their path weights
    // transmittance * bsdfWeight / rrProb multiplied along the chain), src =
    // the index into ids of each; prim[i] = the primary record of ids[i]
    // (the device's eye-ray kernel knows no materials).  The Russian roulette
    // draws from the pass's (seed, pass, pixel, depth) stream.
    struct Chains {
        std::vector<std::vector<alvrl_gather_rec>> recs;
        std::vector<std::vector<uint32_t>> src;
    };
    Chains expand_chains(const std::vector<uint32_t>& ids, bool scat, bool accum,
                         std::vector<alvrl_gather_rec>* prim, uint32_t sample = 0, uint32_t spp = 1) const
    {
        prim->resize(ids.size());
        const uint32_t n = (uint32_t)ids.size();
        const uint32_t W = (uint32_t)scene.width;
        unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        if (n < 4096) nt = 1;
        std::vector<Chains> part(nt);
        auto work = [&](unsigned t) {
            std::vector<float> buf;
            Chains& c = part[t];
            const uint32_t b = (uint32_t)((uint64_t)n * t / nt), e = (uint32_t)((uint64_t)n * (t + 1) / nt);
            for (uint32_t i = b; i < e; i++) {
                scene.make_record((int)(ids[i] % W), (int)(ids[i] / W), scat, reinterpret_cast<float*>(&(*prim)[i]),
                                  seed, cur_pass, sample, spp);
                buf.clear();
                scene.make_chain((int)(ids[i] % W), (int)(ids[i] / W), scat, seed, cur_pass, specRRdepth,
                                 initialSpecularThroughput, &buf, sample, spp);
                const size_t k = buf.size() / kRecWords;
                for (size_t d = 1; d < k; d++) {
                    if (c.recs.size() < d) { c.recs.resize(d); c.src.resize(d); }
                    alvrl_gather_rec r;
                    std::memcpy(&r, &buf[d * kRecWords], sizeof(r));
                    if (accum) r.flags |= ALVRL_REC_ACCUM;
                    c.recs[d - 1].push_back(r);
                    c.src[d - 1].push_back(i);
                }
            }
        };
        if (nt == 1) work(0);
        else {
            std::vector<std::thread> th;
            for (unsigned t = 0; t < nt; t++) th.emplace_back(work, t);
            for (auto& x : th) x.join();
        }
        Chains out;
        for (unsigned t = 0; t < nt; t++) {
            if (out.recs.size() < part[t].recs.size()) {
                out.recs.resize(part[t].recs.size());
                out.src.resize(part[t].recs.size());
            }
            for (size_t d = 0; d < part[t].recs.size(); d++) {
                out.recs[d].insert(out.recs[d].end(), part[t].recs[d].begin(), part[t].recs[d].end());
                out.src[d].insert(out.src[d].end(), part[t].src[d].begin(), part[t].src[d].end());
            }
        }
        return out;
    }

    // The host's records of the built rows gl[i] (alvrl_integrator_prepass_records),
    // in the form expand_chains gives: prim[i] = row i's first record (zero --
    // no hit, no contribution -- if it has none), then level by level the
    // further ones, flagged ALVRL_REC_ACCUM (getLiLuminanceVrlContributions
    // adds a path's segments into the row, :812-813)
    Chains host_rows(const std::vector<uint32_t>& gl, uint32_t rows, std::vector<alvrl_gather_rec>* prim) const
    {
        const uint32_t nb = (uint32_t)gl.size();
        std::vector<uint32_t> bidx(rows, 0xFFFFFFFFu);
        for (uint32_t i = 0; i < nb; i++) bidx[gl[i]] = i;
        prim->assign(nb, alvrl_gather_rec{});
        std::vector<uint32_t> cnt(nb, 0);
        Chains ch;
        for (uint32_t k = 0; k < ext_n; k++) {
            const uint32_t g = ext_row[k];
            if (g >= rows) throw IntegError(ALVRL_ERR_INVALID, "alvrl_integrator_prepass_records: row_of_rec out of range");
            const uint32_t i = bidx[g];
            if (i == 0xFFFFFFFFu) continue;   // a row of another rank's slice
            alvrl_gather_rec r = ext_recs[k];
            r.flags &= ~ALVRL_REC_ACCUM;
            const uint32_t d = cnt[i]++;
            if (d == 0) { (*prim)[i] = r; continue; }
            if (ch.recs.size() < d) { ch.recs.resize(d); ch.src.resize(d); }
            r.flags |= ALVRL_REC_ACCUM;
            ch.recs[d - 1].push_back(r);
            ch.src[d - 1].push_back(i);
        }
        return ch;
    }

    // Building R (:302-333) for the rows of the slices flagged in 'need'.  R is
    // stored as one [vrl][row] block per slice (the reference's
    // R[slice][rep][vrl], transposed): a slice's local matrix is then one
    // contiguous run -- consecutive VRL columns 8 * R_s bytes apart instead of
    // 8 * rows -- which the refinement streams.  Blocks are packed in slice
    // order, so with every slice built global row g of slice s lives at
    // float2 index nv * rep_off[s] + (g - rep_off[s]) + v * R_s.  One launch
    // builds every block and ORs the non-zero VRL mask of Preprocessor::cluster
    // (:843-855) into 'nz'.
    void build_R(const std::vector<char>& need, std::vector<uint8_t>* nz)
    {
        const uint32_t nv = vrls.n;
        const auto& roff = prep->rep_off();
        const auto& rpix = prep->rep_pix();
        const uint32_t ns = prep->num_slices();
        const uint32_t rows = roff[ns];
        const int H = scene.height, W = scene.width;
        const bool scat = !(scene.medium.sigma_s[0] == 0 && scene.medium.sigma_s[1] == 0 && scene.medium.sigma_s[2] == 0);
        row_base.assign(rows, UINT64_MAX);
        row_stride.assign(rows, 0);
        // records of the representative pixel centres (sensor->sampleRay at
        // the pixel centre, :327-328 / :1060-1061), formed on the device from
        // the row-major pixel ids (the RNG ids too)
        std::vector<uint32_t> ids, bstr, gl;
        std::vector<uint64_t> boff;
        uint64_t acc = 0;
        for (uint32_t s2 = 0; s2 < ns; s2++) {
            if (!need[s2]) continue;
            const uint32_t n = roff[s2 + 1] - roff[s2];
            for (uint32_t g = roff[s2]; g < roff[s2 + 1]; g++) {
                row_base[g] = (uint64_t)nv * acc + (g - roff[s2]);
                row_stride[g] = n;
                const uint32_t x = rpix[g] / (uint32_t)H, y = rpix[g] % (uint32_t)H;
                ids.push_back(y * (uint32_t)W + x);
                gl.push_back(g);
                boff.push_back(row_base[g]);
                bstr.push_back(n);
            }
            acc += n;
        }
        const uint32_t nb = (uint32_t)ids.size();
        rows_built = nb;
        const double ta = now_ms();
        rep_recs.ensure(nb);
        rep_ids.ensure(nb);
        rb_off.ensure(nb);
        rb_stride.ensure(nb);
        nz_dev.ensure(nv);
        Rt.ensure((size_t)2 * nv * acc);
        st.ms_alloc += now_ms() - ta;
        if (nb) {
            hchk(hipMemcpyAsync(rep_ids.p, ids.data(), sizeof(uint32_t) * nb, hipMemcpyHostToDevice, stream), "copy rep ids");
            if (!chains && !ext) chk_host(alvrl_scene_records_gpu(&scene_desc, scat ? 1 : 0, rep_ids.p, nb, rep_recs.p, stream));
            hchk(hipMemcpyAsync(rb_off.p, boff.data(), sizeof(uint64_t) * nb, hipMemcpyHostToDevice, stream), "copy row offsets");
            hchk(hipMemcpyAsync(rb_stride.p, bstr.data(), sizeof(uint32_t) * nb, hipMemcpyHostToDevice, stream), "copy row strides");
        }
        // getLiLuminanceVrlContributions follows the row's delta-BSDF chain
        // (:527-539 -> LiInternal :445-511) and the contributions of every
        // level add into the row (:812-813): one launch per depth level, its
        // records flagged ALVRL_REC_ACCUM (a row has at most one record per level)
        Chains ch;
        std::vector<uint32_t> lv_off{0};
        if ((chains || ext) && nb) {
            std::vector<alvrl_gather_rec> prim;
            if (ext) ch = host_rows(gl, rows, &prim);
            else ch = expand_chains(ids, scat, true, &prim);
            hchk(hipMemcpy(rep_recs.p, prim.data(), sizeof(alvrl_gather_rec) * nb, hipMemcpyHostToDevice), "copy records");
            std::vector<alvrl_gather_rec> r;
            std::vector<uint32_t> cid, cstr;
            std::vector<uint64_t> coff;
            for (size_t d = 0; d < ch.recs.size(); d++) {
                for (size_t j = 0; j < ch.recs[d].size(); j++) {
                    const uint32_t i = ch.src[d][j];
                    r.push_back(ch.recs[d][j]);
                    cid.push_back(ids[i]); coff.push_back(boff[i]); cstr.push_back(bstr[i]);
                }
                lv_off.push_back((uint32_t)r.size());
            }
            const size_t n = r.size();
            ch_recs.ensure(n); ch_ids.ensure(n); ch_off.ensure(n); ch_stride.ensure(n);
            if (n) {
                hchk(hipMemcpyAsync(ch_recs.p, r.data(), sizeof(alvrl_gather_rec) * n, hipMemcpyHostToDevice, stream), "copy chain records");
                hchk(hipMemcpyAsync(ch_ids.p, cid.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice, stream), "copy chain ids");
                hchk(hipMemcpyAsync(ch_off.p, coff.data(), sizeof(uint64_t) * n, hipMemcpyHostToDevice, stream), "copy chain offsets");
                hchk(hipMemcpyAsync(ch_stride.p, cstr.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice, stream), "copy chain strides");
                hchk(hipStreamSynchronize(stream), "sync");   // r, cid, ... are freed on return
            }
        }
        hchk(hipMemsetAsync(nz_dev.p, 0, nv, stream), "clear mask");
        hipEvent_t e0, e1;
        hchk(hipEventCreate(&e0), "event"); hchk(hipEventCreate(&e1), "event");
        hchk(hipEventRecord(e0, stream), "event");
        chk(alvrl_build_R_blocks(ctx, rep_recs.p, rep_ids.p, nb, Rt.p, rb_off.p, rb_stride.p, nz_dev.p, stream),
            "alvrl_build_R_blocks");
        for (size_t d = 0; d + 1 < lv_off.size(); d++)
            chk(alvrl_build_R_blocks(ctx, ch_recs.p + lv_off[d], ch_ids.p + lv_off[d], lv_off[d + 1] - lv_off[d], Rt.p,
                                     ch_off.p + lv_off[d], ch_stride.p + lv_off[d], nz_dev.p, stream),
                "alvrl_build_R_blocks (chain level)");
        hchk(hipEventRecord(e1, stream), "event");
        nz->assign(nv, 0);
        if (nv) hchk(hipMemcpyAsync(nz->data(), nz_dev.p, nv, hipMemcpyDeviceToHost, stream), "copy mask");
        hchk(hipStreamSynchronize(stream), "sync");
        float ms = 0;
        hchk(hipEventElapsedTime(&ms, e0, e1), "event");
        st.ms_rbuild += ms;
        hipEventDestroy(e0); hipEventDestroy(e1);
    }

    // The slices of rank `rank` of `world`: longest processing time first over
    // each slice's local-matrix rows (the refinement's and the R build's cost
    // both grow with them; every slice has every column) -- slices by cost,
    // largest first (ties: lower index), each to the least-loaded rank (ties:
    // lower rank) -- or s % world with sliceSharding=roundrobin.  Every rank
    // derives the same assignment from the pass's slice mapping.
    std::vector<uint32_t> slices_of_rank(uint32_t rank, uint32_t world,
                                         const std::vector<std::vector<uint32_t>>& all_rows) const
    {
        const uint32_t ns = (uint32_t)all_rows.size();
        std::vector<uint32_t> mine;
        if (world <= 1 || sliceRoundRobin) {
            for (uint32_t s = rank; s < ns; s += world) mine.push_back(s);
            return mine;
        }
        std::vector<uint32_t> order(ns);
        for (uint32_t s = 0; s < ns; s++) order[s] = s;
        std::stable_sort(order.begin(), order.end(),
                         [&](uint32_t a, uint32_t b) { return all_rows[a].size() > all_rows[b].size(); });
        std::vector<uint64_t> load(world, 0);
        for (uint32_t s : order) {
            uint32_t best = 0;
            for (uint32_t r = 1; r < world; r++)
                if (load[r] < load[best]) best = r;
            load[best] += all_rows[s].size();
            if (best == rank) mine.push_back(s);
        }
        std::sort(mine.begin(), mine.end());
        return mine;
    }

    // buildClusters (:293-346).  With world > 1 the slices are sharded over
    // the ranks (slices_of_rank): this rank builds R for its slices and their
    // neighbours' rows, refines its slices, and the exchange makes the mask
    // and the cluster lists global.
    void build_clusters(uint32_t pass_id, uint32_t rank, uint32_t world, const alvrl_exchange* ex)
    {
        const uint32_t nv = vrls.n;
        // sampleSliceMapping (:293-296)
        prep->set_pass(pass_id);
        prep->sample_slice_mapping(targetPixelUndersampling);
        const auto& roff = prep->rep_off();
        const uint32_t ns = prep->num_slices();
        const uint32_t rows = roff[ns];
        st.rep_rows = rows;
        // local matrices (getLocalMatrix, :779-827): every slice's with world > 1
        // (the assignment's costs), this rank's slices' otherwise
        std::vector<std::vector<uint32_t>> all_rows(world > 1 ? ns : 0);
        std::vector<std::vector<double>> all_w(world > 1 ? ns : 0);
        for (uint32_t s = 0; s < (world > 1 ? ns : 0); s++) prep->local_matrix(s, &all_rows[s], &all_w[s]);
        std::vector<uint32_t> mine;
        if (world > 1) mine = slices_of_rank(rank, world, all_rows);
        else for (uint32_t s = 0; s < ns; s++) mine.push_back(s);
        local_slices = mine;
        const uint32_t nm = (uint32_t)mine.size();
        std::vector<std::vector<uint32_t>> lrows(nm);
        std::vector<std::vector<double>> lw(nm);
        std::vector<char> need(ns, 0);
        for (uint32_t k = 0; k < nm; k++) {
            if (world > 1) { lrows[k].swap(all_rows[mine[k]]); lw[k].swap(all_w[mine[k]]); }
            else prep->local_matrix(mine[k], &lrows[k], &lw[k]);
            need[mine[k]] = 1;
            for (uint32_t g : lrows[k])
                need[(uint32_t)(std::upper_bound(roff.begin(), roff.end(), g) - roff.begin()) - 1] = 1;
        }
        std::vector<uint8_t> nz;
        build_R(need, &nz);
        // Preprocessor::cluster (:838-898): non-zero VRLs in one cluster, zero VRLs in another
        double tx = now_ms();
        if (world > 1) or_reduce(*ex, world, nz.data(), nv);
        st.ms_exchange += now_ms() - tx;
        std::vector<uint32_t> init;
        init.reserve(nv);
        for (uint32_t v = 0; v < nv; v++) if (nz[v]) init.push_back(v);
        const uint32_t nnz = (uint32_t)init.size();
        for (uint32_t v = 0; v < nv; v++) if (!nz[v]) init.push_back(v);
        std::vector<uint32_t> init_off{0};
        if (nnz) init_off.push_back(nnz);
        if (nnz != nv) init_off.push_back(nv);
        if (globalCluster && nnz) {
            // clusterRefinement (Preprocessor.cpp:899-912): the non-zero VRLs
            // refined as one cluster over all rows with globalUndersampling;
            // its clusters (getVrlsPerCluster) plus the zero cluster become
            // every slice's initial clusters.  Needs every row of R.
            if (rows_built != rows) {
                std::vector<uint8_t> unused;
                build_R(std::vector<char>(ns, 1), &unused);
            }
            std::vector<uint32_t> all(rows);
            for (uint32_t r = 0; r < rows; r++) all[r] = r;
            std::vector<double> dw(rows, 1.0 / (double)rows);
            alvrl_cluster_job gj{};
            gj.rows = all.data(); gj.locw = dw.data(); gj.nrows = rows;
            gj.row_off = row_base.data(); gj.row_stride = row_stride.data();
            gj.pixel_undersampling = prep->global_pixel_undersampling();
            gj.undersampling = globalUndersampling;
            gj.depth_correction = 1.0f;
            gj.do_refine = 1;
            gj.stage_refine = gj.stage_sample = kStageGlobalRefine;
            const uint32_t one[2] = {0, nnz};
            std::vector<uint32_t> mem(nnz + 1), moff(nnz + 2);
            uint32_t nc = 0;
            int ok = 0;
            const double tg = now_ms();
            chk(alvrl_refine_members(ctx, Rt.p, rows, &gj, init.data(), one, 1, mem.data(), moff.data(), &nc,
                                     &ok, stream), "alvrl_refine_members (global cluster)");
            st.ms_refine += now_ms() - tg;
            {
                float kms = 0.0f;
                uint64_t ent = 0;
                chk(alvrl_last_refine_ms(ctx, &kms), "alvrl_last_refine_ms");
                chk(alvrl_last_refine_entries(ctx, &ent), "alvrl_last_refine_entries");
                uint64_t sent = 0;
                chk(alvrl_last_refine_split_entries(ctx, &sent), "alvrl_last_refine_split_entries");
                st.ms_refine_kernel += kms;
                st.refine_entries += ent;
                st.refine_split_entries += sent;
            }
            if (!ok) throw IntegError(ALVRL_ERR_NUMERIC, "Couldn't refine global clustering!");
            std::copy(mem.begin(), mem.begin() + nnz, init.begin());
            init_off.assign(moff.begin(), moff.begin() + nc + 1);
            if (nnz != nv) init_off.push_back(nv);
            st.global_clusters = nc;
        }
        // refinePerSlice (:199-252): one device job per slice
        std::vector<std::vector<uint64_t>> loff(nm);
        std::vector<std::vector<uint32_t>> lstr(nm);
        std::vector<alvrl_cluster_job> jobs(nm);
        for (uint32_t k = 0; k < nm; k++) {
            const uint32_t s = mine[k];
            for (uint32_t g : lrows[k]) { loff[k].push_back(row_base[g]); lstr[k].push_back(row_stride[g]); }
            alvrl_cluster_job& j = jobs[k];
            j.rows = lrows[k].data();
            j.row_off = loff[k].data();
            j.row_stride = lstr[k].data();
            j.locw = lw[k].data();
            j.nrows = (uint32_t)lrows[k].size();
            j.pixel_undersampling = prep->slice_undersampling()[s];
            j.undersampling = localUndersampling;
            j.depth_correction = depthCorrection;
            j.do_refine = localRefinement ? 1 : 0;
            j.stage_refine = stage_slice_refine(s);
            j.stage_sample = stage_slice_sample(s);
        }
        job_init = init; job_init_off = init_off; job_slices = mine; job_rows = lrows; job_locw = lw;
        // output lists sized for every VRL in every job: kept between passes
        // (value-initialising 2 x 40 MB per pass cost milliseconds)
        std::vector<uint32_t> off(nm + 1);
        if (rep_buf.size() < (size_t)nm * nv + 1) rep_buf.resize((size_t)nm * nv + 1);
        if (w_buf.size() < (size_t)nm * nv + 1) w_buf.resize((size_t)nm * nv + 1);
        std::vector<uint32_t>& rep = rep_buf;
        std::vector<float>& w = w_buf;
        std::vector<int> refined(nm + 1);
        const double t0 = now_ms() - st.ms_refine;
        if (nm)
            chk(alvrl_refine(ctx, Rt.p, rows, nm, jobs.data(), init.data(), init_off.data(),
                             (uint32_t)init_off.size() - 1, off.data(), rep.data(), w.data(),
                             refined.data(), stream), "alvrl_refine (slices)");
        st.ms_refine = now_ms() - t0;
        st.slices_local = nm;
        if (nm) {
            float kms = 0.0f;
            uint64_t ent = 0;
            chk(alvrl_last_refine_ms(ctx, &kms), "alvrl_last_refine_ms");
            chk(alvrl_last_refine_entries(ctx, &ent), "alvrl_last_refine_entries");
            uint64_t sent = 0;
            chk(alvrl_last_refine_split_entries(ctx, &sent), "alvrl_last_refine_split_entries");
            st.ms_refine_kernel += kms;
            st.refine_entries += ent;
            st.refine_split_entries += sent;
        }
        // every rank gets every slice's list
        SliceClusters m;
        if (world > 1) {
            tx = now_ms();
            m = merge_clusters(*ex, world, ns, nm, mine.data(), refined.data(), off.data(), rep.data(), w.data());
            st.ms_exchange += now_ms() - tx;
        } else {
            m.refined.assign(refined.begin(), refined.begin() + ns);
            m.off.assign(off.begin(), off.begin() + ns + 1);
            m.reps.assign(rep.begin(), rep.begin() + off[ns]);
            m.w.assign(w.begin(), w.begin() + off[ns]);
        }
        // Fall-back clustering (buildClusters :175-186): refine the global
        // clustering of all rows to N/fallBackUndersampling clusters.  Only its
        // users need it -- slices whose refinement failed (:276-282) and pixels
        // without a gather point (:564-571) -- and its counter-RNG streams are
        // its own, so it is built only when one of them exists.  Every rank
        // computes it from all rows (R of the missing slices built here).
        uint32_t failed = 0;
        for (uint32_t s = 0; s < ns; s++) failed += m.refined[s] ? 0 : 1;
        bool need_fb = failed > 0;
        for (uint32_t p : pixel_to_slice) if (p == 0xFFFFFFFFu) { need_fb = true; break; }
        fb_reps.clear(); fb_w.clear();
        if (need_fb) {
            if (rows_built != rows) {
                std::vector<uint8_t> unused;
                build_R(std::vector<char>(ns, 1), &unused);
            }
            std::vector<uint32_t> all(rows);
            for (uint32_t r = 0; r < rows; r++) all[r] = r;
            std::vector<double> dw(rows, 1.0 / (double)rows);
            alvrl_cluster_job fj;
            fj.rows = all.data(); fj.locw = dw.data(); fj.nrows = rows;
            fj.row_off = row_base.data(); fj.row_stride = row_stride.data();
            fj.pixel_undersampling = prep->global_pixel_undersampling();
            fj.undersampling = fallBackUndersampling;
            fj.depth_correction = 1.0f;
            fj.do_refine = 1;
            fj.stage_refine = kStageFallbackRefine;
            fj.stage_sample = kStageFallbackSample;
            std::vector<uint32_t> foff(2), frep(nv + 1);
            std::vector<float> fw(nv + 1);
            int fref = 0;
            const double t1 = now_ms();
            chk(alvrl_refine(ctx, Rt.p, rows, 1, &fj, init.data(), init_off.data(),
                             (uint32_t)init_off.size() - 1, foff.data(), frep.data(), fw.data(), &fref,
                             stream), "alvrl_refine (fall-back)");
            st.ms_refine += now_ms() - t1;
            {
                float kms = 0.0f;
                uint64_t ent = 0;
                chk(alvrl_last_refine_ms(ctx, &kms), "alvrl_last_refine_ms");
                chk(alvrl_last_refine_entries(ctx, &ent), "alvrl_last_refine_entries");
                uint64_t sent = 0;
                chk(alvrl_last_refine_split_entries(ctx, &sent), "alvrl_last_refine_split_entries");
                st.ms_refine_kernel += kms;
                st.refine_entries += ent;
                st.refine_split_entries += sent;
            }
            if (!fref) throw IntegError(ALVRL_ERR_NUMERIC, "couldn't refine global clustering! (but all VRLs should be non-zero!)");
            fb_reps.assign(frep.begin(), frep.begin() + foff[1]);
            fb_w.assign(fw.begin(), fw.begin() + foff[1]);
            st.fallback_built = 1;
        }
        slice_off.assign(ns + 1, 0);
        reps.clear(); weights.clear();
        for (uint32_t s = 0; s < ns; s++) {
            slice_off[s] = (uint32_t)reps.size();
            if (m.refined[s]) {
                reps.insert(reps.end(), m.reps.begin() + m.off[s], m.reps.begin() + m.off[s + 1]);
                weights.insert(weights.end(), m.w.begin() + m.off[s], m.w.begin() + m.off[s + 1]);
            } else {   // "Could not refine slice %d, using fall-back clustering!"
                reps.insert(reps.end(), fb_reps.begin(), fb_reps.end());
                weights.insert(weights.end(), fb_w.begin(), fb_w.end());
            }
        }
        slice_off[ns] = (uint32_t)reps.size();
        st.slices_failed = failed;
        st.clusters_total = reps.size();
        st.rows_built = rows_built;
        chk(alvrl_set_clusters(ctx, ns, slice_off.data(), reps.data(), weights.data(), fb_reps.data(),
                               fb_w.data(), (uint32_t)fb_reps.size()), "alvrl_set_clusters");
    }

    void prepare_render(uint32_t rank, uint32_t world)
    {
        const uint32_t mode = clustered ? 2u : 1u;
        // chains (their Russian roulette) and sensor samples depend on the pass
        const uint32_t S = (uint32_t)sampleCount;
        if (cache_rank == rank && cache_world == world && cache_mode == mode &&
            ((!chains && S == 1) || cache_pass == cur_pass))
            return;
        const int W = scene.width, H = scene.height;
        uint32_t npix = 0;
        chk_host(alvrl_tile_pixels(W, H, rank, world, nullptr, 0, &npix));
        std::vector<uint32_t> pix(npix);
        chk_host(alvrl_tile_pixels(W, H, rank, world, pix.data(), npix, &npix));
        std::vector<alvrl_work_item> items;
        // bucket a level's records by the slice of their pixel (stable; the
        // camera ray's slice at every depth, :550-560) into wave work items
        auto bucket = [&](std::vector<uint32_t>* order, const std::vector<uint32_t>& recpix, uint32_t base) {
            std::vector<uint32_t> sl(recpix.size());
            for (size_t i = 0; i < recpix.size(); i++) {
                const uint32_t x = recpix[i] % (uint32_t)W, y = recpix[i] / (uint32_t)W;
                sl[i] = pixel_to_slice[y + (uint32_t)H * x];   // m_slices[y + H*x] (:560)
            }
            order->resize(recpix.size());
            for (size_t i = 0; i < order->size(); i++) (*order)[i] = (uint32_t)i;
            std::stable_sort(order->begin(), order->end(), [&](uint32_t a, uint32_t b) { return sl[a] < sl[b]; });
            std::vector<uint32_t> s2(sl.size());
            for (size_t i = 0; i < s2.size(); i++) s2[i] = sl[(*order)[i]];
            std::vector<alvrl_work_item> it(s2.size() + 1);
            const uint32_t n = alvrl_make_work_items(s2.data(), (uint32_t)s2.size(), it.data(), (uint32_t)it.size());
            for (uint32_t k = 0; k < n; k++) { it[k].begin += base; items.push_back(it[k]); }
        };
        if (clustered) {
            std::vector<uint32_t> order;
            bucket(&order, pix, 0);
            std::vector<uint32_t> p2(pix.size());
            for (size_t i = 0; i < order.size(); i++) p2[i] = pix[order[i]];
            pix.swap(p2);
            // launch the waves of the longest representative lists first: the
            // last waves to start are then the short ones (C4: 44.5 against
            // 45.7 ms, tools/gather_tail.py); the lists are the pass's, the
            // order a scheduling choice only (every wave's result is the same)
            if (slice_off.size() > 1) {
                auto len = [&](uint32_t sl) -> uint32_t {
                    return sl == 0xFFFFFFFFu || sl + 1 >= slice_off.size() ? (uint32_t)fb_reps.size()
                                                                          : slice_off[sl + 1] - slice_off[sl];
                };
                std::stable_sort(items.begin(), items.end(), [&](const alvrl_work_item& a, const alvrl_work_item& b) {
                    return len(a.slice) > len(b.slice);
                });
            }
        }
        const bool scat = !(scene.medium.sigma_s[0] == 0 && scene.medium.sigma_s[1] == 0 && scene.medium.sigma_s[2] == 0);
        const uint32_t nprim = (uint32_t)pix.size();
        if ((uint64_t)nprim * S > 0x7FFFFFFFull) throw IntegError(ALVRL_ERR_INVALID, "sampleCount too large for the frame");
        // the sensor samples' primary records, sample major: block j holds
        // sample j of every owned pixel (the pixel order and work items of
        // block 0); each block is one accumulation level
        level_rec.assign({0u});
        level_item.assign({0u});
        {
            const size_t nit = items.size();
            for (uint32_t j = 0; j < S; j++) {
                if (j)
                    for (size_t k = 0; k < nit; k++) {
                        alvrl_work_item w = items[k];
                        w.begin += j * nprim;
                        items.push_back(w);
                    }
                level_rec.push_back((j + 1) * nprim);
                level_item.push_back((uint32_t)items.size());
            }
            const std::vector<uint32_t> p0(pix);
            pix.reserve((size_t)nprim * S);
            for (uint32_t j = 1; j < S; j++) pix.insert(pix.end(), p0.begin(), p0.end());
        }
        std::vector<alvrl_gather_rec> extra;   // the chains' records, level by level
        std::vector<alvrl_gather_rec> prim;
        if (chains) {
            prim.resize((size_t)nprim * S);
            const std::vector<uint32_t> ppix(pix.begin(), pix.begin() + nprim);
            for (uint32_t j = 0; j < S; j++) {
                std::vector<alvrl_gather_rec> pj;
                Chains ch = expand_chains(ppix, scat, false, &pj, j, S);
                std::copy(pj.begin(), pj.end(), prim.begin() + (size_t)j * nprim);
                for (size_t d = 0; d < ch.recs.size(); d++) {
                    std::vector<uint32_t> recpix(ch.src[d].size());
                    for (size_t k = 0; k < recpix.size(); k++) recpix[k] = ppix[ch.src[d][k]];
                    const uint32_t base = nprim * S + (uint32_t)extra.size();
                    std::vector<uint32_t> order(recpix.size());
                    for (size_t k = 0; k < order.size(); k++) order[k] = (uint32_t)k;
                    if (clustered) bucket(&order, recpix, base);
                    for (uint32_t k : order) { extra.push_back(ch.recs[d][k]); pix.push_back(recpix[k]); }
                    level_rec.push_back(nprim * S + (uint32_t)extra.size());
                    level_item.push_back((uint32_t)items.size());
                }
            }
        }
        nrec = (uint32_t)pix.size();
        nitems = (uint32_t)items.size();
        rec_buf.ensure(nrec);
        pix_buf.ensure(nrec);
        out_buf.ensure((size_t)3 * nrec);
        hchk(hipMemcpyAsync(pix_buf.p, pix.data(), sizeof(uint32_t) * nrec, hipMemcpyHostToDevice, stream), "copy pixels");
        // the eye-ray first hits of the owned pixels' sensor samples, on the device
        if (chains) {
            if (nprim)
                hchk(hipMemcpyAsync(rec_buf.p, prim.data(), sizeof(alvrl_gather_rec) * prim.size(),
                                    hipMemcpyHostToDevice, stream), "copy records");
        } else
            chk_host(alvrl_scene_records_spp_gpu(&scene_desc, scat ? 1 : 0, seed, cur_pass, S, pix_buf.p, nprim,
                                                 rec_buf.p, stream));
        if (!extra.empty())
            hchk(hipMemcpyAsync(rec_buf.p + (size_t)nprim * S, extra.data(), sizeof(alvrl_gather_rec) * extra.size(),
                                hipMemcpyHostToDevice, stream), "copy chain records");
        if (nitems) {
            item_buf.ensure(nitems);
            hchk(hipMemcpyAsync(item_buf.p, items.data(), sizeof(alvrl_work_item) * nitems, hipMemcpyHostToDevice, stream), "copy items");
        }
        hchk(hipStreamSynchronize(stream), "sync");
        cache_rank = rank; cache_world = world; cache_mode = mode; cache_pass = cur_pass;
    }

    void render(uint32_t rank, uint32_t world, float* d_fb, hipStream_t s)
    {
        if (!have_scene) throw IntegError(ALVRL_ERR_STATE, "render before preprocess");
        if (ext)
            throw IntegError(ALVRL_ERR_STATE, "host-cast scene: gather the host's eye records with "
                                              "alvrl_gather_clustered_host / alvrl_gather_brute_host");
        if (world == 0 || rank >= world) throw IntegError(ALVRL_ERR_INVALID, "bad rank/world");
        prepare_render(rank, world);
        // the caller's stream waits for the records upload (done, synchronous above)
        // false colour (LiInternal, :427-443, 545-599, 794-806): numVrlFalseColor
        // wins over slicesFalseColor; convergenceFalseColor only rewrites the
        // result after a specular (delta-BSDF) chain (:514-521), which the
        // smoke box's diffuse walls never start, so it leaves the image as is
        // With delta-BSDF chains every level's records are gathered in the same
        // launch (their path weights applied in the kernels) and the levels
        // are added into the frame in depth order, one launch each, so that
        // no two additions to a pixel race.  slicesFalseColor stops at the
        // first hit (:461-462); numVrlFalseColor keeps weight 1 down the
        // chain (:502-503), which the false-colour kernel never applies.
        uint32_t levels = (uint32_t)level_rec.size() - 1;
        render_timed = false;   // get_stats' ms_render_kernel: the gather of this render only
        if (numVrlFalseColor || slicesFalseColor) {
            if (!clustered && !numVrlFalseColor)
                throw IntegError(ALVRL_ERR_INVALID, "requested slices false color image without clustering!");
            const int mode = numVrlFalseColor ? ALVRL_FALSE_COLOR_NUM_VRLS : ALVRL_FALSE_COLOR_SLICES;
            if (!numVrlFalseColor) levels = (uint32_t)sampleCount;   // the primary blocks
            chk(alvrl_gather_false_color(ctx, mode, rec_buf.p, clustered ? item_buf.p : nullptr,
                                         clustered ? level_item[levels] : level_rec[levels], out_buf.p, s),
                "alvrl_gather_false_color");
        } else {
            hchk(hipEventRecord(ev_r0, s), "hipEventRecord");
            if (clustered)
                chk(alvrl_gather_clustered(ctx, rec_buf.p, pix_buf.p, item_buf.p, nitems, out_buf.p, s),
                    "alvrl_gather_clustered");
            else
                chk(alvrl_gather_brute(ctx, rec_buf.p, pix_buf.p, nrec, out_buf.p, s), "alvrl_gather_brute");
            hchk(hipEventRecord(ev_r1, s), "hipEventRecord");
            render_timed = true;
        }
        // ImageBlock::put of each sensor sample, normalised by the box
        // filter's weight sum at develop time: the mean over the samples
        if (sampleCount > 1 && level_rec[levels]) {
            const uint32_t nv = 3u * level_rec[levels];
            hipLaunchKernelGGL(k_scale_f32, dim3((nv + 255) / 256), dim3(256), 0, s, out_buf.p, nv,
                               1.0f / (float)sampleCount);
            hchk(hipGetLastError(), "k_scale_f32");
        }
        for (uint32_t d = 0; d < levels; d++)
            chk(alvrl_accumulate_rgb(ctx, out_buf.p + (size_t)3 * level_rec[d], pix_buf.p + level_rec[d],
                                     level_rec[d + 1] - level_rec[d], d_fb, s), "alvrl_accumulate_rgb");
        if (s != stream) {
            // the launches above read rec_buf / pix_buf / out_buf on the
            // caller's stream; the next prepare_render rewrites them on the
            // integrator's own stream, which therefore waits for them
            hipEvent_t ev = nullptr;
            hchk(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
            hipError_t e = hipEventRecord(ev, s);
            if (e == hipSuccess) e = hipStreamWaitEvent(stream, ev, 0);
            (void)hipEventDestroy(ev);
            hchk(e, "order the integrator's stream after the render");
        }
    }
};

static int ierr(int code, const std::string& m)
{
    g_host_err = m;
    return code;
}

#define GUARD(...)                                                           \
    try {                                                                    \
        __VA_ARGS__;                                                         \
    } catch (const IntegError& e) {                                          \
        return ierr(e.code, e.what());                                       \
    } catch (const CommError& e) {                                           \
        return ierr(e.code, e.what());                                       \
    } catch (const std::exception& e) {                                      \
        return ierr(ALVRL_ERR_INVALID, e.what());                            \
    }

extern "C" {

ALVRL_API int alvrl_integrator_create(const char* props, int device, alvrl_integrator** out)
{
    if (!out) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_create: null out");
    std::unique_ptr<alvrl_integrator> it(new alvrl_integrator());
    GUARD({
        std::string p = props ? props : "";
        std::stringstream ss(p);
        std::string kv;
        while (std::getline(ss, kv, ';')) {
            const auto a = kv.find_first_not_of(" \t\n");
            if (a == std::string::npos) continue;
            kv = kv.substr(a);
            const auto eq = kv.find('=');
            if (eq == std::string::npos) throw IntegError(ALVRL_ERR_INVALID, "property without '=': " + kv);
            std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
            while (!k.empty() && (k.back() == ' ' || k.back() == '\t')) k.pop_back();
            it->set(k, v);
        }
        it->validate();
        it->device = device;
        alvrl_config cfg{device, it->volVolSamples, it->volSurfSamples, it->shortVrls ? 1 : 0, it->seed};
        chk(alvrl_ctx_create(&cfg, &it->ctx), "alvrl_ctx_create");
        chk(alvrl_set_rsamples(it->ctx, it->Rsamples), "alvrl_set_rsamples");
        chk(alvrl_set_strict_rbuild(it->ctx, it->strictRbuild ? 1 : 0), "alvrl_set_strict_rbuild");
        hchk(hipSetDevice(device), "hipSetDevice");
        hchk(hipStreamCreateWithFlags(&it->stream, hipStreamNonBlocking), "hipStreamCreate");
        hchk(hipEventCreate(&it->ev_r0), "hipEventCreate");
        hchk(hipEventCreate(&it->ev_r1), "hipEventCreate");
    });
    *out = it.release();
    return ALVRL_OK;
}

ALVRL_API void alvrl_integrator_destroy(alvrl_integrator* it) { delete it; }

ALVRL_API int alvrl_integrator_preprocess(alvrl_integrator* it, const alvrl_scene_desc* s)
{
    if (!it || !s) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_preprocess: null argument");
    GUARD({ hchk(hipSetDevice(it->device), "hipSetDevice"); it->preprocess(*s); });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_preprocess_ext(alvrl_integrator* it, const alvrl_scene_ext* s)
{
    if (!it || !s) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_preprocess_ext: null argument");
    GUARD({ hchk(hipSetDevice(it->device), "hipSetDevice"); it->preprocess_ext(*s); });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_rep_pixels(alvrl_integrator* it, uint32_t pass, uint32_t* pixel_ids, uint32_t cap,
                                          uint32_t* n)
{
    if (!it || !n) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_rep_pixels: null argument");
    GUARD({
        const std::vector<uint32_t> p = it->rep_pixels(pass);
        *n = (uint32_t)p.size();
        if (pixel_ids) {
            if (cap < p.size()) throw IntegError(ALVRL_ERR_INVALID, "alvrl_integrator_rep_pixels: buffer too small");
            std::copy(p.begin(), p.end(), pixel_ids);
        }
    });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_prepass_records(alvrl_integrator* it, uint32_t pass, const alvrl_gather_rec* recs,
                                               const uint32_t* row_of_rec, uint32_t n, uint32_t rank,
                                               uint32_t world, const alvrl_exchange* ex)
{
    if (!it) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_prepass_records: null argument");
    GUARD({
        hchk(hipSetDevice(it->device), "hipSetDevice");
        it->prepass_records(pass, recs, row_of_rec, n, rank, world, ex);
    });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_set_cluster_info(alvrl_integrator* it, uint32_t pass, uint32_t npix,
                                                const uint32_t* p2s, uint32_t nslices, const uint32_t* slice_off,
                                                const uint32_t* reps, const float* weights, uint32_t n_fb,
                                                const uint32_t* fb_reps, const float* fb_weights)
{
    if (!it || (npix && !p2s) || !slice_off || (n_fb && (!fb_reps || !fb_weights)))
        return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_set_cluster_info: null argument");
    const uint32_t nr = slice_off[nslices];
    if (nr && (!reps || !weights)) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_set_cluster_info: null lists");
    GUARD({
        hchk(hipSetDevice(it->device), "hipSetDevice");
        std::vector<uint32_t> a(p2s, p2s + npix), so(slice_off, slice_off + nslices + 1), rp(reps, reps + nr),
            fr(fb_reps, fb_reps + n_fb);
        std::vector<float> w(weights, weights + nr), fw(fb_weights, fb_weights + n_fb);
        it->install_cluster_info(pass, a, so, rp, w, fr, fw);
    });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_prepass(alvrl_integrator* it, uint32_t pass)
{
    if (!it) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_prepass: null argument");
    GUARD({ hchk(hipSetDevice(it->device), "hipSetDevice"); it->prepass(pass); });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_prepass_dist(alvrl_integrator* it, uint32_t pass, uint32_t rank,
                                            uint32_t world, const alvrl_exchange* ex)
{
    if (!it) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_prepass_dist: null argument");
    GUARD({ hchk(hipSetDevice(it->device), "hipSetDevice"); it->prepass(pass, rank, world, ex); });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_render(alvrl_integrator* it, uint32_t rank, uint32_t world, float* d_fb,
                                      void* stream)
{
    if (!it || !d_fb) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_render: null argument");
    GUARD({
        hchk(hipSetDevice(it->device), "hipSetDevice");
        hipStream_t s = stream ? (hipStream_t)stream : it->stream;
        if (!stream) {
            // the integrator's own stream is non-blocking: order it after the
            // caller's work on the null stream (e.g. the frame's zero fill),
            // which it would otherwise race
            hipEvent_t ev = nullptr;
            hchk(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
            hipError_t e = hipEventRecord(ev, nullptr);
            if (e == hipSuccess) e = hipStreamWaitEvent(s, ev, 0);
            (void)hipEventDestroy(ev);
            hchk(e, "order after the null stream");
        }
        it->render(rank, world, d_fb, s);
    });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_set_vrls(alvrl_integrator* it, const float* soa, uint32_t n,
                                        uint64_t particle_count)
{
    if (!it || (!soa && n)) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_set_vrls: null argument");
    if (n && particle_count == 0) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_set_vrls: particle_count must be > 0");
    GUARD({
        it->vrls.n = n;
        it->vrls.particle_count = particle_count;
        it->vrls.soa.assign(soa, soa + 9 * (size_t)n);
        it->vrls_from_file = true;
        it->uploaded_pass = 0xFFFFFFFFu;
    });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_get_stats(alvrl_integrator* it, alvrl_integrator_stats* st)
{
    if (!it || !st) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_get_stats: null argument");
    GUARD({
        uint64_t pre = 0, ren = 0;
        chk(alvrl_get_stats(it->ctx, &pre, &ren), "alvrl_get_stats");
        it->st.contrib_preprocess = pre;
        it->st.contrib_render = ren;
        float ms = 0;
        if (it->render_timed && hipEventSynchronize(it->ev_r1) == hipSuccess &&
            hipEventElapsedTime(&ms, it->ev_r0, it->ev_r1) == hipSuccess)
            it->st.ms_render_kernel = ms;
        *st = it->st;
    });
    return ALVRL_OK;
}

ALVRL_API alvrl_ctx* alvrl_integrator_ctx(alvrl_integrator* it) { return it ? it->ctx : nullptr; }

ALVRL_API int alvrl_integrator_save_cluster_info(alvrl_integrator* it, const char* path)
{
    if (!it || !path) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_save_cluster_info: null argument");
    GUARD({ it->save_cluster_info(path); });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_load_cluster_info(alvrl_integrator* it, const char* path, uint32_t pass)
{
    if (!it || !path) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_load_cluster_info: null argument");
    GUARD({ hchk(hipSetDevice(it->device), "hipSetDevice"); it->load_cluster_info(path, pass); });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_local_slices(alvrl_integrator* it, uint32_t* out, uint32_t cap, uint32_t* n)
{
    if (!it || !n) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_local_slices: null argument");
    *n = (uint32_t)it->local_slices.size();
    if (out && cap < *n) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_local_slices: cap too small");
    if (out) std::copy(it->local_slices.begin(), it->local_slices.end(), out);
    return ALVRL_OK;
}

ALVRL_API uint32_t alvrl_integrator_num_slices(alvrl_integrator* it)
{
    return (it && it->prep) ? it->prep->num_slices() : 0;
}

ALVRL_API int alvrl_integrator_slices(alvrl_integrator* it, uint32_t* p2s, uint32_t n)
{
    if (!it || !p2s) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_slices: null argument");
    if (n < it->pixel_to_slice.size()) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_slices: buffer too small");
    std::copy(it->pixel_to_slice.begin(), it->pixel_to_slice.end(), p2s);
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_reps(alvrl_integrator* it, uint32_t* rep_off, uint32_t* rep_pix, uint32_t cap)
{
    if (!it || !it->prep || !rep_off || !rep_pix) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_reps: no slices");
    const auto& o = it->prep->rep_off();
    const auto& p = it->prep->rep_pix();
    if (cap < p.size()) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_reps: buffer too small");
    std::copy(o.begin(), o.end(), rep_off);
    std::copy(p.begin(), p.end(), rep_pix);
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_clusters(alvrl_integrator* it, uint32_t* slice_off, uint32_t* reps,
                                        float* weights, uint32_t cap, uint32_t* fb_reps, float* fb_w,
                                        uint32_t fb_cap, uint32_t* n_fb)
{
    if (!it || !slice_off || !reps || !weights || !n_fb) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_clusters: null argument");
    if (cap < it->reps.size() || fb_cap < it->fb_reps.size()) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_clusters: buffer too small");
    std::copy(it->slice_off.begin(), it->slice_off.end(), slice_off);
    std::copy(it->reps.begin(), it->reps.end(), reps);
    std::copy(it->weights.begin(), it->weights.end(), weights);
    if (fb_reps) std::copy(it->fb_reps.begin(), it->fb_reps.end(), fb_reps);
    if (fb_w) std::copy(it->fb_w.begin(), it->fb_w.end(), fb_w);
    *n_fb = (uint32_t)it->fb_reps.size();
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_R(alvrl_integrator* it, float* out, uint64_t cap)
{
    if (!it || !out) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_R: null argument");
    const uint64_t need = (uint64_t)2 * it->vrls.n * it->st.rep_rows;
    if (cap < need) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_R: buffer too small");
    if (it->rows_built != it->st.rep_rows)
        return ierr(ALVRL_ERR_STATE, "alvrl_integrator_R: this rank holds R of its own slices only");
    GUARD({
        hchk(hipSetDevice(it->device), "hipSetDevice");
        hchk(hipStreamSynchronize(it->stream), "sync");
        // per-slice [vrl][row] blocks -> one [vrl][rep_rows] matrix
        const auto& ro = it->prep->rep_off();
        const uint64_t nv = it->vrls.n, rows = it->st.rep_rows;
        for (size_t s = 0; need && s + 1 < ro.size(); s++) {
            const uint64_t n = ro[s + 1] - ro[s];
            if (!n) continue;
            hchk(hipMemcpy2D(out + 2 * ro[s], rows * 8, it->Rt.p + 2 * nv * ro[s], n * 8, n * 8, nv,
                             hipMemcpyDeviceToHost), "copy R");
        }
    });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_slice_job(alvrl_integrator* it, uint32_t s, float* R, double* locw, uint32_t cap_rows,
                                         uint32_t* nrows, float* pixel_under, uint32_t* init_vrls,
                                         uint32_t* init_off, uint32_t* ninit)
{
    if (!it || !nrows || !ninit) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_slice_job: null argument");
    const auto k = std::find(it->job_slices.begin(), it->job_slices.end(), s) - it->job_slices.begin();
    if (k == (long)it->job_slices.size())
        return ierr(ALVRL_ERR_STATE, "alvrl_integrator_slice_job: slice not refined on this rank in the last prepass");
    const auto& rows = it->job_rows[k];
    const uint32_t n = (uint32_t)rows.size();
    *nrows = n;
    *ninit = (uint32_t)it->job_init_off.size() - 1;
    // R and locw hold cap_rows rows: refuse before writing anything
    if ((R || locw) && cap_rows < n) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_slice_job: buffer too small");
    if (pixel_under) *pixel_under = it->prep->slice_undersampling()[s];
    if (init_vrls) std::copy(it->job_init.begin(), it->job_init.end(), init_vrls);
    if (init_off) std::copy(it->job_init_off.begin(), it->job_init_off.end(), init_off);
    if (locw) std::copy(it->job_locw[k].begin(), it->job_locw[k].end(), locw);
    if (!R) return ALVRL_OK;
    GUARD({
        hchk(hipSetDevice(it->device), "hipSetDevice");
        hchk(hipStreamSynchronize(it->stream), "sync");
        const uint64_t nv = it->vrls.n;
        // rows that are one contiguous run of a slice block: one 2-D copy
        uint32_t r = 0;
        while (r < n) {
            const uint32_t g = rows[r];
            const uint64_t b = it->row_base[g], st = it->row_stride[g];
            uint32_t q = r + 1;
            while (q < n && it->row_stride[rows[q]] == st && it->row_base[rows[q]] == b + (q - r)) q++;
            hchk(hipMemcpy2D(R + 2 * (uint64_t)r, (uint64_t)n * 8, it->Rt.p + 2 * b, st * 8, (uint64_t)(q - r) * 8,
                             nv, hipMemcpyDeviceToHost), "copy slice R");
            r = q;
        }
    });
    return ALVRL_OK;
}

ALVRL_API int alvrl_integrator_vrls(alvrl_integrator* it, float* soa, uint32_t cap, uint32_t* n, uint64_t* particles)
{
    if (!it || !n || !particles) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_vrls: null argument");
    *n = it->vrls.n;
    *particles = it->vrls.particle_count;
    if (!soa) return ALVRL_OK;
    if (cap < it->vrls.n) return ierr(ALVRL_ERR_INVALID, "alvrl_integrator_vrls: buffer too small");
    for (int pl = 0; pl < 9; pl++)
        std::memcpy(soa + (size_t)pl * cap, it->vrls.soa.data() + (size_t)pl * it->vrls.n, sizeof(float) * it->vrls.n);
    return ALVRL_OK;
}

}  // extern "C"
