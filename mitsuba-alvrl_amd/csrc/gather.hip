// gather.hip -- gfx950 kernels of hot path (a) and the R build of (b).
//
//   k_prepare_vrls     VRL SoA (36 B/VRL, VRL.h:89-96) -> VrlPrep (80 B)
//   k_gather_brute     getVRLContributions, vrlIntegrator.cpp:792-825
//   k_gather_clustered getClusteredVrlContributions, vrlIntegrator.cpp:542-599
//   k_build_R          Rbuilder::run -> getLiLuminanceVrlContributions,
//                      vrlIntegrator.cpp:527-539, 1053-1067
//
// Mapping: a lane owns one eye segment (gather record); a wave walks the VRL
// list in lock step so the VRL index is wave-uniform and VrlPrep arrives in
// SGPRs through the scalar cache (64 pairs share every 80-B VRL fetch).  The
// kernels are VALU/transcendental-bound; HBM traffic per pair is << 1 B.
#include "vrl_device.hpp"

// Resident blocks of 256 per CU the render gathers are compiled for: 4
// (128 VGPRs, four waves per SIMD; a few bytes spilled).  With the two
// samples side by side the compiler's own choice is 139 VGPRs, three waves:
// C2 5.09e10 against 5.18e10 contributions/s at four (profiles/r04/gather_ab.txt).
// Developer A/B: -DALVRL_GATHER_MINB=n, 0 = the compiler's choice.
#ifndef ALVRL_GATHER_MINB
#define ALVRL_GATHER_MINB 4
#endif
#if ALVRL_GATHER_MINB > 0
#define ALVRL_GATHER_BOUNDS __launch_bounds__(256, ALVRL_GATHER_MINB)
#else
#define ALVRL_GATHER_BOUNDS __launch_bounds__(256)
#endif

#ifndef ALVRL_RB_MINB
#define ALVRL_RB_MINB 3   // the R build: three waves per SIMD
#endif

namespace alvrl {

__global__ void __launch_bounds__(256) k_prepare_vrls(const float* __restrict__ soa, uint32_t n,
                                                      VrlPrep* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    VrlPrep p;
    p.sx = soa[0 * (size_t)n + i]; p.sy = soa[1 * (size_t)n + i]; p.sz = soa[2 * (size_t)n + i];
    p.ex = soa[3 * (size_t)n + i]; p.ey = soa[4 * (size_t)n + i]; p.ez = soa[5 * (size_t)n + i];
    p.pr = soa[6 * (size_t)n + i]; p.pg = soa[7 * (size_t)n + i]; p.pb = soa[8 * (size_t)n + i];
    const F3 v = f3(p.ex, p.ey, p.ez) - f3(p.sx, p.sy, p.sz);
    p.vx = v.x; p.vy = v.y; p.vz = v.z;
    const F3 d = nrm(v);
    p.dx = d.x; p.dy = d.y; p.dz = d.z;
    p.len = len(f3(p.sx, p.sy, p.sz) - f3(p.ex, p.ey, p.ez));
    p.c = dot(v, v);
    p.pad0 = p.pad1 = p.pad2 = 0.0f;
    out[i] = p;
}

__device__ __forceinline__ Rec load_rec(const Rec* __restrict__ recs, uint32_t r, bool active)
{
    Rec x;
    if (active) {
        const float4* p = reinterpret_cast<const float4*>(recs + r);
        const float4 a = p[0], b = p[1], c = p[2], d = p[3], e = p[4];
        x.ox = a.x; x.oy = a.y; x.oz = a.z; x.dx = a.w;
        x.dy = b.x; x.dz = b.y; x.px = b.z; x.py = b.w;
        x.pz = c.x; x.nx = c.y; x.ny = c.z; x.nz = c.w;
        x.ar = d.x; x.ag = d.y; x.ab = d.z; x.flags = __float_as_uint(d.w);
        x.wr = e.x; x.wg = e.y; x.wb = e.z; x.depth = __float_as_uint(e.w);
    } else {
        x.ox = x.oy = x.oz = 0.0f; x.dx = 0.0f; x.dy = 0.0f; x.dz = 1.0f;
        x.px = x.py = 0.0f; x.pz = 1.0f; x.nx = x.ny = 0.0f; x.nz = -1.0f;
        x.ar = x.ag = x.ab = 0.0f; x.flags = 0u;
        x.wr = x.wg = x.wb = 1.0f; x.depth = 0u;
    }
    return x;
}

__device__ __forceinline__ void count_pairs(unsigned long long* counter, bool lane_counts,
                                            uint32_t per_lane)
{
    const unsigned long long m = __ballot(lane_counts);
    if ((threadIdx.x & 63) == 0 && m)
        atomicAdd(counter, (unsigned long long)__popcll(m) * per_lane);
}

template <int NVV, int NVS, bool VIS = false>
__global__ void ALVRL_GATHER_BOUNDS k_gather_brute(const Rec* __restrict__ recs,
                                                      const uint32_t* __restrict__ ids, uint32_t nrec,
                                                      const VrlPrep* __restrict__ vp, uint32_t nvrl,
                                                      DevParams P, float normalization,
                                                      float* __restrict__ out,
                                                      unsigned long long* counter)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = r < nrec;
    const Rec rec = load_rec(recs, r, active);
    const RecPre q = prepare_record(rec, P);
    const uint32_t rid = active ? (ids ? ids[r] : r) : 0u;
    float L0 = 0.0f, L1 = 0.0f, L2 = 0.0f;
    if (q.medium) {
        for (uint32_t v = 0; v < nvrl; ++v) {
            const VrlPrep V = vp[v];
            float c[3], m, s;
            integrate_vrl<NVV, NVS, false, VIS>(P, q, V, rid, v, kDomGather, P.nvv, P.nvs, c, &m, &s);
            // vrlContribution *= normalization; Li += vrlContribution (:810, 815)
            L0 += c[0] * normalization; L1 += c[1] * normalization; L2 += c[2] * normalization;
        }
        // the segment's path weight (integrateVRL's 'weight', :668 / :743)
        if (!q.unit) { L0 *= q.w[0]; L1 *= q.w[1]; L2 *= q.w[2]; }
    }
    count_pairs(counter, active && q.medium, nvrl);
    if (active) {
        out[3 * (size_t)r + 0] = L0; out[3 * (size_t)r + 1] = L1; out[3 * (size_t)r + 2] = L2;
    }
}

struct WorkItem { uint32_t slice, begin, count, pad; };

// One pair's colour for the clustered gathers.  The one-wave-per-item kernel
// and the split form of small host batches (k_gather_split_pairs) inline it
// into different loops; this file is built with -ffp-contract=on (a*b+c fused
// only within one source expression, Makefile GATHERFLAGS), so its roundings
// do not depend on the surrounding code and a record's result does not
// depend on which form its batch took (tests/test_gpu_boundary.py).
template <int NVV, int NVS, bool VIS>
__device__ __forceinline__ float3 pair_colour(const DevParams& P, const RecPre& q, const VrlPrep& V, uint32_t rid,
                                           uint32_t v)
{
    float c[3], m, s;
    integrate_vrl<NVV, NVS, false, VIS>(P, q, V, rid, v, kDomGather, P.nvv, P.nvs, c, &m, &s);
    return make_float3(c[0], c[1], c[2]);
}

template <int NVV, int NVS, bool VIS>
__device__ __forceinline__ void gather_item(const Rec* __restrict__ recs, const uint32_t* __restrict__ ids,
                                            const WorkItem& it, const uint32_t* lr, const float* lw, uint32_t k,
                                            const VrlPrep* __restrict__ vp, const DevParams& P, float inv_pc,
                                            float* __restrict__ out, unsigned long long* counter);

template <int NVV, int NVS, bool VIS = false>
__global__ void ALVRL_GATHER_BOUNDS k_gather_clustered(
    const Rec* __restrict__ recs, const uint32_t* __restrict__ ids,
    const WorkItem* __restrict__ items, uint32_t nitems, const VrlPrep* __restrict__ vp,
    const uint32_t* __restrict__ slice_off, const uint32_t* __restrict__ reps,
    const float* __restrict__ weights, const uint32_t* __restrict__ fb_reps,
    const float* __restrict__ fb_w, uint32_t n_fb, DevParams P, float inv_pc,
    float* __restrict__ out, unsigned long long* counter)
{
    const uint32_t item = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (item >= nitems) return;
    const WorkItem it = items[item];
    const uint32_t* lr;
    const float* lw;
    uint32_t k;
    if (it.slice == 0xFFFFFFFFu) { lr = fb_reps; lw = fb_w; k = n_fb; }
    else { const uint32_t b = slice_off[it.slice]; lr = reps + b; lw = weights + b; k = slice_off[it.slice + 1] - b; }
    gather_item<NVV, NVS, VIS>(recs, ids, it, lr, lw, k, vp, P, inv_pc, out, counter);
}

// One work item (<= 64 pixels of one slice, a lane each) over a
// representative list: Li = sum_i w_i * integrateVRL(rep_i) / particleCount.
template <int NVV, int NVS, bool VIS>
__device__ __forceinline__ void gather_item(const Rec* __restrict__ recs, const uint32_t* __restrict__ ids,
                                            const WorkItem& it, const uint32_t* lr, const float* lw, uint32_t k,
                                            const VrlPrep* __restrict__ vp, const DevParams& P, float inv_pc,
                                            float* __restrict__ out, unsigned long long* counter)
{
    const uint32_t lane = threadIdx.x & 63;
    const bool active = lane < it.count;
    const uint32_t r = it.begin + lane;
    const Rec rec = load_rec(recs, r, active);
    const RecPre q = prepare_record(rec, P);
    const uint32_t rid = active ? (ids ? ids[r] : r) : 0u;
    float L0 = 0.0f, L1 = 0.0f, L2 = 0.0f;
    if (q.medium) {
        for (uint32_t i = 0; i < k; ++i) {
            const uint32_t v = lr[i];
            const float w = lw[i];
            const VrlPrep V = vp[v];
            const float3 c = pair_colour<NVV, NVS, VIS>(P, q, V, rid, v);
            // Li += weights->at(i) * integrateVRL(...)  (:587-589)
            L0 += c.x * w; L1 += c.y * w; L2 += c.z * w;
        }
        // Li /= particleCount (:590); return Li * weight (:598)
        L0 *= inv_pc; L1 *= inv_pc; L2 *= inv_pc;
        if (!q.unit) { L0 *= q.w[0]; L1 *= q.w[1]; L2 *= q.w[2]; }
    }
    count_pairs(counter, active && q.medium, k);
    if (active) {
        out[3 * (size_t)r + 0] = L0; out[3 * (size_t)r + 1] = L1; out[3 * (size_t)r + 2] = L2;
    }
}

// Small launches (the plugin's records mode: renderBlock-sized host calls,
// a few hundred work items) leave most of the 4,096 wave slots of the chip
// idle while each item's wave walks its whole representative list.  The split
// form gives every chunk of a list its own wave: k_gather_split_pairs stores
// each pair's integrateVRL colour (the same inlined code as gather_item), and
// k_gather_split_sum adds them in list order with gather_item's own
// accumulation expression, so a record gets the same bits either way
// (tests/test_gpu_boundary.py).  Pair colours: item j's block at
// cbuf[base[j] ...], entry (i * 3 + channel) * 64 + lane.
struct SplitUnit { uint32_t item, first; };

template <int NVV, int NVS, bool VIS>
__global__ void ALVRL_GATHER_BOUNDS k_gather_split_pairs(
    const Rec* __restrict__ recs, const uint32_t* __restrict__ ids, const WorkItem* __restrict__ items,
    const SplitUnit* __restrict__ units, uint32_t nunits, uint32_t chunk, const VrlPrep* __restrict__ vp,
    const uint32_t* __restrict__ slice_off, const uint32_t* __restrict__ reps, const uint32_t* __restrict__ fb_reps,
    uint32_t n_fb, DevParams P, const uint64_t* __restrict__ base, float* __restrict__ cbuf)
{
    const uint32_t unit = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (unit >= nunits) return;
    const SplitUnit u = units[unit];
    const WorkItem it = items[u.item];
    const uint32_t* lr;
    uint32_t k;
    if (it.slice == 0xFFFFFFFFu) { lr = fb_reps; k = n_fb; }
    else { const uint32_t b = slice_off[it.slice]; lr = reps + b; k = slice_off[it.slice + 1] - b; }
    const uint32_t lane = threadIdx.x & 63;
    const bool active = lane < it.count;
    const uint32_t r = it.begin + lane;
    const Rec rec = load_rec(recs, r, active);
    const RecPre q = prepare_record(rec, P);
    const uint32_t rid = active ? (ids ? ids[r] : r) : 0u;
    float* __restrict__ cb = cbuf + base[u.item] + lane;
    const uint32_t end = min(k, u.first + chunk);
    if (q.medium) {
        for (uint32_t i = u.first; i < end; ++i) {
            const uint32_t v = lr[i];
            const VrlPrep V = vp[v];
            const float3 c = pair_colour<NVV, NVS, VIS>(P, q, V, rid, v);
            cb[(size_t)(3 * i + 0) * 64] = c.x;
            cb[(size_t)(3 * i + 1) * 64] = c.y;
            cb[(size_t)(3 * i + 2) * 64] = c.z;
        }
    }
}

__global__ void __launch_bounds__(256) k_gather_split_sum(
    const Rec* __restrict__ recs, const WorkItem* __restrict__ items, uint32_t nitems,
    const uint32_t* __restrict__ slice_off, const float* __restrict__ weights, const float* __restrict__ fb_w,
    uint32_t n_fb, DevParams P, float inv_pc, const uint64_t* __restrict__ base, const float* __restrict__ cbuf,
    float* __restrict__ out, unsigned long long* counter)
{
    const uint32_t item = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (item >= nitems) return;
    const WorkItem it = items[item];
    const float* lw;
    uint32_t k;
    if (it.slice == 0xFFFFFFFFu) { lw = fb_w; k = n_fb; }
    else { const uint32_t b = slice_off[it.slice]; lw = weights + b; k = slice_off[it.slice + 1] - b; }
    const uint32_t lane = threadIdx.x & 63;
    const bool active = lane < it.count;
    const uint32_t r = it.begin + lane;
    const Rec rec = load_rec(recs, r, active);
    const RecPre q = prepare_record(rec, P);
    const float* __restrict__ cb = cbuf + base[item] + lane;
    float L0 = 0.0f, L1 = 0.0f, L2 = 0.0f;
    if (q.medium) {
        for (uint32_t i = 0; i < k; ++i) {
            const float w = lw[i];
            const float c0 = cb[(size_t)(3 * i + 0) * 64], c1 = cb[(size_t)(3 * i + 1) * 64],
                        c2 = cb[(size_t)(3 * i + 2) * 64];
            // as gather_item: Li += weights->at(i) * integrateVRL(...)  (:587-589)
            L0 += c0 * w; L1 += c1 * w; L2 += c2 * w;
        }
        L0 *= inv_pc; L1 *= inv_pc; L2 *= inv_pc;
        if (!q.unit) { L0 *= q.w[0]; L1 *= q.w[1]; L2 *= q.w[2]; }
    }
    count_pairs(counter, active && q.medium, k);
    if (active) {
        out[3 * (size_t)r + 0] = L0; out[3 * (size_t)r + 1] = L1; out[3 * (size_t)r + 2] = L2;
    }
}

// The debug images of LiInternal for a primary ray (weight 1): numVrlFalseColor
// gives |list| / N (clustered, :574-575) or 1 (brute, :800-801) where the
// medium scatters, 0 elsewhere; slicesFalseColor (clustered only) colours the
// slice with the integer hash of :578-583 (grey for the fall-back list), also
// outside the medium (:546).  The stats counter gets the list size, as there.
// items == nullptr: one record per lane (brute).
__global__ void __launch_bounds__(256) k_false_color(const Rec* __restrict__ recs,
                                                     const WorkItem* __restrict__ items, uint32_t n,
                                                     int mode, const uint32_t* __restrict__ slice_off,
                                                     uint32_t n_fb, uint32_t nvrl, float* __restrict__ out,
                                                     unsigned long long* counter)
{
    uint32_t r, k, slice = 0xFFFFFFFFu;
    bool active;
    if (items) {
        const uint32_t item = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
        if (item >= n) return;
        const WorkItem it = items[item];
        const uint32_t lane = threadIdx.x & 63;
        active = lane < it.count;
        r = it.begin + lane;
        slice = it.slice;
        k = slice == 0xFFFFFFFFu ? n_fb : slice_off[slice + 1] - slice_off[slice];
    } else {
        r = blockIdx.x * blockDim.x + threadIdx.x;
        active = r < n;
        k = nvrl;
    }
    const bool medium = active && (__float_as_uint(reinterpret_cast<const float4*>(recs + (active ? r : 0))[3].w) & 4u);
    float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f;
    if (mode == 1) {
        if (medium) c0 = c1 = c2 = items ? (float)k / (float)nvrl : 1.0f;
    } else if (slice == 0xFFFFFFFFu) {
        c0 = c1 = c2 = 0.5f;
    } else {
        const uint32_t s = slice;
        c0 = (float)((double)((s + s * s) % 43u) / 43.0);
        c1 = (float)((double)((7u * s + 2u * s * s + 7u) % 41u) / 41.0);
        c2 = (float)((double)((23u * s + 5u * s * s + s * s * s + 17u) % 53u) / 53.0);
    }
    count_pairs(counter, mode == 1 ? medium : active, k);
    if (active) { out[3 * (size_t)r + 0] = c0; out[3 * (size_t)r + 1] = c1; out[3 * (size_t)r + 2] = c2; }
}

hipError_t launch_false_color(const Rec* recs, const WorkItem* items, uint32_t n, int mode,
                              const uint32_t* slice_off, uint32_t n_fb, uint32_t nvrl, float* out,
                              unsigned long long* counter, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    const dim3 grid(items ? (n + 3) / 4 : (n + 255) / 256), block(256);
    hipLaunchKernelGGL(k_false_color, grid, block, 0, s, recs, items, n, mode, slice_off, n_fb, nvrl, out, counter);
    return hipGetLastError();
}

// R build: lane = representative row, the block's 4 waves interleave over a
// VRL chunk.  Writes Rt[v][row0 + r] = (mean * norm, var * norm * norm).
template <int NVV, int NVS, bool VIS = false>
__global__ void __launch_bounds__(256, ALVRL_RB_MINB) k_build_R(const Rec* __restrict__ recs,
                                                 const uint32_t* __restrict__ ids, uint32_t nrows,
                                                 const VrlPrep* __restrict__ vp, uint32_t nvrl,
                                                 uint32_t chunk, DevParams P, float normalization,
                                                 float2* __restrict__ Rt, uint64_t ld, uint64_t row0,
                                                 unsigned long long* counter)
{
    const uint32_t r = blockIdx.x * 64 + (threadIdx.x & 63);
    const uint32_t wave = threadIdx.x >> 6;
    const bool active = r < nrows;
    const Rec rec = load_rec(recs, r, active);
    const RecPre q = prepare_record(rec, P);
    const uint32_t rid = active ? (ids ? ids[r] : r) : 0u;
    const uint32_t v0 = blockIdx.y * chunk;
    const uint32_t v1 = min(nvrl, v0 + chunk);
    const int nsamp = P.rsamples > 1 ? P.rsamples : 1;
    uint32_t done = 0;
    for (uint32_t v = v0 + wave; v < v1; v += 4) {
        float mean = 0.0f, var = 0.0f;
        if (q.medium) {
            const VrlPrep V = vp[v];
            float c[3];
            if (nsamp == 1) {
                integrate_vrl<NVV, NVS, true, VIS>(P, q, V, rid, v, kDomRbuild, P.nvv, P.nvs, c, &mean, &var);
                mean = mean * normalization;
                var = var * normalization * normalization;
            } else {
                // LiInternal's samples loop: entries are sums over the samples (:812-813)
                for (int si = 0; si < nsamp; si++) {
                    float m, s2;
                    integrate_vrl<NVV, NVS, true, VIS>(P, q, V, rid, v, kDomRbuild, P.nvv, P.nvs, c, &m, &s2,
                                                  (uint32_t)si);
                    mean += m * normalization;
                    var += s2 * normalization * normalization;
                }
            }
        }
        if (active) {
            float2* e = &Rt[(size_t)v * ld + row0 + r];
            if (rec.flags & kRecAccum) { const float2 o = *e; *e = make_float2(o.x + mean, o.y + var); }
            else *e = make_float2(mean, var);
        }
        ++done;
    }
    count_pairs(counter, active && q.medium, done * (uint32_t)nsamp);
}

// The same over per-slice blocks: row r of the launch lives at float2 index
// roff[r] + v * rstride[r].  Lanes of a wave are consecutive rows of one
// block except across slice boundaries, so the stores stay coalesced.  The
// non-zero column test of Preprocessor::cluster rides along: one ballot per
// (wave, VRL), one byte store when a mean is non-zero.
template <int NVV, int NVS, bool VIS = false>
// Three waves per SIMD (<= 168 VGPRs): the R build's one long FP32 chain per
// pair hides more latency than at two (179 VGPRs, 45.2 -> 40.3 ms at C4);
// four (128 VGPRs) spill and lose (49.3 ms)
__global__ void __launch_bounds__(256, ALVRL_RB_MINB) k_build_R_blocks(const Rec* __restrict__ recs,
                                                        const uint32_t* __restrict__ ids, uint32_t nrows,
                                                        const VrlPrep* __restrict__ vp, uint32_t nvrl,
                                                        uint32_t chunk, DevParams P, float normalization,
                                                        float2* __restrict__ Rt,
                                                        const uint64_t* __restrict__ roff,
                                                        const uint32_t* __restrict__ rstride,
                                                        uint8_t* __restrict__ nonzero,
                                                        unsigned long long* counter)
{
    const uint32_t r = blockIdx.x * 64 + (threadIdx.x & 63);
    const uint32_t wave = threadIdx.x >> 6;
    const bool active = r < nrows;
    const Rec rec = load_rec(recs, r, active);
    const RecPre q = prepare_record(rec, P);
    const uint32_t rid = active ? (ids ? ids[r] : r) : 0u;
    const uint64_t base = active ? roff[r] : 0;
    const uint64_t stride = active ? rstride[r] : 0;
    const uint32_t v0 = blockIdx.y * chunk;
    const uint32_t v1 = min(nvrl, v0 + chunk);
    const int nsamp = P.rsamples > 1 ? P.rsamples : 1;
    uint32_t done = 0;
    for (uint32_t v = v0 + wave; v < v1; v += 4) {
        float mean = 0.0f, var = 0.0f;
        if (q.medium) {
            const VrlPrep V = vp[v];
            float c[3];
            if (nsamp == 1) {
                integrate_vrl<NVV, NVS, true, VIS>(P, q, V, rid, v, kDomRbuild, P.nvv, P.nvs, c, &mean, &var);
                mean = mean * normalization;
                var = var * normalization * normalization;
            } else {
                // LiInternal's samples loop: entries are sums over the samples (:812-813)
                for (int si = 0; si < nsamp; si++) {
                    float m, s2;
                    integrate_vrl<NVV, NVS, true, VIS>(P, q, V, rid, v, kDomRbuild, P.nvv, P.nvs, c, &m, &s2,
                                                  (uint32_t)si);
                    mean += m * normalization;
                    var += s2 * normalization * normalization;
                }
            }
        }
        if (active) {
            float2* e = &Rt[base + (uint64_t)v * stride];
            if (rec.flags & kRecAccum) { const float2 o = *e; *e = make_float2(o.x + mean, o.y + var); }
            else *e = make_float2(mean, var);
        }
        if (nonzero && __ballot(active && mean != 0.0f) && (threadIdx.x & 63) == 0) nonzero[v] = 1;
        ++done;
    }
    count_pairs(counter, active && q.medium, done * (uint32_t)nsamp);
}

// Preprocessor::cluster's totalVrlContribution != 0 (means are >= 0): one
// wave per VRL column, rows contiguous.
__global__ void __launch_bounds__(256) k_nonzero_columns(const float2* __restrict__ Rt, uint64_t ld,
                                                         uint32_t nrows, uint32_t nvrl,
                                                         uint8_t* __restrict__ mask)
{
    const uint32_t v = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= nvrl) return;
    const float2* col = Rt + (size_t)v * ld;
    bool nz = false;
    for (uint32_t r = threadIdx.x & 63; r < nrows; r += 64) nz |= col[r].x != 0.0f;
    const unsigned long long b = __ballot(nz);
    if ((threadIdx.x & 63) == 0) mask[v] = b ? 1 : 0;
}

__global__ void __launch_bounds__(256) k_accumulate_rgb(const float* __restrict__ rgb,
                                                        const uint32_t* __restrict__ pix, uint32_t n,
                                                        float* __restrict__ fb)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const size_t p = (size_t)pix[r] * 3;
    fb[p + 0] += rgb[3 * (size_t)r + 0];
    fb[p + 1] += rgb[3 * (size_t)r + 1];
    fb[p + 2] += rgb[3 * (size_t)r + 2];
}

hipError_t launch_nonzero_columns(const float2* Rt, uint64_t ld, uint32_t nrows, uint32_t nvrl,
                                  uint8_t* mask, hipStream_t s)
{
    if (nvrl == 0) return hipSuccess;
    hipLaunchKernelGGL(k_nonzero_columns, dim3((nvrl + 3) / 4), dim3(256), 0, s, Rt, ld, nrows, nvrl, mask);
    return hipGetLastError();
}

hipError_t launch_accumulate_rgb(const float* rgb, const uint32_t* pix, uint32_t n, float* fb, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_accumulate_rgb, dim3((n + 255) / 256), dim3(256), 0, s, rgb, pix, n, fb);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// host-side launchers (called from capi.cpp)
// ---------------------------------------------------------------------------
hipError_t launch_prepare_vrls(const float* soa, uint32_t n, VrlPrep* out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prepare_vrls, dim3((n + 255) / 256), dim3(256), 0, s, soa, n, out);
    return hipGetLastError();
}

hipError_t launch_gather_brute(const Rec* recs, const uint32_t* ids, uint32_t nrec,
                               const VrlPrep* vp, uint32_t nvrl, const DevParams& P,
                               float normalization, float* out, unsigned long long* counter,
                               hipStream_t s)
{
    if (nrec == 0) return hipSuccess;
    const dim3 grid((nrec + 255) / 256), block(256);
    if (P.occ.ntri)   // occluders: shadow tests (generic sample counts only)
        hipLaunchKernelGGL((k_gather_brute<-1, -1, true>), grid, block, 0, s, recs, ids, nrec, vp, nvrl, P, normalization, out, counter);
    else if (P.nvv == 2 && P.nvs == 2 && P.strategy == 0)   // unrolled, 'balance' only
        hipLaunchKernelGGL((k_gather_brute<2, 2>), grid, block, 0, s, recs, ids, nrec, vp, nvrl, P,
                           normalization, out, counter);
    else
        hipLaunchKernelGGL((k_gather_brute<-1, -1>), grid, block, 0, s, recs, ids, nrec, vp, nvrl,
                           P, normalization, out, counter);
    return hipGetLastError();
}

hipError_t launch_gather_clustered(const Rec* recs, const uint32_t* ids, const WorkItem* items,
                                   uint32_t nitems, const VrlPrep* vp, const uint32_t* slice_off,
                                   const uint32_t* reps, const float* weights,
                                   const uint32_t* fb_reps, const float* fb_w, uint32_t n_fb,
                                   const DevParams& P, float inv_pc, float* out,
                                   unsigned long long* counter, hipStream_t s)
{
    if (nitems == 0) return hipSuccess;
    const dim3 grid((nitems + 3) / 4), block(256);
    if (P.occ.ntri)   // occluders: shadow tests (generic sample counts only)
        hipLaunchKernelGGL((k_gather_clustered<-1, -1, true>), grid, block, 0, s, recs, ids, items, nitems, vp, slice_off, reps, weights, fb_reps, fb_w, n_fb, P, inv_pc, out, counter);
    else if (P.nvv == 2 && P.nvs == 2 && P.strategy == 0)   // unrolled, 'balance' only
        hipLaunchKernelGGL((k_gather_clustered<2, 2>), grid, block, 0, s, recs, ids, items, nitems,
                           vp, slice_off, reps, weights, fb_reps, fb_w, n_fb, P, inv_pc, out,
                           counter);
    else
        hipLaunchKernelGGL((k_gather_clustered<-1, -1>), grid, block, 0, s, recs, ids, items,
                           nitems, vp, slice_off, reps, weights, fb_reps, fb_w, n_fb, P, inv_pc,
                           out, counter);
    return hipGetLastError();
}

hipError_t launch_gather_clustered_split(const Rec* recs, const uint32_t* ids, const WorkItem* items,
                                         uint32_t nitems, const SplitUnit* units, uint32_t nunits, uint32_t chunk,
                                         const uint64_t* base, float* cbuf, const VrlPrep* vp,
                                         const uint32_t* slice_off, const uint32_t* reps, const float* weights,
                                         const uint32_t* fb_reps, const float* fb_w, uint32_t n_fb,
                                         const DevParams& P, float inv_pc, float* out,
                                         unsigned long long* counter, hipStream_t s)
{
    if (nitems == 0) return hipSuccess;
    if (nunits) {
        const dim3 grid((nunits + 3) / 4), block(256);
        if (P.occ.ntri)
            hipLaunchKernelGGL((k_gather_split_pairs<-1, -1, true>), grid, block, 0, s, recs, ids, items, units, nunits,
                               chunk, vp, slice_off, reps, fb_reps, n_fb, P, base, cbuf);
        else if (P.nvv == 2 && P.nvs == 2 && P.strategy == 0)
            hipLaunchKernelGGL((k_gather_split_pairs<2, 2, false>), grid, block, 0, s, recs, ids, items, units, nunits,
                               chunk, vp, slice_off, reps, fb_reps, n_fb, P, base, cbuf);
        else
            hipLaunchKernelGGL((k_gather_split_pairs<-1, -1, false>), grid, block, 0, s, recs, ids, items, units,
                               nunits, chunk, vp, slice_off, reps, fb_reps, n_fb, P, base, cbuf);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_gather_split_sum, dim3((nitems + 3) / 4), dim3(256), 0, s, recs, items, nitems, slice_off,
                       weights, fb_w, n_fb, P, inv_pc, base, cbuf, out, counter);
    return hipGetLastError();
}

hipError_t launch_build_R(const Rec* recs, const uint32_t* ids, uint32_t nrows, const VrlPrep* vp,
                          uint32_t nvrl, const DevParams& P, float normalization, float2* Rt,
                          uint64_t ld, uint64_t row0, unsigned long long* counter, hipStream_t s)
{
    if (nrows == 0 || nvrl == 0) return hipSuccess;
    const uint32_t chunk = 256;
    const dim3 grid((nrows + 63) / 64, (nvrl + chunk - 1) / chunk), block(256);
    if (P.occ.ntri)   // occluders: shadow tests (generic sample counts only)
        hipLaunchKernelGGL((k_build_R<-1, -1, true>), grid, block, 0, s, recs, ids, nrows, vp, nvrl, chunk, P, normalization, Rt, ld, row0, counter);
    else if (P.nvv == 2 && P.nvs == 2 && P.strategy == 0)   // unrolled, 'balance' only
        hipLaunchKernelGGL((k_build_R<2, 2>), grid, block, 0, s, recs, ids, nrows, vp, nvrl, chunk,
                           P, normalization, Rt, ld, row0, counter);
    else
        hipLaunchKernelGGL((k_build_R<-1, -1>), grid, block, 0, s, recs, ids, nrows, vp, nvrl,
                           chunk, P, normalization, Rt, ld, row0, counter);
    return hipGetLastError();
}

hipError_t launch_build_R_blocks(const Rec* recs, const uint32_t* ids, uint32_t nrows, const VrlPrep* vp,
                                 uint32_t nvrl, const DevParams& P, float normalization, float2* Rt,
                                 const uint64_t* roff, const uint32_t* rstride, uint8_t* nonzero,
                                 unsigned long long* counter, hipStream_t s)
{
    if (nrows == 0 || nvrl == 0) return hipSuccess;
    const uint32_t chunk = 256;
    const dim3 grid((nrows + 63) / 64, (nvrl + chunk - 1) / chunk), block(256);
    if (P.occ.ntri)   // occluders: shadow tests (generic sample counts only)
        hipLaunchKernelGGL((k_build_R_blocks<-1, -1, true>), grid, block, 0, s, recs, ids, nrows, vp, nvrl, chunk, P, normalization, Rt, roff, rstride, nonzero, counter);
    else if (P.nvv == 2 && P.nvs == 2 && P.strategy == 0)   // unrolled, 'balance' only
        hipLaunchKernelGGL((k_build_R_blocks<2, 2>), grid, block, 0, s, recs, ids, nrows, vp, nvrl, chunk,
                           P, normalization, Rt, roff, rstride, nonzero, counter);
    else
        hipLaunchKernelGGL((k_build_R_blocks<-1, -1>), grid, block, 0, s, recs, ids, nrows, vp, nvrl,
                           chunk, P, normalization, Rt, roff, rstride, nonzero, counter);
    return hipGetLastError();
}

}  // namespace alvrl
