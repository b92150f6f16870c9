// refine.hip -- LightSlice cluster refinement on gfx950.
//
// Restates class Preprocessor::Clustering (src/integrators/vrl/Preprocessor.cpp:
// 287-720) and its helpers (calculateColumnWeigths :985-1008,
// calculateUnclusteredVariance :1022-1048, calculateClusterVariance
// :1058-1120, weightedSample :1534-1580) as ONE persistent workgroup per
// clustering job (a slice's local matrix L_i, or the fall-back matrix).
//
// Work decomposition inside a job (8 waves):
//  * the best-first control flow (priority queue, singleton list, snapshot /
//    restore, convergence constants) runs on lane 0 of wave 0, exactly in the
//    reference's order; the heap is std::push_heap/pop_heap's algorithm;
//  * column work (column weights, projections) runs one wave per VRL column,
//    lanes over the local-matrix rows, with the deterministic wave order that
//    oracle/alvrl_preproc.c uses (lane l sums rows l, l+64, ...; halving tree);
//  * the forward / reverse cluster-variance recurrences (:1075-1109) are
//    sequential along the cluster and parallel over rows (one lane per row),
//    processed in chunks of 64 prefixes; the per-prefix inner products over
//    rows are again one wave each;
//  * the projection sort is a bitonic sort in LDS (<= 4096 keys) or a 1-bit
//    LSD split radix sort in global scratch; keys are (orderable float, vrl),
//    unique, so any correct sort reproduces std::sort on std::pair.
// This file is compiled with -ffp-contract=off: every double/float operation
// is the same IEEE operation the oracle performs, so the resulting cluster
// indices and weights are bit-identical to the CPU restatement.
#include "vrl_device.hpp"

#include <string>
#include <vector>

namespace alvrl {

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kChunk = 64;
constexpr int kBitonicMax = 4096;
constexpr uint32_t kDomCluster = 5u;

struct CNode { float uvar, ivar; uint32_t begin, end; };

struct JobDev {
    const uint32_t* rows;
    const double* locw;
    uint32_t nrows;
    float pixel_under, undersampling, depth_correction;
    int do_refine;
    uint32_t stage_refine, stage_sample;
    // workspace (device, sized by the host)
    uint32_t* vrls;
    float* colw;
    CNode* heap;
    CNode* sh_heap;
    uint32_t* singles;
    uint32_t* sh_singles;
    float* dir;
    unsigned long long* keys0;
    unsigned long long* keys1;
    float* fsu; float* fsi; float* feu; float* fei;
    double* st;        // 3 * nrows: sum, M, sumVars
    double* bufM;      // kChunk * nrows
    double* bufV;
    // outputs
    uint32_t* out_reps;
    float* out_w;
    uint32_t* out_n;
    int* out_refined;
    int* out_err;
};

struct Common {
    const float2* Rt;
    uint64_t ld;
    uint32_t nvrl;
    const uint32_t* init_vrls;
    const uint32_t* init_off;
    uint32_t ninit;
    uint32_t seed, pass;
};

struct Ctl {
    float tracingVar, unclIntVar, clUnderVar, clIntVar;
    float sh_clUnderVar, sh_clIntVar;
    int heap_n, sh_heap_n, singles_n, sh_singles_n;
    int err;
    uint32_t b, e, vrl1, vrl2, draw_k;
    int degenerate;
    float diffLen, nd;
    int go, do_snap, stop, refined;
    double Wcur;
    float res_u, res_i;
    float avg;
    // chunk coefficients
    double W[kChunk + 1];
    double w[kChunk];
    double a[kChunk];
    double bb[kChunk];
    uint32_t cv[kChunk];
    // reductions
    float best_v[kWaves];
    uint32_t best_i[kWaves];
    uint32_t cnt[kWaves];
    uint32_t zeros, lo_or, hi_or, lo_and, hi_and;
};

// ------------------------------------------------------------ helpers --
__device__ __forceinline__ double wave_tree_d(double p)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double o = __shfl_down(p, off, 64);
        if (lane < off) p = p + o;
    }
    return p;
}
__device__ __forceinline__ float wave_tree_f(float p)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float o = __shfl_down(p, off, 64);
        if (lane < off) p = p + o;
    }
    return p;
}

__device__ __forceinline__ float Rmean(const Common& cm, uint32_t row, uint32_t v)
{
    return cm.Rt[(size_t)v * cm.ld + row].x;
}
__device__ __forceinline__ float2 Rmv(const Common& cm, uint32_t row, uint32_t v)
{
    return cm.Rt[(size_t)v * cm.ld + row];
}

// Sequential stream of one (stage, cluster range) (see oracle smp_t).
struct Smp {
    uint32_t seed, pass, a, b, c, k, blk;
    U4 buf;
    __device__ void init(uint32_t s, uint32_t p, uint32_t a_, uint32_t b_, uint32_t c_)
    {
        seed = s; pass = p; a = a_; b = b_; c = c_; k = 0; blk = 0xFFFFFFFFu;
    }
    __device__ float next()
    {
        const uint32_t bl = k >> 2;
        if (bl != blk) { buf = philox4x32_10(a, b, bl, (kDomCluster << 24) | (c & 0xFFFFFFu), seed, pass); blk = bl; }
        const uint32_t s = k & 3;
        const uint32_t x = s == 0 ? buf.x : (s == 1 ? buf.y : (s == 2 ? buf.z : buf.w));
        ++k;
        return u01(x);
    }
};

__device__ __forceinline__ float draw_at(uint32_t seed, uint32_t pass, uint32_t a, uint32_t b,
                                         uint32_t c, uint32_t k)
{
    const U4 r = philox4x32_10(a, b, k >> 2, (kDomCluster << 24) | (c & 0xFFFFFFu), seed, pass);
    const uint32_t s = k & 3;
    return u01(s == 0 ? r.x : (s == 1 ? r.y : (s == 2 ? r.z : r.w)));
}

// weightedSample (Preprocessor.cpp:1534-1580), single lane.
__device__ uint32_t weighted_sample(const float* w, Smp& smp, float* prob, uint32_t begin,
                                    uint32_t end, const uint32_t* ind, int* err)
{
    if (begin >= end) { *err = 1; return begin; }
    if (end == begin + 1) { if (prob) *prob = 1; return begin; }
    float weightSum = 0.0f;
    for (uint32_t i = begin; i < end; i++) weightSum += w[ind[i]];
    float probability;
    uint32_t idx;
    if (weightSum <= 0) {
        int tries = 0;
        do {
            idx = (uint32_t)((float)begin + smp.next() * (float)(end - begin));
            if (++tries > 1000) { *err = 1; idx = begin; break; }
        } while (idx >= end);
        probability = (float)(1.0 / (double)(end - begin));
    } else {
        const float alpha = smp.next() * weightSum;
        float accum = 0.0f;
        idx = begin;
        for (uint32_t i = begin; i < end; i++) {
            accum += w[ind[i]];
            if (accum >= alpha) { idx = i; break; }
        }
        probability = w[ind[idx]] / weightSum;
    }
    if (prob) *prob = probability;
    return idx;
}

// deterministic Box-Muller x (oracle alvrl_o_det_std_normal_x)
__device__ double det_log(double x)
{
    int e = 0;
    while (x < 0.70710678118654752440) { x = x * 2.0; e--; }
    const double z = (x - 1.0) / (x + 1.0), z2 = z * z;
    double term = z, sum = 0.0;
    for (int k = 1; k <= 41; k += 2) { sum = sum + term / (double)k; term = term * z2; }
    return 2.0 * sum + (double)e * 0.69314718055994530942;
}
__device__ double det_cos(double phi)
{
    const double PI_ = 3.14159265358979323846;
    double x = phi;
    if (x > PI_) x = 2.0 * PI_ - x;
    double sign = 1.0;
    if (x > 0.5 * PI_) { x = PI_ - x; sign = -1.0; }
    const double x2 = x * x;
    double term = 1.0, sum = 0.0;
    for (int k = 0; k < 14; k++) { sum = sum + term; term = -term * x2 / (double)((2 * k + 1) * (2 * k + 2)); }
    return sign * sum;
}
__device__ float det_std_normal_x(float sx, float sy)
{
    const double r = sqrt(-2.0 * det_log(1.0 - (double)sx));
    const double phi = 2.0 * 3.14159265358979323846 * (double)sy;
    return (float)(det_cos(phi) * r);
}

// ------------------------------------------------------------- heap --
__device__ __forceinline__ bool cless(const CNode& a, const CNode& b)
{
    return a.uvar + a.ivar < b.uvar + b.ivar;
}
__device__ void push_heap_(CNode* first, long hole, long top, CNode value)
{
    long parent = (hole - 1) / 2;
    while (hole > top && cless(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}
__device__ void adjust_heap(CNode* first, long hole, long len, CNode value)
{
    const long top = hole;
    long second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (cless(first[second], first[second - 1])) second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    push_heap_(first, hole, top, value);
}

// lane-0-only Clustering::addCluster (:549-579)
__device__ void add_cluster(const JobDev& J, Ctl& C, uint32_t begin, uint32_t end, float uvar, float ivar)
{
    if (end == begin) { C.err = 1; return; }
    if (end == begin + 1) {
        J.singles[C.singles_n++] = J.vrls[begin];
        if (uvar != 0) C.err = 1;
        C.clIntVar += ivar;
    } else {
        CNode cn{uvar, ivar, begin, end};
        J.heap[C.heap_n++] = cn;
        push_heap_(J.heap, C.heap_n - 1, 0, cn);
        C.clUnderVar += uvar;
        C.clIntVar += ivar;
    }
}
__device__ CNode pop_multi(const JobDev& J, Ctl& C)
{
    const CNode top = J.heap[0];
    if (C.heap_n > 1) {
        const long last = C.heap_n - 1;
        const CNode value = J.heap[last];
        J.heap[last] = J.heap[0];
        adjust_heap(J.heap, 0, last, value);
    }
    C.heap_n--;
    C.clUnderVar -= top.uvar;
    C.clIntVar -= top.ivar;
    return top;
}

__device__ __forceinline__ uint32_t n_clusters(const Ctl& C) { return (uint32_t)(C.singles_n + C.heap_n); }
__device__ __forceinline__ float unclustered_var(const Ctl& C) { return C.tracingVar + C.unclIntVar; }
__device__ __forceinline__ float clustered_var(const Ctl& C) { return C.tracingVar + C.clUnderVar + C.clIntVar; }
__device__ float conv_const(Ctl& C, uint32_t nvrl, float pu)
{
    const float c = ((float)nvrl * pu + (float)n_clusters(C)) * clustered_var(C);
    if (!isfinite(c) || c <= 0) C.err = 1;
    return c;
}
__device__ float lower_bound(Ctl& C, uint32_t nvrl, float pu)
{
    const float c = ((float)nvrl * pu + (float)n_clusters(C)) * unclustered_var(C);
    if (!isfinite(c) || c <= 0) C.err = 1;
    return c;
}

// collective snapshot / restore (:686-699)
__device__ void snapshot(const JobDev& J, Ctl& C)
{
    const int nh = C.heap_n, ns = C.singles_n;
    for (int i = threadIdx.x; i < nh; i += kThreads) J.sh_heap[i] = J.heap[i];
    for (int i = threadIdx.x; i < ns; i += kThreads) J.sh_singles[i] = J.singles[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        C.sh_clUnderVar = C.clUnderVar; C.sh_clIntVar = C.clIntVar;
        C.sh_heap_n = nh; C.sh_singles_n = ns;
    }
    __syncthreads();
}
__device__ void restore(const JobDev& J, Ctl& C)
{
    const int nh = C.sh_heap_n, ns = C.sh_singles_n;
    for (int i = threadIdx.x; i < nh; i += kThreads) J.heap[i] = J.sh_heap[i];
    for (int i = threadIdx.x; i < ns; i += kThreads) J.singles[i] = J.sh_singles[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        C.clUnderVar = C.sh_clUnderVar; C.clIntVar = C.sh_clIntVar;
        C.heap_n = nh; C.singles_n = ns;
    }
    __syncthreads();
}

// ------------------------------------------------ variance recurrence --
// calculateClusterVariance over vrls[first + n*step], n in [0, m).  With
// fu/fi: the incremental (prefix) variances are written.  Result in C.res_*.
__device__ void cluster_variance(const JobDev& J, const Common& cm, Ctl& C, const uint32_t* order,
                                 long step, uint32_t m, float* fu, float* fi)
{
    const uint32_t R = J.nrows;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (uint32_t r = tid; r < R; r += kThreads) { J.st[r] = 0.0; J.st[R + r] = 0.0; J.st[2 * R + r] = 0.0; }
    if (tid == 0) C.Wcur = 0.0;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < m; c0 += kChunk) {
        const uint32_t cn = min((uint32_t)kChunk, m - c0);
        if (tid == 0) {
            double W = C.Wcur;
            C.W[0] = W;
            for (uint32_t c = 0; c < cn; c++) {
                const uint32_t vrl = order[(long)(c0 + c) * step];
                const double weight = (double)J.colw[vrl];
                if (!isfinite(weight) || weight <= 0) C.err = 1;
                C.cv[c] = vrl;
                C.w[c] = weight;
                W = W + weight;
                C.W[c + 1] = W;
            }
            C.Wcur = W;
        }
        __syncthreads();
        if (tid < (int)cn) {
            const double nW = C.W[tid + 1], oW = C.W[tid];
            C.a[tid] = (nW * nW) / (oW * oW);
            C.bb[tid] = (1.0 / C.w[tid] + 1.0 / oW);
        }
        __syncthreads();
        for (uint32_t r = tid; r < R; r += kThreads) {
            const uint32_t row = J.rows[r];
            double sum = J.st[r], M = J.st[R + r], V = J.st[2 * R + r];
            for (uint32_t c = 0; c < cn; c++) {
                const float2 mv = Rmv(cm, row, C.cv[c]);
                const double x = (double)mv.x;
                const double tmp = C.w[c] * sum - C.W[c] * x;
                if (c0 + c > 0) M = C.a[c] * M + C.bb[c] * (tmp * tmp);
                V = V + (double)mv.y / C.w[c];
                sum = sum + x;
                if (fu) { J.bufM[(size_t)c * R + r] = M; J.bufV[(size_t)c * R + r] = V; }
            }
            J.st[r] = sum; J.st[R + r] = M; J.st[2 * R + r] = V;
        }
        __syncthreads();
        if (fu) {
            for (uint32_t c = wave; c < cn; c += kWaves) {
                const double Wn = C.W[c + 1];
                double pi = 0.0, pu = 0.0;
                for (uint32_t r = lane; r < R; r += 64) {
                    pi = pi + J.locw[r] * (J.bufV[(size_t)c * R + r] * Wn);
                    pu = pu + J.locw[r] * (J.bufM[(size_t)c * R + r] / Wn);
                }
                pi = wave_tree_d(pi);
                pu = wave_tree_d(pu);
                if (lane == 0) {
                    const uint32_t n = c0 + c;
                    fi[n] = (float)pi;
                    fu[n] = n == 0 ? 0.0f : (float)pu;
                }
            }
            __syncthreads();
        }
    }
    if (fu) {
        if (tid == 0) { C.res_u = fu[m - 1]; C.res_i = fi[m - 1]; }
    } else if (wave == 0) {
        const double W = C.Wcur;
        double pu = 0.0, pi = 0.0;
        for (uint32_t r = lane; r < R; r += 64) {
            pu = pu + J.locw[r] * (J.st[R + r] / W);
            pi = pi + J.locw[r] * (J.st[2 * R + r] * W);
        }
        pu = wave_tree_d(pu);
        pi = wave_tree_d(pi);
        if (lane == 0) { C.res_u = (float)pu; C.res_i = (float)pi; }
    }
    __syncthreads();
    if (tid == 0) {
        if (!isfinite(C.res_u) || C.res_u < 0) C.err = 1;
        if (!isfinite(C.res_i) || C.res_i < 0) C.err = 1;
    }
    __syncthreads();
}

// ------------------------------------------------------------- sort --
__device__ __forceinline__ unsigned long long proj_key(float p, uint32_t vrl)
{
    if (p == 0.0f) p = 0.0f;   // -0 == +0 for std::pair's operator<
    uint32_t u = __float_as_uint(p);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | vrl;
}

// Sorts J.keys0[0..m); returns the buffer holding the result.
__device__ unsigned long long* sort_keys(const JobDev& J, Ctl& C, uint32_t m, unsigned long long* lds)
{
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    if (m <= (uint32_t)kBitonicMax) {
        uint32_t n2 = 1;
        while (n2 < m) n2 <<= 1;
        for (uint32_t i = tid; i < n2; i += kThreads) lds[i] = i < m ? J.keys0[i] : ~0ull;
        __syncthreads();
        for (uint32_t k = 2; k <= n2; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = tid; i < n2; i += kThreads) {
                    const uint32_t ixj = i ^ j;
                    if (ixj > i) {
                        const unsigned long long a = lds[i], b = lds[ixj];
                        const bool up = (i & k) == 0;
                        if ((a > b) == up) { lds[i] = b; lds[ixj] = a; }
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t i = tid; i < m; i += kThreads) J.keys0[i] = lds[i];
        __syncthreads();
        return J.keys0;
    }
    // varying bits
    if (tid == 0) { C.lo_or = 0; C.hi_or = 0; C.lo_and = 0xFFFFFFFFu; C.hi_and = 0xFFFFFFFFu; }
    __syncthreads();
    {
        uint32_t lo_o = 0, hi_o = 0, lo_a = 0xFFFFFFFFu, hi_a = 0xFFFFFFFFu;
        for (uint32_t i = tid; i < m; i += kThreads) {
            const unsigned long long k = J.keys0[i];
            lo_o |= (uint32_t)k; hi_o |= (uint32_t)(k >> 32);
            lo_a &= (uint32_t)k; hi_a &= (uint32_t)(k >> 32);
        }
        atomicOr(&C.lo_or, lo_o); atomicOr(&C.hi_or, hi_o);
        atomicAnd(&C.lo_and, lo_a); atomicAnd(&C.hi_and, hi_a);
    }
    __syncthreads();
    const unsigned long long vary = (((unsigned long long)(C.hi_or ^ C.hi_and)) << 32) |
                                    (unsigned long long)(C.lo_or ^ C.lo_and);
    unsigned long long* src = J.keys0;
    unsigned long long* dst = J.keys1;
    for (int bit = 0; bit < 64; bit++) {
        if (!((vary >> bit) & 1ull)) continue;
        // total zeros
        if (tid == 0) C.zeros = 0;
        __syncthreads();
        uint32_t z = 0;
        for (uint32_t i = tid; i < m; i += kThreads) z += ((src[i] >> bit) & 1ull) ? 0u : 1u;
        atomicAdd(&C.zeros, z);
        __syncthreads();
        const uint32_t zeros = C.zeros;
        uint32_t zbase = 0, obase = zeros;
        for (uint32_t t0 = 0; t0 < m; t0 += kThreads) {
            const uint32_t i = t0 + tid;
            const bool valid = i < m;
            const unsigned long long k = valid ? src[i] : 0ull;
            const bool one = valid && ((k >> bit) & 1ull);
            const bool zero = valid && !one;
            const unsigned long long bz = __ballot(zero), bo = __ballot(one);
            const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
            const uint32_t rz = __popcll(bz & lt), ro = __popcll(bo & lt);
            if (lane == 0) C.cnt[wave] = (uint32_t)__popcll(bz) | ((uint32_t)__popcll(bo) << 16);
            __syncthreads();
            uint32_t pz = 0, po = 0, tz = 0, to = 0;
            for (int w = 0; w < kWaves; w++) {
                const uint32_t cz = C.cnt[w] & 0xFFFFu, co = C.cnt[w] >> 16;
                if (w < wave) { pz += cz; po += co; }
                tz += cz; to += co;
            }
            if (zero) dst[zbase + pz + rz] = k;
            if (one) dst[obase + po + ro] = k;
            zbase += tz; obase += to;
            __syncthreads();
        }
        unsigned long long* t = src; src = dst; dst = t;
    }
    return src;
}

// ------------------------------------------------------------ split --
// Clustering::split (:590-684), collective.
__device__ void split(const JobDev& J, const Common& cm, Ctl& C, uint32_t begin, uint32_t end,
                      unsigned long long* lds)
{
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t m = end - begin;
    const uint32_t R = J.nrows;
    if (tid == 0) {
        Smp smp;
        smp.init(cm.seed, cm.pass, begin, end, J.stage_refine);
        const uint32_t vrl1 = J.vrls[weighted_sample(J.colw, smp, nullptr, begin, end, J.vrls, &C.err)];
        const float weight1 = J.colw[vrl1];
        J.colw[vrl1] = 0.0f;
        const uint32_t vrl2 = J.vrls[weighted_sample(J.colw, smp, nullptr, begin, end, J.vrls, &C.err)];
        J.colw[vrl1] = weight1;
        C.vrl1 = vrl1; C.vrl2 = vrl2; C.draw_k = smp.k;
    }
    __syncthreads();
    const uint32_t vrl1 = C.vrl1, vrl2 = C.vrl2;
    if (wave == 0) {
        float p1 = 0.0f, p2 = 0.0f, pd = 0.0f;
        for (uint32_t r = lane; r < R; r += 64) {
            const float a = Rmean(cm, J.rows[r], vrl1), b = Rmean(cm, J.rows[r], vrl2);
            const float d = b - a;
            const float ua = fabsf(a), ub = fabsf(b), ud = fabsf(d);
            p1 = p1 + ua * ua; p2 = p2 + ub * ub; pd = pd + ud * ud;
        }
        p1 = wave_tree_f(p1); p2 = wave_tree_f(p2); pd = wave_tree_f(pd);
        if (lane == 0) {
            const float l1 = sqrtf(p1), l2 = sqrtf(p2), ld_ = sqrtf(pd);
            C.diffLen = ld_;
            C.degenerate = !(l1 != 0 && l2 != 0 && ld_ != 0);
        }
    }
    __syncthreads();
    if (!C.degenerate) {
        const float dl = C.diffLen;
        for (uint32_t r = tid; r < R; r += kThreads) {
            const float a = Rmean(cm, J.rows[r], vrl1), b = Rmean(cm, J.rows[r], vrl2);
            J.dir[r] = (b - a) / dl;
        }
        __syncthreads();
    } else {
        uint32_t k = C.draw_k;
        while (true) {
            for (uint32_t r = tid; r < R; r += kThreads) {
                const float sx = draw_at(cm.seed, cm.pass, begin, end, J.stage_refine, k + 2 * r);
                const float sy = draw_at(cm.seed, cm.pass, begin, end, J.stage_refine, k + 2 * r + 1);
                J.dir[r] = det_std_normal_x(sx, sy);
            }
            __syncthreads();
            if (wave == 0) {
                float p = 0.0f;
                for (uint32_t r = lane; r < R; r += 64) { const float u = fabsf(J.dir[r]); p = p + u * u; }
                p = wave_tree_f(p);
                if (lane == 0) C.nd = sqrtf(p);
            }
            __syncthreads();
            if (C.nd != 0) break;
            k += 2 * R;
            if (k > C.draw_k + 64u * 2u * R) {   // hang guard (p ~ 2^-23 per retry)
                if (tid == 0) C.err = 1;
                __syncthreads();
                break;
            }
        }
        const float nd = C.nd != 0 ? C.nd : 1.0f;
        for (uint32_t r = tid; r < R; r += kThreads) J.dir[r] = J.dir[r] / nd;
        __syncthreads();
    }
    // projections (:625-640), one wave per column
    for (uint32_t j = wave; j < m; j += kWaves) {
        const uint32_t vrl = J.vrls[begin + j];
        float pn = 0.0f;
        for (uint32_t r = lane; r < R; r += 64) {
            const float a = fabsf(Rmean(cm, J.rows[r], vrl));
            pn = pn + a * a;
        }
        pn = wave_tree_f(pn);
        const float nc = sqrtf(__shfl(pn, 0, 64));
        float proj = 0.0f;
        if (nc != 0) {
            float pp = 0.0f;
            for (uint32_t r = lane; r < R; r += 64) pp = pp + J.dir[r] * (Rmean(cm, J.rows[r], vrl) / nc);
            pp = wave_tree_f(pp);
            proj = pp;
        }
        if (lane == 0) J.keys0[j] = proj_key(proj, vrl);
    }
    __syncthreads();
    const unsigned long long* sorted = sort_keys(J, C, m, lds);
    for (uint32_t i = tid; i < m; i += kThreads) J.vrls[begin + i] = (uint32_t)sorted[i];
    __syncthreads();
    cluster_variance(J, cm, C, J.vrls + begin, 1, m, J.fsu, J.fsi);
    cluster_variance(J, cm, C, J.vrls + end - 1, -1, m, J.feu, J.fei);
    // argmin over split position (:664-675)
    float bv = INFINITY;
    uint32_t bi = 0xFFFFFFFFu;
    for (uint32_t i = 1 + tid; i < m; i += kThreads) {
        const float v = J.fsu[i - 1] + J.fsi[i - 1] + J.feu[m - 1 - i] + J.fei[m - 1 - i];
        if (v < bv) { bv = v; bi = i; }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float ov = __shfl_down(bv, off, 64);
        const uint32_t oi = __shfl_down(bi, off, 64);
        if (lane < off && (ov < bv || (ov == bv && oi < bi))) { bv = ov; bi = oi; }
    }
    if (lane == 0) { C.best_v[wave] = bv; C.best_i[wave] = bi; }
    __syncthreads();
    if (tid == 0) {
        float v = INFINITY;
        uint32_t idx = 0xFFFFFFFFu;
        for (int w = 0; w < kWaves; w++)
            if (C.best_v[w] < v || (C.best_v[w] == v && C.best_i[w] < idx)) { v = C.best_v[w]; idx = C.best_i[w]; }
        if (idx == 0xFFFFFFFFu) {
            C.err = 1;
        } else {
            const uint32_t s = begin + idx;
            add_cluster(J, C, begin, s, J.fsu[idx - 1], J.fsi[idx - 1]);
            add_cluster(J, C, s, end, J.feu[m - 1 - idx], J.fei[m - 1 - idx]);
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------- kernel --
__global__ void __launch_bounds__(kThreads) k_refine(const JobDev* __restrict__ jobs, Common cm)
{
    const JobDev J = jobs[blockIdx.x];
    __shared__ Ctl C;
    __shared__ unsigned long long lds[kBitonicMax];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t N = cm.nvrl, R = J.nrows;
    const uint32_t nv = cm.init_off[cm.ninit];
    if (tid == 0) {
        C.tracingVar = C.unclIntVar = C.clUnderVar = C.clIntVar = 0.0f;
        C.heap_n = C.singles_n = C.sh_heap_n = C.sh_singles_n = 0;
        C.err = 0; C.refined = 1;
    }
    __syncthreads();
    for (uint32_t i = tid; i < nv; i += kThreads) J.vrls[i] = cm.init_vrls[i];
    // calculateColumnWeigths (:985-1008)
    for (uint32_t v = wave; v < N; v += kWaves) {
        double p = 0.0;
        for (uint32_t r = lane; r < R; r += 64) {
            const float2 mv = Rmv(cm, J.rows[r], v);
            const double mean = (double)mv.x, var = (double)mv.y;
            const double x = mean * mean + var;
            p = p + J.locw[r] * x;
        }
        p = wave_tree_d(p);
        if (lane == 0) {
            const float cw = (float)sqrt(p > 0.0 ? p : 0.0);
            J.colw[v] = cw;
            if (!isfinite(cw)) C.err = 1;
        }
    }
    __syncthreads();
    if (tid == 0) {
        float acc = 0.0f;
        for (uint32_t v = 0; v < N; v++) acc += J.colw[v];
        float avg = acc / N;
        if (avg == 0) avg = 1.0f;
        C.avg = avg;
    }
    __syncthreads();
    {
        const float add = C.avg * 1e-2f;
        for (uint32_t v = tid; v < N; v += kThreads) J.colw[v] += add;
    }
    __syncthreads();
    // initial clusters
    for (uint32_t i = 0; i < cm.ninit; i++) {
        const uint32_t b = cm.init_off[i], e = cm.init_off[i + 1];
        if (b == e) { if (tid == 0) C.err = 1; __syncthreads(); continue; }
        cluster_variance(J, cm, C, J.vrls + b, 1, e - b, nullptr, nullptr);
        if (tid == 0) add_cluster(J, C, b, e, C.res_u, C.res_i);
        __syncthreads();
    }
    // calculateUnclusteredVariance (:1022-1048): per-row Welford in m_vrls order
    for (uint32_t r = tid; r < R; r += kThreads) {
        const uint32_t row = J.rows[r];
        double mean = 0.0, M2 = 0.0, sv = 0.0;
        for (uint32_t n = 0; n < nv; n++) {
            const float2 mv = Rmv(cm, row, J.vrls[n]);
            sv = sv + (double)mv.y;
            const double x = (double)mv.x;
            const double delta = x - mean;
            mean = mean + delta / (double)(n + 1);
            M2 = M2 + delta * (x - mean);
        }
        J.st[r] = sv; J.st[R + r] = M2;
    }
    __syncthreads();
    if (wave == 0) {
        double pv = 0.0, pm = 0.0;
        for (uint32_t r = lane; r < R; r += 64) {
            pv = pv + J.locw[r] * J.st[r];
            pm = pm + J.locw[r] * J.st[R + r];
        }
        pv = wave_tree_d(pv);
        pm = wave_tree_d(pm);
        if (lane == 0) {
            if (nv <= 1) C.err = 1;
            C.unclIntVar = (float)pv;
            C.tracingVar = (float)(pm - (double)C.unclIntVar);
        }
    }
    __syncthreads();

    // refine (:380-489)
    if (J.do_refine && !C.err) {
        if (J.undersampling > 0) {
            // refineFixedDepth (:387-399)
            const uint32_t target = (uint32_t)(0.5 + (double)((float)N / J.undersampling));
            while (true) {
                if (tid == 0) {
                    C.go = (n_clusters(C) < target && C.heap_n > 0 && !C.err);
                    if (C.go) { const CNode cn = pop_multi(J, C); C.b = cn.begin; C.e = cn.end; }
                }
                __syncthreads();
                if (!C.go) break;
                split(J, cm, C, C.b, C.e, lds);
            }
        } else {
            // refineAdaptively (:402-489)
            const float dc = J.depth_correction;
            int run = 0;
            if (tid == 0) {
                if (C.heap_n <= 0) { run = 0; }
                else if (unclustered_var(C) == 0) { C.refined = 0; run = 0; }
                else run = 1;
                C.go = run;
            }
            __syncthreads();
            if (C.go) {
                __shared__ float best;
                __shared__ int nsplit, bestN;
                if (tid == 0) { best = conv_const(C, N, J.pixel_under); nsplit = 0; bestN = 0; }
                snapshot(J, C);
                while (true) {
                    if (tid == 0) {
                        C.go = C.heap_n > 0 && !C.err;
                        if (C.go) { const CNode cn = pop_multi(J, C); C.b = cn.begin; C.e = cn.end; }
                    }
                    __syncthreads();
                    if (!C.go) break;
                    split(J, cm, C, C.b, C.e, lds);
                    if (tid == 0) {
                        nsplit++;
                        const float curr = conv_const(C, N, J.pixel_under);
                        C.do_snap = 0;
                        if (curr < best) {
                            if (dc == 1) C.do_snap = 1;
                            best = curr;
                            bestN = nsplit;
                        }
                        C.stop = lower_bound(C, N, J.pixel_under) >= best;
                    }
                    __syncthreads();
                    if (C.do_snap) snapshot(J, C);
                    if (C.stop) break;
                }
                restore(J, C);
                if (dc != 1) {
                    const int corrected = (int)(0.5 + dc * bestN);
                    for (int i = 0; i < corrected; i++) {
                        if (tid == 0) {
                            C.go = C.heap_n > 0 && !C.err;
                            if (C.go) { const CNode cn = pop_multi(J, C); C.b = cn.begin; C.e = cn.end; }
                        }
                        __syncthreads();
                        if (!C.go) break;
                        split(J, cm, C, C.b, C.e, lds);
                    }
                }
            }
        }
    }
    __syncthreads();
    // sampleRepresentatives (:354-378)
    if (tid == 0) {
        const int refined = C.err ? 0 : C.refined;
        uint32_t i = 0;
        if (refined) {
            for (int k = C.singles_n - 1; k >= 0; k--) { J.out_reps[i] = J.singles[k]; J.out_w[i] = 1; i++; }
            for (int k = 0; k < C.heap_n; k++) {
                const CNode cn = J.heap[k];
                Smp smp;
                smp.init(cm.seed, cm.pass, cn.begin, cn.end, J.stage_sample);
                float prob = 1.0f;
                const uint32_t j = weighted_sample(J.colw, smp, &prob, cn.begin, cn.end, J.vrls, &C.err);
                J.out_reps[i] = J.vrls[j];
                J.out_w[i] = 1.0f / prob;
                i++;
            }
        }
        *J.out_n = i;
        *J.out_refined = refined;
        *J.out_err = C.err;
    }
}

// ------------------------------------------------------------- host --
static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

struct HostJob {
    const uint32_t* rows;
    const double* locw;
    uint32_t nrows;
    float pixel_under, undersampling, depth_correction;
    int do_refine;
    uint32_t stage_refine, stage_sample;
};

// Runs every clustering job on the device (one workgroup each) and copies the
// representatives back.  Returns 0 or an ALVRL_ERR_* code with *err set.
int refine_jobs(hipStream_t s, const float* d_Rt, uint64_t ld, uint32_t nvrl, uint32_t seed,
                uint32_t pass, uint32_t njobs, const HostJob* jobs, const uint32_t* init_vrls,
                const uint32_t* init_off, uint32_t ninit, uint32_t* out_off, uint32_t* out_reps,
                float* out_w, int* out_refined, float* ms, std::string* err)
{
    if (ms) *ms = 0.0f;
    out_off[0] = 0;
    if (njobs == 0) return 0;
    const uint32_t nv = init_off[ninit];
    if (nv != nvrl) { *err = "alvrl_refine: initial clusters must cover every VRL exactly once"; return 1; }
    for (uint32_t i = 0; i < ninit; i++)
        if (init_off[i + 1] < init_off[i]) { *err = "alvrl_refine: init_off not monotone"; return 1; }
    {
        std::vector<unsigned char> seen(nvrl, 0);
        for (uint32_t i = 0; i < nv; i++) {
            if (init_vrls[i] >= nvrl || seen[init_vrls[i]]) { *err = "alvrl_refine: initial clusters are not a partition of the VRLs"; return 1; }
            seen[init_vrls[i]] = 1;
        }
    }
    const size_t N = nvrl;
    std::vector<size_t> row_off(njobs), job_off(njobs);
    size_t rows_total = 0;
    for (uint32_t j = 0; j < njobs; j++) {
        if (jobs[j].nrows == 0) { *err = "alvrl_refine: job with no rows"; return 1; }
        row_off[j] = rows_total;
        rows_total += jobs[j].nrows;
    }
    auto job_bytes = [&](uint32_t R) {
        return align_up(N * 4) * 2 + align_up(N * sizeof(CNode)) * 2 + align_up(N * 4) * 2 +
               align_up((size_t)R * 4) + align_up(N * 8) * 2 + align_up(N * 4) * 4 +
               align_up((size_t)3 * R * 8) + align_up((size_t)kChunk * R * 8) * 2 +
               align_up(N * 4) * 2 + align_up(16);
    };
    size_t total = align_up(rows_total * 4) + align_up(rows_total * 8) + align_up((size_t)nv * 4) +
                   align_up((size_t)(ninit + 1) * 4) + align_up((size_t)njobs * sizeof(JobDev));
    for (uint32_t j = 0; j < njobs; j++) { job_off[j] = total; total += job_bytes(jobs[j].nrows); }
    char* arena = nullptr;
    hipError_t e = hipMalloc(&arena, total);
    if (e != hipSuccess) { *err = std::string("alvrl_refine: hipMalloc: ") + hipGetErrorString(e); return 4; }
    size_t o = 0;
    uint32_t* d_rows = (uint32_t*)(arena + o); o += align_up(rows_total * 4);
    double* d_locw = (double*)(arena + o); o += align_up(rows_total * 8);
    uint32_t* d_init = (uint32_t*)(arena + o); o += align_up((size_t)nv * 4);
    uint32_t* d_init_off = (uint32_t*)(arena + o); o += align_up((size_t)(ninit + 1) * 4);
    JobDev* d_jobs = (JobDev*)(arena + o);
    std::vector<uint32_t> h_rows(rows_total);
    std::vector<double> h_locw(rows_total);
    std::vector<JobDev> h_jobs(njobs);
    for (uint32_t j = 0; j < njobs; j++) {
        const HostJob& H = jobs[j];
        for (uint32_t r = 0; r < H.nrows; r++) {
            if (H.rows[r] >= ld) { hipFree(arena); *err = "alvrl_refine: row id out of range"; return 1; }
            h_rows[row_off[j] + r] = H.rows[r];
            h_locw[row_off[j] + r] = H.locw[r];
        }
        JobDev& J = h_jobs[j];
        char* p = arena + job_off[j];
        const uint32_t R = H.nrows;
        J.rows = d_rows + row_off[j]; J.locw = d_locw + row_off[j]; J.nrows = R;
        J.pixel_under = H.pixel_under; J.undersampling = H.undersampling;
        J.depth_correction = H.depth_correction; J.do_refine = H.do_refine;
        J.stage_refine = H.stage_refine; J.stage_sample = H.stage_sample;
        J.vrls = (uint32_t*)p; p += align_up(N * 4);
        J.colw = (float*)p; p += align_up(N * 4);
        J.heap = (CNode*)p; p += align_up(N * sizeof(CNode));
        J.sh_heap = (CNode*)p; p += align_up(N * sizeof(CNode));
        J.singles = (uint32_t*)p; p += align_up(N * 4);
        J.sh_singles = (uint32_t*)p; p += align_up(N * 4);
        J.dir = (float*)p; p += align_up((size_t)R * 4);
        J.keys0 = (unsigned long long*)p; p += align_up(N * 8);
        J.keys1 = (unsigned long long*)p; p += align_up(N * 8);
        J.fsu = (float*)p; p += align_up(N * 4);
        J.fsi = (float*)p; p += align_up(N * 4);
        J.feu = (float*)p; p += align_up(N * 4);
        J.fei = (float*)p; p += align_up(N * 4);
        J.st = (double*)p; p += align_up((size_t)3 * R * 8);
        J.bufM = (double*)p; p += align_up((size_t)kChunk * R * 8);
        J.bufV = (double*)p; p += align_up((size_t)kChunk * R * 8);
        J.out_reps = (uint32_t*)p; p += align_up(N * 4);
        J.out_w = (float*)p; p += align_up(N * 4);
        J.out_n = (uint32_t*)p;
        J.out_refined = (int*)(p + 4);
        J.out_err = (int*)(p + 8);
    }
    Common cm;
    cm.Rt = reinterpret_cast<const float2*>(d_Rt); cm.ld = ld; cm.nvrl = nvrl;
    cm.init_vrls = d_init; cm.init_off = d_init_off; cm.ninit = ninit;
    cm.seed = seed; cm.pass = pass;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMemcpyAsync(d_rows, h_rows.data(), rows_total * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_locw, h_locw.data(), rows_total * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_init, init_vrls, (size_t)nv * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_init_off, init_off, (size_t)(ninit + 1) * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_jobs, h_jobs.data(), njobs * sizeof(JobDev), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipEventRecord(e0, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_refine, dim3(njobs), dim3(kThreads), 0, s, d_jobs, cm);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    // gather results
    std::vector<uint32_t> meta(3 * (size_t)njobs);
    for (uint32_t j = 0; j < njobs && e == hipSuccess; j++)
        e = hipMemcpyAsync(&meta[3 * (size_t)j], h_jobs[j].out_n, 12, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    int rc = 0;
    if (e == hipSuccess) {
        uint32_t off = 0;
        for (uint32_t j = 0; j < njobs; j++) {
            const uint32_t n = meta[3 * (size_t)j];
            const int refined = (int)meta[3 * (size_t)j + 1];
            const int jerr = (int)meta[3 * (size_t)j + 2];
            if (jerr) { rc = 5; *err = "alvrl_refine: clustering invariant violated in job " + std::to_string(j); }
            if (n > nvrl) { rc = 5; *err = "alvrl_refine: corrupt representative count"; break; }
            out_refined[j] = refined;
            if (n) {
                e = hipMemcpyAsync(out_reps + off, h_jobs[j].out_reps, (size_t)n * 4, hipMemcpyDeviceToHost, s);
                if (e == hipSuccess) e = hipMemcpyAsync(out_w + off, h_jobs[j].out_w, (size_t)n * 4, hipMemcpyDeviceToHost, s);
                if (e != hipSuccess) break;
            }
            off += n;
            out_off[j + 1] = off;
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess && ms) e = hipEventElapsedTime(ms, e0, e1);
    }
    if (e != hipSuccess) { rc = 3; *err = std::string("alvrl_refine: ") + hipGetErrorString(e); }
    hipFree(arena);
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    return rc;
}

}  // namespace alvrl
