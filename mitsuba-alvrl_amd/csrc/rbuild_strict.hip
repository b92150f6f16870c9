// rbuild_strict.hip -- the R build in the oracle's arithmetic (integrator
// property strictRbuild, alvrl_set_strict_rbuild; the default pipeline).
//
// getLiLuminanceVrlContributions (vrlIntegrator.cpp:527-539) through
// integrateVRL's mean / variance outputs (:603-785) and its samplers
// (:831-1032), HomogeneousMedium::eval (homogeneous.cpp:354-396) and the
// shadow term of Scene::evalTransmittance (scene.cpp:619-679), evaluated
// statement for statement in the order of the CPU restatement
// (oracle/alvrl_oracle.c integrate_vrl_w): IEEE float division and sqrt, no
// contraction (this file is built with -ffp-contract=off and without the
// gathers' approximate division), and the transcendentals of detmath.h, which
// the oracle shares -- evaluated here through detmath_fast.h, which returns
// detmath.h's float for every one of the 2^32 inputs (checked exhaustively
// on the device, k_detmath_exhaustive).  Its R entries are the oracle's bit for
// bit, so the discrete clustering decisions downstream (bit-exact given the
// same R, refine.hip) follow the oracle's own pipeline (tests/test_gpu_strict.py).
//
// Execution model (as gather.hip's k_build_R_blocks): lane = representative
// row, the VRL is wave-uniform and its prepared record (StrictVrl: the
// VRL-only values the restatement derives, computed by the same operations
// once per VRL) is read with scalar loads; the row's own values are hoisted
// out of the VRL loop.  Values the oracle recomputes but that are identical by
// construction (the row's eye segment and vol->surf transmittance, a pair's
// closest points and asinh bounds, |U - V| for the shadow ray, the pdf and
// transmittance exponentials of one distance) are evaluated once: the same
// operations on the same operands give the same bits.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>
#include <mutex>

#include "detmath.h"
#include "detmath_fast.h"
#include "vrl_device.hpp"

#ifndef ALVRL_STRICT_MINB
#define ALVRL_STRICT_MINB 4   // 4 waves/SIMD (<= 128 VGPRs): 127 -> 117 ms at C4 against 3
#endif

namespace alvrl {
namespace strict {

struct V3 { float x, y, z; };
__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 scl(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ float len(V3 a) { return sqrtf(len2(a)); }
__device__ __forceinline__ float dist(V3 a, V3 b) { return len(sub(a, b)); }
__device__ __forceinline__ float dist2(V3 a, V3 b) { return len2(sub(a, b)); }
// normalize(v) = v * (1 / |v|) (operator/ multiplies by the reciprocal)
__device__ __forceinline__ V3 nrm(V3 a) { const float r = 1.0f / len(a); return scl(a, r); }

constexpr float kEps = 1e-4f;
constexpr uint32_t kFlagHit = 1u, kFlagSmooth = 2u, kFlagMedium = 4u;

// The transcendentals of one evaluation: FAST = detmath_fast.h's flag-raising
// forms (a lane whose flag is set re-evaluates its R entry with FAST = false),
// otherwise detmath.h itself.
// Division: the compiler's IEEE expansion (v_div_scale x2, v_rcp, five fmas,
// v_div_fmas, v_div_fixup: 11 VALU, exact for every operand, nothing to check)
// costs less than detmath_fast.h's unscaled core with its zero select and
// range checks (10 + 5): R build alone 90.0 -> 89.3 ms.  ALVRL_STRICT_FASTDIV=1:
// the core (developer A/B).
#ifndef ALVRL_STRICT_FASTDIV
#define ALVRL_STRICT_FASTDIV 0
#endif
// ALVRL_STRICT_STUB_FLAGS (developer timing variant, results invalid): the
// fast forms' range / rounding flags are computed into a dead local
#ifdef ALVRL_STRICT_STUB_FLAGS
#define TX_FLAG(s) d_
#define TXD FxRange d_ = fx_range_init(); (void)d_;
#else
#define TX_FLAG(s) (s)
#define TXD
#endif
template <bool FAST>
struct Tx {
#ifdef ALVRL_STRICT_STUB_TX   // developer timing variant: results invalid
    static __device__ __forceinline__ float exp(float x, FxRange& s) { return __expf(x); }
    static __device__ __forceinline__ float atan(float x, FxRange& s) { return x * 0.7f; }
    static __device__ __forceinline__ float tan(float x, FxRange& s) { return x * 1.3f; }
    static __device__ __forceinline__ float asinh(float x, FxRange& s) { return x * 0.9f; }
    static __device__ __forceinline__ float sinh(float x, FxRange& s) { return x * 1.1f; }
#else
    static __device__ __forceinline__ float exp(float x, FxRange& s) { TXD return FAST ? fx_expf_r(x, TX_FLAG(s)) : dm_expf(x); }
    static __device__ __forceinline__ float atan(float x, FxRange& s) { TXD return FAST ? fx_atanf_r(x, TX_FLAG(s)) : dm_atanf(x); }
    static __device__ __forceinline__ float tan(float x, FxRange& s) { TXD return FAST ? fx_tanf_r(x, TX_FLAG(s)) : dm_tanf(x); }
    static __device__ __forceinline__ float asinh(float x, FxRange& s) { TXD return FAST ? fx_asinhf_r(x, TX_FLAG(s)) : dm_asinhf(x); }
    static __device__ __forceinline__ float sinh(float x, FxRange& s) { TXD return FAST ? fx_sinhf_r(x, TX_FLAG(s)) : dm_sinhf(x); }
#endif
#ifdef ALVRL_STRICT_STUB_DIV   // developer timing variant: results invalid
    static __device__ __forceinline__ float sqrt(float x, FxRange& s) { return __builtin_amdgcn_sqrtf(x); }
    static __device__ __forceinline__ float div(float a, float b, FxRange& s) { return a * __builtin_amdgcn_rcpf(b); }
    static __device__ __forceinline__ float rcp(float b, FxRange& s) { return __builtin_amdgcn_rcpf(b); }
#else
    // IEEE sqrt and reciprocal: their cores without the scaling (flag outside
    // the range where the scaling is the identity), or the compiler's expansion
    static __device__ __forceinline__ float sqrt(float x, FxRange& s) { TXD return FAST ? fx_sqrtf_r(x, TX_FLAG(s)) : sqrtf(x); }
    static __device__ __forceinline__ float div(float a, float b, FxRange& s) { return ALVRL_STRICT_FASTDIV && FAST ? fx_divf_r(a, b, s) : a / b; }
    static __device__ __forceinline__ float rcp(float b, FxRange& s) { TXD return FAST ? fx_rcpf_r(b, TX_FLAG(s)) : 1.0f / b; }
#endif
};
template <bool FAST> __device__ __forceinline__ float lenT(V3 a, FxRange& s) { return Tx<FAST>::sqrt(len2(a), s); }
template <bool FAST> __device__ __forceinline__ float distT(V3 a, V3 b, FxRange& s) { return lenT<FAST>(sub(a, b), s); }
template <bool FAST> __device__ __forceinline__ V3 nrmT(V3 a, FxRange& s)
{
    const float r = Tx<FAST>::rcp(lenT<FAST>(a, s), s);
    return scl(a, r);
}

// The VRL-only values of integrate_vrl_w, by the restatement's own operations
// (k_prepare_strict).  128 B: two s_load_dwordx16.
struct __attribute__((aligned(16))) StrictVrl {
    float sx, sy, sz, ex, ey, ez;   // m_start, m_end
    float pr, pg, pb;               // m_power
    float dx, dy, dz;               // normalize(End - S) (SV, Novak's dirSE, the vol->surf Kulla direction)
    float vx, vy, vz;               // End - S (closest points' v)
    float c;                        // dot(v, v) = len2(v)
    float dSE;                      // distance(S, End)
    float invlen;                   // 1 / distance(End, S)
    float pad[13];
};
static_assert(sizeof(StrictVrl) == 128, "StrictVrl layout");

__global__ void __launch_bounds__(256) k_prepare_strict(const float* __restrict__ soa, uint32_t n,
                                                        StrictVrl* __restrict__ out)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const V3 S = mk(soa[0 * (size_t)n + v], soa[1 * (size_t)n + v], soa[2 * (size_t)n + v]);
    const V3 End = mk(soa[3 * (size_t)n + v], soa[4 * (size_t)n + v], soa[5 * (size_t)n + v]);
    StrictVrl o;
    o.sx = S.x; o.sy = S.y; o.sz = S.z; o.ex = End.x; o.ey = End.y; o.ez = End.z;
    o.pr = soa[6 * (size_t)n + v]; o.pg = soa[7 * (size_t)n + v]; o.pb = soa[8 * (size_t)n + v];
    const V3 sv = nrm(sub(End, S));
    o.dx = sv.x; o.dy = sv.y; o.dz = sv.z;
    const V3 vv = sub(End, S);
    o.vx = vv.x; o.vy = vv.y; o.vz = vv.z;
    o.c = dot(vv, vv);
    o.dSE = dist(S, End);
    o.invlen = 1 / dist(End, S);
    for (int i = 0; i < 13; i++) o.pad[i] = 0.0f;
    out[v] = o;
}

// Draw k of the counter stream (dom, a, b, c): one Philox block of four per
// four draws (oracle draw()).  With a compile-time sample count and
// Rsamples = 1 every k is a constant and the block cache folds away.
struct Draws {
    uint32_t a, b, c, seed, pass, blk;
    U4 buf;
    __device__ __forceinline__ float at(uint32_t k)
    {
        const uint32_t bk = k >> 2;
        if (bk != blk) {
            buf = philox4x32_10(a, b, bk, (kDomRbuild << 24) | (c & 0xFFFFFFu), seed, pass);
            blk = bk;
        }
        const uint32_t j = k & 3u;
        return u01(j == 0 ? buf.x : j == 1 ? buf.y : j == 2 ? buf.z : buf.w);
    }
};

// MaxExpDist::cdf (maxexp.h:83-94)
template <bool FAST>
__device__ __forceinline__ float mxexp_cdf(const DevParams& P, float t, FxRange& slow)
{
    int k = 0;
    while (k < 3 && P.mx_start[k] < t) k++;
    const int i = k > 0 ? k - 1 : 0;
    const float upper = -Tx<FAST>::exp(-P.mx_sigma[i] * t, slow);
    return P.mx_cdf[i] + (upper - P.mx_lower[i]) * P.mx_inv_norm;
}

// HomogeneousMedium::eval (homogeneous.cpp:354-396): transmittance and the
// pdfFailure of the sampling strategy
template <bool FAST>
__device__ __forceinline__ void medium_eval(const DevParams& P, float distance, float tr[3], float* pdf_failure,
                                            FxRange& slow)
{
    const float e0 = Tx<FAST>::exp(P.sigma_t[0] * (-distance), slow);
    const float e1 = Tx<FAST>::exp(P.sigma_t[1] * (-distance), slow);
    const float e2 = Tx<FAST>::exp(P.sigma_t[2] * (-distance), slow);
    float pf = 0.0f;
    if (P.strategy == 0) {
        pf += e0; pf += e1; pf += e2;
        pf = Tx<FAST>::div(pf, 3.0f, slow);
    } else if (P.strategy == 3) {
        pf = 1 - mxexp_cdf<FAST>(P, distance, slow);
    } else {
        pf = Tx<FAST>::exp(-P.density * distance, slow);
    }
    tr[0] = e0; tr[1] = e1; tr[2] = e2;
    *pdf_failure = pf * P.w + (1 - P.w);
    float mx = tr[0] > tr[1] ? tr[0] : tr[1];
    mx = mx > tr[2] ? mx : tr[2];
    if (mx < 1e-20f) tr[0] = tr[1] = tr[2] = 0.0f;
}

// Scene::evalTransmittance(p1, p1OnSurface, p2): exp(-sigma_t |p2 - p1|) per
// channel, zero when an occluder (not a null surface) lies on the segment.
// `remaining` = |p2 - p1|, which the caller has as distance(p1, p2) (the
// squares of negated components are the same floats).
template <bool FAST, bool OCC>
__device__ __forceinline__ void shadow_transmittance(const DevParams& P, V3 p1, bool p1_surface, V3 p2,
                                                     float remaining, float tr[3], FxRange& slow)
{
    const float negLength = 0.0f - remaining;
    for (int i = 0; i < 3; i++) tr[i] = P.sigma_t[i] != 0 ? Tx<FAST>::exp(P.sigma_t[i] * negLength, slow) : 1.0f;
    if (!OCC) return;
    if (P.occ.ntri == 0 || !(remaining > 0)) return;
    const V3 d = sub(p2, p1);
    const V3 dn = scl(d, Tx<FAST>::rcp(remaining, slow));
    const float mint = p1_surface ? 1e-4f : 0.0f;
    const float maxt = remaining * 1.0f;
    if (bvh::occluded(P.occ, bvh::mk(p1.x, p1.y, p1.z), bvh::mk(dn.x, dn.y, dn.z), mint, maxt))
        tr[0] = tr[1] = tr[2] = 0.0f;
}

// isotropic.cpp:76-78, hg.cpp:107-110
template <bool FAST>
__device__ __forceinline__ float phase_eval(const DevParams& P, V3 wi, V3 wo, FxRange& slow)
{
    if (P.phase_type == 0) return kInvFourPi;
    const float g = P.g;
    const float temp = 1.0f + g * g + 2.0f * g * dot(wi, wo);
    return Tx<FAST>::div(kInvFourPi * (1 - g * g), temp * Tx<FAST>::sqrt(temp, slow), slow);
}

// the row's eye segment: everything integrateVRL derives without the VRL
struct Row {
    V3 E, d, U, n, B, dirAB, nd, u;
    float alb[3], wt[3], teus[3], cos_wi;
    float dAB;              // distance(A, B) (Kulla on the eye segment, A = E)
    float a_uu, eps_luu;    // closest points: dot(u, u), kEps * len2(u)
    uint32_t flags, rid, sw;
    bool surf;
};

// getClosestPoints (vrlIntegrator.cpp:962-1032) for S1 = the eye segment E ->
// hit, S2 = the VRL; returns |dP| and the closest point on the VRL
template <bool FAST>
__device__ __forceinline__ float closest_points(const Row& w, V3 S, const V3& vv, float c, V3* S2h, FxRange& slow)
{
    const V3 u = w.u, v = vv, wv = sub(w.E, S);
    const float a = w.a_uu, b = dot(u, v), d = dot(u, wv), e = dot(v, wv);
    const float D = a * c - b * b;
    float sN, sD = D, tN, tD = D;
    if (D < w.eps_luu * c) {
        sN = 0.0f; sD = 1.0f; tN = e; tD = c;
    } else {
        sN = (b * e - c * d);
        tN = (a * e - b * d);
        if (sN < 0.0f) { sN = 0.0f; tN = e; tD = c; }
        else if (sN > sD) { sN = sD; tN = e + b; tD = c; }
    }
    if (tN < 0.0f) {
        tN = 0.0f;
        if (-d < 0.0f) sN = 0.0f;
        else if (-d > a) sN = sD;
        else { sN = -d; sD = a; }
    } else if (tN > tD) {
        tN = tD;
        if ((-d + b) < 0.0f) sN = 0;
        else if ((-d + b) > a) sN = sD;
        else { sN = (-d + b); sD = a; }
    }
    const float sc = Tx<FAST>::div(sN, sD, slow);
    const float tc = Tx<FAST>::div(tN, tD, slow);
    const V3 dP = sub(add(wv, scl(u, sc)), scl(v, tc));
    *S2h = add(S, scl(v, tc));
    return lenT<FAST>(dP, slow);
}

// KullaSampling (vrlIntegrator.cpp:889-914) split into the part fixed by the
// segment A->B and the point D, and the per-uniform sample
struct Kulla { V3 dir, I; float Dis, aa, ab; };

template <bool FAST>
__device__ __forceinline__ Kulla kulla_frame(V3 A, V3 B, V3 dir, float dAB, V3 D, FxRange& slow)
{
    Kulla k;
    k.dir = dir;
    const float dotPr = dot(dir, sub(D, A));
    k.I = add(A, scl(dir, dotPr));
    k.Dis = distT<FAST>(D, k.I, slow);
    const float dAI = distT<FAST>(A, k.I, slow);
    float angle_a = Tx<FAST>::atan(Tx<FAST>::div(dAI, k.Dis, slow), slow);
    float angle_b = Tx<FAST>::atan(Tx<FAST>::div(distT<FAST>(k.I, B, slow), k.Dis, slow), slow);
    if (dotPr > 0) {
        angle_a *= -1;
        if (dAI > dAB) angle_b *= -1;
    }
    k.aa = angle_a; k.ab = angle_b;
    return k;
}

template <bool FAST>
__device__ __forceinline__ float kulla_sample(const Kulla& k, float uniform, V3* result, FxRange& slow)
{
    const float t = k.Dis * Tx<FAST>::tan(((1.0f - uniform) * k.aa) + (uniform * k.ab), slow);
    const float pdf = Tx<FAST>::div(k.Dis, (k.ab - k.aa) * (k.Dis * k.Dis + t * t), slow);
    *result = add(k.I, scl(k.dir, t));
    return pdf;
}

// sampleVtoDistance (vrlIntegrator.cpp:916-953), the uniform-free part
struct Novak {
    int mode;           // 0: zero-length VRL, 1: parallel (uniform on the VRL), 2: Novak
    float h, sinTheta, A0, A1, denom, dVhS;
};

template <bool FAST>
__device__ __forceinline__ Novak novak_frame(const Row& w, V3 S, V3 End, V3 SE, const V3& vv, float c, float dSE,
                                             FxRange& slow)
{
    Novak n;
    n.mode = 0;
    if (dSE == 0) return n;
    const float cosTheta = dot(w.nd, SE);
    const float st2 = 1 - cosTheta * cosTheta;
    n.sinTheta = Tx<FAST>::sqrt(st2 > 0.0f ? st2 : 0.0f, slow);
    if (n.sinTheta < kEps) {
        n.mode = 1;
        return n;
    }
    n.mode = 2;
    V3 Vh;
    n.h = closest_points<FAST>(w, S, vv, c, &Vh, slow);
    n.dVhS = distT<FAST>(Vh, S, slow);
    const float V0c = -1 * n.dVhS;
    const float V1c = distT<FAST>(Vh, End, slow);
    n.A0 = Tx<FAST>::asinh(Tx<FAST>::div(V0c, n.h, slow) * n.sinTheta, slow);
    n.A1 = Tx<FAST>::asinh(Tx<FAST>::div(V1c, n.h, slow) * n.sinTheta, slow);
    n.denom = Tx<FAST>::div(n.A1 - n.A0, n.sinTheta, slow);
    return n;
}

template <bool FAST>
__device__ __forceinline__ float novak_sample(const Novak& n, V3 S, V3 End, V3 SE, float invlen, float uniform,
                                              V3* V, FxRange& slow)
{
    if (n.mode == 0) { *V = S; return 1; }
    if (n.mode == 1) { *V = add(S, scl(sub(End, S), uniform)); return invlen; }
    float newV = n.h * Tx<FAST>::sinh(n.A0 + (uniform * (n.A1 - n.A0)), slow);
    newV = Tx<FAST>::div(newV, n.sinTheta, slow);
    const float result = Tx<FAST>::rcp(Tx<FAST>::sqrt(n.h * n.h + newV * newV * n.sinTheta * n.sinTheta, slow), slow);
    newV += n.dVhS;
    *V = add(S, scl(SE, newV));
    return Tx<FAST>::div(result, n.denom, slow);
}

__device__ __forceinline__ Row make_row(const DevParams& P, const Rec& r, uint32_t rid)
{
    Row w;
    w.E = mk(r.ox, r.oy, r.oz); w.d = mk(r.dx, r.dy, r.dz);
    w.U = mk(r.px, r.py, r.pz); w.n = mk(r.nx, r.ny, r.nz);
    w.alb[0] = r.ar; w.alb[1] = r.ag; w.alb[2] = r.ab;
    w.wt[0] = r.wr; w.wt[1] = r.wg; w.wt[2] = r.wb;      // use_weight: the record's path weight
    w.flags = r.flags;
    w.rid = rid;
    w.sw = ((r.depth & 0xFFu) << 16) | ((r.depth >> 16) & 0xFFFFu);
    const float edist = dist(w.U, w.E);                  // sampleUVKulla :865-871
    w.B = add(w.E, scl(w.d, edist));
    w.dirAB = nrm(sub(w.B, w.E));
    w.dAB = dist(w.E, w.B);
    w.teus[0] = w.teus[1] = w.teus[2] = 0.0f;
    if ((r.flags & kFlagHit) && edist != 0) {
        float pfd;
        FxRange unused = fx_range_init();
        medium_eval<false>(P, edist, w.teus, &pfd, unused);
    }
    w.surf = (w.teus[0] != 0 || w.teus[1] != 0 || w.teus[2] != 0) && (r.flags & kFlagSmooth);
    w.cos_wi = dot(neg(w.d), w.n);
    w.nd = nrm(w.d);
    w.u = sub(w.U, w.E);                                 // closest points: u = S1P1 - S1P0
    w.a_uu = dot(w.u, w.u);
    w.eps_luu = kEps * len2(w.u);
    return w;
}

__device__ __forceinline__ float lum(const float c[3]) { return c[0] * 0.212671f + c[1] * 0.715160f + c[2] * 0.072169f; }
__device__ __forceinline__ bool valid(const float c[3])
{
    for (int i = 0; i < 3; i++)
        if (!isfinite(c[i]) || c[i] < 0.0f) return false;
    return true;
}

// integrate_vrl_w's contribution (mean) and variance outputs for one pair.
// NVV / NVS < 0: the sample counts come from P at run time.
template <int NVV, int NVS, bool OCC, bool FAST>
__device__ __forceinline__ void integrate_R(const DevParams& P, const Row& w, const StrictVrl& L, uint32_t v,
                                            uint32_t koff, float* contrib, float* variance, FxRange& slow)
{
    *contrib = 0; *variance = 0;
    if (!(w.flags & kFlagMedium)) return;
    const V3 S = mk(L.sx, L.sy, L.sz);
    const V3 End = mk(L.ex, L.ey, L.ez);
    const float power[3] = {L.pr, L.pg, L.pb};
    const V3 SV = mk(L.dx, L.dy, L.dz);
    const V3 vv = mk(L.vx, L.vy, L.vz);
    const V3 EU = w.d;
    const int nVV = NVV >= 0 ? NVV : P.nvv, nVS = NVS >= 0 ? NVS : P.nvs;
    // the Philox key schedule is re-derived per VRL (scalar adds) instead of
    // being hoisted out of the VRL loop into twenty SGPRs that spill
    uint32_t seed = P.seed, pass = P.pass;
    asm volatile("" : "+s"(seed), "+s"(pass));
    Draws dr{w.rid, v, w.sw, seed, pass, 0xFFFFFFFFu, U4{0u, 0u, 0u, 0u}};

    // ---- volume to volume (:647-703) ----
    const Novak nv = novak_frame<FAST>(w, S, End, SV, vv, L.c, L.dSE, slow);
    float mean = 0, M2 = 0;
    for (int sample = 0; sample < nVV; sample++) {
        float lumv = 0.0f;
        const float u0 = dr.at(koff + 2 * sample);
        const float u1 = dr.at(koff + 2 * sample + 1);
        V3 V, U;
        float pdf = novak_sample<FAST>(nv, S, End, SV, L.invlen, u0, &V, slow);
        pdf *= kulla_sample<FAST>(kulla_frame<FAST>(w.E, w.B, w.dirAB, w.dAB, V, slow), u1, &U, slow);
        const float dUV = distT<FAST>(U, V, slow);
        if (dUV != 0) {
            const V3 VU = nrmT<FAST>(sub(U, V), slow);
            float tuv[3], teu[3], tsv[3], pf_eu, pf_sv;
            shadow_transmittance<FAST, OCC>(P, U, false, V, dUV, tuv, slow);
            if (!(tuv[0] == 0 && tuv[1] == 0 && tuv[2] == 0)) {
                medium_eval<FAST>(P, distT<FAST>(w.E, U, slow), teu, &pf_eu, slow);
                medium_eval<FAST>(P, distT<FAST>(S, V, slow), tsv, &pf_sv, slow);
                const float rpdf = Tx<FAST>::rcp(pdf, slow);
                const float rd2 = Tx<FAST>::rcp(dist2(U, V), slow);
                const float phU = phase_eval<FAST>(P, neg(VU), neg(EU), slow);
                const float phV = phase_eval<FAST>(P, neg(SV), VU, slow);
                const float rpf = Tx<FAST>::rcp(pf_sv, slow);
                float c[3];
                for (int i = 0; i < 3; i++) {
                    c[i] = w.wt[i];
                    c[i] *= power[i];
                    c[i] *= (P.sigma_s[i] * P.sigma_s[i]) * rpdf;
                    c[i] *= rd2;
                    c[i] *= tsv[i];
                    c[i] *= tuv[i];
                    c[i] *= teu[i];
                    if (P.short_vrls) c[i] *= rpf;
                    c[i] *= phU;
                    c[i] *= phV;
                }
                if (valid(c)) lumv = lum(c);
            }
        }
        const float delta = lumv - mean;                 // :693-699
        mean += delta / (sample + 1);
        M2 += delta * (lumv - mean);
    }
    if (nVV > 0) { *contrib += mean; *variance += M2 / ((nVV - 1) * nVV); }

    // ---- volume to surface (:706-782) ----
    mean = 0; M2 = 0;
    if (w.surf && nVS > 0) {
        const Kulla ks = kulla_frame<FAST>(S, End, SV, L.dSE, w.U, slow);
        for (int sample = 0; sample < nVS; sample++) {
            float lumv = 0.0f;
            const float u = dr.at(koff + 2 * nVV + sample);
            V3 V;
            const float pdf = kulla_sample<FAST>(ks, u, &V, slow);
            const float dUV = distT<FAST>(w.U, V, slow);
            if (dUV != 0) {
                const V3 VU = nrmT<FAST>(sub(w.U, V), slow);
                float tuv[3], tsv[3], pf_sv;
                shadow_transmittance<FAST, OCC>(P, w.U, true, V, dUV, tuv, slow);
                medium_eval<FAST>(P, distT<FAST>(S, V, slow), tsv, &pf_sv, slow);
                // SmoothDiffuse::eval (diffuse.cpp:110-118)
                const float cos_wo = dot(neg(VU), w.n);
                float f[3] = {0, 0, 0};
                if (!(w.cos_wi <= 0 || cos_wo <= 0))
                    for (int i = 0; i < 3; i++) f[i] = w.alb[i] * (kInvPi * cos_wo);
                const float phV = phase_eval<FAST>(P, neg(SV), VU, slow);
                const float rpdf = Tx<FAST>::rcp(pdf, slow);
                const float rd2 = Tx<FAST>::rcp(dist2(w.U, V), slow);
                const float rpf = Tx<FAST>::rcp(pf_sv, slow);
                float c[3];
                for (int i = 0; i < 3; i++) {
                    c[i] = w.wt[i];
                    c[i] *= power[i];
                    c[i] *= P.sigma_s[i] * rpdf;
                    c[i] *= rd2;
                    c[i] *= tsv[i];
                    c[i] *= tuv[i];
                    c[i] *= w.teus[i];
                    if (P.short_vrls) c[i] *= rpf;
                    c[i] *= phV;
                    c[i] *= f[i];
                }
                if (valid(c)) lumv = lum(c);
            }
            const float delta = lumv - mean;
            mean += delta / (sample + 1);
            M2 += delta * (lumv - mean);
        }
    } else {
        // no surface sample contributes: the Welford recurrence over zeros
        // leaves mean = M2 = 0
    }
    if (nVS > 0) { *contrib += mean; *variance += M2 / ((nVS - 1) * nVS); }
}

__device__ __forceinline__ Rec load_rec(const Rec* __restrict__ recs, uint32_t r)
{
    const float4* p = reinterpret_cast<const float4*>(recs + r);
    const float4 a = p[0], b = p[1], c = p[2], d = p[3], e = p[4];
    Rec x;
    x.ox = a.x; x.oy = a.y; x.oz = a.z; x.dx = a.w;
    x.dy = b.x; x.dz = b.y; x.px = b.z; x.py = b.w;
    x.pz = c.x; x.nx = c.y; x.ny = c.z; x.nz = c.w;
    x.ar = d.x; x.ag = d.y; x.ab = d.z; x.flags = __float_as_uint(d.w);
    x.wr = e.x; x.wg = e.y; x.wb = e.z; x.depth = __float_as_uint(e.w);
    return x;
}

// One R entry: the sum over Rsamples of (contribution, variance) scaled by
// the normalization as brute_worker / Rbuilder write it (:812-813).
// RS1: Rsamples = 1 (one sample, draw offset 0).
template <int NVV, int NVS, bool OCC, bool RS1, bool FAST>
__device__ __forceinline__ float2 entry(const DevParams& P, const Row& w, const StrictVrl& L, uint32_t v,
                                       float normalization, FxRange& slow)
{
    const int nsamp = RS1 ? 1 : (P.rsamples > 1 ? P.rsamples : 1);
    float m = 0.0f, s = 0.0f;
    for (int si = 0; si < nsamp; si++) {
        float contribution, variance;
        integrate_R<NVV, NVS, OCC, FAST>(P, w, L, v, RS1 ? 0u : ((uint32_t)si & 0xFFFFu) << 10, &contribution,
                                         &variance, slow);
        m += contribution * normalization;
        s += variance * normalization * normalization;
    }
    return make_float2(m, s);
}

// The queue of entries the fast evaluation could not settle: (launch row,
// VRL) pairs, re-evaluated with detmath.h by k_build_R_strict_fixup.  Keeping
// that evaluation out of the main kernel keeps its code (and instruction cache
// footprint) to the fast form alone.
struct FixQueue {
    uint2* items;
    unsigned long long* count;
    uint32_t cap;
};

__device__ __forceinline__ void store_entry(float2* __restrict__ Rt, uint64_t idx, bool accum, float2 e)
{
    float2* p = &Rt[idx];
    if (accum) { const float2 o = *p; *p = make_float2(o.x + e.x, o.y + e.y); }
    else *p = e;
}

// lane = row, the block's four waves interleave over a 256-VRL chunk, as
// gather.hip's k_build_R / k_build_R_blocks (same outputs, same counters).
// roff == nullptr: dense Rt[v * ld + row0 + r].  A lane whose fast
// transcendentals, division or square root could round differently from the
// oracle's (one entry in ~5,000; about one wave iteration in 80) queues the
// entry instead of storing it.  store = 0: only the queue is written (the
// re-run after a queue overflow, which must not add accumulating rows twice).
template <int NVV, int NVS, bool OCC, bool RS1>
__global__ void __launch_bounds__(256, ALVRL_STRICT_MINB) k_build_R_strict(const Rec* __restrict__ recs,
                                                        const uint32_t* __restrict__ ids, uint32_t nrows,
                                                        const StrictVrl* __restrict__ sv, uint32_t nvrl,
                                                        uint32_t chunk, DevParams P, float normalization,
                                                        float2* __restrict__ Rt, uint64_t ld, uint64_t row0,
                                                        const uint64_t* __restrict__ roff,
                                                        const uint32_t* __restrict__ rstride,
                                                        uint8_t* __restrict__ nonzero,
                                                        unsigned long long* counter, FixQueue fq, int store)
{
    fx_tables_init();
    const uint32_t r = blockIdx.x * 64 + (threadIdx.x & 63);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool active = r < nrows;
    Rec rec;
    if (active) rec = load_rec(recs, r);
    else { rec = Rec{}; rec.flags = 0u; }
    const uint32_t rid = active ? (ids ? ids[r] : r) : 0u;
    const Row w = make_row(P, rec, rid);
    const bool medium = active && (rec.flags & kFlagMedium);
    const uint64_t base = !active ? 0 : roff ? roff[r] : row0 + r;
    const uint64_t stride = !active ? 0 : roff ? rstride[r] : ld;
    const uint32_t v0 = blockIdx.y * chunk;
    const uint32_t v1 = min(nvrl, v0 + chunk);
    const int nsamp = RS1 ? 1 : (P.rsamples > 1 ? P.rsamples : 1);
    uint32_t done = 0;
    for (uint32_t v = v0 + wave; v < v1; v += 4) {
        float2 e = make_float2(0.0f, 0.0f);
        bool slow = false;
        if (medium) {
            const StrictVrl L = sv[v];
            FxRange g = fx_range_init();
            e = entry<NVV, NVS, OCC, RS1, true>(P, w, L, v, normalization, g);
            slow = fx_range_slow(g);
        }
        if (store && active && !slow) store_entry(Rt, base + (uint64_t)v * stride, rec.flags & kRecAccum, e);
        const unsigned long long sb = __ballot(slow);
        if (sb) {   // wave-aggregated append
            unsigned long long at = 0;
            if ((threadIdx.x & 63) == 0) at = atomicAdd(fq.count, (unsigned long long)__popcll(sb));
            at = __shfl(at, 0);
            const uint32_t lane = threadIdx.x & 63;
            const unsigned long long k = at + __popcll(sb & ((1ull << lane) - 1ull));
            if (slow && k < fq.cap) fq.items[k] = make_uint2(r, v);
        }
        if (store && nonzero && __ballot(active && !slow && e.x != 0.0f) && (threadIdx.x & 63) == 0) nonzero[v] = 1;
        ++done;
    }
    const unsigned long long m = __ballot(medium);
    if (store && (threadIdx.x & 63) == 0 && m) atomicAdd(counter, (unsigned long long)__popcll(m) * done * (uint32_t)nsamp);
}

// The queued entries with detmath.h, one lane each (same row set-up, same
// entry, same store and mask as the main kernel)
template <int NVV, int NVS, bool OCC, bool RS1>
__global__ void __launch_bounds__(256) k_build_R_strict_fixup(const Rec* __restrict__ recs,
                                                              const uint32_t* __restrict__ ids,
                                                              const StrictVrl* __restrict__ sv, DevParams P,
                                                              float normalization, float2* __restrict__ Rt,
                                                              uint64_t ld, uint64_t row0,
                                                              const uint64_t* __restrict__ roff,
                                                              const uint32_t* __restrict__ rstride,
                                                              uint8_t* __restrict__ nonzero,
                                                              const uint2* __restrict__ items, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = items[i].x, v = items[i].y;
    const Rec rec = load_rec(recs, r);
    const Row w = make_row(P, rec, ids ? ids[r] : r);
    FxRange unused = fx_range_init();
    const float2 e = entry<NVV, NVS, OCC, RS1, false>(P, w, sv[v], v, normalization, unused);
    const uint64_t base = roff ? roff[r] : row0 + r;
    const uint64_t stride = roff ? rstride[r] : ld;
    store_entry(Rt, base + (uint64_t)v * stride, rec.flags & kRecAccum, e);
    if (nonzero && e.x != 0.0f) nonzero[v] = 1;
}

// detmath.h on the device, elementwise (alvrl_detmath_eval): the host = device
// check of the shared definitions; fn + 8: the detmath_fast.h evaluation
__global__ void __launch_bounds__(256) k_detmath(int fn, const float* __restrict__ in, float* __restrict__ out,
                                                 uint32_t n)
{
    fx_tables_init();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = in[i];
    float y;
    switch (fn) {
    case 0: y = dm_expf(x); break;
    case 1: y = dm_logf(x); break;
    case 2: y = dm_atanf(x); break;
    case 3: y = dm_tanf(x); break;
    case 4: y = dm_asinhf(x); break;
    case 5: y = dm_sinhf(x); break;
    case 8: y = fx_expf(x); break;
    case 10: y = fx_atanf(x); break;
    case 11: y = fx_tanf(x); break;
    case 12: y = fx_asinhf(x); break;
    default: y = fx_sinhf(x); break;
    }
    out[i] = y;
}

// Every float bit pattern in [begin, end): fx_*f(x) against dm_*f(x), bit for
// bit.  out[0] counts mismatches, first[0..15] keeps some mismatching inputs.
template <int FN>
__device__ __forceinline__ void fx_dm(float x, float* f, float* d)
{
    if (FN == 0) { *f = fx_expf(x); *d = dm_expf(x); }
    else if (FN == 2) { *f = fx_atanf(x); *d = dm_atanf(x); }
    else if (FN == 3) { *f = fx_tanf(x); *d = dm_tanf(x); }
    else if (FN == 4) { *f = fx_asinhf(x); *d = dm_asinhf(x); }
    else if (FN == 6) { *f = fx_sqrtf(x); *d = sqrtf(x); }
    else if (FN == 7) { *f = fx_rcpf(x); *d = 1.0f / x; }
    else { *f = fx_sinhf(x); *d = dm_sinhf(x); }
}

template <int FN>
__global__ void __launch_bounds__(256) k_detmath_exhaustive(uint64_t begin, uint64_t end,
                                                            unsigned long long* __restrict__ out,
                                                            uint32_t* __restrict__ first)
{
    fx_tables_init();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t bad = 0;
    for (uint64_t b = begin + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < end; b += stride) {
        const float x = __uint_as_float((uint32_t)b);
        float f, d;
        fx_dm<FN>(x, &f, &d);
        if (__float_as_uint(f) != __float_as_uint(d)) {
            ++bad;
            const unsigned long long k = atomicAdd(out + 1, 1ull);
            if (k < 16) first[k] = (uint32_t)b;
        }
    }
    if (bad) atomicAdd(out, (unsigned long long)bad);
}

// fx_divf(a, b) against IEEE a / b, bit for bit, on n pseudo-random operand
// pairs: even draws are uniform over all 2^32 bit patterns (every exponent,
// zeros, subnormals, infinities, NaNs), odd draws log-uniform magnitudes in
// [2^-44, 2^44] (the fast range and its edges) with random signs.
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_div_check(uint64_t n, uint64_t seed, unsigned long long* __restrict__ out,
                                                   uint32_t* __restrict__ first)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t bad = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t h = mix64(seed ^ (i * 0xD1B54A32D192ED03ull));
        uint32_t ba = (uint32_t)h, bb = (uint32_t)(h >> 32);
        if (i & 1) {   // sign | exponent in [127 - 44, 127 + 44] | mantissa
            ba = (ba & 0x807FFFFFu) | ((83u + ((ba >> 23) & 0xFFu) % 89u) << 23);
            bb = (bb & 0x807FFFFFu) | ((83u + ((bb >> 23) & 0xFFu) % 89u) << 23);
        }
        const float a = __uint_as_float(ba), b = __uint_as_float(bb);
        const float f = fx_divf(a, b), d = a / b;
        if (__float_as_uint(f) != __float_as_uint(d)) {
            ++bad;
            const unsigned long long k = atomicAdd(out + 1, 1ull);
            if (k < 8) { first[2 * k] = ba; first[2 * k + 1] = bb; }
        }
    }
    if (bad) atomicAdd(out, (unsigned long long)bad);
}

}  // namespace strict

hipError_t launch_div_check(uint64_t n, uint64_t seed, unsigned long long* out, uint32_t* first, hipStream_t s)
{
    hipLaunchKernelGGL(strict::k_div_check, dim3(8192), dim3(256), 0, s, n, seed, out, first);
    return hipGetLastError();
}

size_t strict_vrl_bytes() { return sizeof(strict::StrictVrl); }

hipError_t launch_prepare_strict(const float* soa, uint32_t n, void* out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(strict::k_prepare_strict, dim3((n + 255) / 256), dim3(256), 0, s, soa, n,
                       reinterpret_cast<strict::StrictVrl*>(out));
    return hipGetLastError();
}

// the fix-up queue of the strict R build, per device (grown on demand)
static std::mutex g_fix_mu;
struct FixBuf {
    uint2* items = nullptr;
    unsigned long long* count = nullptr;
    unsigned long long* h_count = nullptr;
    uint32_t cap = 0;
};
static FixBuf g_fix[64];

template <int NVV, int NVS, bool OCC, bool RS1>
static hipError_t run_strict(dim3 grid, dim3 block, hipStream_t s, const Rec* recs, const uint32_t* ids,
                             uint32_t nrows, const strict::StrictVrl* sv, uint32_t nvrl, uint32_t chunk,
                             const DevParams& P, float normalization, float2* Rt, uint64_t ld, uint64_t row0,
                             const uint64_t* roff, const uint32_t* rstride, uint8_t* nonzero,
                             unsigned long long* counter)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    // one queue per device; launches of several host threads on one device
    // serialise here (the queue is read back before the next launch uses it)
    std::lock_guard<std::mutex> g(g_fix_mu);
    FixBuf& fb = g_fix[dev];
    if (!fb.count) {
        if ((e = hipMalloc(&fb.count, sizeof(unsigned long long))) != hipSuccess) return e;
        if ((e = hipHostMalloc(&fb.h_count, sizeof(unsigned long long))) != hipSuccess) return e;
    }
    if (fb.cap == 0) {
        // ~0.13 % of the entries are queued (detmath_fast.h's band): room for
        // 0.4 % of this launch's pairs, at least 2^20
        const uint64_t pairs = (uint64_t)grid.x * 64u * nvrl;
        const uint32_t want = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1u << 20, pairs / 256u), 1u << 30);
        if ((e = hipMalloc(&fb.items, sizeof(uint2) * want)) != hipSuccess) return e;
        fb.cap = want;
    }
    for (int attempt = 0; attempt < 2; attempt++) {
        if ((e = hipMemsetAsync(fb.count, 0, sizeof(unsigned long long), s)) != hipSuccess) return e;
        const strict::FixQueue fq{fb.items, fb.count, fb.cap};
        hipLaunchKernelGGL((strict::k_build_R_strict<NVV, NVS, OCC, RS1>), grid, block, 0, s, recs, ids, nrows, sv,
                           nvrl, chunk, P, normalization, Rt, ld, row0, roff, rstride, nonzero, counter, fq,
                           attempt == 0 ? 1 : 0);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(fb.h_count, fb.count, sizeof(unsigned long long), hipMemcpyDeviceToHost, s)) !=
            hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        const unsigned long long n = *fb.h_count;
        if (n <= fb.cap) {
            if (n)
                hipLaunchKernelGGL((strict::k_build_R_strict_fixup<NVV, NVS, OCC, RS1>),
                                   dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, recs, ids, sv, P,
                                   normalization, Rt, ld, row0, roff, rstride, nonzero, fb.items, (uint32_t)n);
            return hipGetLastError();
        }
        // the queue overflowed (its first cap entries were kept, every other
        // entry is stored): grow it and run again to list the queued entries
        // only -- no stores, no counts -- then re-evaluate them
        if (attempt == 1 || n > 0xFFFFFFFFull) return hipErrorOutOfMemory;
        hipFree(fb.items);
        fb.items = nullptr;
        fb.cap = 0;
        if ((e = hipMalloc(&fb.items, sizeof(uint2) * n)) != hipSuccess) return e;
        fb.cap = (uint32_t)n;
    }
    return hipErrorUnknown;
}

template <int NVV, int NVS, bool OCC>
static hipError_t launch_rs(bool rs1, dim3 grid, dim3 block, hipStream_t s, const Rec* recs, const uint32_t* ids,
                            uint32_t nrows, const strict::StrictVrl* sv, uint32_t nvrl, uint32_t chunk,
                            const DevParams& P, float normalization, float2* Rt, uint64_t ld, uint64_t row0,
                            const uint64_t* roff, const uint32_t* rstride, uint8_t* nonzero,
                            unsigned long long* counter)
{
    if (rs1)
        return run_strict<NVV, NVS, OCC, true>(grid, block, s, recs, ids, nrows, sv, nvrl, chunk, P,
                                               normalization, Rt, ld, row0, roff, rstride, nonzero, counter);
    return run_strict<NVV, NVS, OCC, false>(grid, block, s, recs, ids, nrows, sv, nvrl, chunk, P, normalization,
                                            Rt, ld, row0, roff, rstride, nonzero, counter);
}

hipError_t launch_build_R_strict(const Rec* recs, const uint32_t* ids, uint32_t nrows, const void* svrl,
                                 uint32_t nvrl, const DevParams& P, float normalization, float2* Rt, uint64_t ld,
                                 uint64_t row0, const uint64_t* roff, const uint32_t* rstride, uint8_t* nonzero,
                                 unsigned long long* counter, hipStream_t s)
{
    if (nrows == 0 || nvrl == 0) return hipSuccess;
    const uint32_t chunk = 256;
    const dim3 grid((nrows + 63) / 64, (nvrl + chunk - 1) / chunk), block(256);
    const auto* sv = reinterpret_cast<const strict::StrictVrl*>(svrl);
    const bool rs1 = P.rsamples <= 1;
    if (P.occ.ntri)
        return launch_rs<-1, -1, true>(rs1, grid, block, s, recs, ids, nrows, sv, nvrl, chunk, P, normalization, Rt,
                                       ld, row0, roff, rstride, nonzero, counter);
    if (P.nvv == 2 && P.nvs == 2)
        return launch_rs<2, 2, false>(rs1, grid, block, s, recs, ids, nrows, sv, nvrl, chunk, P, normalization, Rt,
                                      ld, row0, roff, rstride, nonzero, counter);
    return launch_rs<-1, -1, false>(rs1, grid, block, s, recs, ids, nrows, sv, nvrl, chunk, P, normalization, Rt,
                                    ld, row0, roff, rstride, nonzero, counter);
}

hipError_t launch_detmath(int fn, const float* in, float* out, uint32_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(strict::k_detmath, dim3((n + 255) / 256), dim3(256), 0, s, fn, in, out, n);
    return hipGetLastError();
}

hipError_t launch_detmath_exhaustive(int fn, uint64_t begin, uint64_t end, unsigned long long* out,
                                     uint32_t* first, hipStream_t s)
{
    if (end <= begin) return hipSuccess;
    const dim3 grid(8192), block(256);
    switch (fn) {
    case 0: hipLaunchKernelGGL(strict::k_detmath_exhaustive<0>, grid, block, 0, s, begin, end, out, first); break;
    case 2: hipLaunchKernelGGL(strict::k_detmath_exhaustive<2>, grid, block, 0, s, begin, end, out, first); break;
    case 3: hipLaunchKernelGGL(strict::k_detmath_exhaustive<3>, grid, block, 0, s, begin, end, out, first); break;
    case 4: hipLaunchKernelGGL(strict::k_detmath_exhaustive<4>, grid, block, 0, s, begin, end, out, first); break;
    case 5: hipLaunchKernelGGL(strict::k_detmath_exhaustive<5>, grid, block, 0, s, begin, end, out, first); break;
    case 6: hipLaunchKernelGGL(strict::k_detmath_exhaustive<6>, grid, block, 0, s, begin, end, out, first); break;
    case 7: hipLaunchKernelGGL(strict::k_detmath_exhaustive<7>, grid, block, 0, s, begin, end, out, first); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace alvrl
