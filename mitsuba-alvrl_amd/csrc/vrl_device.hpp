// vrl_device.hpp -- gfx950 device maths of the ALVRL gather primitive.
//
// integrateVRL (src/integrators/vrl/vrlIntegrator.cpp:603-785) with its
// samplers (:831-1032), HomogeneousMedium::eval / evalTransmittance
// (src/medium/homogeneous.cpp:266-273, 354-396, 'balance' strategy), the
// isotropic / HG phase eval (isotropic.cpp:76-78, hg.cpp:107-110) and
// SmoothDiffuse::eval (diffuse.cpp:110-118), for one (eye segment, VRL) pair.
//
// Execution model: one lane = one eye segment; the VRL being integrated is
// wave-uniform, so its prepared record (VrlPrep) is fetched with scalar loads
// into SGPRs and every pair-independent quantity of the eye segment
// (RecPre) is hoisted out of the VRL loop.  Quantities that the reference
// recomputes per sample but that do not depend on the sample (the
// segment-segment closest points, the asinh bounds of Novak's sampler, the
// equi-angular frame of the vol->surf Kulla sampler) are computed once per
// pair: identical values, fewer transcendentals.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bvh_device.hpp"

namespace alvrl {

constexpr float kEpsilon = 1e-4f;                       // constants.h:27-33
constexpr float kInvFourPi = 0.07957747154594766788f;
constexpr float kInvPi = 0.31830988618379067154f;

constexpr uint32_t kDomGather = 1u;   // render gather draws
constexpr uint32_t kDomRbuild = 2u;   // R-build draws

// Prepared VRL: derived once per VRL set by k_prepare_vrls.  80 B, read with
// s_load_dwordx16 + s_load_dwordx4.
struct __attribute__((aligned(16))) VrlPrep {
    float sx, sy, sz;       // m_start
    float ex, ey, ez;       // m_end
    float vx, vy, vz;       // m_end - m_start
    float pr, pg, pb;       // m_power
    float dx, dy, dz;       // normalize(m_end - m_start)
    float len;              // distance(m_start, m_end)
    float c;                // dot(v, v)
    float pad0, pad1, pad2;
};
static_assert(sizeof(VrlPrep) == 80, "VrlPrep layout");

struct DevParams {
    float sigma_s[3];
    float sigma_t[3];
    float w;                // mediumSamplingWeight
    float g;                // HG asymmetry
    int phase_type;
    int nvv, nvs;
    int short_vrls;
    uint32_t seed, pass;
    int rsamples;           // Rsamples (vrlIntegrator.cpp:194): samples per R entry (0 = 1)
    bvh::View occ;          // occluders blocking U-V and surface-V (ntri == 0: convex container)
    // the medium's sampling strategy (homogeneous.cpp:150-227): 0 balance,
    // 1 single / 2 manual (density), 3 maximum (MaxExpDist, maxexp.h:28-94)
    int strategy;
    float density;
    float mx_sigma[3], mx_cdf[4], mx_start[3], mx_lower[3], mx_inv_norm;
};

// ---------------------------------------------------------------- RNG --
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1)
{
#ifdef ALVRL_EXP_RNG_ROUNDS   // timing-only experiment: fewer rounds (results differ from the oracle)
    constexpr int kRounds = ALVRL_EXP_RNG_ROUNDS;
#else
    constexpr int kRounds = 10;
#endif
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        // one 32x32->64 product per multiplier (v_mad_u64_u32) instead of a
        // v_mul_hi_u32 + v_mul_lo_u32 pair
        const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
        const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        // each three-way XOR as one gfx950 v_bitop3_b32 (truth table 0x96 =
        // A ^ B ^ C; the round key is its SGPR operand) instead of two v_xor_b32:
        // two instructions fewer per round, ~5 % of the gather's VALU stream
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    return U4{c0, c1, c2, c3};
}

// Random::nextFloat (src/libcore/random.cpp:630-639)
__device__ __forceinline__ float u01(uint32_t b)
{
    return __uint_as_float((b >> 9) | 0x3f800000u) - 1.0f;
}

// ------------------------------------------------------------- vectors --
struct F3 { float x, y, z; };
__device__ __forceinline__ F3 f3(float x, float y, float z) { return F3{x, y, z}; }
__device__ __forceinline__ F3 operator-(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ F3 operator+(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ F3 operator*(F3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ F3 neg(F3 a) { return f3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len2(F3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ float len(F3 a) { return sqrtf(len2(a)); }
__device__ __forceinline__ F3 nrm(F3 a) { const float r = 1.0f / len(a); return a * r; }
__device__ __forceinline__ float fmax3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

// Division as v_rcp_f32 (1 ulp) times the numerator: 2 VALU instead of the
// 6 of the range-checked fdiv lowering.  Operands here are far from the
// 2^+-126 limits where the two differ beyond rounding.
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fdiv(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }

// ------------------------------------------------- hyperbolic functions --
// ocml's asinhf / sinhf carry double-float intermediates and cost ~30% of the
// gather (measured, DESIGN.md "gather instruction budget").  These use the
// hardware log2 / exp2 with the cancellation-prone ranges handled explicitly;
// max relative error vs. double asinh / sinh is a few ulp (tools/mathcheck.hip).
constexpr float kLn2 = 0.69314718055994530942f;
constexpr float kLog2e = 1.44269504088896340736f;
constexpr float kLog2eLo = 1.925963033500e-8f;          // log2(e) - (float)log2(e)

// asinh(x) = log1p(|x| + x^2 / (1 + sqrt(1 + x^2))), log1p by Goldberg's
// correction log(u) * y / (u - 1), u = 1 + y; log(2|x|) beyond 2^12.
__device__ __forceinline__ float asinh_fast(float x)
{
    const float ax = fabsf(x);
    const bool big = ax > 4096.0f;
    const float s = sqrtf(fmaf(ax, ax, 1.0f));
    const float y = ax + fdiv(ax * ax, 1.0f + s);
    const float u = 1.0f + y;
    // one hardware log for both ranges: ln(u), or ln(|x|) + ln 2 = ln(2|x|)
    const float l = __builtin_amdgcn_logf(big ? ax : u) * kLn2;
    const float small = (u == 1.0f) ? y : l * fdiv(y, u - 1.0f);
    return copysignf(big ? l + kLn2 : small, x);
}

// ------------------------------------------------- circular functions --
// The Kulla sampler only evaluates tan on (-pi/2, pi/2) and atan of finite
// ratios; ocml's tanf carries a Payne-Hanek reduction for huge arguments,
// evaluated branch-free.  Cody-Waite reduction by pi/2 in three parts and the
// Cephes minimax polynomials (tanf / atanf, public domain) instead.
__device__ __forceinline__ float tan_fast(float x)     // |x| < 3*pi/4
{
    const float j = rintf(x * 0.63661977236758134308f);
    float r = fmaf(j, -1.5703125f, x);
    r = fmaf(j, -4.837512969970703125e-4f, r);
    r = fmaf(j, -7.54978995489188216e-8f, r);
    const float z = r * r;
    float p = fmaf(z, 9.38540185543e-3f, 3.11992232697e-3f);
    p = fmaf(p, z, 2.44301354525e-2f);
    p = fmaf(p, z, 5.34112807005e-2f);
    p = fmaf(p, z, 1.33387994085e-1f);
    p = fmaf(p, z, 3.33331568548e-1f);
    const float t = fmaf(p * z, r, r);
    return j != 0.0f ? -rcp(t) : t;
}

__device__ __forceinline__ float atan_fast(float x)
{
    const float ax = fabsf(x);
    const bool hi = ax > 2.414213562373095f, mid = ax > 0.4142135623730950f;
    const float num = hi ? -1.0f : (mid ? ax - 1.0f : ax);
    const float den = hi ? ax : (mid ? ax + 1.0f : 1.0f);
    const float t = fdiv(num, den);
    const float y0 = hi ? 1.57079632679489661923f : (mid ? 0.78539816339744830962f : 0.0f);
    const float z = t * t;
    float p = fmaf(z, 8.05374449538e-2f, -1.38776856032e-1f);
    p = fmaf(p, z, 1.99777106478e-1f);
    p = fmaf(p, z, -3.33329491539e-1f);
    return copysignf(y0 + fmaf(p * z, t, t), x);
}

// --------------------------------------------------- per eye segment --
struct Rec {
    float ox, oy, oz, dx, dy, dz, px, py, pz, nx, ny, nz, ar, ag, ab;
    uint32_t flags;
    float wr, wg, wb;   // path weight of the segment (LiInternal's 'weight', vrlIntegrator.cpp:503-510)
    uint32_t depth;     // bits 0-15: eye-path vertex of the segment's start (0: camera ray); bits 16-31:
                        // the sensor sample (multi-sample renders); both key its streams
};
static_assert(sizeof(Rec) == 80, "Rec layout");
constexpr uint32_t kRecAccum = 16u;   // ALVRL_REC_ACCUM: the R build adds to the row's entries

struct RecPre {
    F3 E, d, dN, P, n, B, dirAB;
    float lenAB;      // distance(A, B) of the eye Kulla segment
    float a;          // dot(u, u), u = P - E (getClosestPoints)
    float cos_wi;     // Frame::cosTheta(its.wi)
    float teus[3];    // transmittanceEUsurf (vrlIntegrator.cpp:711-719)
    float alb[3];
    float w[3];       // the segment's path weight
    uint32_t depth;
    bool medium, surf, unit;   // unit: weight (1, 1, 1)
};

// MaxExpDist::cdf (maxexp.h:83-94); the interval of t by lower_bound over
// the three starts (the first is 0)
__device__ __forceinline__ float maxexp_cdf(const DevParams& P, float d)
{
    const int i = (P.mx_start[1] < d) + (P.mx_start[2] < d);
    const float upper = -__expf(-P.mx_sigma[i] * d);
    return P.mx_cdf[i] + (upper - P.mx_lower[i]) * P.mx_inv_norm;
}

// ANY_STRATEGY: the generic-sample-count kernels serve every strategy; the
// unrolled (2, 2) kernels are launched for 'balance' only and carry no branch.
template <bool ANY_STRATEGY>
__device__ __forceinline__ void medium_tr(const DevParams& P, float d, float tr[3], float* pf)
{
    // HomogeneousMedium::eval (homogeneous.cpp:354-396): with 'balance' the
    // pdf exponentials and the transmittance exponentials are the same values.
    const float t0 = __expf(P.sigma_t[0] * (-d));
    const float t1 = __expf(P.sigma_t[1] * (-d));
    const float t2 = __expf(P.sigma_t[2] * (-d));
    float s = 0.0f;
    if (!ANY_STRATEGY || P.strategy == 0) {   // wave-uniform
        s += t0; s += t1; s += t2;
        s *= (1.0f / 3.0f);
    } else if (P.strategy == 3) {
        s = 1 - maxexp_cdf(P, d);
    } else {
        s = __expf(-P.density * d);
    }
    *pf = s * P.w + (1 - P.w);
    const bool z = fmax3(t0, t1, t2) < 1e-20f;
    tr[0] = z ? 0.0f : t0; tr[1] = z ? 0.0f : t1; tr[2] = z ? 0.0f : t2;
}

__device__ __forceinline__ void medium_tr_only(const DevParams& P, float d, float tr[3])
{
    const float t0 = __expf(P.sigma_t[0] * (-d));
    const float t1 = __expf(P.sigma_t[1] * (-d));
    const float t2 = __expf(P.sigma_t[2] * (-d));
    const bool z = fmax3(t0, t1, t2) < 1e-20f;
    tr[0] = z ? 0.0f : t0; tr[1] = z ? 0.0f : t1; tr[2] = z ? 0.0f : t2;
}

__device__ __forceinline__ RecPre prepare_record(const Rec& r, const DevParams& P)
{
    RecPre q;
    q.E = f3(r.ox, r.oy, r.oz);
    q.d = f3(r.dx, r.dy, r.dz);
    q.P = f3(r.px, r.py, r.pz);
    q.n = f3(r.nx, r.ny, r.nz);
    q.dN = nrm(q.d);
    const float edist = len(q.P - q.E);               // sampleUVKulla :869
    q.B = q.E + q.d * edist;                          // :871
    q.dirAB = nrm(q.B - q.E);
    q.lenAB = len(q.E - q.B);
    const F3 u = q.P - q.E;
    q.a = dot(u, u);
    q.cos_wi = dot(neg(q.d), q.n);
    q.alb[0] = r.ar; q.alb[1] = r.ag; q.alb[2] = r.ab;
    q.w[0] = r.wr; q.w[1] = r.wg; q.w[2] = r.wb;
    q.unit = r.wr == 1.0f && r.wg == 1.0f && r.wb == 1.0f;
    q.depth = r.depth;
    q.medium = (r.flags & 4u) != 0;
    q.teus[0] = q.teus[1] = q.teus[2] = 0.0f;
    if ((r.flags & 1u) && len(q.P - q.E) != 0) medium_tr_only(P, len(q.P - q.E), q.teus);
    q.surf = (q.teus[0] != 0 || q.teus[1] != 0 || q.teus[2] != 0) && (r.flags & 2u);
    return q;
}

__device__ __forceinline__ float phase(const DevParams& P, F3 wi, F3 wo)
{
    if (P.phase_type == 0) return kInvFourPi;
    const float g = P.g;
    const float temp = 1.0f + g * g + 2.0f * g * dot(wi, wo);
    return fdiv(kInvFourPi * (1 - g * g), temp * sqrtf(temp));
}

__device__ __forceinline__ bool spec_valid(float a, float b, float c)
{
    return isfinite(a) && isfinite(b) && isfinite(c) && a >= 0.0f && b >= 0.0f && c >= 0.0f;
}

__device__ __forceinline__ float luminance(float r, float g, float b)
{
    return r * 0.212671f + g * 0.715160f + b * 0.072169f;
}

// Equi-angular (Kulla) frame of a segment A->B w.r.t. a point D
// (KullaSampling, vrlIntegrator.cpp:889-914).  I = A + dotPr * dir is the foot
// of D on the segment's line, DI = D - I.  The reference's distance(A, I) and
// distance(I, B) are |dotPr| and |lenAB - dotPr| (I, A, B are collinear).
struct KullaFrame { F3 DI; float Dis, rDis, dotPr, aa, ab; };

// atan of two arguments with one reciprocal for both reduced ratios
// (num / den of atan_fast; den is |x|, |x| + 1 or 1, so den1 * den2 only
// overflows where both ratios are -1/|x| ~ 0, which then come out as 0)
__device__ __forceinline__ void atan2_fast(float x1, float x2, float* r1, float* r2)
{
    const float a1 = fabsf(x1), a2 = fabsf(x2);
    const bool hi1 = a1 > 2.414213562373095f, mid1 = a1 > 0.4142135623730950f;
    const bool hi2 = a2 > 2.414213562373095f, mid2 = a2 > 0.4142135623730950f;
    const float n1 = hi1 ? -1.0f : (mid1 ? a1 - 1.0f : a1), d1 = hi1 ? a1 : (mid1 ? a1 + 1.0f : 1.0f);
    const float n2 = hi2 ? -1.0f : (mid2 ? a2 - 1.0f : a2), d2 = hi2 ? a2 : (mid2 ? a2 + 1.0f : 1.0f);
    const float rr = rcp(d1 * d2);
    const float t1 = (n1 * d2) * rr, t2 = (n2 * d1) * rr;
    const float y1 = hi1 ? 1.57079632679489661923f : (mid1 ? 0.78539816339744830962f : 0.0f);
    const float y2 = hi2 ? 1.57079632679489661923f : (mid2 ? 0.78539816339744830962f : 0.0f);
    const float z1 = t1 * t1, z2 = t2 * t2;
    float p1 = fmaf(z1, 8.05374449538e-2f, -1.38776856032e-1f);
    float p2 = fmaf(z2, 8.05374449538e-2f, -1.38776856032e-1f);
    p1 = fmaf(p1, z1, 1.99777106478e-1f);
    p2 = fmaf(p2, z2, 1.99777106478e-1f);
    p1 = fmaf(p1, z1, -3.33329491539e-1f);
    p2 = fmaf(p2, z2, -3.33329491539e-1f);
    *r1 = copysignf(y1 + fmaf(p1 * z1, t1, t1), x1);
    *r2 = copysignf(y2 + fmaf(p2 * z2, t2, t2), x2);
}

__device__ __forceinline__ KullaFrame kulla_frame(F3 A, F3 dir, float lenAB, F3 D)
{
    KullaFrame k;
    const F3 w = D - A;
    k.dotPr = dot(dir, w);
    k.DI = w - dir * k.dotPr;
    // |DI| and its reciprocal from one v_rsq_f32 (Dis = 0: rDis = inf, as rcp(0))
    const float l2 = len2(k.DI);
    const float rDis = __builtin_amdgcn_rsqf(l2);
    k.Dis = l2 > 0.0f ? l2 * rDis : 0.0f;
    k.rDis = rDis;
    const float dAI = fabsf(k.dotPr);
    float aa, ab;
    atan2_fast(dAI * rDis, fabsf(lenAB - k.dotPr) * rDis, &aa, &ab);
    if (k.dotPr > 0) {
        aa = -aa;
        if (dAI > lenAB) ab = -ab;
    }
    k.aa = aa; k.ab = ab;
    return k;
}

// The sampled offset t along the segment from I (result = I + t * dir).
__device__ __forceinline__ float kulla_t(const KullaFrame& k, float u)
{
    return k.Dis * tan_fast(((1.0f - u) * k.aa) + (u * k.ab));
}

// sinh and cosh of x together (cosh for Novak's pdf, see below).
__device__ __forceinline__ void sinhcosh_fast(float x, float* sh, float* ch)
{
    const float ax = fabsf(x);
    const float x2 = ax * ax;
    const float ps = fmaf(ax * x2, fmaf(x2, fmaf(x2, 1.0f / 5040.0f, 1.0f / 120.0f), 1.0f / 6.0f), ax);
    const float pc = fmaf(x2, fmaf(x2, fmaf(x2, 1.0f / 720.0f, 1.0f / 24.0f), 0.5f), 1.0f);
    const float ph = ax * kLog2e;
    const float pl = fmaf(ax, kLog2e, -ph) + ax * kLog2eLo;
    const float e = __builtin_amdgcn_exp2f(ph) * fmaf(pl, kLn2, 1.0f);
    const float re = rcp(e);
    const bool small = ax < 0.25f;
    *sh = copysignf(small ? ps : 0.5f * (e - re), x);
    *ch = small ? pc : 0.5f * (e + re);
}

// ------------------------------------------------ two samples at once --
// The unrolled (2, 2) kernels evaluate a pair's two volVol samples, and its
// two volSurf samples, side by side: per-sample arithmetic on float pairs
// (v_pk_fma/mul/add_f32, two lanes' worth of FP32 per instruction), the
// transcendentals and selects per element.  Every value is formed by the
// same operations as the one-sample code above.
// (the R build's gathers keep the one-sample code unless ALVRL_RB_PACKED:
// their Welford statistics leave fewer registers for the pairs.  Measured on
// MI355X at C4, round 5: packed at 2 waves/SIMD (233 VGPRs, no spill) builds
// R in 41.8 ms against 36.0 ms for this default, so it stays off)
#ifndef ALVRL_RB_PACKED
#define ALVRL_RB_PACKED 0
#endif
typedef float v2f __attribute__((ext_vector_type(2)));
struct V3 { v2f x, y, z; };
__device__ __forceinline__ v2f v2(float a) { return v2f{a, a}; }
__device__ __forceinline__ v2f vfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ v2f vabs(v2f a) { return __builtin_elementwise_abs(a); }
__device__ __forceinline__ v2f vcopysign(v2f a, v2f b) { return __builtin_elementwise_copysign(a, b); }
__device__ __forceinline__ v2f vsel(bool c0, bool c1, v2f a, v2f b) { return v2f{c0 ? a.x : b.x, c1 ? a.y : b.y}; }
__device__ __forceinline__ v2f vrcp(v2f a) { return v2f{rcp(a.x), rcp(a.y)}; }

__device__ __forceinline__ void sinhcosh2(v2f x, v2f* sh, v2f* ch)
{
    const v2f ax = vabs(x);
    const v2f x2 = ax * ax;
    const v2f ps = vfma(ax * x2, vfma(x2, vfma(x2, v2(1.0f / 5040.0f), v2(1.0f / 120.0f)), v2(1.0f / 6.0f)), ax);
    const v2f pc = vfma(x2, vfma(x2, vfma(x2, v2(1.0f / 720.0f), v2(1.0f / 24.0f)), v2(0.5f)), v2(1.0f));
    const v2f ph = ax * kLog2e;
    const v2f pl = vfma(ax, v2(kLog2e), -ph) + ax * kLog2eLo;
    const v2f e = v2f{__builtin_amdgcn_exp2f(ph.x), __builtin_amdgcn_exp2f(ph.y)} * vfma(pl, v2(kLn2), v2(1.0f));
    const v2f re = vrcp(e);
    const bool s0 = ax.x < 0.25f, s1 = ax.y < 0.25f;
    *sh = vcopysign(vsel(s0, s1, ps, 0.5f * (e - re)), x);
    *ch = vsel(s0, s1, pc, 0.5f * (e + re));
}

__device__ __forceinline__ v2f tan2(v2f x)     // tan_fast per element
{
    const v2f xs = x * 0.63661977236758134308f;
    const v2f j = v2f{rintf(xs.x), rintf(xs.y)};
    v2f r = vfma(j, v2(-1.5703125f), x);
    r = vfma(j, v2(-4.837512969970703125e-4f), r);
    r = vfma(j, v2(-7.54978995489188216e-8f), r);
    const v2f z = r * r;
    v2f p = vfma(z, v2(9.38540185543e-3f), v2(3.11992232697e-3f));
    p = vfma(p, z, v2(2.44301354525e-2f));
    p = vfma(p, z, v2(5.34112807005e-2f));
    p = vfma(p, z, v2(1.33387994085e-1f));
    p = vfma(p, z, v2(3.33331568548e-1f));
    const v2f t = vfma(p * z, r, r);
    return vsel(j.x != 0.0f, j.y != 0.0f, -vrcp(t), t);
}

// atan2_fast for each element's pair (x1, x2)
__device__ __forceinline__ void atan2_2(v2f x1, v2f x2, v2f* r1, v2f* r2)
{
    const v2f a1 = vabs(x1), a2 = vabs(x2);
    const bool h10 = a1.x > 2.414213562373095f, h11 = a1.y > 2.414213562373095f;
    const bool m10 = a1.x > 0.4142135623730950f, m11 = a1.y > 0.4142135623730950f;
    const bool h20 = a2.x > 2.414213562373095f, h21 = a2.y > 2.414213562373095f;
    const bool m20 = a2.x > 0.4142135623730950f, m21 = a2.y > 0.4142135623730950f;
    const v2f n1 = vsel(h10, h11, v2(-1.0f), vsel(m10, m11, a1 - 1.0f, a1));
    const v2f d1 = vsel(h10, h11, a1, vsel(m10, m11, a1 + 1.0f, v2(1.0f)));
    const v2f n2 = vsel(h20, h21, v2(-1.0f), vsel(m20, m21, a2 - 1.0f, a2));
    const v2f d2 = vsel(h20, h21, a2, vsel(m20, m21, a2 + 1.0f, v2(1.0f)));
    const v2f rr = vrcp(d1 * d2);
    const v2f t1 = (n1 * d2) * rr, t2 = (n2 * d1) * rr;
    const v2f y1 = vsel(h10, h11, v2(1.57079632679489661923f), vsel(m10, m11, v2(0.78539816339744830962f), v2(0.0f)));
    const v2f y2 = vsel(h20, h21, v2(1.57079632679489661923f), vsel(m20, m21, v2(0.78539816339744830962f), v2(0.0f)));
    const v2f z1 = t1 * t1, z2 = t2 * t2;
    v2f p1 = vfma(z1, v2(8.05374449538e-2f), v2(-1.38776856032e-1f));
    v2f p2 = vfma(z2, v2(8.05374449538e-2f), v2(-1.38776856032e-1f));
    p1 = vfma(p1, z1, v2(1.99777106478e-1f));
    p2 = vfma(p2, z2, v2(1.99777106478e-1f));
    p1 = vfma(p1, z1, v2(-3.33329491539e-1f));
    p2 = vfma(p2, z2, v2(-3.33329491539e-1f));
    *r1 = vcopysign(y1 + vfma(p1 * z1, t1, t1), x1);
    *r2 = vcopysign(y2 + vfma(p2 * z2, t2, t2), x2);
}

struct KullaFrame2 { V3 DI; v2f Dis, rDis, dotPr, aa, ab; };
__device__ __forceinline__ KullaFrame2 kulla_frame2(F3 A, F3 dir, float lenAB, const V3& D)
{
    KullaFrame2 k;
    const V3 w{D.x - A.x, D.y - A.y, D.z - A.z};
    k.dotPr = dir.x * w.x + dir.y * w.y + dir.z * w.z;
    k.DI = V3{w.x - dir.x * k.dotPr, w.y - dir.y * k.dotPr, w.z - dir.z * k.dotPr};
    const v2f l2 = k.DI.x * k.DI.x + k.DI.y * k.DI.y + k.DI.z * k.DI.z;
    const v2f rDis = v2f{__builtin_amdgcn_rsqf(l2.x), __builtin_amdgcn_rsqf(l2.y)};
    k.Dis = vsel(l2.x > 0.0f, l2.y > 0.0f, l2 * rDis, v2(0.0f));
    k.rDis = rDis;
    const v2f dAI = vabs(k.dotPr);
    v2f aa, ab;
    atan2_2(dAI * rDis, vabs(lenAB - k.dotPr) * rDis, &aa, &ab);
    const bool p0 = k.dotPr.x > 0, p1 = k.dotPr.y > 0;
    k.aa = vsel(p0, p1, -aa, aa);
    k.ab = vsel(p0 && dAI.x > lenAB, p1 && dAI.y > lenAB, -ab, ab);
    return k;
}

// medium_tr<false> ('balance') per element
__device__ __forceinline__ void medium_tr2(const DevParams& P, v2f d, v2f tr[3], v2f* pf)
{
    const v2f nd = -d;
    const v2f e0 = P.sigma_t[0] * nd, e1 = P.sigma_t[1] * nd, e2 = P.sigma_t[2] * nd;
    const v2f t0 = v2f{__expf(e0.x), __expf(e0.y)};
    const v2f t1 = v2f{__expf(e1.x), __expf(e1.y)};
    const v2f t2 = v2f{__expf(e2.x), __expf(e2.y)};
    v2f s = v2(0.0f);
    s += t0; s += t1; s += t2;
    s *= (1.0f / 3.0f);
    *pf = s * P.w + (1 - P.w);
    const bool z0 = fmax3(t0.x, t1.x, t2.x) < 1e-20f, z1 = fmax3(t0.y, t1.y, t2.y) < 1e-20f;
    tr[0] = vsel(z0, z1, v2(0.0f), t0); tr[1] = vsel(z0, z1, v2(0.0f), t1); tr[2] = vsel(z0, z1, v2(0.0f), t2);
}

// Pair-constant part of sampleVtoDistance (:916-953) incl. getClosestPoints (:962-1032).
struct NovakFrame { float sinT, rsinT, h, rh, A0, dA, dVhS, ipdf; bool parallel, zero; };

__device__ __forceinline__ NovakFrame novak_frame(const RecPre& q, const VrlPrep& v)
{
    NovakFrame f;
    const F3 S = f3(v.sx, v.sy, v.sz);
    const float cosT = dot(q.dN, f3(v.dx, v.dy, v.dz));
    const float s2 = 1 - cosT * cosT;
    f.zero = v.len == 0.0f;                          // :920-924
    // sinT and 1 / sinT from one v_rsq_f32
    const float rs2 = __builtin_amdgcn_rsqf(s2);
    f.sinT = s2 > 0.0f ? s2 * rs2 : 0.0f;
    f.parallel = f.sinT < kEpsilon;
    f.h = f.rh = f.A0 = f.dA = f.rsinT = f.dVhS = f.ipdf = 0.0f;
    if (!f.parallel && !f.zero) {
        // getClosestPoints(E, its.p, start, end)
        const F3 u = q.P - q.E;
        const F3 vv = f3(v.vx, v.vy, v.vz);
        const F3 w = q.E - S;
        const float a = q.a, b = dot(u, vv), c = v.c, d = dot(u, w), e = dot(vv, w);
        const float D = a * c - b * b;
        float sN, sD = D, tN, tD = D;
        if (D < kEpsilon * a * c) {
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
            if ((-d + b) < 0.0f) sN = 0.0f;
            else if ((-d + b) > a) sN = sD;
            else { sN = (-d + b); sD = a; }
        }
        const float rst = rcp(sD * tD);              // |sD|, |tD| <= a c: no overflow
        const float sc = (sN * tD) * rst, tc = (tN * sD) * rst;
        const F3 dP = (w + u * sc) - vv * tc;
        const float h2 = len2(dP);
        const float rh = __builtin_amdgcn_rsqf(h2);
        f.h = h2 > 0.0f ? h2 * rh : 0.0f;
        // Vh = S + vv tc: distance(Vh, S) = |tc| len, distance(Vh, End) = |tc - 1| len
        f.dVhS = fabsf(tc) * v.len;
        const float V0c = -1 * f.dVhS;
        const float V1c = fabsf(tc - 1.0f) * v.len;
        f.rh = rh;
        const float A0 = asinh_fast((V0c * f.rh) * f.sinT);
        const float A1 = asinh_fast((V1c * f.rh) * f.sinT);
        f.A0 = A0;
        f.dA = A1 - A0;
        f.rsinT = rs2;
        // 1 / pdf = cosh(x) * h * dA / sinT (the sample's pdf without its cosh)
        f.ipdf = (f.h * f.dA) * f.rsinT;
    }
    return f;
}

// One integrateVRL evaluation (vrlIntegrator.cpp:603-785).  Returns RGB in
// out[]; *mean_out / *var_out receive the luminance mean and variance-of-mean
// contributions (:693-703, :772-782).
//
// Evaluated in reduced form; every identity below is exact in real
// arithmetic, so only float rounding separates it from the reference's
// sequence of point constructions:
//  * V = S + SV * newV, so distance(S, V) = |newV| (Novak) or u * len
//    (parallel); the vol->surf V = I + t * SV gives |dotPr + t|;
//  * U = I + t * dirAB with I = E + dotPr * dirAB, so distance(E, U) =
//    |dotPr + t|; U - V = t * dir - DI with DI perpendicular to dir, so
//    distanceSquared(U, V) = Dis^2 + t^2;
//  * Kulla's pdf is Dis / ((ab - aa)(Dis^2 + t^2)), so pdf^-1 * dist^-2 =
//    (ab - aa) / Dis (the equi-angular cancellation);
//  * Novak's 1 / sqrt(h^2 + (newV sinT)^2) with newV sinT = h sinh(x) is
//    1 / (h cosh(x)).
// Directions (VU) are formed only for the HG phase function / the BSDF cosine.
// VIS: occluders present (Scene::evalTransmittance's occluder test,
// scene.cpp:619-679: from U (a medium point, mint 0) or the surface point
// (mint Epsilon) to V, the whole segment).
__device__ __forceinline__ bool blocked(const DevParams& P, F3 p1, bool p1_surface, F3 p2)
{
    const F3 d = p2 - p1;
    const float rem = len(d);
    if (!(rem > 0.0f)) return false;
    const F3 dn = d * (1.0f / rem);
    return bvh::occluded(P.occ, bvh::mk(p1.x, p1.y, p1.z), bvh::mk(dn.x, dn.y, dn.z), p1_surface ? 1e-4f : 0.0f, rem);
}

template <int NVV, int NVS, bool WANT_STATS, bool VIS = false>
__device__ __forceinline__ void integrate_vrl(const DevParams& P, const RecPre& q, const VrlPrep& v,
                                              uint32_t rec_id, uint32_t vrl_id, uint32_t domain,
                                              int nvv_rt, int nvs_rt, float out[3], float* mean_out,
                                              float* var_out, uint32_t rsub = 0u)
{
    const int nVV = NVV >= 0 ? NVV : nvv_rt;
    const int nVS = NVS >= 0 ? NVS : nvs_rt;
    const F3 S = f3(v.sx, v.sy, v.sz);
    const F3 SV = f3(v.dx, v.dy, v.dz);
    float tot0 = 0.0f, tot1 = 0.0f, tot2 = 0.0f;
    float mean = 0.0f, M2 = 0.0f, mean_acc = 0.0f, var_acc = 0.0f;
    const uint32_t k0 = P.seed, k1 = P.pass;
    // stream word: domain, the segment's eye-path depth and the record's
    // sensor sample (its depth word's bits 16-31); the R sample index sits in
    // bits 8-23 of the block counter (a pair's draws use blocks < 2^8), so no
    // two (sensor sample, R sample) pairs of one record share a stream
    const uint32_t c3 = (domain << 24) | ((q.depth & 0xFFu) << 16) | ((q.depth >> 16) & 0xFFFFu);
    const uint32_t cr = (rsub & 0xFFFFu) << 8;

    // draws 0..3: volVol samples 0,1 (V, U); draws 4..7: volSurf / further volVol
    U4 rb = philox4x32_10(rec_id, vrl_id, cr, c3, k0, k1);
    uint32_t cur_blk = 0;
    auto draw = [&](int k) -> float {
        const uint32_t blk = (uint32_t)k >> 2;
        if (blk != cur_blk) { rb = philox4x32_10(rec_id, vrl_id, cr | blk, c3, k0, k1); cur_blk = blk; }
        const uint32_t s = k & 3;
        const uint32_t b = s == 0 ? rb.x : (s == 1 ? rb.y : (s == 2 ? rb.z : rb.w));
        return u01(b);
    };

    const NovakFrame nf = novak_frame(q, v);
    const bool hg = P.phase_type != 0;
    const float ss0 = P.sigma_s[0], ss1 = P.sigma_s[1], ss2 = P.sigma_s[2];

    // ---------------- volume -> volume (:647-703) ----------------
    if constexpr (NVV == 2 && !VIS && (!WANT_STATS || ALVRL_RB_PACKED)) {
        // both samples side by side (see "two samples at once")
        const v2f u0 = v2f{draw(0), draw(2)}, u1 = v2f{draw(1), draw(3)};
        V3 V;
        v2f ipdfV, dSV;
        if (nf.zero) {
            V = V3{v2(S.x), v2(S.y), v2(S.z)}; ipdfV = v2(1.0f); dSV = v2(0.0f);
        } else if (nf.parallel) {
            V = V3{S.x + v.vx * u0, S.y + v.vy * u0, S.z + v.vz * u0};
            ipdfV = v2(v.len);
            dSV = u0 * v.len;
        } else {
            v2f sh, ch;
            sinhcosh2(nf.A0 + (u0 * nf.dA), &sh, &ch);
            const v2f newV = vfma(nf.h * sh, v2(nf.rsinT), v2(nf.dVhS));
            V = V3{S.x + SV.x * newV, S.y + SV.y * newV, S.z + SV.z * newV};
            ipdfV = ch * nf.ipdf;
            dSV = vabs(newV);
        }
        const KullaFrame2 ke = kulla_frame2(q.E, q.dirAB, q.lenAB, V);
        const v2f t = ke.Dis * tan2(((1.0f - u1) * ke.aa) + (u1 * ke.ab));
        const v2f l2 = vfma(ke.Dis, ke.Dis, t * t);
        const v2f dUV = v2f{sqrtf(l2.x), sqrtf(l2.y)};
        const v2f dEU = vabs(ke.dotPr + t);
        const float smin = fminf(fminf(P.sigma_t[0], P.sigma_t[1]), P.sigma_t[2]);
        const v2f sd = smin * dEU;
        const bool zeu0 = sd.x > 46.0517019f, zeu1 = sd.y > 46.0517019f;
        const v2f ndUE = 0.0f - (dUV + dEU);
        v2f tue[3];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const v2f e = P.sigma_t[c] * ndUE;
            tue[c] = vsel(zeu0, zeu1, v2(0.0f), v2f{__expf(e.x), __expf(e.y)});
        }
        v2f tsv[3], pf;
        medium_tr2(P, dSV, tsv, &pf);
        const v2f g = ((ke.ab - ke.aa) * ke.rDis) * ipdfV;
        const v2f rpf = P.short_vrls ? vrcp(pf) : v2(1.0f);
        v2f ph = v2(kInvFourPi * kInvFourPi);
        if (hg) {
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const float tk = t[k], rd = rcp(dUV[k]);
                const F3 VU = (q.dirAB * tk - f3(ke.DI.x[k], ke.DI.y[k], ke.DI.z[k])) * rd;
                ph[k] = phase(P, neg(VU), neg(q.d)) * phase(P, neg(SV), VU);
            }
        }
        const v2f gg = g * rpf * ph;
        v2f c0 = v2(v.pr * (ss0 * ss0)), c1 = v2(v.pg * (ss1 * ss1)), c2 = v2(v.pb * (ss2 * ss2));
        c0 *= tsv[0] * tue[0];
        c1 *= tsv[1] * tue[1];
        c2 *= tsv[2] * tue[2];
        c0 *= gg; c1 *= gg; c2 *= gg;
        if (WANT_STATS && !q.unit) { c0 *= q.w[0]; c1 *= q.w[1]; c2 *= q.w[2]; }
#pragma unroll
        for (int sample = 0; sample < 2; ++sample) {
            float lumv = 0.0f;
            const bool live = l2[sample] != 0 && (tue[0][sample] != 0 || tue[1][sample] != 0 || tue[2][sample] != 0);
            if (live && spec_valid(c0[sample], c1[sample], c2[sample])) {
                const float rn = 1.0f / (float)nVV;
                tot0 += c0[sample] * rn; tot1 += c1[sample] * rn; tot2 += c2[sample] * rn;
                lumv = luminance(c0[sample], c1[sample], c2[sample]);
            }
            if (WANT_STATS) {
                const float delta = lumv - mean;
                mean += delta / (sample + 1);
                M2 += delta * (lumv - mean);
            }
        }
    } else {
#pragma unroll
    for (int sample = 0; sample < (NVV >= 0 ? NVV : 64); ++sample) {
        if (NVV < 0 && sample >= nVV) break;
        float lumv = 0.0f;
        const float u0 = draw(2 * sample), u1 = draw(2 * sample + 1);
        F3 V;
        float ipdfV, dSV;                           // 1 / samplingPDF of V
        if (nf.zero) {                              // sampleVtoDistance :920-924
            V = S; ipdfV = 1.0f; dSV = 0.0f;
        } else if (nf.parallel) {                   // :929-933
            V = S + f3(v.vx, v.vy, v.vz) * u0;
            ipdfV = v.len;
            dSV = u0 * v.len;
        } else {                                    // :935-952
            float sh, ch;
            sinhcosh_fast(nf.A0 + (u0 * nf.dA), &sh, &ch);
            const float newV = fmaf(nf.h * sh, nf.rsinT, nf.dVhS);
            V = S + SV * newV;
            ipdfV = ch * nf.ipdf;                   // pdf = (1 / (h cosh)) sinT / dA
            dSV = fabsf(newV);
        }
        const KullaFrame ke = kulla_frame(q.E, q.dirAB, q.lenAB, V);
        const float t = kulla_t(ke, u1);
        const float l2 = fmaf(ke.Dis, ke.Dis, t * t);
        if (l2 != 0 && !(VIS && blocked(P, q.E + q.dirAB * (ke.dotPr + t), false, V))) {
            const float dUV = sqrtf(l2);
            // T(U, V) T(E, U) in one exponential per channel, exp(-sigma_t (dUV + dEU));
            // evalTransmittance(E, U)'s clamp (every channel below 1e-20) as
            // min sigma_t * dEU > ln 1e20
            const float dEU = fabsf(ke.dotPr + t);
            const float smin = fminf(fminf(P.sigma_t[0], P.sigma_t[1]), P.sigma_t[2]);
            const bool zeu = smin * dEU > 46.0517019f;
            const float dUE = dUV + dEU;
            float tue[3];
            tue[0] = zeu ? 0.0f : __expf(P.sigma_t[0] * (0.0f - dUE));
            tue[1] = zeu ? 0.0f : __expf(P.sigma_t[1] * (0.0f - dUE));
            tue[2] = zeu ? 0.0f : __expf(P.sigma_t[2] * (0.0f - dUE));
            if (tue[0] != 0 || tue[1] != 0 || tue[2] != 0) {
                float tsv[3], pf;
                medium_tr<(NVV < 0)>(P, dSV, tsv, &pf);
                // 1 / samplingPDF / distanceSquared(U, V)
                const float g = ((ke.ab - ke.aa) * ke.rDis) * ipdfV;
                const float rpf = P.short_vrls ? rcp(pf) : 1.0f;
                float ph = kInvFourPi * kInvFourPi;
                if (hg) {
                    const F3 VU = (q.dirAB * t - ke.DI) * rcp(dUV);
                    ph = phase(P, neg(VU), neg(q.d)) * phase(P, neg(SV), VU);
                }
                const float gg = g * rpf * ph;
                float c0 = v.pr * (ss0 * ss0), c1 = v.pg * (ss1 * ss1), c2 = v.pb * (ss2 * ss2);
                c0 *= tsv[0] * tue[0];
                c1 *= tsv[1] * tue[1];
                c2 *= tsv[2] * tue[2];
                c0 *= gg; c1 *= gg; c2 *= gg;
                if (WANT_STATS && !q.unit) { c0 *= q.w[0]; c1 *= q.w[1]; c2 *= q.w[2]; }
                if (spec_valid(c0, c1, c2)) {
                    const float rn = 1.0f / (float)nVV;
                    tot0 += c0 * rn; tot1 += c1 * rn; tot2 += c2 * rn;
                    lumv = luminance(c0, c1, c2);
                }
            }
        }
        if (WANT_STATS) {
            const float delta = lumv - mean;
            mean += delta / (sample + 1);
            M2 += delta * (lumv - mean);
        }
    }
    }
    if (WANT_STATS && nVV > 0) {
        mean_acc += mean;
        var_acc += M2 / ((nVV - 1) * nVV);
    }

    // ---------------- volume -> surface (:706-782) ----------------
    if (nVS > 0) {
        mean = 0.0f; M2 = 0.0f;
        KullaFrame ks;
        float gs = 0.0f, sn = 0.0f, dn = 0.0f, base0 = 0.0f, base1 = 0.0f, base2 = 0.0f;
        if (q.surf) {
            ks = kulla_frame(S, SV, v.len, q.P);    // sampleV -> KullaSampling(S, End, Usurf)
            gs = (ks.ab - ks.aa) * ks.rDis;         // 1 / samplingPDF / distanceSquared(U, V)
            sn = dot(SV, q.n);                      // cos_wo = (t sn - dn) / dUV
            dn = dot(ks.DI, q.n);
            base0 = v.pr * ss0 * q.teus[0];
            base1 = v.pg * ss1 * q.teus[1];
            base2 = v.pb * ss2 * q.teus[2];
        }
        if constexpr (NVS == 2 && !VIS && (!WANT_STATS || ALVRL_RB_PACKED)) {
            // both samples side by side (see "two samples at once")
            v2f c0 = v2(0.0f), c1 = v2(0.0f), c2 = v2(0.0f);
            bool live0 = false, live1 = false;
            if (q.surf) {
                const v2f u = v2f{draw(2 * nVV), draw(2 * nVV + 1)};
                const v2f t = ks.Dis * tan2(((1.0f - u) * ks.aa) + (u * ks.ab));
                const v2f l2 = vfma(v2(ks.Dis), v2(ks.Dis), t * t);
                live0 = l2.x != 0; live1 = l2.y != 0;
                const v2f rdUV = v2f{__builtin_amdgcn_rsqf(l2.x), __builtin_amdgcn_rsqf(l2.y)};
                const v2f dUV = l2 * rdUV;
                const v2f ndUV = 0.0f - dUV;
                v2f tuv[3], tsv[3], pf;
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const v2f e = P.sigma_t[c] * ndUV;
                    tuv[c] = P.sigma_t[c] != 0 ? v2f{__expf(e.x), __expf(e.y)} : v2(1.0f);
                }
                medium_tr2(P, vabs(ks.dotPr + t), tsv, &pf);
                const v2f cos_wo = vfma(t, v2(sn), v2(-dn)) * rdUV;
                const bool bz0 = q.cos_wi <= 0 || cos_wo.x <= 0, bz1 = q.cos_wi <= 0 || cos_wo.y <= 0;
                const v2f fcos = vsel(bz0, bz1, v2(0.0f), kInvPi * cos_wo);
                v2f phV = v2(kInvFourPi);
                if (hg) {
#pragma unroll
                    for (int k = 0; k < 2; k++) phV[k] = phase(P, neg(SV), (ks.DI - SV * t[k]) * rdUV[k]);
                }
                const v2f rpf = P.short_vrls ? vrcp(pf) : v2(1.0f);
                const v2f gg = gs * rpf * phV * fcos;
                c0 = v2(base0 * q.alb[0]); c1 = v2(base1 * q.alb[1]); c2 = v2(base2 * q.alb[2]);
                c0 *= tsv[0] * tuv[0];
                c1 *= tsv[1] * tuv[1];
                c2 *= tsv[2] * tuv[2];
                c0 *= gg; c1 *= gg; c2 *= gg;
                if (WANT_STATS && !q.unit) { c0 *= q.w[0]; c1 *= q.w[1]; c2 *= q.w[2]; }
            }
#pragma unroll
            for (int sample = 0; sample < 2; ++sample) {
                float lumv = 0.0f;
                if ((sample == 0 ? live0 : live1) && spec_valid(c0[sample], c1[sample], c2[sample])) {
                    const float rn = 1.0f / (float)nVS;
                    tot0 += c0[sample] * rn; tot1 += c1[sample] * rn; tot2 += c2[sample] * rn;
                    lumv = luminance(c0[sample], c1[sample], c2[sample]);
                }
                if (WANT_STATS) {
                    const float delta = lumv - mean;
                    mean += delta / (sample + 1);
                    M2 += delta * (lumv - mean);
                }
            }
        } else {
#pragma unroll
        for (int sample = 0; sample < (NVS >= 0 ? NVS : 64); ++sample) {
            if (NVS < 0 && sample >= nVS) break;
            float lumv = 0.0f;
            if (q.surf) {
                const float u = draw(2 * nVV + sample);
                const float t = kulla_t(ks, u);
                const float l2 = fmaf(ks.Dis, ks.Dis, t * t);
                if (l2 != 0 && !(VIS && blocked(P, q.P, true, S + SV * (ks.dotPr + t)))) {
                    const float rdUV = __builtin_amdgcn_rsqf(l2);   // l2 > 0 here
                    const float dUV = l2 * rdUV;
                    float tuv[3], tsv[3], pf;
                    tuv[0] = P.sigma_t[0] != 0 ? __expf(P.sigma_t[0] * (0.0f - dUV)) : 1.0f;
                    tuv[1] = P.sigma_t[1] != 0 ? __expf(P.sigma_t[1] * (0.0f - dUV)) : 1.0f;
                    tuv[2] = P.sigma_t[2] != 0 ? __expf(P.sigma_t[2] * (0.0f - dUV)) : 1.0f;
                    medium_tr<(NVV < 0)>(P, fabsf(ks.dotPr + t), tsv, &pf);
                    const float cos_wo = fmaf(t, sn, -dn) * rdUV;
                    const bool bz = (q.cos_wi <= 0 || cos_wo <= 0);
                    const float fcos = bz ? 0.0f : kInvPi * cos_wo;
                    float phV = kInvFourPi;
                    if (hg) phV = phase(P, neg(SV), (ks.DI - SV * t) * rdUV);
                    const float rpf = P.short_vrls ? rcp(pf) : 1.0f;
                    const float gg = gs * rpf * phV * fcos;
                    float c0 = base0 * q.alb[0], c1 = base1 * q.alb[1], c2 = base2 * q.alb[2];
                    c0 *= tsv[0] * tuv[0];
                    c1 *= tsv[1] * tuv[1];
                    c2 *= tsv[2] * tuv[2];
                    c0 *= gg; c1 *= gg; c2 *= gg;
                    if (WANT_STATS && !q.unit) { c0 *= q.w[0]; c1 *= q.w[1]; c2 *= q.w[2]; }
                    if (spec_valid(c0, c1, c2)) {
                        const float rn = 1.0f / (float)nVS;
                        tot0 += c0 * rn; tot1 += c1 * rn; tot2 += c2 * rn;
                        lumv = luminance(c0, c1, c2);
                    }
                }
            }
            if (WANT_STATS) {
                const float delta = lumv - mean;
                mean += delta / (sample + 1);
                M2 += delta * (lumv - mean);
            }
        }
        }
        if (WANT_STATS) {
            mean_acc += mean;
            var_acc += M2 / ((nVS - 1) * nVS);
        }
    }
    out[0] = tot0; out[1] = tot1; out[2] = tot2;
    if (WANT_STATS) { *mean_out = mean_acc; *var_out = var_acc; }
}

// refine_jobs' device scratch, kept by a context between calls (refine.hip)
struct RefineArenas {
    char* arena = nullptr;
    char* tarena = nullptr;
    char* varena = nullptr;           // the kernel's Common and the jobs' views (k_views)
    size_t arena_cap = 0, tarena_cap = 0, varena_cap = 0;
    void release();
};

}  // namespace alvrl
