/*
 * detmath_fast.h -- device evaluation of detmath.h's float functions, bit for
 * bit, at a fraction of the cost.
 *
 * dm_expf, dm_atanf, dm_tanf, dm_asinhf and dm_sinhf (detmath.h) round a
 * double evaluation whose relative error is ~1e-16 once to float; the oracle,
 * the host tracer and the strict device kernels share them.  Their truncated
 * series without FMA cost 40-80 f64 operations per call, and the strict R build
 * makes ~44 such calls per VRL pair.
 *
 * fx_*f below reach the same float by Ziv's rounding test:
 *
 *   1. a short evaluation in f64 with explicit fma (Cody-Waite reduction and
 *      near-minimax polynomials fitted by tools/detmath_fast_coeffs.py; division
 *      and square root by v_rcp_f64 / v_rsq_f64 plus Newton steps) whose
 *      relative error stays below 2^-43;
 *   2. the float rounding of that value is taken only when it is unambiguous:
 *      the 29 mantissa bits that rounding to float drops must lie further than
 *      kFxBand units of 2^-52 from the halfway point 2^28, i.e. the exact value
 *      and detmath's value (both within 2^-43 relative of the fast one) fall on
 *      the same side of the same float rounding boundary;
 *   3. otherwise -- and for inputs outside the fast range (NaN, infinities,
 *      results near the float subnormal or overflow range, tiny arguments) --
 *      the lane evaluates detmath.h itself: fx_*f per call, or, with the
 *      fx_*f_r forms that only raise a flag, the caller re-evaluates its whole
 *      unit of work (the strict R build: one R entry) with detmath.h.
 *
 * The identity fx_*f(x) == dm_*f(x) is checked for ALL 2^32 float inputs on
 * the device (alvrl_detmath_exhaustive, tests/test_gpu_strict.py), so the
 * strict kernels that use these stay the oracle's arithmetic bit for bit.  The
 * slow branch runs for about one lane in 2^16 (the band) plus the out-of-range
 * inputs, so a wave almost never takes it.
 *
 * Device only (the host keeps detmath.h).  Built without contraction like
 * every strict translation unit; the fmas here are explicit.
 */
#ifndef ALVRL_DETMATH_FAST_H
#define ALVRL_DETMATH_FAST_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "detmath.h"

#define FX_FN static __device__ __forceinline__

// Half-width of the ambiguous band around the float halfway point, in units
// of the double's last place: 2^10 ulp of double is at least 2^-43 relative,
// 4x the largest fast-path error bound (the fits' 2^-45.1 plus evaluation
// rounding) and well above detmath.h's own error (~2 ulp).
#ifndef ALVRL_FX_BAND
#define ALVRL_FX_BAND (1u << 10)
#endif
constexpr uint32_t kFxBand = ALVRL_FX_BAND;

// true when rounding y to float could depend on the last 2^-41 of y
FX_FN bool fx_near_half(double y)
{
    const uint32_t lo = (uint32_t)__double_as_longlong(y) & 0x1FFFFFFFu;
    return (lo - (0x10000000u - kFxBand)) < 2u * kFxBand;
}

FX_FN double fx_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// A polynomial coefficient as the scalar operand of its v_fma_f64: the empty
// asm ties the constant to an SGPR pair and, through its dependence on the
// step's VGPR input, keeps it from being hoisted, shared or kept live (without
// it the compiler moves each coefficient into a VGPR pair, two v_mov_b32 per
// step).  Not volatile: the steps of independent chains still interleave.
FX_FN double fx_kd(double c, double dep)
{
#ifndef ALVRL_FX_VCONST   // developer A/B: leave the constants to the compiler
    asm("" : "+s"(c) : "v"(dep));
#endif
    return c;
}

// 1 / d with two Newton steps on v_rcp_f64 (relative error ~2^-52, not
// correctly rounded; d normal and finite)
FX_FN double fx_rcp(double d)
{
    double r = __builtin_amdgcn_rcp(d);
    double e = fx_fma(-d, r, 1.0);
    r = fx_fma(r, e, r);
    e = fx_fma(-d, r, 1.0);
    return fx_fma(r, e, r);
}

// sqrt(s) for s >= 1 (finite): v_rsq_f64 refined by Goldschmidt steps
FX_FN double fx_sqrt(double s)
{
    const double y = __builtin_amdgcn_rsq(s);
    double g = s * y, h = 0.5 * y;
    double r = fx_fma(-g, h, 0.5);
    g = fx_fma(g, r, g);
    h = fx_fma(h, r, h);
    r = fx_fma(-g, h, 0.5);
    g = fx_fma(g, r, g);
    h = fx_fma(h, r, h);
    const double d = fx_fma(-g, g, s);
    return fx_fma(d, h, g);
}

// exp(x), |x| <= 87.5: x = k ln2 + r, |r| <= ln2/2, degree-9 fit (2^-45.6)
FX_FN double fx_exp_core(double x)
{
    const double t = fx_fma(x, DM_LOG2E, 0x1.8p52);      // k in the low word (round to nearest)
    const double kd = t - 0x1.8p52;
    const int k = (int)(uint32_t)__double_as_longlong(t);
    double r = fx_fma(kd, -DM_LN2, x);
    r = fx_fma(kd, -0x1.abc9e3b39803fp-56, r);     // ln2 - DM_LN2
    double p = fx_fma(r, 0x1.72e1082a74e98p-19, 0x1.a17df15fe496fp-16);
    p = fx_fma(p, r, fx_kd(0x1.a01994c7f6f2cp-13, p));
    p = fx_fma(p, r, fx_kd(0x1.6c162bb7680d6p-10, p));
    p = fx_fma(p, r, fx_kd(0x1.11111123bf2a8p-7, p));
    p = fx_fma(p, r, fx_kd(0x1.55555588b87a9p-5, p));
    p = fx_fma(p, r, fx_kd(0x1.5555555550d87p-3, p));
    p = fx_fma(p, r, fx_kd(0x1.ffffffffe74efp-2, p));
    p = fx_fma(p, r, fx_kd(0x1.0000000000006p+0, p));
    p = fx_fma(p, r, fx_kd(0x1.000000000003dp+0, p));
    return __builtin_amdgcn_ldexp(p, k);
}

// The _r forms return the fast float and set `slow` when it may differ from
// detmath's; the plain forms fall back lane by lane.
FX_FN float fx_expf_r(float x, bool& slow)
{
    const double y = fx_exp_core((double)x);
    // |x| <= 87: the result is a normal float (exp(-87) > 2^-126)
    slow |= !(__builtin_fabsf(x) <= 87.0f) || fx_near_half(y);
    return (float)y;
}

// atan(x): |x| reduced to |t| <= tan(pi/8) with one division
// (t = x, (x - 1)/(x + 1) or -1/x), degree-8 fit of atan(t)/t in t^2 (2^-45.1)
FX_FN float fx_atanf_r(float x, bool& slow)
{
    const double a = __builtin_fabs((double)x);
    const bool hi = a > 0x1.3504f333f9de6p+1;            // tan(3 pi/8)
    const bool mid = !hi && a > DM_TANPI8;
    const double num = hi ? -1.0 : mid ? a - 1.0 : a;
    const double den = hi ? a : mid ? a + 1.0 : 1.0;
    const double t = num * fx_rcp(den);
    const double q = hi ? 2.0 : mid ? 1.0 : 0.0;          // base = q pi/4 (DM_PIO2 = 2 DM_PIO4)
    const double z = t * t;
    double p = fx_fma(z, 0x1.f65f98a1a15d0p-6, -0x1.e13d4fe5e8178p-5);
    p = fx_fma(p, z, fx_kd(0x1.35cf2e1e8527dp-4, p));
    p = fx_fma(p, z, fx_kd(-0x1.73d9d7288a2a9p-4, p));
    p = fx_fma(p, z, fx_kd(0x1.c714d4c310c52p-4, p));
    p = fx_fma(p, z, fx_kd(-0x1.2492291db18d8p-3, p));
    p = fx_fma(p, z, fx_kd(0x1.99999911d787dp-3, p));
    p = fx_fma(p, z, fx_kd(-0x1.55555554e6115p-2, p));
    p = fx_fma(p, z, fx_kd(0x1.fffffffffff0fp-1, p));
    const double r = fx_fma(q, DM_PIO4, t * p);
    const double y = x < 0.0f ? -r : r;
    // 2^-60 <= |x| <= 2^60: normal float results, no tiny-argument edge;
    // atan(+-0) = +0 as in detmath
    const bool zero = x == 0.0f;
    slow |= !zero && (!(a >= 0x1p-60 && a <= 0x1p60) || fx_near_half(y));
    return zero ? 0.0f : (float)y;
}

// tan(x), |x| <= 2^16: x = k pi/2 + r, |r| <= pi/4 (+), sin r / cos r
// (degree-5 / 6 fits in r^2: 2^-47.6, 2^-52.7), one division
FX_FN float fx_tanf_r(float x, bool& slow)
{
    const double xd = (double)x;
    const double tk = fx_fma(xd, DM_TWOOPI, 0x1.8p52);
    const double kd = tk - 0x1.8p52;
    const uint32_t k = (uint32_t)__double_as_longlong(tk);
    double r = fx_fma(kd, -DM_PIO2, xd);
    r = fx_fma(kd, -0x1.1a62633145c07p-54, r);    // pi/2 - DM_PIO2
    const double z = r * r;
    double s = fx_fma(z, -0x1.a9507e8da2551p-26, 0x1.71d73179b8864p-19);
    s = fx_fma(s, z, fx_kd(-0x1.a019f8a2044d2p-13, s));
    s = fx_fma(s, z, fx_kd(0x1.1111110bde5b7p-7, s));
    s = fx_fma(s, z, fx_kd(-0x1.5555555550efdp-3, s));
    s = fx_fma(s, z, fx_kd(0x1.fffffffffffd9p-1, s));
    const double sn = r * s;
    double c = fx_fma(z, 0x1.1b8af4e3db6c4p-29, -0x1.27df4008bd308p-22);
    c = fx_fma(c, z, fx_kd(0x1.a019f7fd83c78p-16, c));
    c = fx_fma(c, z, fx_kd(-0x1.6c16c163c5a2dp-10, c));
    c = fx_fma(c, z, fx_kd(0x1.555555554e7ebp-5, c));
    c = fx_fma(c, z, fx_kd(-0x1.fffffffffff79p-2, c));
    c = fx_fma(c, z, 1.0);
    const bool odd = k & 1u;
    const double num = odd ? -c : sn;
    const double den = odd ? sn : c;
    const double y = num * fx_rcp(den);
    // 2^-30 <= |x| <= 2^16, and |r| >= 2^-40 so the quotient stays in range
    const float ax = __builtin_fabsf(x);
    slow |= !(ax >= 0x1p-30f && ax <= 0x1p16f) || !(__builtin_fabs(r) >= 0x1p-40) || fx_near_half(y);
    return (float)y;
}

// asinh(x), a = |x|:
//   2^-6 <= a <= 2^20: log(w), w = a + sqrt(1 + a^2) = m 2^e with m in
//     [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m - 1)/(m + 1) (m - 1
//     exact), degree-5 fit of atanh(s)/s in s^2 (2^-45.1); w's rounding
//     (2^-52 absolute) stays below 2^-46 relative for a >= 2^-6;
//   a < 2^-6: a (1 - z/6 + 3z^2/40 - 5z^3/112), z = a^2 <= 2^-12 (series
//     remainder 35 z^4 / 1152 < 2^-53)
FX_FN float fx_asinhf_r(float x, bool& slow)
{
    const double a = __builtin_fabs((double)x);
    const double w = a + fx_sqrt(fx_fma(a, a, 1.0));
    int e = __builtin_amdgcn_frexp_exp(w);
    double m = __builtin_amdgcn_frexp_mant(w);               // [1/2, 1)
    const bool up = m < DM_SQRT2 * 0.5;
    m = up ? m * 2.0 : m;
    e = up ? e - 1 : e;
    const double s = (m - 1.0) * fx_rcp(m + 1.0);
    const double z = s * s;
    double p = fx_fma(z, 0x1.9192e67b031d5p-4, 0x1.c620ee4c22144p-4);
    p = fx_fma(p, z, fx_kd(0x1.2494381f492efp-3, p));
    p = fx_fma(p, z, fx_kd(0x1.9999962c0518cp-3, p));
    p = fx_fma(p, z, fx_kd(0x1.5555555671492p-2, p));
    p = fx_fma(p, z, fx_kd(0x1.fffffffffff12p-1, p));
    const double rl = fx_fma((double)e, DM_LN2, (2.0 * s) * p);
    const double za = a * a;
    double q = fx_fma(za, -5.0 / 112.0, 3.0 / 40.0);
    q = fx_fma(q, za, -1.0 / 6.0);
    q = fx_fma(q, za, 1.0);
    const double r = a < 0x1p-6 ? a * q : rl;
    const double y = x < 0.0f ? -r : r;
    const bool zero = x == 0.0f;                             // asinh(+-0) = +0 (detmath)
    slow |= !zero && (!(a >= 0x1p-60 && a <= 0x1p20) || fx_near_half(y));
    return zero ? 0.0f : (float)y;
}

// sinh(x): |x| < 1: x P(x^2) (degree-6 fit of sinh(a)/a, 2^-52.2);
// 1 <= |x| <= 87: (e - 1/e) / 2 with the exp above
FX_FN float fx_sinhf_r(float x, bool& slow)
{
    const double a = __builtin_fabs((double)x);
    double r;
    if (a < 1.0) {
        const double z = a * a;
        double p = fx_fma(z, 0x1.6712f2e298972p-33, 0x1.ae53fbcbba646p-26);
        p = fx_fma(p, z, fx_kd(0x1.71de50a983cefp-19, p));
        p = fx_fma(p, z, fx_kd(0x1.a01a0180d218ap-13, p));
        p = fx_fma(p, z, fx_kd(0x1.1111111125edbp-7, p));
        p = fx_fma(p, z, fx_kd(0x1.5555555555407p-3, p));
        p = fx_fma(p, z, 1.0);
        r = a * p;
    } else {
        const double e = fx_exp_core(a);
        r = fx_fma(0.5, e, -0.5 * fx_rcp(e));
    }
    const double y = x < 0.0f ? -r : r;
    slow |= !(a >= 0x1p-20 && a <= 87.0) || fx_near_half(y);
    return (float)y;
}

// a / b in IEEE single precision, correctly rounded: the core of the
// compiler's IEEE expansion (v_rcp_f32, one Newton step, the quotient and two
// residual corrections) without v_div_scale / v_div_fmas / v_div_fixup, which
// only act on extreme exponents and special values: the flag is raised unless
// |b| and |a| (or a = +-0) lie in [2^-40, 2^40], where the scaling is the
// identity and every intermediate stays finite.  A zero numerator returns its
// own signed zero quotient (a * (1/b)).  Checked against IEEE division on 2^34
// random operand pairs over all exponents (alvrl_detmath_div_check).
FX_FN float fx_divf_r(float a, float b, bool& slow)
{
    float y = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    const float q0 = a * y;
    float r = __builtin_fmaf(-b, q0, a);
    float q = __builtin_fmaf(r, y, q0);
    r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    const uint32_t ea = __float_as_uint(a) & 0x7FFFFFFFu, eb = __float_as_uint(b) & 0x7FFFFFFFu;
    slow |= (eb - 0x2B800000u) > (0x53800000u - 0x2B800000u) ||
            (ea != 0u && (ea - 0x2B800000u) > (0x53800000u - 0x2B800000u));
    return ea == 0u ? q0 : q;
}

// sqrtf(x), correctly rounded, for x = +0 and 2^-100 <= x <= 2^100 (flag
// otherwise): v_sqrt_f32 (within 1 ulp) and the one-ulp correction of the
// compiler's IEEE expansion, without its denormal scaling and special-value
// fix-ups.  x = +0: v_sqrt gives +0 and neither correction applies (y - 1 ulp
// is a NaN, fma(-(y + 1 ulp), +0, +0) = +0).  Checked against IEEE sqrtf on
// every float (alvrl_detmath_exhaustive fn 6).
FX_FN float fx_sqrtf_r(float x, bool& slow)
{
    const float y = __builtin_amdgcn_sqrtf(x);
    const float ym = __uint_as_float(__float_as_uint(y) - 1u);
    const float yp = __uint_as_float(__float_as_uint(y) + 1u);
    float r = __builtin_fmaf(-ym, y, x) <= 0.0f ? ym : y;
    r = __builtin_fmaf(-yp, y, x) > 0.0f ? yp : r;
    slow |= x != 0.0f && (__float_as_uint(x) - 0x0D800000u) > (0x71800000u - 0x0D800000u);   // [2^-100, 2^100]
    return r;
}

FX_FN float fx_divf(float a, float b)
{
    bool slow = false;
    float q = fx_divf_r(a, b, slow);
    if (slow) q = a / b;
    return q;
}

FX_FN float fx_sqrtf(float x)
{
    bool slow = false;
    float y = fx_sqrtf_r(x, slow);
    if (slow) y = sqrtf(x);
    return y;
}

#define FX_PLAIN(name)                                      \
    FX_FN float fx_##name##f(float x)                       \
    {                                                       \
        bool slow = false;                                  \
        float y = fx_##name##f_r(x, slow);                  \
        if (slow) y = dm_##name##f(x);                      \
        return y;                                           \
    }
FX_PLAIN(exp)
FX_PLAIN(atan)
FX_PLAIN(tan)
FX_PLAIN(asinh)
FX_PLAIN(sinh)
#undef FX_PLAIN

#endif /* ALVRL_DETMATH_FAST_H */
