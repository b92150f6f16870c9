/*
 * detmath.h -- deterministic transcendental functions for the bit-exact paths.
 *
 * The reference evaluates the float functions of its samplers and media with
 * the host libm: expf/logf through math::fastexp/fastlog (double exp/log,
 * include/mitsuba/core/math.h:175-199), atanf and tanf in KullaSampling
 * (vrlIntegrator.cpp:889-914), asinhf and sinhf in sampleVtoDistance
 * (:916-957).  glibc and the device library (ocml) round those differently in
 * the last place, so nothing built on them can be compared bit for bit across
 * host and device.  These definitions evaluate each function in double with
 * IEEE +, -, *, / and sqrt only (range reduction plus a truncated series,
 * relative error ~1e-16) and round once to float.  The float results are
 * therefore the correctly rounded values except in cases a few ulps of double
 * wide around a float rounding boundary (tests/test_detmath.py pins them
 * against mpmath), and they are the SAME bits on every compiler that honours
 * IEEE double arithmetic without contraction:
 *
 *   - the oracle (oracle/, gcc -ffp-contract=off),
 *   - the host tracer (csrc/host/scene.cpp, g++ -ffp-contract=off),
 *   - the strict device kernels (csrc/rbuild_strict.hip, csrc/tracer.hip,
 *     hipcc -ffp-contract=off; f64 division and sqrt are correctly rounded).
 *
 * Include it ONLY from translation units built without FMA contraction.
 * Plain C99 / C++17 / HIP: hex-float constants, no tables.
 */
#ifndef ALVRL_DETMATH_H
#define ALVRL_DETMATH_H

#include <stdint.h>
#include <math.h>

#if defined(__HIP__)
#define DM_FN static inline __host__ __device__
#else
#define DM_FN static inline
#endif

#define DM_LN2_HI   0x1.62e42fee00000p-1   /* 33 significant bits: k * LN2_HI is exact */
#define DM_LN2_LO   0x1.a39ef35793c76p-33
#define DM_LN2      0x1.62e42fefa39efp-1
#define DM_LOG2E    0x1.71547652b82fep+0
#define DM_SQRT2    0x1.6a09e667f3bcdp+0
#define DM_PIO2     0x1.921fb54442d18p+0
#define DM_PIO4     0x1.921fb54442d18p-1
#define DM_PIO2_1   0x1.921fb54400000p+0   /* 33 significant bits of pi/2 */
#define DM_PIO2_1T  0x1.0b4611a626331p-34  /* pi/2 - DM_PIO2_1 */
#define DM_TWOOPI   0x1.45f306dc9c883p-1
#define DM_TANPI8   0x1.a827999fcef32p-2

DM_FN double dm_bits_to_d(uint64_t b) { double d; __builtin_memcpy(&d, &b, 8); return d; }
DM_FN uint64_t dm_d_to_bits(double d) { uint64_t b; __builtin_memcpy(&b, &d, 8); return b; }
DM_FN double dm_inf(void) { return dm_bits_to_d(0x7ff0000000000000ull); }
DM_FN double dm_nan(void) { return dm_bits_to_d(0x7ff8000000000000ull); }

/* 2^k for k in [-1022, 1023] */
DM_FN double dm_pow2i(int k) { return dm_bits_to_d((uint64_t)(k + 1023) << 52); }

/* exp(x).  Results below 2^-150 or above 2^128 leave the float range, so
 * |x| is clamped there: x < -110 -> 0, x > 100 -> inf. */
DM_FN double dm_exp(double x)
{
    if (x != x) return x;
    if (x > 100.0) return dm_inf();
    if (x < -110.0) return 0.0;
    const double kd = floor(x * DM_LOG2E + 0.5);
    const double r = (x - kd * DM_LN2_HI) - kd * DM_LN2_LO;   /* |r| <= 0.347 */
    /* sum_{n <= 13} r^n / n!  (truncation r^14 / 14! < 5e-18) */
    double p = 0x1.6124613a86d09p-33;
    p = p * r + 0x1.1eed8eff8d898p-29;
    p = p * r + 0x1.ae64567f544e4p-26;
    p = p * r + 0x1.27e4fb7789f5cp-22;
    p = p * r + 0x1.71de3a556c734p-19;
    p = p * r + 0x1.a01a01a01a01ap-16;
    p = p * r + 0x1.a01a01a01a01ap-13;
    p = p * r + 0x1.6c16c16c16c17p-10;
    p = p * r + 0x1.1111111111111p-7;
    p = p * r + 0x1.5555555555555p-5;
    p = p * r + 0x1.5555555555555p-3;
    p = p * r + 0x1.0000000000000p-1;
    p = p * r + 1.0;
    p = p * r + 1.0;
    return p * dm_pow2i((int)kd);
}

/* log(x): x = m 2^e with m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s),
 * s = (m - 1) / (m + 1), |s| <= 0.1716 (series to s^23, truncation < 1e-18) */
DM_FN double dm_log(double x)
{
    if (x != x) return x;
    if (x <= 0.0) return x == 0.0 ? -dm_inf() : dm_nan();
    if (x == dm_inf()) return x;
    int e = 0;
    if (x < 0x1p-1022) { x = x * 0x1p54; e = -54; }
    const uint64_t b = dm_d_to_bits(x);
    e += (int)((b >> 52) & 0x7ff) - 1023;
    double m = dm_bits_to_d((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
    if (m > DM_SQRT2) { m = m * 0.5; e = e + 1; }
    const double f = m - 1.0;                 /* exact (Sterbenz) */
    const double s = f / (2.0 + f);
    const double z = s * s;
    double p = 0x1.642c8590b2164p-5;
    p = p * z + 0x1.8618618618618p-5;
    p = p * z + 0x1.af286bca1af28p-5;
    p = p * z + 0x1.e1e1e1e1e1e1ep-5;
    p = p * z + 0x1.1111111111111p-4;
    p = p * z + 0x1.3b13b13b13b14p-4;
    p = p * z + 0x1.745d1745d1746p-4;
    p = p * z + 0x1.c71c71c71c71cp-4;
    p = p * z + 0x1.2492492492492p-3;
    p = p * z + 0x1.999999999999ap-3;
    p = p * z + 0x1.5555555555555p-2;
    p = p * z + 1.0;
    const double lm = (2.0 * s) * p;
    const double ed = (double)e;
    return ed * DM_LN2_HI + (ed * DM_LN2_LO + lm);
}

/* log(1 + y), y >= 0, with Goldberg's correction for the rounding of 1 + y */
DM_FN double dm_log1p(double y)
{
    const double u = 1.0 + y;
    if (u == 1.0) return y;
    return dm_log(u) * (y / (u - 1.0));
}

/* asinh(x) = log1p(|x| + x^2 / (1 + sqrt(1 + x^2))) */
DM_FN double dm_asinh(double x)
{
    const double a = fabs(x);
    double r;
    if (a < 0x1p-28) r = a;
    else if (a > 0x1p28) r = dm_log(a) + DM_LN2;
    else r = dm_log1p(a + (a * a) / (1.0 + sqrt(1.0 + a * a)));
    return x < 0.0 ? -r : r;
}

/* sinh(x): Taylor series below 1 (to x^19 / 19!), (e^a - e^-a) / 2 above */
DM_FN double dm_sinh(double x)
{
    if (x != x) return x;
    const double a = fabs(x);
    double r;
    if (a < 0x1p-28) {
        r = a;
    } else if (a < 1.0) {
        const double z = a * a;
        double p = 0x1.2f49b46814157p-57;
        p = p * z + 0x1.952c77030ad4ap-49;
        p = p * z + 0x1.ae7f3e733b81fp-41;
        p = p * z + 0x1.6124613a86d09p-33;
        p = p * z + 0x1.ae64567f544e4p-26;
        p = p * z + 0x1.71de3a556c734p-19;
        p = p * z + 0x1.a01a01a01a01ap-13;
        p = p * z + 0x1.1111111111111p-7;
        p = p * z + 0x1.5555555555555p-3;
        r = a + (a * z) * p;
    } else {
        const double e = dm_exp(a);
        r = 0.5 * e - 0.5 / e;
    }
    return x < 0.0 ? -r : r;
}

/* atan(x): atan(a) = pi/2 - atan(1/a) above 1, pi/4 + atan((t-1)/(t+1))
 * above tan(pi/8); series to t^43 on |t| <= 0.4143 (truncation < 1e-18) */
DM_FN double dm_atan(double x)
{
    if (x != x) return x;
    const double a = fabs(x);
    const int inv = a > 1.0;
    double t = inv ? 1.0 / a : a;
    const int mid = t > DM_TANPI8;
    if (mid) t = (t - 1.0) / (t + 1.0);
    const double z = t * t;
    double p = -0x1.7d05f417d05f4p-6;
    p = p * z + 0x1.8f9c18f9c18fap-6;
    p = p * z + -0x1.a41a41a41a41ap-6;
    p = p * z + 0x1.bacf914c1bad0p-6;
    p = p * z + -0x1.d41d41d41d41dp-6;
    p = p * z + 0x1.f07c1f07c1f08p-6;
    p = p * z + -0x1.0842108421084p-5;
    p = p * z + 0x1.1a7b9611a7b96p-5;
    p = p * z + -0x1.2f684bda12f68p-5;
    p = p * z + 0x1.47ae147ae147bp-5;
    p = p * z + -0x1.642c8590b2164p-5;
    p = p * z + 0x1.8618618618618p-5;
    p = p * z + -0x1.af286bca1af28p-5;
    p = p * z + 0x1.e1e1e1e1e1e1ep-5;
    p = p * z + -0x1.1111111111111p-4;
    p = p * z + 0x1.3b13b13b13b14p-4;
    p = p * z + -0x1.745d1745d1746p-4;
    p = p * z + 0x1.c71c71c71c71cp-4;
    p = p * z + -0x1.2492492492492p-3;
    p = p * z + 0x1.999999999999ap-3;
    p = p * z + -0x1.5555555555555p-2;
    p = p * z + 1.0;
    double r = t * p;
    if (mid) r = DM_PIO4 + r;
    if (inv) r = DM_PIO2 - r;
    return x < 0.0 ? -r : r;
}

/* tan(x) for |x| < 2^19: x = k pi/2 + r (Cody-Waite, two parts),
 * |r| <= pi/4, sin r / cos r by their series to r^21 / r^20 */
DM_FN double dm_tan(double x)
{
    if (x != x || fabs(x) == dm_inf()) return dm_nan();
    const double kd = floor(x * DM_TWOOPI + 0.5);
    const double r = (x - kd * DM_PIO2_1) - kd * DM_PIO2_1T;
    const double z = r * r;
    double s = 0x1.71b8ef6dcf572p-66;
    s = s * z + -0x1.2f49b46814157p-57;
    s = s * z + 0x1.952c77030ad4ap-49;
    s = s * z + -0x1.ae7f3e733b81fp-41;
    s = s * z + 0x1.6124613a86d09p-33;
    s = s * z + -0x1.ae64567f544e4p-26;
    s = s * z + 0x1.71de3a556c734p-19;
    s = s * z + -0x1.a01a01a01a01ap-13;
    s = s * z + 0x1.1111111111111p-7;
    s = s * z + -0x1.5555555555555p-3;
    const double sn = r + (r * z) * s;
    double c = 0x1.e542ba4020225p-62;
    c = c * z + -0x1.6827863b97d97p-53;
    c = c * z + 0x1.ae7f3e733b81fp-45;
    c = c * z + -0x1.93974a8c07c9dp-37;
    c = c * z + 0x1.1eed8eff8d898p-29;
    c = c * z + -0x1.27e4fb7789f5cp-22;
    c = c * z + 0x1.a01a01a01a01ap-16;
    c = c * z + -0x1.6c16c16c16c17p-10;
    c = c * z + 0x1.5555555555555p-5;
    c = c * z + -0x1.0000000000000p-1;
    const double cs = 1.0 + z * c;
    const int64_t k = (int64_t)kd;
    return (k & 1) ? -(cs / sn) : sn / cs;
}

/* the float functions of the reference, rounded once from double */
DM_FN float dm_expf(float x) { return (float)dm_exp((double)x); }
DM_FN float dm_logf(float x) { return (float)dm_log((double)x); }
DM_FN float dm_atanf(float x) { return (float)dm_atan((double)x); }
DM_FN float dm_tanf(float x) { return (float)dm_tan((double)x); }
DM_FN float dm_asinhf(float x) { return (float)dm_asinh((double)x); }
DM_FN float dm_sinhf(float x) { return (float)dm_sinh((double)x); }

#endif /* ALVRL_DETMATH_H */
