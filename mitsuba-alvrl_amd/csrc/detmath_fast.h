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
// of the double's last place: 2^13 ulp of double is at least 2^-40 relative,
// 5x the largest fast-path error bound (2^-42.5: exp's Taylor q, reduction
// and table; the other fits' <= 2^-43.5, plus evaluation rounding) and well
// above detmath.h's own error (~2 ulp).  A lane lands in the band once in
// 2^15 calls (~44 calls per R entry: 0.13 % of the entries go to the fix-up
// queue, whose re-evaluation costs well under 1 % of the build).
#ifndef ALVRL_FX_BAND
#define ALVRL_FX_BAND (1u << 13)
#endif
constexpr uint32_t kFxBand = ALVRL_FX_BAND;

// true when rounding y to float could depend on the last 2^-41 of y
FX_FN bool fx_near_half(double y)
{
    const uint32_t lo = (uint32_t)__double_as_longlong(y) & 0x1FFFFFFFu;
    return (lo - (0x10000000u - kFxBand)) < 2u * kFxBand;
}

// The flags of one unit of work (the strict R build: one R entry) as running
// extremes instead of a boolean per operation.  A flag per operation costs a
// compare and a lane-mask OR each (and, at every divergent join, a mask
// merged into a VGPR): with ~120 checked operations per entry the flags were
// 18 % of the build (profiles/r06/ab/strict_flags_r6b.txt).  Here each checked
// operand adds one or two integer operations to a running minimum / maximum,
// and the flag is read once per entry (fx_range_slow).  Every predicate below
// flags at least what the per-operation form flags (the boolean sink of the
// same functions), so the exhaustive checks of that form carry over:
//
//   q_*: the operands of fx_divf / fx_rcpf in the doubled frame w = 2 (bits &
//        0x7FFFFFFF) - 2 (the shift drops the sign; +-0 wraps to 0xFFFFFFFE):
//        a divisor must satisfy w in [2 (L - 1), 2 (H - 1)], L = bits(2^-40),
//        H = bits(2^40) -- so a zero, tiny, huge or non-finite one is flagged;
//        a numerator enters the minimum as w (zero passes, as in fx_divf_r) and
//        the maximum as 2 (bits & 0x7FFFFFFF) (zero passes; |a| = 2^40 itself
//        is flagged, which fx_divf_r does not: conservative);
//   s_*: fx_sqrtf's argument bits (sign included) in the maximum, bits - 1 in
//        the minimum: +0 passes, every negative value (-0 included, which
//        fx_sqrtf_r lets through: conservative) and every value outside
//        [2^-100, 2^100] is flagged;
//   h_mn: the rounding test of the transcendentals, min over calls of
//        8 (lo29 - (2^28 - band)) mod 2^32, flagged below 8 (2 band) --
//        exactly fx_near_half's predicate;
//   slow: the transcendentals' argument ranges, as in their boolean form.
struct FxRange {
    uint32_t q_mx, q_mn, s_mx, s_mn, h_mn;
    bool slow;
};
constexpr uint32_t kFxQLo = 2u * (0x2B800000u - 1u), kFxQHi = 2u * (0x53800000u - 1u);
constexpr uint32_t kFxSLo = 0x0D800000u - 1u, kFxSHi = 0x71800000u;
FX_FN FxRange fx_range_init() { return FxRange{0u, 0xFFFFFFFFu, 0u, 0xFFFFFFFFu, 0xFFFFFFFFu, false}; }
FX_FN bool fx_range_slow(const FxRange& g)
{
    return g.slow || g.q_mn < kFxQLo || g.q_mx > kFxQHi || g.s_mn < kFxSLo || g.s_mx > kFxSHi ||
           g.h_mn < ((2u * kFxBand) << 3);
}
FX_FN uint32_t fx_umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
FX_FN uint32_t fx_umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

// The two sinks of the fast functions' checks: a boolean (per operation) or
// the running extremes.  rng = the argument lies outside the function's fast
// range; y = the fast double whose float rounding must be unambiguous.
FX_FN void fx_sink_tx(bool& s, bool rng, double y) { s |= rng || fx_near_half(y); }
// (ALVRL_STUB_TXRANGE / _NEARHALF / _QS: developer timing variants that drop
// one class of checks; results invalid for the fix-up decision)
FX_FN void fx_sink_tx(FxRange& g, bool rng, double y)
{
#ifndef ALVRL_STUB_TXRANGE
    g.slow |= rng;
#endif
#ifdef ALVRL_STUB_NEARHALF
    return;
#endif
    // the 29 dropped bits moved to the top of a word (one v_lshl_add_u32):
    // 8 (lo29 - (2^28 - band)) mod 2^32
    const uint32_t t = ((uint32_t)__double_as_longlong(y) << 3) - ((0x10000000u - kFxBand) << 3);
    g.h_mn = fx_umin(g.h_mn, t);
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

// 1 / d with Newton steps on v_rcp_f64 (d normal and finite; not correctly
// rounded).  One step (ALVRL_FX_RCP_STEPS) squares v_rcp_f64's relative error.
#ifndef ALVRL_FX_RCP_STEPS
#define ALVRL_FX_RCP_STEPS 1
#endif
FX_FN double fx_rcp(double d)
{
    double r = __builtin_amdgcn_rcp(d);
    for (int i = 0; i < ALVRL_FX_RCP_STEPS; i++) {
        const double e = fx_fma(-d, r, 1.0);
        r = fx_fma(r, e, r);
    }
    return r;
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

// 2^(j/256), j = 0..255 (Python's float pow, within 1 ulp: 2^-52 relative),
// the table of fx_exp_core.  Each kernel that evaluates fx_expf / fx_sinhf
// copies it to LDS first (fx_tables_init, all threads of the block).
__device__ __constant__ const double kFxExp2Tab[256] = {
    0x1.0000000000000p+0, 0x1.00b1afa5abcbfp+0, 0x1.0163da9fb3335p+0, 0x1.02168143b0281p+0,
    0x1.02c9a3e778061p+0, 0x1.037d42e11bbccp+0, 0x1.04315e86e7f85p+0, 0x1.04e5f72f654b1p+0,
    0x1.059b0d3158574p+0, 0x1.0650a0e3c1f89p+0, 0x1.0706b29ddf6dep+0, 0x1.07bd42b72a836p+0,
    0x1.0874518759bc8p+0, 0x1.092bdf66607e0p+0, 0x1.09e3ecac6f383p+0, 0x1.0a9c79b1f3919p+0,
    0x1.0b5586cf9890fp+0, 0x1.0c0f145e46c85p+0, 0x1.0cc922b7247f7p+0, 0x1.0d83b23395decp+0,
    0x1.0e3ec32d3d1a2p+0, 0x1.0efa55fdfa9c5p+0, 0x1.0fb66affed31bp+0, 0x1.1073028d7233ep+0,
    0x1.11301d0125b51p+0, 0x1.11edbab5e2ab6p+0, 0x1.12abdc06c31ccp+0, 0x1.136a814f204abp+0,
    0x1.1429aaea92de0p+0, 0x1.14e95934f312ep+0, 0x1.15a98c8a58e51p+0, 0x1.166a45471c3c2p+0,
    0x1.172b83c7d517bp+0, 0x1.17ed48695bbc0p+0, 0x1.18af9388c8deap+0, 0x1.1972658375d2fp+0,
    0x1.1a35beb6fcb75p+0, 0x1.1af99f8138a1cp+0, 0x1.1bbe084045cd4p+0, 0x1.1c82f95281c6bp+0,
    0x1.1d4873168b9aap+0, 0x1.1e0e75eb44027p+0, 0x1.1ed5022fcd91dp+0, 0x1.1f9c18438ce4dp+0,
    0x1.2063b88628cd6p+0, 0x1.212be3578a819p+0, 0x1.21f49917ddc96p+0, 0x1.22bdda27912d1p+0,
    0x1.2387a6e756238p+0, 0x1.2451ffb82140ap+0, 0x1.251ce4fb2a63fp+0, 0x1.25e85711ece75p+0,
    0x1.26b4565e27cddp+0, 0x1.2780e341ddf29p+0, 0x1.284dfe1f56381p+0, 0x1.291ba7591bb70p+0,
    0x1.29e9df51fdee1p+0, 0x1.2ab8a66d10f13p+0, 0x1.2b87fd0dad990p+0, 0x1.2c57e39771b2fp+0,
    0x1.2d285a6e4030bp+0, 0x1.2df961f641589p+0, 0x1.2ecafa93e2f56p+0, 0x1.2f9d24abd886bp+0,
    0x1.306fe0a31b715p+0, 0x1.31432edeeb2fdp+0, 0x1.32170fc4cd831p+0, 0x1.32eb83ba8ea32p+0,
    0x1.33c08b26416ffp+0, 0x1.3496266e3fa2dp+0, 0x1.356c55f929ff1p+0, 0x1.36431a2de883bp+0,
    0x1.371a7373aa9cbp+0, 0x1.37f26231e754ap+0, 0x1.38cae6d05d866p+0, 0x1.39a401b7140efp+0,
    0x1.3a7db34e59ff7p+0, 0x1.3b57fbfec6cf4p+0, 0x1.3c32dc313a8e5p+0, 0x1.3d0e544ede173p+0,
    0x1.3dea64c123422p+0, 0x1.3ec70df1c5175p+0, 0x1.3fa4504ac801cp+0, 0x1.40822c367a024p+0,
    0x1.4160a21f72e2ap+0, 0x1.423fb2709468ap+0, 0x1.431f5d950a897p+0, 0x1.43ffa3f84b9d4p+0,
    0x1.44e086061892dp+0, 0x1.45c2042a7d232p+0, 0x1.46a41ed1d0057p+0, 0x1.4786d668b3237p+0,
    0x1.486a2b5c13cd0p+0, 0x1.494e1e192aed2p+0, 0x1.4a32af0d7d3dep+0, 0x1.4b17dea6db7d7p+0,
    0x1.4bfdad5362a27p+0, 0x1.4ce41b817c114p+0, 0x1.4dcb299fddd0dp+0, 0x1.4eb2d81d8abffp+0,
    0x1.4f9b2769d2ca7p+0, 0x1.508417f4531eep+0, 0x1.516daa2cf6642p+0, 0x1.5257de83f4eefp+0,
    0x1.5342b569d4f82p+0, 0x1.542e2f4f6ad27p+0, 0x1.551a4ca5d920fp+0, 0x1.56070dde910d2p+0,
    0x1.56f4736b527dap+0, 0x1.57e27dbe2c4cfp+0, 0x1.58d12d497c7fdp+0, 0x1.59c0827ff07ccp+0,
    0x1.5ab07dd485429p+0, 0x1.5ba11fba87a03p+0, 0x1.5c9268a5946b7p+0, 0x1.5d84590998b93p+0,
    0x1.5e76f15ad2148p+0, 0x1.5f6a320dceb71p+0, 0x1.605e1b976dc09p+0, 0x1.6152ae6cdf6f4p+0,
    0x1.6247eb03a5585p+0, 0x1.633dd1d1929fdp+0, 0x1.6434634ccc320p+0, 0x1.652b9febc8fb7p+0,
    0x1.6623882552225p+0, 0x1.671c1c70833f6p+0, 0x1.68155d44ca973p+0, 0x1.690f4b19e9538p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6b052fa75173ep+0, 0x1.6c012750bdabfp+0, 0x1.6cfdcddd47645p+0,
    0x1.6dfb23c651a2fp+0, 0x1.6ef9298593ae5p+0, 0x1.6ff7df9519484p+0, 0x1.70f7466f42e87p+0,
    0x1.71f75e8ec5f74p+0, 0x1.72f8286ead08ap+0, 0x1.73f9a48a58174p+0, 0x1.74fbd35d7cbfdp+0,
    0x1.75feb564267c9p+0, 0x1.77024b1ab6e09p+0, 0x1.780694fde5d3fp+0, 0x1.790b938ac1cf6p+0,
    0x1.7a11473eb0187p+0, 0x1.7b17b0976cfdbp+0, 0x1.7c1ed0130c132p+0, 0x1.7d26a62ff86f0p+0,
    0x1.7e2f336cf4e62p+0, 0x1.7f3878491c491p+0, 0x1.80427543e1a12p+0, 0x1.814d2add106d9p+0,
    0x1.82589994cce13p+0, 0x1.8364c1eb941f7p+0, 0x1.8471a4623c7adp+0, 0x1.857f4179f5b21p+0,
    0x1.868d99b4492edp+0, 0x1.879cad931a436p+0, 0x1.88ac7d98a6699p+0, 0x1.89bd0a478580fp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8be05bad61778p+0, 0x1.8cf3216b5448cp+0, 0x1.8e06a5e0866d9p+0,
    0x1.8f1ae99157736p+0, 0x1.902fed0282c8ap+0, 0x1.9145b0b91ffc6p+0, 0x1.925c353aa2fe2p+0,
    0x1.93737b0cdc5e5p+0, 0x1.948b82b5f98e5p+0, 0x1.95a44cbc8520fp+0, 0x1.96bdd9a7670b3p+0,
    0x1.97d829fde4e50p+0, 0x1.98f33e47a22a2p+0, 0x1.9a0f170ca07bap+0, 0x1.9b2bb4d53fe0dp+0,
    0x1.9c49182a3f090p+0, 0x1.9d674194bb8d5p+0, 0x1.9e86319e32323p+0, 0x1.9fa5e8d07f29ep+0,
    0x1.a0c667b5de565p+0, 0x1.a1e7aed8eb8bbp+0, 0x1.a309bec4a2d33p+0, 0x1.a42c980460ad8p+0,
    0x1.a5503b23e255dp+0, 0x1.a674a8af46052p+0, 0x1.a799e1330b358p+0, 0x1.a8bfe53c12e59p+0,
    0x1.a9e6b5579fdbfp+0, 0x1.ab0e521356ebap+0, 0x1.ac36bbfd3f37ap+0, 0x1.ad5ff3a3c2774p+0,
    0x1.ae89f995ad3adp+0, 0x1.afb4ce622f2ffp+0, 0x1.b0e07298db666p+0, 0x1.b20ce6c9a8952p+0,
    0x1.b33a2b84f15fbp+0, 0x1.b468415b749b1p+0, 0x1.b59728de5593ap+0, 0x1.b6c6e29f1c52ap+0,
    0x1.b7f76f2fb5e47p+0, 0x1.b928cf22749e4p+0, 0x1.ba5b030a1064ap+0, 0x1.bb8e0b79a6f1fp+0,
    0x1.bcc1e904bc1d2p+0, 0x1.bdf69c3f3a207p+0, 0x1.bf2c25bd71e09p+0, 0x1.c06286141b33dp+0,
    0x1.c199bdd85529cp+0, 0x1.c2d1cd9fa652cp+0, 0x1.c40ab5fffd07ap+0, 0x1.c544778fafb22p+0,
    0x1.c67f12e57d14bp+0, 0x1.c7ba88988c933p+0, 0x1.c8f6d9406e7b5p+0, 0x1.ca3405751c4dbp+0,
    0x1.cb720dcef9069p+0, 0x1.ccb0f2e6d1675p+0, 0x1.cdf0b555dc3fap+0, 0x1.cf3155b5bab74p+0,
    0x1.d072d4a07897cp+0, 0x1.d1b532b08c968p+0, 0x1.d2f87080d89f2p+0, 0x1.d43c8eacaa1d6p+0,
    0x1.d5818dcfba487p+0, 0x1.d6c76e862e6d3p+0, 0x1.d80e316c98398p+0, 0x1.d955d71ff6075p+0,
    0x1.da9e603db3285p+0, 0x1.dbe7cd63a8315p+0, 0x1.dd321f301b460p+0, 0x1.de7d5641c0658p+0,
    0x1.dfc97337b9b5fp+0, 0x1.e11676b197d17p+0, 0x1.e264614f5a129p+0, 0x1.e3b333b16ee12p+0,
    0x1.e502ee78b3ff6p+0, 0x1.e653924676d76p+0, 0x1.e7a51fbc74c83p+0, 0x1.e8f7977cdb740p+0,
    0x1.ea4afa2a490dap+0, 0x1.eb9f4867cca6ep+0, 0x1.ecf482d8e67f1p+0, 0x1.ee4aaa2188510p+0,
    0x1.efa1bee615a27p+0, 0x1.f0f9c1cb6412ap+0, 0x1.f252b376bba97p+0, 0x1.f3ac948dd7274p+0,
    0x1.f50765b6e4540p+0, 0x1.f6632798844f8p+0, 0x1.f7bfdad9cbe14p+0, 0x1.f91d802243c89p+0,
    0x1.fa7c1819e90d8p+0, 0x1.fbdba3692d514p+0, 0x1.fd3c22b8f71f1p+0, 0x1.fe9d96b2a23d9p+0,
};
__shared__ double fx_exp2_lds[256];

// Every thread of the block calls this before its first fx_expf / fx_sinhf
FX_FN void fx_tables_init()
{
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) fx_exp2_lds[i] = kFxExp2Tab[i];
    __syncthreads();
}

// exp(x), |x| <= 87.5: x = (256 k + j) ln2/256 + r, |r| <= ln2/512:
// 2^k 2^(j/256) (1 + r + r^2 q(r)), q = 1/2 + r/6 (2^-42.7 relative on exp),
// one-constant reduction (error <= 32,300 x 2^-61.4 ln2/256 absolute on r:
// 2^-46.4), the table entry (2^-52): within 2^-42.5 overall, 5x inside the
// rounding test's band (2^-40)
FX_FN double fx_exp_core(double x)
{
    const double t = fx_fma(x, 0x1.71547652b82fep+8, 0x1.8p52);   // 256/ln2; n in the low word
    const double kd = t - 0x1.8p52;
    const int n = (int)(uint32_t)__double_as_longlong(t);
    const double r = fx_fma(kd, -0x1.62e42fefa39efp-9, x);         // ln2/256
    const double r2 = r * r;
    // q = 1/2 + r/6 (Taylor; 2^-42.7 relative on exp over |r| <= ln2/512,
    // tools/detmath_fast_coeffs.py): 1/2 is an inline operand of v_fma_f64
    // and 1/6 an SGPR pair, so no constant is moved into VGPRs per call
    const double q = fx_fma(r, fx_kd(0x1.5555555555555p-3, r), 0.5);
    const double p = fx_fma(r2, q, r);
    const double T = fx_exp2_lds[n & 255];
    return __builtin_amdgcn_ldexp(fx_fma(T, p, T), n >> 8);
}

// The _r forms return the fast float and set `slow` when it may differ from
// detmath's; the plain forms fall back lane by lane.
template <class FL>
FX_FN float fx_expf_r(float x, FL& slow)
{
    const double y = fx_exp_core((double)x);
    // |x| <= 87: the result is a normal float (exp(-87) > 2^-126)
    fx_sink_tx(slow, !(__builtin_fabsf(x) <= 87.0f), y);
    return (float)y;
}

// atan(x): |x| reduced to |t| <= tan(pi/8) with one division
// (t = x, (x - 1)/(x + 1) or -1/x), degree-8 fit of atan(t)/t in t^2 (2^-45.1)
template <class FL>
FX_FN float fx_atanf_r(float x, FL& slow)
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
    fx_sink_tx(slow, !zero && !(a >= 0x1p-60 && a <= 0x1p60), zero ? 0.0 : y);
    return zero ? 0.0f : (float)y;
}

// tan(x), |x| <= 2^16: x = k pi/2 + r, |r| <= pi/4 (+), sin r / cos r
// (degree-5 fits in r^2: 2^-47.6, 2^-43.5), one division
template <class FL>
FX_FN float fx_tanf_r(float x, FL& slow)
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
    double c = fx_fma(z, -0x1.23c5c0cad2c16p-22, 0x1.a00e9682df8e9p-16);
    c = fx_fma(c, z, fx_kd(-0x1.6c16b2d3e066cp-10, c));
    c = fx_fma(c, z, fx_kd(0x1.5555554476398p-5, c));
    c = fx_fma(c, z, fx_kd(-0x1.ffffffffe3762p-2, c));
    c = fx_fma(c, z, fx_kd(0x1.ffffffffffe0bp-1, c));
    const bool odd = k & 1u;
    const double num = odd ? -c : sn;
    const double den = odd ? sn : c;
    const double y = num * fx_rcp(den);
    // 2^-30 <= |x| <= 2^16, and |r| >= 2^-40 so the quotient stays in range
    const float ax = __builtin_fabsf(x);
    fx_sink_tx(slow, !(ax >= 0x1p-30f && ax <= 0x1p16f) || !(__builtin_fabs(r) >= 0x1p-40), y);
    return (float)y;
}

// asinh(x), a = |x|:
//   2^-6 <= a <= 2^20: log(w), w = a + sqrt(1 + a^2) = m 2^e with m in
//     [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m - 1)/(m + 1) (m - 1
//     exact), degree-5 fit of atanh(s)/s in s^2 (2^-45.1); w's rounding
//     (2^-52 absolute) stays below 2^-46 relative for a >= 2^-6;
//   a < 2^-6: a (1 - z/6 + 3z^2/40 - 5z^3/112), z = a^2 <= 2^-12 (series
//     remainder 35 z^4 / 1152 < 2^-53)
template <class FL>
FX_FN float fx_asinhf_r(float x, FL& slow)
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
    fx_sink_tx(slow, !zero && !(a >= 0x1p-60 && a <= 0x1p20), zero ? 0.0 : y);
    return zero ? 0.0f : (float)y;
}

// sinh(x): |x| < 1: x P(x^2) (degree-5 fit of sinh(a)/a, 2^-43.5);
// 1 <= |x| <= 87: (e - 1/e) / 2 with the exp above
template <class FL>
FX_FN float fx_sinhf_r(float x, FL& slow)
{
    const double a = __builtin_fabs((double)x);
    double r;
    if (a < 1.0) {
        const double z = a * a;
        double p = fx_fma(z, 0x1.b6be36e12230dp-26, 0x1.71cb623ab9f8ap-19);
        p = fx_fma(p, z, fx_kd(0x1.a01a28c329346p-13, p));
        p = fx_fma(p, z, fx_kd(0x1.111110ec59911p-7, p));
        p = fx_fma(p, z, fx_kd(0x1.5555555587b48p-3, p));
        p = fx_fma(p, z, fx_kd(0x1.ffffffffffd34p-1, p));
        r = a * p;
    } else {
        const double e = fx_exp_core(a);
        r = fx_fma(0.5, e, -0.5 * fx_rcp(e));
    }
    const double y = x < 0.0f ? -r : r;
    fx_sink_tx(slow, !(a >= 0x1p-20 && a <= 87.0), y);
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

// 1 / b in IEEE single precision, correctly rounded: v_rcp_f32 and two
// residual corrections y += y * (1 - b y) (Markstein), for |b| in
// [2^-40, 2^40] (flag otherwise).  Checked against IEEE 1.0f / b on every
// float (alvrl_detmath_exhaustive fn 7).
FX_FN float fx_rcpf_r(float b, bool& slow)
{
    float y = __builtin_amdgcn_rcpf(b);
    float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    const uint32_t eb = __float_as_uint(b) & 0x7FFFFFFFu;
    slow |= (eb - 0x2B800000u) > (0x53800000u - 0x2B800000u);
    return y;
}

// The same cores with the checks folded into the running extremes (FxRange)
FX_FN float fx_divf_r(float a, float b, FxRange& g)
{
    float y = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    const float q0 = a * y;
    float r = __builtin_fmaf(-b, q0, a);
    float q = __builtin_fmaf(r, y, q0);
    r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
#ifndef ALVRL_STUB_QS
    const uint32_t ba = __float_as_uint(a), bb = __float_as_uint(b);
    const uint32_t wb = (bb << 1) - 2u, wa = (ba << 1) - 2u;
    g.q_mx = fx_umax(fx_umax(g.q_mx, wb), ba << 1);
    g.q_mn = fx_umin(fx_umin(g.q_mn, wb), wa);
#endif
    return (__float_as_uint(a) << 1) == 0u ? q0 : q;
}

FX_FN float fx_sqrtf_r(float x, FxRange& g)
{
    const float y = __builtin_amdgcn_sqrtf(x);
    const float ym = __uint_as_float(__float_as_uint(y) - 1u);
    const float yp = __uint_as_float(__float_as_uint(y) + 1u);
    float r = __builtin_fmaf(-ym, y, x) <= 0.0f ? ym : y;
    r = __builtin_fmaf(-yp, y, x) > 0.0f ? yp : r;
#ifndef ALVRL_STUB_QS
    const uint32_t bx = __float_as_uint(x);
    g.s_mx = fx_umax(g.s_mx, bx);
    g.s_mn = fx_umin(g.s_mn, bx - 1u);
#endif
    return r;
}

FX_FN float fx_rcpf_r(float b, FxRange& g)
{
    float y = __builtin_amdgcn_rcpf(b);
    float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
#ifndef ALVRL_STUB_QS
    const uint32_t wb = (__float_as_uint(b) << 1) - 2u;
    g.q_mx = fx_umax(g.q_mx, wb);
    g.q_mn = fx_umin(g.q_mn, wb);
#endif
    return y;
}

FX_FN float fx_rcpf(float b)
{
    FxRange g = fx_range_init();
    float y = fx_rcpf_r(b, g);
    if (fx_range_slow(g)) y = 1.0f / b;
    return y;
}

FX_FN float fx_divf(float a, float b)
{
    FxRange g = fx_range_init();
    float q = fx_divf_r(a, b, g);
    if (fx_range_slow(g)) q = a / b;
    return q;
}

FX_FN float fx_sqrtf(float x)
{
    FxRange g = fx_range_init();
    float y = fx_sqrtf_r(x, g);
    if (fx_range_slow(g)) y = sqrtf(x);
    return y;
}

// (through the running extremes: the exhaustive checks of k_detmath_exhaustive
// and k_div_check cover the form the strict R build uses)
#define FX_PLAIN(name)                                      \
    FX_FN float fx_##name##f(float x)                       \
    {                                                       \
        FxRange g = fx_range_init();                        \
        float y = fx_##name##f_r(x, g);                     \
        if (fx_range_slow(g)) y = dm_##name##f(x);          \
        return y;                                           \
    }
FX_PLAIN(exp)
FX_PLAIN(atan)
FX_PLAIN(tan)
FX_PLAIN(asinh)
FX_PLAIN(sinh)
#undef FX_PLAIN

#endif /* ALVRL_DETMATH_FAST_H */
