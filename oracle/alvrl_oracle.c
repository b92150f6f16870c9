/*
 * alvrl_oracle.c -- CPU restatement of the ALVRL gather path.
 * TEST INFRASTRUCTURE ONLY (see alvrl_oracle.h for scope, citations and the
 * "parity unpinned" status).  Compiled two ways by oracle/Makefile:
 *   liboracle.so       strict IEEE (-O2 -ffp-contract=off), the parity checker
 *   liboracle_fast.so  the reference's own flags (build/config-linux-gcc.py:7),
 *                      used only as bench.py's timed CPU baseline.
 */
#include "alvrl_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "detmath.h"

/* include/mitsuba/core/constants.h:27-33 (SINGLE_PRECISION) */
#define EPSILON       1e-4f
#define INV_FOURPI    0.07957747154594766788f
#define INV_PI        0.31830988618379067154f
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ===================================================================== */
/*  Counter RNG: Philox4x32-10 (Salmon et al., SC'11; Random123)           */
/* ===================================================================== */
static inline uint32_t mulhilo32(uint32_t a, uint32_t b, uint32_t *hi)
{
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

void alvrl_o_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint32_t hi0, hi1;
        uint32_t lo0 = mulhilo32(0xD2511F53u, c0, &hi0);
        uint32_t lo1 = mulhilo32(0xCD9E8D57u, c2, &hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Random::nextFloat, src/libcore/random.cpp:630-639 */
float alvrl_o_u01(uint32_t bits)
{
    union { uint32_t u; float f; } x;
    x.u = (bits >> 9) | 0x3f800000u;
    return x.f - 1.0f;
}

/* Random-access draw k of the stream (dom, a, b, c). */
static float draw(uint32_t seed, uint32_t pass, uint32_t dom, uint32_t a, uint32_t b,
                  uint32_t c, uint32_t k)
{
    uint32_t ctr[4] = { a, b, k >> 2, (dom << 24) | (c & 0xFFFFFFu) };
    uint32_t key[2] = { seed, pass };
    uint32_t out[4];
    alvrl_o_philox4x32_10(ctr, key, out);
    return alvrl_o_u01(out[k & 3]);
}

/* Sequential sampler over one stream (Sampler::next1D / next2D). */
typedef struct {
    uint32_t seed, pass, dom, a, b, c, k;
    uint32_t buf[4];
    uint32_t buf_block;
} seq_sampler;

static void seq_init(seq_sampler *s, uint32_t seed, uint32_t pass, uint32_t dom,
                     uint32_t a, uint32_t b, uint32_t c)
{
    s->seed = seed; s->pass = pass; s->dom = dom;
    s->a = a; s->b = b; s->c = c; s->k = 0; s->buf_block = 0xFFFFFFFFu;
}

static float seq_next(seq_sampler *s)
{
    uint32_t blk = s->k >> 2;
    if (blk != s->buf_block) {
        uint32_t ctr[4] = { s->a, s->b, blk, (s->dom << 24) | (s->c & 0xFFFFFFu) };
        uint32_t key[2] = { s->seed, s->pass };
        alvrl_o_philox4x32_10(ctr, key, s->buf);
        s->buf_block = blk;
    }
    float v = alvrl_o_u01(s->buf[s->k & 3]);
    s->k++;
    return v;
}

/* ===================================================================== */
/*  Vector helpers (include/mitsuba/core/vector.h, point.h semantics)      */
/* ===================================================================== */
typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = { x, y, z }; return r; }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 scl(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float len2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline float len(v3 a) { return sqrtf(len2(a)); }
static inline float dist(v3 a, v3 b) { return len(sub(a, b)); }
static inline float dist2(v3 a, v3 b) { return len2(sub(a, b)); }
/* normalize(v) = v / v.length(), and operator/ multiplies by the reciprocal */
static inline v3 nrm(v3 a) { float r = 1.0f / len(a); return scl(a, r); }
static inline v3 cross(v3 a, v3 b)
{
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline v3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }

/* math::fastexp / fastlog on Linux/x86_64 (include/mitsuba/core/math.h:175-199)
 * and the float atan / tan / asinh / sinh of the samplers (vrlIntegrator.cpp:
 * 889-957).  The parity checker evaluates them with the deterministic
 * definitions of detmath.h (double, rounded once to float: the correctly
 * rounded value outside a few ulps of double around float rounding
 * boundaries, tests/test_detmath.py), which the strict device kernels share,
 * so that the strict R build and the tracer reproduce it bit for bit
 * (deviation 3).  The timed CPU baseline
 * (liboracle_fast.so, -DALVRL_O_LIBM) calls libm as the reference does. */
#ifdef ALVRL_O_LIBM
static inline float fastexp(float v) { return (float)exp((double)v); }
static inline float fastlog(float v) { return (float)log((double)v); }
#define m_atanf atanf
#define m_tanf tanf
#define m_asinhf asinhf
#define m_sinhf sinhf
#else
static inline float fastexp(float v) { return dm_expf(v); }
static inline float fastlog(float v) { return dm_logf(v); }
#define m_atanf dm_atanf
#define m_tanf dm_tanf
#define m_asinhf dm_asinhf
#define m_sinhf dm_sinhf
#endif
static inline float safe_sqrt(float v) { return sqrtf(v > 0.0f ? v : 0.0f); }

/* Spectrum::isValid, include/mitsuba/core/spectrum.h:467-472 */
static inline int spec_valid(const float s[3])
{
    for (int i = 0; i < 3; i++)
        if (!isfinite(s[i]) || s[i] < 0.0f) return 0;
    return 1;
}
/* Spectrum::getLuminance, spectrum.h:638-640 */
static inline float lum(const float s[3])
{
    return s[0] * 0.212671f + s[1] * 0.715160f + s[2] * 0.072169f;
}

/* ===================================================================== */
/*  Medium / phase / BSDF                                                  */
/* ===================================================================== */
void alvrl_o_medium_init(alvrl_o_medium *m, const float sigma_s[3], const float sigma_a[3],
                         float w, int phase_type, float g)
{
    for (int i = 0; i < 3; i++) {
        m->sigma_s[i] = sigma_s[i];
        m->sigma_a[i] = sigma_a[i];
        m->sigma_t[i] = sigma_s[i] + sigma_a[i];
    }
    /* homogeneous.cpp:168-184: highest albedo, clamped to >= 0.5 */
    if (w == -1) {
        for (int i = 0; i < 3; i++) {
            float albedo = m->sigma_s[i] / m->sigma_t[i];
            if (albedo > w && m->sigma_t[i] != 0) w = albedo;
        }
        if (w > 0) w = w > 0.5f ? w : 0.5f;
    }
    m->sampling_weight = w;
    m->phase_type = phase_type;
    m->phase_g = g;
    m->strategy = ALVRL_O_BALANCE;
    m->density = 0.0f;
}

int alvrl_o_medium_strategy(alvrl_o_medium *m, int strategy, int channel, float density)
{
    m->strategy = strategy;
    m->density = 0.0f;
    if (strategy == ALVRL_O_BALANCE) return 0;
    if (strategy == ALVRL_O_SINGLE) {   /* homogeneous.cpp:188-204 */
        if (channel < 0) {
            float smallest = INFINITY;
            channel = 0;
            for (int i = 0; i < 3; i++)
                if (m->sigma_t[i] < smallest) { smallest = m->sigma_t[i]; channel = i; }
        }
        if (channel > 2) return -1;
        m->density = m->sigma_t[channel];
        return 0;
    }
    if (strategy == ALVRL_O_MANUAL) { m->density = density; return 0; }   /* :221-223 */
    if (strategy != ALVRL_O_MAXIMUM) return -1;
    /* MaxExpDist(sigmaT) (maxexp.h:30-57) */
    float s[3] = { m->sigma_t[0], m->sigma_t[1], m->sigma_t[2] };
    for (int i = 0; i < 3; i++)          /* std::sort(.., std::greater<Float>()) */
        for (int j = i + 1; j < 3; j++)
            if (s[j] > s[i]) { float t = s[i]; s[i] = s[j]; s[j] = t; }
    float cdf[4];
    cdf[0] = 0;
    for (int i = 0; i < 3; i++) {
        if (i > 0 && s[i] == s[i - 1]) return -1;
        float lower = (i == 0) ? -1 : -powf(s[i] / s[i - 1], -s[i] / (s[i] - s[i - 1]));
        float upper = (i == 2) ? 0 : -powf(s[i + 1] / s[i], -s[i] / (s[i + 1] - s[i]));
        cdf[i + 1] = cdf[i] + (upper - lower);
        m->mx_start[i] = (i == 0) ? 0 : fastlog(s[i] / s[i - 1]) / (s[i] - s[i - 1]);
        m->mx_lower[i] = lower;
        m->mx_sigma[i] = s[i];
    }
    m->mx_norm = cdf[3];
    m->mx_inv_norm = 1 / m->mx_norm;
    for (int i = 0; i < 4; i++) m->mx_cdf[i] = cdf[i] * m->mx_inv_norm;
    return 0;
}

/* std::max(0, lower_bound(a, a + n, x) - a - 1) */
static int interval_of(const float *a, int n, float x)
{
    int k = 0;
    while (k < n && a[k] < x) k++;
    return k > 0 ? k - 1 : 0;
}

/* MaxExpDist::sample (maxexp.h:59-73).  The index is clamped to the last
 * interval (the reference's SAssert is compiled out: u = 1 above a rounded
 * m_cdf[n] would read past its arrays). */
static float maxexp_sample(const alvrl_o_medium *m, float u, float *pdf)
{
    int i = interval_of(m->mx_cdf, 4, u);
    if (i > 2) i = 2;
    float t = -fastlog(fastexp(-m->mx_start[i] * m->mx_sigma[i]) - m->mx_norm * (u - m->mx_cdf[i])) / m->mx_sigma[i];
    *pdf = m->mx_sigma[i] * fastexp(-m->mx_sigma[i] * t) * m->mx_inv_norm;
    return t;
}

/* MaxExpDist::cdf (maxexp.h:83-94) */
static float maxexp_cdf(const alvrl_o_medium *m, float t)
{
    int i = interval_of(m->mx_start, 3, t);
    float upper = -fastexp(-m->mx_sigma[i] * t);
    return m->mx_cdf[i] + (upper - m->mx_lower[i]) * m->mx_inv_norm;
}

/* HomogeneousMedium::sampleDistance's draws (homogeneous.cpp:277-296): the
 * sampled distance (INFINITY: no medium interaction) and, for 'maximum',
 * the pdf of the sample. */
static float medium_sample_distance(const alvrl_o_medium *m, seq_sampler *smp, float *pdf_max)
{
    float rnd = seq_next(smp), w = m->sampling_weight;
    if (!(rnd < w)) return INFINITY;   /* no medium interaction */
    rnd /= w;
    if (m->strategy == ALVRL_O_MAXIMUM) return maxexp_sample(m, 1 - rnd, pdf_max);
    float density = m->density;
    if (m->strategy == ALVRL_O_BALANCE) {   /* a random channel each time */
        int ch = (int)(seq_next(smp) * 3);
        if (ch > 2) ch = 2;
        density = m->sigma_t[ch];
    }
    return -fastlog(1 - rnd) / density;
}
/* The pdfs of sampleDistance (:317-346) at the distance used: pdfSuccess and
 * pdfFailure with the sampling weight applied. */
static void medium_pdfs(const alvrl_o_medium *m, float sampled, float pdf_max, float *ps, float *pf)
{
    float w = m->sampling_weight, s = 0.0f, f = 0.0f;
    if (m->strategy == ALVRL_O_MAXIMUM) {
        f = 1 - maxexp_cdf(m, sampled);
        s = pdf_max;
    } else if (m->strategy == ALVRL_O_BALANCE) {
        for (int i = 0; i < 3; i++) {
            float tmp = fastexp(-m->sigma_t[i] * sampled);
            f += tmp;
            s += m->sigma_t[i] * tmp;
        }
        f /= 3; s /= 3;
    } else {
        f = fastexp(-m->density * sampled);
        s = m->density * f;
    }
    *ps = s * w;
    *pf = w * f + (1 - w);
}

/* HomogeneousMedium::eval (homogeneous.cpp:354-396).  Only the fields used
 * by integrateVRL are produced. */
static void medium_eval(const alvrl_o_medium *m, float distance, float tr[3], float *pdf_failure)
{
    float pf = 0.0f;
    if (m->strategy == ALVRL_O_BALANCE) {
        for (int i = 0; i < 3; i++) {
            float temp = fastexp(-m->sigma_t[i] * distance);
            pf += temp;
        }
        pf /= 3;
    } else if (m->strategy == ALVRL_O_MAXIMUM) {
        pf = 1 - maxexp_cdf(m, distance);
    } else {
        pf = fastexp(-m->density * distance);
    }
    for (int i = 0; i < 3; i++) tr[i] = fastexp(m->sigma_t[i] * (-distance));
    *pdf_failure = pf * m->sampling_weight + (1 - m->sampling_weight);
    float mx = tr[0] > tr[1] ? tr[0] : tr[1];
    mx = mx > tr[2] ? mx : tr[2];
    if (mx < 1e-20f) tr[0] = tr[1] = tr[2] = 0.0f;
}

/* HomogeneousMedium::evalTransmittance (homogeneous.cpp:266-273) as used by
 * Scene::evalTransmittance (scene.cpp:619-679) when no surface blocks the
 * segment (convex container: every interior pair is mutually visible). */
/* TriangleT::rayIntersect, include/mitsuba/core/triangle.h:109-145 */
static int tri_intersect(const float *tri, v3 o, v3 d, float *u, float *v, float *t)
{
    v3 p0 = mk(tri[0], tri[1], tri[2]), p1 = mk(tri[3], tri[4], tri[5]), p2 = mk(tri[6], tri[7], tri[8]);
    v3 edge1 = sub(p1, p0), edge2 = sub(p2, p0);
    v3 pvec = cross(d, edge2);
    float det = dot(edge1, pvec);
    if (det == 0) return 0;
    float inv_det = 1.0f / det;
    v3 tvec = sub(o, p0);
    *u = dot(tvec, pvec) * inv_det;
    if (*u < 0.0f || *u > 1.0f) return 0;
    v3 qvec = cross(tvec, edge1);
    *v = dot(d, qvec) * inv_det;
    if (*v >= 0.0f && *u + *v <= 1.0f) { *t = dot(edge2, qvec) * inv_det; return 1; }
    return 0;
}

/* The occluder part of Scene::evalTransmittance(p1, p1OnSurface, p2, false)
 * (scene.cpp:619-679): the segment's ray has mint = Epsilon (1e-4) from a
 * surface, 0 from a medium point; any triangle hit in [mint, remaining]
 * blocks.  The box walls cannot (both points are inside). */
static int segment_visible(const float *occ, const uint32_t *mat, uint32_t nocc, v3 p1, int p1_surface, v3 p2)
{
    if (!nocc) return 1;
    v3 d = sub(p2, p1);
    float remaining = len(d);
    if (!(remaining > 0)) return 1;
    d = scl(d, 1.0f / remaining);
    float mint = p1_surface ? 1e-4f : 0.0f;
    float maxt = remaining * 1.0f;
    for (uint32_t i = 0; i < nocc; i++) {
        if (mat && mat[i] == ALVRL_O_MAT_NULL) continue;   /* ENull: passes (scene.cpp:636-637) */
        float u, v, t;
        if (tri_intersect(occ + 9 * (size_t)i, p1, d, &u, &v, &t) && !(t < mint || t > maxt)) return 0;
    }
    return 1;
}

static void shadow_transmittance(const alvrl_o_params *P, v3 p1, int p1_surface, v3 p2, float tr[3])
{
    const alvrl_o_medium *m = &P->medium;
    v3 d = sub(p2, p1);
    float remaining = len(d);
    float negLength = 0.0f - remaining;
    for (int i = 0; i < 3; i++)
        tr[i] = m->sigma_t[i] != 0 ? fastexp(m->sigma_t[i] * negLength) : 1.0f;
    if (!segment_visible(P->occ, P->occ_mat, P->nocc, p1, p1_surface, p2)) tr[0] = tr[1] = tr[2] = 0.0f;
}

/* isotropic.cpp:76-78, hg.cpp:107-110 */
static float phase_eval(const alvrl_o_medium *m, v3 wi, v3 wo)
{
    if (m->phase_type == 0) return INV_FOURPI;
    float g = m->phase_g;
    float temp = 1.0f + g * g + 2.0f * g * dot(wi, wo);
    return INV_FOURPI * (1 - g * g) / (temp * sqrtf(temp));
}

/* ===================================================================== */
/*  Samplers (vrlIntegrator.cpp:831-1032)                                  */
/* ===================================================================== */
/* getClosestPoints, vrlIntegrator.cpp:962-1032 */
static float closest_points(v3 S1P0, v3 S1P1, v3 S2P0, v3 S2P1, v3 *S1h, v3 *S2h)
{
    v3 u = sub(S1P1, S1P0);
    v3 v = sub(S2P1, S2P0);
    v3 w = sub(S1P0, S2P0);
    float a = dot(u, u);
    float b = dot(u, v);
    float c = dot(v, v);
    float d = dot(u, w);
    float e = dot(v, w);
    float D = a * c - b * b;
    float sc, sN, sD = D;
    float tc, tN, tD = D;

    if (D < EPSILON * len2(u) * len2(v)) {
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
    sc = sN / sD;
    tc = tN / tD;
    v3 dP = sub(add(w, scl(u, sc)), scl(v, tc));
    *S1h = add(S1P0, scl(sub(S1P1, S1P0), sc));
    *S2h = add(S2P0, scl(sub(S2P1, S2P0), tc));
    return len(dP);
}

/* KullaSampling, vrlIntegrator.cpp:889-914 (equi-angular sampling) */
static float kulla(v3 A, v3 B, v3 D, v3 *result, float uniform)
{
    v3 dir = nrm(sub(B, A));
    float dotPr = dot(dir, sub(D, A));
    v3 I = add(A, scl(dir, dotPr));
    float Dis = dist(D, I);
    float angle_a = m_atanf(dist(A, I) / Dis);
    float angle_b = m_atanf(dist(I, B) / Dis);
    if (dotPr > 0) {
        angle_a *= -1;
        if (dist(A, I) > dist(A, B)) angle_b *= -1;
    }
    float t = Dis * m_tanf(((1.0f - uniform) * angle_a) + (uniform * angle_b));
    float pdf = Dis / ((angle_b - angle_a) * (Dis * Dis + t * t));
    *result = add(I, scl(dir, t));
    return pdf;
}

static inline float Afun(float x, float h, float sinTheta) { return m_asinhf((x / h) * sinTheta); }

/* sampleVtoDistance, vrlIntegrator.cpp:916-953 (Novak et al. 2012) */
static float sample_v_to_distance(v3 E, v3 d, v3 hitp, v3 S, v3 End, v3 *V, float uniform)
{
    if (dist(S, End) == 0) { *V = S; return 1; }
    float cosTheta = dot(nrm(d), nrm(sub(End, S)));
    float sinTheta = safe_sqrt(1 - cosTheta * cosTheta);
    if (sinTheta < EPSILON) {
        *V = add(S, scl(sub(End, S), uniform));
        return 1 / dist(End, S);
    }
    v3 Uh, Vh;
    float h = closest_points(E, hitp, S, End, &Uh, &Vh);
    float V0c = -1 * dist(Vh, S);
    float V1c = dist(Vh, End);
    float newV = h * m_sinhf(Afun(V0c, h, sinTheta)
                           + (uniform * (Afun(V1c, h, sinTheta) - Afun(V0c, h, sinTheta))));
    newV = newV / sinTheta;
    float result = 1.0f / sqrtf(h * h + newV * newV * sinTheta * sinTheta);
    float denom = (Afun(V1c, h, sinTheta) - Afun(V0c, h, sinTheta)) / sinTheta;
    newV += dist(Vh, S);
    *V = add(S, scl(nrm(sub(End, S)), newV));
    return result / denom;
}

/* Exported single-function entry points: per-function known-answer fixtures
 * (tests/golden/make_golden.py).  Points are float[3]. */
static v3 v3p(const float *p) { v3 r = {p[0], p[1], p[2]}; return r; }
static void v3s(v3 a, float *p) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }

float alvrl_o_closest_points(const float s1p0[3], const float s1p1[3], const float s2p0[3],
                             const float s2p1[3], float s1h[3], float s2h[3])
{
    v3 a, b;
    float h = closest_points(v3p(s1p0), v3p(s1p1), v3p(s2p0), v3p(s2p1), &a, &b);
    v3s(a, s1h); v3s(b, s2h);
    return h;
}

float alvrl_o_kulla(const float A[3], const float B[3], const float D[3], float uniform, float res[3])
{
    v3 r;
    float pdf = kulla(v3p(A), v3p(B), v3p(D), &r, uniform);
    v3s(r, res);
    return pdf;
}

float alvrl_o_sample_v_to_distance(const float E[3], const float d[3], const float hitp[3],
                                   const float S[3], const float End[3], float uniform, float V[3])
{
    v3 r;
    float pdf = sample_v_to_distance(v3p(E), v3p(d), v3p(hitp), v3p(S), v3p(End), &r, uniform);
    v3s(r, V);
    return pdf;
}

/* detmath.h's float functions over an array (fn: 0 exp, 1 log, 2 atan,
 * 3 tan, 4 asinh, 5 sinh): tests/test_detmath.py */
void alvrl_o_detmath(int fn, const float *in, float *out, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++) {
        float x = in[i], y;
        switch (fn) {
        case 0: y = dm_expf(x); break;
        case 1: y = dm_logf(x); break;
        case 2: y = dm_atanf(x); break;
        case 3: y = dm_tanf(x); break;
        case 4: y = dm_asinhf(x); break;
        default: y = dm_sinhf(x); break;
        }
        out[i] = y;
    }
}

void alvrl_o_medium_eval(const alvrl_o_medium *m, float distance, float tr[3], float *pdf_failure)
{
    medium_eval(m, distance, tr, pdf_failure);
}

/* ===================================================================== */
/*  integrateVRL, vrlIntegrator.cpp:603-785                                */
/* ===================================================================== */
/* 'rsub' is the sample index of an R entry with Rsamples > 1 (LiInternal's
 * samples loop, vrlIntegrator.cpp:427-443), in bits 8-23 of the block counter
 * (the draws' block index stays below 2^8); the stream word carries the
 * record's eye-path depth in bits 16-23 and its sensor sample in bits 0-15,
 * so R sample r of sensor sample j never meets another (j', r') stream.  use_weight: integrateVRL's
 * 'weight' argument (:605) is the record's path weight, the first factor of
 * every sample's contribution (:668, :743), as getVRLContributions passes it
 * (:808); getClusteredVrlContributions calls with the default 1 and
 * multiplies its sum instead (:598). */
static void integrate_vrl_w(const alvrl_o_params *P, const float *rec, uint32_t rec_id,
                            const float *vs, uint32_t nvrl, uint32_t vrl_id, uint32_t domain,
                            uint32_t rsub, int use_weight, float out_rgb[3], float *contrib, float *variance)
{
    const alvrl_o_medium *m = &P->medium;
    uint32_t flags, depth;
    memcpy(&flags, &rec[15], 4);
    memcpy(&depth, &rec[19], 4);
    const uint32_t sw = ((depth & 0xFFu) << 16) | ((depth >> 16) & 0xFFFFu);
    const uint32_t koff = (rsub & 0xFFFFu) << 10;   /* + k: counter word (k >> 2) | rsub << 8 */
    const float wt[3] = { use_weight ? rec[16] : 1.0f, use_weight ? rec[17] : 1.0f, use_weight ? rec[18] : 1.0f };
    if (contrib) *contrib = 0;
    if (variance) *variance = 0;
    out_rgb[0] = out_rgb[1] = out_rgb[2] = 0.0f;
    if (!(flags & ALVRL_O_FLAG_MEDIUM)) return;   /* :614-617 */

    v3 E = ld3(rec + 0), dray = ld3(rec + 3), Usurf = ld3(rec + 6), nrmS = ld3(rec + 9);
    v3 S = mk(vs[0 * nvrl + vrl_id], vs[1 * nvrl + vrl_id], vs[2 * nvrl + vrl_id]);
    v3 End = mk(vs[3 * nvrl + vrl_id], vs[4 * nvrl + vrl_id], vs[5 * nvrl + vrl_id]);
    float power[3] = { vs[6 * nvrl + vrl_id], vs[7 * nvrl + vrl_id], vs[8 * nvrl + vrl_id] };
    v3 SV = nrm(sub(End, S));
    v3 EU = dray;
    const int nVV = P->vol_vol_samples, nVS = P->vol_surf_samples;
    float total[3] = { 0, 0, 0 };

    /* sampleUVKulla's eye segment end (:865-871); its.t is finite here */
    float edist = dist(Usurf, E);
    v3 A = E, B = add(E, scl(dray, edist));

    /* ---- volume to volume (:647-703) ---- */
    float mean = 0, M2 = 0;
    for (int sample = 0; sample < nVV; sample++) {
        float lumv = 0.0f;
        float u0 = draw(P->seed, P->pass, domain, rec_id, vrl_id, sw, koff + 2 * sample);
        float u1 = draw(P->seed, P->pass, domain, rec_id, vrl_id, sw, koff + 2 * sample + 1);
        v3 V, U;
        float pdf = sample_v_to_distance(E, dray, Usurf, S, End, &V, u0);
        pdf *= kulla(A, B, V, &U, u1);
        if (dist(U, V) == 0) goto vv_welford;
        {
            v3 VU = nrm(sub(U, V));
            float tuv[3], teu[3], tsv[3], pf_eu, pf_sv;
            shadow_transmittance(P, U, 0, V, tuv);
            if (tuv[0] == 0 && tuv[1] == 0 && tuv[2] == 0) goto vv_welford;
            medium_eval(m, dist(E, U), teu, &pf_eu);
            medium_eval(m, dist(S, V), tsv, &pf_sv);
            float c[3];
            float rpdf = 1.0f / pdf;
            float rd2 = 1 / dist2(U, V);
            float phU = phase_eval(m, neg(VU), neg(EU));
            float phV = phase_eval(m, neg(SV), VU);
            float rpf = 1.0f / pf_sv;
            for (int i = 0; i < 3; i++) {
                c[i] = wt[i];
                c[i] *= power[i];
                c[i] *= (m->sigma_s[i] * m->sigma_s[i]) * rpdf;
                c[i] *= rd2;
                c[i] *= tsv[i];
                c[i] *= tuv[i];
                c[i] *= teu[i];
                if (P->short_vrls) c[i] *= rpf;
                c[i] *= phU;
                c[i] *= phV;
            }
            if (spec_valid(c)) {
                float rn = 1.0f / (float)nVV;
                for (int i = 0; i < 3; i++) total[i] += c[i] * rn;
                lumv = lum(c);
            }
        }
    vv_welford: {
            /* :693-699, evaluated online in the same order */
            float delta = lumv - mean;
            mean += delta / (sample + 1);
            M2 += delta * (lumv - mean);
        }
    }
    if (contrib && nVV > 0) *contrib += mean;
    if (variance && nVV > 0) *variance += M2 / ((nVV - 1) * nVV);

    /* ---- volume to surface (:706-782) ---- */
    v3 U = Usurf;
    float teus[3] = { 0, 0, 0 };
    if (flags & ALVRL_O_FLAG_HIT) {
        if (dist(Usurf, E) != 0) {
            float pfd;
            medium_eval(m, dist(Usurf, E), teus, &pfd);
        }
    }
    mean = 0; M2 = 0;
    int do_surf = (teus[0] != 0 || teus[1] != 0 || teus[2] != 0) && (flags & ALVRL_O_FLAG_SMOOTH);
    for (int sample = 0; sample < nVS; sample++) {
        float lumv = 0.0f;
        if (do_surf) {
            float u = draw(P->seed, P->pass, domain, rec_id, vrl_id, sw, koff + 2 * nVV + sample);
            v3 V;
            float pdf = kulla(S, End, U, &V, u);
            if (dist(U, V) != 0) {
                v3 VU = nrm(sub(U, V));
                float tuv[3], tsv[3], pf_sv;
                shadow_transmittance(P, U, 1, V, tuv);
                medium_eval(m, dist(S, V), tsv, &pf_sv);
                /* SmoothDiffuse::eval (diffuse.cpp:110-118), wi = its.wi, wo = toLocal(-VU) */
                v3 mVU = neg(VU);
                float cos_wi = dot(neg(dray), nrmS);
                float cos_wo = dot(mVU, nrmS);
                float f[3] = { 0, 0, 0 };
                if (!(cos_wi <= 0 || cos_wo <= 0))
                    for (int i = 0; i < 3; i++) f[i] = rec[12 + i] * (INV_PI * cos_wo);
                float phV = phase_eval(m, neg(SV), VU);
                float rpdf = 1.0f / pdf;
                float rd2 = 1 / dist2(U, V);
                float rpf = 1.0f / pf_sv;
                float c[3];
                for (int i = 0; i < 3; i++) {
                    c[i] = wt[i];
                    c[i] *= power[i];
                    c[i] *= m->sigma_s[i] * rpdf;
                    c[i] *= rd2;
                    c[i] *= tsv[i];
                    c[i] *= tuv[i];
                    c[i] *= teus[i];
                    if (P->short_vrls) c[i] *= rpf;
                    c[i] *= phV;
                    c[i] *= f[i];
                }
                if (spec_valid(c)) {
                    float rn = 1.0f / (float)nVS;
                    for (int i = 0; i < 3; i++) total[i] += c[i] * rn;
                    lumv = lum(c);
                }
            }
        }
        float delta = lumv - mean;
        mean += delta / (sample + 1);
        M2 += delta * (lumv - mean);
    }
    if (contrib && nVS > 0) *contrib += mean;
    if (variance && nVS > 0) *variance += M2 / ((nVS - 1) * nVS);

    out_rgb[0] = total[0]; out_rgb[1] = total[1]; out_rgb[2] = total[2];
}

/* ===================================================================== */
/*  Gathers                                                                */
/* ===================================================================== */
void alvrl_o_integrate_vrl(const alvrl_o_params *P, const float *rec, uint32_t rec_id,
                           const float *vs, uint32_t nvrl, uint32_t vrl_id,
                           uint32_t domain, float out_rgb[3], float *contrib, float *variance)
{
    integrate_vrl_w(P, rec, rec_id, vs, nvrl, vrl_id, domain, 0u, 0, out_rgb, contrib, variance);
}

typedef struct {
    const alvrl_o_params *P;
    const float *recs; uint32_t nrec; const uint32_t *rec_ids;
    const float *vs; uint32_t nvrl; uint64_t pc; uint32_t domain;
    float *out; float *R;
    /* clustered */
    const uint32_t *slice_of_rec, *slice_off, *reps, *fb_reps;
    const float *weights, *fb_weights; uint32_t n_fb;
    uint32_t r0, r1;
    uint64_t count;
} gjob;

/* getVRLContributions, vrlIntegrator.cpp:792-825 */
static void *brute_worker(void *arg)
{
    gjob *j = (gjob *)arg;
    float normalization = (float)(1.0 / (double)j->pc);
    for (uint32_t r = j->r0; r < j->r1; r++) {
        const float *rec = j->recs + (size_t)r * ALVRL_O_REC_WORDS;
        uint32_t flags;
        memcpy(&flags, &rec[15], 4);
        float Li[3] = { 0, 0, 0 };
        uint32_t rid = j->rec_ids ? j->rec_ids[r] : r;
        /* R rows: LiInternal with samples = Rsamples; the entries are sums
         * over the samples (:812-813), the radiance their mean (:445) */
        const uint32_t ns = (j->R && j->P->r_samples > 1) ? (uint32_t)j->P->r_samples : 1u;
        if (flags & ALVRL_O_FLAG_MEDIUM) {
            for (uint32_t s = 0; s < ns; s++) {
                for (uint32_t v = 0; v < j->nvrl; v++) {
                    float c[3], contribution, variance;
                    integrate_vrl_w(j->P, rec, rid, j->vs, j->nvrl, v, j->domain, s, 1, c,
                                    &contribution, &variance);
                    for (int i = 0; i < 3; i++) c[i] *= normalization;
                    if (j->R) {
                        float *e = j->R + 2 * ((size_t)r * j->nvrl + v);
                        e[0] += contribution * normalization;
                        e[1] += variance * normalization * normalization;
                    }
                    for (int i = 0; i < 3; i++) Li[i] += c[i];
                }
                j->count += j->nvrl;
            }
            if (ns > 1)
                for (int i = 0; i < 3; i++) Li[i] /= (float)ns;
        }
        for (int i = 0; i < 3; i++) j->out[3 * (size_t)r + i] = Li[i];
    }
    return NULL;
}

/* getClusteredVrlContributions, vrlIntegrator.cpp:542-599 */
static void *clustered_worker(void *arg)
{
    gjob *j = (gjob *)arg;
    for (uint32_t r = j->r0; r < j->r1; r++) {
        const float *rec = j->recs + (size_t)r * ALVRL_O_REC_WORDS;
        uint32_t flags;
        memcpy(&flags, &rec[15], 4);
        float Li[3] = { 0, 0, 0 };
        uint32_t rid = j->rec_ids ? j->rec_ids[r] : r;
        if (flags & ALVRL_O_FLAG_MEDIUM) {
            uint32_t s = j->slice_of_rec[r];
            const uint32_t *vr;
            const float *w;
            uint32_t k;
            if (s == 0xFFFFFFFFu) { vr = j->fb_reps; w = j->fb_weights; k = j->n_fb; }
            else {
                vr = j->reps + j->slice_off[s];
                w = j->weights + j->slice_off[s];
                k = j->slice_off[s + 1] - j->slice_off[s];
            }
            for (uint32_t i = 0; i < k; i++) {
                float c[3];
                alvrl_o_integrate_vrl(j->P, rec, rid, j->vs, j->nvrl, vr[i], j->domain, c, NULL, NULL);
                for (int ch = 0; ch < 3; ch++) Li[ch] += c[ch] * w[i];
            }
            float rp = 1.0f / (float)j->pc;   /* Li /= particleCount (spectrum.h:447-455) */
            for (int ch = 0; ch < 3; ch++) Li[ch] *= rp;
            for (int ch = 0; ch < 3; ch++) Li[ch] = Li[ch] * rec[16 + ch];   /* return Li * weight (:598) */
            j->count += k;
        }
        for (int ch = 0; ch < 3; ch++) j->out[3 * (size_t)r + ch] = Li[ch];
    }
    return NULL;
}

static uint64_t run_jobs(gjob *proto, void *(*fn)(void *), uint32_t nrec, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > nrec && nrec > 0) nthreads = (int)nrec;
    gjob *jobs = (gjob *)calloc((size_t)nthreads, sizeof(gjob));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = *proto;
        jobs[t].r0 = (uint32_t)(((uint64_t)t * nrec) / nthreads);
        jobs[t].r1 = (uint32_t)(((uint64_t)(t + 1) * nrec) / nthreads);
        jobs[t].count = 0;
        if (nthreads > 1) pthread_create(&th[t], NULL, fn, &jobs[t]);
        else fn(&jobs[t]);
    }
    uint64_t total = 0;
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        total += jobs[t].count;
    }
    free(jobs);
    free(th);
    return total;
}

uint64_t alvrl_o_gather_brute(const alvrl_o_params *P, const float *recs, uint32_t nrec,
                              const uint32_t *rec_ids, const float *vrl_soa, uint32_t nvrl,
                              uint64_t particle_count, uint32_t domain,
                              float *out_rgb, float *R_rows, int nthreads)
{
    gjob j;
    memset(&j, 0, sizeof(j));
    j.P = P; j.recs = recs; j.nrec = nrec; j.rec_ids = rec_ids; j.vs = vrl_soa; j.nvrl = nvrl;
    j.pc = particle_count; j.domain = domain; j.out = out_rgb; j.R = R_rows;
    if (R_rows) memset(R_rows, 0, sizeof(float) * 2 * (size_t)nrec * nvrl);
    return run_jobs(&j, brute_worker, nrec, nthreads);
}

uint64_t alvrl_o_gather_clustered(const alvrl_o_params *P, const float *recs, uint32_t nrec,
                                  const uint32_t *rec_ids, const uint32_t *slice_of_rec,
                                  const float *vrl_soa, uint32_t nvrl, uint64_t particle_count,
                                  const uint32_t *slice_off, const uint32_t *reps, const float *weights,
                                  const uint32_t *fb_reps, const float *fb_weights, uint32_t n_fb,
                                  float *out_rgb, int nthreads)
{
    gjob j;
    memset(&j, 0, sizeof(j));
    j.P = P; j.recs = recs; j.nrec = nrec; j.rec_ids = rec_ids; j.vs = vrl_soa; j.nvrl = nvrl;
    j.pc = particle_count; j.domain = ALVRL_O_DOM_GATHER; j.out = out_rgb;
    j.slice_of_rec = slice_of_rec; j.slice_off = slice_off; j.reps = reps; j.weights = weights;
    j.fb_reps = fb_reps; j.fb_weights = fb_weights; j.n_fb = n_fb;
    return run_jobs(&j, clustered_worker, nrec, nthreads);
}

/* ===================================================================== */
/*  Smoke-box scene harness                                                */
/* ===================================================================== */
void alvrl_o_scene_default(alvrl_o_scene *s, int width, int height)
{
    /* BASELINE.md "homogeneous smoke box" */
    memset(s, 0, sizeof(*s));
    s->cam_origin[0] = 0; s->cam_origin[1] = 0; s->cam_origin[2] = -0.9f;
    s->cam_target[0] = 0; s->cam_target[1] = 0; s->cam_target[2] = 1.0f;
    s->cam_up[0] = 0; s->cam_up[1] = 1; s->cam_up[2] = 0;
    s->fov_x_deg = 60.0f;
    s->width = width; s->height = height;
    for (int i = 0; i < 3; i++) {
        s->box_min[i] = -1.0f; s->box_max[i] = 1.0f;
        s->albedo[i] = 0.5f;
        s->light_intensity[i] = 10.0f;
    }
    s->light_pos[0] = 0; s->light_pos[1] = 0.8f; s->light_pos[2] = 0;
    s->occ_eta = 1.5046f / 1.000277f;   /* bk7 / air (ior.h:43, 60) */
}

/* fresnelDielectricExt (src/libcore/util.cpp:651-681) */
static float fresnel_dielectric_ext(float cos_theta_i, float *cos_theta_t, float eta)
{
    if (eta == 1) {
        *cos_theta_t = -cos_theta_i;
        return 0.0f;
    }
    float scale = (cos_theta_i > 0) ? 1 / eta : eta;
    float cos_t_sqr = 1 - (1 - cos_theta_i * cos_theta_i) * (scale * scale);
    if (cos_t_sqr <= 0.0f) {
        *cos_theta_t = 0.0f;
        return 1.0f;
    }
    float ci = fabsf(cos_theta_i);
    float ct = sqrtf(cos_t_sqr);
    float Rs = (ci - eta * ct) / (ci + eta * ct);
    float Rp = (eta * ci - ct) / (eta * ci + ct);
    *cos_theta_t = (cos_theta_i > 0) ? -ct : ct;
    return 0.5f * (Rs * Rs + Rp * Rp);
}

/* Perspective pinhole with Mitsuba's conventions (perspective.cpp:126-155,
 * 247-269; Transform::lookAt): camera-space x = 'left', y = up, z = forward,
 * sample (0,0) = upper-left.  Evaluated analytically in float. */
void alvrl_o_camera_ray(const alvrl_o_scene *s, float px, float py, float o[3], float d[3])
{
    v3 org = ld3(s->cam_origin), tgt = ld3(s->cam_target), up = ld3(s->cam_up);
    v3 fwd = nrm(sub(tgt, org));
    v3 left = nrm(cross(up, fwd));
    v3 nup = cross(fwd, left);
    float aspect = (float)s->width / (float)s->height;
    float tanh_ = tanf(0.5f * s->fov_x_deg * (float)(M_PI / 180.0));
    float sx = px * (1.0f / (float)s->width);
    float sy = py * (1.0f / (float)s->height);
    float xc = (1.0f - 2.0f * sx) * tanh_;
    float yc = ((1.0f - 2.0f * sy) / aspect) * tanh_;
    v3 dc = nrm(mk(xc, yc, 1.0f));
    v3 dw = mk(left.x * dc.x + nup.x * dc.y + fwd.x * dc.z,
               left.y * dc.x + nup.y * dc.y + fwd.y * dc.z,
               left.z * dc.x + nup.z * dc.y + fwd.z * dc.z);
    o[0] = org.x; o[1] = org.y; o[2] = org.z;
    d[0] = dw.x; d[1] = dw.y; d[2] = dw.z;
}

/* ray.mint of sampleRay (perspective.cpp:258-260): nearClip (1e-2) / d.z in camera space */
static float camera_mint(const alvrl_o_scene *s, float px, float py)
{
    float aspect = (float)s->width / (float)s->height;
    float tanh_ = tanf(0.5f * s->fov_x_deg * (float)(M_PI / 180.0));
    float sx = px * (1.0f / (float)s->width);
    float sy = py * (1.0f / (float)s->height);
    float xc = (1.0f - 2.0f * sx) * tanh_;
    float yc = ((1.0f - 2.0f * sy) / aspect) * tanh_;
    v3 dc = nrm(mk(xc, yc, 1.0f));
    return 1e-2f * (1.0f / dc.z);
}

/* Ray / inner-box-wall intersection from inside the box.  Returns t and the
 * inward wall normal (the walls' BSDF is one-sided diffuse facing inward). */
static float box_hit(const alvrl_o_scene *s, v3 o, v3 d, v3 *n)
{
    float best = INFINITY;
    int axis = -1;
    float oo[3] = { o.x, o.y, o.z }, dd[3] = { d.x, d.y, d.z };
    for (int a = 0; a < 3; a++) {
        float t;
        if (dd[a] > 0) t = (s->box_max[a] - oo[a]) / dd[a];
        else if (dd[a] < 0) t = (s->box_min[a] - oo[a]) / dd[a];
        else continue;
        if (t < best) { best = t; axis = a; }
    }
    float nn[3] = { 0, 0, 0 };
    if (axis >= 0) nn[axis] = dd[axis] > 0 ? -1.0f : 1.0f;
    *n = mk(nn[0], nn[1], nn[2]);
    return best;
}

/* Scene::rayIntersect over the walls and the occluders (shape kd-tree leaf
 * test t in [mint, maxt], skdtree.h:248-262; hit record skdtree.h:350-396:
 * barycentric position, face normal).  Ties: the walls, then the lowest
 * triangle index (the reference's kd-tree order is unspecified there). */
static float first_hit(const alvrl_o_scene *s, v3 o, v3 d, float mint, v3 *n, v3 *p, int *tri)
{
    float best = box_hit(s, o, d, n);
    int bi = -1;
    float bu = 0.0f, bv = 0.0f;
    for (uint32_t i = 0; i < s->nocc; i++) {
        float u, v, t;
        if (!tri_intersect(s->occ + 9 * (size_t)i, o, d, &u, &v, &t)) continue;
        if (t < mint || !(t < best)) continue;
        best = t; bi = (int)i; bu = u; bv = v;
    }
    *tri = bi;
    if (bi < 0) { *p = add(o, scl(d, best)); return best; }
    const float *q = s->occ + 9 * (size_t)bi;
    v3 p0 = mk(q[0], q[1], q[2]), p1 = mk(q[3], q[4], q[5]), p2 = mk(q[6], q[7], q[8]);
    float b0 = 1 - bu - bv;
    *p = add(add(scl(p0, b0), scl(p1, bu)), scl(p2, bv));
    v3 fn = cross(sub(p1, p0), sub(p2, p0));
    float l = len(fn);
    if (!(fn.x == 0 && fn.y == 0 && fn.z == 0)) fn = scl(fn, 1.0f / l);
    *n = fn;
    return best;
}

float alvrl_o_first_hit(const alvrl_o_scene *s, const float o[3], const float d[3], float mint,
                        float n[3], float p[3], int *tri)
{
    v3 nn, pp;
    float t = first_hit(s, ld3(o), ld3(d), mint, &nn, &pp, tri);
    n[0] = nn.x; n[1] = nn.y; n[2] = nn.z;
    p[0] = pp.x; p[1] = pp.y; p[2] = pp.z;
    return t;
}

/* The sensor sample of pixel (x, y), sample j of spp (renderBlock,
 * integrator.cpp:240-247): the pixel centre when the sampler takes one
 * sample, else offset + rRec.nextSample2D(), here draws 0 and 1 of the
 * counter stream (seed, pass, dom 8, pixel, sample). */
void alvrl_o_pixel_sample(uint32_t seed, uint32_t pass, int x, int y, int width, uint32_t sample, uint32_t spp,
                          float *px, float *py)
{
    if (spp <= 1) {
        *px = (float)x + 0.5f;
        *py = (float)y + 0.5f;
        return;
    }
    const uint32_t pixel = (uint32_t)y * (uint32_t)width + (uint32_t)x;
    *px = (float)x + draw(seed, pass, ALVRL_O_DOM_PIXEL, pixel, sample, 0u, 0u);
    *py = (float)y + draw(seed, pass, ALVRL_O_DOM_PIXEL, pixel, sample, 0u, 1u);
}

/* The diffuse reflectance of occluder tri: its own (occ_albedos) or the
 * shared occ_albedo */
static const float *occ_alb(const alvrl_o_scene *s, int tri)
{
    return s->occ_albedos ? s->occ_albedos + 3 * (size_t)tri : s->occ_albedo;
}

/* The record of sensor sample j of pixel (x, y); its depth word carries the
 * sample index in bits 16-31 (the gather's streams are keyed by it). */
void alvrl_o_make_record_s(const alvrl_o_scene *s, int medium_scatters, int x, int y, uint32_t seed, uint32_t pass,
                           uint32_t sample, uint32_t spp, float *rec)
{
    float o[3], d[3], px, py;
    alvrl_o_pixel_sample(seed, pass, x, y, s->width, sample, spp, &px, &py);
    alvrl_o_camera_ray(s, px, py, o, d);
    v3 O = ld3(o), D = ld3(d), n, p;
    int tri;
    float t = first_hit(s, O, D, camera_mint(s, px, py), &n, &p, &tri);
    static const float zero3[3] = { 0.0f, 0.0f, 0.0f };
    uint32_t mt = (tri >= 0 && s->occ_mat) ? s->occ_mat[tri] : ALVRL_O_MAT_DIFFUSE;
    const float *alb = mt != ALVRL_O_MAT_DIFFUSE ? zero3 : (tri >= 0 ? occ_alb(s, tri) : s->albedo);
    uint32_t flags = 0;
    if (isfinite(t)) flags |= ALVRL_O_FLAG_HIT | (mt == ALVRL_O_MAT_DIFFUSE ? ALVRL_O_FLAG_SMOOTH : ALVRL_O_FLAG_DELTA);
    if (medium_scatters) flags |= ALVRL_O_FLAG_MEDIUM;
    rec[0] = O.x; rec[1] = O.y; rec[2] = O.z;
    rec[3] = D.x; rec[4] = D.y; rec[5] = D.z;
    rec[6] = p.x; rec[7] = p.y; rec[8] = p.z;
    rec[9] = n.x; rec[10] = n.y; rec[11] = n.z;
    rec[12] = alb[0]; rec[13] = alb[1]; rec[14] = alb[2];
    memcpy(&rec[15], &flags, 4);
    rec[16] = rec[17] = rec[18] = 1.0f;   /* the camera ray: weight 1, depth 0 */
    uint32_t depth = sample << 16;
    memcpy(&rec[19], &depth, 4);
}

void alvrl_o_make_record(const alvrl_o_scene *s, int medium_scatters, int x, int y, float *rec)
{
    alvrl_o_make_record_s(s, medium_scatters, x, y, 0u, 0u, 0u, 1u, rec);
}

static uint32_t mat_of(const alvrl_o_scene *s, int tri)
{
    return (tri >= 0 && s->occ_mat) ? s->occ_mat[tri] : ALVRL_O_MAT_DIFFUSE;
}

static void frame_of(v3 a, v3 *b, v3 *c);

void alvrl_o_make_slice_record(const alvrl_o_scene *s, int x, int y, float *rec)
{
    float o[3], d[3];
    alvrl_o_camera_ray(s, (float)x + 0.5f, (float)y + 0.5f, o, d);
    v3 O = ld3(o), D = ld3(d), n, p;
    int tri;
    float t = first_hit(s, O, D, camera_mint(s, (float)x + 0.5f, (float)y + 0.5f), &n, &p, &tri);
    uint32_t flags = 0;
    v3 gp = p, gn = n;
    if (isfinite(t)) {
        flags = ALVRL_O_FLAG_HIT;
        for (;;) {   /* Preprocessor.cpp:1157-1169: keep going through null surfaces */
            gp = p; gn = n;
            if (mat_of(s, tri) != ALVRL_O_MAT_NULL) break;
            t = first_hit(s, O, D, t + 1e-4f, &n, &p, &tri);   /* Ray(ray, its.t + Epsilon, ray.maxt) */
            if (!isfinite(t)) break;
        }
    }
    for (int k = 0; k < ALVRL_O_REC_WORDS; k++) rec[k] = 0.0f;
    rec[0] = O.x; rec[1] = O.y; rec[2] = O.z;
    rec[3] = D.x; rec[4] = D.y; rec[5] = D.z;
    rec[6] = gp.x; rec[7] = gp.y; rec[8] = gp.z;
    rec[9] = gn.x; rec[10] = gn.y; rec[11] = gn.z;
    memcpy(&rec[15], &flags, 4);
    rec[16] = rec[17] = rec[18] = 1.0f;
}

uint32_t alvrl_o_make_chain(const alvrl_o_scene *s, const alvrl_o_medium *m, int medium_scatters, int x, int y,
                            uint32_t seed, uint32_t pass, int spec_rr_depth, float init_throughput,
                            float *recs, uint32_t cap)
{
    return alvrl_o_make_chain_s(s, m, medium_scatters, x, y, seed, pass, spec_rr_depth, init_throughput, 0u, 1u,
                                recs, cap);
}

/* One LiInternal call (:398-524): the record of the ray's hit, then each
 * delta component's continuation, depth first.  depth: rRec.depth. */
typedef struct {
    const alvrl_o_scene *s;
    const alvrl_o_medium *m;
    int medium_scatters, spec_rr_depth;
    uint32_t seed, pass, pixel, sample, cap, nrec;
    float *recs;
} chain_ctx;

static void chain_node(chain_ctx *cx, v3 O, v3 D, float mint, const float weight[3], const float thr[3], int depth)
{
    const alvrl_o_scene *s = cx->s;
    if (cx->nrec >= cx->cap || cx->nrec >= 256) return;
    v3 n, p;
    int tri;
    float t = first_hit(s, O, D, mint, &n, &p, &tri);
    if (!isfinite(t)) return;                                               /* :414-419 */
    uint32_t mt = mat_of(s, tri);
    uint32_t flags = ALVRL_O_FLAG_HIT | (mt == ALVRL_O_MAT_DIFFUSE ? ALVRL_O_FLAG_SMOOTH : ALVRL_O_FLAG_DELTA) |
                     (cx->medium_scatters ? ALVRL_O_FLAG_MEDIUM : 0u);
    const float *alb = tri >= 0 ? occ_alb(s, tri) : s->albedo;
    float *rec = cx->recs + (size_t)cx->nrec * ALVRL_O_REC_WORDS;
    rec[0] = O.x; rec[1] = O.y; rec[2] = O.z;
    rec[3] = D.x; rec[4] = D.y; rec[5] = D.z;
    rec[6] = p.x; rec[7] = p.y; rec[8] = p.z;
    rec[9] = n.x; rec[10] = n.y; rec[11] = n.z;
    for (int i = 0; i < 3; i++) rec[12 + i] = mt == ALVRL_O_MAT_DIFFUSE ? alb[i] : 0.0f;
    memcpy(&rec[15], &flags, 4);
    for (int i = 0; i < 3; i++) rec[16 + i] = weight[i];
    const uint32_t kw = cx->nrec | (cx->sample << 16);
    memcpy(&rec[19], &kw, 4);
    cx->nrec++;
    if (mt == ALVRL_O_MAT_DIFFUSE) return;                                  /* no delta component (:447-448) */
    /* rRec.medium->eval(Ray(ray, 0, its.t)) (:450-460) */
    float tr[3];
    for (int i = 0; i < 3; i++) tr[i] = fastexp(cx->m->sigma_t[i] * (-t));
    {
        float mx = tr[0] > tr[1] ? tr[0] : tr[1];
        mx = mx > tr[2] ? mx : tr[2];
        if (mx < 1e-20f) tr[0] = tr[1] = tr[2] = 0;
    }
    if (tr[0] == 0 && tr[1] == 0 && tr[2] == 0) return;
    v3 fs, ft;
    frame_of(n, &fs, &ft);
    v3 mwi = neg(D);
    float cos_wi = dot(mwi, n);
    seq_sampler smp;
    seq_init(&smp, cx->seed, cx->pass, 7u, cx->pixel, kw, 0u);
    int ncomp = mt == ALVRL_O_MAT_DIELECTRIC ? 2 : 1;
    for (int c = 0; c < ncomp; c++) {                                       /* :467-511 */
        float bw[3];
        float beta = 1.0f;                                                  /* bRec.eta */
        v3 wol;
        if (mt == ALVRL_O_MAT_MIRROR) {                                     /* conductor.cpp:254-268 */
            if (cos_wi <= 0) continue;
            wol = mk(-dot(mwi, fs), -dot(mwi, ft), cos_wi);
            for (int i = 0; i < 3; i++) bw[i] = s->occ_spec[i];
        } else if (mt == ALVRL_O_MAT_NULL) {                                /* null.cpp:53-63 */
            wol = mk(-dot(mwi, fs), -dot(mwi, ft), -cos_wi);
            bw[0] = bw[1] = bw[2] = 1.0f;
        } else {                                                            /* dielectric.cpp:365-385, ERadiance */
            float cos_t;
            float F = fresnel_dielectric_ext(cos_wi, &cos_t, s->occ_eta);
            float inv_eta = 1 / s->occ_eta;
            if (c == 0) {
                wol = mk(-dot(mwi, fs), -dot(mwi, ft), cos_wi);
                bw[0] = bw[1] = bw[2] = F;
            } else {
                float scale = -(cos_t < 0 ? inv_eta : s->occ_eta);
                wol = mk(scale * dot(mwi, fs), scale * dot(mwi, ft), cos_t);
                beta = cos_t < 0 ? s->occ_eta : inv_eta;
                float factor = cos_t < 0 ? inv_eta : s->occ_eta;
                bw[0] = bw[1] = bw[2] = factor * factor * (1 - F);
            }
            if (bw[0] == 0) continue;
        }
        /* Russian roulette (:480-492) */
        float thr2[3];
        for (int i = 0; i < 3; i++) thr2[i] = ((thr[i] * tr[i]) * bw[i]) * (beta * beta);
        float maxRR = depth >= cx->spec_rr_depth ? 0.98f : 1.0f;
        float mx = thr2[0] > thr2[1] ? thr2[0] : thr2[1];
        mx = mx > thr2[2] ? mx : thr2[2];
        float rrProb = maxRR < mx ? maxRR : mx;
        if (rrProb <= 0 || (rrProb < 1 && seq_next(&smp) > rrProb)) continue;
        float thr_c[3], w_c[3];
        for (int i = 0; i < 3; i++) {
            thr_c[i] = thr2[i] / rrProb;
            w_c[i] = ((weight[i] * tr[i]) * bw[i]) / rrProb;                 /* :505 */
        }
        v3 D2 = add(add(scl(fs, wol.x), scl(ft, wol.y)), scl(n, wol.z));    /* its.toWorld(bRec.wo) */
        chain_node(cx, p, D2, 1e-4f, w_c, thr_c, depth + 1);
    }
}

/* The eye path of sensor sample j of spp: record k's depth word is
 * k | (j << 16), and the Russian roulette draws from the (pixel, k | (j << 16))
 * stream (sample 0: the single-sample streams). */
uint32_t alvrl_o_make_chain_s(const alvrl_o_scene *s, const alvrl_o_medium *m, int medium_scatters, int x, int y,
                              uint32_t seed, uint32_t pass, int spec_rr_depth, float init_throughput,
                              uint32_t sample, uint32_t spp, float *recs, uint32_t cap)
{
    float o[3], d[3], px, py;
    alvrl_o_pixel_sample(seed, pass, x, y, s->width, sample, spp, &px, &py);
    alvrl_o_camera_ray(s, px, py, o, d);   /* the sensor sample (integrator.cpp:240-247) */
    chain_ctx cx;
    cx.s = s; cx.m = m; cx.medium_scatters = medium_scatters; cx.spec_rr_depth = spec_rr_depth;
    cx.seed = seed; cx.pass = pass; cx.pixel = (uint32_t)y * (uint32_t)s->width + (uint32_t)x;
    cx.sample = sample; cx.cap = cap; cx.nrec = 0; cx.recs = recs;
    float weight[3] = { 1.0f, 1.0f, 1.0f };
    float thr[3] = { init_throughput, init_throughput, init_throughput };   /* throughputWithEtaSq */
    chain_node(&cx, ld3(o), ld3(d), camera_mint(s, px, py), weight, thr, 1);   /* rRec.depth 1 */
    return cx.nrec;
}

void alvrl_o_make_records(const alvrl_o_scene *s, int medium_scatters, float *recs)
{
    for (int y = 0; y < s->height; y++)
        for (int x = 0; x < s->width; x++)
            alvrl_o_make_record(s, medium_scatters, x, y,
                                recs + ((size_t)y * s->width + x) * ALVRL_O_REC_WORDS);
}

/* ===================================================================== */
/*  VRL tracer (vrlTracer.h:13-230) in the smoke box                       */
/* ===================================================================== */
/* warp::squareToUniformSphere, src/libcore/warp.cpp:25-31 */
static v3 uniform_sphere(float sx, float sy)
{
    float z = 1.0f - 2.0f * sy;
    float r = safe_sqrt(1.0f - z * z);
    float theta = (float)(2.0f * M_PI * sx);
    /* sin/cos evaluated in double and rounded once: the correctly rounded float
       value, reproducible on the device (tracer.hip) -- libm's sinf/cosf are not */
    float sp = (float)sin((double)theta), cp = (float)cos((double)theta);
    return mk(r * cp, r * sp, z);
}

/* warp::squareToUniformDiskConcentric + squareToCosineHemisphere (warp.cpp:43-52, 81-102) */
static v3 cosine_hemisphere(float sx, float sy)
{
    float r1 = 2.0f * sx - 1.0f;
    float r2 = 2.0f * sy - 1.0f;
    float phi, r;
    if (r1 == 0 && r2 == 0) { r = phi = 0; }
    else if (r1 * r1 > r2 * r2) { r = r1; phi = (float)((M_PI / 4.0f) * (r2 / r1)); }
    else { r = r2; phi = (float)((M_PI / 2.0f) - (r1 / r2) * (M_PI / 4.0f)); }
    float sp = (float)sin((double)phi), cp = (float)cos((double)phi);
    float px = r * cp, py = r * sp;
    float z = safe_sqrt(1.0f - px * px - py * py);
    if (z == 0) z = 1e-10f;
    return mk(px, py, z);
}

/* coordinateSystem, src/libcore/util.cpp:592-601 (Frame(n), frame.h:55-57) */
static void frame_of(v3 a, v3 *b, v3 *c)
{
    if (fabsf(a.x) > fabsf(a.y)) {
        float invLen = 1.0f / sqrtf(a.x * a.x + a.z * a.z);
        *c = mk(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / sqrtf(a.y * a.y + a.z * a.z);
        *c = mk(0.0f, a.z * invLen, -a.y * invLen);
    }
    *b = cross(*c, a);
}

typedef struct {
    float *soa; uint32_t cap, n;
    v3 start; float power[3];
    int sigma_s_zero;
} vrl_sink;

/* vrlVector::put filter (VRL.h:148-158) */
static void vrl_put(vrl_sink *k, v3 end)
{
    if (k->sigma_s_zero) return;
    if (k->power[0] == 0 && k->power[1] == 0 && k->power[2] == 0) return;
    if (dist(k->start, end) == 0) return;
    if (k->n >= k->cap) return;
    uint32_t i = k->n++, c = k->cap;
    k->soa[0 * c + i] = k->start.x; k->soa[1 * c + i] = k->start.y; k->soa[2 * c + i] = k->start.z;
    k->soa[3 * c + i] = end.x; k->soa[4 * c + i] = end.y; k->soa[5 * c + i] = end.z;
    k->soa[6 * c + i] = k->power[0]; k->soa[7 * c + i] = k->power[1]; k->soa[8 * c + i] = k->power[2];
}

/* vrlTracer::endCurrentVrl (vrlTracer.h:83-89) */
static void end_current(vrl_sink *k, v3 p)
{
    if (dist(k->start, p) == 0) return;
    vrl_put(k, p);
}

/* The area emitter's sampling table: TriMesh::prepareSamplingTable
 * (trimesh.cpp:388-403) appends Triangle::surfaceArea (0.5 |sideA x sideB|)
 * to a DiscreteDistribution (a running float sum) and normalizes it
 * (pmf.h:101-114: cdf[i] *= 1 / sum for i >= 1, the last entry 1). */
typedef struct { float *cdf; uint32_t n; float area; } area_table;

static void area_table_init(area_table *t, const float *tris, uint32_t n)
{
    t->n = n;
    t->cdf = (float *)calloc((size_t)n + 1, sizeof(float));
    t->cdf[0] = 0.0f;
    for (uint32_t i = 0; i < n; i++) {
        const float *q = tris + 9 * (size_t)i;
        v3 sideA = sub(ld3(q + 3), ld3(q)), sideB = sub(ld3(q + 6), ld3(q));
        t->cdf[i + 1] = t->cdf[i] + 0.5f * len(cross(sideA, sideB));
    }
    t->area = t->cdf[n];
    if (t->area > 0) {
        float norm = 1.0f / t->area;
        for (uint32_t i = 1; i <= n; i++) t->cdf[i] *= norm;
        t->cdf[n] = 1.0f;
    }
}

/* Scene::sampleEmitterPosition (scene.cpp:958-974; one emitter: sample.x is
 * kept and the pdf is 1) -> AreaEmitter::samplePosition (area.cpp:94-98) ->
 * TriMesh::samplePosition (trimesh.cpp:412-423: the triangle by
 * m_areaDistr.sampleReuse(sample.y), pmf.h:124-169) -> Triangle::sample with
 * squareToUniformTriangle (triangle.cpp:24-59, warp.cpp:76-79); power =
 * m_power = radiance * pi * area (area.cpp:198); then sampleDirection: a
 * cosine-weighted direction in Frame(n), weight 1 (area.cpp:115-123). */
static v3 area_emission(const alvrl_o_scene *s, const area_table *t, float sx, float sy, float dx, float dy,
                        v3 *dir, float power[3])
{
    uint32_t lb = 0;
    while (lb <= t->n && t->cdf[lb] < sy) lb++;            /* std::lower_bound */
    int64_t idx = (int64_t)lb - 1;
    if (idx < 0) idx = 0;
    if (idx > (int64_t)t->n - 1) idx = (int64_t)t->n - 1;
    /* a zero-area triangle is skipped (past the last one the reference would read outside the table) */
    while (idx + 1 < (int64_t)t->n && t->cdf[idx + 1] - t->cdf[idx] == 0) idx++;
    float y = (sy - t->cdf[idx]) / (t->cdf[idx + 1] - t->cdf[idx]);
    float a = safe_sqrt(1.0f - sx);
    float bx = 1 - a, by = a * y;
    const float *q = s->emit + 9 * (size_t)idx;
    v3 p0 = ld3(q), sideA = sub(ld3(q + 3), p0), sideB = sub(ld3(q + 6), p0);
    v3 p = add(add(p0, scl(sideA, bx)), scl(sideB, by));
    v3 nn = nrm(cross(sideA, sideB));
    for (int i = 0; i < 3; i++) power[i] = (s->emit_radiance[i] * (float)M_PI) * t->area;
    v3 l = cosine_hemisphere(dx, dy), fs, ft;
    frame_of(nn, &fs, &ft);
    *dir = add(add(scl(fs, l.x), scl(ft, l.y)), scl(nn, l.z));
    return p;
}

static void trace_particle(const alvrl_o_scene *s, const alvrl_o_medium *m, const area_table *at,
                           seq_sampler *smp, int short_vrls, int max_depth, int rr_depth, vrl_sink *k)
{
    /* sampleEmitterPosition (scene.cpp:958-974) + PointEmitter::samplePosition (point.cpp:81-89) */
    float sx = seq_next(smp), sy = seq_next(smp);
    float power[3];
    /* PointEmitter::sampleDirection (point.cpp:99-106) */
    float dx = seq_next(smp), dy = seq_next(smp);
    v3 dir, o;
    if (at) {
        o = area_emission(s, at, sx, sy, dx, dy, &dir, power);
    } else {
        for (int i = 0; i < 3; i++) power[i] = s->light_intensity[i] * (float)(4 * M_PI);
        dir = uniform_sphere(dx, dy);
        o = ld3(s->light_pos);
    }
    if (power[0] == 0 && power[1] == 0 && power[2] == 0) return;
    /* handleEmission: m_vrls->nextParticle() is counted by the caller */
    k->start = o;
    for (int i = 0; i < 3; i++) k->power[i] = power[i];

    int depth = 1;
    float thr[3] = { 1, 1, 1 };
    float eta = 1.0f;
    float mint = 1e-4f;   /* Ray() default (Epsilon); 0 after a medium, Epsilon after a surface */
    while (!(thr[0] == 0 && thr[1] == 0 && thr[2] == 0) && (depth <= max_depth || max_depth < 0)) {
        v3 n, hp;
        int tri;
        float its_t = first_hit(s, o, dir, mint, &n, &hp, &tri);
        int its_valid = isfinite(its_t);
        /* HomogeneousMedium::sampleDistance (homogeneous.cpp:275-352) */
        float pdf_max = 0.0f;
        float sampled = medium_sample_distance(m, smp, &pdf_max);
        float distSurf = its_t - 0.0f;
        int success = 1;
        v3 mp = o;
        if (sampled < distSurf) {
            float mt = sampled + 0.0f;
            mp = add(o, scl(dir, mt));
            if (mp.x == o.x && mp.y == o.y && mp.z == o.z) success = 0;
        } else {
            sampled = distSurf;
            success = 0;
        }
        float pf, ps;
        medium_pdfs(m, sampled, pdf_max, &ps, &pf);
        float mtr[3];
        for (int i = 0; i < 3; i++) mtr[i] = fastexp(m->sigma_t[i] * (-sampled));
        {
            float mx = mtr[0] > mtr[1] ? mtr[0] : mtr[1];
            mx = mx > mtr[2] ? mx : mtr[2];
            if (mx < 1e-20f) mtr[0] = mtr[1] = mtr[2] = 0;
        }
        if (success) {
            /* medium interaction (vrlTracer.h:143-172) */
            float rps = 1.0f / ps;
            for (int i = 0; i < 3; i++) thr[i] *= mtr[i] * m->sigma_s[i] * rps;
            float px_ = seq_next(smp), py_ = seq_next(smp);
            v3 wo = uniform_sphere(px_, py_);   /* isotropic phase sample: weight 1 */
            v3 endPoint = short_vrls ? mp : hp;
            end_current(k, endPoint);
            k->start = mp;
            for (int i = 0; i < 3; i++) k->power[i] = thr[i] * power[i];
            o = mp; dir = wo; mint = 0.0f;
        } else if (its_valid) {
            /* surface interaction (vrlTracer.h:173-213) */
            float rpf = 1.0f / pf;
            for (int i = 0; i < 3; i++) thr[i] *= mtr[i] * rpf;
            v3 p = hp;
            const float *alb = tri >= 0 ? occ_alb(s, tri) : s->albedo;
            v3 fs, ft;
            frame_of(n, &fs, &ft);
            v3 mwi = neg(dir);
            float cos_wi = dot(mwi, n);       /* Frame::cosTheta(toLocal(-ray.d)) */
            float bx = seq_next(smp), by = seq_next(smp);
            float bw[3] = { 0, 0, 0 };
            v3 wol = mk(0, 0, 0);
            uint32_t mt = mat_of(s, tri);
            if (mt == ALVRL_O_MAT_DIFFUSE) {          /* SmoothDiffuse::sample */
                if (!(cos_wi <= 0)) {
                    wol = cosine_hemisphere(bx, by);
                    for (int i = 0; i < 3; i++) bw[i] = alb[i];
                }
            } else if (mt == ALVRL_O_MAT_MIRROR) {    /* SmoothConductor::sample (conductor.cpp:254-268) */
                if (!(cos_wi <= 0)) {
                    wol = mk(-dot(mwi, fs), -dot(mwi, ft), cos_wi);
                    for (int i = 0; i < 3; i++) bw[i] = s->occ_spec[i];
                }
            } else if (mt == ALVRL_O_MAT_DIELECTRIC) {   /* SmoothDielectric::sample, both components,
                                                           EImportance (dielectric.cpp:335-364) */
                float cos_t;
                float F = fresnel_dielectric_ext(cos_wi, &cos_t, s->occ_eta);
                if (bx <= F) {
                    wol = mk(-dot(mwi, fs), -dot(mwi, ft), cos_wi);
                } else {
                    float inv_eta = 1 / s->occ_eta;
                    float scale = -(cos_t < 0 ? inv_eta : s->occ_eta);
                    wol = mk(scale * dot(mwi, fs), scale * dot(mwi, ft), cos_t);
                    eta *= cos_t < 0 ? s->occ_eta : inv_eta;
                }
                bw[0] = bw[1] = bw[2] = 1.0f;
            } else {                                  /* Null::sample (null.cpp:53-63) */
                wol = mk(-dot(mwi, fs), -dot(mwi, ft), -cos_wi);
                bw[0] = bw[1] = bw[2] = 1.0f;
            }
            if (bw[0] == 0 && bw[1] == 0 && bw[2] == 0) { end_current(k, p); break; }
            v3 wo = add(add(scl(fs, wol.x), scl(ft, wol.y)), scl(n, wol.z));
            float wiDotGeoN = dot(n, mwi), woDotGeoN = dot(n, wo);
            if (wiDotGeoN * cos_wi <= 0 || woDotGeoN * wol.z <= 0) { end_current(k, p); break; }
            for (int i = 0; i < 3; i++) thr[i] *= bw[i];
            end_current(k, p);
            k->start = p;
            for (int i = 0; i < 3; i++) k->power[i] = thr[i] * power[i];
            o = p; dir = wo; mint = 1e-4f;
        } else {
            break;
        }
        if (depth++ >= rr_depth) {
            float mx = thr[0] > thr[1] ? thr[0] : thr[1];
            mx = mx > thr[2] ? mx : thr[2];
            float q = mx * eta * eta;
            if (q > 0.95f) q = 0.95f;
            if (seq_next(smp) >= q) break;
            float rq = 1.0f / q;
            for (int i = 0; i < 3; i++) thr[i] *= rq;
        }
    }
}

uint32_t alvrl_o_trace_vrls(const alvrl_o_scene *s, const alvrl_o_medium *m, uint32_t seed,
                            uint32_t pass, uint32_t target, int short_vrls, int max_depth,
                            int rr_depth, float *vrl_soa, uint32_t cap, uint64_t *particles)
{
    vrl_sink k;
    memset(&k, 0, sizeof(k));
    k.soa = vrl_soa; k.cap = cap; k.n = 0;
    k.sigma_s_zero = (m->sigma_s[0] == 0 && m->sigma_s[1] == 0 && m->sigma_s[2] == 0);
    area_table at;
    memset(&at, 0, sizeof(at));
    if (s->emit && s->nemit) area_table_init(&at, s->emit, s->nemit);
    uint64_t p = 0;
    while (k.n < target && k.n < cap) {
        seq_sampler smp;
        seq_init(&smp, seed, pass, ALVRL_O_DOM_TRACER, (uint32_t)p, (uint32_t)(p >> 32), 0);
        p++;   /* handleEmission -> nextParticle() (the light always emits) */
        trace_particle(s, m, at.cdf ? &at : NULL, &smp, short_vrls, max_depth, rr_depth, &k);
        if (k.sigma_s_zero && p > 1000000) break;
    }
    free(at.cdf);
    if (particles) *particles = p;
    return k.n;
}


/* ===================================================================== */
/*  volpath with onlyVRLpaths (src/integrators/path/volpath.cpp:110-457)   */
/* ===================================================================== */
#define ALVRL_O_DOM_VOLPATH 6u

/* Scene::sampleAttenuatedEmitterDirect + PointEmitter::sampleDirect
 * (scene.cpp:854-898, point.cpp:131-147), one emitter (emPdf = 1) */
static void vp_light_direct(const alvrl_o_scene *s, const alvrl_o_medium *m, v3 ref, int on_surface,
                            float val[3], v3 *dir)
{
    v3 L = ld3(s->light_pos);
    v3 d = sub(L, ref);
    float dist = len(d);
    float invDist = 1.0f / dist;
    d = scl(d, invDist);
    *dir = d;
    /* evalTransmittance(ref, on_surface, light, false): medium + occluders */
    v3 d0 = sub(L, ref);
    float remaining = len(d0);
    float negLength = 0.0f - remaining;
    float tr[3];
    for (int i = 0; i < 3; i++) tr[i] = m->sigma_t[i] != 0 ? fastexp(m->sigma_t[i] * negLength) : 1.0f;
    if (!segment_visible(s->occ, s->occ_mat, s->nocc, ref, on_surface, L)) tr[0] = tr[1] = tr[2] = 0.0f;
    for (int i = 0; i < 3; i++) {
        val[i] = s->light_intensity[i] * (invDist * invDist);
        val[i] *= tr[i] * 1.0f;
    }
}

static void vp_li(const alvrl_o_scene *s, const alvrl_o_medium *m, const alvrl_o_volpath_params *vp,
                  seq_sampler *smp, v3 o, v3 dir, float mint, float Li[3])
{
    Li[0] = Li[1] = Li[2] = 0.0f;
    int first_ok = 0, second_ok = 0, prev_diffuse = 0, prev_volume = 0;
    v3 n, hp;
    int tri;
    float its_t = first_hit(s, o, dir, mint, &n, &hp, &tri);
    float thr[3] = { 1, 1, 1 };
    float eta = 1.0f;
    int depth = 1;
    while (depth <= vp->max_depth || vp->max_depth < 0) {
        if (vp->only_vrl_paths && depth > 2 && !(first_ok && second_ok)) break;   /* :144-145 */
        float pdf_max = 0.0f;
        float sampled = medium_sample_distance(m, smp, &pdf_max);
        float distSurf = its_t - 0.0f;
        int success = 1;
        v3 mp = o;
        if (sampled < distSurf) {
            mp = add(o, scl(dir, sampled + 0.0f));
            if (mp.x == o.x && mp.y == o.y && mp.z == o.z) success = 0;
        } else {
            sampled = distSurf;
            success = 0;
        }
        float pf, ps;
        medium_pdfs(m, sampled, pdf_max, &ps, &pf);
        float mtr[3];
        for (int i = 0; i < 3; i++) mtr[i] = fastexp(m->sigma_t[i] * (-sampled));
        {
            float mx = mtr[0] > mtr[1] ? mtr[0] : mtr[1];
            mx = mx > mtr[2] ? mx : mtr[2];
            if (mx < 1e-20f) mtr[0] = mtr[1] = mtr[2] = 0;
        }
        if (success) {   /* :150-267 */
            if (depth == 1 && vp->vrl_vol_to_vol) first_ok = 1;
            if (depth == 2) second_ok = 1;
            if (depth >= vp->max_depth && vp->max_depth != -1) break;
            float rps = 1.0f / ps;
            for (int i = 0; i < 3; i++) thr[i] *= (m->sigma_s[i] * mtr[i]) * rps;
            /* "(!rRec.depth==2 || (...))" parses as "((!depth) == 2 || (...))" (:183-190) */
            int nee = !vp->only_vrl_paths ||
                      (depth != 1 && (prev_volume || prev_diffuse) && (!prev_diffuse || vp->vrl_vol_to_surf) &&
                       (!prev_volume || vp->vrl_vol_to_vol));
            if (nee) {
                (void)seq_next(smp); (void)seq_next(smp);
                float val[3];
                v3 ld;
                vp_light_direct(s, m, mp, 0, val, &ld);
                if (!(val[0] == 0 && val[1] == 0 && val[2] == 0))
                    for (int i = 0; i < 3; i++) Li[i] += ((thr[i] * val[i]) * INV_FOURPI) * 1.0f;
            }
            float px_ = seq_next(smp), py_ = seq_next(smp);
            v3 wo = uniform_sphere(px_, py_);
            o = mp; dir = wo;
            its_t = first_hit(s, o, dir, 0.0f, &n, &hp, &tri);
            prev_volume = 1;
            prev_diffuse = 0;
        } else {   /* :268-435 */
            float rpf = 1.0f / pf;
            for (int i = 0; i < 3; i++) thr[i] *= mtr[i] * rpf;
            if (!isfinite(its_t)) break;
            if (depth >= vp->max_depth && vp->max_depth != -1) break;
            const float *alb = tri >= 0 ? occ_alb(s, tri) : s->albedo;
            v3 p = hp;
            float cos_wi = dot(neg(dir), n);
            if (!vp->only_vrl_paths || (first_ok && second_ok)) {   /* :319-350 */
                (void)seq_next(smp); (void)seq_next(smp);
                float val[3];
                v3 ld;
                vp_light_direct(s, m, p, 1, val, &ld);
                if (!(val[0] == 0 && val[1] == 0 && val[2] == 0)) {
                    float cos_wo = dot(ld, n);
                    if (!(cos_wi <= 0 || cos_wo <= 0)) {
                        float k = INV_PI * cos_wo;
                        for (int i = 0; i < 3; i++) Li[i] += ((thr[i] * val[i]) * (alb[i] * k)) * 1.0f;
                    }
                }
            }
            float bx = seq_next(smp), by = seq_next(smp);   /* diffuse.cpp:140-150 */
            if (cos_wi <= 0) break;
            v3 wol = cosine_hemisphere(bx, by);
            v3 fs, ft;
            frame_of(n, &fs, &ft);
            v3 wo = add(add(scl(fs, wol.x), scl(ft, wol.y)), scl(n, wol.z));
            if (depth == 1 && vp->vrl_vol_to_surf) first_ok = 1;   /* :377-382 */
            prev_volume = 0;
            prev_diffuse = 1;
            for (int i = 0; i < 3; i++) thr[i] *= alb[i];
            o = p; dir = wo;
            its_t = first_hit(s, o, dir, 1e-4f, &n, &hp, &tri);
        }
        if (depth++ >= vp->rr_depth) {   /* :437-446 */
            float mx = thr[0] > thr[1] ? thr[0] : thr[1];
            mx = mx > thr[2] ? mx : thr[2];
            float q = mx * eta * eta;
            if (q > 0.95f) q = 0.95f;
            if (seq_next(smp) >= q) break;
            float rq = 1.0f / q;
            for (int i = 0; i < 3; i++) thr[i] *= rq;
        }
    }
    if (vp->only_vrl_paths && !(first_ok && second_ok)) Li[0] = Li[1] = Li[2] = 0.0f;   /* :453-455 */
}

void alvrl_o_volpath(const alvrl_o_scene *s, const alvrl_o_medium *m, const alvrl_o_volpath_params *vp,
                     uint32_t seed, uint32_t pass, uint32_t spp, const uint32_t *pixel_ids, uint32_t n,
                     float *out_rgb)
{
    for (uint32_t i = 0; i < n; i++) {
        uint32_t id = pixel_ids ? pixel_ids[i] : i;
        float px = (float)(id % (uint32_t)s->width) + 0.5f, py = (float)(id / (uint32_t)s->width) + 0.5f;
        float o[3], d[3];
        alvrl_o_camera_ray(s, px, py, o, d);
        float mint = camera_mint(s, px, py);
        float acc[3] = { 0, 0, 0 };
        for (uint32_t k = 0; k < spp; k++) {
            seq_sampler smp;
            seq_init(&smp, seed, pass, ALVRL_O_DOM_VOLPATH, id, k, 0);
            float li[3];
            vp_li(s, m, vp, &smp, ld3(o), ld3(d), mint, li);
            for (int c = 0; c < 3; c++) acc[c] += li[c];
        }
        float r = 1.0f / (float)spp;
        for (int c = 0; c < 3; c++) out_rgb[3 * (size_t)i + c] = acc[c] * r;
    }
}
