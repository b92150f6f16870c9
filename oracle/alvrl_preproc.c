/*
 * alvrl_preproc.c -- CPU restatement of LightSlice preprocessing
 * (src/integrators/vrl/Preprocessor.cpp).  TEST INFRASTRUCTURE ONLY.
 *
 * Third-party arithmetic the reference leans on (not vendored):
 *  - boost::numeric::ublas vector ops: restated as sequential element loops
 *    (inner_prod / norm_1 / norm_2 = plain in-order sums, norm_2 unscaled).
 *  - boost::heap::priority_queue: a std::vector driven by std::push_heap /
 *    std::pop_heap; restated with libstdc++'s __push_heap / __adjust_heap, and
 *    its iteration order is the underlying vector order.
 * Random draws come from Philox streams keyed by (stage, cluster range) so that
 * refinement does not depend on thread count (the reference clones samplers
 * per worker thread, Preprocessor.cpp:738, so it has no canonical stream).
 */
#include "alvrl_oracle.h"
#include "alvrl_preproc.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>
#include <unistd.h>

#define UINT32_T_MAX 0xffffffffu
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ---------------------------------------------------------------- RNG -- */
typedef struct {
    uint32_t seed, pass, dom, a, b, c, k, blk;
    uint32_t buf[4];
} smp_t;

static void smp_init(smp_t *s, uint32_t seed, uint32_t pass, uint32_t dom, uint32_t a,
                     uint32_t b, uint32_t c)
{
    s->seed = seed; s->pass = pass; s->dom = dom; s->a = a; s->b = b; s->c = c;
    s->k = 0; s->blk = 0xFFFFFFFFu;
}

static float smp_next(smp_t *s)
{
    uint32_t blk = s->k >> 2;
    if (blk != s->blk) {
        uint32_t ctr[4] = { s->a, s->b, blk, (s->dom << 24) | (s->c & 0xFFFFFFu) };
        uint32_t key[2] = { s->seed, s->pass };
        alvrl_o_philox4x32_10(ctr, key, s->buf);
        s->blk = blk;
    }
    float v = alvrl_o_u01(s->buf[s->k & 3]);
    s->k++;
    return v;
}

/* ---------------------------------------------------- matrix accessor -- */
/* Local matrix M: rows are global row ids into Rt[v*ld + row] (mean,var). */
typedef struct {
    const float *Rt;
    uint64_t ld;
    const uint32_t *rows;
    uint32_t nrows;
    uint32_t nvrl;
} mat_t;

static inline float m_mean(const mat_t *M, uint32_t r, uint32_t v)
{
    return M->Rt[2 * ((uint64_t)v * M->ld + M->rows[r])];
}
static inline float m_var(const mat_t *M, uint32_t r, uint32_t v)
{
    return M->Rt[2 * ((uint64_t)v * M->ld + M->rows[r]) + 1];
}

/* ------------------------------------------- deterministic reductions -- */
/* Every reduction over the ROWS of a local matrix (uBLAS inner_prod / norm_2,
 * an in-order loop in the reference source that its -funsafe-math-optimizations
 * build is free to re-associate, so the reference has no canonical rounding
 * here) uses one fixed order that a 64-lane wavefront evaluates directly:
 * lane l sums rows l, l+64, l+128, ... in ascending order starting from 0,
 * then lanes are combined by the halving tree p[l] += p[l+32] (l<32),
 * p[l] += p[l+16] (l<16), ..., p[0] += p[1].  The device refinement kernel
 * (refine.hip) uses the identical order, which makes cluster indices
 * bit-exact between the two. */
#define WS_LANES 64
static double wsum_d(const double *t, uint32_t R)
{
    double p[WS_LANES];
    for (int l = 0; l < WS_LANES; l++) p[l] = 0.0;
    for (uint32_t r = 0; r < R; r++) p[r % WS_LANES] = p[r % WS_LANES] + t[r];
    for (int off = WS_LANES / 2; off >= 1; off >>= 1)
        for (int l = 0; l < off; l++) p[l] = p[l] + p[l + off];
    return p[0];
}
/* The per-prefix row sums of a split's two calculateClusterVariance passes
 * (inc_u / inc_i below) use a second fixed order, the one the device's split
 * engine forms without moving the per-row terms between waves: each 64-row
 * block is reduced by the halving tree on its own (rows past R enter as +0.0),
 * and the block totals are added in ascending block order.  Like wsum_d this
 * is a re-association of the reference's in-order inner_prod (:1107-1117). */
static double wsum_blk(const double *t, uint32_t R)
{
    double acc = 0.0;
    for (uint32_t b = 0; b * WS_LANES < R; b++) {
        double p[WS_LANES];
        for (int l = 0; l < WS_LANES; l++) {
            uint32_t r = b * WS_LANES + (uint32_t)l;
            p[l] = r < R ? t[r] : 0.0;
        }
        for (int off = WS_LANES / 2; off >= 1; off >>= 1)
            for (int l = 0; l < off; l++) p[l] = p[l] + p[l + off];
        acc = b == 0 ? p[0] : acc + p[0];
    }
    return acc;
}
static float wsum_f(const float *t, uint32_t R)
{
    float p[WS_LANES];
    for (int l = 0; l < WS_LANES; l++) p[l] = 0.0f;
    for (uint32_t r = 0; r < R; r++) p[r % WS_LANES] = p[r % WS_LANES] + t[r];
    for (int off = WS_LANES / 2; off >= 1; off >>= 1)
        for (int l = 0; l < off; l++) p[l] = p[l] + p[l + off];
    return p[0];
}

/* Deterministic standard normal from two uniforms (Box-Muller, the maths of
 * warp::squareToStdNormal, warp.cpp:131-137), evaluated with +,-,*,/,sqrt
 * only so that host and device agree bit for bit (libm / ocml cos and log
 * differ in the last ulp).  Returns the x component, as Preprocessor.cpp:619. */
static double det_log(double x)   /* x in (0, 1] */
{
    int e = 0;
    while (x < 0.70710678118654752440) { x = x * 2.0; e--; }
    /* log(x) = 2 atanh(z), z = (x-1)/(x+1), |z| <= 0.1716 */
    double z = (x - 1.0) / (x + 1.0), z2 = z * z, term = z, sum = 0.0;
    for (int k = 1; k <= 41; k += 2) { sum = sum + term / (double)k; term = term * z2; }
    return 2.0 * sum + (double)e * 0.69314718055994530942;
}
static double det_cos(double phi)  /* phi in [0, 2pi) */
{
    const double PI_ = 3.14159265358979323846;
    double x = phi;
    if (x > PI_) x = 2.0 * PI_ - x;          /* cos symmetric: x in [0, pi] */
    double sign = 1.0;
    if (x > 0.5 * PI_) { x = PI_ - x; sign = -1.0; }   /* x in [0, pi/2] */
    double x2 = x * x, term = 1.0, sum = 0.0;
    for (int k = 0; k < 14; k++) { sum = sum + term; term = -term * x2 / (double)((2 * k + 1) * (2 * k + 2)); }
    return sign * sum;
}
float alvrl_o_det_std_normal_x(float sx, float sy)
{
    double r = sqrt(-2.0 * det_log(1.0 - (double)sx));
    double phi = 2.0 * 3.14159265358979323846 * (double)sy;
    return (float)(det_cos(phi) * r);
}

/* --------------------------------------------------- heap (libstdc++) -- */
typedef struct { float uvar, ivar; uint32_t begin, end; } cnode;

static inline int cnode_less(const cnode *a, const cnode *b)
{
    /* ClusterNode::operator< (Preprocessor.cpp:292-293) */
    return a->uvar + a->ivar < b->uvar + b->ivar;
}

static void c_push_heap_(cnode *first, long hole, long top, cnode value)
{
    long parent = (hole - 1) / 2;
    while (hole > top && cnode_less(&first[parent], &value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}
static void c_adjust_heap(cnode *first, long hole, long len, cnode value)
{
    long top = hole, second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (cnode_less(&first[second], &first[second - 1])) second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    c_push_heap_(first, hole, top, value);
}

typedef struct { cnode *v; long n, cap; } cheap;
static void cheap_push(cheap *h, cnode x)
{
    if (h->n == h->cap) { h->cap = h->cap ? 2 * h->cap : 64; h->v = (cnode *)realloc(h->v, sizeof(cnode) * h->cap); }
    h->v[h->n++] = x;
    cnode val = h->v[h->n - 1];
    c_push_heap_(h->v, h->n - 1, 0, val);
}
static cnode cheap_pop(cheap *h)
{
    cnode top = h->v[0];
    if (h->n > 1) {
        long last = h->n - 1;
        cnode value = h->v[last];
        h->v[last] = h->v[0];
        c_adjust_heap(h->v, 0, last, value);
    }
    h->n--;
    return top;
}
static void cheap_copy(cheap *dst, const cheap *src)
{
    if (dst->cap < src->n) { dst->cap = src->n > 64 ? src->n : 64; dst->v = (cnode *)realloc(dst->v, sizeof(cnode) * dst->cap); }
    if (src->n) memcpy(dst->v, src->v, sizeof(cnode) * src->n);
    dst->n = src->n;
}

/* singleton list with push_front: stored appended, iterated in reverse */
typedef struct { uint32_t *v; long n, cap; } ulist;
static void ulist_push_front(ulist *l, uint32_t x)
{
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 64; l->v = (uint32_t *)realloc(l->v, sizeof(uint32_t) * l->cap); }
    l->v[l->n++] = x;
}
static void ulist_copy(ulist *dst, const ulist *src)
{
    if (dst->cap < src->n) { dst->cap = src->n > 64 ? src->n : 64; dst->v = (uint32_t *)realloc(dst->v, sizeof(uint32_t) * dst->cap); }
    if (src->n) memcpy(dst->v, src->v, sizeof(uint32_t) * src->n);
    dst->n = src->n;
}

/* ------------------------------------------------------ Clustering -- */
/* per-thread scratch of a split: row vectors (R + 1 entries each) */
typedef struct {
    double *sum, *Mv, *sumVars, *scr;
    float *fa, *fb, *fc, *fd;
} scratch_t;

static void scratch_alloc(scratch_t *S, uint32_t R)
{
    S->sum = (double *)calloc((size_t)R * 4 + 4, sizeof(double));
    S->Mv = S->sum + R + 1; S->sumVars = S->Mv + R + 1; S->scr = S->sumVars + R + 1;
    S->fa = (float *)calloc((size_t)R * 4 + 4, sizeof(float));
    S->fb = S->fa + R + 1; S->fc = S->fb + R + 1; S->fd = S->fc + R + 1;
}
static void scratch_free(scratch_t *S) { free(S->sum); free(S->fa); S->sum = NULL; S->fa = NULL; }

struct spec_pool;
typedef struct {
    mat_t M;
    const double *locw;
    uint32_t *vrls;        /* m_vrls */
    uint32_t nv;           /* size of m_vrls */
    float *colw;           /* m_columnWeights, indexed by vrl id */
    float tracingVar, unclIntVar, clUnderVar, clIntVar;
    float pixelUndersampling, depthCorrection;
    cheap pq; ulist singles;
    float sh_clUnderVar, sh_clIntVar;
    cheap sh_pq; ulist sh_singles;
    uint32_t seed, pass, stage;
    int err;
    scratch_t S;           /* the refining thread's scratch */
    int par;               /* threads for the inner loops of big splits on the refining thread */
    struct spec_pool *spec;   /* speculative split workers, or NULL (sequential) */
    uint16_t *gen;         /* diagnostic: split-tree depth of the cluster starting at [begin] */
    uint16_t cur_gen;
} clustering_t;

/* Diagnostic pop trace (test infrastructure): when set, every cluster the
 * refinement pops is recorded as (begin, end, depth in the split tree). */
static uint32_t *g_pop_trace;
static uint32_t g_pop_cap, g_pop_n;
void alvrl_o_set_pop_trace(uint32_t *buf, uint32_t cap) { g_pop_trace = buf; g_pop_cap = cap; g_pop_n = 0; }
uint32_t alvrl_o_pop_trace_n(void) { return g_pop_n; }

/* weightedSample, Preprocessor.cpp:1534-1580.  The running float sums of the
 * reference (weightSum += w, accum += w, in index order) are taken in one
 * fixed blocked order that a 64-lane wavefront evaluates directly -- the
 * reference's -funsafe-math-optimizations build (build/config-linux-gcc.py:7)
 * may reassociate them, so it has no canonical rounding here either:
 *   block b = indices [64b, 64b + 64) (missing ones weigh 0);
 *   within each row of 16: Hillis-Steele inclusive scan, y[l] += y[l - k]
 *     for k = 1, 2, 4, 8 (lanes with l % 16 >= k, simultaneous);
 *   row bases b0 = 0, b1 = t0, b2 = b1 + t1, b3 = b2 + t2 (t_r = row total);
 *   block prefix P[l] = b_row + y[l], block total = b3 + t3;
 *   block bases S_0 = 0, S_{b+1} = S_b + total_b; prefix(64b + l) = S_b + P[l].
 * weightSum = S_nb; the pick is the first index whose prefix >= alpha. */
static float ws_block(const float x[64], float P[64])
{
    float y[64], t[64];
    memcpy(y, x, sizeof(y));
    for (int k = 1; k <= 8; k <<= 1) {
        memcpy(t, y, sizeof(t));
        for (int l = 0; l < 64; l++)
            if (l % 16 >= k) y[l] = t[l] + t[l - k];
    }
    const float b1 = y[15], b2 = b1 + y[31], b3 = b2 + y[47];
    const float base[4] = { 0.0f, b1, b2, b3 };
    for (int l = 0; l < 64; l++) P[l] = base[l / 16] + y[l];
    return b3 + y[63];
}

/* excl: an index whose weight counts as 0 (split's second draw, which the
 * reference takes with the first pick's weight temporarily zeroed,
 * Preprocessor.cpp:597-602; ~0u = none) */
static void ws_load(const float *weights, const uint32_t *ind, size_t ind_base, size_t begin, size_t end,
                    size_t b, uint32_t excl, float x[64])
{
    for (int l = 0; l < 64; l++) {
        size_t i = begin + 64 * b + (size_t)l;
        size_t id = i < end ? (ind ? ind[i - ind_base] : i) : 0;
        x[l] = i < end && id != excl ? weights[id] : 0.0f;
    }
}

/* ind: the index array, ind[i - ind_base] for i in [begin, end) */
static size_t weighted_sample(const float *weights, smp_t *smp, float *prob, size_t begin,
                              size_t end, const uint32_t *ind, size_t ind_base, uint32_t excl, int *err)
{
    if (begin >= end) { *err = 1; return begin; }
    if (end == begin + 1) { if (prob) *prob = 1; return begin; }
    const size_t nb = (end - begin + 63) / 64;
    float x[64], P[64];
    float weightSum = 0.0f;
    for (size_t b = 0; b < nb; b++) {
        ws_load(weights, ind, ind_base, begin, end, b, excl, x);
        weightSum = weightSum + ws_block(x, P);
    }
    float probability;
    size_t idx;
    if (weightSum <= 0) {
        int tries = 0;
        do {
            idx = (size_t)((float)begin + smp_next(smp) * (float)(end - begin));
            if (++tries > 1000) { *err = 1; idx = begin; break; }   /* hang guard, as on the device */
        } while (idx >= end);
        probability = (float)(1.0 / (double)(end - begin));
    } else {
        float alpha = smp_next(smp) * weightSum;
        float S = 0.0f;
        idx = begin;
        int found = 0;
        for (size_t b = 0; b < nb && !found; b++) {
            ws_load(weights, ind, ind_base, begin, end, b, excl, x);
            const float tot = ws_block(x, P);
            for (int l = 0; l < 64 && begin + 64 * b + (size_t)l < end; l++)
                if (S + P[l] >= alpha) { idx = begin + 64 * b + (size_t)l; found = 1; break; }
            S = S + tot;
        }
        probability = weights[ind ? ind[idx - ind_base] : idx] / weightSum;
    }
    if (prob) *prob = probability;
    return idx;
}

/* calculateColumnWeigths, Preprocessor.cpp:985-1008 */
static int column_weights(const mat_t *M, const double *w, float *colw, double *tmp)
{
    for (uint32_t v = 0; v < M->nvrl; v++) {
        for (uint32_t r = 0; r < M->nrows; r++) {
            double mean = (double)m_mean(M, r, v);
            double var = (double)m_var(M, r, v);
            double x = mean * mean + var;
            tmp[r] = w[r] * x;
        }
        double ip = wsum_d(tmp, M->nrows);
        colw[v] = (float)sqrt(ip > 0.0 ? ip : 0.0);
        if (!isfinite(colw[v])) return 1;
    }
    float acc = 0.0f;
    for (uint32_t v = 0; v < M->nvrl; v++) acc += colw[v];
    float averageWeight = acc / M->nvrl;
    if (averageWeight == 0) averageWeight = 1.0;
    for (uint32_t v = 0; v < M->nvrl; v++) colw[v] += averageWeight * 1e-2f;
    return 0;
}

/* calculateUnclusteredVariance, Preprocessor.cpp:1022-1048 */
static int unclustered_variance(const mat_t *M, const double *w, const uint32_t *vb,
                                const uint32_t *ve, float *tracerVar, float *intVar)
{
    uint32_t R = M->nrows;
    double *mean = (double *)calloc(R, sizeof(double));
    double *M2 = (double *)calloc(R, sizeof(double));
    double *sv = (double *)calloc(R, sizeof(double));
    size_t n = 0;
    for (const uint32_t *it = vb; it != ve; ++it) {
        n++;
        double rn = 1.0 / (double)n;            /* -freciprocal-math form, see cluster_variance */
        for (uint32_t r = 0; r < R; r++) {
            sv[r] += (double)m_var(M, r, *it);
            double x = (double)m_mean(M, r, *it);
            double delta = x - mean[r];
            mean[r] += delta * rn;
            M2[r] += delta * (x - mean[r]);
        }
    }
    int rc = 0;
    if (n <= 1) rc = 1;
    for (uint32_t r = 0; r < R; r++) sv[r] = w[r] * sv[r];
    double ipv = wsum_d(sv, R);
    *intVar = (float)ipv;
    for (uint32_t r = 0; r < R; r++) M2[r] = w[r] * M2[r];
    double ipm = wsum_d(M2, R);
    *tracerVar = (float)(ipm - (double)*intVar);
    free(mean); free(M2); free(sv);
    return rc;
}

/* calculateClusterVariance, Preprocessor.cpp:1058-1120.  'vrls' is walked
 * forward (step=+1) or backward (step=-1) over n entries.  The row-vector
 * divisions by the loop-invariant scalars weight and weightSum (:1093,
 * :1100-1106) are taken in their -freciprocal-math form (the reference is
 * built with -funsafe-math-optimizations, build/config-linux-gcc.py:7):
 * one reciprocal per column, a multiply per row. */
static int cluster_variance(const clustering_t *C, const scratch_t *S, const uint32_t *first, long step,
                            uint32_t n_items, float *inc_u, float *inc_i, float *res_u, float *res_i)
{
    const mat_t *M = &C->M;
    uint32_t R = M->nrows;
    double *sum = S->sum, *Mv = S->Mv, *sumVars = S->sumVars;
    for (uint32_t r = 0; r < R; r++) { sum[r] = 0; Mv[r] = 0; sumVars[r] = 0; }
    double weightSum = 0;
    if (n_items == 0) return 1;
    for (uint32_t n = 0; n < n_items; n++) {
        uint32_t vrl = first[(long)n * step];
        double weight = (double)C->colw[vrl];
        if (!isfinite(weight) || weight <= 0) return 1;
        double newWeightSum = weightSum + weight;
        double a = (newWeightSum * newWeightSum) / (weightSum * weightSum);
        double rweight = 1.0 / weight;
        double bcoef = (rweight + 1.0 / weightSum);
        for (uint32_t r = 0; r < R; r++) {
            double x = (double)m_mean(M, r, vrl);
            double tmp = weight * sum[r] - weightSum * x;
            if (n > 0) Mv[r] = a * Mv[r] + bcoef * (tmp * tmp);
            sumVars[r] += (double)m_var(M, r, vrl) * rweight;
            sum[r] = sum[r] + x;
        }
        weightSum = newWeightSum;
        if (inc_u) {
            double rws = 1.0 / weightSum;
            double *t = S->scr;
            for (uint32_t r = 0; r < R; r++) t[r] = C->locw[r] * (sumVars[r] * weightSum);
            double ipi = wsum_blk(t, R);
            if (n == 0) {
                inc_u[n] = 0;
            } else {
                for (uint32_t r = 0; r < R; r++) t[r] = C->locw[r] * (Mv[r] * rws);
                inc_u[n] = (float)wsum_blk(t, R);
            }
            inc_i[n] = (float)ipi;
        }
    }
    /* with per-prefix outputs the totals are the last prefix's (same order) */
    double (*wsum)(const double *, uint32_t) = inc_u ? wsum_blk : wsum_d;
    double rws = 1.0 / weightSum;
    double *t = S->scr;
    for (uint32_t r = 0; r < R; r++) t[r] = C->locw[r] * (Mv[r] * rws);
    double ipu = wsum(t, R);
    for (uint32_t r = 0; r < R; r++) t[r] = C->locw[r] * (sumVars[r] * weightSum);
    double ipi = wsum(t, R);
    *res_u = (float)ipu;
    *res_i = (float)ipi;
    if (!isfinite(*res_u) || *res_u < 0) return 1;
    if (!isfinite(*res_i) || *res_i < 0) return 1;
    return 0;
}

/* Clustering::addCluster, Preprocessor.cpp:549-579 */
static void add_cluster(clustering_t *C, uint32_t begin, uint32_t end, float uvar, float ivar)
{
    if (end == begin) { C->err = 1; return; }
    if (C->gen) C->gen[begin] = (uint16_t)(C->cur_gen + 1);
    if (end == begin + 1) {
        ulist_push_front(&C->singles, C->vrls[begin]);
        if (uvar != 0) C->err = 1;
        C->clIntVar += ivar;
    } else {
        cnode cn = { uvar, ivar, begin, end };
        cheap_push(&C->pq, cn);
        C->clUnderVar += uvar;
        C->clIntVar += ivar;
    }
}

static cnode pop_multi(clustering_t *C)
{
    cnode cn = cheap_pop(&C->pq);
    C->cur_gen = C->gen ? C->gen[cn.begin] : 0;
    if (g_pop_trace && g_pop_n < g_pop_cap) {
        g_pop_trace[3 * g_pop_n] = cn.begin; g_pop_trace[3 * g_pop_n + 1] = cn.end;
        g_pop_trace[3 * g_pop_n + 2] = C->cur_gen; g_pop_n++;
    }
    C->clUnderVar -= cn.uvar;
    C->clIntVar -= cn.ivar;
    return cn;
}

static float norm2f(const float *v, uint32_t n, float *scr)
{
    for (uint32_t i = 0; i < n; i++) { float u = fabsf(v[i]); scr[i] = u * u; }
    return sqrtf(wsum_f(scr, n));
}

typedef struct { float p; uint32_t v; } projpair;
static int projpair_cmp(const void *a, const void *b)
{
    const projpair *x = (const projpair *)a, *y = (const projpair *)b;
    if (x->p < y->p) return -1;
    if (y->p < x->p) return 1;
    return x->v < y->v ? -1 : (x->v > y->v ? 1 : 0);
}

/* Inner loops of a big split on several threads (test-infrastructure speed-up
 * for the C5-sized checks, see the speculative splits below): the
 * projections of disjoint column chunks, and the forward and reverse variance
 * passes side by side.  Every value is computed by the same code in the same
 * order as sequentially. */
typedef struct {
    const mat_t *M;
    const float *direction;
    const uint32_t *v;
    projpair *proj;
    uint32_t j0, j1;
} proj_job;

static void project_range(const proj_job *x, float *c1, float *fd)
{
    const mat_t *M = x->M;
    const uint32_t R = M->nrows;
    for (uint32_t j = x->j0; j < x->j1; j++) {
        uint32_t vrl = x->v[j];
        for (uint32_t r = 0; r < R; r++) c1[r] = m_mean(M, r, vrl);
        float nc = norm2f(c1, R, fd);
        float projection;
        if (nc == 0) {
            projection = 0;
        } else {
            for (uint32_t r = 0; r < R; r++) fd[r] = x->direction[r] * (c1[r] / nc);
            projection = wsum_f(fd, R);
        }
        x->proj[j].p = projection;
        x->proj[j].v = vrl;
    }
}

static void *proj_thread(void *arg)
{
    const proj_job *x = (const proj_job *)arg;
    float *buf = (float *)malloc(sizeof(float) * 2 * ((size_t)x->M->nrows + 1));
    project_range(x, buf, buf + x->M->nrows + 1);
    free(buf);
    return NULL;
}

typedef struct {
    const clustering_t *C;
    scratch_t S;
    const uint32_t *first;
    long step;
    uint32_t n;
    float *inc_u, *inc_i;
    float ru, ri;
    int rc;
} var_job;

static int cluster_variance(const clustering_t *C, const scratch_t *S, const uint32_t *first, long step,
                            uint32_t n_items, float *inc_u, float *inc_i, float *res_u, float *res_i);
static void *var_thread(void *arg)
{
    var_job *x = (var_job *)arg;
    x->rc = cluster_variance(x->C, &x->S, x->first, x->step, x->n, x->inc_u, x->inc_i, &x->ru, &x->ri);
    return NULL;
}

/* The outcome of one split: the two children (begin, split point, end) with
 * their variances.  ok = 0: no split point (the caller's error). */
typedef struct {
    int ok, err;
    uint32_t split;
    float u1, i1, u2, i2;
} split_res;

/* Clustering::split, Preprocessor.cpp:590-684, without its side effects on
 * the clustering state: v = the cluster's ids (positions [begin, end), v[0]
 * is position begin) are sorted in place; the children's variances come back
 * in *out.  Reads only C's immutable inputs (matrix, column weights, locality
 * weights, stream keys), so speculative splits run it on worker threads. */
static void split_compute(const clustering_t *C, const scratch_t *S, uint32_t begin, uint32_t end,
                          uint32_t *v, split_res *out)
{
    memset(out, 0, sizeof(*out));
    uint32_t clusterSize = end - begin;
    if (clusterSize < 2) return;
    const mat_t *M = &C->M;
    uint32_t R = M->nrows;
    int err = 0;
    smp_t smp;
    smp_init(&smp, C->seed, C->pass, ALVRL_O_DOM_CLUSTER, begin, end, C->stage);

    /* the second centre is drawn with the first one's weight zeroed (:597-602) */
    uint32_t vrl1 = v[weighted_sample(C->colw, &smp, NULL, begin, end, v, begin, ~0u, &err) - begin];
    uint32_t vrl2 = v[weighted_sample(C->colw, &smp, NULL, begin, end, v, begin, vrl1, &err) - begin];

    float *direction = S->fa, *c1 = S->fb, *c2 = S->fc, *fd = S->fd;
    for (uint32_t r = 0; r < R; r++) { c1[r] = m_mean(M, r, vrl1); c2[r] = m_mean(M, r, vrl2); }
    float vrl1len = norm2f(c1, R, fd);
    float vrl2len = norm2f(c2, R, fd);
    for (uint32_t r = 0; r < R; r++) c2[r] = c2[r] - c1[r];   /* diff */
    float diffLen = norm2f(c2, R, fd);
    if (vrl1len != 0 && vrl2len != 0 && diffLen != 0) {
        for (uint32_t r = 0; r < R; r++) direction[r] = c2[r] / diffLen;
    } else {
        float nd;
        int guard = 0;
        do {
            for (uint32_t r = 0; r < R; r++) {
                /* warp::squareToStdNormal(next2D()).x (warp.cpp:131-137) */
                float sx = smp_next(&smp), sy = smp_next(&smp);
                direction[r] = alvrl_o_det_std_normal_x(sx, sy);
            }
            nd = norm2f(direction, R, fd);
            if (nd == 0 && ++guard > 64) { err = 1; nd = 1.0f; }   /* hang guard, as on the device */
        } while (nd == 0);
        for (uint32_t r = 0; r < R; r++) direction[r] = direction[r] / nd;
    }

    projpair *proj = (projpair *)malloc(sizeof(projpair) * clusterSize);
    const int par = clusterSize >= (1u << 14) ? C->par : 0;
    if (par > 1) {
        pthread_t th[64];
        int spawned[64];
        proj_job pj[64];
        const int nt = par < 64 ? par : 64;
        const uint32_t chunk = (clusterSize + (uint32_t)nt - 1) / (uint32_t)nt;
        for (int t = 0; t < nt; t++) {
            uint32_t j0 = (uint32_t)t * chunk, j1 = j0 + chunk;
            if (j0 > clusterSize) j0 = clusterSize;
            if (j1 > clusterSize) j1 = clusterSize;
            proj_job x = { M, direction, v, proj, j0, j1 };
            pj[t] = x;
            spawned[t] = t > 0 && pthread_create(&th[t], NULL, proj_thread, &pj[t]) == 0;
        }
        proj_thread(&pj[0]);
        for (int t = 1; t < nt; t++) {
            if (spawned[t]) pthread_join(th[t], NULL);
            else proj_thread(&pj[t]);
        }
    } else {
        proj_job x = { M, direction, v, proj, 0, clusterSize };
        project_range(&x, c1, fd);
    }
    qsort(proj, clusterSize, sizeof(projpair), projpair_cmp);
    for (uint32_t j = 0; j < clusterSize; j++) v[j] = proj[j].v;
    free(proj);

    float *fsu = (float *)malloc(sizeof(float) * clusterSize * 4);
    float *fsi = fsu + clusterSize, *feu = fsu + 2 * clusterSize, *fei = fsu + 3 * clusterSize;
    float v1u, v1i, v2u, v2i;
    if (par > 1) {   /* the two directions on two threads, each with its own scratch */
        var_job vj = { C, { 0 }, v + clusterSize - 1, -1, clusterSize, feu, fei, 0, 0, 0 };
        scratch_alloc(&vj.S, R);
        pthread_t th;
        const int spawned = pthread_create(&th, NULL, var_thread, &vj) == 0;
        if (cluster_variance(C, S, v, 1, clusterSize, fsu, fsi, &v1u, &v1i)) err = 1;
        if (spawned) pthread_join(th, NULL);
        else var_thread(&vj);
        v2u = vj.ru; v2i = vj.ri;
        if (vj.rc) err = 1;
        scratch_free(&vj.S);
    } else {
        if (cluster_variance(C, S, v, 1, clusterSize, fsu, fsi, &v1u, &v1i)) err = 1;
        if (cluster_variance(C, S, v + clusterSize - 1, -1, clusterSize, feu, fei, &v2u, &v2i)) err = 1;
    }
    float bestVariance = INFINITY;
    uint32_t bestIndex = UINT32_T_MAX;
    for (uint32_t i = 1; i < clusterSize; ++i) {
        float thisVar = fsu[i - 1] + fsi[i - 1] + feu[clusterSize - 1 - i] + fei[clusterSize - 1 - i];
        if (thisVar < bestVariance) { bestVariance = thisVar; bestIndex = i; }
    }
    out->err = err;
    if (bestIndex != UINT32_T_MAX) {
        out->ok = 1;
        out->split = begin + bestIndex;
        out->u1 = fsu[bestIndex - 1]; out->i1 = fsi[bestIndex - 1];
        out->u2 = feu[clusterSize - 1 - bestIndex]; out->i2 = fei[clusterSize - 1 - bestIndex];
    } else {
        out->err = 1;
    }
    free(fsu);
}

/* the split's effect on the clustering (:680-683): the two children */
static int split_apply(clustering_t *C, uint32_t begin, uint32_t end, const split_res *r)
{
    if (r->err) C->err = 1;
    if (!r->ok) return 0;
    add_cluster(C, begin, r->split, r->u1, r->i1);
    add_cluster(C, r->split, end, r->u2, r->i2);
    return 1;
}

static int spec_take(clustering_t *C, uint32_t begin, uint32_t end, split_res *r);
static void spec_offer(clustering_t *C);

/* Clustering::split (:590-684) of the popped cluster [begin, end): its
 * speculative result when a worker has it (identical: the split depends only
 * on the cluster's ids and its stream), else computed here. */
static int split(clustering_t *C, uint32_t begin, uint32_t end)
{
    split_res r;
    if (!(C->spec && spec_take(C, begin, end, &r)))
        split_compute(C, &C->S, begin, end, C->vrls + begin, &r);
    int ok = split_apply(C, begin, end, &r);
    if (C->spec) spec_offer(C);
    return ok;
}

static uint32_t n_clusters(const clustering_t *C) { return (uint32_t)(C->singles.n + C->pq.n); }

static float unclustered_var(const clustering_t *C) { return C->tracingVar + C->unclIntVar; }
static float clustered_var(const clustering_t *C) { return C->tracingVar + C->clUnderVar + C->clIntVar; }
static float convergence_constant(clustering_t *C)
{
    float c = ((float)C->M.nvrl * C->pixelUndersampling + (float)n_clusters(C)) * clustered_var(C);
    if (!isfinite(c) || c <= 0) C->err = 1;
    return c;
}
static float lower_bound(clustering_t *C)
{
    float c = ((float)C->M.nvrl * C->pixelUndersampling + (float)n_clusters(C)) * unclustered_var(C);
    if (!isfinite(c) || c <= 0) C->err = 1;
    return c;
}

static void snapshot(clustering_t *C)
{
    C->sh_clUnderVar = C->clUnderVar; C->sh_clIntVar = C->clIntVar;
    cheap_copy(&C->sh_pq, &C->pq); ulist_copy(&C->sh_singles, &C->singles);
}
static void restore(clustering_t *C)
{
    C->clUnderVar = C->sh_clUnderVar; C->clIntVar = C->sh_clIntVar;
    cheap_copy(&C->pq, &C->sh_pq); ulist_copy(&C->singles, &C->sh_singles);
}

/* ------------------------------------------------ speculative splits -- */
/* Test-infrastructure speed-up, not part of the restatement: a split's result
 * depends only on its cluster's ids and its stream (keyed by the cluster's
 * range), and live clusters are disjoint ranges of vrls, so worker threads
 * may split the clusters near the top of the heap ahead of the sequential
 * loop, each on a private copy of the range.  The loop commits a finished
 * result when it pops that cluster and computes anything else itself, so the
 * outcome is the sequential one bit for bit (the same idea as the device's
 * team mode, refine.hip).  Used while no restore() can intervene: it stops
 * before refineAdaptively's restore, and is off for small jobs.
 *   ALVRL_ORACLE_THREADS   workers (default min(16, online CPUs), 0 = off)
 *   ALVRL_ORACLE_SPEC_MIN  job size (rows x VRLs) from which it is used
 *                          (default 2^24; tests set 0 to exercise it) */
typedef struct {
    uint32_t begin, end;
    int state;                 /* 0 queued, 1 running, 2 done */
    uint32_t *buf;             /* the sorted ids, when done */
    split_res res;
} spec_entry;

struct spec_pool {
    pthread_mutex_t mu;
    pthread_cond_t cv_work, cv_done;
    pthread_t *th;
    int nth, stop;
    const clustering_t *C;
    spec_entry *e;
    long n, cap;
    uint64_t task_min;         /* rows x cluster size below which a split is not offered */
    long width;                /* heap entries examined per offer */
};

static void *spec_worker(void *arg)
{
    struct spec_pool *P = (struct spec_pool *)arg;
    const clustering_t *C = P->C;
    scratch_t S;
    scratch_alloc(&S, C->M.nrows);
    pthread_mutex_lock(&P->mu);
    while (!P->stop) {
        long k = 0;
        while (k < P->n && P->e[k].state != 0) k++;
        if (k == P->n) { pthread_cond_wait(&P->cv_work, &P->mu); continue; }
        spec_entry *x = &P->e[k];
        x->state = 1;
        const uint32_t b = x->begin, e = x->end;
        pthread_mutex_unlock(&P->mu);
        uint32_t *buf = (uint32_t *)malloc(sizeof(uint32_t) * (e - b));
        memcpy(buf, C->vrls + b, sizeof(uint32_t) * (e - b));
        split_res r;
        split_compute(C, &S, b, e, buf, &r);
        pthread_mutex_lock(&P->mu);
        for (k = 0; k < P->n; k++)      /* entries move when others are removed */
            if (P->e[k].begin == b && P->e[k].end == e) break;
        P->e[k].buf = buf;
        P->e[k].res = r;
        P->e[k].state = 2;
        pthread_cond_broadcast(&P->cv_done);
    }
    pthread_mutex_unlock(&P->mu);
    scratch_free(&S);
    return NULL;
}

static void spec_remove(struct spec_pool *P, long k)
{
    P->e[k] = P->e[P->n - 1];
    P->n--;
}

static void spec_start(clustering_t *C)
{
    const char *t = getenv("ALVRL_ORACLE_THREADS");
    const char *m = getenv("ALVRL_ORACLE_SPEC_MIN");
    long nth = t ? atol(t) : sysconf(_SC_NPROCESSORS_ONLN);
    if (!t && nth > 16) nth = 16;
    const uint64_t job_min = m ? (uint64_t)atoll(m) : (1ull << 24);
    if (nth < 1 || (uint64_t)C->M.nrows * C->nv < job_min) return;
    struct spec_pool *P = (struct spec_pool *)calloc(1, sizeof(*P));
    pthread_mutex_init(&P->mu, NULL);
    pthread_cond_init(&P->cv_work, NULL);
    pthread_cond_init(&P->cv_done, NULL);
    P->C = C;
    P->task_min = m ? 0 : (1u << 16);
    P->width = 2 * nth + 8;
    P->th = (pthread_t *)calloc((size_t)nth, sizeof(pthread_t));
    for (long i = 0; i < nth; i++)
        if (pthread_create(&P->th[P->nth], NULL, spec_worker, P) == 0) P->nth++;
    C->spec = P;
    C->par = P->nth;
}

/* join the workers and drop every pending result */
static void spec_stop(clustering_t *C)
{
    struct spec_pool *P = C->spec;
    if (!P) return;
    pthread_mutex_lock(&P->mu);
    P->stop = 1;
    pthread_cond_broadcast(&P->cv_work);
    pthread_mutex_unlock(&P->mu);
    for (int i = 0; i < P->nth; i++) pthread_join(P->th[i], NULL);
    for (long k = 0; k < P->n; k++) free(P->e[k].buf);
    free(P->e); free(P->th);
    pthread_mutex_destroy(&P->mu);
    pthread_cond_destroy(&P->cv_work);
    pthread_cond_destroy(&P->cv_done);
    free(P);
    C->spec = NULL;
    C->par = 0;
}

/* the popped cluster [begin, end): 1 = a worker's result, committed here */
static int spec_take(clustering_t *C, uint32_t begin, uint32_t end, split_res *r)
{
    struct spec_pool *P = C->spec;
    pthread_mutex_lock(&P->mu);
    for (;;) {
        long k = 0;
        while (k < P->n && !(P->e[k].begin == begin && P->e[k].end == end)) k++;
        if (k == P->n) { pthread_mutex_unlock(&P->mu); return 0; }
        if (P->e[k].state == 0) { spec_remove(P, k); pthread_mutex_unlock(&P->mu); return 0; }
        if (P->e[k].state == 1) { pthread_cond_wait(&P->cv_done, &P->mu); continue; }
        memcpy(C->vrls + begin, P->e[k].buf, sizeof(uint32_t) * (end - begin));
        *r = P->e[k].res;
        free(P->e[k].buf);
        spec_remove(P, k);
        pthread_mutex_unlock(&P->mu);
        return 1;
    }
}

/* queue the multi-clusters near the top of the heap not queued yet */
static void spec_offer(clustering_t *C)
{
    struct spec_pool *P = C->spec;
    const uint64_t R = C->M.nrows;
    int added = 0;
    pthread_mutex_lock(&P->mu);
    for (long i = 0; i < C->pq.n && i < P->width; i++) {
        const cnode *cn = &C->pq.v[i];
        if (cn->end - cn->begin < 2 || (uint64_t)(cn->end - cn->begin) * R < P->task_min) continue;
        long k = 0;
        while (k < P->n && !(P->e[k].begin == cn->begin && P->e[k].end == cn->end)) k++;
        if (k < P->n) continue;
        if (P->n == P->cap) {
            P->cap = P->cap ? 2 * P->cap : 64;
            P->e = (spec_entry *)realloc(P->e, sizeof(spec_entry) * P->cap);
        }
        spec_entry x = { cn->begin, cn->end, 0, NULL, { 0, 0, 0, 0, 0, 0, 0 } };
        P->e[P->n++] = x;
        added = 1;
    }
    if (added) pthread_cond_broadcast(&P->cv_work);
    pthread_mutex_unlock(&P->mu);
}

/* Clustering ctor, Preprocessor.cpp:301-341 */
static int clustering_init(clustering_t *C, const mat_t *M, const double *locw,
                           const uint32_t *init_vrls, const uint32_t *init_off, uint32_t ninit,
                           float pixelUndersampling, float depthCorrection,
                           uint32_t seed, uint32_t pass, uint32_t stage)
{
    memset(C, 0, sizeof(*C));
    C->M = *M; C->locw = locw;
    C->pixelUndersampling = pixelUndersampling; C->depthCorrection = depthCorrection;
    C->seed = seed; C->pass = pass; C->stage = stage;
    double n1 = 0.0;
    for (uint32_t r = 0; r < M->nrows; r++) n1 += fabs(locw[r]);
    if (fabs((float)n1 - 1) > 1e-3) return 1;
    if (pixelUndersampling <= 0 || pixelUndersampling > 1) return 1;
    uint32_t R = M->nrows;
    scratch_alloc(&C->S, R);
    C->colw = (float *)malloc(sizeof(float) * (M->nvrl ? M->nvrl : 1));
    if (column_weights(M, locw, C->colw, C->S.sum)) return 1;
    C->nv = init_off[ninit];
    C->vrls = (uint32_t *)malloc(sizeof(uint32_t) * (C->nv ? C->nv : 1));
    memcpy(C->vrls, init_vrls, sizeof(uint32_t) * C->nv);
    if (g_pop_trace) C->gen = (uint16_t *)calloc(C->nv ? C->nv : 1, sizeof(uint16_t));
    C->cur_gen = (uint16_t)-1;
    for (uint32_t i = 0; i < ninit; i++) {
        uint32_t b = init_off[i], e = init_off[i + 1];
        float u = 0, iv = 0;
        if (b == e) { C->err = 1; continue; }
        if (cluster_variance(C, &C->S, C->vrls + b, 1, e - b, NULL, NULL, &u, &iv)) C->err = 1;
        add_cluster(C, b, e, u, iv);
    }
    if (unclustered_variance(M, locw, C->vrls, C->vrls + C->nv, &C->tracingVar, &C->unclIntVar))
        C->err = 1;
    return C->err;
}

static void clustering_free(clustering_t *C)
{
    scratch_free(&C->S); free(C->colw); free(C->vrls); free(C->gen);
    free(C->pq.v); free(C->singles.v); free(C->sh_pq.v); free(C->sh_singles.v);
}

/* refineFixedDepth, Preprocessor.cpp:387-399 */
static int refine_fixed(clustering_t *C, float undersampling)
{
    uint32_t target = (uint32_t)(0.5 + (double)((float)C->M.nvrl / undersampling));
    if (n_clusters(C) >= target || C->pq.n <= 0) return 1;
    while (n_clusters(C) < target && C->pq.n > 0) {
        cnode cn = pop_multi(C);
        if (!split(C, cn.begin, cn.end)) C->err = 1;
        if (C->err) return 0;
    }
    return 1;
}

/* refineAdaptively, Preprocessor.cpp:402-489 */
static int refine_adaptive(clustering_t *C)
{
    float dc = C->depthCorrection;
    if (C->pq.n <= 0) return 1;
    if (unclustered_var(C) == 0) return 0;
    float best = convergence_constant(C);
    int nsplit = 0, bestN = 0;
    snapshot(C);
    while (C->pq.n > 0) {
        cnode cn = pop_multi(C);
        if (!split(C, cn.begin, cn.end)) C->err = 1;
        nsplit++;
        float curr = convergence_constant(C);
        if (curr < best) {
            if (dc == 1) snapshot(C);
            best = curr;
            bestN = nsplit;
        }
        if (lower_bound(C) >= best) break;
        if (C->err) return 0;
    }
    spec_stop(C);      /* before restore(): the replay below is sequential */
    restore(C);
    if (dc != 1) {
        /* the replay pops the restored clusters; their ids are what the
         * discarded splits left, so only results computed from here on count */
        spec_start(C);
        if (C->spec) spec_offer(C);
        int corrected = (int)(0.5 + dc * bestN);
        for (int i = 0; i < corrected; i++) {
            if (C->pq.n == 0) break;
            cnode cn = pop_multi(C);
            if (!split(C, cn.begin, cn.end)) C->err = 1;
        }
    }
    return C->err ? 0 : 1;
}

static int refine(clustering_t *C, float undersampling)
{
    spec_start(C);
    if (C->spec) spec_offer(C);
    int ok = undersampling <= 0 ? refine_adaptive(C) : refine_fixed(C, undersampling);
    spec_stop(C);
    return ok;
}

/* Clustering::sampleRepresentatives, Preprocessor.cpp:354-378 */
static uint32_t sample_reps(clustering_t *C, uint32_t stage, uint32_t *reps, float *w)
{
    uint32_t i = 0;
    for (long k = C->singles.n - 1; k >= 0; k--) { reps[i] = C->singles.v[k]; w[i] = 1; i++; }
    for (long k = 0; k < C->pq.n; k++) {
        const cnode *cn = &C->pq.v[k];
        smp_t smp;
        smp_init(&smp, C->seed, C->pass, ALVRL_O_DOM_CLUSTER, cn->begin, cn->end, stage);
        float prob = 1.0f;
        size_t j = weighted_sample(C->colw, &smp, &prob, cn->begin, cn->end, C->vrls, 0, ~0u, &C->err);
        reps[i] = C->vrls[j];
        w[i] = 1.0f / prob;
        i++;
    }
    return i;
}

/* Clustering::getVrlsPerCluster, Preprocessor.cpp:526-543: singletons in
 * std::list order (push_front, so newest first), then the heap's clusters in
 * its underlying vector order.  out_vrls gets C->nv ids, out_off the
 * (clusters + 1) offsets; returns the cluster count. */
static uint32_t vrls_per_cluster(const clustering_t *C, uint32_t *out_vrls, uint32_t *out_off)
{
    uint32_t c = 0, at = 0;
    out_off[0] = 0;
    for (long k = C->singles.n - 1; k >= 0; k--) { out_vrls[at++] = C->singles.v[k]; out_off[++c] = at; }
    for (long k = 0; k < C->pq.n; k++) {
        const cnode *cn = &C->pq.v[k];
        for (uint32_t j = cn->begin; j < cn->end; j++) out_vrls[at++] = C->vrls[j];
        out_off[++c] = at;
    }
    return c;
}

int alvrl_o_cluster_members(const float *Rt, uint64_t ld, const uint32_t *rows, uint32_t nrows,
                            const double *locw, uint32_t nvrl,
                            const uint32_t *init_vrls, const uint32_t *init_off, uint32_t ninit,
                            float pixelUndersampling, float undersampling, uint32_t seed, uint32_t pass,
                            uint32_t stage_refine, uint32_t *out_vrls, uint32_t *out_off,
                            uint32_t *nclusters, int *refined)
{
    mat_t M = { Rt, ld, rows, nrows, nvrl };
    clustering_t C;
    int rc = clustering_init(&C, &M, locw, init_vrls, init_off, ninit, pixelUndersampling, 1.0f,
                             seed, pass, stage_refine);
    if (rc) { clustering_free(&C); return -1; }
    int ok = refine(&C, undersampling);
    if (refined) *refined = ok;
    *nclusters = vrls_per_cluster(&C, out_vrls, out_off);
    int err = C.err;
    clustering_free(&C);
    return err ? -2 : 0;
}

int alvrl_o_cluster_refine(const float *Rt, uint64_t ld, const uint32_t *rows, uint32_t nrows,
                           const double *locw, uint32_t nvrl,
                           const uint32_t *init_vrls, const uint32_t *init_off, uint32_t ninit,
                           float pixelUndersampling, float undersampling, float depthCorrection,
                           int do_refine, uint32_t seed, uint32_t pass, uint32_t stage_refine,
                           uint32_t stage_sample, uint32_t *reps, float *weights, uint32_t *nreps,
                           int *refined)
{
    mat_t M = { Rt, ld, rows, nrows, nvrl };
    clustering_t C;
    int rc = clustering_init(&C, &M, locw, init_vrls, init_off, ninit, pixelUndersampling,
                             depthCorrection, seed, pass, stage_refine);
    if (rc) { clustering_free(&C); return -1; }
    int ok = 1;
    if (do_refine) ok = refine(&C, undersampling);
    if (refined) *refined = ok;
    if (ok) *nreps = sample_reps(&C, stage_sample, reps, weights);
    else *nreps = 0;
    int err = C.err;
    clustering_free(&C);
    return err ? -2 : 0;
}

/* ===================================================================== */
/*  Preprocessor: slicing + representatives + localities + clusters         */
/* ===================================================================== */
typedef struct { float x, y, z; } p3;

typedef struct {
    uint32_t minInd, maxInd;
    float distance;
    unsigned char dim;
    float split;
    p3 posC, dirC;
} snode;

static inline int snode_less(const snode *a, const snode *b) { return a->distance < b->distance; }

static void s_push_heap_(snode *first, long hole, long top, snode value)
{
    long parent = (hole - 1) / 2;
    while (hole > top && snode_less(&first[parent], &value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}
static void s_adjust_heap(snode *first, long hole, long len, snode value)
{
    long top = hole, second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (snode_less(&first[second], &first[second - 1])) second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    s_push_heap_(first, hole, top, value);
}

static float slice_distance(p3 p1, p3 d1, p3 p2, p3 d2)
{
    float dx = p1.x - p2.x, dy = p1.y - p2.y, dz = p1.z - p2.z;
    float ex = d1.x - d2.x, ey = d1.y - d2.y, ez = d1.z - d2.z;
    return sqrtf((dx * dx + dy * dy + dz * dz) + (ex * ex + ey * ey + ez * ez));
}

/* findSplitPoint, Preprocessor.cpp:1451-1487 */
static void find_split_point(p3 mx, p3 mn, unsigned char *dim, float *split, float *extent)
{
    float dx = mx.x - mn.x, dy = mx.y - mn.y, dz = mx.z - mn.z;
    if (dx == 0 && dy == 0 && dz == 0) { *extent = 0; *dim = 0; *split = NAN; return; }
    if (dx > dy) {
        if (dx > dz) { *dim = 0; *split = (float)(mn.x + 0.5 * dx); *extent = dx; }
        else { *dim = 2; *split = (float)(mn.z + 0.5 * dz); *extent = dz; }
    } else {
        if (dy > dz) { *dim = 1; *split = (float)(mn.y + 0.5 * dy); *extent = dy; }
        else { *dim = 2; *split = (float)(mn.z + 0.5 * dz); *extent = dz; }
    }
}

static int make_snode(snode *sn, uint32_t minI, uint32_t maxI, const p3 *pos, const p3 *dir,
                      const uint32_t *idx)
{
    sn->minInd = minI; sn->maxInd = maxI;
    if (minI >= maxI) return 1;
    if (minI + 1 == maxI) {
        sn->distance = 0; sn->dim = 0; sn->split = NAN;
        sn->posC.x = sn->posC.y = sn->posC.z = NAN;
        sn->dirC = sn->posC;
        return 0;
    }
    p3 mxp = { -INFINITY, -INFINITY, -INFINITY }, mnp = { INFINITY, INFINITY, INFINITY };
    p3 mxd = mxp, mnd = mnp;
    for (uint32_t i = minI; i < maxI; i++) {
        p3 p = pos[idx[i]], d = dir[idx[i]];
        if (p.x < mnp.x) { mnp.x = p.x; }
        if (p.y < mnp.y) { mnp.y = p.y; }
        if (p.z < mnp.z) { mnp.z = p.z; }
        if (p.x > mxp.x) { mxp.x = p.x; }
        if (p.y > mxp.y) { mxp.y = p.y; }
        if (p.z > mxp.z) { mxp.z = p.z; }
        if (d.x < mnd.x) { mnd.x = d.x; }
        if (d.y < mnd.y) { mnd.y = d.y; }
        if (d.z < mnd.z) { mnd.z = d.z; }
        if (d.x > mxd.x) { mxd.x = d.x; }
        if (d.y > mxd.y) { mxd.y = d.y; }
        if (d.z > mxd.z) { mxd.z = d.z; }
    }
    sn->distance = slice_distance(mnp, mnd, mxp, mxd);
    unsigned char dp, dd;
    float sp, sd, ep, ed;
    find_split_point(mxp, mnp, &dp, &sp, &ep);
    find_split_point(mxd, mnd, &dd, &sd, &ed);
    if (ep == 0 && ed == 0) return 1;
    if (ep > ed) { sn->dim = dp; sn->split = sp; }
    else { sn->dim = (unsigned char)(3 + dd); sn->split = sd; }
    sn->posC.x = mnp.x + 0.5f * (mxp.x - mnp.x);
    sn->posC.y = mnp.y + 0.5f * (mxp.y - mnp.y);
    sn->posC.z = mnp.z + 0.5f * (mxp.z - mnp.z);
    sn->dirC.x = mnd.x + 0.5f * (mxd.x - mnd.x);
    sn->dirC.y = mnd.y + 0.5f * (mxd.y - mnd.y);
    sn->dirC.z = mnd.z + 0.5f * (mxd.z - mnd.z);
    return 0;
}

static inline int is_larger(p3 p, p3 d, int dim, float split)
{
    switch (dim) {
    case 0: return p.x > split;
    case 1: return p.y > split;
    case 2: return p.z > split;
    case 3: return d.x > split;
    case 4: return d.y > split;
    default: return d.z > split;
    }
}

struct alvrl_o_prep {
    alvrl_o_prep_params prm;
    int W, H;
    uint32_t nslices;
    /* slice s: gather points idx[slice_lo[s] .. slice_hi[s]) (pixel ids, column-major) */
    uint32_t *slice_lo, *slice_hi, *idx;
    p3 *posC, *dirC;
    uint32_t *reps_off, *reps_pix;   /* representative pixel ids (column-major id) */
    float *slice_under;
    float global_under;
    /* localities: per slice list of (slice, distance) sorted like std::set<pair> */
    uint32_t *loc_off, *loc_slice;
    float *loc_dist;
};

alvrl_o_prep *alvrl_o_prep_create(const alvrl_o_prep_params *p)
{
    alvrl_o_prep *P = (alvrl_o_prep *)calloc(1, sizeof(alvrl_o_prep));
    P->prm = *p;
    P->global_under = -1;
    return P;
}

void alvrl_o_prep_destroy(alvrl_o_prep *P)
{
    if (!P) return;
    free(P->slice_lo); free(P->slice_hi); free(P->idx); free(P->posC); free(P->dirC);
    free(P->reps_off); free(P->reps_pix); free(P->slice_under);
    free(P->loc_off); free(P->loc_slice); free(P->loc_dist);
    free(P);
}

/* buildSlices + getSlices + getSlicesPQ, Preprocessor.cpp:1130-1418.
 * pixel_to_slice has W*H entries indexed y + H*x (vrlIntegrator.cpp:560). */
int alvrl_o_prep_build_slices(alvrl_o_prep *P, const alvrl_o_scene *s, uint32_t *pixel_to_slice)
{
    int W = s->width, H = s->height;
    uint32_t n = (uint32_t)W * (uint32_t)H;
    P->W = W; P->H = H;
    p3 *pos = (p3 *)malloc(sizeof(p3) * n), *dir = (p3 *)malloc(sizeof(p3) * n);
    float bd[3] = { s->box_max[0] - s->box_min[0], s->box_max[1] - s->box_min[1],
                    s->box_max[2] - s->box_min[2] };
    float diag = sqrtf(bd[0] * bd[0] + bd[1] * bd[1] + bd[2] * bd[2]);
    float directionScale = diag / 8 * P->prm.slice_curvature_factor;
    int ngood = 0;
    for (int i = 0; i < W; i++) {
        for (int j = 0; j < H; j++) {
            float rec[ALVRL_O_REC_WORDS];
            alvrl_o_make_slice_record(s, i, j, rec);   /* through null surfaces (:1157-1169) */
            uint32_t flags;
            memcpy(&flags, &rec[15], 4);
            uint32_t k = (uint32_t)i * H + j;
            if (flags & ALVRL_O_FLAG_HIT) {
                pos[k].x = rec[6]; pos[k].y = rec[7]; pos[k].z = rec[8];
                dir[k].x = directionScale * rec[9];
                dir[k].y = directionScale * rec[10];
                dir[k].z = directionScale * rec[11];
                ngood++;
            } else {
                pos[k].x = pos[k].y = pos[k].z = NAN;
                dir[k] = pos[k];
            }
        }
    }
    uint32_t *idx = (uint32_t *)malloc(sizeof(uint32_t) * n);
    for (uint32_t i = 0; i < n; i++) { idx[i] = i; pixel_to_slice[i] = UINT32_T_MAX; }
#define FINITE3(q) (isfinite((q).x) && isfinite((q).y) && isfinite((q).z))
    uint32_t first = 0;
    while (first < n && !FINITE3(pos[first])) first++;
    for (uint32_t i = first + 1; i < n; i++) {
        if (!FINITE3(pos[i])) { idx[i] = idx[first]; idx[first] = i; first++; }
    }
    /* getSlicesPQ */
    long cap = 2 * (long)P->prm.target_num_slices + 8, hn = 0;
    snode *heap = (snode *)malloc(sizeof(snode) * cap);
    int rc = 0;
    if (first < n) {
        snode sn;
        rc |= make_snode(&sn, first, n, pos, dir, idx);
        heap[hn++] = sn; s_push_heap_(heap, hn - 1, 0, sn);
        while (hn < (long)P->prm.target_num_slices && heap[0].distance > 0 && !rc) {
            snode top = heap[0];
            if (hn > 1) { snode val = heap[hn - 1]; heap[hn - 1] = heap[0]; s_adjust_heap(heap, 0, hn - 1, val); }
            hn--;
            size_t lo = top.minInd, hi = top.maxInd - 1;
            size_t i = lo - 1, j = hi + 1;
            while (1) {
                while (1) { i++; if (is_larger(pos[idx[i]], dir[idx[i]], top.dim, top.split) || i == hi) break; }
                while (1) { j--; if (!is_larger(pos[idx[j]], dir[idx[j]], top.dim, top.split) || j == lo) break; }
                if (i >= j) break;
                uint32_t t = idx[i]; idx[i] = idx[j]; idx[j] = t;
            }
            snode a, b;
            rc |= make_snode(&a, top.minInd, (uint32_t)(j + 1), pos, dir, idx);
            rc |= make_snode(&b, (uint32_t)(j + 1), top.maxInd, pos, dir, idx);
            if (hn + 2 > cap) { cap *= 2; heap = (snode *)realloc(heap, sizeof(snode) * cap); }
            heap[hn++] = a; s_push_heap_(heap, hn - 1, 0, a);
            heap[hn++] = b; s_push_heap_(heap, hn - 1, 0, b);
        }
    }
    P->nslices = (uint32_t)hn;
    P->slice_lo = (uint32_t *)malloc(sizeof(uint32_t) * (hn + 1));
    P->slice_hi = (uint32_t *)malloc(sizeof(uint32_t) * (hn + 1));
    P->posC = (p3 *)malloc(sizeof(p3) * (hn + 1));
    P->dirC = (p3 *)malloc(sizeof(p3) * (hn + 1));
    for (long k = 0; k < hn; k++) {
        P->slice_lo[k] = heap[k].minInd; P->slice_hi[k] = heap[k].maxInd;
        P->posC[k] = heap[k].posC; P->dirC[k] = heap[k].dirC;
        for (uint32_t i = heap[k].minInd; i < heap[k].maxInd; i++) pixel_to_slice[idx[i]] = (uint32_t)k;
    }
    P->idx = idx;
    free(heap); free(pos); free(dir);
    (void)ngood;
    return rc ? -1 : 0;
}

uint32_t alvrl_o_prep_num_slices(const alvrl_o_prep *P) { return P->nslices; }

/* Slice::sampleRepresentativePixels (Preprocessor.cpp:66-121), sampleSliceMapping
 * (:1502-1525) and buildLocalities (:1241-1293).  rep_pix receives pixel ids in
 * the column-major numbering (id = x*H + y); rep_off has nslices+1 entries. */
int alvrl_o_prep_sample_slice_mapping(alvrl_o_prep *P, float targetUnder, uint32_t *rep_off,
                                      uint32_t *rep_pix, uint32_t cap, float *slice_under,
                                      float *global_under)
{
    uint32_t ns = P->nslices;
    free(P->reps_off); free(P->reps_pix); free(P->slice_under);
    P->reps_off = (uint32_t *)malloc(sizeof(uint32_t) * (ns + 1));
    P->reps_pix = (uint32_t *)malloc(sizeof(uint32_t) * (cap ? cap : 1));
    P->slice_under = (float *)malloc(sizeof(float) * (ns + 1));
    size_t totalPix = 0, totalRep = 0;
    uint32_t outn = 0;
    for (uint32_t s = 0; s < ns; s++) {
        P->reps_off[s] = outn;
        size_t np = P->slice_hi[s] - P->slice_lo[s];
        const uint32_t *gp = P->idx + P->slice_lo[s];
        size_t target = (size_t)(0.5 + (double)((float)np / targetUnder));
        if (target < 2) target = np < 2 ? np : 2;
        smp_t smp;
        smp_init(&smp, P->prm.seed, P->prm.pass, ALVRL_O_DOM_REPS, s, 0, 0);
        if (outn + (target < np ? target : np) > cap) return -1;
        if (np <= target) {
            for (size_t i = 0; i < np; i++) P->reps_pix[outn++] = gp[i];
        } else if (np <= 2 * target) {
            uint32_t *ind = (uint32_t *)malloc(sizeof(uint32_t) * np);
            for (size_t i = 0; i < np; i++) ind[i] = (uint32_t)i;
            for (size_t i = np - 1; i > 0; i--) {
                size_t k = (size_t)((float)(i + 1) * smp_next(&smp));
                uint32_t t = ind[i]; ind[i] = ind[k]; ind[k] = t;
            }
            for (size_t i = 0; i < target; i++) P->reps_pix[outn++] = gp[ind[i]];
            free(ind);
        } else {
            uint32_t *ind = (uint32_t *)malloc(sizeof(uint32_t) * target);
            size_t n = 0;
            while (n < target) {
                int unique;
                do {
                    ind[n] = (uint32_t)(smp_next(&smp) * (float)np);
                    unique = 1;
                    for (size_t i = 0; i < n; i++) if (ind[i] == ind[n]) { unique = 0; break; }
                } while (!unique);
                n++;
            }
            for (size_t i = 0; i < target; i++) P->reps_pix[outn++] = gp[ind[i]];
            free(ind);
        }
        size_t nrep = outn - P->reps_off[s];
        P->slice_under[s] = (float)nrep / (float)np;
        totalRep += nrep; totalPix += np;
    }
    P->reps_off[ns] = outn;
    /* buildLocalities */
    free(P->loc_off); free(P->loc_slice); free(P->loc_dist);
    uint32_t nc = P->prm.neighbour_count;
    P->loc_off = (uint32_t *)calloc(ns + 1, sizeof(uint32_t));
    uint32_t per = ns <= nc ? (ns ? ns - 1 : 0) : nc;
    P->loc_slice = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)ns * per + 1));
    P->loc_dist = (float *)malloc(sizeof(float) * ((size_t)ns * per + 1));
    if (ns <= nc) {
        for (uint32_t i = 0; i < ns; i++) {
            P->loc_off[i] = i * per;
            uint32_t c = 0;
            for (uint32_t j = 0; j < ns; j++) if (i != j) {
                P->loc_slice[i * per + c] = j;
                P->loc_dist[i * per + c] = slice_distance(P->posC[i], P->dirC[i], P->posC[j], P->dirC[j]);
                c++;
            }
        }
    } else if (nc > 0) {
        float *dist = (float *)malloc(sizeof(float) * nc);
        uint32_t *ind = (uint32_t *)calloc(nc, sizeof(uint32_t));
        uint32_t maxInd = 0;   /* not reset per slice (Preprocessor.cpp:1263) */
        for (uint32_t i = 0; i < ns; i++) {
            for (uint32_t j = 0; j < nc; j++) dist[j] = INFINITY;
            for (uint32_t j = 0; j < ns; j++) {
                if (i == j) continue;
                float d = slice_distance(P->posC[i], P->dirC[i], P->posC[j], P->dirC[j]);
                if (d < dist[maxInd]) {
                    dist[maxInd] = d; ind[maxInd] = j;
                    for (uint32_t k = 0; k < nc; k++) if (dist[k] > dist[maxInd]) maxInd = k;
                }
            }
            /* std::set<pair<uint32,Float>> insertion: sort, drop duplicates */
            P->loc_off[i] = i * per;
            uint32_t c = 0;
            for (uint32_t x = 0; x < nc; x++) {
                uint32_t sl = ind[x]; float dd = dist[x];
                uint32_t pos = c, dup = 0;
                for (uint32_t q = 0; q < c; q++) {
                    uint32_t qs = P->loc_slice[i * per + q]; float qd = P->loc_dist[i * per + q];
                    if (qs == sl && qd == dd) { dup = 1; break; }
                }
                if (dup) continue;
                while (pos > 0) {
                    uint32_t qs = P->loc_slice[i * per + pos - 1]; float qd = P->loc_dist[i * per + pos - 1];
                    if (qs < sl || (qs == sl && qd < dd)) break;
                    P->loc_slice[i * per + pos] = qs; P->loc_dist[i * per + pos] = qd;
                    pos--;
                }
                P->loc_slice[i * per + pos] = sl; P->loc_dist[i * per + pos] = dd;
                c++;
            }
            if (c != per) return -3;
        }
        free(dist); free(ind);
    }
    P->loc_off[ns] = ns * per;
    P->global_under = (float)totalRep / (float)totalPix;
    memcpy(rep_off, P->reps_off, sizeof(uint32_t) * (ns + 1));
    memcpy(rep_pix, P->reps_pix, sizeof(uint32_t) * outn);
    if (slice_under) memcpy(slice_under, P->slice_under, sizeof(float) * ns);
    if (global_under) *global_under = P->global_under;
    return 0;
}

/* getLocalMatrix, Preprocessor.cpp:779-827: rows (global row ids) + weights. */
static uint32_t local_matrix(const alvrl_o_prep *P, uint32_t i, uint32_t *rows, double *w)
{
    uint32_t n = 0;
    uint32_t r0 = P->reps_off[i], r1 = P->reps_off[i + 1];
    for (uint32_t r = r0; r < r1; r++) rows[n++] = r;
    uint32_t ni = r1 - r0;
    if (P->prm.neighbour_weight <= 0) {
        for (uint32_t k = 0; k < ni; k++) w[k] = 1.0 / (double)ni;
        return n;
    }
    uint32_t lo = P->loc_off[i], hi = P->loc_off[i + 1];
    float *nw = (float *)malloc(sizeof(float) * (hi - lo + 1));
    float summed = 0;
    for (uint32_t q = lo; q < hi; q++) {
        uint32_t sl = P->loc_slice[q];
        for (uint32_t r = P->reps_off[sl]; r < P->reps_off[sl + 1]; r++) rows[n++] = r;
        nw[q - lo] = (float)(1.0 / (double)P->loc_dist[q]);
        summed += nw[q - lo];
    }
    float nwgt = P->prm.neighbour_weight;
    float sliceWeight = summed * (1 - nwgt) / nwgt;
    float normalization = 1 / (sliceWeight + summed);
    uint32_t m = 0;
    for (uint32_t k = 0; k < ni; k++) w[m++] = (double)(sliceWeight * normalization / (float)ni);
    for (uint32_t q = lo; q < hi; q++) {
        uint32_t sl = P->loc_slice[q];
        uint32_t cnt = P->reps_off[sl + 1] - P->reps_off[sl];
        for (uint32_t k = 0; k < cnt; k++) w[m++] = (double)(nw[q - lo] * normalization / (float)cnt);
    }
    free(nw);
    return n;
}

uint32_t alvrl_o_prep_local_rows(const alvrl_o_prep *P, uint32_t slice, uint32_t *rows, double *w)
{
    return local_matrix(P, slice, rows, w);
}

/* cluster() (Preprocessor.cpp:838-898; with globalCluster, clusterRefinement
 * :899-912 refines the non-zero VRLs over all rows and its clusters become
 * the initial clusters), then buildClusters (:133-197) + refinePerSlice
 * (:199-252) + refineSlice (:254-283).
 * Rt is [nvrl][rows_total] (mean,var) pairs, rows in slice-major order.
 * Outputs: per-slice CSR (slice_off[ns+1], reps, weights), fallback list. */
int alvrl_o_prep_build_clusters(alvrl_o_prep *P, const float *Rt, uint32_t nvrl,
                                uint32_t *slice_off, uint32_t *reps, float *weights, uint32_t cap,
                                uint32_t *gc_reps, float *gc_w, uint32_t *n_gc,
                                uint32_t *fb_reps, float *fb_w, uint32_t *n_fb)
{
    uint32_t ns = P->nslices;
    uint32_t rows_total = P->reps_off[ns];
    uint64_t ld = rows_total;
    /* ---- global cluster (cluster()) on Rflat ---- */
    uint32_t *all_rows = (uint32_t *)malloc(sizeof(uint32_t) * (rows_total + 1));
    for (uint32_t r = 0; r < rows_total; r++) all_rows[r] = r;
    uint32_t *init = (uint32_t *)malloc(sizeof(uint32_t) * (nvrl + 1));
    uint32_t *init_off = (uint32_t *)calloc(nvrl + 2, sizeof(uint32_t)), ninit = 0;
    uint32_t nz = 0;
    for (uint32_t v = 0; v < nvrl; v++) {
        float sum = 0;
        for (uint32_t r = 0; r < rows_total; r++) sum += Rt[2 * ((uint64_t)v * ld + r)];
        if (sum != 0) init[nz++] = v;
    }
    uint32_t nzero = 0;
    double *dw = (double *)malloc(sizeof(double) * (rows_total + 1));
    for (uint32_t r = 0; r < rows_total; r++) dw[r] = 1.0 / (double)rows_total;
    int rc = 0;
    if (nz && P->prm.global_cluster) {
        /* clusterRefinement (:899-912): all non-zero VRLs in one cluster over
         * Rflat, refined with globalUndersampling; getVrlsPerCluster */
        uint32_t one[2] = { 0, nz }, nc = 0;
        uint32_t *members = (uint32_t *)malloc(sizeof(uint32_t) * (nz + 1));
        int ok = 0;
        if (alvrl_o_cluster_members(Rt, ld, all_rows, rows_total, dw, nvrl, init, one, 1,
                                    P->global_under, P->prm.global_undersampling, P->prm.seed,
                                    P->prm.pass, ALVRL_O_STAGE_GLOBAL_REFINE, members, init_off,
                                    &nc, &ok) || !ok)
            rc = -7;   /* "Couldn't refine global clustering!" */
        memcpy(init, members, sizeof(uint32_t) * nz);
        free(members);
        ninit = nc;
    } else if (nz) {
        init_off[1] = nz; ninit = 1;
    }
    for (uint32_t v = 0; v < nvrl; v++) {
        float sum = 0;
        for (uint32_t r = 0; r < rows_total; r++) sum += Rt[2 * ((uint64_t)v * ld + r)];
        if (sum == 0) init[nz + nzero++] = v;
    }
    if (nzero) { init_off[ninit + 1] = nz + nzero; ninit++; }
    if (!rc) {
        mat_t M = { Rt, ld, all_rows, rows_total, nvrl };
        clustering_t C;
        if (clustering_init(&C, &M, dw, init, init_off, ninit, P->global_under, 1.0f,
                            P->prm.seed, P->prm.pass, ALVRL_O_STAGE_FALLBACK_REFINE)) rc = -2;
        if (!rc) {
            *n_gc = sample_reps(&C, ALVRL_O_STAGE_GLOBAL_SAMPLE, gc_reps, gc_w);
            if (!refine(&C, P->prm.fallback_undersampling)) rc = -3;
            *n_fb = sample_reps(&C, ALVRL_O_STAGE_FALLBACK_SAMPLE, fb_reps, fb_w);
        }
        if (C.err) rc = rc ? rc : -4;
        clustering_free(&C);
    }
    if (rc) { free(all_rows); free(init); free(init_off); free(dw); return rc; }
    /* ---- refinePerSlice ---- */
    uint32_t *rows = all_rows;
    double *w = dw;
    uint32_t out = 0;
    for (uint32_t s = 0; s < ns; s++) {
        slice_off[s] = out;
        uint32_t nr = local_matrix(P, s, rows, w);
        uint32_t got = 0;
        int refined = 0;
        if (out + nvrl > cap) { rc = -5; break; }
        int e = alvrl_o_cluster_refine(Rt, ld, rows, nr, w, nvrl, init, init_off, ninit,
                                       P->slice_under[s], P->prm.local_undersampling,
                                       P->prm.depth_correction, P->prm.local_refinement,
                                       P->prm.seed, P->prm.pass, ALVRL_O_STAGE_SLICE_REFINE(s),
                                       ALVRL_O_STAGE_SLICE_SAMPLE(s), reps + out, weights + out,
                                       &got, &refined);
        if (e) { rc = -6; break; }
        if (!refined) {
            memcpy(reps + out, fb_reps, sizeof(uint32_t) * *n_fb);
            memcpy(weights + out, fb_w, sizeof(float) * *n_fb);
            got = *n_fb;
        }
        out += got;
    }
    slice_off[ns] = out;
    free(all_rows); free(init); free(init_off); free(dw);
    return rc;
}
