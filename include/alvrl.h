/*
 * alvrl.h -- C ABI of the MI355X-native ALVRL hot path (libalvrl.so).
 *
 * This is the drop-in boundary: everything a Mitsuba 0.x 'vrl' integrator
 * plugin (src/integrators/vrl/vrlIntegrator.cpp, exported through
 * MTS_EXPORT_PLUGIN at :1127 and driven through the ProgressiveMonteCarlo-
 * Integrator vtable, include/mitsuba/render/integrator.h:482-511) needs from
 * the device.  Plain C types only: no torch, no HIP types in signatures
 * (streams are passed as void* = hipStream_t, NULL = the context's stream,
 * ordered after the work already queued on the null stream).
 * Errors are int status codes (ALVRL_OK = 0) plus alvrl_last_error(); no C++
 * exception crosses this boundary (the reference throws from Log(EError),
 * src/libcore/logger.cpp:147; the shim in INTEGRATION.md maps a non-zero
 * status back to Log(EError)).
 *
 * Each entry point names the reference interface it replaces.
 */
#ifndef ALVRL_H
#define ALVRL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define ALVRL_API __attribute__((visibility("default")))
#else
#define ALVRL_API
#endif

#define ALVRL_ABI_VERSION 2

enum {
    ALVRL_OK = 0,
    ALVRL_ERR_INVALID = 1,   /* bad argument (reference: Log(EError, ...) on bad parameters) */
    ALVRL_ERR_STATE = 2,     /* call order violated (e.g. gather before upload_vrls) */
    ALVRL_ERR_HIP = 3,       /* HIP runtime failure */
    ALVRL_ERR_NOMEM = 4,
    ALVRL_ERR_NUMERIC = 5,   /* an invariant of the clustering maths failed (reference: SLog(EError)) */
    ALVRL_ERR_COMM = 6       /* the caller's collective (alvrl_exchange) failed */
};

/* Record-flag bits of alvrl_gather_rec.flags */
#define ALVRL_REC_HIT     1u   /* rRec.its.isValid()                          (vrlIntegrator.cpp:712) */
#define ALVRL_REC_SMOOTH  2u   /* bsdf->getType() & BSDF::ESmooth             (vrlIntegrator.cpp:726-727) */
#define ALVRL_REC_MEDIUM  4u   /* rRec.medium && !getSigmaS().isZero()         (vrlIntegrator.cpp:614, 795) */
#define ALVRL_REC_DELTA   8u   /* its BSDF has a delta component: the eye path continues (:449-511) */
#define ALVRL_REC_ACCUM  16u   /* R build: add to the row's entries (a deeper segment of the row's
                                  eye path; vrlContributions accumulate over the recursion, :812-813) */

/* Integrator properties that shape the device maths.
 * Replaces the Properties parsing in vrlIntegrator(const Properties&), vrlIntegrator.cpp:128-208. */
typedef struct {
    int device;             /* HIP device ordinal */
    int vol_vol_samples;    /* "volVolSamples"  (default 2; 0 or >= 2), :148-151 */
    int vol_surf_samples;   /* "volSurfSamples" (default 2; 0 or >= 2), :153-156 */
    int short_vrls;         /* "shortVrls" (default true), :135 */
    uint32_t seed;          /* sampler seed: replaces the SFMT /dev/urandom seeding (random.cpp:473-489) */
} alvrl_config;

/* Homogeneous medium + phase function of the (single) medium the VRLs live in.
 * Replaces HomogeneousMedium(const Properties&) (src/medium/homogeneous.cpp:156-227)
 * with its distance-sampling "strategy" -- which sets the tracer's distances
 * and pdfs (sampleDistance, :275-352) and the pdfFailure the gather divides
 * by (eval, :354-396) -- and IsotropicPhaseFunction / HGPhaseFunction eval.
 * A zero-filled tail (strategy, channel, sampling_density) is the default
 * 'balance' strategy. */
#define ALVRL_STRATEGY_BALANCE 0  /* a random channel's sigma_t per sample */
#define ALVRL_STRATEGY_SINGLE 1   /* one channel's sigma_t (:188-214) */
#define ALVRL_STRATEGY_MANUAL 2   /* "samplingDensity" (:221-223) */
#define ALVRL_STRATEGY_MAXIMUM 3  /* MaxExpDist over sigma_t (maxexp.h:28-94); channels must differ */
typedef struct {
    float sigma_s[3];
    float sigma_a[3];
    float sampling_weight;  /* "mediumSamplingWeight"; -1 = auto (max albedo, >= 0.5) */
    int phase_type;         /* 0 = isotropic (isotropic.cpp:76-78), 1 = HG (hg.cpp:107-110) */
    float phase_g;
    int strategy;           /* ALVRL_STRATEGY_* */
    int channel;            /* 'single': 1 + "channel" (0: the smallest sigma_t, :191-202) */
    float sampling_density; /* 'manual': "samplingDensity" */
} alvrl_medium_desc;

/* One eye segment ("gather record"), 80 B.  What LiInternal knows at the point
 * it calls getVRLContributions / getClusteredVrlContributions
 * (vrlIntegrator.cpp:418-443): ray.o, ray.d, rRec.its.{p, shFrame.n}, the
 * diffuse reflectance of its BSDF and the medium/hit flags, and -- for the
 * segments of a specular chain (LiInternal's recursion through delta BSDFs,
 * :445-511) -- the path weight the recursion passes down and the segment's
 * depth along the eye path. */
typedef struct {
    float o[3];        /* E  = ray.o */
    float d[3];        /* ray.d */
    float p[3];        /* Usurf = rRec.its.p */
    float n[3];        /* rRec.its.shFrame.n */
    float albedo[3];   /* SmoothDiffuse reflectance (diffuse.cpp:110-118) */
    uint32_t flags;    /* ALVRL_REC_* */
    float weight[3];   /* LiInternal's 'weight' (:503-510): the gathered radiance and the
                          R entries' luminance samples are multiplied by it; (1, 1, 1) for a
                          camera ray */
    uint32_t depth;    /* eye-path vertex the segment starts at (0: the camera ray); keys the
                          segment's own sample streams (< 256) */
} alvrl_gather_rec;

/* A wave-sized run of slice-bucketed records for the clustered gather:
 * records [begin, begin+count) all use the representative list of 'slice'
 * (UINT32_MAX = the fall-back list, vrlIntegrator.cpp:564-571). count <= 64. */
typedef struct {
    uint32_t slice;
    uint32_t begin;
    uint32_t count;
    uint32_t pad;
} alvrl_work_item;

typedef struct alvrl_ctx alvrl_ctx;

/* ---- lifecycle ------------------------------------------------------ */
/* Replaces vrlIntegrator::vrlIntegrator(const Properties&) (:128-208) for the
 * device state; returns ALVRL_OK and *out, or an error (see alvrl_last_error(NULL)). */
ALVRL_API int alvrl_ctx_create(const alvrl_config *cfg, alvrl_ctx **out);
/* Replaces the implicit destruction of m_vrls / m_ci (ref<> members, :1089-1090). */
ALVRL_API void alvrl_ctx_destroy(alvrl_ctx *ctx);
/* Last error of this context on the calling thread (ctx == NULL: global). */
ALVRL_API const char *alvrl_last_error(const alvrl_ctx *ctx);
ALVRL_API int alvrl_abi_version(void);
/* "src <hash> ...": the first 16 hex digits of the SHA-1 of the library's
 * sources (the .hip, .hpp, host .cpp/.hpp and include .h files, concatenated
 * in path order, mitsuba-alvrl_amd/Makefile SRC_HASH) it was built from; the Python binding recomputes it from the tree
 * (alvrl.build_info) so a prebuilt library is checked against its sources. */
ALVRL_API const char *alvrl_build_id(void);

/* ---- per-scene / per-pass state (set in preprocess/prepass; immutable
 *      while gathers run, vrlIntegrator.cpp:237-356) -------------------- */
/* Replaces scene->getMedia()[0] / vrl.m_medium lookups (:244-249, 607). */
ALVRL_API int alvrl_set_medium(alvrl_ctx *ctx, const alvrl_medium_desc *m);
/* Progressive pass index (integrator.cpp:396-433): keys the counter RNG. */
ALVRL_API int alvrl_set_pass(alvrl_ctx *ctx, uint32_t pass);
/* Occluder triangles (9 floats each: p0 p1 p2) for the visibility part of
 * Scene::evalTransmittance (scene.cpp:619-679) in every gather and R build:
 * a U-V (vol->vol) or surface-V (vol->surf) connection crossing one
 * contributes 0, unless its material (NULL: none is) is ALVRL_MAT_NULL
 * (alvrl_host.h): a null-BSDF surface lets the connection pass (:636-637).
 * Replaces the scene's ShapeKDTree (skdtree.h) for these queries with a BVH
 * built here and kept on the device.  ntri == 0: the convex container (no
 * tests).  Waits for every launch on the device first. */
ALVRL_API int alvrl_set_occluders(alvrl_ctx *ctx, const float *tris, uint32_t ntri, const uint32_t *material);
/* Replaces m_vrls = tracer->randomWalk(...) / new vrlVector(fs, medium) and
 * registerResource(m_vrls) (:276-287, 353).  soa = 9 arrays of n floats:
 * start xyz, end xyz, power rgb (VRL.h:89-96).  particle_count = vrlVector::
 * getParticleCount() (VRL.h:164-166), the 1/particleCount normalisation.
 * soa_on_device != 0: soa is a device pointer.  Waits for every launch on the
 * device first (the records are overwritten in place). */
ALVRL_API int alvrl_upload_vrls(alvrl_ctx *ctx, const float *soa, uint32_t n,
                                uint64_t particle_count, int soa_on_device);
ALVRL_API uint32_t alvrl_num_vrls(const alvrl_ctx *ctx);

/* Replaces m_ci->m_selectedVrls / m_clusterWeight / m_fallBackVrls /
 * m_fallBackWeight (vrlClusterInfo, :17-115; written by buildClusters at :341-346).
 * CSR on the host: slice s uses reps[slice_off[s] .. slice_off[s+1]).  The
 * device lists are overwritten in place.  The call takes the context's state
 * lock exclusively (the gathers and R builds hold it shared from their checks
 * to their enqueue, so none is enqueued during the update) and then waits for
 * the whole device (hipDeviceSynchronize): a gather still reading the
 * previous lists on any stream -- the caller's included -- finishes first.
 * That wait also waits for unrelated work on other streams of the device
 * (e.g. a collective in flight); call it between passes, as the prepass does.
 * alvrl_upload_vrls and alvrl_set_occluders behave the same way. */
ALVRL_API int alvrl_set_clusters(alvrl_ctx *ctx, uint32_t nslices, const uint32_t *slice_off,
                                 const uint32_t *reps, const float *weights,
                                 const uint32_t *fb_reps, const float *fb_weights, uint32_t n_fb);

/* ---- hot path (a): per-record VRL gather ------------------------------ */
/* Threading (renderBlock runs on every LocalWorker at once, renderproc.cpp:
 * 52-86): the gathers may be called concurrently from any number of host
 * threads on one context.  Each calling thread gets its own HIP stream (the
 * NULL-stream and host-pointer variants use it), its own grow-only device
 * scratch for the host-pointer variants (no allocation per call) and its own
 * timing events: alvrl_last_kernel_ms reports the calling thread's last launch. */
/* Replaces getVRLContributions (:792-825) -> integrateVRL (:603-785) for every
 * VRL.  d_recs / d_rec_ids / d_out_rgb are device pointers; d_rec_ids may be
 * NULL (record id = index).  The record id keys the sampling uniforms.
 * d_out_rgb[3*r..] = Li of record r (already * 1/particleCount). */
ALVRL_API int alvrl_gather_brute(alvrl_ctx *ctx, const alvrl_gather_rec *d_recs,
                                 const uint32_t *d_rec_ids, uint32_t nrec, float *d_out_rgb,
                                 void *stream);
/* Replaces getClusteredVrlContributions (:542-599): sum_k w_k * integrateVRL(rep_k)
 * / particleCount over the record's slice list.  Records must be bucketed by
 * slice and described by wave work items (alvrl_make_work_items). */
ALVRL_API int alvrl_gather_clustered(alvrl_ctx *ctx, const alvrl_gather_rec *d_recs,
                                     const uint32_t *d_rec_ids, const alvrl_work_item *d_items,
                                     uint32_t nitems, float *d_out_rgb, void *stream);
/* The false-colour debug images of LiInternal (vrlIntegrator.cpp:199-201,
 * 545-599, 794-806) for primary rays, instead of a gather:
 *   ALVRL_FALSE_COLOR_NUM_VRLS ("numVrlFalseColor"): |slice list| / N with
 *     d_items (clustered, :574-575), 1 without (brute, :800-801), where the
 *     record's medium scatters, else 0;
 *   ALVRL_FALSE_COLOR_SLICES ("slicesFalseColor", clustered only, :576-583):
 *     the slice's hash colour, grey 0.5 for the fall-back list.
 * n = work items (d_items != NULL) or records.  The render counter grows by
 * the list sizes as the reference's stats do (:593-596). */
#define ALVRL_FALSE_COLOR_NUM_VRLS 1
#define ALVRL_FALSE_COLOR_SLICES 2
ALVRL_API int alvrl_gather_false_color(alvrl_ctx *ctx, int mode, const alvrl_gather_rec *d_recs,
                                       const alvrl_work_item *d_items, uint32_t n, float *d_out_rgb,
                                       void *stream);
/* Host helper: build work items from a slice-sorted slice-of-record array
 * (host memory).  Returns the number of items written (<= cap). */
ALVRL_API uint32_t alvrl_make_work_items(const uint32_t *slice_of_rec_sorted, uint32_t nrec,
                                         alvrl_work_item *items, uint32_t cap);

/* ---- hot path (b) part 1: reduced transport matrix R ------------------ */
/* "Rsamples" (vrlIntegrator.cpp:194, default 1): gather samples per R entry.
 * getLiLuminanceVrlContributions runs LiInternal with samples = Rsamples and
 * the entries accumulate, so they are SUMS over the samples (:427-443,
 * :812-813).  Sample i draws from stream (R domain, i). */
ALVRL_API int alvrl_set_rsamples(alvrl_ctx *ctx, int rsamples);

/* Replaces Rbuilder::run (:1053-1067) -> getLiLuminanceVrlContributions
 * (:527-539) with Rsamples = 1.  Writes (mean, var) float pairs to
 * d_Rt[2*(v*ld + row0 + r) + {0,1}] for record r of d_recs and VRL v, i.e. R
 * stored VRL-major with the representative rows contiguous. */
ALVRL_API int alvrl_build_R(alvrl_ctx *ctx, const alvrl_gather_rec *d_recs,
                            const uint32_t *d_rec_ids, uint32_t nrows, float *d_Rt, uint64_t ld,
                            uint64_t row0, void *stream);

/* Replaces the zero / non-zero split of Preprocessor::cluster (:843-855,
 * totalVrlContribution :936-945): out_mask[v] = 1 iff some row of R has a
 * non-zero mean for VRL v (every mean is >= 0, so this equals sum != 0).
 * Rows [0, nrows) of d_Rt; out_mask is host memory (nvrl bytes). */
ALVRL_API int alvrl_nonzero_columns(alvrl_ctx *ctx, const float *d_Rt, uint64_t ld, uint32_t nrows,
                                    uint8_t *out_mask, void *stream);

/* alvrl_build_R for rows scattered over per-slice blocks, in one launch:
 * row r's pair for VRL v goes to float2 index d_row_off[r] + v * d_row_stride[r]
 * (device arrays).  If d_nonzero (device, nvrl bytes) is given, every VRL
 * with a non-zero mean in these rows sets d_nonzero[v] = 1 (never clears it),
 * which is alvrl_nonzero_columns fused into the build. */
ALVRL_API int alvrl_build_R_blocks(alvrl_ctx *ctx, const alvrl_gather_rec *d_recs,
                                   const uint32_t *d_rec_ids, uint32_t nrows, float *d_Rt,
                                   const uint64_t *d_row_off, const uint32_t *d_row_stride,
                                   uint8_t *d_nonzero, void *stream);

/* The R build in the CPU restatement's arithmetic (no replaced reference
 * function: a mode of alvrl_build_R / alvrl_build_R_blocks).  on != 0: both
 * evaluate integrateVRL (vrlIntegrator.cpp:603-785) statement for statement
 * as oracle/alvrl_oracle.c does, with IEEE division / sqrt, no contraction and
 * the deterministic transcendentals of csrc/detmath.h, so every R entry is the
 * oracle's bit for bit and the clustering downstream reproduces the oracle's
 * own pipeline.  Slower than the fast build.  A bare
 * context starts with the fast build; the integrator pipeline
 * (alvrl_integrator_create) turns this on unless its property "strictRbuild"
 * is false. */
ALVRL_API int alvrl_set_strict_rbuild(alvrl_ctx *ctx, int on);

/* csrc/detmath.h on the current device, elementwise over n floats (device
 * pointers; fn 0 exp, 1 log, 2 atan, 3 tan, 4 asinh, 5 sinh): the host =
 * device check of the definitions the strict paths share with the oracle.
 * fn + 8 (8, 10-13) evaluates the strict kernels' fast form
 * (csrc/detmath_fast.h) instead. */
ALVRL_API int alvrl_detmath_eval(int fn, const float *d_in, float *d_out, uint32_t n, void *stream);

/* The fast form against detmath.h for every float bit pattern in [begin, end)
 * (end <= 2^32), on the current device, synchronous: *mismatches = the number
 * of inputs whose results differ in any bit, first[0 .. min(nfirst, 16)) =
 * some of them (0xFFFFFFFF past the last).  fn 0 exp, 2 atan, 3 tan,
 * 4 asinh, 5 sinh, 6 sqrt (the fast square root against IEEE sqrtf), 7 rcp
 * (the fast reciprocal against IEEE 1.0f / x). */
ALVRL_API int alvrl_detmath_exhaustive(int fn, uint64_t begin, uint64_t end, uint64_t *mismatches,
                                       uint32_t *first, uint32_t nfirst);

/* The strict kernels' fast division (csrc/detmath_fast.h fx_divf) against
 * IEEE a / b on n pseudo-random operand pairs (half uniform over all bit
 * patterns, half log-uniform in [2^-44, 2^44]), on the current device,
 * synchronous: *mismatches = pairs whose quotients differ in any bit,
 * first[0 .. min(nfirst, 16)) = (a, b) bit patterns of some of them. */
ALVRL_API int alvrl_detmath_div_check(uint64_t n, uint64_t seed, uint64_t *mismatches, uint32_t *first,
                                      uint32_t nfirst);

/* ---- hot path (b) part 2: cluster refinement ------------------------- */
/* One Clustering (Preprocessor.cpp:287-720): ctor (column weights, initial
 * clusters, unclustered variances, :301-341), optional refine() (:380-489),
 * sampleRepresentatives() (:354-378).  Host pointers. */
typedef struct {
    const uint32_t *rows;     /* local matrix rows = row ids into R (getLocalMatrix, :779-827) */
    const double *locw;       /* locality weights, one per row (sum 1) */
    uint32_t nrows;
    float pixel_undersampling;/* m_sliceUndersampling[i] or m_globalPixelUndersampling */
    float undersampling;      /* refine(): <= 0 adaptive (:402-489), > 0 fixed depth (:387-399) */
    float depth_correction;   /* "depthCorrection" */
    int do_refine;            /* 0: only sampleRepresentatives (localRefinement=false, :270-274) */
    uint32_t stage_refine;    /* counter-RNG stream ids of the split / sampling draws */
    uint32_t stage_sample;
    /* Optional R layout per row (NULL: entry (v, r) is d_Rt[rows[r] + v * ld]).
     * Otherwise entry (v, r) is the float2 at index row_off[r] + v * row_stride[r]
     * -- e.g. R stored as one [vrl][row] block per slice, which keeps a slice's
     * local matrix contiguous (rows is then ignored and may be NULL). */
    const uint64_t *row_off;
    const uint32_t *row_stride;
} alvrl_cluster_job;

/* Replaces refinePerSlice -> refineSlice (Preprocessor.cpp:199-283) and the
 * fall-back refinement in buildClusters (:175-186): runs every job on the
 * device, one persistent workgroup per job, all jobs concurrently.
 *   d_Rt, ld      : R as written by alvrl_build_R
 *   init_vrls/off : the global clusters (Preprocessor::cluster, :838-898), host
 * Outputs (host): per job the representatives and weights in CSR
 * (out_off[njobs+1], capacity njobs * nvrl entries) and out_refined[j]
 * (0 = refine() returned false, the caller substitutes the fall-back list). */
ALVRL_API int alvrl_refine(alvrl_ctx *ctx, const float *d_Rt, uint64_t ld, uint32_t njobs,
                           const alvrl_cluster_job *jobs, const uint32_t *init_vrls,
                           const uint32_t *init_off, uint32_t ninit, uint32_t *out_off,
                           uint32_t *out_reps, float *out_weights, int *out_refined,
                           void *stream);
/* clusterRefinement (Preprocessor.cpp:899-912, the globalCluster option):
 * one Clustering ctor + refine(job->undersampling), then getVrlsPerCluster
 * (:526-543) -- singletons in list order, then the heap's clusters.  The
 * initial clusters may list a subset of the VRLs (the non-zero ones).
 * out_vrls: init_off[ninit] ids; out_off: *n_clusters + 1 offsets (capacity
 * init_off[ninit] + 1).  job->do_refine and depth_correction are ignored. */
ALVRL_API int alvrl_refine_members(alvrl_ctx *ctx, const float *d_Rt, uint64_t ld,
                                   const alvrl_cluster_job *job, const uint32_t *init_vrls,
                                   const uint32_t *init_off, uint32_t ninit, uint32_t *out_vrls,
                                   uint32_t *out_off, uint32_t *n_clusters, int *out_refined,
                                   void *stream);
/* Milliseconds the device spent in the last alvrl_refine call (HIP events). */
ALVRL_API int alvrl_last_refine_ms(alvrl_ctx *ctx, float *ms);
/* R entries (float2, 8 B each) the last alvrl_refine had to read, summed over
 * its jobs: nrows * (3 * nvrl + the columns of every cluster it split) --
 * column weights, initial cluster variances and the unclustered variance read
 * the whole local matrix once, and each split's cluster is counted once. */
ALVRL_API int alvrl_last_refine_entries(alvrl_ctx *ctx, uint64_t *entries);
/* Of those, the splits' share: nrows * (the columns of every cluster split).
 * A split reads them three times (Clustering::split, Preprocessor.cpp:590-684:
 * the projections, then the forward and the reverse calculateClusterVariance
 * pass), so the refinement's algorithmic bytes (one count per
 * split pass) are 8 * (entries + 2 * split_entries). */
ALVRL_API int alvrl_last_refine_split_entries(alvrl_ctx *ctx, uint64_t *entries);

/* ---- framebuffer --------------------------------------------------- */
/* ImageBlock::put of 1-spp box-filtered samples (imageblock.h:124-131):
 * d_fb[3*d_pixel[r] + c] += d_rgb[3*r + c] for r < n. */
ALVRL_API int alvrl_accumulate_rgb(alvrl_ctx *ctx, const float *d_rgb, const uint32_t *d_pixel,
                                   uint32_t n, float *d_fb, void *stream);

/* ---- statistics ------------------------------------------------------- */
/* statsVrlsPreprocess / statsVrlsRender (:119-122, 593-596, 819-822): number
 * of integrateVRL evaluations.  Synchronises the context's counters. */
ALVRL_API int alvrl_get_stats(alvrl_ctx *ctx, uint64_t *preprocess, uint64_t *render);
ALVRL_API int alvrl_reset_stats(alvrl_ctx *ctx);

/* ---- host-pointer conveniences for the Mitsuba shim's renderBlock ----- */
/* Same as alvrl_gather_brute / alvrl_gather_clustered with host arrays;
 * slice_of_rec may be unsorted (UINT32_MAX = fall-back).  Blocking.
 * Calls from several threads are merged: one caller stages every request
 * queued so far in pinned memory and runs them as one launch (a record's
 * result is the same bits in any batch); rec_ids NULL keys a record's streams
 * by its index in its own call.  alvrl_last_kernel_ms of a thread whose
 * request another thread launched is not updated. */
ALVRL_API int alvrl_gather_brute_host(alvrl_ctx *ctx, const alvrl_gather_rec *recs,
                                      const uint32_t *rec_ids, uint32_t nrec, float *out_rgb);
ALVRL_API int alvrl_gather_clustered_host(alvrl_ctx *ctx, const alvrl_gather_rec *recs,
                                          const uint32_t *rec_ids, const uint32_t *slice_of_rec,
                                          uint32_t nrec, float *out_rgb);
/* Diagnostic: launches of the host-pointer gathers and the requests they
 * carried, [0] brute, [1] clustered, since the context was created. */
ALVRL_API int alvrl_host_batch_stats(alvrl_ctx *ctx, uint64_t batches[2], uint64_t requests[2]);

/* ---- timing of the last kernel launched on the context (HIP events) --- */
/* Milliseconds between the begin/end events recorded around the most recent
 * gather / R-build launch, on the stream it ran on.  Synchronises. */
ALVRL_API int alvrl_last_kernel_ms(alvrl_ctx *ctx, float *ms);

#ifdef __cplusplus
}
#endif
#endif /* ALVRL_H */
