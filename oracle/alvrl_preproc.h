/*
 * alvrl_preproc.h -- CPU restatement of LightSlice preprocessing
 * (src/integrators/vrl/Preprocessor.cpp).  TEST INFRASTRUCTURE ONLY.
 */
#ifndef ALVRL_PREPROC_H
#define ALVRL_PREPROC_H

#include <stdint.h>
#include "alvrl_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Philox stream 'c' word for the clustering stages. */
#define ALVRL_O_STAGE_GLOBAL_SAMPLE    0u
#define ALVRL_O_STAGE_FALLBACK_REFINE  1u
#define ALVRL_O_STAGE_FALLBACK_SAMPLE  2u
#define ALVRL_O_STAGE_SLICE_REFINE(s)  (3u + 2u * (uint32_t)(s))
#define ALVRL_O_STAGE_SLICE_SAMPLE(s)  (4u + 2u * (uint32_t)(s))
#define ALVRL_O_STAGE_GLOBAL_REFINE    0xFFFFFFFEu   /* clusterRefinement (globalCluster) */

/* Preprocessor ctor arguments (Preprocessor.cpp:20-39, vrlIntegrator.cpp:158-197). */
typedef struct {
    uint32_t target_num_slices;       /* targetNumSlices (100) */
    uint32_t neighbour_count;         /* neighbourCount (0) */
    float neighbour_weight;           /* neighbourWeight (0) */
    int global_cluster;               /* globalCluster (false) */
    int local_refinement;             /* localRefinement (true) */
    float global_undersampling;       /* globalUndersampling (-1) */
    float local_undersampling;        /* localUndersampling (-1 = adaptive) */
    float fallback_undersampling;     /* fallBackUndersampling (5) */
    float depth_correction;           /* depthCorrection (1) */
    float slice_curvature_factor;     /* sliceCurvatureFactor (0.5) */
    uint32_t seed, pass;
} alvrl_o_prep_params;

typedef struct alvrl_o_prep alvrl_o_prep;

alvrl_o_prep *alvrl_o_prep_create(const alvrl_o_prep_params *p);
void alvrl_o_prep_destroy(alvrl_o_prep *P);
int alvrl_o_prep_build_slices(alvrl_o_prep *P, const alvrl_o_scene *s, uint32_t *pixel_to_slice);
uint32_t alvrl_o_prep_num_slices(const alvrl_o_prep *P);
int alvrl_o_prep_sample_slice_mapping(alvrl_o_prep *P, float target_pixel_undersampling,
                                      uint32_t *rep_off, uint32_t *rep_pix, uint32_t cap,
                                      float *slice_under, float *global_under);
uint32_t alvrl_o_prep_local_rows(const alvrl_o_prep *P, uint32_t slice, uint32_t *rows, double *w);
int alvrl_o_prep_build_clusters(alvrl_o_prep *P, const float *Rt, uint32_t nvrl,
                                uint32_t *slice_off, uint32_t *reps, float *weights, uint32_t cap,
                                uint32_t *gc_reps, float *gc_w, uint32_t *n_gc,
                                uint32_t *fb_reps, float *fb_w, uint32_t *n_fb);

/* One Clustering: ctor + (optional) refine + sampleRepresentatives. */
int alvrl_o_cluster_refine(const float *Rt, uint64_t ld, const uint32_t *rows, uint32_t nrows,
                           const double *locw, uint32_t nvrl,
                           const uint32_t *init_vrls, const uint32_t *init_off, uint32_t ninit,
                           float pixel_undersampling, float undersampling, float depth_correction,
                           int do_refine, uint32_t seed, uint32_t pass, uint32_t stage_refine,
                           uint32_t stage_sample, uint32_t *reps, float *weights, uint32_t *nreps,
                           int *refined);

/* ctor + refine(undersampling) + getVrlsPerCluster (Preprocessor.cpp:526-543):
 * out_vrls (init_off[ninit] ids) and out_off (clusters + 1), depthCorrection 1. */
int alvrl_o_cluster_members(const float *Rt, uint64_t ld, const uint32_t *rows, uint32_t nrows,
                            const double *locw, uint32_t nvrl,
                            const uint32_t *init_vrls, const uint32_t *init_off, uint32_t ninit,
                            float pixel_undersampling, float undersampling, uint32_t seed, uint32_t pass,
                            uint32_t stage_refine, uint32_t *out_vrls, uint32_t *out_off,
                            uint32_t *nclusters, int *refined);

#ifdef __cplusplus
}
#endif
#endif
