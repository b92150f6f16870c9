/*
 * alvrl_host.h -- host-side harness of libalvrl.so (C ABI).
 *
 * Not part of the device boundary (include/alvrl.h): these entry points are
 * the standalone stand-ins for what a Mitsuba host provides around the vrl
 * plugin -- the smoke-box scene (Sensor::sampleRay + Scene::rayIntersect for an
 * inside-the-box camera), the VRL tracer (vrlTracer.h), the ASCII VRL file
 * format (VRL.h:43-54, 120-128) and the LightSlice slicing step
 * (Preprocessor::buildSlices / sampleSliceMapping / buildLocalities /
 * getLocalMatrix, Preprocessor.cpp:66-121, 779-827, 1130-1525) -- plus the
 * integrator pipeline that drives include/alvrl.h like vrlIntegrator does.
 */
#ifndef ALVRL_HOST_H
#define ALVRL_HOST_H

#include <stdint.h>
#include "alvrl.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    float cam_origin[3], cam_target[3], cam_up[3];
    float fov_x_deg;
    int width, height;
    float box_min[3], box_max[3];
    float albedo[3];
    float light_pos[3];
    float light_intensity[3];
    alvrl_medium_desc medium;
    /* Optional occluders inside the box: n_occluders triangles, 9 floats
     * each (p0, p1, p2; counter-clockwise seen from the lit side: the face
     * normal is normalize(cross(p1 - p0, p2 - p0)), skdtree.h:367-396), with
     * a one-sided diffuse BSDF of reflectance occluder_albedo.  They are hit
     * by eye rays and particles and block the gather's U-V and surface-V
     * connections (Scene::evalTransmittance, scene.cpp:619-679).  The array
     * is read during the call that receives the descriptor (and copied by
     * alvrl_integrator_preprocess). */
    const float *occluders;
    uint32_t n_occluders;
    float occluder_albedo[3];
    /* Per-occluder BSDF (NULL: every triangle diffuse), ALVRL_MAT_*:
     *   DIFFUSE  one-sided diffuse of reflectance occluder_albedo (diffuse.cpp);
     *   MIRROR   one-sided smooth conductor, material "none" (Fresnel 1) and
     *            specular reflectance occluder_specular (conductor.cpp:254-268):
     *            a delta BSDF, so eye paths continue past it (LiInternal's
     *            specular chains, vrlIntegrator.cpp:445-511);
     *   NULL     index-matched interface (null.cpp:38-76): light passes through
     *            unchanged; transparent to Scene::evalTransmittance
     *            (scene.cpp:633-676), skipped by buildSlices (Preprocessor.cpp:
     *            1157-1169), it cuts VRLs (vrlTracer.h:173-213);
     *   DIELECTRIC  smooth dielectric interface with m_eta = occluder_eta
     *            (dielectric.cpp, specular reflectance and transmittance 1): a
     *            delta BSDF with two components, so LiInternal's chains branch
     *            into reflection and transmission (bRec.component = i, :467-511);
     *            particles reflect with probability F, else refract
     *            (dielectric.cpp:335-364); blocks shadow segments. */
    const uint32_t *occluder_material;
    float occluder_specular[3];
    float occluder_eta;   /* intIOR / extIOR of DIELECTRIC triangles (<= 0: bk7 / air, ior.h:43, 60) */
    /* Optional area emitter (src/emitters/area.cpp on a triangle mesh),
     * replacing the point light when n_emitter_tris > 0: 9 floats per
     * triangle (p0, p1, p2), emitting radiance emitter_radiance on the side of
     * normalize(cross(p1 - p0, p2 - p0)).  Particles start at a point drawn
     * uniformly by area (TriMesh::samplePosition, trimesh.cpp:388-423;
     * Triangle::sample, triangle.cpp:24-59) with power radiance * pi * area
     * (area.cpp:198) and a cosine-weighted direction (area.cpp:115-123).  The
     * emitter is no surface of its own: list its triangles among the
     * occluders too for eye rays and shadow tests to see it. */
    const float *emitter_tris;
    uint32_t n_emitter_tris;
    float emitter_radiance[3];
    /* Optional per-occluder diffuse reflectance, 3 floats per triangle in
     * [0, 1] (NULL: occluder_albedo for every DIFFUSE triangle): each
     * shape's own SmoothDiffuse -- e.g. an area emitter's mesh, to which
     * Mitsuba gives an all-absorbing one (shape.cpp:49-56).  Read like
     * occluders. */
    const float *occluder_albedos;
} alvrl_scene_desc;
#define ALVRL_MAT_DIFFUSE 0u
#define ALVRL_MAT_MIRROR 1u
#define ALVRL_MAT_NULL 2u
#define ALVRL_MAT_DIELECTRIC 3u

/* The benchmark scene of BASELINE.md ("homogeneous smoke box"). */
ALVRL_API void alvrl_scene_default(alvrl_scene_desc *s, int width, int height);

/* Gather records of pixel centres.  pixel_ids (row-major y*W+x) may be NULL:
 * all pixels in row-major order (n must be W*H then). */
ALVRL_API int alvrl_scene_records(const alvrl_scene_desc *s, int medium_scatters,
                                  const uint32_t *pixel_ids, uint32_t n, alvrl_gather_rec *out);

/* The same records on the current HIP device (Sensor::sampleRay +
 * Scene::rayIntersect through the occluder BVH: the GPU eye-ray first hit),
 * bit-identical to alvrl_scene_records.  d_pixel_ids: device array (NULL:
 * pixels 0..n-1); d_out: n device records, written on 'stream' (NULL: the
 * null stream); returns after they are written. */
ALVRL_API int alvrl_scene_records_gpu(const alvrl_scene_desc *s, int medium_scatters, const uint32_t *d_pixel_ids,
                                      uint32_t n, alvrl_gather_rec *d_out, void *stream);
/* LiInternal's eye path of pixel (x, y) (vrlIntegrator.cpp:398-524): the
 * record of the first hit, then, while the hit surface has a delta BSDF
 * (mirror, null) and the segment's transmittance is non-zero, the specular
 * chain's next hit (bsdf->sample(bRec, Point2(0.5)), :470-476) with Russian
 * roulette on throughputWithEtaSq = init_throughput * ... (:480-492; maxRR
 * 0.98 from depth spec_rr_depth on), drawing from the (seed, pass, pixel,
 * depth) eye stream.  Record k carries depth k and the path weight
 * prod transmittance * bsdfWeight / rrProb (:505).  The gather adds every
 * record's weighted contribution to its pixel.  *n = records (<= cap, at
 * most 256); ALVRL_ERR_INVALID if cap is too small. */
ALVRL_API int alvrl_scene_chain(const alvrl_scene_desc *s, int medium_scatters, uint32_t seed, uint32_t pass,
                                int spec_rr_depth, float init_throughput, int x, int y, alvrl_gather_rec *out,
                                uint32_t cap, uint32_t *n);
/* Multi-sample renders (renderBlock's sample loop, integrator.cpp:240-264):
 * sensor sample j of spp is the pixel centre when spp == 1, else (x, y) +
 * rRec.nextSample2D(), drawn from the counter stream (seed, pass, dom 8,
 * pixel, j).  A record's depth word carries j in bits 16-31, and the gathers
 * key their streams by it (bits 0-15 of the stream word), so sample 0 gives
 * the single-sample records and contributions.  alvrl_scene_records_spp:
 * n * spp records, sample major (record j * n + i = pixel_ids[i], sample j).
 * alvrl_scene_chain_spp: alvrl_scene_chain's eye path from sensor sample j
 * (record k's depth word k | (j << 16); its roulette draws from (pixel,
 * k | (j << 16))).  spp <= 65535. */
ALVRL_API int alvrl_scene_records_spp(const alvrl_scene_desc *s, int medium_scatters, uint32_t seed, uint32_t pass,
                                      uint32_t spp, const uint32_t *pixel_ids, uint32_t n, alvrl_gather_rec *out);
ALVRL_API int alvrl_scene_records_spp_gpu(const alvrl_scene_desc *s, int medium_scatters, uint32_t seed,
                                          uint32_t pass, uint32_t spp, const uint32_t *d_pixel_ids, uint32_t n,
                                          alvrl_gather_rec *d_out, void *stream);
ALVRL_API int alvrl_scene_chain_spp(const alvrl_scene_desc *s, int medium_scatters, uint32_t seed, uint32_t pass,
                                    int spec_rr_depth, float init_throughput, int x, int y, uint32_t sample,
                                    uint32_t spp, alvrl_gather_rec *out, uint32_t cap, uint32_t *n);
/* The slicing record of pixel (x, y) (buildSlices, Preprocessor.cpp:1140-1170):
 * the first hit that is not a null surface; HIT flag, position and normal. */
ALVRL_API int alvrl_scene_slice_record(const alvrl_scene_desc *s, int x, int y, alvrl_gather_rec *out);

/* ---- reference integrator: volpath with onlyVRLpaths --------------------
 * VolumetricPathTracer::Li (src/integrators/path/volpath.cpp:110-457) on the
 * current HIP device: the path-traced ground truth of exactly the light
 * transport the VRLs represent (eye -> volume or diffuse surface -> volume
 * -> light path), for statistical checks of the VRL method (SURVEY 8(f)
 * row 4).  Pixel centres, isotropic phase; counter-RNG stream (seed, pass,
 * pixel id, sample).  d_out_rgb: 3 floats per pixel, the mean over spp. */
typedef struct {
    int max_depth;        /* maxDepth (-1: unbounded) */
    int rr_depth;         /* rrDepth (5) */
    int only_vrl_paths;   /* onlyVRLpaths (1) */
    int vrl_vol_to_vol;   /* vrlVolToVol (1) */
    int vrl_vol_to_surf;  /* vrlVolToSurf (1) */
} alvrl_volpath_params;
ALVRL_API void alvrl_volpath_default(alvrl_volpath_params *p);
ALVRL_API int alvrl_volpath_render(const alvrl_scene_desc *s, const alvrl_volpath_params *p, uint32_t seed,
                                   uint32_t pass, uint32_t spp, const uint32_t *d_pixel_ids, uint32_t n,
                                   float *d_out_rgb, void *stream);
/* Multi-GPU image partition of alvrl_integrator_render: 64x64 tiles in
 * row-major tile order, tile t owned by rank t % world (the
 * reference's analogue is the block scheduler handing 32x32 blocks to workers,
 * blockedrenderprocess.cpp).  Writes the owned pixel ids (row-major y*W+x,
 * tile by tile, rows within a tile) to out if out != NULL and cap suffices;
 * *n = count.  ALVRL_ERR_INVALID for world == 0, rank >= world or cap < count. */
ALVRL_API int alvrl_tile_pixels(int width, int height, uint32_t rank, uint32_t world,
                                uint32_t *out, uint32_t cap, uint32_t *n);

/* vrlTracer::randomWalk (vrlTracer.h:13-52).  soa receives 9 planes of
 * stride 'cap'; *n = #VRLs (>= target unless cap is hit), *particles =
 * particleCount.  Returns ALVRL_ERR_INVALID if cap < the VRLs produced. */
ALVRL_API int alvrl_trace_vrls(const alvrl_scene_desc *s, uint32_t seed, uint32_t pass,
                               uint32_t target, int short_vrls, int max_depth, int rr_depth,
                               float *soa, uint32_t cap, uint32_t *n, uint64_t *particles);
/* The same walk on the current HIP device (csrc/tracer.hip, SURVEY 8(f) row
 * 2): one lane per particle, bit-identical VRL set and particle count.
 * soa == NULL: size query (*n, *particles). */
ALVRL_API int alvrl_trace_vrls_gpu(const alvrl_scene_desc *s, uint32_t seed, uint32_t pass,
                                   uint32_t target, int short_vrls, int max_depth, int rr_depth,
                                   float *soa, uint32_t cap, uint32_t *n, uint64_t *particles);

/* vrlVector(Stream*, const Medium*) (VRL.h:120-128) / a separator-correct
 * serializeAscii (VRL.h:65-73). */
ALVRL_API int alvrl_read_vrl_file(const char *path, const alvrl_medium_desc *m, float *soa,
                                  uint32_t cap, uint32_t *n, uint64_t *particles);
ALVRL_API int alvrl_write_vrl_file(const char *path, const float *soa, uint32_t n);

/* Message of the last failing alvrl_scene_* / alvrl_trace_* / alvrl_*_vrl_file /
 * alvrl_integrator_* call on this thread. */
ALVRL_API const char *alvrl_host_last_error(void);

/* ---- vrl integrator pipeline (vrlIntegrator.cpp) ---------------------- */
typedef struct alvrl_integrator alvrl_integrator;

/* props: "name=value" pairs separated by ';' with the reference's parameter
 * names and defaults (vrlIntegrator.cpp:128-208, integrator.cpp:272-277, 348-349),
 * plus "seed" (counter-RNG key) and "vrlSeed" (tracer key). */
ALVRL_API int alvrl_integrator_create(const char *props, int device, alvrl_integrator **out);
ALVRL_API void alvrl_integrator_destroy(alvrl_integrator *it);
/* vrlIntegrator::preprocess (:237-267): scene, optional vrlFile, buildSlices. */
ALVRL_API int alvrl_integrator_preprocess(alvrl_integrator *it, const alvrl_scene_desc *s);
/* vrlIntegrator::prepass (:270-356) for pass 'pass' (0-based): trace or reuse
 * VRLs, sample representatives, build R, cluster, upload cluster info.
 * Every slice on this GPU (see alvrl_integrator_prepass_dist for the
 * slice-sharded form). */
ALVRL_API int alvrl_integrator_prepass(alvrl_integrator *it, uint32_t pass);
/* SamplingIntegrator::render for the pixels this rank owns: 64x64 tiles dealt
 * round-robin (tile t -> rank t % world).  Adds Li of every owned pixel into
 * d_framebuffer (device, W*H*3 floats, row-major) on 'stream' (NULL: the
 * integrator's stream, ordered after the work already queued on the null
 * stream, e.g. the caller's zero fill of d_framebuffer). */
ALVRL_API int alvrl_integrator_render(alvrl_integrator *it, uint32_t rank, uint32_t world,
                                      float *d_framebuffer, void *stream);
/* Preloaded VRLs (the vrlFile mode, :243-252 / :280-287): every pass reuses
 * this set instead of tracing; soa = 9 planes of stride n. */
ALVRL_API int alvrl_integrator_set_vrls(alvrl_integrator *it, const float *soa, uint32_t n,
                                        uint64_t particle_count);
/* ---- multi-GPU prepass ------------------------------------
 * The one collective the slice-sharded prepass needs, supplied by the
 * caller's communicator (RCCL through torch.distributed, MPI, ...): every
 * rank passes the same 'bytes' and receives world * bytes in rank order.
 * Returns 0 on success; anything else aborts the prepass with ALVRL_ERR_COMM. */
typedef struct {
    void *user;
    int (*allgather)(void *user, const void *send, uint64_t bytes, void *recv);
} alvrl_exchange;

/* vrlIntegrator::prepass with the LightSlice work sharded by slice: rank r
 * builds R for, and refines, its share of the slices (plus the rows of their
 * neighbour slices when neighbourCount > 0): by default the longest-
 * processing-time assignment on the slices' local-matrix rows (every rank
 * derives the same one; alvrl_integrator_local_slices lists this rank's),
 * s % world == r with the property sliceSharding=roundrobin; the non-zero VRL mask
 * of Preprocessor::cluster (:843-855) is OR-reduced over ranks, and the
 * per-slice cluster lists are all-gathered so every rank can render any
 * tile.  Results are identical to alvrl_integrator_prepass on one GPU.  The
 * fall-back clustering (needed only if a slice fails to refine or a pixel
 * has no slice) is computed by every rank over all rows.  world == 1 (ex
 * may be NULL) is alvrl_integrator_prepass. */
ALVRL_API int alvrl_integrator_prepass_dist(alvrl_integrator *it, uint32_t pass, uint32_t rank,
                                            uint32_t world, const alvrl_exchange *ex);

/* Building blocks of the exchange, exported for hosts that orchestrate the
 * prepass themselves and for the CPU tests.
 * Variable-size all-gather: counts[r] = bytes of rank r; with recv != NULL
 * (cap bytes) rank r's data lands at recv + sum(counts[<r]).  Call with
 * recv == NULL first to learn the counts. */
ALVRL_API int alvrl_exchange_allgatherv(const alvrl_exchange *ex, uint32_t world, const void *send,
                                        uint64_t bytes, void *recv, uint64_t cap, uint64_t *counts);
/* Element-wise OR of n bytes over ranks, in place. */
ALVRL_API int alvrl_exchange_or(const alvrl_exchange *ex, uint32_t world, uint8_t *buf, uint64_t n);
/* Merge per-slice cluster lists: this rank holds n_local slices (ids
 * local_slice[], refined flags, CSR local_off/local_reps/local_w); the
 * output is the CSR over all nslices slices (a slice no rank reports gets
 * refined = 0 and no clusters).  *total = clusters of all slices; returns
 * ALVRL_ERR_INVALID if cap is smaller (call again with a larger buffer). */
ALVRL_API int alvrl_exchange_clusters(const alvrl_exchange *ex, uint32_t world, uint32_t nslices,
                                      uint32_t n_local, const uint32_t *local_slice,
                                      const int *local_refined, const uint32_t *local_off,
                                      const uint32_t *local_reps, const float *local_w,
                                      int *refined, uint32_t *slice_off, uint32_t *reps,
                                      float *weights, uint64_t cap, uint64_t *total);

/* An alvrl_exchange whose ranks are threads of this process -- one library
 * integrator per GPU driven from one host thread each (the Mitsuba plugin's
 * amdDevices; the reference renders in one process with one worker per core,
 * src/mitsuba/mitsuba.cpp:280-282, src/librender/renderproc.cpp:119-135).
 * Rank r's exchange is alvrl_local_exchange_rank(g, r); all ranks must call
 * the collectives in the same order.  A rank left waiting 600 s fails the
 * call with ALVRL_ERR_COMM instead of hanging.  Destroy after every rank has
 * returned. */
typedef struct alvrl_local_exchange alvrl_local_exchange;
ALVRL_API int alvrl_local_exchange_create(uint32_t world, alvrl_local_exchange **out);
ALVRL_API const alvrl_exchange *alvrl_local_exchange_rank(alvrl_local_exchange *g, uint32_t rank);
ALVRL_API void alvrl_local_exchange_destroy(alvrl_local_exchange *g);
/* Mark the group broken: every rank waiting in a collective, or arriving at
 * one later, fails it with ALVRL_ERR_COMM at once.  A rank whose prepass
 * failed before its collective calls this so its peers do not wait for the
 * timeout; the group is not reused afterwards. */
ALVRL_API void alvrl_local_exchange_abort(alvrl_local_exchange *g);

/* The same in-process ranks over RCCL: one communicator per device
 * (ncclCommInitAll over devices[0..world), which must be distinct), so the
 * prepass's collective moves device to device over xGMI -- rank r's
 * alvrl_exchange stages its bytes on devices[r] and runs ncclAllGather -- and
 * the frame's tiles are summed on the devices: alvrl_device_exchange_reduce_frame
 * is one ncclReduce (sum, in place) of every rank's n-float framebuffer into
 * rank 0's on 'stream' (NULL: the rank's own), which a single D2H copy then
 * hands to the host (north_star's "single RCCL gather of the framebuffer").
 * Every rank calls it, each from its own thread.  The multi-GPU form of
 * Mitsuba's one-process rendering (renderproc.cpp:142-160). */
typedef struct alvrl_device_exchange alvrl_device_exchange;
ALVRL_API int alvrl_device_exchange_create(const int *devices, uint32_t world, alvrl_device_exchange **out);
ALVRL_API const alvrl_exchange *alvrl_device_exchange_rank(alvrl_device_exchange *g, uint32_t rank);
ALVRL_API int alvrl_device_exchange_reduce_frame(alvrl_device_exchange *g, uint32_t rank, float *d_fb, uint64_t n,
                                                 void *stream);
ALVRL_API void alvrl_device_exchange_destroy(alvrl_device_exchange *g);
/* ncclCommAbort on every rank's communicator: collectives in flight or
 * started later fail instead of waiting for a rank that will not join; the
 * group is not reused afterwards (destroy it). */
ALVRL_API void alvrl_device_exchange_abort(alvrl_device_exchange *g);

/* ---- host-cast scenes (the Mitsuba plugin's "records" mode) ------------
 * For scenes the descriptor above cannot express -- area and other emitters,
 * any shapes and BSDFs, a medium in any container -- the host application
 * casts every eye ray with its own scene; the library keeps the per-pair work
 * (R, the clustering and the gathers) and the VRLs: it traces them per pass
 * itself over a descriptor of the scene's light transport (`tracer` below:
 * vrlTracer.h:91-230 restated, on the device with the integrator property
 * gpuTracer), or they come from vrlFile, or the host sets them with
 * alvrl_integrator_set_vrls before each prepass.
 *
 *   preprocess  alvrl_integrator_preprocess_ext: buildSlices
 *               (Preprocessor.cpp:1130-1193) over the host's gather point of
 *               every pixel centre ray (null surfaces passed, :1157-1169);
 *   prepass     alvrl_integrator_rep_pixels (sampleSliceMapping of the pass,
 *               :1502-1525) -> the host casts each representative pixel's
 *               eye path (sensor->sampleRay at the pixel centre, :327-328;
 *               LiInternal's delta-BSDF chains, :445-511, one record per
 *               segment with its path weight) -> alvrl_integrator_prepass_records
 *               (R rows, buildClusters, cluster lists; slice-sharded with
 *               world > 1 as alvrl_integrator_prepass_dist);
 *   render      the host's eye records through alvrl_gather_clustered_host /
 *               alvrl_gather_brute_host on alvrl_integrator_ctx (slice of a
 *               pixel: alvrl_integrator_slices); alvrl_integrator_render is
 *               refused (it casts the descriptor's camera rays). */
typedef struct {
    int width, height;
    float scene_min[3], scene_max[3];   /* Scene::getAABB(): buildSlices' direction scale (:1137) */
    alvrl_medium_desc medium;           /* the homogeneous medium the VRLs live in */
    /* W*H records, row-major (y*W + x): the gather point of the ray through
     * the pixel centre -- ALVRL_REC_HIT, p and the shading normal; no HIT
     * flag for a ray that leaves the scene (the pixel gets no slice).
     * NULL: no slicing -- a render worker that receives its slices and
     * cluster lists through alvrl_integrator_set_cluster_info (wakeup,
     * vrlIntegrator.cpp:378-384); such an integrator cannot run a prepass. */
    const alvrl_gather_rec *slice_recs;
    /* every triangle of the scene, 9 floats each, for the gathers' occluder
     * test (Scene::evalTransmittance, scene.cpp:619-679); ALVRL_MAT_NULL
     * triangles let a shadow segment pass (NULL material list: all block) */
    const float *triangles;
    uint32_t n_triangles;
    const uint32_t *triangle_material;
    /* The VRL tracer's scene (NULL: the VRLs come from vrlFile or
     * alvrl_integrator_set_vrls): its medium container (box_min / box_max,
     * albedo), occluders with materials, the point light or area emitter
     * (camera fields unused).  Copied by alvrl_integrator_preprocess_ext; each
     * prepass then traces the pass's VRLs over it (seed vrlSeed, the pass,
     * vrlTargetNum, shortVrls, maxParticleDepth, rrDepth), on the device with
     * gpuTracer=true, exactly as alvrl_integrator_prepass does for a
     * descriptor scene. */
    const alvrl_scene_desc *tracer;
} alvrl_scene_ext;

ALVRL_API int alvrl_integrator_preprocess_ext(alvrl_integrator *it, const alvrl_scene_ext *s);
/* The representative pixels of pass 'pass' in R-row order (row-major pixel
 * ids y*W + x): rows rep_off[s]..rep_off[s+1] of alvrl_integrator_reps are
 * slice s's.  cap may be 0 with pixel_ids NULL to learn *n. */
ALVRL_API int alvrl_integrator_rep_pixels(alvrl_integrator *it, uint32_t pass, uint32_t *pixel_ids, uint32_t cap,
                                          uint32_t *n);
/* The prepass of pass 'pass' over the host's records: recs[i] belongs to R
 * row row_of_rec[i] (the index into alvrl_integrator_rep_pixels' list); a
 * row's records are its eye path's segments in LiInternal's order and add
 * into the row (getLiLuminanceVrlContributions, :527-539, 812-813); a row
 * without records (its ray left the scene) is zero.  Each record's gathers
 * draw from the counter streams of the row's pixel id.  world > 1: this rank
 * builds and refines slices s % world == rank only (ex as in
 * alvrl_integrator_prepass_dist; world == 1 may pass NULL). */
ALVRL_API int alvrl_integrator_prepass_records(alvrl_integrator *it, uint32_t pass, const alvrl_gather_rec *recs,
                                               const uint32_t *row_of_rec, uint32_t n, uint32_t rank,
                                               uint32_t world, const alvrl_exchange *ex);
/* The vrlClusterInfo resource in memory (bindUsedResources / wakeup,
 * vrlIntegrator.cpp:371-384: a render worker receives m_vrls and m_ci
 * instead of running the prepass): the pass's VRLs are set or traced as a
 * prepass would, then these lists are installed.  Same arrays as
 * alvrl_cluster_info_write; npix must be the scene's pixel count. */
ALVRL_API int alvrl_integrator_set_cluster_info(alvrl_integrator *it, uint32_t pass, uint32_t npix,
                                                const uint32_t *pixel_to_slice, uint32_t nslices,
                                                const uint32_t *slice_off, const uint32_t *reps,
                                                const float *weights, uint32_t n_fb, const uint32_t *fb_reps,
                                                const float *fb_weights);

/* Timing / statistics of the last prepass and render. */
typedef struct {
    uint64_t vrls, particles, slices, rep_rows, clusters_total;
    uint64_t contrib_preprocess, contrib_render;
    double ms_trace, ms_slices, ms_rbuild, ms_refine, ms_render_kernel, ms_prepass_wall;
    uint32_t slices_failed;
    int fallback_built;
    /* slices this rank refined and R rows it built (all of them at world 1),
     * and the host time spent in the exchange of the last prepass */
    uint64_t slices_local, rows_built;
    double ms_exchange;
    /* device time of the last prepass's refinement and R-build kernels (HIP
     * events) and the R entries its refinement read (alvrl_last_refine_entries) */
    double ms_refine_kernel;
    uint64_t refine_entries;
    uint64_t global_clusters;   /* clusters of the globalCluster refinement (0 if off) */
    uint64_t refine_split_entries;   /* the splits' share of refine_entries (alvrl_last_refine_split_entries) */
    /* host wall time of the last prepass's device allocations (R and its row
     * tables grown with hipMalloc; zero once they are large enough) */
    double ms_alloc;
} alvrl_integrator_stats;
ALVRL_API int alvrl_integrator_get_stats(alvrl_integrator *it, alvrl_integrator_stats *st);
/* The device context the integrator drives (for low-level access). */
ALVRL_API alvrl_ctx *alvrl_integrator_ctx(alvrl_integrator *it);
/* Copies of host-side state for tests: pixel->slice map (column-major,
 * y + H*x, vrlIntegrator.cpp:560), representative rows, cluster CSR. */
ALVRL_API int alvrl_integrator_slices(alvrl_integrator *it, uint32_t *pixel_to_slice, uint32_t n);
ALVRL_API uint32_t alvrl_integrator_num_slices(alvrl_integrator *it);
/* The slices the last prepass refined on this integrator, ascending (all of
 * them at world 1).  out may be NULL to learn *n. */
ALVRL_API int alvrl_integrator_local_slices(alvrl_integrator *it, uint32_t *out, uint32_t cap, uint32_t *n);
ALVRL_API int alvrl_integrator_reps(alvrl_integrator *it, uint32_t *rep_off, uint32_t *rep_pix,
                                    uint32_t cap);
ALVRL_API int alvrl_integrator_clusters(alvrl_integrator *it, uint32_t *slice_off, uint32_t *reps,
                                        float *weights, uint32_t cap, uint32_t *fb_reps,
                                        float *fb_weights, uint32_t fb_cap, uint32_t *n_fb);
/* R of the last prepass, [nvrl][rep_rows] (mean, var) pairs (host copy). */
ALVRL_API int alvrl_integrator_R(alvrl_integrator *it, float *out, uint64_t cap_floats);
ALVRL_API int alvrl_integrator_vrls(alvrl_integrator *it, float *soa, uint32_t cap, uint32_t *n,
                                    uint64_t *particles);
/* The clustering job of slice s in the last prepass, as refineSlice hands it
 * to a Clustering (Preprocessor.cpp:254-283; getLocalMatrix :779-827;
 * initial clusters of cluster() :838-898): the local matrix [nvrl][nrows]
 * (mean, var) pairs (R may be null), locality weights, the slice's pixel
 * undersampling and the initial clusters (init_vrls: nvrl ids, init_off:
 * ninit + 1 offsets).  Null output buffers are skipped; *nrows and *ninit
 * are always set.  For checking the device refinement of one slice. */
ALVRL_API int alvrl_integrator_slice_job(alvrl_integrator *it, uint32_t s, float *R, double *locw,
                                         uint32_t cap_rows, uint32_t *nrows, float *pixel_under,
                                         uint32_t *init_vrls, uint32_t *init_off, uint32_t *ninit);

/* ---- on-disk formats -------------------------------
 * vrlClusterInfo stream (vrlIntegrator.cpp:29-101, the resource the
 * reference ships to remote render workers): ULong counts, UInt ids, Float
 * weights, little-endian.  pixel_to_slice is m_slices (y + H*x); per-slice
 * lists as CSR (slice_off has nslices + 1 entries); the global-cluster and
 * fall-back lists.  The reader fixes the reference's slip at :56-59 (the
 * fall-back ids go to the id list, not the weights). */
typedef struct alvrl_cluster_info alvrl_cluster_info;
ALVRL_API int alvrl_cluster_info_write(const char *path, uint32_t npix, const uint32_t *pixel_to_slice,
                                       uint32_t nslices, const uint32_t *slice_off, const uint32_t *reps,
                                       const float *weights, uint32_t n_global, const uint32_t *global_reps,
                                       const float *global_w, uint32_t n_fb, const uint32_t *fb_reps,
                                       const float *fb_w);
ALVRL_API int alvrl_cluster_info_read(const char *path, alvrl_cluster_info **out);
ALVRL_API void alvrl_cluster_info_free(alvrl_cluster_info *ci);
ALVRL_API int alvrl_cluster_info_sizes(const alvrl_cluster_info *ci, uint32_t *npix, uint32_t *nslices,
                                       uint32_t *nreps, uint32_t *n_global, uint32_t *n_fb);
/* any output may be NULL; sizes from alvrl_cluster_info_sizes */
ALVRL_API int alvrl_cluster_info_get(const alvrl_cluster_info *ci, uint32_t *pixel_to_slice,
                                     uint32_t *slice_off, uint32_t *reps, float *weights,
                                     uint32_t *global_reps, float *global_w, uint32_t *fb_reps, float *fb_w);
/* The integrator's cluster info after prepass, to a file; and the reverse:
 * install a saved one for pass 'pass' (VRLs traced or reused as prepass
 * would, no R build or refinement), as a remote worker renders with the
 * m_ci it receives.  The file's pixel count must match the scene. */
ALVRL_API int alvrl_integrator_save_cluster_info(alvrl_integrator *it, const char *path);
ALVRL_API int alvrl_integrator_load_cluster_info(alvrl_integrator *it, const char *path, uint32_t pass);

/* Single-part scanline OpenEXR, no compression, channels B/G/R, FLOAT
 * (half = 0) or HALF (half = 1) -- the hdrfilm output of a pass; rgb is
 * row-major W*H*3.  The reader takes files of this layout (rgb == NULL:
 * size query). */
ALVRL_API int alvrl_write_exr(const char *path, const float *rgb, int width, int height, int half);
ALVRL_API int alvrl_read_exr(const char *path, float *rgb, uint64_t cap_floats, int *width, int *height);
/* mtsutil rms (src/utils/rms.cpp:36-110): gamma, robust fraction dropped at
 * both ends of the sorted deviations, relative = deviations / reference
 * (zero-reference entries masked). */
ALVRL_API int alvrl_image_rms(const float *sample, const float *reference, uint64_t n, double gamma,
                              double robust_fraction, int relative, double *out);
/* dumpPass file name (integrator.cpp:361-378) with the vrl integrator's
 * passFileSuffix (vrlIntegrator.cpp:357-364) and hdrfilm's ".exr". */
ALVRL_API int alvrl_pass_file_name(char *out, uint64_t cap, const char *dest, int pass, double prepass_cpu,
                                   double prepass_wall, double render_cpu, double render_wall,
                                   double vrls_preprocess, double vrls_render);

#ifdef __cplusplus
}
#endif
#endif /* ALVRL_HOST_H */
