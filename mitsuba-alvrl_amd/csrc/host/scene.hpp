// scene.hpp -- standalone smoke-box scene: the minimal stand-in for the parts
// of Mitsuba's Scene / Sensor / Shape / Emitter that the vrl integrator calls
// (out of scope per SURVEY.md 2; restated only as far as the benchmark scene
// needs them):
//   perspective pinhole  src/sensors/perspective.cpp:126-155, 247-269
//   ray / box walls      one-sided diffuse walls of an axis-aligned box, seen
//                        from inside
//   occluders            optional triangles inside the box (a TriMesh with a
//                        one-sided diffuse BSDF): TriangleT::rayIntersect
//                        (include/mitsuba/core/triangle.h:109-145), the hit
//                        record of skdtree.h:350-396, and the visibility
//                        part of Scene::evalTransmittance (scene.cpp:619-679);
//                        without them every interior pair is mutually visible
//   point light          src/emitters/point.cpp:81-106
//   homogeneous fog      src/medium/homogeneous.cpp (balance / single /
//                        manual / maximum distance sampling)
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace alvrl {
namespace host {

struct V3 { float x, y, z; };

// words of a gather record (alvrl_gather_rec): o, d, p, n, albedo, flags,
// path weight (3), eye-path depth
constexpr int kRecWords = 20;

inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
inline V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
float dot(V3 a, V3 b);
float length(V3 a);
V3 normalize(V3 a);
V3 cross(V3 a, V3 b);

struct MediumParams {
    float sigma_s[3] = {0.8f, 0.6f, 0.4f};
    float sigma_a[3] = {0.05f, 0.05f, 0.05f};
    float sigma_t[3] = {0.85f, 0.65f, 0.45f};
    float sampling_weight = -1.0f;   // resolved by resolve()
    int phase_type = 0;              // 0 isotropic, 1 HG
    float phase_g = 0.0f;
    int strategy = 0;                // ALVRL_STRATEGY_* (homogeneous.cpp:150-227)
    int channel = 0;                 // 'single': 1 + channel (0: the smallest sigma_t)
    float density = 0.0f;            // 'manual': samplingDensity; after resolve() m_samplingDensity
    // MaxExpDist (maxexp.h:28-94) after resolve(): sigma_t sorted decreasingly,
    // the normalised CDF at the interval starts, the starts, the lower terms
    float mx_sigma[3] = {0, 0, 0}, mx_cdf[4] = {0, 0, 0, 0}, mx_start[3] = {0, 0, 0}, mx_lower[3] = {0, 0, 0};
    float mx_norm = 0.0f, mx_inv_norm = 0.0f;
    const char* problem() const;     // what resolve() cannot accept, or nullptr
    void resolve();                  // sigma_t, the auto sampling weight (:168-184), the strategy's terms
    // sampleDistance's pdfs at the distance used (:317-346), the sampling weight
    // applied; pdf_max: MaxExpDist::sample's pdf ('maximum')
    void pdfs(float sampled, float pdf_max, float* ps, float* pf) const;
    float maxexp_sample(float u, float* pdf) const;   // maxexp.h:59-73
    float maxexp_cdf(float t) const;                  // maxexp.h:83-94
};

struct SmokeBox {
    V3 cam_origin = v3(0.0f, 0.0f, -0.9f);
    V3 cam_target = v3(0.0f, 0.0f, 1.0f);
    V3 cam_up = v3(0.0f, 1.0f, 0.0f);
    float fov_x_deg = 60.0f;
    int width = 1024, height = 1024;
    float box_min[3] = {-1.0f, -1.0f, -1.0f};
    float box_max[3] = {1.0f, 1.0f, 1.0f};
    float albedo[3] = {0.5f, 0.5f, 0.5f};
    V3 light_pos = v3(0.0f, 0.8f, 0.0f);
    float light_intensity[3] = {10.0f, 10.0f, 10.0f};
    MediumParams medium;
    std::vector<float> occ;           // occluder triangles, 9 floats each (p0, p1, p2)
    float occ_albedo[3] = {0.5f, 0.5f, 0.5f};
    std::vector<float> occ_alb;       // per triangle reflectance, 3 floats each (empty: occ_albedo for all)
    const float* occ_albedo_of(int tri) const { return occ_alb.empty() ? occ_albedo : &occ_alb[3 * (size_t)tri]; }
    std::vector<uint32_t> occ_mat;    // per triangle ALVRL_MAT_* (empty: all diffuse)
    float occ_spec[3] = {1.0f, 1.0f, 1.0f};
    // dielectric triangles: m_eta = intIOR / extIOR (dielectric.cpp:149-158; bk7 / air, ior.h:43, 60)
    float occ_eta = 1.5046f / 1.000277f;
    // area emitter (alvrl_scene_desc::emitter_tris): triangles, radiance, and
    // TriMesh's sampling table (prepare_emitter): the normalized area CDF of
    // DiscreteDistribution (pmf.h:101-114) and the surface area
    std::vector<float> emit;
    float emit_radiance[3] = {0.0f, 0.0f, 0.0f};
    std::vector<float> emit_cdf;
    float emit_area = 0.0f;
    bool area_light() const { return !emit.empty(); }
    void prepare_emitter();
    // Scene::sampleEmitterPosition + Emitter::sampleDirection of the area
    // emitter for the tracer's draws (sx, sy) and (dx, dy): origin, direction
    // and power (vrlTracer.h:109-120)
    void sample_area_emission(float sx, float sy, float dx, float dy, V3* o, V3* d, float power[3]) const;
    // the BSDF of a hit: 0 diffuse (walls: tri < 0), 1 mirror, 2 null, 3 dielectric
    uint32_t mat(int tri) const { return (tri < 0 || occ_mat.empty()) ? 0u : occ_mat[(size_t)tri]; }
    bool has_delta() const
    {
        for (uint32_t m : occ_mat) if (m != 0u) return true;
        return false;
    }

    // Sensor::sampleRay through pixel sample (px, py); *mint = nearClip / d.z
    // in camera space (perspective.cpp:247-263, nearClip 1e-2).
    void camera_ray(float px, float py, V3* o, V3* d, float* mint = nullptr) const;
    // First hit of a ray starting inside the box: t and inward normal.
    float box_hit(V3 o, V3 d, V3* n) const;
    // Scene::rayIntersect over the walls and the occluders, t >= mint; the
    // walls win ties, then the lowest triangle index.  *tri = -1 for a wall;
    // *p = its.p (ray(t) for a wall, barycentric for a triangle).
    float first_hit(V3 o, V3 d, float mint, V3* n, V3* p, int* tri) const;
    // The occluder part of Scene::evalTransmittance(p1, p1OnSurface, p2,
    // p2OnSurface): false if a triangle lies on the segment (the walls
    // cannot: both points are inside the box); null triangles let it pass.
    bool visible(V3 p1, bool p1_surface, V3 p2, bool p2_surface) const;
    // The eye path of pixel centre (x, y) through delta BSDFs: LiInternal's
    // recursion (vrlIntegrator.cpp:386-524) as gather records, one per
    // segment, each with the weight the recursion passes down (:503-510).
    // A delta BSDF's every delta component is followed (bRec.component = i,
    // :467-511): a dielectric branches into reflection and transmission, so
    // the records form a tree, emitted depth first (component 0's subtree
    // before component 1's).  Record k (pre-order index, = its depth on a
    // path without branches) has depth word k | (j << 16) for sensor sample j
    // of spp (pixel_sample); the Russian roulette of its components (from
    // initialSpecularThroughput, maxRR 0.98 past specularForcedRRdepth,
    // :475-492) draws in component order from the stream (seed, pass, dom 7,
    // pixel, k | (j << 16)).  Appends kRecWords floats per record (<= 256).
    void make_chain(int x, int y, bool medium_scatters, uint32_t seed, uint32_t pass, int spec_rr_depth,
                    float init_throughput, std::vector<float>* out, uint32_t sample = 0, uint32_t spp = 1) const;
    // buildSlices' gather point of pixel (x, y) (Preprocessor.cpp:1144-1170):
    // the camera ray's first hit, continued through null surfaces; a record
    // with the hit flag, position and normal of that point.
    void make_slice_record(int x, int y, float rec[kRecWords]) const;
    uint32_t n_occ() const { return (uint32_t)(occ.size() / 9); }
    // The sensor sample of pixel (x, y), sample j of spp (renderBlock,
    // integrator.cpp:240-247): the pixel centre for one sample per pixel,
    // else (x, y) + rRec.nextSample2D(), here draws 0 and 1 of the stream
    // (seed, pass, dom 8, pixel, j).
    void pixel_sample(int x, int y, uint32_t seed, uint32_t pass, uint32_t sample, uint32_t spp, float* px,
                      float* py) const;
    // Gather record (alvrl_gather_rec layout) of pixel centre (x, y), or of
    // its sensor sample j of spp; the depth word carries j in bits 16-31.
    void make_record(int x, int y, bool medium_scatters, float rec[kRecWords], uint32_t seed = 0,
                     uint32_t pass = 0, uint32_t sample = 0, uint32_t spp = 1) const;
    float scene_diagonal() const;   // distance(getAABB().min, getAABB().max)

private:
    void chain_node(V3 O, V3 D, float mint, const float weight[3], const float thr[3], int depth, uint32_t pixel,
                    uint32_t sample, bool medium_scatters, uint32_t seed, uint32_t pass, int spec_rr_depth,
                    std::vector<float>* out, uint32_t* k) const;
};

// fresnelDielectricExt (src/libcore/util.cpp:651-681): unpolarized Fresnel
// reflectance and the signed cosine of the transmitted direction.
float fresnel_dielectric_ext(float cos_theta_i, float* cos_theta_t, float eta);

// TriangleT::rayIntersect (triangle.h:109-145): t of the hit, or false.
bool tri_intersect(const float* tri, V3 o, V3 d, float* u, float* v, float* t);

// vrlVector: SoA planes (start xyz, end xyz, power rgb), VRL.h:105-194.
struct VrlSet {
    std::vector<float> soa;   // 9 * n, plane stride n
    uint32_t n = 0;
    uint64_t particle_count = 0;
};

// vrlTracer::randomWalk (vrlTracer.h:13-230) in the smoke box, with the
// counter-based stream (seed, pass, particle index) instead of one sequential
// sampler, so the VRL set does not depend on how particles are scheduled.
VrlSet trace_vrls(const SmokeBox& s, uint32_t seed, uint32_t pass, uint32_t target, bool short_vrls,
                  int max_depth, int rr_depth);

// ASCII VRL file I/O: one VRL per line "sx sy sz ex ey ez r g b"
// (VRL.h:43-54 reader, vrlVector(Stream*, Medium*) :120-128).  particleCount =
// number of lines that pass the put-filter.  The writer separates fields with
// spaces (the reference's serializeAscii, VRL.h:65-73, writes none and cannot
// be read back).
bool read_vrl_file(const char* path, const MediumParams& m, VrlSet* out, std::string* err);
bool write_vrl_file(const char* path, const VrlSet& v, std::string* err);

}  // namespace host
}  // namespace alvrl
