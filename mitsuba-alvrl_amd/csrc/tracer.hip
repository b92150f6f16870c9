// tracer.hip -- vrlTracer::randomWalk (vrlTracer.h:13-230) on the GPU,
// SURVEY.md 8(f) row 2.  One lane per particle: particle p draws from its own
// counter-based stream (seed, pass, p), exactly as the host tracer
// (csrc/host/scene.cpp trace_particle) and the oracle do, so the VRL set is
// the host's bit for bit.  Built with -ffp-contract=off and IEEE division /
// square root like the host; sin, cos, exp and log are evaluated in double
// and rounded once, as on the host.
//
// Two passes per batch of particles: count each particle's VRLs, then (after
// a prefix sum on the host picks the particles the sequential loop would have
// traced -- it stops after the particle that brings the set to the target)
// write them at their final positions in the SoA planes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "alvrl_host.h"
#include "bvh_device.hpp"
#include "host/bvh.hpp"
#include "host/scene.hpp"
#include "detmath.h"

namespace alvrl {
namespace host {
extern thread_local std::string g_host_err;
SmokeBox to_box(const alvrl_scene_desc& s);   // host_capi.cpp
const char* scene_problem(const alvrl_scene_desc& s);
}
}  // namespace alvrl

namespace {

constexpr double kPi = 3.14159265358979323846;
constexpr uint32_t kDomTracer = 3u;

struct TScene {
    float light_pos[3], power[3];
    float box_min[3], box_max[3], albedo[3];
    float sigma_s[3], sigma_t[3], w;
    int strategy;                 // the medium's sampling strategy (MediumParams)
    float density, mx_sigma[3], mx_cdf[4], mx_start[3], mx_lower[3], mx_norm, mx_inv_norm;
    int sigma_s_zero;
    alvrl::bvh::View bv;          // occluders (ntri == 0: none)
    float occ_albedo[3];
    const float* occ_alb;         // per-triangle reflectance (3 floats, by triangle index), or nullptr
    // area emitter (SmokeBox::emit; nemit == 0: the point light): triangles,
    // the normalized area CDF (nemit + 1 entries), radiance and surface area
    const float* emit;
    const float* emit_cdf;
    uint32_t nemit;
    float emit_radiance[3], emit_area;
};

struct F3 { float x, y, z; };
__device__ __forceinline__ F3 f3(float x, float y, float z) { return F3{x, y, z}; }
__device__ __forceinline__ F3 add(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ F3 sub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ F3 mul(F3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len(F3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ F3 cross(F3 a, F3 b)
{
    return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float safe_sqrt(float v) { return sqrtf(v > 0.0f ? v : 0.0f); }
// math::fastexp / fastlog (math.h:185-199): detmath.h, bit for bit the host's and the oracle's
__device__ __forceinline__ float fastexp(float v) { return dm_expf(v); }
__device__ __forceinline__ float fastlog(float v) { return dm_logf(v); }

// HomogeneousMedium::sampleDistance (homogeneous.cpp:275-352) as the host's
// MediumParams / sample_distance: the same float operations, so the same
// values.  'maximum' follows MaxExpDist (maxexp.h:59-94).
__device__ __forceinline__ int interval_of(const float* a, int n, float x)
{
    int k = 0;
    while (k < n && a[k] < x) k++;
    return k > 0 ? k - 1 : 0;
}

__device__ __forceinline__ float maxexp_sample(const TScene& sc, float u, float* pdf)
{
    const int i = min(interval_of(sc.mx_cdf, 4, u), 2);
    const float t = -fastlog(fastexp(-sc.mx_start[i] * sc.mx_sigma[i]) - sc.mx_norm * (u - sc.mx_cdf[i])) / sc.mx_sigma[i];
    *pdf = sc.mx_sigma[i] * fastexp(-sc.mx_sigma[i] * t) * sc.mx_inv_norm;
    return t;
}

__device__ __forceinline__ float maxexp_cdf(const TScene& sc, float t)
{
    const int i = interval_of(sc.mx_start, 3, t);
    const float upper = -fastexp(-sc.mx_sigma[i] * t);
    return sc.mx_cdf[i] + (upper - sc.mx_lower[i]) * sc.mx_inv_norm;
}

__device__ __forceinline__ void medium_pdfs(const TScene& sc, float sampled, float pdf_max, float* ps, float* pf)
{
    const float w = sc.w;
    float s = 0.0f, f = 0.0f;
    if (sc.strategy == 3) {
        f = 1 - maxexp_cdf(sc, sampled);
        s = pdf_max;
    } else if (sc.strategy == 0) {
        for (int i = 0; i < 3; i++) {
            const float tmp = fastexp(-sc.sigma_t[i] * sampled);
            f += tmp;
            s += sc.sigma_t[i] * tmp;
        }
        f /= 3; s /= 3;
    } else {
        f = fastexp(-sc.density * sampled);
        s = sc.density * f;
    }
    *ps = s * w;
    *pf = w * f + (1 - w);
}

// Random123 Philox4x32-10 and Random::nextFloat (random.cpp:630-639), as the host
struct Stream {
    uint32_t seed, pass, a, b, k, blk;
    uint32_t buf[4];
    __device__ float next()
    {
        const uint32_t bl = k >> 2;
        if (bl != blk) {
            uint32_t c0 = a, c1 = b, c2 = bl, c3 = (kDomTracer << 24);
            uint32_t k0 = seed, k1 = pass;
            for (int r = 0; r < 10; r++) {
                if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
                const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
                const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
                c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
            }
            buf[0] = c0; buf[1] = c1; buf[2] = c2; buf[3] = c3;
            blk = bl;
        }
        const uint32_t u = (buf[k & 3] >> 9) | 0x3f800000u;
        ++k;
        return __uint_as_float(u) - 1.0f;
    }
};

// sampleDistance's draws (homogeneous.cpp:277-296): the distance (INFINITY:
// no medium interaction) and, for 'maximum', the pdf of the sample
template <class S>
__device__ __forceinline__ float sample_distance(const TScene& sc, S& smp, float* pdf_max)
{
    float rnd = smp.next();
    const float w = sc.w;
    if (!(rnd < w)) return INFINITY;
    rnd /= w;
    if (sc.strategy == 3) return maxexp_sample(sc, 1 - rnd, pdf_max);
    float density = sc.density;
    if (sc.strategy == 0) {   // a random channel each time
        int ch = (int)(smp.next() * 3);
        if (ch > 2) ch = 2;
        density = sc.sigma_t[ch];
    }
    return -fastlog(1 - rnd) / density;
}

__device__ F3 uniform_sphere(float sx, float sy)   // warp.cpp:25-31
{
    const float z = 1.0f - 2.0f * sy;
    const float r = safe_sqrt(1.0f - z * z);
    const float theta = (float)(2.0f * kPi * sx);
    return f3(r * (float)cos((double)theta), r * (float)sin((double)theta), z);
}

__device__ F3 cosine_hemisphere(float sx, float sy)   // warp.cpp:43-52, 81-102
{
    const float r1 = 2.0f * sx - 1.0f, r2 = 2.0f * sy - 1.0f;
    float phi, r;
    if (r1 == 0 && r2 == 0) { r = phi = 0; }
    else if (r1 * r1 > r2 * r2) { r = r1; phi = (float)((kPi / 4.0f) * (r2 / r1)); }
    else { r = r2; phi = (float)((kPi / 2.0f) - (r1 / r2) * (kPi / 4.0f)); }
    const float px = r * (float)cos((double)phi), py = r * (float)sin((double)phi);
    float z = safe_sqrt(1.0f - px * px - py * py);
    if (z == 0) z = 1e-10f;
    return f3(px, py, z);
}

__device__ void frame_of(F3 a, F3* b, F3* c)   // coordinateSystem, util.cpp:592-601
{
    if (fabsf(a.x) > fabsf(a.y)) {
        const float invLen = 1.0f / sqrtf(a.x * a.x + a.z * a.z);
        *c = f3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        const float invLen = 1.0f / sqrtf(a.y * a.y + a.z * a.z);
        *c = f3(0.0f, a.z * invLen, -a.y * invLen);
    }
    *b = cross(*c, a);
}

__device__ float box_hit(const TScene& sc, F3 o, F3 d, F3* n)   // first wall hit from inside
{
    float best = INFINITY;
    int axis = -1;
    const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    for (int a = 0; a < 3; a++) {
        float t;
        if (dd[a] > 0) t = (sc.box_max[a] - oo[a]) / dd[a];
        else if (dd[a] < 0) t = (sc.box_min[a] - oo[a]) / dd[a];
        else continue;
        if (t < best) { best = t; axis = a; }
    }
    float nn[3] = {0.0f, 0.0f, 0.0f};
    if (axis >= 0) nn[axis] = dd[axis] > 0 ? -1.0f : 1.0f;
    *n = f3(nn[0], nn[1], nn[2]);
    return best;
}

// Scene::rayIntersect over the walls and the occluders (host SmokeBox::first_hit):
// t, normal, its.p (ray(t) on a wall, barycentric on a triangle), occluder or not
// *tri: the occluder's index (-1: a wall)
__device__ float first_hit(const TScene& sc, F3 o, F3 d, float mint, F3* n, F3* p, int* tri)
{
    float best = box_hit(sc, o, d, n);
    int id = -1, slot = -1;
    float bu = 0.0f, bv = 0.0f;
    alvrl::bvh::closest(sc.bv, alvrl::bvh::mk(o.x, o.y, o.z), alvrl::bvh::mk(d.x, d.y, d.z), mint, &best, &id, &slot,
                        &bu, &bv);
    *tri = id;
    if (id < 0) {
        *p = add(o, mul(d, best));
        return best;
    }
    const float* q = sc.bv.tris + 9 * (size_t)slot;
    const F3 p0 = f3(q[0], q[1], q[2]), p1 = f3(q[3], q[4], q[5]), p2 = f3(q[6], q[7], q[8]);
    const float b0 = 1 - bu - bv;
    *p = add(add(mul(p0, b0), mul(p1, bu)), mul(p2, bv));
    F3 fn = cross(sub(p1, p0), sub(p2, p0));
    const float l = len(fn);
    if (!(fn.x == 0 && fn.y == 0 && fn.z == 0)) fn = mul(fn, 1.0f / l);
    *n = fn;
    return best;
}

// the diffuse reflectance of what first_hit hit: the occluder's own or the shared one, or the walls'
__device__ __forceinline__ const float* albedo_of(const TScene& sc, int tri)
{
    return tri < 0 ? sc.albedo : sc.occ_alb ? sc.occ_alb + 3 * (size_t)tri : sc.occ_albedo;
}

// vrlVector::put + the current VRL (vrlTracer.h:56-89, VRL.h:148-158); counts,
// or writes into the SoA planes at 'pos' when soa != nullptr
struct Sink {
    F3 start;
    float power[3];
    int sigma_s_zero;
    uint32_t n;
    float* soa;
    uint64_t pos, stride;
    __device__ void put(F3 end)
    {
        if (sigma_s_zero) return;
        if (power[0] == 0 && power[1] == 0 && power[2] == 0) return;
        if (len(sub(start, end)) == 0) return;
        if (soa) {
            const uint64_t i = pos + n;
            const float v[9] = {start.x, start.y, start.z, end.x, end.y, end.z, power[0], power[1], power[2]};
#pragma unroll
            for (int pl = 0; pl < 9; pl++) soa[(uint64_t)pl * stride + i] = v[pl];
        }
        n++;
    }
    __device__ void end_current(F3 p)
    {
        if (len(sub(start, p)) == 0) return;
        put(p);
    }
};

// SmokeBox::sample_area_emission (host/scene.cpp), the same operations:
// Scene::sampleEmitterPosition with one emitter, TriMesh::samplePosition,
// Triangle::sample, AreaEmitter::sampleDirection (area.cpp:94-123)
__device__ F3 area_emission(const TScene& sc, float sx, float sy, float dx, float dy, F3* dir, float power[3])
{
    const uint32_t n = sc.nemit;
    uint32_t lb = 0;
    while (lb <= n && sc.emit_cdf[lb] < sy) lb++;   // std::lower_bound
    uint32_t idx = lb > 0 ? lb - 1 : 0;
    if (idx > n - 1) idx = n - 1;
    while (idx + 1 < n && sc.emit_cdf[idx + 1] - sc.emit_cdf[idx] == 0) ++idx;
    const float y = (sy - sc.emit_cdf[idx]) / (sc.emit_cdf[idx + 1] - sc.emit_cdf[idx]);
    const float a = safe_sqrt(1.0f - sx);
    const float bx = 1 - a, by = a * y;
    const float* t = sc.emit + 9 * (size_t)idx;
    const F3 p0 = f3(t[0], t[1], t[2]);
    const F3 sideA = sub(f3(t[3], t[4], t[5]), p0), sideB = sub(f3(t[6], t[7], t[8]), p0);
    const F3 o = add(add(p0, mul(sideA, bx)), mul(sideB, by));
    const F3 c = cross(sideA, sideB);
    const F3 nn = mul(c, 1.0f / len(c));
    for (int i = 0; i < 3; i++) power[i] = (sc.emit_radiance[i] * (float)kPi) * sc.emit_area;
    const F3 l = cosine_hemisphere(dx, dy);
    F3 fs, ft;
    frame_of(nn, &fs, &ft);
    *dir = add(add(mul(fs, l.x), mul(ft, l.y)), mul(nn, l.z));
    return o;
}

__device__ void trace_particle(const TScene& sc, Stream& smp, bool short_vrls, int max_depth, int rr_depth, Sink& k)
{
    const float sx = smp.next(), sy = smp.next();   // sampleEmitterPosition (scene.cpp:958-974)
    const float dx = smp.next(), dy = smp.next();   // sampleDirection (point.cpp:99-106, area.cpp:115-123)
    float power[3];
    F3 dir, o;
    if (sc.nemit) {
        o = area_emission(sc, sx, sy, dx, dy, &dir, power);
    } else {
        dir = uniform_sphere(dx, dy);
        o = f3(sc.light_pos[0], sc.light_pos[1], sc.light_pos[2]);
        for (int i = 0; i < 3; i++) power[i] = sc.power[i];
    }
    if (power[0] == 0 && power[1] == 0 && power[2] == 0) return;
    k.start = o;
    for (int i = 0; i < 3; i++) k.power[i] = power[i];
    int depth = 1;
    float thr[3] = {1.0f, 1.0f, 1.0f};
    const float eta = 1.0f;
    float mint = 1e-4f;   // Ray() default mint (Epsilon), then 0 after a medium and Epsilon after a surface
    while (!(thr[0] == 0 && thr[1] == 0 && thr[2] == 0) && (depth <= max_depth || max_depth < 0)) {
        F3 n, hp;
        int hit_tri;
        const float its_t = first_hit(sc, o, dir, mint, &n, &hp, &hit_tri);
        const bool its_valid = isfinite(its_t);
        // HomogeneousMedium::sampleDistance (homogeneous.cpp:275-352), balance
        float pdf_max = 0.0f;
        float sampled = sample_distance(sc, smp, &pdf_max);
        const float distSurf = its_t - 0.0f;
        bool success = true;
        F3 mp = o;
        if (sampled < distSurf) {
            mp = add(o, mul(dir, sampled + 0.0f));
            if (mp.x == o.x && mp.y == o.y && mp.z == o.z) success = false;
        } else {
            sampled = distSurf;
            success = false;
        }
        float pf, ps;
        medium_pdfs(sc, sampled, pdf_max, &ps, &pf);
        float mtr[3];
        for (int i = 0; i < 3; i++) mtr[i] = fastexp(sc.sigma_t[i] * (-sampled));
        {
            float mx = mtr[0] > mtr[1] ? mtr[0] : mtr[1];
            mx = mx > mtr[2] ? mx : mtr[2];
            if (mx < 1e-20f) mtr[0] = mtr[1] = mtr[2] = 0;
        }
        if (success) {   // vrlTracer.h:143-172
            const float rps = 1.0f / ps;
            for (int i = 0; i < 3; i++) thr[i] *= mtr[i] * sc.sigma_s[i] * rps;
            const float px_ = smp.next(), py_ = smp.next();
            const F3 wo = uniform_sphere(px_, py_);
            const F3 endPoint = short_vrls ? mp : hp;
            k.end_current(endPoint);
            k.start = mp;
            for (int i = 0; i < 3; i++) k.power[i] = thr[i] * power[i];
            o = mp; dir = wo; mint = 0.0f;
        } else if (its_valid) {   // vrlTracer.h:173-213
            const float rpf = 1.0f / pf;
            for (int i = 0; i < 3; i++) thr[i] *= mtr[i] * rpf;
            const F3 p = hp;
            const float* alb = albedo_of(sc, hit_tri);
            F3 fs, ft;
            frame_of(n, &fs, &ft);
            const F3 mwi = f3(-dir.x, -dir.y, -dir.z);
            const float cos_wi = dot(mwi, n);
            const float bx = smp.next(), by = smp.next();
            float bw[3] = {0, 0, 0};
            F3 wol = f3(0, 0, 0);
            if (!(cos_wi <= 0)) {
                wol = cosine_hemisphere(bx, by);
                for (int i = 0; i < 3; i++) bw[i] = alb[i];
            }
            if (bw[0] == 0 && bw[1] == 0 && bw[2] == 0) { k.end_current(p); break; }
            const F3 wo = add(add(mul(fs, wol.x), mul(ft, wol.y)), mul(n, wol.z));
            const float wiDotGeoN = dot(n, mwi), woDotGeoN = dot(n, wo);
            if (wiDotGeoN * cos_wi <= 0 || woDotGeoN * wol.z <= 0) { k.end_current(p); break; }
            for (int i = 0; i < 3; i++) thr[i] *= bw[i];
            k.end_current(p);
            k.start = p;
            for (int i = 0; i < 3; i++) k.power[i] = thr[i] * power[i];
            o = p; dir = wo; mint = 1e-4f;
        } else {
            break;
        }
        if (depth++ >= rr_depth) {
            float mx = thr[0] > thr[1] ? thr[0] : thr[1];
            mx = mx > thr[2] ? mx : thr[2];
            float q = mx * eta * eta;
            if (q > 0.95f) q = 0.95f;
            if (smp.next() >= q) break;
            const float rq = 1.0f / q;
            for (int i = 0; i < 3; i++) thr[i] *= rq;
        }
    }
}

struct TArgs {
    uint32_t seed, pass;
    int short_vrls, max_depth, rr_depth;
};

__global__ void __launch_bounds__(256) k_trace_count(TScene sc, TArgs a, uint64_t p0, uint32_t P, uint32_t* counts)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const uint64_t p = p0 + i;
    Stream smp{a.seed, a.pass, (uint32_t)p, (uint32_t)(p >> 32), 0u, 0xFFFFFFFFu, {0, 0, 0, 0}};
    Sink k{};
    k.sigma_s_zero = sc.sigma_s_zero;
    k.soa = nullptr;
    trace_particle(sc, smp, a.short_vrls != 0, a.max_depth, a.rr_depth, k);
    counts[i] = k.n;
}

__global__ void __launch_bounds__(256) k_trace_write(TScene sc, TArgs a, uint64_t p0, uint32_t P,
                                                     const uint64_t* offs, float* soa, uint64_t stride)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const uint64_t p = p0 + i;
    Stream smp{a.seed, a.pass, (uint32_t)p, (uint32_t)(p >> 32), 0u, 0xFFFFFFFFu, {0, 0, 0, 0}};
    Sink k{};
    k.sigma_s_zero = sc.sigma_s_zero;
    k.soa = soa;
    k.pos = offs[i];
    k.stride = stride;
    trace_particle(sc, smp, a.short_vrls != 0, a.max_depth, a.rr_depth, k);
}

int terr(int code, const std::string& m)
{
    alvrl::host::g_host_err = m;
    return code;
}

template <typename T>
struct DMem {
    T* p = nullptr;
    ~DMem() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t n) { return hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)); }
};

// The scene's occluder BVH on the device (built on the host, host/bvh.cpp).
struct DevBvh {
    DMem<alvrl::BvhNode> nodes;
    DMem<float> tris;
    DMem<uint32_t> ids;
    alvrl::bvh::View view{nullptr, nullptr, nullptr, 0u};
    hipError_t upload(const std::vector<float>& occ)
    {
        const uint32_t nt = (uint32_t)(occ.size() / 9);
        if (nt == 0) return hipSuccess;
        alvrl::BvhHost b;
        try {
            b = alvrl::build_bvh(occ.data(), nt);
        } catch (const std::exception&) {
            return hipErrorInvalidValue;   // deeper than the traversal stacks hold
        }
        hipError_t e = nodes.alloc(b.nodes.size());
        if (e == hipSuccess) e = tris.alloc(b.tris.size());
        if (e == hipSuccess) e = ids.alloc(b.ids.size());
        if (e == hipSuccess) e = hipMemcpy(nodes.p, b.nodes.data(), b.nodes.size() * sizeof(alvrl::BvhNode), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(tris.p, b.tris.data(), b.tris.size() * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(ids.p, b.ids.data(), b.ids.size() * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) view = alvrl::bvh::View{nodes.p, tris.p, ids.p, nt};
        return e;
    }
};

// The last BVH built on each device, keyed by the occluder triangles: the
// integrator's calls for one scene (records every render cache refresh and R
// build, the tracer every pass) reuse it instead of rebuilding it each call.
// The cache is never destroyed (its device memory lives until the process
// exits; freeing it from a static destructor could run after the HIP runtime
// is gone); a caller keeps its BVH alive by holding the shared pointer.
std::shared_ptr<DevBvh> cached_bvh(const std::vector<float>& occ, hipError_t* err)
{
    static std::mutex mu;
    static auto* cache = new std::map<int, std::pair<std::vector<float>, std::shared_ptr<DevBvh>>>();
    int dev = 0;
    *err = hipGetDevice(&dev);
    if (*err != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache->find(dev);
    if (it != cache->end() && it->second.first == occ) return it->second.second;
    auto b = std::make_shared<DevBvh>();
    *err = b->upload(occ);
    if (*err != hipSuccess) return nullptr;
    (*cache)[dev] = {occ, b};
    return b;
}

// The camera of SmokeBox::camera_ray with its per-scene terms formed on the
// host (the same float operations, so the same values).
struct TCam {
    float o[3], fwd[3], left[3], nup[3];
    float tanh_, aspect, inv_w, inv_h;
    uint32_t width;
    int scat;
};

// Sensor::sampleRay at the pixel centre + Scene::rayIntersect (host
// SmokeBox::make_record, bit for bit): the GPU eye-ray first hit of SURVEY
// 8(f) row 1.  pix == nullptr: pixel i.
// Sensor sample j of spp > 1 (SmokeBox::pixel_sample): draws 0 and 1 of the
// counter stream (seed, pass, dom 8, pixel, j).
constexpr uint32_t kDomPixel = 8u;
__device__ __forceinline__ void pixel_jitter(uint32_t seed, uint32_t pass, uint32_t pixel, uint32_t j, float* u,
                                             float* v)
{
    uint32_t c0 = pixel, c1 = j, c2 = 0u, c3 = kDomPixel << 24;
    uint32_t k0 = seed, k1 = pass;
    for (int r = 0; r < 10; r++) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
    *u = __uint_as_float((c0 >> 9) | 0x3f800000u) - 1.0f;
    *v = __uint_as_float((c1 >> 9) | 0x3f800000u) - 1.0f;
}

// spp records per pixel, sample major: record j * n + i is pixel pix[i],
// sensor sample j (its depth word j << 16); spp == 1: pixel centres.
__global__ void __launch_bounds__(256) k_eye_records(TCam c, TScene sc, const uint32_t* __restrict__ pix,
                                                     uint32_t n, uint32_t spp, uint32_t seed, uint32_t pass,
                                                     float* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * spp) return;
    const uint32_t j = i / n, ii = i - j * n;
    const uint32_t id = pix ? pix[ii] : ii;
    float px = (float)(id % c.width) + 0.5f, py = (float)(id / c.width) + 0.5f;
    if (spp > 1) {
        float u, v;
        pixel_jitter(seed, pass, id, j, &u, &v);
        px = (float)(id % c.width) + u;
        py = (float)(id / c.width) + v;
    }
    const float sx = px * c.inv_w, sy = py * c.inv_h;
    const float xc = (1.0f - 2.0f * sx) * c.tanh_;
    const float yc = ((1.0f - 2.0f * sy) / c.aspect) * c.tanh_;
    F3 dc = f3(xc, yc, 1.0f);
    dc = mul(dc, 1.0f / len(dc));
    const float mint = 1e-2f * (1.0f / dc.z);
    const F3 O = f3(c.o[0], c.o[1], c.o[2]);
    const F3 D = f3(c.left[0] * dc.x + c.nup[0] * dc.y + c.fwd[0] * dc.z,
                    c.left[1] * dc.x + c.nup[1] * dc.y + c.fwd[1] * dc.z,
                    c.left[2] * dc.x + c.nup[2] * dc.y + c.fwd[2] * dc.z);
    F3 nn, p;
    int tri;
    const float t = first_hit(sc, O, D, mint, &nn, &p, &tri);
    uint32_t flags = 0;
    if (isfinite(t)) flags |= 1u | 2u;
    if (c.scat) flags |= 4u;
    const float* a = albedo_of(sc, tri);
    float* r = out + 20 * (size_t)i;   // alvrl_gather_rec: 20 words
    const float v[15] = {O.x, O.y, O.z, D.x, D.y, D.z, p.x, p.y, p.z, nn.x, nn.y, nn.z, a[0], a[1], a[2]};
#pragma unroll
    for (int k = 0; k < 15; k++) r[k] = v[k];
    r[15] = __uint_as_float(flags);
    r[16] = 1.0f; r[17] = 1.0f; r[18] = 1.0f;   // a camera ray: path weight 1, depth 0
    r[19] = __uint_as_float(j << 16);
}

// ----------------------------------------------------- volpath reference --
// VolumetricPathTracer::Li_original with onlyVRLpaths (src/integrators/path/
// volpath.cpp:120-457): the path-traced ground truth of the light transport
// VRLs represent, for the statistical parity of the VRL
// method.  One lane per pixel, its samples in order; draws from the counter
// stream (seed, pass, dom 6, pixel, sample) in the reference's order:
// sampleDistance (1-2), medium NEE (2, when requested), phase sample (2),
// surface NEE (2, when requested), BSDF sample (2), Russian roulette (1).
// Isotropic phase, point light (EDiscrete: every MIS weight is 1), diffuse
// walls and occluders, strictNormals off, no emitter is hit by a ray.
constexpr uint32_t kDomVolpath = 6u;

struct VStream {
    uint32_t seed, pass, a, b, k, blk;
    uint32_t buf[4];
    __device__ float next()
    {
        const uint32_t bl = k >> 2;
        if (bl != blk) {
            uint32_t c0 = a, c1 = b, c2 = bl, c3 = (kDomVolpath << 24);
            uint32_t k0 = seed, k1 = pass;
            for (int r = 0; r < 10; r++) {
                if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
                const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
                const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
                c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
            }
            buf[0] = c0; buf[1] = c1; buf[2] = c2; buf[3] = c3;
            blk = bl;
        }
        const uint32_t u = (buf[k & 3] >> 9) | 0x3f800000u;
        ++k;
        return __uint_as_float(u) - 1.0f;
    }
};

struct VParams {
    int max_depth, rr_depth, only_vrl, vol_to_vol, vol_to_surf;
    float intensity[3];
};

// evalTransmittance(p1, p1OnSurface, light, false) (scene.cpp:619-679):
// medium transmittance over the whole segment, 0 behind an occluder
__device__ void attenuation(const TScene& sc, F3 p1, bool p1_surface, F3 p2, float tr[3])
{
    const F3 d0 = sub(p2, p1);
    const float remaining = len(d0);
    const float negLength = 0.0f - remaining;
    for (int i = 0; i < 3; i++) tr[i] = sc.sigma_t[i] != 0 ? fastexp(sc.sigma_t[i] * negLength) : 1.0f;
    if (sc.bv.ntri && remaining > 0) {
        const F3 d = mul(d0, 1.0f / remaining);
        if (alvrl::bvh::occluded(sc.bv, alvrl::bvh::mk(p1.x, p1.y, p1.z), alvrl::bvh::mk(d.x, d.y, d.z),
                                 p1_surface ? 1e-4f : 0.0f, remaining))
            tr[0] = tr[1] = tr[2] = 0.0f;
    }
}

// Scene::sampleAttenuatedEmitterDirect + PointEmitter::sampleDirect
// (scene.cpp:854-898, point.cpp:131-147): value and unit direction to the light
__device__ void light_direct(const TScene& sc, const VParams& vp, F3 ref, bool on_surface, float val[3], F3* dir)
{
    const F3 L = f3(sc.light_pos[0], sc.light_pos[1], sc.light_pos[2]);
    F3 d = sub(L, ref);
    const float dist = len(d);
    const float invDist = 1.0f / dist;
    d = mul(d, invDist);
    *dir = d;
    float tr[3];
    attenuation(sc, ref, on_surface, L, tr);
    for (int i = 0; i < 3; i++) {
        val[i] = vp.intensity[i] * (invDist * invDist);
        val[i] *= tr[i] * 1.0f;   // / emPdf (one emitter)
    }
}

__device__ void volpath_li(const TScene& sc, const VParams& vp, VStream& smp, F3 o, F3 dir, float mint, float Li[3])
{
    Li[0] = Li[1] = Li[2] = 0.0f;
    bool first_ok = false, second_ok = false, prev_diffuse = false, prev_volume = false;
    F3 n, hp;
    int hit_tri;
    float its_t = first_hit(sc, o, dir, mint, &n, &hp, &hit_tri);
    float thr[3] = {1.0f, 1.0f, 1.0f};
    const float eta = 1.0f;
    int depth = 1;
    bool indirect = true;   // rRec.type keeps EIndirect*Radiance (ERadiance / ERadianceNoEmission)
    while (depth <= vp.max_depth || vp.max_depth < 0) {
        if (vp.only_vrl && depth > 2 && !(first_ok && second_ok)) break;   // :144-145
        // HomogeneousMedium::sampleDistance over Ray(ray, 0, its.t)
        float pdf_max = 0.0f;
        float sampled = sample_distance(sc, smp, &pdf_max);
        const float distSurf = its_t - 0.0f;
        bool success = true;
        F3 mp = o;
        if (sampled < distSurf) {
            mp = add(o, mul(dir, sampled + 0.0f));
            if (mp.x == o.x && mp.y == o.y && mp.z == o.z) success = false;
        } else {
            sampled = distSurf;
            success = false;
        }
        float pf, ps;
        medium_pdfs(sc, sampled, pdf_max, &ps, &pf);
        float mtr[3];
        for (int i = 0; i < 3; i++) mtr[i] = fastexp(sc.sigma_t[i] * (-sampled));
        {
            float mx = mtr[0] > mtr[1] ? mtr[0] : mtr[1];
            mx = mx > mtr[2] ? mx : mtr[2];
            if (mx < 1e-20f) mtr[0] = mtr[1] = mtr[2] = 0;
        }
        if (success) {   // :150-267
            if (depth == 1 && vp.vol_to_vol) first_ok = true;
            if (depth == 2) second_ok = true;
            if (depth >= vp.max_depth && vp.max_depth != -1) break;
            const float rps = 1.0f / ps;
            for (int i = 0; i < 3; i++) thr[i] *= (sc.sigma_s[i] * mtr[i]) * rps;
            // luminaire sampling; the reference's "(!rRec.depth==2 || ...)" is
            // "((!depth) == 2 || ...)", i.e. the bracket alone (:183-190)
            const bool nee = !vp.only_vrl ||
                             (depth != 1 && (prev_volume || prev_diffuse) && (!prev_diffuse || vp.vol_to_surf) &&
                              (!prev_volume || vp.vol_to_vol));
            if (nee) {
                (void)smp.next(); (void)smp.next();   // rRec.nextSample2D() (unused by a point light)
                float val[3];
                F3 ld;
                light_direct(sc, vp, mp, false, val, &ld);
                if (!(val[0] == 0 && val[1] == 0 && val[2] == 0)) {
                    const float phaseVal = 0.079577471545947667884f;   // IsotropicPhaseFunction::eval, 1/(4 pi)
                    for (int i = 0; i < 3; i++) Li[i] += ((thr[i] * val[i]) * phaseVal) * 1.0f;
                }
            }
            // phase sampling (isotropic: weight 1)
            const float px_ = smp.next(), py_ = smp.next();
            const F3 wo = uniform_sphere(px_, py_);
            o = mp; dir = wo;
            its_t = first_hit(sc, o, dir, 0.0f, &n, &hp, &hit_tri);
            if (!indirect) break;
            prev_volume = true;
            prev_diffuse = false;
        } else {   // :268-435
            const float rpf = 1.0f / pf;
            for (int i = 0; i < 3; i++) thr[i] *= mtr[i] * rpf;
            if (!isfinite(its_t)) break;
            if (depth >= vp.max_depth && vp.max_depth != -1) break;
            const float* alb = albedo_of(sc, hit_tri);
            const F3 p = hp;
            const float cos_wi = dot(f3(-dir.x, -dir.y, -dir.z), n);
            if (!vp.only_vrl || (first_ok && second_ok)) {   // :319-350 (ESmooth diffuse)
                (void)smp.next(); (void)smp.next();
                float val[3];
                F3 ld;
                light_direct(sc, vp, p, true, val, &ld);
                if (!(val[0] == 0 && val[1] == 0 && val[2] == 0)) {
                    const float cos_wo = dot(ld, n);
                    if (!(cos_wi <= 0 || cos_wo <= 0)) {
                        const float k = 0.31830988618379067154f * cos_wo;   // INV_PI * cosTheta(wo)
                        for (int i = 0; i < 3; i++) Li[i] += ((thr[i] * val[i]) * (alb[i] * k)) * 1.0f;
                    }
                }
            }
            // BSDF sampling (diffuse.cpp:140-150)
            const float bx = smp.next(), by = smp.next();
            if (cos_wi <= 0) break;   // bsdfWeight.isZero()
            const F3 wol = cosine_hemisphere(bx, by);
            F3 fs, ft;
            frame_of(n, &fs, &ft);
            const F3 wo = add(add(mul(fs, wol.x), mul(ft, wol.y)), mul(n, wol.z));
            if (depth == 1 && vp.vol_to_surf) first_ok = true;   // :377-382 (inside the medium, smooth)
            prev_volume = false;
            prev_diffuse = true;
            for (int i = 0; i < 3; i++) thr[i] *= alb[i];
            o = p; dir = wo;
            its_t = first_hit(sc, o, dir, 1e-4f, &n, &hp, &hit_tri);
            if (!indirect) break;
        }
        if (depth++ >= vp.rr_depth) {   // :437-446
            float mx = thr[0] > thr[1] ? thr[0] : thr[1];
            mx = mx > thr[2] ? mx : thr[2];
            float q = mx * eta * eta;
            if (q > 0.95f) q = 0.95f;
            if (smp.next() >= q) break;
            const float rq = 1.0f / q;
            for (int i = 0; i < 3; i++) thr[i] *= rq;
        }
    }
    if (vp.only_vrl && !(first_ok && second_ok)) Li[0] = Li[1] = Li[2] = 0.0f;   // :453-455
}

__global__ void __launch_bounds__(256) k_volpath(TCam c, TScene sc, VParams vp, uint32_t seed, uint32_t pass,
                                                 uint32_t spp, const uint32_t* __restrict__ pix, uint32_t n,
                                                 float* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t id = pix ? pix[i] : i;
    const float px = (float)(id % c.width) + 0.5f, py = (float)(id / c.width) + 0.5f;
    const float sx = px * c.inv_w, sy = py * c.inv_h;
    const float xc = (1.0f - 2.0f * sx) * c.tanh_;
    const float yc = ((1.0f - 2.0f * sy) / c.aspect) * c.tanh_;
    F3 dc = f3(xc, yc, 1.0f);
    dc = mul(dc, 1.0f / len(dc));
    const float mint = 1e-2f * (1.0f / dc.z);
    const F3 O = f3(c.o[0], c.o[1], c.o[2]);
    const F3 D = f3(c.left[0] * dc.x + c.nup[0] * dc.y + c.fwd[0] * dc.z,
                    c.left[1] * dc.x + c.nup[1] * dc.y + c.fwd[1] * dc.z,
                    c.left[2] * dc.x + c.nup[2] * dc.y + c.fwd[2] * dc.z);
    float acc[3] = {0.0f, 0.0f, 0.0f};
    for (uint32_t s = 0; s < spp; s++) {
        VStream smp{seed, pass, id, s, 0u, 0xFFFFFFFFu, {0, 0, 0, 0}};
        float li[3];
        volpath_li(sc, vp, smp, O, D, mint, li);
        for (int k = 0; k < 3; k++) acc[k] += li[k];
    }
    const float r = 1.0f / (float)spp;
    for (int k = 0; k < 3; k++) out[3 * (size_t)i + k] = acc[k] * r;
}

TScene make_tscene(const alvrl::host::SmokeBox& box)
{
    TScene sc;
    sc.light_pos[0] = box.light_pos.x; sc.light_pos[1] = box.light_pos.y; sc.light_pos[2] = box.light_pos.z;
    for (int i = 0; i < 3; i++) {
        sc.power[i] = box.light_intensity[i] * (float)(4 * kPi);
        sc.box_min[i] = box.box_min[i]; sc.box_max[i] = box.box_max[i];
        sc.albedo[i] = box.albedo[i];
        sc.sigma_s[i] = box.medium.sigma_s[i];
        sc.sigma_t[i] = box.medium.sigma_t[i];
        sc.occ_albedo[i] = box.occ_albedo[i];
    }
    sc.occ_alb = nullptr;   // set by the caller that uploads box.occ_alb (upload_albedos)
    sc.w = box.medium.sampling_weight;
    sc.strategy = box.medium.strategy;
    sc.density = box.medium.density;
    for (int i = 0; i < 3; i++) {
        sc.mx_sigma[i] = box.medium.mx_sigma[i]; sc.mx_start[i] = box.medium.mx_start[i];
        sc.mx_lower[i] = box.medium.mx_lower[i];
    }
    for (int i = 0; i < 4; i++) sc.mx_cdf[i] = box.medium.mx_cdf[i];
    sc.mx_norm = box.medium.mx_norm;
    sc.mx_inv_norm = box.medium.mx_inv_norm;
    sc.sigma_s_zero = (sc.sigma_s[0] == 0 && sc.sigma_s[1] == 0 && sc.sigma_s[2] == 0) ? 1 : 0;
    sc.bv = alvrl::bvh::View{nullptr, nullptr, nullptr, 0u};
    sc.emit = nullptr;
    sc.emit_cdf = nullptr;
    sc.nemit = (uint32_t)(box.emit.size() / 9);
    for (int i = 0; i < 3; i++) sc.emit_radiance[i] = box.emit_radiance[i];
    sc.emit_area = box.emit_area;
    return sc;
}

TCam make_tcam(const alvrl::host::SmokeBox& box, int scat)
{
    using namespace alvrl::host;
    TCam c;
    const V3 fwd = normalize(box.cam_target - box.cam_origin);
    const V3 left = normalize(cross(box.cam_up, fwd));
    const V3 nup = cross(fwd, left);
    const float vv[4][3] = {{box.cam_origin.x, box.cam_origin.y, box.cam_origin.z}, {fwd.x, fwd.y, fwd.z},
                            {left.x, left.y, left.z}, {nup.x, nup.y, nup.z}};
    for (int k = 0; k < 3; k++) { c.o[k] = vv[0][k]; c.fwd[k] = vv[1][k]; c.left[k] = vv[2][k]; c.nup[k] = vv[3][k]; }
    c.aspect = (float)box.width / (float)box.height;
    c.tanh_ = std::tan(0.5f * box.fov_x_deg * (float)(kPi / 180.0));
    c.inv_w = 1.0f / (float)box.width;
    c.inv_h = 1.0f / (float)box.height;
    c.width = (uint32_t)box.width;
    c.scat = scat;
    return c;
}

}  // namespace

extern "C" {

ALVRL_API void alvrl_volpath_default(alvrl_volpath_params* p)
{
    if (!p) return;
    p->max_depth = -1;       // MonteCarloIntegrator maxDepth
    p->rr_depth = 5;         // rrDepth
    p->only_vrl_paths = 1;   // volpath.cpp:79-81
    p->vrl_vol_to_vol = 1;
    p->vrl_vol_to_surf = 1;
}

// the occluders' own reflectances on the device (SmokeBox::occ_alb), for TScene::occ_alb
static bool upload_albedos(const alvrl::host::SmokeBox& box, DMem<float>& d, TScene& sc)
{
    if (box.occ_alb.empty()) return true;
    if (d.alloc(box.occ_alb.size()) != hipSuccess) return false;
    if (hipMemcpy(d.p, box.occ_alb.data(), box.occ_alb.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return false;
    sc.occ_alb = d.p;
    return true;
}

ALVRL_API int alvrl_volpath_render(const alvrl_scene_desc* s, const alvrl_volpath_params* p, uint32_t seed,
                                   uint32_t pass, uint32_t spp, const uint32_t* d_pixel_ids, uint32_t n,
                                   float* d_out_rgb, void* stream)
{
    if (!s || !p || (!d_out_rgb && n)) return terr(ALVRL_ERR_INVALID, "alvrl_volpath_render: null argument");
    if (spp == 0) return terr(ALVRL_ERR_INVALID, "alvrl_volpath_render: spp must be > 0");
    if (s->medium.phase_type != 0)
        return terr(ALVRL_ERR_INVALID, "alvrl_volpath_render: only the isotropic phase function is supported");
    if (const char* m = alvrl::host::scene_problem(*s)) return terr(ALVRL_ERR_INVALID, m);
    const alvrl::host::SmokeBox box = alvrl::host::to_box(*s);
    if (box.has_delta())
        return terr(ALVRL_ERR_INVALID, "alvrl_volpath_render: mirror / null occluders are not supported by the volpath reference");
    if (box.area_light())
        return terr(ALVRL_ERR_INVALID, "alvrl_volpath_render: the volpath reference samples the point light only");
    const uint64_t npix = (uint64_t)box.width * (uint64_t)box.height;
    if (!d_pixel_ids && n > npix) return terr(ALVRL_ERR_INVALID, "alvrl_volpath_render: n > W*H without pixel ids");
    if (n == 0) return ALVRL_OK;
    TScene sc = make_tscene(box);
    hipError_t be = hipSuccess;
    const std::shared_ptr<DevBvh> bv = cached_bvh(box.occ, &be);
    if (!bv) return terr(ALVRL_ERR_HIP, "alvrl_volpath_render: BVH upload");
    sc.bv = bv->view;
    DMem<float> d_alb;
    if (!upload_albedos(box, d_alb, sc)) return terr(ALVRL_ERR_HIP, "alvrl_volpath_render: albedo upload");
    const TCam c = make_tcam(box, 1);
    VParams vp;
    vp.max_depth = p->max_depth; vp.rr_depth = p->rr_depth; vp.only_vrl = p->only_vrl_paths ? 1 : 0;
    vp.vol_to_vol = p->vrl_vol_to_vol ? 1 : 0; vp.vol_to_surf = p->vrl_vol_to_surf ? 1 : 0;
    for (int i = 0; i < 3; i++) vp.intensity[i] = box.light_intensity[i];
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_volpath, dim3((n + 255) / 256), dim3(256), 0, st, c, sc, vp, seed, pass, spp, d_pixel_ids, n,
                       d_out_rgb);
    if (hipGetLastError() != hipSuccess) return terr(ALVRL_ERR_HIP, "alvrl_volpath_render: launch");
    if (hipStreamSynchronize(st) != hipSuccess) return terr(ALVRL_ERR_HIP, "alvrl_volpath_render: sync");
    return ALVRL_OK;
}

// Gather records of pixel centres on the current HIP device (the host
// alvrl_scene_records, bit for bit).  d_pixel_ids (device, row-major y*W+x)
// may be NULL: pixels 0..n-1.  d_out: n device records.  Stream-ordered on
// 'stream' (the occluder BVH is built and uploaded synchronously first).
ALVRL_API int alvrl_scene_records_gpu(const alvrl_scene_desc* s, int medium_scatters, const uint32_t* d_pixel_ids,
                                      uint32_t n, alvrl_gather_rec* d_out, void* stream)
{
    return alvrl_scene_records_spp_gpu(s, medium_scatters, 0u, 0u, 1u, d_pixel_ids, n, d_out, stream);
}

// The sensor samples of alvrl_scene_records_spp (the host's, bit for bit):
// n * spp device records, sample major.
ALVRL_API int alvrl_scene_records_spp_gpu(const alvrl_scene_desc* s, int medium_scatters, uint32_t seed,
                                          uint32_t pass, uint32_t spp, const uint32_t* d_pixel_ids, uint32_t n,
                                          alvrl_gather_rec* d_out, void* stream)
{
    if (!s || (!d_out && n)) return terr(ALVRL_ERR_INVALID, "alvrl_scene_records_gpu: null argument");
    if (spp == 0 || spp > 0xFFFFu || (uint64_t)spp * n > 0xFFFFFFFFull)
        return terr(ALVRL_ERR_INVALID, "alvrl_scene_records_spp_gpu: spp out of range");
    if (const char* m = alvrl::host::scene_problem(*s)) return terr(ALVRL_ERR_INVALID, m);
    const alvrl::host::SmokeBox box = alvrl::host::to_box(*s);
    if (box.has_delta())
        return terr(ALVRL_ERR_INVALID, "alvrl_scene_records_gpu: mirror / null occluders: the eye paths are formed "
                                       "on the host (alvrl_scene_records, the integrator's chain records)");
    const uint64_t npix = (uint64_t)box.width * (uint64_t)box.height;
    if (!d_pixel_ids && n > npix) return terr(ALVRL_ERR_INVALID, "alvrl_scene_records_gpu: n > W*H without pixel ids");
    if (n == 0) return ALVRL_OK;
    TScene sc = make_tscene(box);
    hipError_t be = hipSuccess;
    const std::shared_ptr<DevBvh> bv = cached_bvh(box.occ, &be);
    if (!bv) return terr(ALVRL_ERR_HIP, "alvrl_scene_records_gpu: BVH upload");
    sc.bv = bv->view;
    DMem<float> d_alb;
    if (!upload_albedos(box, d_alb, sc)) return terr(ALVRL_ERR_HIP, "alvrl_scene_records_gpu: albedo upload");
    const TCam c = make_tcam(box, medium_scatters && !sc.sigma_s_zero ? 1 : 0);
    hipStream_t st = (hipStream_t)stream;
    const uint32_t total = n * spp;
    hipLaunchKernelGGL(k_eye_records, dim3((total + 255) / 256), dim3(256), 0, st, c, sc, d_pixel_ids, n, spp, seed,
                       pass, reinterpret_cast<float*>(d_out));
    if (hipGetLastError() != hipSuccess) return terr(ALVRL_ERR_HIP, "alvrl_scene_records_gpu: launch");
    // stream-ordered callers may replace the cached BVH after return: wait for the kernel
    if (hipStreamSynchronize(st) != hipSuccess) return terr(ALVRL_ERR_HIP, "alvrl_scene_records_gpu: sync");
    return ALVRL_OK;
}

// The GPU form of alvrl_trace_vrls (same arguments and results); runs on the
// current HIP device.
ALVRL_API int alvrl_trace_vrls_gpu(const alvrl_scene_desc* s, uint32_t seed, uint32_t pass, uint32_t target,
                                   int short_vrls, int max_depth, int rr_depth, float* soa, uint32_t cap,
                                   uint32_t* n, uint64_t* particles)
{
    if (!s || !n || !particles) return terr(ALVRL_ERR_INVALID, "alvrl_trace_vrls_gpu: null argument");
    // the scene as the host tracer resolves it (to_box + MediumParams::resolve)
    if (const char* m = alvrl::host::scene_problem(*s)) return terr(ALVRL_ERR_INVALID, m);
    const alvrl::host::SmokeBox box = alvrl::host::to_box(*s);
    if (box.has_delta())
        return terr(ALVRL_ERR_INVALID, "alvrl_trace_vrls_gpu: mirror / null occluders are traced on the host (alvrl_trace_vrls)");
    TScene sc = make_tscene(box);
    hipError_t be = hipSuccess;
    const std::shared_ptr<DevBvh> bvh = cached_bvh(box.occ, &be);
    if (!bvh) return terr(ALVRL_ERR_HIP, "alvrl_trace_vrls_gpu: BVH upload");
    sc.bv = bvh->view;
    DMem<float> d_alb;
    if (!upload_albedos(box, d_alb, sc)) return terr(ALVRL_ERR_HIP, "alvrl_trace_vrls_gpu: albedo upload");
    const TArgs a{seed, pass, short_vrls, max_depth, rr_depth};
    *n = 0;
    if (target == 0) { *particles = 0; return ALVRL_OK; }
    if (sc.sigma_s_zero) { *particles = 1000001; return ALVRL_OK; }   // the host loop's bound
    const float* pw = sc.nemit ? sc.emit_radiance : sc.power;
    if (pw[0] == 0 && pw[1] == 0 && pw[2] == 0)
        return terr(ALVRL_ERR_INVALID, "alvrl_trace_vrls_gpu: the light emits nothing (the VRL target is unreachable)");
    // the area emitter's triangles and sampling table on the device
    DMem<float> d_emit, d_cdf;
    if (sc.nemit) {
        if (d_emit.alloc(box.emit.size()) != hipSuccess || d_cdf.alloc(box.emit_cdf.size()) != hipSuccess)
            return terr(ALVRL_ERR_NOMEM, "alvrl_trace_vrls_gpu: device memory");
        if (hipMemcpy(d_emit.p, box.emit.data(), box.emit.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(d_cdf.p, box.emit_cdf.data(), box.emit_cdf.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
            return terr(ALVRL_ERR_HIP, "alvrl_trace_vrls_gpu: copy");
        sc.emit = d_emit.p;
        sc.emit_cdf = d_cdf.p;
    }
    // count pass, batch by batch, until the running total reaches the target
    const uint32_t P = std::min<uint32_t>(1u << 20, std::max<uint32_t>(4096u, target));
    DMem<uint32_t> d_cnt;
    if (d_cnt.alloc(P) != hipSuccess) return terr(ALVRL_ERR_NOMEM, "alvrl_trace_vrls_gpu: device memory");
    std::vector<uint32_t> counts;
    uint64_t total = 0, used = 0;
    for (uint64_t p0 = 0; used == 0; p0 += P) {
        if (p0 > (1ull << 32)) return terr(ALVRL_ERR_INVALID, "alvrl_trace_vrls_gpu: target not reached");
        hipLaunchKernelGGL(k_trace_count, dim3((P + 255) / 256), dim3(256), 0, 0, sc, a, p0, P, d_cnt.p);
        if (hipGetLastError() != hipSuccess) return terr(ALVRL_ERR_HIP, "alvrl_trace_vrls_gpu: launch");
        const size_t base = counts.size();
        counts.resize(base + P);
        if (hipMemcpy(counts.data() + base, d_cnt.p, P * 4, hipMemcpyDeviceToHost) != hipSuccess)
            return terr(ALVRL_ERR_HIP, "alvrl_trace_vrls_gpu: copy");
        for (uint32_t i = 0; i < P; i++) {
            total += counts[base + i];
            if (total >= target) { used = base + i + 1; break; }
        }
    }
    *particles = used;
    *n = (uint32_t)total;
    if (!soa) return ALVRL_OK;   // size query
    if (total > cap) return terr(ALVRL_ERR_INVALID, "alvrl_trace_vrls_gpu: capacity too small");
    // write pass: every particle's VRLs at its exclusive prefix offset
    std::vector<uint64_t> offs(used);
    uint64_t o = 0;
    for (uint64_t i = 0; i < used; i++) { offs[i] = o; o += counts[i]; }
    DMem<uint64_t> d_off;
    DMem<float> d_soa;
    if (d_off.alloc(used) != hipSuccess || d_soa.alloc(9 * total) != hipSuccess)
        return terr(ALVRL_ERR_NOMEM, "alvrl_trace_vrls_gpu: device memory");
    if (hipMemcpy(d_off.p, offs.data(), used * 8, hipMemcpyHostToDevice) != hipSuccess)
        return terr(ALVRL_ERR_HIP, "alvrl_trace_vrls_gpu: copy");
    for (uint64_t p0 = 0; p0 < used; p0 += P) {
        const uint32_t np = (uint32_t)std::min<uint64_t>(P, used - p0);
        hipLaunchKernelGGL(k_trace_write, dim3((np + 255) / 256), dim3(256), 0, 0, sc, a, p0, np, d_off.p + p0,
                           d_soa.p, total);
        if (hipGetLastError() != hipSuccess) return terr(ALVRL_ERR_HIP, "alvrl_trace_vrls_gpu: launch");
    }
    if (hipMemcpy2D(soa, (size_t)cap * 4, d_soa.p, total * 4, total * 4, 9, hipMemcpyDeviceToHost) != hipSuccess)
        return terr(ALVRL_ERR_HIP, "alvrl_trace_vrls_gpu: copy");
    return ALVRL_OK;
}

}  // extern "C"
