// scene.cpp -- smoke-box harness and the VRL tracer (see scene.hpp).
// Compiled with g++ -ffp-contract=off: float semantics identical to the
// oracle's restatement, so records and VRL sets agree bit for bit with it.
#include "scene.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "detmath.h"

namespace alvrl {
namespace host {

namespace {
constexpr double kPi = 3.14159265358979323846;
constexpr uint32_t kDomTracer = 3u;
constexpr uint32_t kDomEye = 7u;   // Russian roulette of the eye paths' specular chains
constexpr uint32_t kDomPixel = 8u;   // sensor sample offsets of multi-sample renders

// math::fastexp / fastlog (math.h:185-199) with the deterministic definitions
// the oracle and tracer.hip share (detmath.h, DESIGN.md section 8 deviation 3)
inline float fastexp(float v) { return dm_expf(v); }
inline float fastlog(float v) { return dm_logf(v); }
inline float safe_sqrt(float v) { return std::sqrt(v > 0.0f ? v : 0.0f); }
}  // namespace

float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
float length(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
V3 normalize(V3 a) { const float r = 1.0f / length(a); return a * r; }
V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }

void MediumParams::resolve()
{
    for (int i = 0; i < 3; i++) sigma_t[i] = sigma_s[i] + sigma_a[i];
    float w = sampling_weight;
    if (w == -1) {
        for (int i = 0; i < 3; i++) {
            const float albedo = sigma_s[i] / sigma_t[i];
            if (albedo > w && sigma_t[i] != 0) w = albedo;
        }
        if (w > 0) w = w > 0.5f ? w : 0.5f;
    }
    sampling_weight = w;
    density = strategy == 2 ? density : 0.0f;
    if (strategy == 1) {   // homogeneous.cpp:188-204
        int ch = channel - 1;
        if (ch < 0) {
            float smallest = INFINITY;
            ch = 0;
            for (int i = 0; i < 3; i++)
                if (sigma_t[i] < smallest) { smallest = sigma_t[i]; ch = i; }
        }
        density = sigma_t[ch];
    } else if (strategy == 3) {   // MaxExpDist(sigmaT), maxexp.h:30-57
        float s[3] = {sigma_t[0], sigma_t[1], sigma_t[2]};
        std::sort(s, s + 3, [](float a, float b) { return a > b; });
        float cdf[4];
        cdf[0] = 0;
        for (int i = 0; i < 3; i++) {
            const float lower = (i == 0) ? -1 : -std::pow(s[i] / s[i - 1], -s[i] / (s[i] - s[i - 1]));
            const float upper = (i == 2) ? 0 : -std::pow(s[i + 1] / s[i], -s[i] / (s[i + 1] - s[i]));
            cdf[i + 1] = cdf[i] + (upper - lower);
            mx_start[i] = (i == 0) ? 0 : fastlog(s[i] / s[i - 1]) / (s[i] - s[i - 1]);
            mx_lower[i] = lower;
            mx_sigma[i] = s[i];
        }
        mx_norm = cdf[3];
        mx_inv_norm = 1 / mx_norm;
        for (int i = 0; i < 4; i++) mx_cdf[i] = cdf[i] * mx_inv_norm;
    }
}

const char* MediumParams::problem() const
{
    if (strategy < 0 || strategy > 3) return "alvrl_medium_desc: unknown sampling strategy";
    if (strategy == 1 && (channel < 0 || channel > 3)) return "alvrl_medium_desc: 'single' channel out of range";
    if (strategy == 3) {
        float s[3];
        for (int i = 0; i < 3; i++) s[i] = sigma_s[i] + sigma_a[i];
        if (s[0] == s[1] || s[1] == s[2] || s[0] == s[2])
            return "alvrl_medium_desc: 'maximum' needs sigma_t to vary across channels (maxexp.h:37-38)";
    }
    return nullptr;
}

namespace {
// std::max(0, lower_bound(a, a + n, x) - a - 1)
int interval_of(const float* a, int n, float x)
{
    int k = 0;
    while (k < n && a[k] < x) k++;
    return k > 0 ? k - 1 : 0;
}
}  // namespace

float MediumParams::maxexp_sample(float u, float* pdf) const
{
    // the index clamped to the last interval (u = 1 above a rounded m_cdf[n])
    const int i = std::min(interval_of(mx_cdf, 4, u), 2);
    const float t = -fastlog(fastexp(-mx_start[i] * mx_sigma[i]) - mx_norm * (u - mx_cdf[i])) / mx_sigma[i];
    *pdf = mx_sigma[i] * fastexp(-mx_sigma[i] * t) * mx_inv_norm;
    return t;
}

float MediumParams::maxexp_cdf(float t) const
{
    const int i = interval_of(mx_start, 3, t);
    const float upper = -fastexp(-mx_sigma[i] * t);
    return mx_cdf[i] + (upper - mx_lower[i]) * mx_inv_norm;
}

void MediumParams::pdfs(float sampled, float pdf_max, float* ps, float* pf) const
{
    const float w = sampling_weight;
    float s = 0.0f, f = 0.0f;
    if (strategy == 3) {
        f = 1 - maxexp_cdf(sampled);
        s = pdf_max;
    } else if (strategy == 0) {
        for (int i = 0; i < 3; i++) {
            const float tmp = fastexp(-sigma_t[i] * sampled);
            f += tmp;
            s += sigma_t[i] * tmp;
        }
        f /= 3; s /= 3;
    } else {
        f = fastexp(-density * sampled);
        s = density * f;
    }
    *ps = s * w;
    *pf = w * f + (1 - w);
}

void SmokeBox::camera_ray(float px, float py, V3* o, V3* d, float* mint) const
{
    const V3 fwd = normalize(cam_target - cam_origin);
    const V3 left = normalize(cross(cam_up, fwd));
    const V3 nup = cross(fwd, left);
    const float aspect = (float)width / (float)height;
    const float tanh_ = std::tan(0.5f * fov_x_deg * (float)(kPi / 180.0));
    const float sx = px * (1.0f / (float)width);
    const float sy = py * (1.0f / (float)height);
    const float xc = (1.0f - 2.0f * sx) * tanh_;
    const float yc = ((1.0f - 2.0f * sy) / aspect) * tanh_;
    const V3 dc = normalize(v3(xc, yc, 1.0f));
    if (mint) *mint = 1e-2f * (1.0f / dc.z);
    *o = cam_origin;
    *d = v3(left.x * dc.x + nup.x * dc.y + fwd.x * dc.z,
            left.y * dc.x + nup.y * dc.y + fwd.y * dc.z,
            left.z * dc.x + nup.z * dc.y + fwd.z * dc.z);
}

float SmokeBox::box_hit(V3 o, V3 d, V3* n) const
{
    float best = INFINITY;
    int axis = -1;
    const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    for (int a = 0; a < 3; a++) {
        float t;
        if (dd[a] > 0) t = (box_max[a] - oo[a]) / dd[a];
        else if (dd[a] < 0) t = (box_min[a] - oo[a]) / dd[a];
        else continue;
        if (t < best) { best = t; axis = a; }
    }
    float nn[3] = {0.0f, 0.0f, 0.0f};
    if (axis >= 0) nn[axis] = dd[axis] > 0 ? -1.0f : 1.0f;
    *n = v3(nn[0], nn[1], nn[2]);
    return best;
}

float fresnel_dielectric_ext(float cos_theta_i, float* cos_theta_t, float eta)
{
    if (eta == 1) {
        *cos_theta_t = -cos_theta_i;
        return 0.0f;
    }
    const float scale = (cos_theta_i > 0) ? 1 / eta : eta;
    const float cos_t_sqr = 1 - (1 - cos_theta_i * cos_theta_i) * (scale * scale);
    if (cos_t_sqr <= 0.0f) {   // total internal reflection
        *cos_theta_t = 0.0f;
        return 1.0f;
    }
    const float ci = std::fabs(cos_theta_i);
    const float ct = std::sqrt(cos_t_sqr);
    const float Rs = (ci - eta * ct) / (ci + eta * ct);
    const float Rp = (eta * ci - ct) / (eta * ci + ct);
    *cos_theta_t = (cos_theta_i > 0) ? -ct : ct;
    return 0.5f * (Rs * Rs + Rp * Rp);
}

bool tri_intersect(const float* tri, V3 o, V3 d, float* u, float* v, float* t)
{
    const V3 p0 = v3(tri[0], tri[1], tri[2]), p1 = v3(tri[3], tri[4], tri[5]), p2 = v3(tri[6], tri[7], tri[8]);
    const V3 edge1 = p1 - p0, edge2 = p2 - p0;
    const V3 pvec = cross(d, edge2);
    const float det = dot(edge1, pvec);
    if (det == 0) return false;
    const float inv_det = 1.0f / det;
    const V3 tvec = o - p0;
    *u = dot(tvec, pvec) * inv_det;
    if (*u < 0.0f || *u > 1.0f) return false;
    const V3 qvec = cross(tvec, edge1);
    *v = dot(d, qvec) * inv_det;
    if (*v >= 0.0f && *u + *v <= 1.0f) {   // inverted comparison (catches NaNs)
        *t = dot(edge2, qvec) * inv_det;
        return true;
    }
    return false;
}

float SmokeBox::first_hit(V3 o, V3 d, float mint, V3* n, V3* p, int* tri) const
{
    float best = box_hit(o, d, n);
    int bi = -1;
    float bu = 0.0f, bv = 0.0f;
    const uint32_t nt = n_occ();
    for (uint32_t i = 0; i < nt; i++) {   // shape kd-tree leaf test, t in [mint, maxt] (skdtree.h:248-262)
        float u, v, t;
        if (!tri_intersect(&occ[9 * (size_t)i], o, d, &u, &v, &t)) continue;
        if (t < mint || !(t < best)) continue;
        best = t; bi = (int)i; bu = u; bv = v;
    }
    *tri = bi;
    if (bi < 0) {
        *p = o + d * best;
        return best;
    }
    // fillIntersectionRecord (skdtree.h:350-396): barycentric position, face normal
    const float* q = &occ[9 * (size_t)bi];
    const V3 p0 = v3(q[0], q[1], q[2]), p1 = v3(q[3], q[4], q[5]), p2 = v3(q[6], q[7], q[8]);
    const float b0 = 1 - bu - bv;
    *p = (p0 * b0 + p1 * bu) + p2 * bv;
    V3 fn = cross(p1 - p0, p2 - p0);
    const float len = length(fn);
    if (!(fn.x == 0 && fn.y == 0 && fn.z == 0)) fn = fn * (1.0f / len);
    *n = fn;
    return best;
}

bool SmokeBox::visible(V3 p1, bool p1_surface, V3 p2, bool p2_surface) const
{
    const uint32_t nt = n_occ();
    if (nt == 0) return true;
    V3 d = p2 - p1;
    const float remaining = length(d);
    if (!(remaining > 0)) return true;   // the loop of scene.cpp:634 does not run
    d = d * (1.0f / remaining);
    const float mint = p1_surface ? 1e-4f : 0.0f;                     // Epsilon
    const float maxt = remaining * (p2_surface ? (1 - 1e-3f) : 1.0f);   // ShadowEpsilon
    for (uint32_t i = 0; i < nt; i++) {
        if (mat((int)i) == 2u) continue;   // ENull: passes (scene.cpp:636-637)
        float u, v, t;
        if (tri_intersect(&occ[9 * (size_t)i], p1, d, &u, &v, &t) && !(t < mint || t > maxt)) return false;
    }
    return true;
}

void SmokeBox::make_record(int x, int y, bool medium_scatters, float rec[kRecWords], uint32_t seed, uint32_t pass,
                           uint32_t sample, uint32_t spp) const
{
    V3 O, D, n, p;
    float mint, px, py;
    pixel_sample(x, y, seed, pass, sample, spp, &px, &py);
    camera_ray(px, py, &O, &D, &mint);   // renderBlock's sensor sample, integrator.cpp:240-247
    int tri;
    const float t = first_hit(O, D, mint, &n, &p, &tri);
    const uint32_t m = mat(tri);
    uint32_t flags = 0;
    if (std::isfinite(t)) flags |= 1u | (m == 0u ? 2u : 8u);   // ESmooth (diffuse) or EDelta
    if (medium_scatters) flags |= 4u;
    static const float kZero[3] = {0.0f, 0.0f, 0.0f};
    const float* a = m != 0u ? kZero : (tri >= 0 ? occ_albedo_of(tri) : albedo);
    rec[0] = O.x; rec[1] = O.y; rec[2] = O.z;
    rec[3] = D.x; rec[4] = D.y; rec[5] = D.z;
    rec[6] = p.x; rec[7] = p.y; rec[8] = p.z;
    rec[9] = n.x; rec[10] = n.y; rec[11] = n.z;
    rec[12] = a[0]; rec[13] = a[1]; rec[14] = a[2];
    std::memcpy(&rec[15], &flags, 4);
    rec[16] = rec[17] = rec[18] = 1.0f;   // the camera ray: path weight 1, depth 0
    const uint32_t depth = sample << 16;
    std::memcpy(&rec[19], &depth, 4);
}

void SmokeBox::make_slice_record(int x, int y, float rec[kRecWords]) const
{
    V3 O, D, n, p;
    float mint;
    camera_ray((float)x + 0.5f, (float)y + 0.5f, &O, &D, &mint);
    int tri;
    float t = first_hit(O, D, mint, &n, &p, &tri);
    uint32_t flags = 0;
    V3 gp = p, gn = n;
    if (std::isfinite(t)) {
        flags = 1u;
        while (true) {   // Preprocessor.cpp:1157-1169
            gp = p; gn = n;
            if (mat(tri) != 2u) break;
            t = first_hit(O, D, t + 1e-4f, &n, &p, &tri);   // Ray(ray, its.t + Epsilon, ray.maxt)
            if (!std::isfinite(t)) break;
        }
    }
    for (int k = 0; k < kRecWords; k++) rec[k] = 0.0f;
    rec[0] = O.x; rec[1] = O.y; rec[2] = O.z;
    rec[3] = D.x; rec[4] = D.y; rec[5] = D.z;
    rec[6] = gp.x; rec[7] = gp.y; rec[8] = gp.z;
    rec[9] = gn.x; rec[10] = gn.y; rec[11] = gn.z;
    std::memcpy(&rec[15], &flags, 4);
    rec[16] = rec[17] = rec[18] = 1.0f;
}

float SmokeBox::scene_diagonal() const
{
    const float a = box_max[0] - box_min[0], b = box_max[1] - box_min[1], c = box_max[2] - box_min[2];
    return std::sqrt(a * a + b * b + c * c);
}

// ---------------------------------------------------------------- tracer --
namespace {

void philox(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

struct Stream {   // Sampler::next1D over the (dom, a, b, c) Philox stream
    uint32_t seed, pass, dom, a, b, c, k = 0, blk = 0xFFFFFFFFu;
    uint32_t buf[4];
    float next()
    {
        const uint32_t bl = k >> 2;
        if (bl != blk) {
            const uint32_t ctr[4] = {a, b, bl, (dom << 24) | (c & 0xFFFFFFu)};
            const uint32_t key[2] = {seed, pass};
            philox(ctr, key, buf);
            blk = bl;
        }
        union { uint32_t u; float f; } x;
        x.u = (buf[k & 3] >> 9) | 0x3f800000u;   // Random::nextFloat, random.cpp:630-639
        ++k;
        return x.f - 1.0f;
    }
};

V3 uniform_sphere(float sx, float sy)   // warp.cpp:25-31
{
    const float z = 1.0f - 2.0f * sy;
    const float r = safe_sqrt(1.0f - z * z);
    const float theta = (float)(2.0f * kPi * sx);
    // sin/cos in double, rounded once (the oracle and tracer.hip do the same)
    return v3(r * (float)std::cos((double)theta), r * (float)std::sin((double)theta), z);
}

V3 cosine_hemisphere(float sx, float sy)   // warp.cpp:43-52, 81-102
{
    const float r1 = 2.0f * sx - 1.0f, r2 = 2.0f * sy - 1.0f;
    float phi, r;
    if (r1 == 0 && r2 == 0) { r = phi = 0; }
    else if (r1 * r1 > r2 * r2) { r = r1; phi = (float)((kPi / 4.0f) * (r2 / r1)); }
    else { r = r2; phi = (float)((kPi / 2.0f) - (r1 / r2) * (kPi / 4.0f)); }
    const float px = r * (float)std::cos((double)phi), py = r * (float)std::sin((double)phi);
    float z = safe_sqrt(1.0f - px * px - py * py);
    if (z == 0) z = 1e-10f;
    return v3(px, py, z);
}

void frame_of(V3 a, V3* b, V3* c)   // coordinateSystem, util.cpp:592-601
{
    if (std::fabs(a.x) > std::fabs(a.y)) {
        const float invLen = 1.0f / std::sqrt(a.x * a.x + a.z * a.z);
        *c = v3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        const float invLen = 1.0f / std::sqrt(a.y * a.y + a.z * a.z);
        *c = v3(0.0f, a.z * invLen, -a.y * invLen);
    }
    *b = cross(*c, a);
}

struct Sink {   // vrlVector::put + the tracer's current VRL (vrlTracer.h:56-89, VRL.h:148-158)
    std::vector<float> s[9];
    V3 start;
    float power[3];
    bool sigma_s_zero;
    void put(V3 end)
    {
        if (sigma_s_zero) return;
        if (power[0] == 0 && power[1] == 0 && power[2] == 0) return;
        if (length(start - end) == 0) return;
        s[0].push_back(start.x); s[1].push_back(start.y); s[2].push_back(start.z);
        s[3].push_back(end.x); s[4].push_back(end.y); s[5].push_back(end.z);
        s[6].push_back(power[0]); s[7].push_back(power[1]); s[8].push_back(power[2]);
    }
    void end_current(V3 p)
    {
        if (length(start - p) == 0) return;
        put(p);
    }
    uint32_t size() const { return (uint32_t)s[0].size(); }
};

// sampleDistance's draws (homogeneous.cpp:277-296): the distance (INFINITY:
// no medium interaction) and, for 'maximum', the pdf of the sample
float sample_distance(const MediumParams& m, Stream& smp, float* pdf_max)
{
    float rnd = smp.next();
    const float w = m.sampling_weight;
    if (!(rnd < w)) return INFINITY;
    rnd /= w;
    if (m.strategy == 3) return m.maxexp_sample(1 - rnd, pdf_max);
    float density = m.density;
    if (m.strategy == 0) {   // a random channel each time
        int ch = (int)(smp.next() * 3);
        if (ch > 2) ch = 2;
        density = m.sigma_t[ch];
    }
    return -fastlog(1 - rnd) / density;
}

void trace_particle(const SmokeBox& sc, Stream& smp, bool short_vrls, int max_depth, int rr_depth, Sink& k)
{
    const MediumParams& m = sc.medium;
    const float sx = smp.next(), sy = smp.next();   // sampleEmitterPosition (scene.cpp:958-974)
    float power[3];
    const float dx = smp.next(), dy = smp.next();   // sampleDirection (point.cpp:99-106, area.cpp:115-123)
    V3 dir, o;
    if (sc.area_light()) {
        sc.sample_area_emission(sx, sy, dx, dy, &o, &dir, power);
    } else {
        for (int i = 0; i < 3; i++) power[i] = sc.light_intensity[i] * (float)(4 * kPi);
        dir = uniform_sphere(dx, dy);
        o = sc.light_pos;
    }
    if (power[0] == 0 && power[1] == 0 && power[2] == 0) return;
    k.start = o;
    for (int i = 0; i < 3; i++) k.power[i] = power[i];
    int depth = 1;
    float thr[3] = {1.0f, 1.0f, 1.0f};
    float eta = 1.0f;
    float mint = 1e-4f;   // Ray() default mint (Epsilon), then 0 after a medium and Epsilon after a surface
    while (!(thr[0] == 0 && thr[1] == 0 && thr[2] == 0) && (depth <= max_depth || max_depth < 0)) {
        V3 n, hp;
        int tri;
        const float its_t = sc.first_hit(o, dir, mint, &n, &hp, &tri);
        const bool its_valid = std::isfinite(its_t);
        // HomogeneousMedium::sampleDistance (homogeneous.cpp:275-352)
        float pdf_max = 0.0f;
        float sampled = sample_distance(m, smp, &pdf_max);
        const float distSurf = its_t - 0.0f;
        bool success = true;
        V3 mp = o;
        if (sampled < distSurf) {
            mp = o + dir * (sampled + 0.0f);
            if (mp.x == o.x && mp.y == o.y && mp.z == o.z) success = false;
        } else {
            sampled = distSurf;
            success = false;
        }
        float pf, ps;
        m.pdfs(sampled, pdf_max, &ps, &pf);
        float mtr[3];
        for (int i = 0; i < 3; i++) mtr[i] = fastexp(m.sigma_t[i] * (-sampled));
        {
            float mx = mtr[0] > mtr[1] ? mtr[0] : mtr[1];
            mx = mx > mtr[2] ? mx : mtr[2];
            if (mx < 1e-20f) mtr[0] = mtr[1] = mtr[2] = 0;
        }
        if (success) {   // vrlTracer.h:143-172
            const float rps = 1.0f / ps;
            for (int i = 0; i < 3; i++) thr[i] *= mtr[i] * m.sigma_s[i] * rps;
            const float px_ = smp.next(), py_ = smp.next();
            const V3 wo = uniform_sphere(px_, py_);
            const V3 endPoint = short_vrls ? mp : hp;
            k.end_current(endPoint);
            k.start = mp;
            for (int i = 0; i < 3; i++) k.power[i] = thr[i] * power[i];
            o = mp; dir = wo; mint = 0.0f;
        } else if (its_valid) {   // vrlTracer.h:173-213
            const float rpf = 1.0f / pf;
            for (int i = 0; i < 3; i++) thr[i] *= mtr[i] * rpf;
            const V3 p = hp;
            const float* alb = tri >= 0 ? sc.occ_albedo_of(tri) : sc.albedo;
            V3 fs, ft;
            frame_of(n, &fs, &ft);
            const V3 mwi = -dir;
            const float cos_wi = dot(mwi, n);
            const float bx = smp.next(), by = smp.next();   // bsdf->sample(bRec, next2D())
            float bw[3] = {0, 0, 0};
            V3 wol = v3(0, 0, 0);
            const uint32_t mt = sc.mat(tri);
            if (mt == 0u) {          // SmoothDiffuse::sample (diffuse.cpp:120-133)
                if (!(cos_wi <= 0)) {
                    wol = cosine_hemisphere(bx, by);
                    for (int i = 0; i < 3; i++) bw[i] = alb[i];
                }
            } else if (mt == 1u) {   // SmoothConductor::sample (conductor.cpp:254-268), material none
                if (!(cos_wi <= 0)) {
                    wol = v3(-dot(mwi, fs), -dot(mwi, ft), cos_wi);   // reflect(wi)
                    for (int i = 0; i < 3; i++) bw[i] = sc.occ_spec[i];
                }
            } else if (mt == 3u) {   // SmoothDielectric::sample, both components, EImportance (dielectric.cpp:335-364)
                float cos_t;
                const float F = fresnel_dielectric_ext(cos_wi, &cos_t, sc.occ_eta);
                if (bx <= F) {
                    wol = v3(-dot(mwi, fs), -dot(mwi, ft), cos_wi);
                } else {
                    const float inv_eta = 1 / sc.occ_eta;
                    const float scale = -(cos_t < 0 ? inv_eta : sc.occ_eta);   // refract(wi, cosThetaT)
                    wol = v3(scale * dot(mwi, fs), scale * dot(mwi, ft), cos_t);
                    eta *= cos_t < 0 ? sc.occ_eta : inv_eta;                   // bRec.eta
                }
                bw[0] = bw[1] = bw[2] = 1.0f;                                 // importance: factor 1
            } else {                 // Null::sample (null.cpp:53-63): wo = -wi
                wol = v3(-dot(mwi, fs), -dot(mwi, ft), -cos_wi);
                bw[0] = bw[1] = bw[2] = 1.0f;
            }
            if (bw[0] == 0 && bw[1] == 0 && bw[2] == 0) { k.end_current(p); break; }
            const V3 wo = (fs * wol.x + ft * wol.y) + n * wol.z;
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

}  // namespace

// TriMesh::prepareSamplingTable (trimesh.cpp:388-403): Triangle::surfaceArea
// (triangle.cpp: 0.5 |cross(p1 - p0, p2 - p0)|) appended to a
// DiscreteDistribution (running float sum), normalized (pmf.h:101-114)
void SmokeBox::prepare_emitter()
{
    const size_t n = emit.size() / 9;
    emit_cdf.assign(1, 0.0f);
    for (size_t i = 0; i < n; i++) {
        const float* t = &emit[9 * i];
        const V3 p0 = v3(t[0], t[1], t[2]), p1 = v3(t[3], t[4], t[5]), p2 = v3(t[6], t[7], t[8]);
        const float a = 0.5f * length(cross(p1 - p0, p2 - p0));
        emit_cdf.push_back(emit_cdf.back() + a);
    }
    emit_area = emit_cdf.back();
    if (emit_area > 0) {
        const float norm = 1.0f / emit_area;
        for (size_t i = 1; i < emit_cdf.size(); i++) emit_cdf[i] *= norm;
        emit_cdf.back() = 1.0f;
    }
}

void SmokeBox::sample_area_emission(float sx, float sy, float dx, float dy, V3* o, V3* d, float power[3]) const
{
    // Scene::sampleEmitterPosition: one emitter, so m_emitterPDF.sampleReuse
    // leaves sample.x as it is and the pdf is 1 (pmf.h:124-169)
    // TriMesh::samplePosition: the triangle by m_areaDistr.sampleReuse(sample.y)
    const size_t n = emit_cdf.size() - 1;
    size_t lb = (size_t)(std::lower_bound(emit_cdf.begin(), emit_cdf.end(), sy) - emit_cdf.begin());
    size_t idx = std::min(n - 1, (size_t)std::max((ptrdiff_t)0, (ptrdiff_t)lb - 1));
    // a zero-area triangle is skipped (the reference's loop would read past the table
    // if the last one had zero area)
    while (idx + 1 < n && emit_cdf[idx + 1] - emit_cdf[idx] == 0) ++idx;
    const float y = (sy - emit_cdf[idx]) / (emit_cdf[idx + 1] - emit_cdf[idx]);
    // Triangle::sample with warp::squareToUniformTriangle (warp.cpp:76-79)
    const float a = safe_sqrt(1.0f - sx);
    const float bx = 1 - a, by = a * y;
    const float* t = &emit[9 * idx];
    const V3 p0 = v3(t[0], t[1], t[2]), p1 = v3(t[3], t[4], t[5]), p2 = v3(t[6], t[7], t[8]);
    const V3 sideA = p1 - p0, sideB = p2 - p0;
    *o = (p0 + sideA * bx) + sideB * by;
    const V3 nn = normalize(cross(sideA, sideB));
    // AreaEmitter::samplePosition returns m_power = m_radiance * M_PI * area
    // (area.cpp:94-98, 198); sampleDirection: a cosine-weighted direction in
    // Frame(pRec.n), weight 1 (area.cpp:115-123)
    for (int i = 0; i < 3; i++) power[i] = (emit_radiance[i] * (float)kPi) * emit_area;
    const V3 l = cosine_hemisphere(dx, dy);
    V3 fs, ft;
    frame_of(nn, &fs, &ft);
    *d = (fs * l.x + ft * l.y) + nn * l.z;
}

void SmokeBox::pixel_sample(int x, int y, uint32_t seed, uint32_t pass, uint32_t sample, uint32_t spp, float* px,
                            float* py) const
{
    if (spp <= 1) {
        *px = (float)x + 0.5f;
        *py = (float)y + 0.5f;
        return;
    }
    Stream smp{seed, pass, kDomPixel, (uint32_t)y * (uint32_t)width + (uint32_t)x, sample, 0u};
    *px = (float)x + smp.next();
    *py = (float)y + smp.next();
}

void SmokeBox::make_chain(int x, int y, bool medium_scatters, uint32_t seed, uint32_t pass, int spec_rr_depth,
                          float init_throughput, std::vector<float>* out, uint32_t sample, uint32_t spp) const
{
    V3 O, D;
    float mint, px, py;
    pixel_sample(x, y, seed, pass, sample, spp, &px, &py);
    camera_ray(px, py, &O, &D, &mint);   // the sensor sample (integrator.cpp:240-247)
    const uint32_t pixel = (uint32_t)y * (uint32_t)width + (uint32_t)x;
    const float weight[3] = {1.0f, 1.0f, 1.0f};
    const float thr[3] = {init_throughput, init_throughput, init_throughput};   // throughputWithEtaSq (:381)
    uint32_t k = 0;
    chain_node(O, D, mint, weight, thr, 1, pixel, sample, medium_scatters, seed, pass, spec_rr_depth, out, &k);
}

// One LiInternal call (:398-524): the record of the ray's hit, then each
// delta component's continuation.  depth: rRec.depth (1 for the sensor ray).
void SmokeBox::chain_node(V3 O, V3 D, float mint, const float weight[3], const float thr[3], int depth,
                          uint32_t pixel, uint32_t sample, bool medium_scatters, uint32_t seed, uint32_t pass,
                          int spec_rr_depth, std::vector<float>* out, uint32_t* k) const
{
    if (*k >= 256) return;
    V3 n, p;
    int tri;
    const float t = first_hit(O, D, mint, &n, &p, &tri);
    if (!std::isfinite(t)) return;                                        // :414-419
    const uint32_t m = mat(tri);
    const uint32_t flags = 1u | (m == 0u ? 2u : 8u) | (medium_scatters ? 4u : 0u);
    const float* a = tri >= 0 ? occ_albedo_of(tri) : albedo;
    const size_t o = out->size();
    out->resize(o + kRecWords);
    float* rec = out->data() + o;
    rec[0] = O.x; rec[1] = O.y; rec[2] = O.z;
    rec[3] = D.x; rec[4] = D.y; rec[5] = D.z;
    rec[6] = p.x; rec[7] = p.y; rec[8] = p.z;
    rec[9] = n.x; rec[10] = n.y; rec[11] = n.z;
    for (int i = 0; i < 3; i++) rec[12 + i] = m == 0u ? a[i] : 0.0f;
    std::memcpy(&rec[15], &flags, 4);
    for (int i = 0; i < 3; i++) rec[16 + i] = weight[i];
    const uint32_t kw = *k | (sample << 16);
    std::memcpy(&rec[19], &kw, 4);
    ++*k;
    if (m == 0u) return;                                                  // no delta component (:447-448)
    // transmittance of the segment, rRec.medium->eval(Ray(ray, 0, its.t)) (:450-460)
    float tr[3];
    for (int i = 0; i < 3; i++) tr[i] = fastexp(medium.sigma_t[i] * (-t));
    {
        float mx = tr[0] > tr[1] ? tr[0] : tr[1];
        mx = mx > tr[2] ? mx : tr[2];
        if (mx < 1e-20f) tr[0] = tr[1] = tr[2] = 0;
    }
    if (tr[0] == 0 && tr[1] == 0 && tr[2] == 0) return;
    V3 fs, ft;
    frame_of(n, &fs, &ft);
    const V3 mwi = -D;
    const float cos_wi = dot(mwi, n);
    Stream smp{seed, pass, kDomEye, pixel, kw, 0u};
    const int ncomp = m == 3u ? 2 : 1;
    for (int c = 0; c < ncomp; c++) {   // the delta components (:467-511), bsdf->sample(bRec, Point2(0.5f))
        float bw[3];
        float beta = 1.0f;              // bRec.eta
        V3 wol;
        if (m == 1u) {                  // conductor.cpp:254-268
            if (cos_wi <= 0) continue;
            wol = v3(-dot(mwi, fs), -dot(mwi, ft), cos_wi);
            for (int i = 0; i < 3; i++) bw[i] = occ_spec[i];
        } else if (m == 2u) {           // null.cpp:53-63
            wol = v3(-dot(mwi, fs), -dot(mwi, ft), -cos_wi);
            bw[0] = bw[1] = bw[2] = 1.0f;
        } else {                        // dielectric.cpp:365-385, one component, ERadiance
            float cos_t;
            const float F = fresnel_dielectric_ext(cos_wi, &cos_t, occ_eta);
            const float inv_eta = 1 / occ_eta;
            if (c == 0) {
                wol = v3(-dot(mwi, fs), -dot(mwi, ft), cos_wi);
                bw[0] = bw[1] = bw[2] = F;
            } else {
                const float scale = -(cos_t < 0 ? inv_eta : occ_eta);
                wol = v3(scale * dot(mwi, fs), scale * dot(mwi, ft), cos_t);
                beta = cos_t < 0 ? occ_eta : inv_eta;
                const float factor = cos_t < 0 ? inv_eta : occ_eta;
                bw[0] = bw[1] = bw[2] = factor * factor * (1 - F);
            }
            if (bw[0] == 0) continue;
        }
        // Russian roulette (:480-492)
        float thr2[3];
        for (int i = 0; i < 3; i++) thr2[i] = ((thr[i] * tr[i]) * bw[i]) * (beta * beta);
        const float maxRR = depth >= spec_rr_depth ? 0.98f : 1.0f;
        float mx = thr2[0] > thr2[1] ? thr2[0] : thr2[1];
        mx = mx > thr2[2] ? mx : thr2[2];
        const float rrProb = maxRR < mx ? maxRR : mx;
        if (rrProb <= 0 || (rrProb < 1 && smp.next() > rrProb)) continue;
        float thr_c[3], w_c[3];
        for (int i = 0; i < 3; i++) {
            thr_c[i] = thr2[i] / rrProb;
            w_c[i] = ((weight[i] * tr[i]) * bw[i]) / rrProb;                  // weight * transmittance * bsdfWeight / rrProb (:505)
        }
        const V3 D2 = (fs * wol.x + ft * wol.y) + n * wol.z;                 // its.toWorld(bRec.wo)
        // RayDifferential(its.p, wo): mint = Epsilon
        chain_node(p, D2, 1e-4f, w_c, thr_c, depth + 1, pixel, sample, medium_scatters, seed, pass, spec_rr_depth,
                   out, k);
    }
}

VrlSet trace_vrls(const SmokeBox& sc, uint32_t seed, uint32_t pass, uint32_t target, bool short_vrls,
                  int max_depth, int rr_depth)
{
    Sink k;
    const MediumParams& m = sc.medium;
    k.sigma_s_zero = (m.sigma_s[0] == 0 && m.sigma_s[1] == 0 && m.sigma_s[2] == 0);
    uint64_t p = 0;
    while (k.size() < target) {   // vrlTracer::randomWalk, vrlTracer.h:29-39
        Stream smp{seed, pass, kDomTracer, (uint32_t)p, (uint32_t)(p >> 32), 0u};
        p++;   // handleEmission -> nextParticle (the point light always emits)
        trace_particle(sc, smp, short_vrls, max_depth, rr_depth, k);
        if (k.sigma_s_zero && p > 1000000) break;
    }
    VrlSet out;
    out.n = k.size();
    out.particle_count = p;
    out.soa.resize(9 * (size_t)out.n);
    for (int pl = 0; pl < 9; pl++)
        std::memcpy(&out.soa[(size_t)pl * out.n], k.s[pl].data(), sizeof(float) * out.n);
    return out;
}

bool read_vrl_file(const char* path, const MediumParams& m, VrlSet* out, std::string* err)
{
    std::ifstream f(path);
    if (!f) { *err = std::string("cannot open VRL file ") + path; return false; }
    Sink k;
    k.sigma_s_zero = (m.sigma_s[0] == 0 && m.sigma_s[1] == 0 && m.sigma_s[2] == 0);
    std::string line;
    while (std::getline(f, line)) {
        std::stringstream ss(line);
        float v[9];
        int got = 0;
        while (got < 9 && (ss >> v[got])) got++;
        if (got == 0) continue;
        if (got != 9) break;   // the reference stops at the first unparsable line (VRL.h:121-126)
        for (int i = 6; i < 9; i++)
            if (!std::isfinite(v[i]) || v[i] < 0) { *err = "invalid parsed VRL power"; return false; }   // VRL.h:51-53
        k.start = v3(v[0], v[1], v[2]);
        k.power[0] = v[6]; k.power[1] = v[7]; k.power[2] = v[8];
        k.put(v3(v[3], v[4], v[5]));
    }
    out->n = k.size();
    out->particle_count = out->n;   // m_numParticles = size() (VRL.h:127)
    out->soa.resize(9 * (size_t)out->n);
    for (int pl = 0; pl < 9; pl++)
        std::memcpy(&out->soa[(size_t)pl * out->n], k.s[pl].data(), sizeof(float) * out->n);
    return true;
}

bool write_vrl_file(const char* path, const VrlSet& v, std::string* err)
{
    FILE* f = std::fopen(path, "w");
    if (!f) { *err = std::string("cannot write VRL file ") + path; return false; }
    for (uint32_t i = 0; i < v.n; i++) {
        for (int pl = 0; pl < 9; pl++)
            std::fprintf(f, pl ? " %.9g" : "%.9g", (double)v.soa[(size_t)pl * v.n + i]);
        std::fputc('\n', f);
    }
    std::fclose(f);
    return true;
}

}  // namespace host
}  // namespace alvrl
