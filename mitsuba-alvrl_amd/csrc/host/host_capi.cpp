// host_capi.cpp -- C ABI of the host harness (include/alvrl_host.h): scene
// records, VRL tracer, VRL file I/O.  The integrator pipeline entry points
// live in integrator.hip (they drive the device).
#include "alvrl_host.h"

#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>

#include "scene.hpp"

using namespace alvrl::host;

namespace alvrl {
namespace host {
thread_local std::string g_host_err;
// HomogeneousMedium(props) of a descriptor, unresolved (MediumParams::problem, resolve)
MediumParams medium_of(const alvrl_medium_desc& d)
{
    MediumParams m;
    for (int i = 0; i < 3; i++) { m.sigma_s[i] = d.sigma_s[i]; m.sigma_a[i] = d.sigma_a[i]; }
    m.sampling_weight = d.sampling_weight;
    m.phase_type = d.phase_type;
    m.phase_g = d.phase_g;
    m.strategy = d.strategy;
    m.channel = d.channel;
    m.density = d.sampling_density;
    return m;
}
// what is wrong with a scene descriptor, or nullptr
const char* scene_problem(const alvrl_scene_desc& s)
{
    if (s.width <= 0 || s.height <= 0) return "alvrl_scene_desc: width and height must be > 0";
    if (const char* m = medium_of(s.medium).problem()) return m;
    if (s.n_occluders && !s.occluders) return "alvrl_scene_desc: n_occluders > 0 without occluders";
    if (s.occluders && s.occluder_material)
        for (uint32_t i = 0; i < s.n_occluders; i++)
            if (s.occluder_material[i] > ALVRL_MAT_DIELECTRIC) return "alvrl_scene_desc: unknown occluder material";
    if (s.n_emitter_tris && !s.emitter_tris) return "alvrl_scene_desc: n_emitter_tris > 0 without emitter_tris";
    if (s.occluders && s.occluder_albedos)
        for (size_t i = 0; i < 3 * (size_t)s.n_occluders; i++)
            if (!(s.occluder_albedos[i] >= 0.0f && s.occluder_albedos[i] <= 1.0f))
                return "alvrl_scene_desc: occluder_albedos must lie in [0, 1]";
    if (s.n_emitter_tris) {
        for (size_t i = 0; i < 9 * (size_t)s.n_emitter_tris; i++)
            if (!std::isfinite(s.emitter_tris[i])) return "alvrl_scene_desc: non-finite emitter vertex";
        for (int i = 0; i < 3; i++)
            if (!std::isfinite(s.emitter_radiance[i]) || s.emitter_radiance[i] < 0)
                return "alvrl_scene_desc: emitter radiance must be finite and >= 0";
        SmokeBox b;
        b.emit.assign(s.emitter_tris, s.emitter_tris + 9 * (size_t)s.n_emitter_tris);
        b.prepare_emitter();
        if (!(b.emit_area > 0)) return "alvrl_scene_desc: the emitter triangles have no area";
    }
    return nullptr;
}
SmokeBox to_box(const alvrl_scene_desc& s)
{
    SmokeBox b;
    b.cam_origin = v3(s.cam_origin[0], s.cam_origin[1], s.cam_origin[2]);
    b.cam_target = v3(s.cam_target[0], s.cam_target[1], s.cam_target[2]);
    b.cam_up = v3(s.cam_up[0], s.cam_up[1], s.cam_up[2]);
    b.fov_x_deg = s.fov_x_deg;
    b.width = s.width; b.height = s.height;
    for (int i = 0; i < 3; i++) {
        b.box_min[i] = s.box_min[i]; b.box_max[i] = s.box_max[i];
        b.albedo[i] = s.albedo[i]; b.light_intensity[i] = s.light_intensity[i];
    }
    b.light_pos = v3(s.light_pos[0], s.light_pos[1], s.light_pos[2]);
    b.medium = medium_of(s.medium);
    b.medium.resolve();
    if (s.occluders && s.n_occluders) b.occ.assign(s.occluders, s.occluders + 9 * (size_t)s.n_occluders);
    for (int i = 0; i < 3; i++) b.occ_albedo[i] = s.occluder_albedo[i];
    if (s.occluders && s.n_occluders && s.occluder_albedos)
        b.occ_alb.assign(s.occluder_albedos, s.occluder_albedos + 3 * (size_t)s.n_occluders);
    if (s.occluders && s.n_occluders && s.occluder_material)
        b.occ_mat.assign(s.occluder_material, s.occluder_material + s.n_occluders);
    for (int i = 0; i < 3; i++) b.occ_spec[i] = s.occluder_specular[i];
    if (s.occluder_eta > 0) b.occ_eta = s.occluder_eta;
    if (s.emitter_tris && s.n_emitter_tris) {
        b.emit.assign(s.emitter_tris, s.emitter_tris + 9 * (size_t)s.n_emitter_tris);
        for (int i = 0; i < 3; i++) b.emit_radiance[i] = s.emitter_radiance[i];
        b.prepare_emitter();
    }
    return b;
}
}  // namespace host
}  // namespace alvrl

static int herr(int code, const std::string& m)
{
    g_host_err = m;
    return code;
}

extern "C" {

ALVRL_API void alvrl_scene_default(alvrl_scene_desc* s, int width, int height)
{
    std::memset(s, 0, sizeof(*s));
    const SmokeBox b;
    s->cam_origin[0] = b.cam_origin.x; s->cam_origin[1] = b.cam_origin.y; s->cam_origin[2] = b.cam_origin.z;
    s->cam_target[0] = b.cam_target.x; s->cam_target[1] = b.cam_target.y; s->cam_target[2] = b.cam_target.z;
    s->cam_up[0] = b.cam_up.x; s->cam_up[1] = b.cam_up.y; s->cam_up[2] = b.cam_up.z;
    s->fov_x_deg = b.fov_x_deg;
    s->width = width; s->height = height;
    for (int i = 0; i < 3; i++) {
        s->box_min[i] = b.box_min[i]; s->box_max[i] = b.box_max[i];
        s->albedo[i] = b.albedo[i]; s->light_intensity[i] = b.light_intensity[i];
        s->medium.sigma_s[i] = b.medium.sigma_s[i]; s->medium.sigma_a[i] = b.medium.sigma_a[i];
    }
    s->light_pos[0] = b.light_pos.x; s->light_pos[1] = b.light_pos.y; s->light_pos[2] = b.light_pos.z;
    s->medium.sampling_weight = -1.0f;
    s->medium.phase_type = 0;
    s->medium.phase_g = 0.0f;
    s->occluders = nullptr;
    s->n_occluders = 0;
    for (int i = 0; i < 3; i++) s->occluder_albedo[i] = b.occ_albedo[i];
    s->occluder_material = nullptr;
    for (int i = 0; i < 3; i++) s->occluder_specular[i] = b.occ_spec[i];
    s->occluder_eta = b.occ_eta;
}

ALVRL_API int alvrl_scene_records(const alvrl_scene_desc* s, int medium_scatters, const uint32_t* ids,
                                  uint32_t n, alvrl_gather_rec* out)
{
    if (!s || (!out && n)) return herr(ALVRL_ERR_INVALID, "alvrl_scene_records: null argument");
    if (const char* m = scene_problem(*s)) return herr(ALVRL_ERR_INVALID, m);
    const SmokeBox b = to_box(*s);
    const uint64_t npix = (uint64_t)b.width * (uint64_t)b.height;
    if (!ids && n != npix) return herr(ALVRL_ERR_INVALID, "alvrl_scene_records: n must be W*H without pixel ids");
    const bool scat = medium_scatters && !(b.medium.sigma_s[0] == 0 && b.medium.sigma_s[1] == 0 && b.medium.sigma_s[2] == 0);
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t p = ids ? ids[i] : i;
        if (p >= npix) return herr(ALVRL_ERR_INVALID, "alvrl_scene_records: pixel id out of range");
        b.make_record((int)(p % (uint32_t)b.width), (int)(p / (uint32_t)b.width), scat,
                      reinterpret_cast<float*>(&out[i]));
    }
    return ALVRL_OK;
}

ALVRL_API int alvrl_scene_records_spp(const alvrl_scene_desc* s, int medium_scatters, uint32_t seed, uint32_t pass,
                                      uint32_t spp, const uint32_t* ids, uint32_t n, alvrl_gather_rec* out)
{
    if (!s || (!out && n)) return herr(ALVRL_ERR_INVALID, "alvrl_scene_records_spp: null argument");
    if (spp == 0 || (uint64_t)spp * n > 0xFFFFFFFFull || spp > 0xFFFFu)
        return herr(ALVRL_ERR_INVALID, "alvrl_scene_records_spp: spp out of range");
    if (const char* m = scene_problem(*s)) return herr(ALVRL_ERR_INVALID, m);
    const SmokeBox b = to_box(*s);
    const uint64_t npix = (uint64_t)b.width * (uint64_t)b.height;
    if (!ids && n != npix) return herr(ALVRL_ERR_INVALID, "alvrl_scene_records_spp: n must be W*H without pixel ids");
    const bool scat = medium_scatters && !(b.medium.sigma_s[0] == 0 && b.medium.sigma_s[1] == 0 && b.medium.sigma_s[2] == 0);
    for (uint32_t j = 0; j < spp; j++)
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t p = ids ? ids[i] : i;
            if (p >= npix) return herr(ALVRL_ERR_INVALID, "alvrl_scene_records_spp: pixel id out of range");
            b.make_record((int)(p % (uint32_t)b.width), (int)(p / (uint32_t)b.width), scat,
                          reinterpret_cast<float*>(&out[(size_t)j * n + i]), seed, pass, j, spp);
        }
    return ALVRL_OK;
}

ALVRL_API int alvrl_scene_chain(const alvrl_scene_desc* s, int medium_scatters, uint32_t seed, uint32_t pass,
                                int spec_rr_depth, float init_throughput, int x, int y, alvrl_gather_rec* out,
                                uint32_t cap, uint32_t* n)
{
    return alvrl_scene_chain_spp(s, medium_scatters, seed, pass, spec_rr_depth, init_throughput, x, y, 0, 1, out,
                                 cap, n);
}

ALVRL_API int alvrl_scene_chain_spp(const alvrl_scene_desc* s, int medium_scatters, uint32_t seed, uint32_t pass,
                                    int spec_rr_depth, float init_throughput, int x, int y, uint32_t sample,
                                    uint32_t spp, alvrl_gather_rec* out, uint32_t cap, uint32_t* n)
{
    if (spp == 0 || sample >= spp || spp > 0xFFFFu) return herr(ALVRL_ERR_INVALID, "alvrl_scene_chain: sample out of range");
    if (!s || !n || (!out && cap)) return herr(ALVRL_ERR_INVALID, "alvrl_scene_chain: null argument");
    if (const char* m = scene_problem(*s)) return herr(ALVRL_ERR_INVALID, m);
    const SmokeBox b = to_box(*s);
    if (x < 0 || y < 0 || x >= b.width || y >= b.height) return herr(ALVRL_ERR_INVALID, "alvrl_scene_chain: pixel out of range");
    const bool scat = medium_scatters && !(b.medium.sigma_s[0] == 0 && b.medium.sigma_s[1] == 0 && b.medium.sigma_s[2] == 0);
    std::vector<float> recs;
    b.make_chain(x, y, scat, seed, pass, spec_rr_depth, init_throughput, &recs, sample, spp);
    const uint32_t k = (uint32_t)(recs.size() / kRecWords);
    *n = k;
    if (k > cap) return herr(ALVRL_ERR_INVALID, "alvrl_scene_chain: capacity too small");
    if (k) std::memcpy(out, recs.data(), sizeof(float) * recs.size());
    return ALVRL_OK;
}

ALVRL_API int alvrl_scene_slice_record(const alvrl_scene_desc* s, int x, int y, alvrl_gather_rec* out)
{
    if (!s || !out) return herr(ALVRL_ERR_INVALID, "alvrl_scene_slice_record: null argument");
    if (const char* m = scene_problem(*s)) return herr(ALVRL_ERR_INVALID, m);
    const SmokeBox b = to_box(*s);
    if (x < 0 || y < 0 || x >= b.width || y >= b.height) return herr(ALVRL_ERR_INVALID, "alvrl_scene_slice_record: pixel out of range");
    b.make_slice_record(x, y, reinterpret_cast<float*>(out));
    return ALVRL_OK;
}

ALVRL_API int alvrl_tile_pixels(int width, int height, uint32_t rank, uint32_t world, uint32_t* out,
                                uint32_t cap, uint32_t* n)
{
    if (!n || width < 0 || height < 0) return herr(ALVRL_ERR_INVALID, "alvrl_tile_pixels: bad argument");
    if (world == 0 || rank >= world) return herr(ALVRL_ERR_INVALID, "alvrl_tile_pixels: bad rank/world");
    const int T = 64;
    const int tx = (width + T - 1) / T, ty = (height + T - 1) / T;
    uint32_t k = 0;
    for (int t = 0; t < tx * ty; t++) {
        if ((uint32_t)t % world != rank) continue;
        const int x0 = (t % tx) * T, y0 = (t / tx) * T;
        const int x1 = x0 + T < width ? x0 + T : width, y1 = y0 + T < height ? y0 + T : height;
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) {
                if (out && k < cap) out[k] = (uint32_t)(y * width + x);
                k++;
            }
    }
    *n = k;
    if (out && k > cap) return herr(ALVRL_ERR_INVALID, "alvrl_tile_pixels: capacity too small");
    return ALVRL_OK;
}

ALVRL_API int alvrl_trace_vrls(const alvrl_scene_desc* s, uint32_t seed, uint32_t pass, uint32_t target,
                               int short_vrls, int max_depth, int rr_depth, float* soa, uint32_t cap,
                               uint32_t* n, uint64_t* particles)
{
    if (!s || !soa || !n || !particles) return herr(ALVRL_ERR_INVALID, "alvrl_trace_vrls: null argument");
    if (const char* m = scene_problem(*s)) return herr(ALVRL_ERR_INVALID, m);
    const SmokeBox b = to_box(*s);
    const VrlSet v = trace_vrls(b, seed, pass, target, short_vrls != 0, max_depth, rr_depth);
    if (v.n > cap) return herr(ALVRL_ERR_INVALID, "alvrl_trace_vrls: capacity too small (" + std::to_string(v.n) + " VRLs)");
    for (int pl = 0; pl < 9; pl++)
        std::memcpy(soa + (size_t)pl * cap, v.soa.data() + (size_t)pl * v.n, sizeof(float) * v.n);
    *n = v.n;
    *particles = v.particle_count;
    return ALVRL_OK;
}

ALVRL_API int alvrl_read_vrl_file(const char* path, const alvrl_medium_desc* m, float* soa, uint32_t cap,
                                  uint32_t* n, uint64_t* particles)
{
    if (!path || !m || !n || !particles) return herr(ALVRL_ERR_INVALID, "alvrl_read_vrl_file: null argument");
    MediumParams mp;
    for (int i = 0; i < 3; i++) { mp.sigma_s[i] = m->sigma_s[i]; mp.sigma_a[i] = m->sigma_a[i]; }
    mp.resolve();
    VrlSet v;
    std::string err;
    if (!read_vrl_file(path, mp, &v, &err)) return herr(ALVRL_ERR_INVALID, err);
    *n = v.n;
    *particles = v.particle_count;
    if (!soa) return ALVRL_OK;   // size query
    if (v.n > cap) return herr(ALVRL_ERR_INVALID, "alvrl_read_vrl_file: capacity too small");
    for (int pl = 0; pl < 9; pl++)
        std::memcpy(soa + (size_t)pl * cap, v.soa.data() + (size_t)pl * v.n, sizeof(float) * v.n);
    return ALVRL_OK;
}

ALVRL_API int alvrl_write_vrl_file(const char* path, const float* soa, uint32_t n)
{
    if (!path || (!soa && n)) return herr(ALVRL_ERR_INVALID, "alvrl_write_vrl_file: null argument");
    VrlSet v;
    v.n = n;
    v.soa.assign(soa, soa + 9 * (size_t)n);
    std::string err;
    if (!write_vrl_file(path, v, &err)) return herr(ALVRL_ERR_INVALID, err);
    return ALVRL_OK;
}

ALVRL_API const char* alvrl_host_last_error(void) { return g_host_err.c_str(); }

}  // extern "C"
