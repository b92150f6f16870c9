// formats.cpp -- on-disk formats around the vrl integrator,
// C ABI in include/alvrl_host.h:
//  * vrlClusterInfo stream layout (vrlIntegrator.cpp:29-101), so cluster lists
//    can be checkpointed and handed to another process, as the reference hands
//    m_ci to remote workers (bindUsedResources / wakeup, :353-354);
//  * uncompressed scanline OpenEXR (the hdrfilm output of a pass) and its
//    reader for this writer's files;
//  * mtsutil rms (src/utils/rms.cpp) and the dumpPass file name
//    (integrator.cpp:361-378 + vrlIntegrator::passFileSuffix, :357-364).
#include "alvrl_host.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iomanip>
#include <sstream>
#include <string>
#include <vector>

namespace alvrl {
namespace host {
extern thread_local std::string g_host_err;
}
}  // namespace alvrl
using alvrl::host::g_host_err;

namespace {

int ferr(int code, const std::string& m)
{
    g_host_err = m;
    return code;
}

// Mitsuba Stream primitives in little-endian order (a FileStream on x86 is
// host order): writeULong = 8 bytes, writeUInt = 4, writeFloat = 4 (Float is
// single precision in the reference's builds).
struct Out {
    std::vector<unsigned char> b;
    void u64(uint64_t v) { for (int i = 0; i < 8; i++) b.push_back((unsigned char)(v >> (8 * i))); }
    void u32(uint32_t v) { for (int i = 0; i < 4; i++) b.push_back((unsigned char)(v >> (8 * i))); }
    void f32(float f) { uint32_t v; std::memcpy(&v, &f, 4); u32(v); }
    void i32(int32_t v) { u32((uint32_t)v); }
    void u8(uint8_t v) { b.push_back(v); }
    void str(const char* s) { while (*s) b.push_back((unsigned char)*s++); b.push_back(0); }
};
struct In {
    const unsigned char* p;
    size_t n, o = 0;
    bool ok = true;
    bool need(size_t k) { if (o + k > n) ok = false; return ok; }
    uint64_t u64() { if (!need(8)) return 0; uint64_t v = 0; for (int i = 0; i < 8; i++) v |= (uint64_t)p[o + i] << (8 * i); o += 8; return v; }
    uint32_t u32() { if (!need(4)) return 0; uint32_t v = 0; for (int i = 0; i < 4; i++) v |= (uint32_t)p[o + i] << (8 * i); o += 4; return v; }
    float f32() { const uint32_t v = u32(); float f; std::memcpy(&f, &v, 4); return f; }
};

bool read_file(const char* path, std::vector<unsigned char>* out)
{
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    unsigned char buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof(buf), f)) > 0) out->insert(out->end(), buf, buf + k);
    std::fclose(f);
    return true;
}
bool write_file(const char* path, const std::vector<unsigned char>& b)
{
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    const bool ok = std::fwrite(b.data(), 1, b.size(), f) == b.size();
    return std::fclose(f) == 0 && ok;
}

}  // namespace

struct alvrl_cluster_info {
    std::vector<uint32_t> slices;                 // m_slices, y + H*x
    std::vector<uint32_t> slice_off, reps;        // m_selectedVrls as CSR
    std::vector<float> weights;                   // m_clusterWeight, same CSR
    std::vector<uint32_t> gc_reps, fb_reps;
    std::vector<float> gc_w, fb_w;
};

extern "C" {

ALVRL_API int alvrl_cluster_info_write(const char* path, uint32_t npix, const uint32_t* pixel_to_slice,
                                       uint32_t nslices, const uint32_t* slice_off, const uint32_t* reps,
                                       const float* weights, uint32_t n_global, const uint32_t* global_reps,
                                       const float* global_w, uint32_t n_fb, const uint32_t* fb_reps,
                                       const float* fb_w)
{
    if (!path || (npix && !pixel_to_slice) || (nslices && (!slice_off || !reps || !weights)) ||
        (n_global && (!global_reps || !global_w)) || (n_fb && (!fb_reps || !fb_w)))
        return ferr(ALVRL_ERR_INVALID, "alvrl_cluster_info_write: null argument");
    Out o;
    o.u64(npix);
    for (uint32_t i = 0; i < npix; i++) o.u32(pixel_to_slice[i]);
    o.u64(nslices);                                  // m_selectedVrls
    for (uint32_t s = 0; s < nslices; s++) {
        if (slice_off[s + 1] < slice_off[s]) return ferr(ALVRL_ERR_INVALID, "alvrl_cluster_info_write: bad slice_off");
        o.u64(slice_off[s + 1] - slice_off[s]);
        for (uint32_t j = slice_off[s]; j < slice_off[s + 1]; j++) o.u32(reps[j]);
    }
    o.u64(nslices);                                  // m_clusterWeight
    for (uint32_t s = 0; s < nslices; s++) {
        o.u64(slice_off[s + 1] - slice_off[s]);
        for (uint32_t j = slice_off[s]; j < slice_off[s + 1]; j++) o.f32(weights[j]);
    }
    o.u64(n_global);
    for (uint32_t i = 0; i < n_global; i++) o.u32(global_reps[i]);
    o.u64(n_global);
    for (uint32_t i = 0; i < n_global; i++) o.f32(global_w[i]);
    o.u64(n_fb);
    for (uint32_t i = 0; i < n_fb; i++) o.u32(fb_reps[i]);
    o.u64(n_fb);
    for (uint32_t i = 0; i < n_fb; i++) o.f32(fb_w[i]);
    if (!write_file(path, o.b)) return ferr(ALVRL_ERR_INVALID, std::string("cannot write ") + path);
    return ALVRL_OK;
}

// The reader of vrlClusterInfo(Stream*, InstanceManager*) with its slip at
// :56-59 fixed: the fall-back representatives are read into m_fallBackVrls
// (the reference reads them into m_fallBackWeight and then overwrites it).
ALVRL_API int alvrl_cluster_info_read(const char* path, alvrl_cluster_info** out)
{
    if (!path || !out) return ferr(ALVRL_ERR_INVALID, "alvrl_cluster_info_read: null argument");
    std::vector<unsigned char> b;
    if (!read_file(path, &b)) return ferr(ALVRL_ERR_INVALID, std::string("cannot open ") + path);
    In in{b.data(), b.size()};
    auto* ci = new alvrl_cluster_info();
    auto cnt = [&](uint64_t per) -> uint64_t {       // a count whose payload must fit the file
        const uint64_t n = in.u64();
        if (in.ok && n > (in.n - in.o) / per) in.ok = false;
        return in.ok ? n : 0;
    };
    const uint64_t np = cnt(4);
    ci->slices.resize(np);
    for (auto& v : ci->slices) v = in.u32();
    const uint64_t ns = cnt(8);
    ci->slice_off.assign(1, 0);
    for (uint64_t s = 0; s < ns && in.ok; s++) {
        const uint64_t k = cnt(4);
        for (uint64_t j = 0; j < k; j++) ci->reps.push_back(in.u32());
        ci->slice_off.push_back((uint32_t)ci->reps.size());
    }
    const uint64_t nw = cnt(8);
    if (in.ok && nw != ns) in.ok = false;
    for (uint64_t s = 0; s < nw && in.ok; s++) {
        const uint64_t k = cnt(4);
        if (k != ci->slice_off[s + 1] - ci->slice_off[s]) { in.ok = false; break; }
        for (uint64_t j = 0; j < k; j++) ci->weights.push_back(in.f32());
    }
    uint64_t k = cnt(4);
    for (uint64_t i = 0; i < k; i++) ci->gc_reps.push_back(in.u32());
    k = cnt(4);
    for (uint64_t i = 0; i < k; i++) ci->gc_w.push_back(in.f32());
    k = cnt(4);
    for (uint64_t i = 0; i < k; i++) ci->fb_reps.push_back(in.u32());
    k = cnt(4);
    for (uint64_t i = 0; i < k; i++) ci->fb_w.push_back(in.f32());
    if (!in.ok || in.o != in.n || ci->gc_reps.size() != ci->gc_w.size() || ci->fb_reps.size() != ci->fb_w.size()) {
        delete ci;
        return ferr(ALVRL_ERR_INVALID, std::string("malformed vrlClusterInfo stream: ") + path);
    }
    *out = ci;
    return ALVRL_OK;
}

ALVRL_API void alvrl_cluster_info_free(alvrl_cluster_info* ci) { delete ci; }

ALVRL_API int alvrl_cluster_info_sizes(const alvrl_cluster_info* ci, uint32_t* npix, uint32_t* nslices,
                                       uint32_t* nreps, uint32_t* n_global, uint32_t* n_fb)
{
    if (!ci) return ferr(ALVRL_ERR_INVALID, "alvrl_cluster_info_sizes: null argument");
    if (npix) *npix = (uint32_t)ci->slices.size();
    if (nslices) *nslices = (uint32_t)ci->slice_off.size() - 1;
    if (nreps) *nreps = (uint32_t)ci->reps.size();
    if (n_global) *n_global = (uint32_t)ci->gc_reps.size();
    if (n_fb) *n_fb = (uint32_t)ci->fb_reps.size();
    return ALVRL_OK;
}

ALVRL_API int alvrl_cluster_info_get(const alvrl_cluster_info* ci, uint32_t* pixel_to_slice, uint32_t* slice_off,
                                     uint32_t* reps, float* weights, uint32_t* global_reps, float* global_w,
                                     uint32_t* fb_reps, float* fb_w)
{
    if (!ci) return ferr(ALVRL_ERR_INVALID, "alvrl_cluster_info_get: null argument");
    auto cp = [](const auto& v, auto* dst) { if (dst) std::copy(v.begin(), v.end(), dst); };
    cp(ci->slices, pixel_to_slice);
    cp(ci->slice_off, slice_off);
    cp(ci->reps, reps);
    cp(ci->weights, weights);
    cp(ci->gc_reps, global_reps);
    cp(ci->gc_w, global_w);
    cp(ci->fb_reps, fb_reps);
    cp(ci->fb_w, fb_w);
    return ALVRL_OK;
}

// ---------------------------------------------------------------- EXR --
// Single-part scanline OpenEXR, NO_COMPRESSION, one scanline per block,
// channels B, G, R (alphabetical, as the format requires), FLOAT or HALF.
namespace {
uint16_t f2h(float f)
{
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t mant = x & 0x7FFFFFu;
    int exp = (int)((x >> 23) & 0xFF);
    if (exp == 255) return (uint16_t)(sign | 0x7C00u | (mant ? 0x200u : 0u));
    exp = exp - 127 + 15;
    if (exp >= 31) return (uint16_t)(sign | 0x7C00u);
    if (exp <= 0) {
        if (exp < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        const int shift = 14 - exp;
        uint32_t h = mant >> shift;
        const uint32_t rem = mant & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) h++;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)exp << 10) | (mant >> 13);
    const uint32_t rem = mant & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;   // round to nearest even (may carry into exp)
    return (uint16_t)(sign | h);
}
float h2f(uint16_t h)
{
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1Fu, mant = h & 0x3FFu, x;
    if (exp == 0) {
        if (mant == 0) x = sign;
        else {
            exp = 127 - 15 + 1;
            while (!(mant & 0x400u)) { mant <<= 1; exp--; }
            x = sign | (exp << 23) | ((mant & 0x3FFu) << 13);
        }
    } else if (exp == 31) x = sign | 0x7F800000u | (mant << 13);
    else x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    float f;
    std::memcpy(&f, &x, 4);
    return f;
}
}  // namespace

ALVRL_API int alvrl_write_exr(const char* path, const float* rgb, int width, int height, int half)
{
    if (!path || !rgb || width <= 0 || height <= 0) return ferr(ALVRL_ERR_INVALID, "alvrl_write_exr: bad argument");
    Out o;
    o.u32(20000630u);                 // magic 76 2f 31 01
    o.u32(2u);                        // version 2, single-part scanline
    const int32_t pt = half ? 1 : 2;  // HALF / FLOAT
    o.str("channels"); o.str("chlist");
    o.i32(3 * (2 + 16) + 1);
    for (const char* c : {"B", "G", "R"}) { o.str(c); o.i32(pt); o.u8(0); o.u8(0); o.u8(0); o.u8(0); o.i32(1); o.i32(1); }
    o.u8(0);
    o.str("compression"); o.str("compression"); o.i32(1); o.u8(0);
    o.str("dataWindow"); o.str("box2i"); o.i32(16); o.i32(0); o.i32(0); o.i32(width - 1); o.i32(height - 1);
    o.str("displayWindow"); o.str("box2i"); o.i32(16); o.i32(0); o.i32(0); o.i32(width - 1); o.i32(height - 1);
    o.str("lineOrder"); o.str("lineOrder"); o.i32(1); o.u8(0);
    o.str("pixelAspectRatio"); o.str("float"); o.i32(4); o.f32(1.0f);
    o.str("screenWindowCenter"); o.str("v2f"); o.i32(8); o.f32(0.0f); o.f32(0.0f);
    o.str("screenWindowWidth"); o.str("float"); o.i32(4); o.f32(1.0f);
    o.u8(0);
    const size_t bpc = half ? 2 : 4;
    const uint64_t line = 8 + 3 * bpc * (size_t)width;
    const uint64_t table = o.b.size();
    for (int y = 0; y < height; y++) o.u64(table + 8 * (uint64_t)height + line * (uint64_t)y);
    for (int y = 0; y < height; y++) {
        o.i32(y);
        o.i32((int32_t)(3 * bpc * (size_t)width));
        for (int c = 2; c >= 0; c--)          // B, G, R
            for (int x = 0; x < width; x++) {
                const float v = rgb[3 * ((size_t)y * width + x) + c];
                if (half) { const uint16_t h = f2h(v); o.u8((uint8_t)h); o.u8((uint8_t)(h >> 8)); }
                else o.f32(v);
            }
    }
    if (!write_file(path, o.b)) return ferr(ALVRL_ERR_INVALID, std::string("cannot write ") + path);
    return ALVRL_OK;
}

// Reads the files alvrl_write_exr writes (uncompressed scanline, B/G/R).
ALVRL_API int alvrl_read_exr(const char* path, float* rgb, uint64_t cap_floats, int* width, int* height)
{
    if (!path || !width || !height) return ferr(ALVRL_ERR_INVALID, "alvrl_read_exr: null argument");
    std::vector<unsigned char> b;
    if (!read_file(path, &b)) return ferr(ALVRL_ERR_INVALID, std::string("cannot open ") + path);
    In in{b.data(), b.size()};
    if (in.u32() != 20000630u || (in.u32() & 0xFFu) != 2u) return ferr(ALVRL_ERR_INVALID, "not an OpenEXR file");
    int32_t w = 0, h = 0, pt = -1, comp = -1;
    auto cstr = [&]() { std::string s; while (in.need(1) && b[in.o]) s += (char)b[in.o++]; in.o++; return s; };
    while (in.ok) {
        const std::string name = cstr();
        if (name.empty()) break;
        const std::string type = cstr();
        const int32_t size = (int32_t)in.u32();
        const size_t at = in.o;
        if (size < 0 || !in.need((size_t)size)) break;
        if (name == "channels") {
            int nc = 0;
            while (in.o < at + size && b[in.o]) {
                const std::string cn = cstr();
                const int32_t t = (int32_t)in.u32();
                in.o += 12;
                if (pt >= 0 && t != pt) return ferr(ALVRL_ERR_INVALID, "mixed channel types");
                pt = t;
                if (cn != (nc == 0 ? "B" : nc == 1 ? "G" : "R")) return ferr(ALVRL_ERR_INVALID, "channels must be B, G, R");
                nc++;
            }
            if (nc != 3) return ferr(ALVRL_ERR_INVALID, "channels must be B, G, R");
        } else if (name == "compression") {
            comp = b[at];
        } else if (name == "dataWindow") {
            In d{b.data() + at, (size_t)size};
            const int32_t x0 = (int32_t)d.u32(), y0 = (int32_t)d.u32(), x1 = (int32_t)d.u32(), y1 = (int32_t)d.u32();
            w = x1 - x0 + 1; h = y1 - y0 + 1;
        }
        in.o = at + size;
    }
    if (!in.ok || comp != 0 || (pt != 1 && pt != 2) || w <= 0 || h <= 0)
        return ferr(ALVRL_ERR_INVALID, "unsupported OpenEXR file (uncompressed scanline B/G/R only)");
    *width = w; *height = h;
    if (!rgb) return ALVRL_OK;
    if (cap_floats < 3ull * w * h) return ferr(ALVRL_ERR_INVALID, "alvrl_read_exr: buffer too small");
    const size_t bpc = pt == 1 ? 2 : 4;
    for (int y = 0; y < h; y++) {
        In t{b.data(), b.size(), in.o + 8 * (size_t)y};
        In s{b.data(), b.size(), (size_t)t.u64()};
        const int32_t yy = (int32_t)s.u32();
        const int32_t sz = (int32_t)s.u32();
        if (!t.ok || !s.ok || yy < 0 || yy >= h || (size_t)sz != 3 * bpc * (size_t)w || !s.need((size_t)sz))
            return ferr(ALVRL_ERR_INVALID, "malformed scanline block");
        for (int c = 2; c >= 0; c--)
            for (int x = 0; x < w; x++) {
                float v;
                if (bpc == 2) { v = h2f((uint16_t)(b[s.o] | (b[s.o + 1] << 8))); s.o += 2; }
                else v = s.f32();
                rgb[3 * ((size_t)yy * w + x) + c] = v;
            }
    }
    return ALVRL_OK;
}

// mtsutil rms <gamma> a b [robust fraction] [relative] (src/utils/rms.cpp:36-110)
ALVRL_API int alvrl_image_rms(const float* sample, const float* reference, uint64_t n, double gamma,
                              double robust_fraction, int relative, double* out)
{
    if (!sample || !reference || !out || n == 0) return ferr(ALVRL_ERR_INVALID, "alvrl_image_rms: bad argument");
    size_t drop = 0;
    if (robust_fraction > 0) {
        drop = (size_t)(0.5 + (double)n * robust_fraction);
        if (2 * drop >= n) return ferr(ALVRL_ERR_INVALID, "robustFraction: dropping more elements than there are available!");
    }
    std::vector<double> d(n);
    for (uint64_t i = 0; i < n; i++) {
        const double s = std::pow((double)sample[i], 1.0 / gamma);
        const double r = std::pow((double)reference[i], 1.0 / gamma);
        d[i] = relative ? (r == 0 ? 0 : (s - r) / r) : s - r;
    }
    if (drop > 0) std::sort(d.begin(), d.end());
    for (size_t i = drop; i < n - drop; i++) d[i] = d[i] * d[i];
    std::sort(d.begin() + drop, d.end() - drop);
    double acc = 0;
    for (size_t i = drop; i < n - drop; i++) acc += d[i];
    *out = std::sqrt(acc / (double)(n - 2 * drop));
    return ALVRL_OK;
}

// ProgressiveMonteCarloIntegrator::dumpPass file name with the vrl
// integrator's passFileSuffix; hdrfilm replaces the placeholder extension
// ".blahExtensionTODO" by ".exr".
ALVRL_API int alvrl_pass_file_name(char* out, uint64_t cap, const char* dest, int pass, double prepass_cpu,
                                   double prepass_wall, double render_cpu, double render_wall,
                                   double vrls_preprocess, double vrls_render)
{
    if (!out || !dest) return ferr(ALVRL_ERR_INVALID, "alvrl_pass_file_name: null argument");
    std::stringstream s;
    s << dest << "_pass" << std::setfill('0') << std::setw(3) << pass
      << std::fixed << std::scientific << std::setprecision(4)
      << "_precpu" << prepass_cpu << "_prewall" << prepass_wall
      << "_rencpu" << render_cpu << "_renwall" << render_wall;
    // passFileSuffix (:358-363): the statistics counters read as float
    s << std::fixed << std::scientific << std::setprecision(4)
      << "_prevrl" << (float)vrls_preprocess << "_renvrl" << (float)vrls_render << ".exr";
    const std::string r = s.str();
    if (r.size() + 1 > cap) return ferr(ALVRL_ERR_INVALID, "alvrl_pass_file_name: buffer too small");
    std::memcpy(out, r.c_str(), r.size() + 1);
    return ALVRL_OK;
}

}  // extern "C"
