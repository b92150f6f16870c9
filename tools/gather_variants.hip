// gather_variants.hip -- A/B harness for the brute gather kernel on one GPU.
// Builds C2-shaped inputs with libalvrl.so's host harness, runs kernel
// variants interleaved in one process (cdna_hip_programming.md rule 24) and
// prints ms per variant and the max relative difference to variant 0.
//   hipcc --offload-arch=gfx950 -O3 -fno-hip-fp32-correctly-rounded-divide-sqrt \
//     -fgpu-flush-denormals-to-zero -I../include -I../mitsuba-alvrl_amd/csrc \
//     gather_variants.hip -L../mitsuba-alvrl_amd -lalvrl -o gather_variants
#include "../include/alvrl_host.h"
#include <hip/hip_runtime.h>
// ablation stubs (build-time -D): replace a transcendental family by a cheap
// stand-in to price it; outputs are meaningless in those builds.
#ifdef STUB_TAN
#define tanf(x) ((x) * 1.0001f)
#endif
#ifdef STUB_ATAN
#define atanf(x) ((x) * 0.9999f)
#endif
#ifdef STUB_HYP
#define sinhf(x) ((x) * 1.0001f)
#define asinhf(x) ((x) * 0.9999f)
#endif
#ifdef STUB_EXP
#define __expf(x) ((x) * 1.0001f + 1.0f)
#endif
#include "vrl_device.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace alvrl;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ Rec ld(const Rec* recs, uint32_t r, bool a)
{
    Rec x;
    if (a) { x = recs[r]; } else { x = Rec{0,0,0,0,0,1,0,0,1,0,0,-1,0,0,0,0u}; }
    return x;
}

template <int MINW>
__device__ __forceinline__ void body(const Rec* recs, uint32_t nrec, const VrlPrep* vp, uint32_t nvrl,
                                     DevParams P, float norm, float* out)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = r < nrec;
    const RecPre q = prepare_record(ld(recs, r, active), P);
    float L0 = 0, L1 = 0, L2 = 0;
    if (q.medium) {
        for (uint32_t v = 0; v < nvrl; ++v) {
            const VrlPrep V = vp[v];
            float c[3], m, s;
            integrate_vrl<2, 2, false>(P, q, V, r, v, kDomGather, 2, 2, c, &m, &s);
            L0 += c[0] * norm; L1 += c[1] * norm; L2 += c[2] * norm;
        }
    }
    if (active) { out[3 * r] = L0; out[3 * r + 1] = L1; out[3 * r + 2] = L2; }
}

__global__ void __launch_bounds__(256) kv0(const Rec* a, uint32_t b, const VrlPrep* c, uint32_t d, DevParams P, float n, float* o) { body<0>(a, b, c, d, P, n, o); }
__global__ void __launch_bounds__(256, 5) kv5(const Rec* a, uint32_t b, const VrlPrep* c, uint32_t d, DevParams P, float n, float* o) { body<5>(a, b, c, d, P, n, o); }
__global__ void __launch_bounds__(256, 6) kv6(const Rec* a, uint32_t b, const VrlPrep* c, uint32_t d, DevParams P, float n, float* o) { body<6>(a, b, c, d, P, n, o); }
__global__ void __launch_bounds__(256, 8) kv8(const Rec* a, uint32_t b, const VrlPrep* c, uint32_t d, DevParams P, float n, float* o) { body<8>(a, b, c, d, P, n, o); }

// two VRLs per iteration: two independent dependency chains per lane
__global__ void __launch_bounds__(256) kvu2(const Rec* recs, uint32_t nrec, const VrlPrep* vp, uint32_t nvrl, DevParams P, float norm, float* out)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = r < nrec;
    const RecPre q = prepare_record(ld(recs, r, active), P);
    float L0 = 0, L1 = 0, L2 = 0;
    if (q.medium) {
        uint32_t v = 0;
        for (; v + 1 < nvrl; v += 2) {
            const VrlPrep A = vp[v], B = vp[v + 1];
            float ca[3], cb[3], m, s;
            integrate_vrl<2, 2, false>(P, q, A, r, v, kDomGather, 2, 2, ca, &m, &s);
            integrate_vrl<2, 2, false>(P, q, B, r, v + 1, kDomGather, 2, 2, cb, &m, &s);
            L0 += ca[0] * norm; L1 += ca[1] * norm; L2 += ca[2] * norm;
            L0 += cb[0] * norm; L1 += cb[1] * norm; L2 += cb[2] * norm;
        }
        for (; v < nvrl; ++v) {
            const VrlPrep A = vp[v];
            float ca[3], m, s;
            integrate_vrl<2, 2, false>(P, q, A, r, v, kDomGather, 2, 2, ca, &m, &s);
            L0 += ca[0] * norm; L1 += ca[1] * norm; L2 += ca[2] * norm;
        }
    }
    if (active) { out[3 * r] = L0; out[3 * r + 1] = L1; out[3 * r + 2] = L2; }
}

typedef void (*KFn)(const Rec*, uint32_t, const VrlPrep*, uint32_t, DevParams, float, float*);

int main(int argc, char** argv)
{
    const int W = argc > 1 ? atoi(argv[1]) : 1024, H = argc > 2 ? atoi(argv[2]) : 512;
    const uint32_t NV = argc > 3 ? atoi(argv[3]) : 4000;
    alvrl_scene_desc sd;
    alvrl_scene_default(&sd, W, H);
    std::vector<float> soa(9 * (size_t)(NV + 8192));
    uint32_t nv = 0; uint64_t pc = 0;
    if (alvrl_trace_vrls(&sd, 0x5EED0001u, 0, NV, 1, -1, 5, soa.data(), NV + 8192, &nv, &pc)) { printf("trace failed\n"); return 1; }
    const uint32_t n = (uint32_t)W * H;
    std::vector<alvrl_gather_rec> recs(n);
    alvrl_scene_records(&sd, 1, nullptr, n, recs.data());
    // prepared VRLs on the host (same maths as k_prepare_vrls, host float)
    std::vector<VrlPrep> vp(nv);
    const size_t cap = NV + 8192;
    for (uint32_t i = 0; i < nv; i++) {
        VrlPrep p{};
        p.sx = soa[0 * cap + i]; p.sy = soa[1 * cap + i]; p.sz = soa[2 * cap + i];
        p.ex = soa[3 * cap + i]; p.ey = soa[4 * cap + i]; p.ez = soa[5 * cap + i];
        p.pr = soa[6 * cap + i]; p.pg = soa[7 * cap + i]; p.pb = soa[8 * cap + i];
        p.vx = p.ex - p.sx; p.vy = p.ey - p.sy; p.vz = p.ez - p.sz;
        const float l = std::sqrt(p.vx * p.vx + p.vy * p.vy + p.vz * p.vz);
        p.dx = p.vx / l; p.dy = p.vy / l; p.dz = p.vz / l;
        p.len = l; p.c = p.vx * p.vx + p.vy * p.vy + p.vz * p.vz;
        vp[i] = p;
    }
    DevParams P{};
    const float ss[3] = {0.8f, 0.6f, 0.4f};
    for (int i = 0; i < 3; i++) { P.sigma_s[i] = ss[i]; P.sigma_t[i] = ss[i] + 0.05f; }
    P.w = 0.8f / 0.85f; P.phase_type = 0; P.nvv = 2; P.nvs = 2; P.short_vrls = 1; P.seed = 0xA1B2C3D4u; P.pass = 0;
    Rec* d_recs; VrlPrep* d_vp; float* d_out;
    CK(hipMalloc(&d_recs, sizeof(Rec) * n)); CK(hipMalloc(&d_vp, sizeof(VrlPrep) * nv)); CK(hipMalloc(&d_out, 4 * 3 * (size_t)n * 8));
    CK(hipMemcpy(d_recs, recs.data(), sizeof(Rec) * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vp, vp.data(), sizeof(VrlPrep) * nv, hipMemcpyHostToDevice));
    const char* names[] = {"base", "minw5", "minw6", "minw8", "unroll2"};
    KFn fns[] = {kv0, kv5, kv6, kv8, kvu2};
    const int NVAR = 5;
    std::vector<std::vector<float>> res(NVAR, std::vector<float>(3 * (size_t)n));
    std::vector<double> tot(NVAR, 0.0);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const float norm = (float)(1.0 / (double)pc);
    for (int rep = 0; rep < 4; rep++) {
        for (int k = 0; k < NVAR; k++) {
            float* o = d_out + 3 * (size_t)n * k;
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(fns[k], dim3((n + 255) / 256), dim3(256), 0, 0, d_recs, n, d_vp, nv, P, norm, o);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0) tot[k] += ms;
            if (rep == 0) CK(hipMemcpy(res[k].data(), o, 4 * 3 * (size_t)n, hipMemcpyDeviceToHost));
        }
    }
    const double pairs = (double)n * nv;
    for (int k = 0; k < NVAR; k++) {
        double mx = 0;
        for (size_t i = 0; i < res[k].size(); i++) {
            const double a = res[0][i], b = res[k][i];
            if (a != 0) mx = std::fmax(mx, std::fabs(a - b) / std::fabs(a));
        }
        const double ms = tot[k] / 3;
        printf("%-10s %9.2f ms  %.3e pairs/s  maxrel_vs_base %.2e\n", names[k], ms, pairs / (ms * 1e-3), mx);
    }
    return 0;
}
