// ubench_f64.hip -- gfx950 latency / throughput of the operations the
// refinement recurrence is built from: dependent and independent f64 mul/add
// chains, f32 for comparison, and LDS broadcast ds_read_b128 latency.
// One workgroup of NW waves on one CU; s_memtime ticks per operation.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off ubench_f64.hip -o ubench_f64
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 4096;

template <int CHAINS>
__global__ void k_f64(double* out, double a, double b, long long* t)
{
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x + c;
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) x[c] = x[c] * a + b;   // mul + add (no contraction)
    }
    const long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s += x[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

template <int CHAINS>
__global__ void k_f32(float* out, float a, float b, long long* t)
{
    float x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = threadIdx.x + c;
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) x[c] = x[c] * a + b;
    }
    const long long t1 = clock64();
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s += x[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

struct __attribute__((aligned(16))) C4 { double a, b; };
__global__ void k_lds(double* out, long long* t)
{
    __shared__ C4 buf[64];
    if (threadIdx.x < 64) { buf[threadIdx.x].a = 1.0 + threadIdx.x * 1e-9; buf[threadIdx.x].b = 0; }
    __syncthreads();
    double acc = 0;
    int idx = 0;
    const long long t0 = clock64();
    for (int i = 0; i < N; i++) {                       // dependent broadcast reads
        const C4 v = buf[idx];
        acc += v.a;
        idx = ((int)v.b + i) & 63;
    }
    const long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

__global__ void k_barrier(double* out, long long* t)
{
    double acc = threadIdx.x;
    const long long t0 = clock64();
    for (int i = 0; i < N / 16; i++) { acc = acc * 1.0000001 + 1e-9; __syncthreads(); }
    const long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

template <int OFF>
__device__ __forceinline__ uint32_t flp(uint32_t v)
{
    if constexpr (OFF == 32) return __builtin_amdgcn_permlane32_swap(v, v, false, false)[1];
    else if constexpr (OFF == 16) return __builtin_amdgcn_permlane16_swap(v, v, false, false)[1];
    else return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x100 + OFF, 0xF, 0xF, false);
}
template <int OFF>
__device__ __forceinline__ double flpd(double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    return __longlong_as_double((long long)(((unsigned long long)flp<OFF>((uint32_t)(u >> 32)) << 32) | flp<OFF>((uint32_t)u)));
}
__global__ void k_tree(double* out, long long* t)
{
    double p[4];
    for (int q = 0; q < 4; q++) p[q] = threadIdx.x + q;
    const long long t0 = clock64();
    for (int i = 0; i < N / 16; i++) {
#define LV(O) { double o[4]; for (int q = 0; q < 4; q++) o[q] = flpd<O>(p[q]); for (int q = 0; q < 4; q++) p[q] = p[q] + o[q]; }
        LV(32) LV(16) LV(8) LV(4) LV(2) LV(1)
#undef LV
    }
    const long long t1 = clock64();
    out[threadIdx.x] = p[0] + p[1] + p[2] + p[3];
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

int main()
{
    double* d; float* f; long long* t;
    (void)hipMalloc(&d, 4096 * 8); (void)hipMalloc(&f, 4096 * 4); (void)hipMalloc(&t, 8);
    long long h;
    auto run = [&](const char* name, void (*launch)(int), int nw, double ops_per_iter) {
        launch(nw * 64);
        (void)hipDeviceSynchronize();
        launch(nw * 64);
        (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
        printf("%-34s waves/WG %d: %8.2f ticks per iteration, %6.2f ticks per op per wave\n", name, nw,
               (double)h / N, (double)h / N / ops_per_iter);
    };
#define L64(C) [](int n) { hipLaunchKernelGGL(k_f64<C>, dim3(1), dim3(n), 0, 0, (double*)0, 1.0000001, 1e-9, (long long*)0); }
    // (lambdas cannot capture; use globals)
    static double* gd; static float* gf; static long long* gt;
    gd = d; gf = f; gt = t;
    run("f64 mul+add, 1 chain", [](int n) { hipLaunchKernelGGL(k_f64<1>, dim3(1), dim3(n), 0, 0, gd, 1.0000001, 1e-9, gt); }, 1, 2);
    run("f64 mul+add, 4 chains", [](int n) { hipLaunchKernelGGL(k_f64<4>, dim3(1), dim3(n), 0, 0, gd, 1.0000001, 1e-9, gt); }, 1, 8);
    run("f64 mul+add, 16 chains", [](int n) { hipLaunchKernelGGL(k_f64<16>, dim3(1), dim3(n), 0, 0, gd, 1.0000001, 1e-9, gt); }, 1, 32);
    run("f64 mul+add, 16 chains", [](int n) { hipLaunchKernelGGL(k_f64<16>, dim3(1), dim3(n), 0, 0, gd, 1.0000001, 1e-9, gt); }, 8, 32);
    run("f32 mul+add, 1 chain", [](int n) { hipLaunchKernelGGL(k_f32<1>, dim3(1), dim3(n), 0, 0, gf, 1.0000001f, 1e-9f, gt); }, 1, 2);
    run("f32 mul+add, 16 chains", [](int n) { hipLaunchKernelGGL(k_f32<16>, dim3(1), dim3(n), 0, 0, gf, 1.0000001f, 1e-9f, gt); }, 1, 32);
    run("f32 mul+add, 16 chains", [](int n) { hipLaunchKernelGGL(k_f32<16>, dim3(1), dim3(n), 0, 0, gf, 1.0000001f, 1e-9f, gt); }, 8, 32);
    run("LDS broadcast b128 dependent", [](int n) { hipLaunchKernelGGL(k_lds, dim3(1), dim3(n), 0, 0, gd, gt); }, 1, 1);
    run("LDS broadcast b128 dependent", [](int n) { hipLaunchKernelGGL(k_lds, dim3(1), dim3(n), 0, 0, gd, gt); }, 8, 1);
    run("__syncthreads (+1 f64 op)", [](int n) { hipLaunchKernelGGL(k_barrier, dim3(1), dim3(n), 0, 0, gd, gt); }, 1, 1.0 / 16 * 16);
    run("__syncthreads (+1 f64 op)", [](int n) { hipLaunchKernelGGL(k_barrier, dim3(1), dim3(n), 0, 0, gd, gt); }, 8, 1.0 / 16 * 16);
    run("4 double trees (6 levels)", [](int n) { hipLaunchKernelGGL(k_tree, dim3(1), dim3(n), 0, 0, gd, gt); }, 1, 1.0 / 16 * 16);
    run("4 double trees (6 levels)", [](int n) { hipLaunchKernelGGL(k_tree, dim3(1), dim3(n), 0, 0, gd, gt); }, 8, 1.0 / 16 * 16);
    // clock calibration: s_memtime ticks vs wall time
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_f64<1>, dim3(1), dim3(64), 0, 0, gd, 1.0000001, 1e-9, gt);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    printf("calibration: %lld ticks in a kernel of %.3f ms wall (ticks/ns <= %.2f)\n", h, ms, h / (ms * 1e6));
    return 0;
}
