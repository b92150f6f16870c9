// ubench_valu.hip -- gfx950 VALU throughput per instruction class at full
// occupancy (8 waves/SIMD, independent chains): f32 / f64 fma, v_mov, f32
// IEEE division, trans.  Prints wave-instruction rate per SIMD and the cycles
// one wave64 instruction holds its SIMD.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/ubench_valu.hip -o tools/ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 4096;
constexpr int CH = 8;

template <typename T>
__global__ void __launch_bounds__(256) k_fma(T* out, T a, T b)
{
    T x[CH];
    for (int c = 0; c < CH; c++) x[c] = (T)(threadIdx.x + c);
    for (int i = 0; i < ITER; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = __builtin_fma(x[c], a, b);
    T s = 0;
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_div(float* out, float a)
{
    float x[CH];
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c + 1.0f;
    for (int i = 0; i < ITER / 8; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = a / x[c];
    float s = 0;
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the IEEE f32 division's core without its scaling and fix-up (v_div_scale,
// v_div_fmas, v_div_fixup): rcp, one Newton step, quotient and two residual
// corrections (operands and quotient in the normal range)
__device__ __forceinline__ float div_core(float a, float b)
{
    float y = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    float q = a * y;
    float r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}

__global__ void __launch_bounds__(256) k_divc(float* out, float a)
{
    float x[CH];
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c + 1.0f;
    for (int i = 0; i < ITER / 8; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = div_core(a, x[c]);
    float s = 0;
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__device__ __forceinline__ float sqrt_core(float x)
{
    const float y = __builtin_amdgcn_sqrtf(x);
    const float ym = __uint_as_float(__float_as_uint(y) - 1u);
    const float yp = __uint_as_float(__float_as_uint(y) + 1u);
    float r = __builtin_fmaf(-ym, y, x) <= 0.0f ? ym : y;
    return __builtin_fmaf(-yp, y, x) > 0.0f ? yp : r;
}

__global__ void __launch_bounds__(256) k_sqrtc(float* out, float a)
{
    float x[CH];
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c + 1.0f;
    for (int i = 0; i < ITER / 8; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = sqrt_core(x[c] + a);
    float s = 0;
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_fmaf(float* out, float a, float b)
{
    float x[CH];
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c;
    for (int i = 0; i < ITER; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = __builtin_fmaf(x[c], a, b);
    float s = 0;
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_sqrt(float* out, float a)
{
    float x[CH];
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c + 1.0f;
    for (int i = 0; i < ITER / 8; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = sqrtf(x[c] + a);
    float s = 0;
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    const int blocks = cus * 8;   // 8 blocks of 4 waves per CU: 8 waves / SIMD
    float* of; double* od;
    hipMalloc(&of, sizeof(float) * blocks * 256);
    hipMalloc(&od, sizeof(double) * blocks * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch, double ops_per_thread) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double waveinst = ops_per_thread * blocks * 4;     // wave64 instructions (4 waves per block)
        const double per_simd_ns = waveinst / (cus * 4) / (ms * 1e6);
        std::printf("%-10s %8.3f ms  %.3f wave-inst/ns/SIMD  = %.2f cyc/inst at %d MHz\n", name, ms, per_simd_ns,
                    (clk / 1e3) / 1e3 / per_simd_ns, clk / 1000);
    };
    run("fma_f32", [&] { hipLaunchKernelGGL(k_fmaf, dim3(blocks), dim3(256), 0, 0, of, 0.999f, 0.5f); },
        (double)ITER * CH);
    run("fma_f64", [&] { hipLaunchKernelGGL(k_fma<double>, dim3(blocks), dim3(256), 0, 0, od, 0.999, 0.5); },
        (double)ITER * CH);
    run("div_f32", [&] { hipLaunchKernelGGL(k_div, dim3(blocks), dim3(256), 0, 0, of, 3.0f); }, (double)ITER / 8 * CH);
    run("sqrt_f32", [&] { hipLaunchKernelGGL(k_sqrt, dim3(blocks), dim3(256), 0, 0, of, 0.5f); },
        (double)ITER / 8 * CH);
    run("divcore", [&] { hipLaunchKernelGGL(k_divc, dim3(blocks), dim3(256), 0, 0, of, 3.0f); }, (double)ITER / 8 * CH);
    run("sqrtcore", [&] { hipLaunchKernelGGL(k_sqrtc, dim3(blocks), dim3(256), 0, 0, of, 0.5f); },
        (double)ITER / 8 * CH);
    return 0;
}
