// ubench_colw_mfma.hip -- does MFMA pay for LightSlice's reduced-matrix products?
//
// The candidate (BASELINE.json north_star): calculateColumnWeigths
// (Preprocessor.cpp:985-1008) for S slices that share a row block (the
// neighbour-weighted local matrices of getLocalMatrix, :779-827, when
// neighbourCount > 0): W[S x N] = Loc[S x rows] . X[rows x N] with
// X = mean^2 + var of R's entries.  S = 1 is the default (neighbourCount = 0):
// one GEMV per slice.  R is stored as the refinement reads it: one slice block
// [vrl][row] of float2 (mean, var), columns 8 * rows bytes apart.
//
// Three kernels over the same block:
//   valu   one wave per column, lanes over rows (the production order: lane l
//          sums rows l, l+64, ..., then the halving tree), S outputs per column;
//   mfma   v_mfma_f64_16x16x4_f64: a wave owns 16 columns, B = X (lane l holds
//          4 consecutive rows of column l & 15 -> the k order of the 4 MFMAs of
//          a 16-row step is permuted, A follows it), A = Loc padded to 16 rows;
//   peak   back-to-back independent f64 MFMAs (the box's f64 matrix rate).
// And the f64 MFMA's numerics: is D bit for bit the k-ordered fma chain
// fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0,c))))?
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_colw_mfma tools/ubench_colw_mfma.hip
//   tools/ubench_colw_mfma            (prints one JSON line per case)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef double double4_t __attribute__((ext_vector_type(4)));

constexpr int kSmax = 4;

__device__ __forceinline__ double tree(double p)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) p += __shfl_down(p, off, 64);
    return p;
}

// one wave per column
__global__ void __launch_bounds__(256) k_colw_valu(const float2* __restrict__ R, uint32_t rows, uint32_t n,
                                                   const double* __restrict__ loc, int S, double* __restrict__ out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t v = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); v < n; v += nw) {
        double acc[kSmax] = {0.0, 0.0, 0.0, 0.0};
        for (uint32_t r = lane; r < rows; r += 64) {
            const float2 e = R[(size_t)v * rows + r];
            const double x = (double)e.x * (double)e.x + (double)e.y;
#pragma unroll
            for (int s = 0; s < kSmax; s++)
                if (s < S) acc[s] += loc[(size_t)s * rows + r] * x;
        }
#pragma unroll
        for (int s = 0; s < kSmax; s++)
            if (s < S) {
                const double t = tree(acc[s]);
                if (lane == 0) out[(size_t)s * n + v] = t;
            }
    }
}

// one wave per 16 columns on v_mfma_f64_16x16x4_f64
__global__ void __launch_bounds__(256) k_colw_mfma(const float2* __restrict__ R, uint32_t rows, uint32_t n,
                                                   const double* __restrict__ loc, int S, double* __restrict__ out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane & 15, h = lane >> 4;
    const uint32_t ntile = (n + 15) / 16;
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t t = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < ntile; t += nw) {
        const uint32_t v = t * 16 + j;
        const bool colok = v < n;
        double4_t acc = {0.0, 0.0, 0.0, 0.0};
        for (uint32_t k0 = 0; k0 < rows; k0 += 16) {
            // this lane's 4 consecutive rows of column v: k0 + 4h + q, q = 0..3
            double x[4], a[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t r = k0 + 4 * h + (uint32_t)q;
                float2 e = make_float2(0.0f, 0.0f);
                if (colok && r < rows) e = R[(size_t)v * rows + r];
                x[q] = (double)e.x * (double)e.x + (double)e.y;
                // A[i = lane & 15][k = h] of MFMA q: Loc row i at row k0 + 4h + q
                a[q] = ((int)j < S && r < rows) ? loc[(size_t)j * rows + r] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < 4; q++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], x[q], acc, 0, 0, 0);
        }
        // D[i][col]: col = lane & 15, i = (lane >> 4) + 4 * reg
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            const int i = (int)h + 4 * reg;
            if (i < S && colok) out[(size_t)i * n + v] = acc[reg];
        }
    }
}

// independent back-to-back f64 MFMAs: the matrix rate
__global__ void __launch_bounds__(256) k_mfma_peak(double* out, int iters)
{
    const double a = 1.0 + 1e-9 * threadIdx.x, b = 1.0 - 1e-9 * threadIdx.x;
    double4_t c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    const double4_t s = c0 + c1 + c2 + c3;
    if (s[0] == 12345.0) out[threadIdx.x] = s[1];
}

// one MFMA on given operands: A/B one f64 per lane, C/D 4 per lane
__global__ void k_mfma_once(const double* A, const double* B, const double* Cin, double* D)
{
    const uint32_t l = threadIdx.x;
    double4_t c = {Cin[4 * l], Cin[4 * l + 1], Cin[4 * l + 2], Cin[4 * l + 3]};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(A[l], B[l], c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[4 * l + r] = c[r];
}

static float time_ms(void (*launch)(void*), void* arg, int reps)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    launch(arg);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, nullptr));
    for (int i = 0; i < reps; i++) launch(arg);
    CK(hipEventRecord(e1, nullptr));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

struct Args { const float2* R; uint32_t rows, n; const double* loc; int S; double* out; int grid; };
static void launch_valu(void* p) { Args& a = *(Args*)p; hipLaunchKernelGGL(k_colw_valu, dim3(a.grid), dim3(256), 0, 0, a.R, a.rows, a.n, a.loc, a.S, a.out); }
static void launch_mfma(void* p) { Args& a = *(Args*)p; hipLaunchKernelGGL(k_colw_mfma, dim3(a.grid), dim3(256), 0, 0, a.R, a.rows, a.n, a.loc, a.S, a.out); }

int main()
{
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(-1.0, 1.0);

    // 1. numerics of v_mfma_f64_16x16x4_f64: A[i][k] lane (k<<4)|i, B[k][j] lane (k<<4)|j,
    //    C/D[i][j] at lane (i & 3) << 4 | j, reg i >> 2 (col = lane & 15, row = (lane >> 4) + 4 reg)
    {
        const int trials = 2000;
        long fma_chain = 0, fma_rev = 0, sep = 0, total = 0;
        std::vector<double> A(64), B(64), C(256), D(256);
        double *dA, *dB, *dC, *dD;
        CK(hipMalloc(&dA, 64 * 8)); CK(hipMalloc(&dB, 64 * 8)); CK(hipMalloc(&dC, 256 * 8)); CK(hipMalloc(&dD, 256 * 8));
        for (int t = 0; t < trials; t++) {
            // wide dynamic range with cancellation: products and C of similar size
            for (auto& x : A) x = U(rng) * std::ldexp(1.0, (int)(rng() % 40) - 20);
            for (auto& x : B) x = U(rng) * std::ldexp(1.0, (int)(rng() % 40) - 20);
            for (auto& x : C) x = U(rng) * std::ldexp(1.0, (int)(rng() % 40) - 20);
            CK(hipMemcpy(dA, A.data(), 64 * 8, hipMemcpyHostToDevice));
            CK(hipMemcpy(dB, B.data(), 64 * 8, hipMemcpyHostToDevice));
            CK(hipMemcpy(dC, C.data(), 256 * 8, hipMemcpyHostToDevice));
            hipLaunchKernelGGL(k_mfma_once, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
            CK(hipMemcpy(D.data(), dD, 256 * 8, hipMemcpyDeviceToHost));
            for (int i = 0; i < 16; i++)
                for (int jj = 0; jj < 16; jj++) {
                    const int lane = ((i & 3) << 4) | jj, reg = i >> 2;
                    const double c = C[4 * lane + reg], d = D[4 * lane + reg];
                    double f = c, r = c, s = c;
                    for (int k = 0; k < 4; k++) f = std::fma(A[(k << 4) | i], B[(k << 4) | jj], f);
                    for (int k = 3; k >= 0; k--) r = std::fma(A[(k << 4) | i], B[(k << 4) | jj], r);
                    for (int k = 0; k < 4; k++) s = s + A[(k << 4) | i] * B[(k << 4) | jj];
                    fma_chain += d == f; fma_rev += d == r; sep += d == s; total++;
                }
        }
        std::printf("{\"case\": \"f64 mfma numerics\", \"results\": %ld, \"equal_fma_chain_k_order\": %ld, "
                    "\"equal_fma_chain_reverse\": %ld, \"equal_mul_then_add\": %ld}\n", total, fma_chain, fma_rev, sep);
        CK(hipFree(dA)); CK(hipFree(dB)); CK(hipFree(dC)); CK(hipFree(dD));
    }

    // 2. the f64 matrix rate on this box
    double peak_tf = 0;
    {
        double* d; CK(hipMalloc(&d, 256 * 8));
        const int iters = 4096, grid = ncu * 8;
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        hipLaunchKernelGGL(k_mfma_peak, dim3(grid), dim3(256), 0, 0, d, 16);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, nullptr));
        hipLaunchKernelGGL(k_mfma_peak, dim3(grid), dim3(256), 0, 0, d, iters);
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double flops = (double)grid * 4 /*waves*/ * iters * 4 /*mfma*/ * (2.0 * 16 * 16 * 4);
        peak_tf = flops / (ms * 1e-3) / 1e12;
        std::printf("{\"case\": \"f64 mfma peak\", \"tflops\": %.2f, \"ms\": %.3f, \"cus\": %d, \"clock_mhz\": %d}\n",
                    peak_tf, ms, ncu, clk_khz / 1000);
        CK(hipFree(d));
    }

    // 3. column weights of one slice block, S = 1 (default) and S = 4 (neighbours)
    const uint32_t shapes[][2] = {{164, 100003}, {214, 100003}, {655, 1000000}};
    for (auto& sh : shapes) {
        const uint32_t rows = sh[0], n = sh[1];
        std::vector<float2> hR((size_t)rows * n);
        for (auto& e : hR) { const float m = (float)std::fabs(U(rng)) * 1e-3f; e = make_float2(m, m * m * 0.1f); }
        float2* dR; CK(hipMalloc(&dR, hR.size() * 8));
        CK(hipMemcpy(dR, hR.data(), hR.size() * 8, hipMemcpyHostToDevice));
        for (int S : {1, 4}) {
            std::vector<double> loc((size_t)S * rows);
            for (auto& x : loc) x = std::fabs(U(rng)) / rows;
            double *dloc, *o1, *o2;
            CK(hipMalloc(&dloc, loc.size() * 8));
            CK(hipMemcpy(dloc, loc.data(), loc.size() * 8, hipMemcpyHostToDevice));
            CK(hipMalloc(&o1, (size_t)S * n * 8)); CK(hipMalloc(&o2, (size_t)S * n * 8));
            Args a1{dR, rows, n, dloc, S, o1, ncu * 16}, a2{dR, rows, n, dloc, S, o2, ncu * 16};
            const float t_valu = time_ms(launch_valu, &a1, 20);
            const float t_mfma = time_ms(launch_mfma, &a2, 20);
            std::vector<double> h1((size_t)S * n), h2((size_t)S * n);
            CK(hipMemcpy(h1.data(), o1, h1.size() * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h2.data(), o2, h2.size() * 8, hipMemcpyDeviceToHost));
            double maxrel = 0; long bitequal = 0;
            for (size_t i = 0; i < h1.size(); i++) {
                maxrel = std::max(maxrel, std::fabs(h1[i] - h2[i]) / std::max(std::fabs(h1[i]), 1e-300));
                bitequal += h1[i] == h2[i];
            }
            const double bytes = (double)rows * n * 8, useful = 2.0 * S * rows * n;
            const double padded = 2.0 * 16 * ((rows + 15) / 16 * 16) * ((n + 15) / 16 * 16);
            std::printf("{\"case\": \"column weights\", \"rows\": %u, \"columns\": %u, \"slices_S\": %d, "
                        "\"valu_ms\": %.4f, \"valu_GBps\": %.0f, \"mfma_ms\": %.4f, \"mfma_GBps\": %.0f, "
                        "\"mfma_util_useful\": %.5f, \"mfma_util_issued\": %.5f, \"flop_per_byte\": %.3f, "
                        "\"max_rel_diff\": %.2e, \"bit_equal_frac\": %.3f}\n",
                        rows, n, S, t_valu, bytes / (t_valu * 1e-3) / 1e9, t_mfma, bytes / (t_mfma * 1e-3) / 1e9,
                        useful / (t_mfma * 1e-3) / 1e12 / peak_tf, padded / (t_mfma * 1e-3) / 1e12 / peak_tf,
                        useful / bytes, maxrel, (double)bitequal / h1.size());
            CK(hipFree(dloc)); CK(hipFree(o1)); CK(hipFree(o2));
        }
        CK(hipFree(dR));
    }
    return 0;
}
