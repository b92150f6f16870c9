// pmc_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access widths k_refine uses (MI355X_MICROARCH.md leaves 8-B-per-lane
// loads and agent-scope atomics uncalibrated).  Each kernel moves a known
// number of bytes over a 1 GiB buffer (4x the Infinity Cache):
//   ld16      float4 per lane, streaming                      (guide: FETCH x2)
//   ld8       float2 per lane, streaming
//   ld8_cols  float2 per lane over 1312-B column runs at random 8-B offsets
//             (164 rows x 8 B: one slice's R column, k_refine's pattern)
//   st16/st8  streaming stores
//   cas       agent-scope relaxed compare-and-swap polls on 256 words
//   ldpoll    agent-scope relaxed loads of 256 words
// Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
// Run:   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- tools/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr size_t kBytes = size_t(1) << 30;

__global__ void ld16(const float4* __restrict__ a, size_t n, float* out)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;
}

__global__ void ld8(const float2* __restrict__ a, size_t n, float* out)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 12345.f) out[0] = s;
}

// one wave per column run of 164 float2 (3 loads per lane, the last partial)
__global__ void ld8_cols(const float2* __restrict__ a, const unsigned* __restrict__ starts, unsigned ncols, float* out)
{
    const unsigned lane = threadIdx.x & 63, w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const unsigned nw = (gridDim.x * blockDim.x) >> 6;
    float s = 0.f;
    for (unsigned c = w; c < ncols; c += nw) {
        const float2* col = a + starts[c];
        for (unsigned r = lane; r < 164; r += 64) {
            const float2 v = col[r];
            s += v.x + v.y;
        }
    }
    if (s == 12345.f) out[0] = s;
}

__global__ void st16(float4* __restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

__global__ void st8(float2* __restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float2(1.f, (float)i);
}

// thread 0 of each block: `iters` CAS attempts on word blockIdx.x % 256
__global__ void cas(unsigned* w, unsigned iters)
{
    if (threadIdx.x != 0) return;
    unsigned* p = w + (blockIdx.x & 255) * 32;
    for (unsigned k = 0; k < iters; k++) {
        unsigned e = k;
        __hip_atomic_compare_exchange_strong(p, &e, k + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void ldpoll(unsigned* w, unsigned iters, unsigned* out)
{
    if (threadIdx.x != 0) return;
    unsigned* p = w + (blockIdx.x & 255) * 32;
    unsigned s = 0;
    for (unsigned k = 0; k < iters; k++) s += __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 12345u) out[0] = s;
}

int main()
{
    void* buf;
    float* out;
    unsigned* words;
    CK(hipMalloc(&buf, kBytes));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&words, 256 * 128));
    CK(hipMemset(buf, 0, kBytes));
    CK(hipMemset(words, 0, 256 * 128));
    const unsigned ncols = (unsigned)(kBytes / 1312);
    unsigned* starts_h = (unsigned*)std::malloc(ncols * 4ull);
    unsigned long long x = 88172645463325252ull;
    const unsigned maxs = (unsigned)(kBytes / 8) - 164;
    for (unsigned c = 0; c < ncols; c++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        starts_h[c] = (unsigned)(x % maxs);
    }
    unsigned* starts;
    CK(hipMalloc(&starts, ncols * 4ull));
    CK(hipMemcpy(starts, starts_h, ncols * 4ull, hipMemcpyHostToDevice));
    const int G = 2048, B = 256;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char* name, double bytes, auto&& launch) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-9s bytes %.0f  %.3f ms  %.2f TB/s\n", name, bytes, ms, bytes / ms * 1e-9);
    };
    timed("ld16", (double)kBytes, [&] { ld16<<<G, B>>>((const float4*)buf, kBytes / 16, out); });
    timed("ld8", (double)kBytes, [&] { ld8<<<G, B>>>((const float2*)buf, kBytes / 8, out); });
    timed("ld8_cols", (double)ncols * 1312, [&] { ld8_cols<<<G, B>>>((const float2*)buf, starts, ncols, out); });
    timed("st16", (double)kBytes, [&] { st16<<<G, B>>>((float4*)buf, kBytes / 16); });
    timed("st8", (double)kBytes, [&] { st8<<<G, B>>>((float2*)buf, kBytes / 8); });
    const unsigned iters = 4096;
    timed("cas", 1024.0 * iters, [&] { cas<<<1024, 64>>>(words, iters); });
    timed("ldpoll", 1024.0 * iters, [&] { ldpoll<<<1024, 64>>>(words, iters, (unsigned*)out); });
    CK(hipDeviceSynchronize());
    std::printf("ncols %u (1312 B each); cas/ldpoll: 1024 blocks x %u ops\n", ncols, iters);
    return 0;
}
