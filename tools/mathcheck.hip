// mathcheck.hip -- accuracy of the gather's fast device functions against
// host double precision, on log-spaced sweeps of both signs.  Prints the max
// relative error (and in float ulps) per function and magnitude band.
//   hipcc --offload-arch=gfx950 -O3 -fgpu-flush-denormals-to-zero \
//     -fno-hip-fp32-correctly-rounded-divide-sqrt -I../mitsuba-alvrl_amd/csrc mathcheck.hip -o mathcheck
#include "vrl_device.hpp"

#include <cmath>
#include <cstdio>
#include <vector>

using namespace alvrl;

enum { F_ASINH, F_SINH, F_COSH, F_OCML_ASINH, F_OCML_SINH, F_TAN, F_OCML_TAN, F_ATAN, F_OCML_ATAN, F_N };

__global__ void k_eval(const float* x, float* y, int n, int f)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = x[i];
    float r = 0;
    switch (f) {
    case F_ASINH: r = asinh_fast(v); break;
    case F_SINH: { float c; sinhcosh_fast(v, &r, &c); } break;
    case F_COSH: { float sh; sinhcosh_fast(v, &sh, &r); } break;
    case F_OCML_ASINH: r = asinhf(v); break;
    case F_OCML_SINH: r = sinhf(v); break;
    case F_TAN: r = tan_fast(v); break;
    case F_OCML_TAN: r = tanf(v); break;
    case F_ATAN: r = atan_fast(v); break;
    case F_OCML_ATAN: r = atanf(v); break;
    }
    y[i] = r;
}

int main()
{
    std::vector<float> xs;
    for (int e = -30; e <= 20; e++)          // |x| in [2^-30, 2^21)
        for (int k = 0; k < 4096; k++) {
            const float m = std::ldexp(1.0f + k / 4096.0f, e);
            xs.push_back(m);
            xs.push_back(-m);
        }
    for (int k = 0; k < 1 << 16; k++) {       // dense approach to pi/2 for tan
        const float m = std::nextafter(1.5707963267948966f, 0.0f) - std::ldexp((float)k, -16) * 0.5f;
        xs.push_back(m);
        xs.push_back(-m);
    }
    const int n = (int)xs.size();
    float *dx, *dy;
    (void)hipMalloc(&dx, 4 * n); (void)hipMalloc(&dy, 4 * n);
    (void)hipMemcpy(dx, xs.data(), 4 * n, hipMemcpyHostToDevice);
    const char* names[F_N] = {"asinh_fast", "sinhcosh.sh", "sinhcosh.ch", "ocml asinhf", "ocml sinhf", "tan_fast", "ocml tanf", "atan_fast", "ocml atanf"};
    std::vector<float> ys(n);
    for (int f = 0; f < F_N; f++) {
        hipLaunchKernelGGL(k_eval, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dy, n, f);
        (void)hipMemcpy(ys.data(), dy, 4 * n, hipMemcpyDeviceToHost);
        const double bands[] = {0, 1e-3, 0.25, 1, 1.5, 1.5707, 8, 90, 1e30};
        for (int b = 0; b + 1 < 9; b++) {
            double mx = 0, mxu = 0, xat = 0;
            for (int i = 0; i < n; i++) {
                const double a = std::fabs((double)xs[i]);
                if (a < bands[b] || a >= bands[b + 1]) continue;
                const bool s = (f == F_SINH || f == F_OCML_SINH), ch = (f == F_COSH);
                const bool tn = (f == F_TAN || f == F_OCML_TAN), at = (f == F_ATAN || f == F_OCML_ATAN);
                if ((s || ch) && a > 88) continue;                          // overflow range
                if (tn && a >= 1.5707963267948966) continue;        // sampler domain
                const double xd = xs[i];
                const double t = ch ? std::cosh(xd) : s ? std::sinh(xd) : tn ? std::tan(xd) : at ? std::atan(xd) : std::asinh(xd);
                const double err = std::fabs((double)ys[i] - t) / std::fabs(t);
                const double ulp = std::ldexp(1.0, std::ilogb((float)t) - 23);
                const double eu = std::fabs((double)ys[i] - t) / ulp;
                if (err > mx) { mx = err; xat = xs[i]; }
                if (eu > mxu) mxu = eu;
            }
            printf("%-12s |x| in [%g, %g): max rel %.3e (%.2f ulp) at x=%g\n", names[f], bands[b], bands[b + 1], mx, mxu, xat);
        }
    }
    return 0;
}
