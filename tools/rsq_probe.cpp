// Accuracy of the f64 reciprocal square root estimate (v_rsq_f64) and of one and two Newton steps
// (multifrontal.hip rsqrt_nr), against 1 / sqrtl(d) on the host in long double. Diagnostics only.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/rsq_probe tools/rsq_probe.cpp
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__global__ void probe(const double* d, double* y0, double* y1, double* y2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = d[i];
    double y = __builtin_amdgcn_rsq(x);
    y0[i] = y;
    const double h = 0.5 * x;
    y = y * fma(-h * y, y, 1.5);
    y1[i] = y;
    y = y * fma(-h * y, y, 1.5);
    y2[i] = y;
}

int main() {
    const int n = 1 << 20;
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-12.0, 12.0);
    std::vector<double> d(n);
    for (auto& x : d) x = std::pow(10.0, u(g)) * (1.0 + 1e-3 * (double)(g() % 1000));
    double *dd, *a, *b, *c;
    if (hipMalloc(&dd, n * 8) || hipMalloc(&a, n * 8) || hipMalloc(&b, n * 8) || hipMalloc(&c, n * 8)) return 1;
    if (hipMemcpy(dd, d.data(), n * 8, hipMemcpyHostToDevice)) return 1;
    hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, dd, a, b, c, n);
    if (hipDeviceSynchronize()) return 1;
    std::vector<double> y0(n), y1(n), y2(n);
    if (hipMemcpy(y0.data(), a, n * 8, hipMemcpyDeviceToHost) || hipMemcpy(y1.data(), b, n * 8, hipMemcpyDeviceToHost) ||
        hipMemcpy(y2.data(), c, n * 8, hipMemcpyDeviceToHost))
        return 1;
    double e0 = 0, e1 = 0, e2 = 0;
    for (int i = 0; i < n; ++i) {
        const long double ex = 1.0L / sqrtl((long double)d[i]);
        const long double ulp = (long double)std::nextafter((double)ex, INFINITY) - (long double)(double)ex;
        e0 = std::max(e0, (double)(fabsl((long double)y0[i] - ex) / ulp));
        e1 = std::max(e1, (double)(fabsl((long double)y1[i] - ex) / ulp));
        e2 = std::max(e2, (double)(fabsl((long double)y2[i] - ex) / ulp));
    }
    printf("max error in ulps over %d values (1e-12 .. 1e12): v_rsq_f64 %.3g, one Newton step %.3g, two %.3g\n", n, e0, e1, e2);
    return 0;
}
