// Dependent-chain latencies of the instructions on the pivot loop's critical path (diagnostic):
// one wavefront, each chain N steps long between two s_memtime reads. Prints core cycles per step.
// Build: hipcc -O3 --offload-arch=gfx950 tools/lat_probe.hip -o gpurun_exp/lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 512;

__device__ __forceinline__ double readlane_d(double x, int l) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double rsqrt_nr(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

__device__ __forceinline__ double rcp_nr(double d) {
    double y = __builtin_amdgcn_rcp(d);
    y = fma(fma(-d, y, 1.0), y, y);
    return fma(fma(-d, y, 1.0), y, y);
}

__global__ __launch_bounds__(64) void probe(unsigned long long* out, double* sink, double seed, int jl) {
    __shared__ double buf[128];
    const int lane = threadIdx.x;
    double x = seed + lane * 1e-3;
    unsigned long long t0, t1;
    int q = 0;
#define TIME(BODY)                                                             \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                \
    t0 = __builtin_amdgcn_s_memtime();                                         \
    for (int i = 0; i < N; ++i) { BODY; }                                      \
    asm volatile("" : "+v"(x));                                                \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                \
    t1 = __builtin_amdgcn_s_memtime();                                         \
    if (lane == 0) out[q] = t1 - t0;                                           \
    ++q;
    TIME(x = fma(x, 0.999999, 1e-9); asm volatile("" : "+v"(x)))                       // 0 fma f64
    TIME(x = x * 0.999999; asm volatile("" : "+v"(x)))                                 // 1 mul f64
    TIME(x = __builtin_amdgcn_rsq(x); asm volatile("" : "+v"(x)))                     // 2 v_rsq_f64
    TIME(x = rsqrt_nr(x); asm volatile("" : "+v"(x)))                                  // 3 rsq + 2 Newton
    TIME(x = rcp_nr(x); asm volatile("" : "+v"(x)))                                    // 4 rcp + 2 Newton
    TIME(x = readlane_d(x, jl) + 1e-9; asm volatile("" : "+v"(x)))                     // 5 readlane pair + add
    TIME(buf[lane] = x; __builtin_amdgcn_wave_barrier(); x = buf[(lane + 1) & 63] + 1e-9;
         __builtin_amdgcn_wave_barrier(); asm volatile("" : "+v"(x)))                 // 6 LDS write->read
    TIME(const double d = readlane_d(x, jl); x = fma(x, rsqrt_nr(d > 0 ? d : 1.0), 1e-9);
         asm volatile("" : "+v"(x)))                                                   // 7 readlane + rsqrt_nr + fma
    TIME(const double d = readlane_d(x, jl); const bool bad = !(d > 0.0); const double dd = bad ? 1e-300 : d;
         x = lane == jl ? dd * rsqrt_nr(dd) : x * rsqrt_nr(dd); asm volatile("" : "+v"(x)))   // 8 pivot column form
    {
        float xf = (float)x;
        TIME(xf = fmaf(xf, 0.999f, 1e-6f); asm volatile("" : "+v"(xf)))                // 9 fma f32
        x += xf;
    }
    TIME(x = __builtin_amdgcn_sqrt(x); asm volatile("" : "+v"(x)))                    // 10 v_sqrt_f64
    TIME(x = __builtin_amdgcn_rcp(x); asm volatile("" : "+v"(x)))                     // 11 v_rcp_f64
    TIME(x = __shfl(x, jl) + 1e-9; asm volatile("" : "+v"(x)))                         // 12 shfl (bpermute)
    TIME(x += (double)(__builtin_amdgcn_s_memtime() & 1); asm volatile("" : "+v"(x)))  // 13 s_memtime + use
    TIME(x += (double)(__builtin_amdgcn_s_memrealtime() & 1); asm volatile("" : "+v"(x)))   // 14 s_memrealtime + use
    sink[lane] = x;
}

int main() {
    unsigned long long* d_out;
    double* d_sink;
    hipMalloc(&d_out, 64 * sizeof(unsigned long long));
    hipMalloc(&d_sink, 64 * sizeof(double));
    const char* names[] = {"v_fma_f64", "v_mul_f64", "v_rsq_f64", "rsq+2 Newton", "rcp+2 Newton",
                           "readlane pair + add", "LDS write->read", "readlane + rsqrt_nr + fma",
                           "pivot column form", "v_fma_f32", "v_sqrt_f64", "v_rcp_f64", "shfl + add", "s_memtime + use",
                           "s_memrealtime + use"};
    unsigned long long h[64];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_out, d_sink, 1.2345, 5);
        hipDeviceSynchronize();
    }
    hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    printf("dependent-chain latency, one wave alone (core cycles per step, %d steps):\n", N);
    for (int i = 0; i < 15; ++i) printf("  %-28s %7.1f\n", names[i], (double)h[i] / N);
    return 0;
}
