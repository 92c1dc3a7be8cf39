// Does a kernel launched with hipExtAnyOrderLaunch run beside the previous kernel of the same stream
// (AQL barrier bit clear), eagerly and inside a captured hipGraph? Two kernels that each spin ~40 us
// on a few CUs: ~40 us total if they overlap, ~80 us if serialised (diagnostics).
// Build: hipcc --offload-arch=gfx950 -O2 tools/anyorder_probe.cpp -o tools/anyorder_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { auto e_ = (x); if (e_ != hipSuccess) { std::printf("error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

__global__ void spin(unsigned long long ticks, unsigned long long* out) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long* out;
    CK(hipMalloc(&out, 1024 * sizeof(unsigned long long)));
    const unsigned long long T = 4000;   // 40 us at 100 MHz
    auto run = [&](const char* name, auto&& body, int reps) -> int {
        body();
        CK(hipStreamSynchronize(s));
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) body();
        CK(hipStreamSynchronize(s));
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
        std::printf("%-52s %8.1f us per pair\n", name, us);
        return 0;
    };
    void* args[] = {(void*)&T, (void*)&out};
    auto a = [&]() { hipLaunchKernelGGL(spin, dim3(4), dim3(64), 0, s, T, out); };
    auto b_normal = [&]() { hipLaunchKernelGGL(spin, dim3(4), dim3(64), 0, s, T, out + 512); };
    auto b_any = [&]() { (void)hipExtLaunchKernel((const void*)spin, dim3(4), dim3(64), args, 0, s, nullptr, nullptr, hipExtAnyOrderLaunch); };
    if (run("eager: A then B (normal)", [&] { a(); b_normal(); }, 20)) return 1;
    if (run("eager: A then B (hipExtAnyOrderLaunch)", [&] { a(); b_any(); }, 20)) return 1;
    hipGraph_t g1, g2;
    hipGraphExec_t x1, x2;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    a(); b_normal();
    CK(hipStreamEndCapture(s, &g1));
    CK(hipGraphInstantiate(&x1, g1, nullptr, nullptr, 0));
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    a(); b_any();
    CK(hipStreamEndCapture(s, &g2));
    CK(hipGraphInstantiate(&x2, g2, nullptr, nullptr, 0));
    if (run("graph: A then B (normal)", [&] { (void)hipGraphLaunch(x1, s); }, 20)) return 1;
    if (run("graph: A then B (hipExtAnyOrderLaunch)", [&] { (void)hipGraphLaunch(x2, s); }, 20)) return 1;
    // fork / join through a second stream inside a graph (the solver's current form)
    hipStream_t side;
    hipEvent_t ef, ej;
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
    hipGraph_t g3;
    hipGraphExec_t x3;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(ef, s));
    CK(hipStreamWaitEvent(side, ef, 0));
    hipLaunchKernelGGL(spin, dim3(4), dim3(64), 0, side, T, out);
    CK(hipEventRecord(ej, side));
    b_normal();
    CK(hipStreamWaitEvent(s, ej, 0));
    CK(hipStreamEndCapture(s, &g3));
    CK(hipGraphInstantiate(&x3, g3, nullptr, nullptr, 0));
    if (run("graph: A on a forked stream beside B, joined", [&] { (void)hipGraphLaunch(x3, s); }, 20)) return 1;
    return 0;
}
