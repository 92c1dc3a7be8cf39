// Latency of small RCCL all-gathers with a one-rank communicator (the W = 1 sharded path's
// exchanges), eager and inside a captured hipGraph, beside a device-to-device copy and an empty
// kernel (diagnostics). Build: hipcc --offload-arch=gfx950 -O2 tools/rccl_latency.cpp -lrccl
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { auto e_ = (x); if (e_ != 0) { std::printf("error %d at %s:%d\n", (int)e_, __FILE__, __LINE__); return 1; } } while (0)

__global__ void empty_kernel(double* p) { if (threadIdx.x == 1023) p[0] = 1.0; }

int main() {
    ncclUniqueId id;
    ncclComm_t comm;
    CK(ncclGetUniqueId(&id));
    CK(ncclCommInitRank(&comm, 1, id, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    double *a, *b;
    const size_t n = 256;   // 2 KB
    CK(hipMalloc(&a, n * sizeof(double)));
    CK(hipMalloc(&b, n * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 200;
    auto timed = [&](const char* name, auto&& body) -> int {
        for (int i = 0; i < 10; ++i) body();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) body();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        const double host_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-44s %8.2f us per op (device), %8.2f us (host)\n", name, ms * 1e3 / reps, host_us);
        return 0;
    };
    if (timed("ncclAllGather 2 KB, 1 rank, eager", [&] { ncclAllGather(a, b, n, ncclDouble, comm, s); })) return 1;
    if (timed("hipMemcpyAsync D2D 2 KB, eager", [&] { (void)hipMemcpyAsync(b, a, n * sizeof(double), hipMemcpyDeviceToDevice, s); })) return 1;
    if (timed("empty kernel, eager", [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, a); })) return 1;
    // graphs of 10 ops each
    auto graph_of = [&](auto&& op, hipGraphExec_t* ex) -> int {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < 10; ++i) { op(); hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, a); }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(ex, g, nullptr, nullptr, 0));
        return 0;
    };
    hipGraphExec_t gx_nccl, gx_copy, gx_kern;
    if (graph_of([&] { ncclAllGather(a, b, n, ncclDouble, comm, s); }, &gx_nccl)) return 1;
    if (graph_of([&] { (void)hipMemcpyAsync(b, a, n * sizeof(double), hipMemcpyDeviceToDevice, s); }, &gx_copy)) return 1;
    if (graph_of([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, b); }, &gx_kern)) return 1;
    if (timed("graph: 10 x (ncclAllGather + kernel) / 10", [&] { (void)hipGraphLaunch(gx_nccl, s); })) return 1;
    if (timed("graph: 10 x (memcpy D2D + kernel) / 10", [&] { (void)hipGraphLaunch(gx_copy, s); })) return 1;
    if (timed("graph: 10 x (kernel + kernel) / 10", [&] { (void)hipGraphLaunch(gx_kern, s); })) return 1;
    std::printf("(graph lines: per graph launch of 10 pairs; divide by 10 for one pair)\n");
    ncclCommDestroy(comm);
    return 0;
}
