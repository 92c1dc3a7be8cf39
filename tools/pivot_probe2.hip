// What a two-pivot step of the front loop spends its cycles on (diagnostic; companion of
// tools/pivot_probe.hip): the same step with the front size a compile-time constant (no scalar
// branches over column groups), without exec-mask branches (stores to a scratch slot instead of
// predicated), its dependency chain alone, and its trailing update alone. One wavefront alone.
// Build: hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize tools/pivot_probe2.hip -o gpurun_exp/pivot_probe2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

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
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// MODE 0: full step, predicated stores (product-like) with m, k compile-time
// MODE 1: full step, branch-free stores (scratch slot)
// MODE 2: chain only (pivots, L columns; no LDS broadcast, no trailing update, no stores)
// MODE 3: trailing update only (fixed L columns through the LDS broadcast)
// MODE 4: full step branch-free, no forward step
// MODE 5: full step (predicated stores), the pivot pair of each trailing column read by readlane
//         into scalar registers instead of the LDS broadcast
// MODE 6: trailing update only, readlane form
// MODE 7: full step (predicated stores), LDS broadcast with each group of 8 pairs read at once
template <int M, int K, int MODE>
__global__ __launch_bounds__(64) void step(const double* A, double* L, double* wout, unsigned long long* cyc,
                                           double* rows_out) {
    __shared__ __attribute__((aligned(16))) double colbuf[2 * (M + 2) + 4];
    const int lane = threadIdx.x;
    const bool live = lane < M;
    double row[M];
#pragma unroll
    for (int c = 0; c < M; ++c) row[c] = (live && c <= lane) ? A[lane * M + c] : 0.0;
    double wi = live ? 1.0 + 0.01 * lane : 0.0;
    double* Lj = L + lane;
    double* const Lsink = L + 64 * 64 * 4 + lane;   // branch-free stores of the lanes that write nothing
    int nbad = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma nounroll
    for (int j = 0; j + 1 < K; j += 2) {
        double l0, l1, inv0, inv1;
        if (MODE == 3 || MODE == 6) {
            l0 = 0.01 * (lane + j);
            l1 = 0.02 * (lane + j);
            inv0 = inv1 = 1.0;
        } else {
            double d0 = readlane_d(row[0], j);
            const bool bad0 = !(d0 > 0.0);
            nbad += bad0;
            d0 = bad0 ? 1e-300 : d0;
            inv0 = rsqrt_nr(d0);
            const double l00 = d0 * inv0;
            l0 = lane == j ? l00 : row[0] * inv0;
            const double lj1 = readlane_d(l0, j + 1);
            const double f1 = fma(-l0, lj1, row[1]);
            double d1 = readlane_d(f1, j + 1);
            const bool bad1 = !(d1 > 0.0);
            nbad += bad1;
            d1 = bad1 ? 1e-300 : d1;
            inv1 = rsqrt_nr(d1);
            const double l11 = d1 * inv1;
            l1 = lane == j + 1 ? l11 : f1 * inv1;
        }
        if (MODE == 2) {
            // keep the chain's results alive; shift the window so the next step's pivot depends on this one
#pragma unroll
            for (int t = 0; t < M - 2; ++t) row[t] = row[t + 2];
            row[0] += 1e-30 * l0;
            row[1] += 1e-30 * l1;
            continue;
        }
        double2* cp = reinterpret_cast<double2*>(colbuf);
        if (MODE == 0 || MODE == 5 || MODE == 7) {
            if (MODE != 5 && lane > j + 1 && lane < M) cp[lane - j - 2] = make_double2(l0, l1);
            if (live) {
                if (lane >= j) __builtin_nontemporal_store(l0, Lj);
                if (lane >= j + 1) __builtin_nontemporal_store(l1, Lj + M);
            }
        } else if (MODE != 3 && MODE != 6) {
            const bool wc = lane > j + 1 && lane < M;
            cp[wc ? lane - j - 2 : M + 1] = make_double2(l0, l1);   // slot M + 1: scratch
            __builtin_nontemporal_store(l0, (live && lane >= j) ? Lj : Lsink);
            __builtin_nontemporal_store(l1, (live && lane >= j + 1) ? Lj + M : Lsink + 64);
        } else {
            if (lane > j + 1 && lane < M) cp[lane - j - 2] = make_double2(l0, l1);
        }
        Lj += 2 * M;
        if (MODE != 4 && MODE != 3 && MODE != 6) {
            const double y0 = readlane_d(wi, j) * inv0;
            if (lane == j) wi = y0;
            else if (lane > j) wi -= l0 * y0;
            const double y1 = readlane_d(wi, j + 1) * inv1;
            if (lane == j + 1) wi = y1;
            else if (lane > j + 1) wi -= l1 * y1;
        }
        if (MODE == 5 || MODE == 6) {
#pragma unroll
            for (int t = 0; t < M - 2; ++t) {
                const double cx = readlane_d(l0, j + 2 + t), cy = readlane_d(l1, j + 2 + t);
                row[t] = fma(-l1, cy, fma(-l0, cx, row[t + 2]));
            }
        } else if (MODE == 7) {
            wave_sync();
#pragma unroll
            for (int t0 = 0; t0 < M - 2; t0 += 8) {
                double2 c[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) c[u] = t0 + u < M - 2 ? cp[t0 + u] : make_double2(0.0, 0.0);
#pragma unroll
                for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(c[u].x), "+v"(c[u].y));
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (t0 + u < M - 2) row[t0 + u] = fma(-l1, c[u].y, fma(-l0, c[u].x, row[t0 + u + 2]));
            }
        } else {
            wave_sync();
#pragma unroll
            for (int t = 0; t < M - 2; ++t) {
                const double2 c = cp[t];
                row[t] = fma(-l1, c.y, fma(-l0, c.x, row[t + 2]));
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    asm volatile("" : "+v"(row[0]), "+v"(wi));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[0] = t1 - t0;
    if (lane == 0) cyc[1] = nbad;
    wout[lane] = wi;
#pragma unroll
    for (int c = 0; c < M; ++c) rows_out[lane * M + c] = row[c];
}

template <int M, int K, int MODE>
void run(const char* name, const double* dA, double* dL, double* dw, unsigned long long* dc, double* dr) {
    std::vector<double> tot;
    unsigned long long h[2];
    for (int rep = 0; rep < 20; ++rep) {
        hipLaunchKernelGGL((step<M, K, MODE>), dim3(1), dim3(64), 0, 0, dA, dL, dw, dc, dr);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
        if (rep >= 3) tot.push_back((double)h[0]);
    }
    std::sort(tot.begin(), tot.end());
    printf("  %-44s m %2d k %2d: %6.0f cycles per two-pivot step\n", name, M, K, tot[tot.size() / 2] / (K / 2));
}

template <int M, int K>
void suite(double* dA, double* dL, double* dw, unsigned long long* dc, double* dr) {
    std::vector<double> A(M * M);
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j) A[i * M + j] = (i == j ? 4.0 * M : 0.0) + 1.0 / (1.0 + i + j);
    (void)hipMemcpy(dA, A.data(), M * M * 8, hipMemcpyHostToDevice);
    run<M, K, 0>("static m, predicated stores", dA, dL, dw, dc, dr);
    run<M, K, 1>("static m, branch-free stores", dA, dL, dw, dc, dr);
    run<M, K, 4>("static m, branch-free, no forward step", dA, dL, dw, dc, dr);
    run<M, K, 2>("chain only (pivots + L columns)", dA, dL, dw, dc, dr);
    run<M, K, 3>("trailing update only (LDS broadcast + FMAs)", dA, dL, dw, dc, dr);
    run<M, K, 5>("static m, readlane broadcast", dA, dL, dw, dc, dr);
    run<M, K, 6>("trailing update only, readlane broadcast", dA, dL, dw, dc, dr);
    run<M, K, 7>("static m, LDS pairs read 8 at once", dA, dL, dw, dc, dr);
}

int main() {
    double *dA, *dL, *dw, *dr;
    unsigned long long* dc;
    (void)hipMalloc(&dA, 64 * 64 * 8);
    (void)hipMalloc(&dL, 64 * 64 * 8 * 8);
    (void)hipMalloc(&dw, 64 * 8);
    (void)hipMalloc(&dr, 64 * 64 * 8);
    (void)hipMalloc(&dc, 64 * 8);
    printf("two-pivot step anatomy, one wavefront alone (core cycles):\n");
    suite<18, 6>(dA, dL, dw, dc, dr);
    suite<42, 18>(dA, dL, dw, dc, dr);
    return 0;
}
