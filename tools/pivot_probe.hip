// The multifrontal front's two-pivot loop (hip/multifrontal.hip factor_front_reg, product form) in
// isolation (diagnostic): one wavefront factors an m x m SPD front's first k columns with the rows
// in registers, s_memtime around every two-pivot step. Variants drop the L-panel stores or the fused
// forward step, to see what the step's cycles are made of. Prints the median cycles per step.
// Build: hipcc -O3 --offload-arch=gfx950 -fno-slp-vectorize tools/pivot_probe.hip -o gpurun_exp/pivot_probe
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

template <int MAXM, bool STORE_L, bool FORWARD, bool STAMP, bool FAST>
__global__ __launch_bounds__(64) void pivots(const double* A, int m, int k, double* L, double* wout,
                                             unsigned long long* cyc, double* rows_out) {
    __shared__ __attribute__((aligned(16))) double colbuf[2 * MAXM];
    const int lane = threadIdx.x;
    const bool live = lane < m;
    double row[MAXM];
#pragma unroll
    for (int c = 0; c < MAXM; ++c) row[c] = (live && c <= lane && c < m) ? A[lane * m + c] : 0.0;
    double wi = live ? 1.0 + 0.01 * lane : 0.0;
    double* Lj = L + lane;
    int nbad = 0;
    int j = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t = __builtin_amdgcn_s_memtime();
    const unsigned long long tstart = t;
    // FAST: a11 and A(j+1, j) read with the pivot (d1 = a11 - L(j+1,j)^2 needs no second readlane
    // of the updated column), the non-positive-pivot substitute selected after the rsqrt (its value
    // computed once), and the next step's first two columns updated from readlanes of lanes j+2, j+3
    // instead of the LDS broadcast
    const double inv_bad = rsqrt_nr(1e-300), l_bad = 1e-300 * inv_bad;
    if (FAST) {
#pragma nounroll
        for (; j + 1 < k; j += 2) {
            const double d0r = readlane_d(row[0], j), a10 = readlane_d(row[0], j + 1), a11 = readlane_d(row[1], j + 1);
            const bool bad0 = !(d0r > 0.0);
            nbad += bad0;
            const double r0 = rsqrt_nr(d0r);
            const double inv0 = bad0 ? inv_bad : r0, l00 = bad0 ? l_bad : d0r * r0;
            const double l0 = lane == j ? l00 : row[0] * inv0;
            const double lj1 = a10 * inv0;                       // = l0 of lane j + 1
            const double f1 = fma(-l0, lj1, row[1]);
            const double d1r = fma(-lj1, lj1, a11);               // = f1 of lane j + 1
            const bool bad1 = !(d1r > 0.0);
            nbad += bad1;
            const double r1 = rsqrt_nr(d1r);
            const double inv1 = bad1 ? inv_bad : r1, l11 = bad1 ? l_bad : d1r * r1;
            const double l1 = lane == j + 1 ? l11 : f1 * inv1;
            double2* cp = reinterpret_cast<double2*>(colbuf);
            if (lane > j + 1 && lane < m) cp[lane - j - 2] = make_double2(l0, l1);
            if (STORE_L && live) {
                if (lane >= j) __builtin_nontemporal_store(l0, Lj);
                if (lane >= j + 1) __builtin_nontemporal_store(l1, Lj + m);
            }
            Lj += 2 * m;
            // the next pivots' columns (t = 0, 1) from lanes j + 2, j + 3 directly
            const double p0 = readlane_d(l0, j + 2), p1 = readlane_d(l1, j + 2);
            const double q0 = readlane_d(l0, j + 3), q1 = readlane_d(l1, j + 3);
            const double n0 = fma(-l1, p1, fma(-l0, p0, row[2]));
            const double n1 = fma(-l1, q1, fma(-l0, q0, row[3]));
            if (FORWARD) {
                const double y0 = readlane_d(wi, j) * inv0;
                if (lane == j) wi = y0;
                else if (lane > j) wi -= l0 * y0;
                const double y1 = readlane_d(wi, j + 1) * inv1;
                if (lane == j + 1) wi = y1;
                else if (lane > j + 1) wi -= l1 * y1;
            }
            wave_sync();
            const int nt = m - j - 2;
#pragma unroll
            for (int t0 = 0; t0 < MAXM - 2; t0 += 8) {
                if (t0 < nt) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int tt = t0 + u;
                        if (tt >= 2 && tt < MAXM - 2) {
                            const double2 c = cp[tt];
                            row[tt] = fma(-l1, c.y, fma(-l0, c.x, row[tt + 2]));
                        }
                    }
                }
            }
            row[0] = n0;
            row[1] = n1;
            __builtin_amdgcn_wave_barrier();
            if (STAMP) {
                asm volatile("" : "+v"(row[0]));
                const unsigned long long t1 = __builtin_amdgcn_s_memtime();
                if (lane == 0) cyc[j / 2] = t1 - t;
                t = t1;
            }
        }
    }
#pragma nounroll
    for (; j + 1 < k; j += 2) {
        double d0 = readlane_d(row[0], j);
        const bool bad0 = !(d0 > 0.0);
        nbad += bad0;
        d0 = bad0 ? 1e-300 : d0;
        const double inv0 = rsqrt_nr(d0), l00 = d0 * inv0;
        const double l0 = lane == j ? l00 : row[0] * inv0;
        const double lj1 = readlane_d(l0, j + 1);
        const double f1 = fma(-l0, lj1, row[1]);
        double d1 = readlane_d(f1, j + 1);
        const bool bad1 = !(d1 > 0.0);
        nbad += bad1;
        d1 = bad1 ? 1e-300 : d1;
        const double inv1 = rsqrt_nr(d1), l11 = d1 * inv1;
        const double l1 = lane == j + 1 ? l11 : f1 * inv1;
        double2* cp = reinterpret_cast<double2*>(colbuf);
        if (lane > j + 1 && lane < m) cp[lane - j - 2] = make_double2(l0, l1);
        if (STORE_L && live) {
            if (lane >= j) __builtin_nontemporal_store(l0, Lj);
            if (lane >= j + 1) __builtin_nontemporal_store(l1, Lj + m);
        }
        Lj += 2 * m;
        if (FORWARD) {
            const double y0 = readlane_d(wi, j) * inv0;
            if (lane == j) wi = y0;
            else if (lane > j) wi -= l0 * y0;
            const double y1 = readlane_d(wi, j + 1) * inv1;
            if (lane == j + 1) wi = y1;
            else if (lane > j + 1) wi -= l1 * y1;
        }
        wave_sync();
        const int nt = m - j - 2;
#pragma unroll
        for (int t0 = 0; t0 < MAXM - 2; t0 += 8) {
            if (t0 < nt) {
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int tt = t0 + u;
                    if (tt < MAXM - 2) {
                        const double2 c = cp[tt];
                        row[tt] = fma(-l1, c.y, fma(-l0, c.x, row[tt + 2]));
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (STAMP) {
            asm volatile("" : "+v"(row[0]));
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            if (lane == 0) cyc[j / 2] = t1 - t;
            t = t1;
        }
    }
    asm volatile("" : "+v"(row[0]), "+v"(wi));
    const unsigned long long tend = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[63] = tend - tstart;
    if (lane == 0) cyc[62] = nbad;
    wout[lane] = wi;
#pragma unroll
    for (int c = 0; c < MAXM; ++c) rows_out[lane * MAXM + c] = row[c];
}

template <int MAXM, bool S, bool F, bool ST, bool FA = false>
void run(const char* name, int m, int k, const double* dA, double* dL, double* dw, unsigned long long* dc, double* dr) {
    std::vector<double> tot;
    std::vector<unsigned long long> h(64);
    std::vector<double> per;
    for (int rep = 0; rep < 20; ++rep) {
        hipLaunchKernelGGL((pivots<MAXM, S, F, ST, FA>), dim3(1), dim3(64), 0, 0, dA, m, k, dL, dw, dc, dr);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h.data(), dc, 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        if (rep < 3) continue;
        tot.push_back((double)h[63]);
        if (ST)
            for (int s = 0; s < k / 2; ++s) per.push_back((double)h[s]);
    }
    std::sort(tot.begin(), tot.end());
    std::sort(per.begin(), per.end());
    printf("  %-34s m %2d k %2d: loop %7.0f cycles = %6.0f per two-pivot step%s", name, m, k, tot[tot.size() / 2],
           tot[tot.size() / 2] / (k / 2), ST ? "" : "\n");
    if (ST) printf("; stamped steps: median %6.0f, min %6.0f\n", per[per.size() / 2], per[0]);
}

int main() {
    const int MM = 48;
    std::vector<double> A(MM * MM);
    for (int i = 0; i < MM; ++i)
        for (int j = 0; j < MM; ++j) A[i * MM + j] = (i == j ? 4.0 * MM : 0.0) + 1.0 / (1.0 + i + j);
    double *dA[2], *dL, *dw, *dr;
    unsigned long long* dc;
    (void)hipMalloc(&dL, 64 * 64 * 8 * 8);
    (void)hipMalloc(&dw, 64 * 8);
    (void)hipMalloc(&dr, 64 * 64 * 8);
    (void)hipMalloc(&dc, 64 * 8);
    for (int v = 0; v < 2; ++v) (void)hipMalloc(&dA[v], MM * MM * 8);
    auto upload = [&](int m) {   // the leading m x m block, row-major with stride m
        std::vector<double> B(m * m);
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < m; ++j) B[i * m + j] = A[i * MM + j];
        (void)hipMemcpy(dA[0], B.data(), m * m * 8, hipMemcpyHostToDevice);
    };
    printf("two-pivot steps of the front loop, one wavefront alone (core cycles):\n");
    const int cases[][2] = {{18, 6}, {42, 18}, {24, 12}};
    for (auto& c : cases) {
        const int m = c[0], k = c[1];
        upload(m);
        run<48, true, true, false>("product (L stores, forward)", m, k, dA[0], dL, dw, dc, dr);
        run<48, true, true, true>("product, stamped", m, k, dA[0], dL, dw, dc, dr);
        run<48, false, true, false>("no L stores", m, k, dA[0], dL, dw, dc, dr);
        run<48, true, false, false>("no forward step", m, k, dA[0], dL, dw, dc, dr);
        run<48, false, false, false>("neither", m, k, dA[0], dL, dw, dc, dr);
        if (m <= 24) run<24, true, true, false>("product, rows of 24 (MAXM 24)", m, k, dA[0], dL, dw, dc, dr);
        std::vector<double> r1(64 * 48), w1(64), L1(64 * 64 * 8), r2(64 * 48), w2(64), L2(64 * 64 * 8);
        run<48, true, true, false>("(check: product)", m, k, dA[0], dL, dw, dc, dr);
        (void)hipMemcpy(r1.data(), dr, r1.size() * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(w1.data(), dw, w1.size() * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(L1.data(), dL, L1.size() * 8, hipMemcpyDeviceToHost);
        (void)hipMemset(dL, 0, L1.size() * 8);
        run<48, true, true, false, true>("fast (product outputs)", m, k, dA[0], dL, dw, dc, dr);
        (void)hipMemcpy(r2.data(), dr, r2.size() * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(w2.data(), dw, w2.size() * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(L2.data(), dL, L2.size() * 8, hipMemcpyDeviceToHost);
        int diff = 0;
        for (int i = 0; i < m; ++i) {
            for (int c = 0; c < 48; ++c) diff += c <= i - k && r1[i * 48 + c] != r2[i * 48 + c];   // the trailing block
            diff += w1[i] != w2[i];
        }
        for (int q = 0; q < k * m; ++q) diff += L1[q] != L2[q];
        printf("  fast vs product: %d differing values (trailing rows, forward results, L)\n", diff);
        run<48, true, true, true, true>("fast, stamped", m, k, dA[0], dL, dw, dc, dr);
    }
    return 0;
}
