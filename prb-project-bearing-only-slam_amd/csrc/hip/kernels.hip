// HIP kernels of one Gauss-Newton iteration for 2-D bearing-only SLAM on MI355X (gfx950).
//
// J+H build (the hot path, reference slam/solver.cpp:28-69 + solver_jacobians.cpp:9-168), one
// launch, no LDS and no atomics. H is written block-sparse in observation order (host/plan.hpp
// BlockLayout), every value exactly once:
//   * pose lanes (lpp per pose): each lane walks a segment of its pose's bearings (sorted by
//     landmark) — error, Jacobian, robust kernel (scales e only, solver.cpp:37-41) — accumulating
//     the pose's diagonal block and b in registers and storing each pose-landmark block H_pl as it
//     goes (lists are wave-interleaved, so every step of a wave reads 64 consecutive records and
//     writes 64 consecutive blocks); lane 0 of the group also walks the pose's odometry edges (both sides accumulate
//     H_ss = H_dd, the source side stores H_sd = -H_ss and counts chi^2). The group's partial sums
//     are combined with a fixed butterfly (deterministic) and stored with the damping (:64-69).
//   * landmark lanes: one per landmark, walking its bearings for H_ll and b_l (+ damping).
// A bearing is evaluated twice (pose side, landmark side): the arithmetic is cheap next to the
// memory traffic, and no lane ever reads what another writes.
#include "kernels.hpp"

#include "../host/bos_math.hpp"

namespace bos {
namespace dev {

namespace {

template <typename T> struct alignas(4 * sizeof(T)) V4 { T x, y, z, w; };
template <typename T> struct alignas(2 * sizeof(T)) V2 { T x, y; };

template <typename T> __device__ __forceinline__ V4<T> load4(const T* p) { return *(const V4<T>*)p; }
template <typename T> __device__ __forceinline__ V2<T> load2(const T* p) { return *(const V2<T>*)p; }
// six values at an even offset of the block array (8-byte aligned for fp32, 16 for fp64)
template <typename T> __device__ __forceinline__ void store6(T* p, T a, T b, T c, T d, T e, T f) {
    V2<T>* q = (V2<T>*)p;
    q[0] = V2<T>{a, b};
    q[1] = V2<T>{c, d};
    q[2] = V2<T>{e, f};
}

template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Odometry edge (solver_jacobians.cpp:97-168) seen from one endpoint. J_dst = -J_src exactly in
// the reference's Jacobian (:137-146: (DR' R_s)^T = -R_s^T DR', DR' antisymmetric), so
// H_ss = H_dd = J_s^T Omega J_s, H_sd = -H_ss, b_d = -b_s. Returns rho = e^T Omega e; h = H_ss
// (00, 10, 11, 20, 21, 22), g = b_s.
template <typename T>
__device__ __forceinline__ T odometry_hb(const LinParams<T>& P, int k, const V4<T>& S, T ths, const V4<T>& D, T thd,
                                         T h[6], T g[3]) {
    const T xs = S.x, ys = S.y, cs = S.z, ss = S.w, xd = D.x, yd = D.y;
    const T tx = xd - xs, ty = yd - ys;
    const T e0 = (cs * tx + ss * ty) - P.o_z[3 * k];                                // :106, :319
    const T e1 = (-ss * tx + cs * ty) - P.o_z[3 * k + 1];
    const T e2 = bos::normalized_angle<T>(bos::normalized_angle<T>(thd - ths) - P.o_z[3 * k + 2]);
    const T t0 = -ss * xd + cs * yd, t1 = -cs * xd - ss * yd;                       // :139
    // J_s = [[-cs, -ss, t0], [ss, -cs, t1], [0, 0, -1]]
    const T* u = P.o_om + 6 * k;
    const T o00 = u[0], o01 = u[1], o02 = u[2], o11 = u[3], o12 = u[4], o22 = u[5];
    T Oe0 = o00 * e0 + o01 * e1 + o02 * e2;
    T Oe1 = o01 * e0 + o11 * e1 + o12 * e2;
    T Oe2 = o02 * e0 + o12 * e1 + o22 * e2;
    const T rho = e0 * Oe0 + e1 * Oe1 + e2 * Oe2;                                   // solver.cpp:54
    if (rho > P.kt) {                                                               // :55-57
        const T sc = sqrt(P.kt / rho);
        Oe0 *= sc; Oe1 *= sc; Oe2 *= sc;
    }
    // Omega J_s, column by column
    const T a00 = -o00 * cs + o01 * ss, a01 = -o00 * ss - o01 * cs, a02 = o00 * t0 + o01 * t1 - o02;
    const T a10 = -o01 * cs + o11 * ss, a11 = -o01 * ss - o11 * cs, a12 = o01 * t0 + o11 * t1 - o12;
    const T a20 = -o02 * cs + o12 * ss, a21 = -o02 * ss - o12 * cs, a22 = o02 * t0 + o12 * t1 - o22;
    // H_ss = J_s^T (Omega J_s)
    h[0] = -cs * a00 + ss * a10;
    h[1] = -ss * a00 - cs * a10;
    h[2] = -ss * a01 - cs * a11;
    h[3] = t0 * a00 + t1 * a10 - a20;
    h[4] = t0 * a01 + t1 * a11 - a21;
    h[5] = t0 * a02 + t1 * a12 - a22;
    g[0] = -cs * Oe0 + ss * Oe1;
    g[1] = -ss * Oe0 - cs * Oe1;
    g[2] = t0 * Oe0 + t1 * Oe1 - Oe2;
    return rho;
}

template <typename T, bool HAS_W, bool HAS_DUPS, int LPP>
__device__ __forceinline__ void pose_lanes(const LinParams<T>& P, double& chi, int& nrob) {
    const int g = P.p_begin * LPP + blockIdx.x * kBlock + threadIdx.x;   // lane; shards start at a wave
    const int p = g / LPP, sub = g % LPP, t = g & 63;
    const bool active = p < P.p_end;
    T h[6] = {0, 0, 0, 0, 0, 0}, gb[3] = {0, 0, 0};
    if (active) {
        const V4<T> X = load4(P.pc + 4 * p);
        const int n = P.pl_cnt[g];
        int sl = P.pw_base[g >> 6] + t;   // slot of item j: + 64 j
        T acc[6] = {0, 0, 0, 0, 0, 0};
        // two-stage software pipeline: record j+2 and the landmark of item j+1 are in flight while
        // item j is evaluated
        BRec<T> nxt, nxt2;
        V2<T> Lnxt;
        if (n > 0) { nxt = P.pb[sl]; Lnxt = load2(P.lc + 2 * nxt.idx); }
        if (n > 1) nxt2 = P.pb[sl + 64];
        for (int j = 0; j < n; ++j, sl += 64) {
            const BRec<T> cur = nxt;
            const V2<T> Lm = Lnxt;
            if (j + 1 < n) { nxt = nxt2; Lnxt = load2(P.lc + 2 * nxt.idx); }
            if (j + 2 < n) nxt2 = P.pb[sl + 128];
            T J[5];
            T e = bos::bearing_error_jacobian<T>(X.x, X.y, X.z, X.w, Lm.x, Lm.y, cur.z, J);   // :9-95
            const T w = HAS_W ? P.pb_w[sl] : (T)1;
            const T rho = e * w * e;                                                       // solver.cpp:37
            chi += (double)rho;
            if (rho > P.kt) {                                                              // :38-40
                e *= sqrt(P.kt / rho);
                ++nrob;
            }
            // H += (J^T w) J, b += (J^T w) e (:44-45)
            const T w0 = J[0] * w, w1 = J[1] * w, w2 = J[2] * w;
            h[0] += w0 * J[0]; h[1] += w1 * J[0]; h[2] += w1 * J[1];
            h[3] += w2 * J[0]; h[4] += w2 * J[1]; h[5] += w2 * J[2];
            gb[0] += w0 * e; gb[1] += w1 * e; gb[2] += w2 * e;
            const T o0 = w0 * J[3], o1 = w0 * J[4], o2 = w1 * J[3], o3 = w1 * J[4], o4 = w2 * J[3], o5 = w2 * J[4];
            T* blk = P.hval + P.off_pl + 6 * sl;
            if (HAS_DUPS) {   // observations of one pair are adjacent: sum, store at the last one
                acc[0] += o0; acc[1] += o1; acc[2] += o2; acc[3] += o3; acc[4] += o4; acc[5] += o5;
                if (j + 1 == n || nxt.idx != cur.idx) {
                    store6(blk, acc[0], acc[1], acc[2], acc[3], acc[4], acc[5]);
#pragma unroll
                    for (int q = 0; q < 6; ++q) acc[q] = (T)0;
                }
            } else {
                store6(blk, o0, o1, o2, o3, o4, o5);
            }
        }
        if (sub == 0) {
            const T th = P.pth[p];
            T acc6[6] = {0, 0, 0, 0, 0, 0};
            const int x1 = P.po_ptr[p + 1];
            for (int x = P.po_ptr[p]; x < x1; ++x) {
                const int ent = P.po_ent[x], k = ent >> 1;
                const bool dst_side = ent & 1;
                const int q = dst_side ? P.o_src[k] : P.o_dst[k];
                const V4<T> Q = load4(P.pc + 4 * q);
                const T thq = P.pth[q];
                T he[6], ge[3];
                const T rho = dst_side ? odometry_hb<T>(P, k, Q, thq, X, th, he, ge)
                                       : odometry_hb<T>(P, k, X, th, Q, thq, he, ge);
#pragma unroll
                for (int v = 0; v < 6; ++v) h[v] += he[v];
                if (dst_side) {
                    gb[0] -= ge[0]; gb[1] -= ge[1]; gb[2] -= ge[2];
                    continue;
                }
                gb[0] += ge[0]; gb[1] += ge[1]; gb[2] += ge[2];
                chi += (double)rho;
                if (rho > P.kt) ++nrob;
                const int ub = P.po_blk[x];
                T* ob = P.hval + P.off_pp + 6 * ub;
                if (HAS_DUPS) {
#pragma unroll
                    for (int v = 0; v < 6; ++v) acc6[v] -= he[v];
                    if (x + 1 == x1 || P.po_blk[x + 1] != ub) {
                        store6(ob, acc6[0], acc6[1], acc6[2], acc6[3], acc6[4], acc6[5]);
#pragma unroll
                        for (int v = 0; v < 6; ++v) acc6[v] = (T)0;
                    }
                } else {
                    store6(ob, -he[0], -he[1], -he[2], -he[3], -he[4], -he[5]);
                }
            }
        }
    }
    // combine the lane group's partial sums (fixed butterfly: deterministic)
#pragma unroll
    for (int o = 1; o < LPP; o <<= 1) {
#pragma unroll
        for (int v = 0; v < 6; ++v) h[v] += __shfl_xor(h[v], o);
#pragma unroll
        for (int v = 0; v < 3; ++v) gb[v] += __shfl_xor(gb[v], o);
    }
    if (active && sub == 0) {
        const T lam = P.lambda;
        store6(P.hval + 6 * p, h[0] + lam, h[1], h[2] + lam, h[3], h[4], h[5] + lam);
        T* bp = P.b + 3 * p;
        bp[0] = gb[0]; bp[1] = gb[1]; bp[2] = gb[2];
    }
}

template <typename T, bool HAS_W>
__device__ __forceinline__ void landmark_lane(const LinParams<T>& P) {
    const int l = P.l_begin + (blockIdx.x - P.pose_blocks) * kBlock + threadIdx.x;   // shards start at a wave
    if (l >= P.l_end) return;
    const V2<T> Lm = load2(P.lc + 2 * l);
    T h00 = 0, h10 = 0, h11 = 0, g0 = 0, g1 = 0;
    const int n = P.ll_cnt[l];
    int sl = P.lw_base[l >> 6] + (l & 63);
    BRec<T> nxt, nxt2;
    V4<T> Xnxt;
    if (n > 0) { nxt = P.lb[sl]; Xnxt = load4(P.pc + 4 * nxt.idx); }
    if (n > 1) nxt2 = P.lb[sl + 64];
    for (int j = 0; j < n; ++j, sl += 64) {
        const BRec<T> cur = nxt;
        const V4<T> X = Xnxt;
        if (j + 1 < n) { nxt = nxt2; Xnxt = load4(P.pc + 4 * nxt.idx); }
        if (j + 2 < n) nxt2 = P.lb[sl + 128];
        T J[5];
        T e = bos::bearing_error_jacobian<T>(X.x, X.y, X.z, X.w, Lm.x, Lm.y, cur.z, J);
        const T w = HAS_W ? P.lb_w[sl] : (T)1;
        const T rho = e * w * e;
        if (rho > P.kt) e *= sqrt(P.kt / rho);
        const T w3 = J[3] * w, w4 = J[4] * w;
        h00 += w3 * J[3]; h10 += w4 * J[3]; h11 += w4 * J[4];
        g0 += w3 * e; g1 += w4 * e;
    }
    T* hl = P.hval + P.off_ldiag + 3 * l;
    hl[0] = h00 + P.lambda; hl[1] = h10; hl[2] = h11 + P.lambda;
    T* bl = P.b + 3 * P.NP + 2 * l;
    bl[0] = g0; bl[1] = g1;
}

template <typename T, bool HAS_W, bool HAS_DUPS, int LPP>
__global__ __launch_bounds__(kBlock) void linearize_kernel(const LinParams<T> P) {
    if ((int)blockIdx.x >= P.pose_blocks) {   // block-uniform branch
        landmark_lane<T, HAS_W>(P);
        return;
    }
    double chi = 0.0;
    int nrob = 0;
    pose_lanes<T, HAS_W, HAS_DUPS, LPP>(P, chi, nrob);
    // per-block chi^2 / robust count in a fixed order
    __shared__ double sc[kBlock / 64];
    __shared__ int sr[kBlock / 64];
    chi = wave_sum(chi);
    nrob = (int)wave_sum((double)nrob);
    if ((threadIdx.x & 63) == 0) { sc[threadIdx.x >> 6] = chi; sr[threadIdx.x >> 6] = nrob; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double c = 0.0;
        int r = 0;
        for (int w = 0; w < kBlock / 64; ++w) { c += sc[w]; r += sr[w]; }
        P.chi2_part[blockIdx.x] = c;
        P.nrob_part[blockIdx.x] = r;
    }
}

// State::apply_boxplus (framework/state.cpp:69-80): dx = -x (the solve ran on +b)
template <typename T> __global__ void boxplus_kernel(const UpdateParams<T> U) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double m = 0.0;
    if (i < U.NP) {
        if (i != U.fixed) {
            const int d = U.node_dof[i];
            const double dx = -U.x[d], dy = -U.x[d + 1], dth = -U.x[d + 2];
            double x = U.pose[3 * i], y = U.pose[3 * i + 1], th = U.pose[3 * i + 2];
            bos::boxplus_pose<double>(x, y, th, dx, dy, dth);
            U.pose[3 * i] = x;
            U.pose[3 * i + 1] = y;
            U.pose[3 * i + 2] = th;
            U.pc[4 * i] = (T)x;
            U.pc[4 * i + 1] = (T)y;
            U.pc[4 * i + 2] = cos((T)th);
            U.pc[4 * i + 3] = sin((T)th);
            U.pth[i] = (T)th;
            m = fmax(fabs(dx), fmax(fabs(dy), fabs(dth)));
        }
    } else if (i < U.NP + U.NL) {
        const int j = i - U.NP;
        const int d = U.node_dof[i];
        const double dx = -U.x[d], dy = -U.x[d + 1];
        const double x = U.lm[2 * j] + dx, y = U.lm[2 * j + 1] + dy;
        U.lm[2 * j] = x;
        U.lm[2 * j + 1] = y;
        U.lc[2 * j] = (T)x;
        U.lc[2 * j + 1] = (T)y;
        m = fmax(fabs(dx), fabs(dy));
    }
    // max is order independent: deterministic
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0 && m > 0.0)
        atomicMax(U.max_dx_bits, (unsigned long long)__double_as_longlong(m));
}

__global__ void reduce_stats_kernel(const double* chi_part, const int32_t* nrob_part, int n, double* chi_out,
                                    int32_t* nrob_out) {
    __shared__ double sc[256];
    __shared__ long long sr[256];
    double c = 0.0;
    long long r = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) { c += chi_part[i]; r += nrob_part[i]; }
    sc[threadIdx.x] = c;
    sr[threadIdx.x] = r;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) { sc[threadIdx.x] += sc[threadIdx.x + o]; sr[threadIdx.x] += sr[threadIdx.x + o]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { *chi_out = sc[0]; *nrob_out = (int32_t)sr[0]; }
}

template <typename T> __global__ void to_f64_kernel(const T* in, double* out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (double)in[i];
}

template <typename T> __global__ void gather_f64_kernel(const T* in, const int32_t* idx, double* out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (double)in[idx[i]];
}

__global__ void scatter_dense_kernel(const int32_t* rowptr, const int32_t* colind, const double* val, int n,
                                     double* dense) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    for (int e = rowptr[r]; e < rowptr[r + 1]; ++e) dense[(int64_t)colind[e] * n + r] = val[e];  // col-major lower
}

}  // namespace

template <typename T, bool W, bool D>
hipError_t launch_lin_lpp(const LinParams<T>& p, int lpp, int grid, hipStream_t s) {
    switch (lpp) {
        case 1: hipLaunchKernelGGL((linearize_kernel<T, W, D, 1>), dim3(grid), dim3(kBlock), 0, s, p); break;
        case 2: hipLaunchKernelGGL((linearize_kernel<T, W, D, 2>), dim3(grid), dim3(kBlock), 0, s, p); break;
        case 4: hipLaunchKernelGGL((linearize_kernel<T, W, D, 4>), dim3(grid), dim3(kBlock), 0, s, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_linearize(const LinParams<T>& p, int lpp, bool has_w, bool has_dups, hipStream_t s) {
    const int grid = p.pose_blocks + (p.l_end - p.l_begin + kBlock - 1) / kBlock;
    if (grid == 0) return hipSuccess;
    if (has_w) return has_dups ? launch_lin_lpp<T, true, true>(p, lpp, grid, s) : launch_lin_lpp<T, true, false>(p, lpp, grid, s);
    return has_dups ? launch_lin_lpp<T, false, true>(p, lpp, grid, s) : launch_lin_lpp<T, false, false>(p, lpp, grid, s);
}

template <typename T> hipError_t launch_boxplus(const UpdateParams<T>& p, hipStream_t s) {
    const int n = p.NP + p.NL;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL((boxplus_kernel<T>), dim3((n + 255) / 256), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_reduce_stats(const double* chi_part, const int32_t* nrob_part, int n, double* chi_out,
                               int32_t* nrob_out, hipStream_t s) {
    hipLaunchKernelGGL(reduce_stats_kernel, dim3(1), dim3(256), 0, s, chi_part, nrob_part, n, chi_out, nrob_out);
    return hipGetLastError();
}

template <typename T> hipError_t launch_to_f64(const T* in, double* out, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL((to_f64_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_gather_f64(const T* in, const int32_t* idx, double* out, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL((gather_f64_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, in, idx, out, n);
    return hipGetLastError();
}

hipError_t launch_scatter_dense(const int32_t* rowptr, const int32_t* colind, const double* val, int n, double* dense,
                                hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_dense_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rowptr, colind, val, n, dense);
    return hipGetLastError();
}

template hipError_t launch_linearize<double>(const LinParams<double>&, int, bool, bool, hipStream_t);
template hipError_t launch_linearize<float>(const LinParams<float>&, int, bool, bool, hipStream_t);
template hipError_t launch_boxplus<double>(const UpdateParams<double>&, hipStream_t);
template hipError_t launch_boxplus<float>(const UpdateParams<float>&, hipStream_t);
template hipError_t launch_to_f64<double>(const double*, double*, int64_t, hipStream_t);
template hipError_t launch_to_f64<float>(const float*, double*, int64_t, hipStream_t);
template hipError_t launch_gather_f64<double>(const double*, const int32_t*, double*, int64_t, hipStream_t);
template hipError_t launch_gather_f64<float>(const float*, const int32_t*, double*, int64_t, hipStream_t);

}  // namespace dev
}  // namespace bos
