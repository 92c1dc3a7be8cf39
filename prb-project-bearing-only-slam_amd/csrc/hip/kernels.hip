// HIP kernels of one Gauss-Newton iteration for 2-D bearing-only SLAM on MI355X (gfx950).
//
// J+H build (the hot path, reference slam/solver.cpp:28-69 + solver_jacobians.cpp:9-168):
// ONE launch, two kinds of workgroups:
//   * pose-centric tasks: a wavefront owns a run of whole poses; lane = one bearing or one side
//     of an odometry edge incident to those poses. It evaluates e and J, applies the robust
//     kernel (scales e only, solver.cpp:37-41/54-58), reduces the pose-diagonal 3x3 blocks and
//     b_pose across its lanes through LDS in a fixed order (deterministic, no atomics), writes
//     the off-diagonal blocks whose CSR row belongs to the pose, and the chi^2 partial.
//   * landmark-centric tasks: the same for whole landmarks (2x2 diagonal, b_landmark and the
//     landmark-row off-diagonal blocks). A bearing is evaluated once on each side instead of
//     being scattered with atomics: recomputing ~100 flops is cheaper than a scattered 40-byte
//     atomic/partial round trip through HBM.
// All outputs of the two task kinds are disjoint, so the launch has no inter-workgroup
// communication. Damping (solver.cpp:64-69) is folded into the diagonal writes.
#include "kernels.hpp"

#include "../host/bos_math.hpp"

namespace bos {
namespace dev {

namespace {

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// position of entry (r, c) of the diagonal block of a node whose rows start at row0 with `base`
// entries of off-diagonal blocks before the diagonal (host/plan.cpp layout)
__device__ __forceinline__ int diag_pos(int row0, int base, int r, int c) {
    return row0 + r * base + ((r * (r + 1)) >> 1) + base + c;
}
// position of entry (r, c) of an off-diagonal block whose row-0 entry is at slot
__device__ __forceinline__ int off_pos(int slot, int base, int r, int c) {
    return slot + r * base + ((r * (r + 1)) >> 1) + c;
}

template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// lower-triangle index rv (0..5) -> (r, c)
__device__ __forceinline__ void tri_rc(int rv, int& r, int& c) {
    r = (rv >= 1) + (rv >= 3);
    c = rv - ((r * (r + 1)) >> 1);
}

template <typename T, bool HAS_W, bool HAS_GROUPS>
__device__ __forceinline__ void pose_task(const LinParams<T>& P, int t, int lane, T (*red)[64], T (*offr)[64]) {
    const int s0 = P.a_task[t], s1 = P.a_task[t + 1];
    const int i0 = P.a_seg_item[s0], i1 = P.a_seg_item[s1];
    const int nseg = s1 - s0;
    // reducer role: lane -> (segment rs, value rv) of the 9 reduced values per pose
    const int rs = lane / 9, rv = lane - 9 * (lane / 9);
    const bool reducer = rs < nseg;
    int r_beg = 0, r_end = 0;
    if (reducer) { r_beg = P.a_seg_item[s0 + rs]; r_end = P.a_seg_item[s0 + rs + 1]; }
    T acc = (T)0;
    double chi = 0.0;
    int nrob = 0;
    for (int c0 = i0; c0 < i1; c0 += 64) {
        const int i = c0 + lane;
        T v[9], off[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) { v[k] = (T)0; off[k] = (T)0; }
        int slot = -1, grp = i, ncol = 0, base = 0;
        if (i < i1) {
            int s = s0;
            while (s + 1 < s1 && P.a_seg_item[s + 1] <= i) ++s;
            const int p = P.a_seg_node[s];
            const int other = P.a_other[i];
            slot = P.a_slot[i];
            if (HAS_GROUPS) grp = P.a_grp[i];
            if (slot >= 0) base = P.p_base[p];
            if (other >= 0) {
                // ---- bearing (solver_jacobians.cpp:9-95), pose side
                const T px = P.pc[4 * p], py = P.pc[4 * p + 1], c = P.pc[4 * p + 2], sn = P.pc[4 * p + 3];
                const T lx = P.lc[2 * other], ly = P.lc[2 * other + 1];
                T J[5];
                T e = bos::bearing_error_jacobian<T>(px, py, c, sn, lx, ly, P.a_z[i], J);
                const T w = HAS_W ? P.a_w[i] : (T)1;
                const T rho = e * w * e;                                    // solver.cpp:37
                chi += (double)rho;
                if (rho > P.kt) { e *= sqrt(P.kt / rho); ++nrob; }          // :38-40
                T wJ[3];
#pragma unroll
                for (int r = 0; r < 3; ++r) wJ[r] = J[r] * w;
                v[0] = wJ[0] * J[0];
                v[1] = wJ[1] * J[0]; v[2] = wJ[1] * J[1];
                v[3] = wJ[2] * J[0]; v[4] = wJ[2] * J[1]; v[5] = wJ[2] * J[2];
                v[6] = wJ[0] * e; v[7] = wJ[1] * e; v[8] = wJ[2] * e;       // :45
#pragma unroll
                for (int r = 0; r < 3; ++r) { off[3 * r] = wJ[r] * J[3]; off[3 * r + 1] = wJ[r] * J[4]; }
                ncol = 2;
            } else {
                // ---- odometry edge side (solver_jacobians.cpp:97-168)
                const int code = -other - 1;
                const int k = code >> 1, side = code & 1;
                const int ps = P.o_src[k], pd = P.o_dst[k];
                const T xs = P.pc[4 * ps], ys = P.pc[4 * ps + 1], cs = P.pc[4 * ps + 2], ss = P.pc[4 * ps + 3];
                const T xd = P.pc[4 * pd], yd = P.pc[4 * pd + 1];
                T e[3], J[18];
                bos::odometry_error_jacobian<T>(xs, ys, P.pth[ps], cs, ss, xd, yd, P.pth[pd], P.o_z[3 * k],
                                                P.o_z[3 * k + 1], P.o_z[3 * k + 2], e, J);
                const T* u = P.o_om + 6 * k;
                const T Om[9] = {u[0], u[1], u[2], u[1], u[3], u[4], u[2], u[4], u[5]};
                T Oe[3];
#pragma unroll
                for (int r = 0; r < 3; ++r) Oe[r] = Om[3 * r] * e[0] + Om[3 * r + 1] * e[1] + Om[3 * r + 2] * e[2];
                const T rho = e[0] * Oe[0] + e[1] * Oe[1] + e[2] * Oe[2];  // solver.cpp:54
                if (side == 0) chi += (double)rho;
                if (rho > P.kt) {                                           // :55-57
                    const T sc = sqrt(P.kt / rho);
#pragma unroll
                    for (int r = 0; r < 3; ++r) Oe[r] *= sc;
                    if (side == 0) ++nrob;
                }
                const int me = 3 * side, ot = 3 - me;
                T OJ[9];   // Omega * J_me
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        OJ[3 * r + c] = Om[3 * r] * J[me + c] + Om[3 * r + 1] * J[6 + me + c] + Om[3 * r + 2] * J[12 + me + c];
#pragma unroll
                for (int rv2 = 0; rv2 < 6; ++rv2) {
                    int r, c;
                    tri_rc(rv2, r, c);
                    v[rv2] = J[me + r] * OJ[c] + J[6 + me + r] * OJ[3 + c] + J[12 + me + r] * OJ[6 + c];
                }
#pragma unroll
                for (int r = 0; r < 3; ++r) v[6 + r] = J[me + r] * Oe[0] + J[6 + me + r] * Oe[1] + J[12 + me + r] * Oe[2];
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        off[3 * r + c] = OJ[r] * J[ot + c] + OJ[3 + r] * J[6 + ot + c] + OJ[6 + r] * J[12 + ot + c];
                ncol = 3;
            }
        }
#pragma unroll
        for (int k = 0; k < 9; ++k) red[k][lane] = v[k];
        if (HAS_GROUPS) {
#pragma unroll
            for (int k = 0; k < 9; ++k) offr[k][lane] = off[k];
        }
        wave_lds_sync();
        if (slot >= 0) {
            if (HAS_GROUPS) {
                for (int j = grp - c0; j < lane; ++j)
#pragma unroll
                    for (int k = 0; k < 9; ++k) off[k] += offr[k][j];
            }
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < ncol; ++c) P.val[off_pos(slot, base, r, c)] = off[3 * r + c];
        }
        if (reducer) {
            const int lo = max(r_beg, c0) - c0, hi = min(r_end, c0 + 64) - c0;
            for (int j = lo; j < hi; ++j) acc += red[rv][j];
        }
        wave_lds_sync();
    }
    if (reducer) {
        const int p = P.a_seg_node[s0 + rs];
        if (rv < 6) {
            const int row0 = P.p_row0[p];
            if (row0 >= 0) {
                int r, c;
                tri_rc(rv, r, c);
                P.val[diag_pos(row0, P.p_base[p], r, c)] = acc + (r == c ? P.lambda : (T)0);
            }
        } else {
            P.b[P.p_bpos[p] + rv - 6] = acc;
        }
    }
    chi = wave_sum(chi);
    const int nr = (int)wave_sum((double)nrob);
    if (lane == 0) { P.chi2_part[t] = chi; P.nrob_part[t] = nr; }
}

template <typename T, bool HAS_W, bool HAS_GROUPS>
__device__ __forceinline__ void lm_task(const LinParams<T>& P, int t, int lane, T (*red)[64], T (*offr)[64]) {
    const int s0 = P.b_task[t], s1 = P.b_task[t + 1];
    const int i0 = P.b_seg_item[s0], i1 = P.b_seg_item[s1];
    const int nseg = s1 - s0;
    const int rs = lane / 5, rv = lane - 5 * (lane / 5);
    const bool reducer = rs < nseg;
    int r_beg = 0, r_end = 0;
    if (reducer) { r_beg = P.b_seg_item[s0 + rs]; r_end = P.b_seg_item[s0 + rs + 1]; }
    T acc = (T)0;
    for (int c0 = i0; c0 < i1; c0 += 64) {
        const int i = c0 + lane;
        T v[5], off[6];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = (T)0;
#pragma unroll
        for (int k = 0; k < 6; ++k) off[k] = (T)0;
        int slot = -1, grp = i, base = 0;
        if (i < i1) {
            int s = s0;
            while (s + 1 < s1 && P.b_seg_item[s + 1] <= i) ++s;
            const int l = P.b_seg_node[s];
            const int p = P.b_other[i];
            slot = P.b_slot[i];
            if (HAS_GROUPS) grp = P.b_grp[i];
            if (slot >= 0) base = P.l_base[l];
            const T px = P.pc[4 * p], py = P.pc[4 * p + 1], c = P.pc[4 * p + 2], sn = P.pc[4 * p + 3];
            const T lx = P.lc[2 * l], ly = P.lc[2 * l + 1];
            T J[5];
            T e = bos::bearing_error_jacobian<T>(px, py, c, sn, lx, ly, P.b_z[i], J);
            const T w = HAS_W ? P.b_w[i] : (T)1;
            const T rho = e * w * e;
            if (rho > P.kt) e *= sqrt(P.kt / rho);
            const T wJ3 = J[3] * w, wJ4 = J[4] * w;
            v[0] = wJ3 * J[3];
            v[1] = wJ4 * J[3]; v[2] = wJ4 * J[4];
            v[3] = wJ3 * e; v[4] = wJ4 * e;
            // landmark rows (2) x pose cols (3): H(l, p) = (J_l w) J_p
#pragma unroll
            for (int c2 = 0; c2 < 3; ++c2) { off[c2] = wJ3 * J[c2]; off[3 + c2] = wJ4 * J[c2]; }
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) red[k][lane] = v[k];
        if (HAS_GROUPS) {
#pragma unroll
            for (int k = 0; k < 6; ++k) offr[k][lane] = off[k];
        }
        wave_lds_sync();
        if (slot >= 0) {
            if (HAS_GROUPS) {
                for (int j = grp - c0; j < lane; ++j)
#pragma unroll
                    for (int k = 0; k < 6; ++k) off[k] += offr[k][j];
            }
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int c2 = 0; c2 < 3; ++c2) P.val[off_pos(slot, base, r, c2)] = off[3 * r + c2];
        }
        if (reducer) {
            const int lo = max(r_beg, c0) - c0, hi = min(r_end, c0 + 64) - c0;
            for (int j = lo; j < hi; ++j) acc += red[rv][j];
        }
        wave_lds_sync();
    }
    if (reducer) {
        const int l = P.b_seg_node[s0 + rs];
        if (rv < 3) {
            const int r = rv >= 1, cc = rv - r;
            P.val[diag_pos(P.l_row0[l], P.l_base[l], r, cc)] = acc + (r == cc ? P.lambda : (T)0);
        } else {
            P.b[P.l_bpos[l] + rv - 3] = acc;
        }
    }
}

template <typename T, bool HAS_W, bool HAS_GROUPS>
__global__ __launch_bounds__(kBlock) void linearize_kernel(const LinParams<T> P) {
    __shared__ T red[kWavesPerBlock][9][64];
    __shared__ T offr[kWavesPerBlock][HAS_GROUPS ? 9 : 1][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if ((int)blockIdx.x < P.nblk_pose) {
        const int t = blockIdx.x * kWavesPerBlock + wave;
        if (t < P.ntask_pose) pose_task<T, HAS_W, HAS_GROUPS>(P, t, lane, red[wave], offr[wave]);
    } else {
        const int t = (blockIdx.x - P.nblk_pose) * kWavesPerBlock + wave;
        if (t < P.ntask_lm) lm_task<T, HAS_W, HAS_GROUPS>(P, t, lane, red[wave], offr[wave]);
    }
}

template <typename T> __global__ void refresh_cache_kernel(const UpdateParams<T> U) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < U.NP) {
        const double x = U.pose[3 * i], y = U.pose[3 * i + 1], th = U.pose[3 * i + 2];
        U.pc[4 * i] = (T)x;
        U.pc[4 * i + 1] = (T)y;
        U.pc[4 * i + 2] = cos((T)th);
        U.pc[4 * i + 3] = sin((T)th);
        U.pth[i] = (T)th;
    } else if (i < U.NP + U.NL) {
        const int j = i - U.NP;
        U.lc[2 * j] = (T)U.lm[2 * j];
        U.lc[2 * j + 1] = (T)U.lm[2 * j + 1];
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

__global__ void scatter_dense_kernel(const int32_t* rowptr, const int32_t* colind, const double* val, int n,
                                     double* dense) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    for (int e = rowptr[r]; e < rowptr[r + 1]; ++e) dense[(int64_t)colind[e] * n + r] = val[e];  // col-major lower
}

}  // namespace

template <typename T>
hipError_t launch_linearize(const LinParams<T>& p, bool has_w, bool has_groups, hipStream_t s) {
    const int nblk_lm = (p.ntask_lm + kWavesPerBlock - 1) / kWavesPerBlock;
    const int grid = p.nblk_pose + nblk_lm;
    if (grid == 0) return hipSuccess;
    if (has_w) {
        if (has_groups) hipLaunchKernelGGL((linearize_kernel<T, true, true>), dim3(grid), dim3(kBlock), 0, s, p);
        else hipLaunchKernelGGL((linearize_kernel<T, true, false>), dim3(grid), dim3(kBlock), 0, s, p);
    } else {
        if (has_groups) hipLaunchKernelGGL((linearize_kernel<T, false, true>), dim3(grid), dim3(kBlock), 0, s, p);
        else hipLaunchKernelGGL((linearize_kernel<T, false, false>), dim3(grid), dim3(kBlock), 0, s, p);
    }
    return hipGetLastError();
}

template <typename T> hipError_t launch_refresh_cache(const UpdateParams<T>& p, hipStream_t s) {
    const int n = p.NP + p.NL;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL((refresh_cache_kernel<T>), dim3((n + 255) / 256), dim3(256), 0, s, p);
    return hipGetLastError();
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

hipError_t launch_scatter_dense(const int32_t* rowptr, const int32_t* colind, const double* val, int n, double* dense,
                                hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_dense_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rowptr, colind, val, n, dense);
    return hipGetLastError();
}

template hipError_t launch_linearize<double>(const LinParams<double>&, bool, bool, hipStream_t);
template hipError_t launch_linearize<float>(const LinParams<float>&, bool, bool, hipStream_t);
template hipError_t launch_refresh_cache<double>(const UpdateParams<double>&, hipStream_t);
template hipError_t launch_refresh_cache<float>(const UpdateParams<float>&, hipStream_t);
template hipError_t launch_boxplus<double>(const UpdateParams<double>&, hipStream_t);
template hipError_t launch_boxplus<float>(const UpdateParams<float>&, hipStream_t);
template hipError_t launch_to_f64<double>(const double*, double*, int64_t, hipStream_t);
template hipError_t launch_to_f64<float>(const float*, double*, int64_t, hipStream_t);

}  // namespace dev
}  // namespace bos
