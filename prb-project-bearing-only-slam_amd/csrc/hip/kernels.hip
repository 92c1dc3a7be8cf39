// HIP kernels of one Gauss-Newton iteration for 2-D bearing-only SLAM on MI355X (gfx950).
//
// J+H build (the hot path, reference slam/solver.cpp:28-69 + solver_jacobians.cpp:9-168), one
// launch. A wavefront owns a task = a contiguous range of nodes in elimination order (host/plan.cpp
// build_tasks), so the CSR rows it produces are ONE contiguous span of the value array:
//   1. lane = one observation incident to the task's nodes: error, Jacobian, robust kernel
//      (scales e only, solver.cpp:37-41/54-58); its per-side contributions (diagonal block + b)
//      go to LDS slots and its off-diagonal block, when the block's row lives in this task, goes
//      straight into the LDS image of the rows;
//   2. lanes (node, value) reduce the slots in a fixed order (deterministic, no atomics) into the
//      diagonal blocks (+ damping, solver.cpp:64-69) and b;
//   3. the row image and b are stored with coalesced writes.
// An observation whose endpoints lie in two tasks is evaluated in both; no workgroup reads what
// another writes, so the launch has no inter-workgroup communication.
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

// Contributions of one side of an observation go to slots[v][2 * entry + side]: pose side 9
// values (H 00,10,11,20,21,22, b 0..2), landmark side 5 values (H 00,10,11, b 0,1).

template <typename T, bool HAS_W, bool HAS_DUPS>
__device__ __forceinline__ void eval_bearing(const LinParams<T>& P, int i, int ll, T* rows, T (*slots)[kSlots],
                                             double& chi, int& nrob) {
    const int meta = P.be_meta[i];
    const int p = P.be_pose[i], l = P.be_lm[i];
    const T px = P.pc[4 * p], py = P.pc[4 * p + 1], c = P.pc[4 * p + 2], sn = P.pc[4 * p + 3];
    const T lx = P.lc[2 * l], ly = P.lc[2 * l + 1];
    T J[5];
    T e = bos::bearing_error_jacobian<T>(px, py, c, sn, lx, ly, P.be_z[i], J);   // solver_jacobians.cpp:9-95
    const T w = HAS_W ? P.be_w[i] : (T)1;
    const T rho = e * w * e;                                                        // solver.cpp:37
    if (meta & 4) chi += (double)rho;
    if (rho > P.kt) {                                                               // solver.cpp:38-40
        e *= sqrt(P.kt / rho);
        if (meta & 4) ++nrob;
    }
    // H += (J^T w) J, b += (J^T w) e  (solver.cpp:44-45)
    const T wJ0 = J[0] * w, wJ1 = J[1] * w, wJ2 = J[2] * w, wJ3 = J[3] * w, wJ4 = J[4] * w;
    if (meta & 1) {
        slots[0][2 * ll] = wJ0 * J[0];
        slots[1][2 * ll] = wJ1 * J[0];
        slots[2][2 * ll] = wJ1 * J[1];
        slots[3][2 * ll] = wJ2 * J[0];
        slots[4][2 * ll] = wJ2 * J[1];
        slots[5][2 * ll] = wJ2 * J[2];
        slots[6][2 * ll] = wJ0 * e;
        slots[7][2 * ll] = wJ1 * e;
        slots[8][2 * ll] = wJ2 * e;
    }
    if (meta & 2) {
        slots[0][2 * ll + 1] = wJ3 * J[3];
        slots[1][2 * ll + 1] = wJ4 * J[3];
        slots[2][2 * ll + 1] = wJ4 * J[4];
        slots[3][2 * ll + 1] = wJ3 * e;
        slots[4][2 * ll + 1] = wJ4 * e;
    }
    if (meta & 8) {
        const T wo = HAS_DUPS ? P.be_woff[i] : w;
        T* blk = rows + (meta >> 8);
        if (meta & 16) {   // landmark rows (2) x pose cols (3)
            const int base = P.node_base[P.NP + l];
            const T a0 = J[3] * wo, a1 = J[4] * wo;
            blk[0] = a0 * J[0]; blk[1] = a0 * J[1]; blk[2] = a0 * J[2];
            blk += base + 1;
            blk[0] = a1 * J[0]; blk[1] = a1 * J[1]; blk[2] = a1 * J[2];
        } else {           // pose rows (3) x landmark cols (2)
            const int base = P.node_base[p];
            const T a0 = J[0] * wo, a1 = J[1] * wo, a2 = J[2] * wo;
            blk[0] = a0 * J[3]; blk[1] = a0 * J[4];
            blk += base + 1;
            blk[0] = a1 * J[3]; blk[1] = a1 * J[4];
            blk += base + 2;
            blk[0] = a2 * J[3]; blk[1] = a2 * J[4];
        }
    }
}

// Odometry edge (solver_jacobians.cpp:97-168). J_dst = -J_src exactly in the reference's
// Jacobian (:137-146: (DR' R_s)^T = -R_s^T DR' since DR' is antisymmetric), so
// H_ss = H_dd = J_s^T Omega J_s, H_sd = -H_ss, b_d = -b_s.
template <typename T, bool HAS_DUPS>
__device__ __forceinline__ void eval_odometry(const LinParams<T>& P, int j, int ll, T* rows, T (*slots)[kSlots],
                                              double& chi, int& nrob) {
    const int meta = P.oe_meta[j];
    const int k = P.oe_edge[j];
    const int ps = P.o_src[k], pd = P.o_dst[k];
    const T xs = P.pc[4 * ps], ys = P.pc[4 * ps + 1], cs = P.pc[4 * ps + 2], ss = P.pc[4 * ps + 3];
    const T xd = P.pc[4 * pd], yd = P.pc[4 * pd + 1];
    const T tx = xd - xs, ty = yd - ys;
    const T e0 = (cs * tx + ss * ty) - P.o_z[3 * k];                                // :106, :319
    const T e1 = (-ss * tx + cs * ty) - P.o_z[3 * k + 1];
    const T e2 = bos::normalized_angle<T>(bos::normalized_angle<T>(P.pth[pd] - P.pth[ps]) - P.o_z[3 * k + 2]);
    const T t0 = -ss * xd + cs * yd, t1 = -cs * xd - ss * yd;                       // :139
    // J_s = [[-cs, -ss, t0], [ss, -cs, t1], [0, 0, -1]]
    const T* u = P.o_om + 6 * k;
    const T o00 = u[0], o01 = u[1], o02 = u[2], o11 = u[3], o12 = u[4], o22 = u[5];
    T Oe0 = o00 * e0 + o01 * e1 + o02 * e2;
    T Oe1 = o01 * e0 + o11 * e1 + o12 * e2;
    T Oe2 = o02 * e0 + o12 * e1 + o22 * e2;
    const T rho = e0 * Oe0 + e1 * Oe1 + e2 * Oe2;                                   // solver.cpp:54
    if (meta & 4) chi += (double)rho;
    if (rho > P.kt) {                                                               // :55-57
        const T sc = sqrt(P.kt / rho);
        Oe0 *= sc; Oe1 *= sc; Oe2 *= sc;
        if (meta & 4) ++nrob;
    }
    // Omega J_s, column by column
    const T a00 = -o00 * cs + o01 * ss, a01 = -o00 * ss - o01 * cs, a02 = o00 * t0 + o01 * t1 - o02;
    const T a10 = -o01 * cs + o11 * ss, a11 = -o01 * ss - o11 * cs, a12 = o01 * t0 + o11 * t1 - o12;
    const T a20 = -o02 * cs + o12 * ss, a21 = -o02 * ss - o12 * cs, a22 = o02 * t0 + o12 * t1 - o22;
    // H_ss = J_s^T (Omega J_s): J_s^T row r = column r of J_s
    const T h00 = -cs * a00 + ss * a10;
    const T h10 = -ss * a00 - cs * a10;
    const T h11 = -ss * a01 - cs * a11;
    const T h20 = t0 * a00 + t1 * a10 - a20;
    const T h21 = t0 * a01 + t1 * a11 - a21;
    const T h22 = t0 * a02 + t1 * a12 - a22;
    const T b0 = -cs * Oe0 + ss * Oe1, b1 = -ss * Oe0 - cs * Oe1, b2 = t0 * Oe0 + t1 * Oe1 - Oe2;
    if (meta & 1) {
        slots[0][2 * ll] = h00; slots[1][2 * ll] = h10; slots[2][2 * ll] = h11;
        slots[3][2 * ll] = h20; slots[4][2 * ll] = h21; slots[5][2 * ll] = h22;
        slots[6][2 * ll] = b0; slots[7][2 * ll] = b1; slots[8][2 * ll] = b2;
    }
    if (meta & 2) {
        slots[0][2 * ll + 1] = h00; slots[1][2 * ll + 1] = h10; slots[2][2 * ll + 1] = h11;
        slots[3][2 * ll + 1] = h20; slots[4][2 * ll + 1] = h21; slots[5][2 * ll + 1] = h22;
        slots[6][2 * ll + 1] = -b0; slots[7][2 * ll + 1] = -b1; slots[8][2 * ll + 1] = -b2;
    }
    if (meta & 8) {
        T g00 = h00, g10 = h10, g11 = h11, g20 = h20, g21 = h21, g22 = h22;
        if (HAS_DUPS) {   // summed information of a duplicate group
            const T* v = P.oe_omoff + 6 * j;
            const T q00 = -v[0] * cs + v[1] * ss, q01 = -v[0] * ss - v[1] * cs, q02 = v[0] * t0 + v[1] * t1 - v[2];
            const T q10 = -v[1] * cs + v[3] * ss, q11 = -v[1] * ss - v[3] * cs, q12 = v[1] * t0 + v[3] * t1 - v[4];
            const T q20 = -v[2] * cs + v[4] * ss, q21 = -v[2] * ss - v[4] * cs, q22 = v[2] * t0 + v[4] * t1 - v[5];
            g00 = -cs * q00 + ss * q10; g10 = -ss * q00 - cs * q10; g11 = -ss * q01 - cs * q11;
            g20 = t0 * q00 + t1 * q10 - q20; g21 = t0 * q01 + t1 * q11 - q21; g22 = t0 * q02 + t1 * q12 - q22;
        }
        // H_sd = -H_ss (symmetric), rows of the owner x cols of the other pose
        const int base = P.node_base[(meta & 16) ? pd : ps];
        T* blk = rows + (meta >> 8);
        blk[0] = -g00; blk[1] = -g10; blk[2] = -g20;
        blk += base + 1;
        blk[0] = -g10; blk[1] = -g11; blk[2] = -g21;
        blk += base + 2;
        blk[0] = -g20; blk[1] = -g21; blk[2] = -g22;
    }
}

// per-wave LDS tables of a task (kMaxTaskNodes nodes, <= 2 x 64 contribution slots)
struct TaskTables {
    int32_t node_base[kMaxTaskNodes];
    int16_t node_rel[kMaxTaskNodes];    // row start relative to the task's first value (< kStageCap)
    int16_t node_dof[kMaxTaskNodes];    // relative to the task's first dof
    int16_t node_cl[kMaxTaskNodes + 1]; // contribution-list range, relative to the task's first
    uint8_t node_pose[kMaxTaskNodes];
    uint8_t pair_node[9 * kMaxTaskNodes];
    uint8_t pair_val[9 * kMaxTaskNodes];
    uint16_t cl[kSlots];
};

template <typename T, bool HAS_W, bool HAS_DUPS>
__device__ __forceinline__ void range_task(const LinParams<T>& P, int t, int lane, T* rowimg, T (*slots)[kSlots],
                                           T* bimg, TaskTables& tb) {
    const int q0 = P.task_q[t], q1 = P.task_q[t + 1];
    const int flags = P.task_flags[t];
    const bool staged = flags & 1, single = flags & 2;
    const int v0 = P.pos_row0[q0], v1 = P.pos_row0[q1];
    const int d0 = P.pos_dof[q0], d1 = P.pos_dof[q1];
    T* rows = staged ? rowimg : P.val + v0;
    T* bb = staged ? bimg : P.b + d0;
    const int be0 = P.task_be[t], nb = P.task_be[t + 1] - be0;
    const int oe0 = P.task_oe[t], ne = nb + P.task_oe[t + 1] - oe0;
    const int nn = q1 - q0;
    // prologue: node table and contribution lists into LDS (independent of the entry loads)
    int npairs = 0;
    if (!single) {
        const int cl0 = P.cl_ptr[q0], ncl = P.cl_ptr[q1] - cl0;
        int nv = 0;
        if (lane < nn) {
            const int q = q0 + lane;
            const bool pose = P.pos_node[q] < P.NP;
            nv = pose ? 9 : 5;
            tb.node_rel[lane] = (int16_t)(P.pos_row0[q] - v0);
            tb.node_base[lane] = P.pos_base[q];
            tb.node_dof[lane] = (int16_t)(P.pos_dof[q] - d0);
            tb.node_cl[lane] = (int16_t)(P.cl_ptr[q] - cl0);
            tb.node_pose[lane] = pose;
        }
        if (lane == 0) tb.node_cl[nn] = (int16_t)ncl;
        for (int x = lane; x < ncl; x += 64) tb.cl[x] = P.cl[cl0 + x];
        // exclusive prefix sum of the value counts -> pair table
        int incl = nv;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        npairs = __shfl(incl, 63);
        for (int v = 0; v < nv; ++v) {
            tb.pair_node[incl - nv + v] = (uint8_t)lane;
            tb.pair_val[incl - nv + v] = (uint8_t)v;
        }
    }
    double chi = 0.0;
    int nrob = 0;
    T acc = (T)0;   // single-node tasks: lane v < size accumulates value v over all chunks
    for (int c0 = 0; c0 < ne; c0 += 64) {
        const int e = c0 + lane;
#pragma unroll
        for (int v = 0; v < 9; ++v) { slots[v][2 * lane] = (T)0; slots[v][2 * lane + 1] = (T)0; }
        if (e < nb) eval_bearing<T, HAS_W, HAS_DUPS>(P, be0 + e, lane, rows, slots, chi, nrob);
        else if (e < ne) eval_odometry<T, HAS_DUPS>(P, oe0 + (e - nb), lane, rows, slots, chi, nrob);
        wave_lds_sync();
        if (single) {
            const int cnt = min(64, ne - c0);
            if (lane < 9)
                for (int j = 0; j < cnt; ++j) acc += slots[lane][2 * j] + slots[lane][2 * j + 1];
            wave_lds_sync();
        }
    }
    // reduce per node in a fixed order and write the diagonal blocks (+ damping) and b
    if (single) {
        const bool pose = P.pos_node[q0] < P.NP;
        const int base = P.pos_base[q0];
        if (lane < (pose ? 9 : 5)) {
            const int nh = pose ? 6 : 3;
            if (lane < nh) {
                int r, c;
                tri_rc(lane, r, c);
                rows[r * base + ((r * (r + 1)) >> 1) + base + c] = acc + (r == c ? P.lambda : (T)0);
            } else {
                bb[lane - nh] = acc;
            }
        }
    } else {
        for (int pj = lane; pj < npairs; pj += 64) {
            const int j = tb.pair_node[pj], v = tb.pair_val[pj];
            T sum = (T)0;
            for (int x = tb.node_cl[j]; x < tb.node_cl[j + 1]; ++x) sum += slots[v][tb.cl[x]];
            const int base = tb.node_base[j], rel = tb.node_rel[j];
            const int nh = tb.node_pose[j] ? 6 : 3;
            if (v < nh) {
                int r, c;
                tri_rc(v, r, c);
                rows[rel + r * base + ((r * (r + 1)) >> 1) + base + c] = sum + (r == c ? P.lambda : (T)0);
            } else {
                bb[tb.node_dof[j] + v - nh] = sum;
            }
        }
    }
    wave_lds_sync();
    if (staged) {
        for (int x = lane; x < v1 - v0; x += 64) P.val[v0 + x] = rowimg[x];
        for (int x = lane; x < d1 - d0; x += 64) P.b[d0 + x] = bimg[x];
    }
    chi = wave_sum(chi);
    const int nr = (int)wave_sum((double)nrob);
    if (lane == 0) { P.chi2_part[t] = chi; P.nrob_part[t] = nr; }
}

template <typename T, bool HAS_W, bool HAS_DUPS>
__global__ __launch_bounds__(kBlock) void linearize_kernel(const LinParams<T> P) {
    __shared__ T rowimg[kWavesPerBlock][kStageCap];
    __shared__ T slots[kWavesPerBlock][9][kSlots];
    __shared__ T bimg[kWavesPerBlock][kBCap];
    __shared__ TaskTables tables[kWavesPerBlock];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = blockIdx.x * kWavesPerBlock + wave;
    if (t < P.ntask) range_task<T, HAS_W, HAS_DUPS>(P, t, lane, rowimg[wave], slots[wave], bimg[wave], tables[wave]);
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
hipError_t launch_linearize(const LinParams<T>& p, bool has_w, bool has_dups, hipStream_t s) {
    const int grid = (p.ntask + kWavesPerBlock - 1) / kWavesPerBlock;
    if (grid == 0) return hipSuccess;
    if (has_w) {
        if (has_dups) hipLaunchKernelGGL((linearize_kernel<T, true, true>), dim3(grid), dim3(kBlock), 0, s, p);
        else hipLaunchKernelGGL((linearize_kernel<T, true, false>), dim3(grid), dim3(kBlock), 0, s, p);
    } else {
        if (has_dups) hipLaunchKernelGGL((linearize_kernel<T, false, true>), dim3(grid), dim3(kBlock), 0, s, p);
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
