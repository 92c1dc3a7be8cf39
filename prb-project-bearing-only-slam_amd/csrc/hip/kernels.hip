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

#include <algorithm>
#include <cstdlib>

#include "../host/bos_math.hpp"


namespace bos {
namespace dev {

namespace {

template <typename T> struct alignas(4 * sizeof(T)) V4 { T x, y, z, w; };
template <typename T> struct alignas(2 * sizeof(T)) V2 { T x, y; };

template <typename T> __device__ __forceinline__ V4<T> load4(const T* p) { return *(const V4<T>*)p; }
template <typename T> __device__ __forceinline__ V2<T> load2(const T* p) { return *(const V2<T>*)p; }
// Six values at an even offset of the block array (8-byte aligned for fp32, 16 for fp64), stored
// non-temporal: the block array is written once per build and read by the next kernel, so it is
// streamed out instead of occupying L2 (measured: back-to-back build 15.9 -> 13.8 us fp32; the
// in-step build and the solver's reads of it unchanged).
template <typename T> __device__ __forceinline__ void store6(T* p, T a, T b, T c, T d, T e, T f) {
    typedef T v2 __attribute__((ext_vector_type(2)));
    v2* q = (v2*)p;
    __builtin_nontemporal_store(v2{a, b}, q);
    __builtin_nontemporal_store(v2{c, d}, q + 1);
    __builtin_nontemporal_store(v2{e, f}, q + 2);
}


template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Timeline diagnostics (bos_debug_linearize_timeline only; null in every product launch): per wave,
// [block, wave, kind, t_start, t_loop, t_loop_end, t_end, hw_id | xcc << 32], realtime clock (100 MHz).
__device__ __forceinline__ void stamp(const unsigned long long* base, unsigned long long* st, int k) {
    if (base) st[k] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void stamp_flush(unsigned long long* diag, const unsigned long long* st, int kind) {
    if (!diag || (threadIdx.x & 63)) return;
    unsigned long long* d = diag + 8 * ((int64_t)blockIdx.x * (kJhWg / 64) + (threadIdx.x >> 6));
    d[0] = blockIdx.x; d[1] = threadIdx.x >> 6; d[2] = kind;
    d[3] = st[0]; d[4] = st[1]; d[5] = st[2]; d[6] = __builtin_amdgcn_s_memrealtime();
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);           // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);         // HW_REG_XCC_ID
    d[7] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
}

// Odometry edge (solver_jacobians.cpp:97-168) seen from one endpoint. J_dst = -J_src exactly in
// the reference's Jacobian (:137-146: (DR' R_s)^T = -R_s^T DR', DR' antisymmetric), so
// H_ss = H_dd = J_s^T Omega J_s, H_sd = -H_ss, b_d = -b_s. Returns rho = e^T Omega e; h = H_ss
// (00, 10, 11, 20, 21, 22), g = b_s. z = measurement, u = upper triangle of Omega.
template <typename T>
__device__ __forceinline__ T odometry_hb(T kt, const T z[3], const T u[6], const V4<T>& S, T ths, const V4<T>& D,
                                         T thd, T h[6], T g[3]) {
    const T xs = S.x, ys = S.y, cs = S.z, ss = S.w, xd = D.x, yd = D.y;
    const T tx = xd - xs, ty = yd - ys;
    const T e0 = (cs * tx + ss * ty) - z[0];                                        // :106, :319
    const T e1 = (-ss * tx + cs * ty) - z[1];
    const T e2 = bos::normalized_angle<T>(bos::normalized_angle<T>(thd - ths) - z[2]);
    const T t0 = -ss * xd + cs * yd, t1 = -cs * xd - ss * yd;                       // :139
    // J_s = [[-cs, -ss, t0], [ss, -cs, t1], [0, 0, -1]]
    const T o00 = u[0], o01 = u[1], o02 = u[2], o11 = u[3], o12 = u[4], o22 = u[5];
    T Oe0 = o00 * e0 + o01 * e1 + o02 * e2;
    T Oe1 = o01 * e0 + o11 * e1 + o12 * e2;
    T Oe2 = o02 * e0 + o12 * e1 + o22 * e2;
    const T rho = e0 * Oe0 + e1 * Oe1 + e2 * Oe2;                                   // solver.cpp:54
    if (rho > kt) {                                                                 // :55-57
        const T sc = sqrt(kt / rho);
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

// Inputs of one odometry entry of a pose, gathered before any of them is used.
template <typename T> struct OdoIn {
    int ent, blk;     // edge << 1 | destination side; pose-pose block (source side)
    V4<T> Q;          // the other pose: x, y, cos, sin
    T thq;
    T z[3], u[6];
};

template <typename T> __device__ __forceinline__ void odo_fetch_ids(const LinParams<T>& P, int x, OdoIn<T>& o, int& oth) {
    o.ent = P.po_ent[x];
    o.blk = P.po_blk[x];
    oth = P.po_oth[x];
}

template <typename T> __device__ __forceinline__ void odo_fetch_data(const LinParams<T>& P, int oth, OdoIn<T>& o) {
    o.Q = load4(P.pc + 4 * oth);
    o.thq = P.pth[oth];
    const int k = o.ent >> 1;
#pragma unroll
    for (int v = 0; v < 3; ++v) o.z[v] = P.o_z[3 * k + v];
    const V2<T>* u = (const V2<T>*)(P.o_om + P.om_stride * k);
#pragma unroll
    for (int v = 0; v < 3; ++v) { const V2<T> q = u[v]; o.u[2 * v] = q.x; o.u[2 * v + 1] = q.y; }
}

// One odometry entry of pose p (pose state X, th): the entry's edge seen from p's side. Both sides
// add H_ss = H_dd to the pose's diagonal block; b gets +b_s (source) or -b_s (destination); the
// source side counts chi^2; the lower pose of the pair adds H_sd = -H_ss to the pair's block (edges
// in both directions between two poses share it). Source and destination are chosen by selects,
// so lanes on different sides of their edges run one instruction stream.
template <typename T, bool HAS_DUPS>
__device__ __forceinline__ void odometry_entry(const LinParams<T>& P, int x, int x1, const OdoIn<T>& o, const V4<T>& X,
                                               T th, T h[6], T gb[3], T acc6[6], double& chi, int& nrob) {
    const bool dst_side = o.ent & 1;
    const V4<T> S = dst_side ? o.Q : X, D = dst_side ? X : o.Q;
    const T ths = dst_side ? o.thq : th, thd = dst_side ? th : o.thq;
    T he[6], ge[3];
    const T rho = odometry_hb<T>(P.kt, o.z, o.u, S, ths, D, thd, he, ge);
#pragma unroll
    for (int v = 0; v < 6; ++v) h[v] += he[v];
#pragma unroll
    for (int v = 0; v < 3; ++v) gb[v] += dst_side ? -ge[v] : ge[v];   // a + (-b) == a - b exactly
    if (!dst_side) {
        chi += (double)rho;
        if (rho > P.kt) ++nrob;
    }
    if (o.blk < 0) return;
    T* ob = P.hval + P.off_pp + 6 * o.blk;
    if (HAS_DUPS) {
#pragma unroll
        for (int v = 0; v < 6; ++v) acc6[v] -= he[v];
        if (x + 1 == x1 || P.po_blk[x + 1] != o.blk) {
            store6(ob, acc6[0], acc6[1], acc6[2], acc6[3], acc6[4], acc6[5]);
#pragma unroll
            for (int v = 0; v < 6; ++v) acc6[v] = (T)0;
        }
    } else {
        store6(ob, -he[0], -he[1], -he[2], -he[3], -he[4], -he[5]);
    }
}

// One bearing seen from its pose (solver_jacobians.cpp:9-95, solver.cpp:37-45), in two parts: the
// evaluation (error, Jacobian, robust kernel; the pose-landmark block o = J_p^T w J_l and its factors
// jf) and the accumulation of the pose's diagonal block h, b, chi^2 and robust count from the terms
// (interleaved lane groups accumulate another lane's terms: pose_lanes).
template <typename T> struct BearingTerms {
    T j0, j1, j2, e, w, rho;   // pose Jacobian, robust-scaled error, information, e w e before scaling
    int rob;                   // the robust kernel scaled e
};

template <typename T>
__device__ __forceinline__ BearingTerms<T> pose_bearing_eval(const LinParams<T>& P, const V4<T>& X, const V2<T>& Lm,
                                                             T z, T w, T o[6], T jf[3]) {
    T J[5];
    T e = bos::bearing_error_jacobian<T>(X.x, X.y, X.z, X.w, Lm.x, Lm.y, z, J);   // :9-95
    const T rho = e * w * e;                                                       // solver.cpp:37
    int rob = 0;
    if (rho > P.kt) {                                                              // :38-40
        e *= sqrt(P.kt / rho);
        rob = 1;
    }
    const T w0 = J[0] * w, w1 = J[1] * w, w2 = J[2] * w;
    o[0] = w0 * J[3]; o[1] = w0 * J[4]; o[2] = w1 * J[3]; o[3] = w1 * J[4]; o[4] = w2 * J[3]; o[5] = w2 * J[4];
    jf[0] = J[2]; jf[1] = J[3]; jf[2] = J[4];
    return BearingTerms<T>{J[0], J[1], J[2], e, w, rho, rob};
}

// H += (J^T w) J, b += (J^T w) e (:44-45), each term one explicit fused multiply-add: the
// instruction sequence must not depend on where the terms come from (this lane's registers, with w
// a compile-time 1 when the problem has no bearing information, or another lane's shuffle), or
// the compiler's contraction and packing choices would round the two differently
template <typename T>
__device__ __forceinline__ void pose_bearing_acc(const BearingTerms<T>& b, T h[6], T gb[3], double& chi, int& nrob) {
    chi += (double)b.rho;
    nrob += b.rob;
    const T w0 = b.j0 * b.w, w1 = b.j1 * b.w, w2 = b.j2 * b.w;
    h[0] = fma(w0, b.j0, h[0]); h[1] = fma(w1, b.j0, h[1]); h[2] = fma(w1, b.j1, h[2]);
    h[3] = fma(w2, b.j0, h[3]); h[4] = fma(w2, b.j1, h[4]); h[5] = fma(w2, b.j2, h[5]);
    gb[0] = fma(w0, b.e, gb[0]); gb[1] = fma(w1, b.e, gb[1]); gb[2] = fma(w2, b.e, gb[2]);
}

// lane src's terms (a bearing of the same pose evaluated by another lane of the group)
template <typename T> __device__ __forceinline__ BearingTerms<T> shfl_terms(const BearingTerms<T>& b, int src) {
    return BearingTerms<T>{__shfl(b.j0, src), __shfl(b.j1, src), __shfl(b.j2, src), __shfl(b.e, src),
                           __shfl(b.w, src), __shfl(b.rho, src), __shfl(b.rob, src)};
}

// The pose-landmark block of a bearing: stored at its slot, or (duplicate pairs) summed over the
// run of equal landmarks and stored at the run's last slot (records of earlier slots of a run carry
// kRunCont in their index).
// Three values at slot s of a factored pose-landmark region (LinParams::pl_factored), streamed out
template <typename T> __device__ __forceinline__ void store3(T* p, T a, T b, T c) {
    __builtin_nontemporal_store(a, p);
    __builtin_nontemporal_store(b, p + 1);
    __builtin_nontemporal_store(c, p + 2);
}

template <typename T, bool HAS_DUPS>
__device__ __forceinline__ void put_pl(T* plbase, int64_t slot, const T o[6], T acc[6], bool last, bool factored,
                                       const T jf[3]) {
    if (!HAS_DUPS && factored) {   // (uniform branch: one value per launch)
        store3(plbase + 3 * slot, jf[0], jf[1], jf[2]);
        return;
    }
    if (HAS_DUPS) {
#pragma unroll
        for (int q = 0; q < 6; ++q) acc[q] += o[q];
        if (last) {
            store6(plbase + 6 * slot, acc[0], acc[1], acc[2], acc[3], acc[4], acc[5]);
#pragma unroll
            for (int q = 0; q < 6; ++q) acc[q] = (T)0;
        }
    } else {
        store6(plbase + 6 * slot, o[0], o[1], o[2], o[3], o[4], o[5]);
    }
}

// Interleaved lane groups (LPP > 1 without duplicate pairs, plan.cpp build_layout): item i of a pose
// goes to lane i % LPP of its group, and the group's first lane accumulates every item in pose order
// (its own, then each other lane's of the same round, shuffled to it) after the odometry entries —
// the operations and order of one lane per pose, so H, b and the blocks are bit-identical to LPP = 1;
// the other lanes evaluate their bearings (gathers, atan2, Jacobians) side by side and store their
// blocks. A lane's count word then holds its own count (bits 0-15) and the group's round count
// (its first lane's count, bits 16-29).
template <typename T, bool HAS_W, bool HAS_DUPS, int LPP>
__device__ __forceinline__ void pose_lanes(const LinParams<T>& P, int g, double& chi, int& nrob,
                                           unsigned long long* st) {
    constexpr bool ILV = LPP > 1 && !HAS_DUPS;
    const int grp = g / LPP, sub = g % LPP, t = g & 63;
    // group i runs pose i unless a table says otherwise (sharded ranks): one dependent load fewer
    // at the head of both of the lane's load chains
    const int p = grp < P.n_groups ? (P.lane_pose ? P.lane_pose[grp] : grp) : -1;
    const bool active = p >= 0;
    T h[6] = {0, 0, 0, 0, 0, 0}, gb[3] = {0, 0, 0};
    if (active) {
        // Dependent load stages, the bearing chain (count/base -> records -> landmarks) and the
        // odometry chain (entry range -> entry ids -> other pose + edge data) issued side by side.
        const V4<T> X = load4(P.pc + 4 * p);
        const int cnt = P.pl_cnt[g];
        const int n = ILV ? cnt & 0xffff : cnt & ~kOdoChain;
        const int nloop = ILV ? (cnt >> 16) & 0x3fff : n;   // the group's rounds (interleaved) or own items
        const bool chain = cnt & kOdoChain;   // (first lane of the group only)
        const int sl = P.pw_base[g >> 6] + t;   // slot of item j: sl + S j
        const int S = P.pw_stride[g >> 6];
        const int jl = n > 0 ? n - 1 : 0;       // record reads past the lane's last item: clamped to it
        auto at = [&](int j) { return sl + S * min(j, jl); };
        const bool odo = sub == 0;
        int x0 = 0, x1 = 0;
        T th = (T)0;
        if (odo) { x0 = P.po_ptr[p]; x1 = P.po_ptr[p + 1]; th = P.pth[p]; }
        // a chain pose's two entries follow from p (edge p - 1 from its destination side, edge p from
        // its source side): its edge and other-pose loads wait for no index load; only the pair
        // block's index (a store address) is loaded
        auto ids = [&](int i, OdoIn<T>& o, int& oth) {
            if (chain) {
                o.ent = i == 0 ? ((p - 1) << 1) | 1 : p << 1;
                oth = i == 0 ? p - 1 : p + 1;
                o.blk = i == 0 ? -1 : P.po_blk[x0 + 1];
            } else {
                odo_fetch_ids(P, x0 + i, o, oth);
            }
        };
        // Bearing items run in pairs with two register sets (A: even items, B: odd items). Per set,
        // the record index is loaded two pairs ahead, the full record and the landmark gather one
        // pair ahead; every register is refilled by a load right after its last use, so no loaded
        // value is ever copied (a copy waits for its load) and each gather has a whole pair of items
        // to land. Reads past the lane's last item are clamped to it (cache hits; never evaluated).
        const int32_t* ip = P.pb_idx;
        const T* zp = P.pb_z;
        int iA = ip[at(0)], iB = ip[at(1)];
        OdoIn<T> oa, ob;
        int otha = 0, othb = 0;
        if (chain || x0 < x1) ids(0, oa, otha);
        if (chain || x0 + 1 < x1) ids(1, ob, othb);
        V2<T> LA = load2(P.lc + 2 * (iA & kIdxMask)), LB = load2(P.lc + 2 * (iB & kIdxMask));
        T zA = zp[at(0)], zB = zp[at(1)];
        bool lastA = !(iA & kRunCont), lastB = !(iB & kRunCont);
        T wA = HAS_W ? P.pb_w[at(0)] : (T)1, wB = HAS_W ? P.pb_w[at(1)] : (T)1;
        iA = ip[at(2)];
        iB = ip[at(3)];
        // odometry first: its arithmetic covers the landmark gathers of items 0 and 1
        T acc6[6] = {0, 0, 0, 0, 0, 0};
        auto odometry = [&]() {
            if (x0 < x1) odo_fetch_data(P, otha, oa);
            if (x0 + 1 < x1) odo_fetch_data(P, othb, ob);
            if (x0 < x1) odometry_entry<T, HAS_DUPS>(P, x0, x1, oa, X, th, h, gb, acc6, chi, nrob);
            if (x0 + 1 < x1) odometry_entry<T, HAS_DUPS>(P, x0 + 1, x1, ob, X, th, h, gb, acc6, chi, nrob);
            for (int x = x0 + 2; x < x1; ++x) {
                OdoIn<T> oc;
                int othc;
                odo_fetch_ids(P, x, oc, othc);
                odo_fetch_data(P, othc, oc);
                odometry_entry<T, HAS_DUPS>(P, x, x1, oc, X, th, h, gb, acc6, chi, nrob);
            }
        };
        odometry();
        T acc[6] = {0, 0, 0, 0, 0, 0}, o[6], jf[3];
        const bool factored = P.pl_factored != 0;
        T* const plbase = P.hval + P.off_pl;
        stamp(P.diag_stamps, st, 1);
        const int src0 = (threadIdx.x & 63 & ~(LPP - 1));   // the group's first lane in the wave
        // (interleaved) the other lanes' terms of this round, after this lane's own, in lane order
        auto peers = [&](const BearingTerms<T>& mine, bool valid) {
#pragma unroll
            for (int k = 1; k < LPP; ++k) {
                const BearingTerms<T> q = shfl_terms(mine, src0 + k);
                if (__shfl((int)valid, src0 + k)) pose_bearing_acc<T>(q, h, gb, chi, nrob);
            }
        };
        for (int j = 0; j < nloop; j += 2) {
            // item j (set A), then refill A: item j + 2's gather and z, item j + 4's index
            {
                // (interleaved: every lane of the group evaluates, valid or not — a round past a
                // lane's last item reads clamped records and stores zeros to a padding slot of its
                // wave — so the shuffles run with the whole group active)
                const bool vA = !ILV || j < n;
                const BearingTerms<T> bA = pose_bearing_eval<T>(P, X, LA, zA, wA, o, jf);
                if (vA) pose_bearing_acc<T>(bA, h, gb, chi, nrob);
                if constexpr (ILV) {
                    peers(bA, vA);
                    if (!vA) {
#pragma unroll
                        for (int q = 0; q < 6; ++q) o[q] = (T)0;
                        jf[0] = jf[1] = jf[2] = (T)0;
                    }
                }
            }
            put_pl<T, HAS_DUPS>(plbase, sl + (int64_t)S * j, o, acc, lastA, factored, jf);
            lastA = !(iA & kRunCont);
            LA = load2(P.lc + 2 * (iA & kIdxMask));
            zA = zp[at(j + 2)];
            if (HAS_W) wA = P.pb_w[at(j + 2)];
            iA = ip[at(j + 4)];
            // item j + 1 (set B). Its block is stored even past the lane's last item (a padding slot
            // of the lane's wave: pose-lane waves have an even number of slots per lane), so both
            // paths issue the same memory operations and the loop's waits stay exact.
            if constexpr (ILV) {
                const bool vB = j + 1 < n;
                const BearingTerms<T> bB = pose_bearing_eval<T>(P, X, LB, zB, wB, o, jf);
                if (vB) pose_bearing_acc<T>(bB, h, gb, chi, nrob);
                peers(bB, vB);
                if (!vB) {
#pragma unroll
                    for (int q = 0; q < 6; ++q) o[q] = (T)0;
                    jf[0] = jf[1] = jf[2] = (T)0;
                }
            } else if (j + 1 < n) {
                pose_bearing_acc<T>(pose_bearing_eval<T>(P, X, LB, zB, wB, o, jf), h, gb, chi, nrob);
            } else {
#pragma unroll
                for (int q = 0; q < 6; ++q) o[q] = (T)0;
                jf[0] = jf[1] = jf[2] = (T)0;
            }
            put_pl<T, HAS_DUPS>(plbase, sl + (int64_t)S * (j + 1), o, acc, lastB, factored, jf);
            lastB = !(iB & kRunCont);
            LB = load2(P.lc + 2 * (iB & kIdxMask));
            zB = zp[at(j + 3)];
            if (HAS_W) wB = P.pb_w[at(j + 3)];
            iB = ip[at(j + 5)];
        }
        stamp(P.diag_stamps, st, 2);
    }
    if constexpr (ILV) {   // the first lane holds the pose's sums; the others' chi^2 / counts are not theirs
        if (sub != 0) { chi = 0.0; nrob = 0; }
    } else {
        // combine the lane group's partial sums (fixed butterfly: deterministic)
#pragma unroll
        for (int o = 1; o < LPP; o <<= 1) {
#pragma unroll
            for (int v = 0; v < 6; ++v) h[v] += __shfl_xor(h[v], o);
#pragma unroll
            for (int v = 0; v < 3; ++v) gb[v] += __shfl_xor(gb[v], o);
        }
    }
    if (active && sub == 0) {
        const T lam = P.lambda;
        store6(P.hval + 6 * p, h[0] + lam, h[1], h[2] + lam, h[3], h[4], h[5] + lam);
        T* bp = P.b + 3 * p;
        bp[0] = gb[0]; bp[1] = gb[1]; bp[2] = gb[2];
    }
}

// One bearing seen from its landmark: the landmark's diagonal block and b.
template <typename T>
__device__ __forceinline__ void landmark_bearing(const LinParams<T>& P, const V4<T>& X, const V2<T>& Lm, T z, T w,
                                                 T hl[3], T gl[2]) {
    T J[5];
    T e = bos::bearing_error_jacobian<T>(X.x, X.y, X.z, X.w, Lm.x, Lm.y, z, J);
    const T rho = e * w * e;
    if (rho > P.kt) e *= sqrt(P.kt / rho);
    const T w3 = J[3] * w, w4 = J[4] * w;
    hl[0] += w3 * J[3]; hl[1] += w4 * J[3]; hl[2] += w4 * J[4];
    gl[0] += w3 * e; gl[1] += w4 * e;
}

template <typename T, bool HAS_W>
__device__ __forceinline__ void landmark_lane(const LinParams<T>& P, int g, unsigned long long* st) {
    if (g >= P.n_lm_lanes) return;
    int l, n, p0;
    if (P.ll_hdr) {   // (uniform: one value per launch)
        const int2 h = P.ll_hdr[g];
        l = h.x & 0xfffff;
        n = (int)((uint32_t)h.x >> 20);
        p0 = h.y;
    } else {
        l = P.ll_lm[g];
        n = P.ll_cnt[g];
        p0 = P.ll_run ? P.ll_run[g] : -1;
    }
    const int sl = P.lw_base[g >> 6] + (g & 63);
    const int S = P.lw_stride[g >> 6];
    const int jl = n > 0 ? n - 1 : 0;
    auto at = [&](int j) { return sl + S * min(j, jl); };
    const V2<T> Lm = load2(P.lc + 2 * l);
    T hl[3] = {0, 0, 0}, gl[2] = {0, 0};
    const T* zp = P.lb_z;
    if (p0 >= 0) {
        // consecutive poses p0 + j: every load of the lane is independent of the others (one latency
        // per pair instead of the index -> pose chain). Paired registers, one pair ahead.
        const T* xp = P.pc + 4 * (int64_t)p0;
        auto xat = [&](int j) { return xp + 4 * min(j, jl); };
        V4<T> XA = load4(xat(0)), XB = load4(xat(1));
        T zA = zp[at(0)], zB = zp[at(1)];
        T wA = HAS_W ? P.lb_w[at(0)] : (T)1, wB = HAS_W ? P.lb_w[at(1)] : (T)1;
        stamp(P.diag_stamps, st, 1);
        for (int j = 0; j < n; j += 2) {
            landmark_bearing<T>(P, XA, Lm, zA, wA, hl, gl);
            XA = load4(xat(j + 2));
            zA = zp[at(j + 2)];
            if (HAS_W) wA = P.lb_w[at(j + 2)];
            if (j + 1 < n) landmark_bearing<T>(P, XB, Lm, zB, wB, hl, gl);
            XB = load4(xat(j + 3));
            zB = zp[at(j + 3)];
            if (HAS_W) wB = P.lb_w[at(j + 3)];
        }
        stamp(P.diag_stamps, st, 2);
        T* hp = P.hval + P.off_ldiag + 3 * l;
        hp[0] = hl[0] + P.lambda; hp[1] = hl[1]; hp[2] = hl[2] + P.lambda;
        T* bl = P.b + 3 * P.NP + 2 * l;
        bl[0] = gl[0]; bl[1] = gl[1];
        return;
    }
    // paired register sets as in pose_lanes (reads past the last item clamped to it)
    const int32_t* ip = P.lb_idx;
    int iA = ip[at(0)], iB = ip[at(1)];
    V4<T> XA = load4(P.pc + 4 * iA), XB = load4(P.pc + 4 * iB);
    T zA = zp[at(0)], zB = zp[at(1)];
    T wA = HAS_W ? P.lb_w[at(0)] : (T)1, wB = HAS_W ? P.lb_w[at(1)] : (T)1;
    iA = ip[at(2)];
    iB = ip[at(3)];
    stamp(P.diag_stamps, st, 1);
    for (int j = 0; j < n; j += 2) {
        landmark_bearing<T>(P, XA, Lm, zA, wA, hl, gl);
        XA = load4(P.pc + 4 * iA);
        zA = zp[at(j + 2)];
        if (HAS_W) wA = P.lb_w[at(j + 2)];
        iA = ip[at(j + 4)];
        if (j + 1 < n) landmark_bearing<T>(P, XB, Lm, zB, wB, hl, gl);
        XB = load4(P.pc + 4 * iB);
        zB = zp[at(j + 3)];
        if (HAS_W) wB = P.lb_w[at(j + 3)];
        iB = ip[at(j + 5)];
    }
    stamp(P.diag_stamps, st, 2);
    T* hp = P.hval + P.off_ldiag + 3 * l;
    hp[0] = hl[0] + P.lambda; hp[1] = hl[1]; hp[2] = hl[2] + P.lambda;
    T* bl = P.b + 3 * P.NP + 2 * l;
    bl[0] = gl[0]; bl[1] = gl[1];
}

// XCD-aware block order: blocks b and b + 8 share an XCD (and its L2), so a segment [s0, s1) of
// the grid is renumbered to give each XCD a contiguous run of it; the pose (landmark) blocks an
// XCD runs then cover a stretch of the trajectory, and the landmark (pose) cache lines their
// gathers fetch come from that stretch only, instead of every XCD's L2 fetching all of them.
__device__ __forceinline__ int64_t xcd_contiguous(int64_t b, int64_t s0, int64_t s1) {
    const int64_t n = s1 - s0, i = b - s0, g = i & 7, q = n >> 3, rmd = n & 7;
    return s0 + g * q + (g < rmd ? g : rmd) + (i >> 3);
}

// Launch order of the J+H units (kJhWg lanes each; kJhSub per block of lanes): pose units first,
// then landmark units, each range XCD-contiguous (above). Pose waves are the longer chains (~12.7 us
// against ~8.5 us per wave cold at config 3), so they get the head start (measured: interleaving
// the two kinds in proportion, or one-wave units spreading the pose waves over every CU, is no
// faster). Returns true for a pose unit; u = the unit's index in its range.
__device__ __forceinline__ bool jh_unit(int64_t i, int64_t n_units, int64_t n_pose_units, int64_t& u) {
    if (i < n_pose_units) {
        u = xcd_contiguous(i, 0, n_pose_units);
        return true;
    }
    u = xcd_contiguous(i, n_pose_units, n_units) - n_pose_units;
    return false;
}

// chi^2 / robust count of a pose workgroup, its waves summed in order (deterministic), one partial
// per workgroup (the stats kernel sums them in a fixed order)
__device__ __forceinline__ void pose_wg_partials(double* chi2_part, int32_t* nrob_part, int g, double chi, int nrob) {
    __shared__ double sc[kJhWg / 64];
    __shared__ int sr[kJhWg / 64];
    chi = wave_sum(chi);
    nrob = (int)wave_sum((double)nrob);
    if ((threadIdx.x & 63) == 0) { sc[threadIdx.x >> 6] = chi; sr[threadIdx.x >> 6] = nrob; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double c = 0.0;
        int r = 0;
        for (int w = 0; w < kJhWg / 64; ++w) { c += sc[w]; r += sr[w]; }
        chi2_part[g / kJhWg] = c;
        nrob_part[g / kJhWg] = r;
    }
}

template <typename T, bool HAS_W, bool HAS_DUPS, int LPP, int MINW>
__global__ __launch_bounds__(kJhWg, MINW) void linearize_kernel(const LinParams<T> P) {
    int64_t u;
    const bool pose = jh_unit(blockIdx.x, gridDim.x, (int64_t)P.n_pose_run * kJhSub, u);
    unsigned long long st[3] = {0, 0, 0};
    if (P.t_start && blockIdx.x == 0 && threadIdx.x == 0) *P.t_start = __builtin_amdgcn_s_memrealtime();
    stamp(P.diag_stamps, st, 0);
    if (!pose) {   // workgroup-uniform branch
        landmark_lane<T, HAS_W>(P, (int)(((int64_t)P.lm_b0 * kJhSub + u) * kJhWg + threadIdx.x), st);
        stamp_flush(P.diag_stamps, st, 1);
        return;
    }
    const int g = (int)(((int64_t)P.pose_b0 * kJhSub + u) * kJhWg + threadIdx.x);
    double chi = 0.0;
    int nrob = 0;
    pose_lanes<T, HAS_W, HAS_DUPS, LPP>(P, g, chi, nrob, st);
    stamp_flush(P.diag_stamps, st, 0);
    pose_wg_partials(P.chi2_part, P.nrob_part, g, chi, nrob);
}

// max that propagates NaN (fmax returns the non-NaN operand): a non-finite update must not read
// as convergence
__device__ __forceinline__ double nan_max(double a, double b) { return (a != a || b != b) ? a + b : fmax(a, b); }

// State::apply_boxplus (framework/state.cpp:69-80): dx = -x (the solve ran on +b). Skipped (state
// untouched) when the solver reports an aborted factorization.
template <typename T> __global__ __launch_bounds__(kUpdateBlock) void boxplus_kernel(const UpdateParams<T> U) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = U.nodes ? (t < U.n_nodes ? U.nodes[t] : -1) : t;
    double m = 0.0;
    if (U.t_start && blockIdx.x == 0 && threadIdx.x == 0) *U.t_start = __builtin_amdgcn_s_memrealtime();
    // the node's dof, its state and the abort word are loaded together (one dependent hop, to the
    // solution, follows); nothing is written when the solver aborted
    const bool is_pose = i >= 0 && i < U.NP && i != U.fixed, is_lm = i >= U.NP && i < U.NP + U.NL;
    const int d = is_pose || is_lm ? U.node_dof[i] : 0;
    int32_t inf = U.info ? *U.info : 0;
    if (U.ex_hdr)
        for (int q = 0; q < U.ex_world; ++q) inf |= (int32_t)U.ex_hdr[q * U.ex_stride] & kStepAbort;
    if (is_pose) {
        double x = U.pose[3 * i], y = U.pose[3 * i + 1], th = U.pose[3 * i + 2];
        const double dx = -U.x[d], dy = -U.x[d + 1], dth = -U.x[d + 2];
        if (!(inf & kStepAbort)) {
            bos::boxplus_pose<double>(x, y, th, dx, dy, dth);
            U.pose[3 * i] = x;
            U.pose[3 * i + 1] = y;
            U.pose[3 * i + 2] = th;
            U.pc[4 * i] = (T)x;
            U.pc[4 * i + 1] = (T)y;
            U.pc[4 * i + 2] = cos((T)th);
            U.pc[4 * i + 3] = sin((T)th);
            U.pth[i] = (T)th;
            m = nan_max(fabs(dx), nan_max(fabs(dy), fabs(dth)));
        }
    } else if (is_lm) {
        const int j = i - U.NP;
        const double lx = U.lm[2 * j], ly = U.lm[2 * j + 1];
        const double dx = -U.x[d], dy = -U.x[d + 1];
        if (!(inf & kStepAbort)) {
            const double x = lx + dx, y = ly + dy;
            U.lm[2 * j] = x;
            U.lm[2 * j + 1] = y;
            U.lc[2 * j] = (T)x;
            U.lc[2 * j + 1] = (T)y;
            m = nan_max(fabs(dx), fabs(dy));
        }
    }
    // block max into its partial slot (max is order independent: deterministic; no atomics, which
    // would serialize on one address)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = nan_max(m, __shfl_xor(m, o));
    __shared__ double sm[kUpdateBlock / 64];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = sm[0];
        for (int w = 1; w < kUpdateBlock / 64; ++w) b = nan_max(b, sm[w]);
        U.max_part[blockIdx.x] = b;
    }
}

// This thread's share of the J+H chi^2 / robust-count partials (one per pose workgroup), in a
// fixed order: four loads in flight per thread and step
template <typename R>
__device__ __forceinline__ void sum_partials(const double* chi_part, const int32_t* nrob_part, int n, double& c, R& r) {
    for (int i0 = threadIdx.x; i0 < n; i0 += 4 * blockDim.x) {
        double v[4];
        int w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = min(i0 + k * (int)blockDim.x, n - 1);
            v[k] = chi_part[i];
            w[k] = nrob_part[i];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool in = i0 + k * (int)blockDim.x < n;
            c += in ? v[k] : 0.0;
            r += in ? w[k] : 0;
        }
    }
}

__global__ void reduce_stats_kernel(const double* chi_part, const int32_t* nrob_part, int n, double chi_const,
                                    int32_t nrob_const, const double* max_part, int n_max, int32_t* info,
                                    StepStatus* out, StepStatus* mirror) {
    __shared__ double sc[256];
    __shared__ double sm[256];
    __shared__ long long sr[256];
    double c = 0.0, m = 0.0;
    long long r = 0;
    const int32_t inf = info && threadIdx.x == 0 ? *info : 0;   // loaded with the partials
    if (nrob_part) {
        sum_partials(chi_part, nrob_part, n, c, r);
    } else if (threadIdx.x == 0) {   // an all-reduced header
        c = chi_part[0];
        r = (long long)chi_part[1];
    }
    if (max_part)
        for (int i = threadIdx.x; i < n_max; i += blockDim.x) m = nan_max(m, max_part[i]);
    sc[threadIdx.x] = c;
    sm[threadIdx.x] = m;
    sr[threadIdx.x] = r;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            sc[threadIdx.x] += sc[threadIdx.x + o];
            sr[threadIdx.x] += sr[threadIdx.x + o];
            sm[threadIdx.x] = nan_max(sm[threadIdx.x], sm[threadIdx.x + o]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out->chi2 = sc[0] + chi_const;
        out->n_robust = (int32_t)sr[0] + nrob_const;
        out->max_dx = sm[0];
        out->info = inf;
        out->aborted |= inf & kStepAbort;
        if (info) *info = 0;
        out->stamp[3] = __builtin_amdgcn_s_memrealtime();
        out->seq += 1;
        if (mirror) {   // the summary, then (after a system-scope release) its sequence number: a host
                        // that sees the new seq sees the whole summary (read_stats polls it)
            const StepStatus v = *out;
            mirror->chi2 = v.chi2;
            mirror->max_dx = v.max_dx;
            mirror->n_robust = v.n_robust;
            mirror->info = v.info;
            mirror->aborted = v.aborted;
            for (int k = 0; k < 8; ++k) mirror->stamp[k] = v.stamp[k];
            __threadfence_system();
            __hip_atomic_store(&mirror->seq, v.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// triangulate_one_landmark (slam/triangulation.cpp:21-62): the rows [sin(th + z), -cos(th + z)],
// rhs sin(th + z) px - cos(th + z) py, solved by the reference with Eigen's column-pivoted
// Householder QR; here (as in the host build, host/triangulation.cpp) by column-pivoted modified
// Gram-Schmidt with one re-orthogonalisation and Eigen's nonzeroPivots() rank rule, so a rank-1
// system (one observation) gets the basic solution. The same operation sequence as the host code,
// without FP contraction; the rows are computed once and kept in scratch for the later passes.
template <typename T> __global__ __launch_bounds__(256) void triangulate_kernel(const TriParams<T> P) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= P.NL) return;
    const int x0 = P.lm_ptr[l], x1 = P.lm_ptr[l + 1], M = x1 - x0;
    double n0 = 0.0, n1 = 0.0;
    for (int x = x0; x < x1; ++x) {
        const int k = P.lm_obs[x];
        const double* p = P.pose + 3 * (int64_t)P.b_pose[k];
        const double ang = p[2] + P.b_z[k];
        const double sn = sin(ang), cs = cos(ang);
        const double a0 = sn, a1 = -cs, r = sn * p[0] - cs * p[1];
        double* w = P.scratch + 3 * (int64_t)x;
        w[0] = a0; w[1] = a1; w[2] = r;
        n0 += a0 * a0;
        n1 += a1 * a1;
    }
    double ox = 0.0, oy = 0.0;
    const bool swap = n1 > n0;                     // pivot: the first column of maximal norm
    const double r00 = sqrt(fmax(n0, n1));
    if (M > 0 && r00 != 0.0) {
        auto c0 = [&](const double* w) { return swap ? w[1] : w[0]; };
        auto c1 = [&](const double* w) { return swap ? w[0] : w[1]; };
        double qb0 = 0.0;
        for (int x = x0; x < x1; ++x) { const double* w = P.scratch + 3 * (int64_t)x; qb0 += (c0(w) / r00) * w[2]; }
        double x_piv, x_oth = 0.0;
        bool rank2 = false;
        double r01 = 0.0, r11 = 0.0, qb1 = 0.0;
        if (M >= 2) {
            // two MGS passes: d1 = q0 . c1, c1' = c1 - d1 q0; d2 = q0 . c1', c1'' = c1' - d2 q0
            double d1 = 0.0, d2 = 0.0;
            for (int x = x0; x < x1; ++x) { const double* w = P.scratch + 3 * (int64_t)x; d1 += (c0(w) / r00) * c1(w); }
            for (int x = x0; x < x1; ++x) {
                const double* w = P.scratch + 3 * (int64_t)x;
                const double q = c0(w) / r00;
                d2 += q * (c1(w) - d1 * q);
            }
            r01 = d1 + d2;
            double rem = 0.0;
            for (int x = x0; x < x1; ++x) {
                const double* w = P.scratch + 3 * (int64_t)x;
                const double q = c0(w) / r00;
                const double v = (c1(w) - d1 * q) - d2 * q;
                rem += v * v;
            }
            const double eps = 2.220446049250313e-16;
            const double thr = (r00 * eps) * (r00 * eps) / (double)M * (double)(M - 1);
            if (!(rem < thr)) {
                rank2 = true;
                r11 = sqrt(rem);
                for (int x = x0; x < x1; ++x) {
                    const double* w = P.scratch + 3 * (int64_t)x;
                    const double q = c0(w) / r00;
                    qb1 += (((c1(w) - d1 * q) - d2 * q) / r11) * w[2];
                }
            }
        }
        if (rank2) {
            x_oth = qb1 / r11;
            x_piv = (qb0 - r01 * x_oth) / r00;
        } else {
            x_piv = qb0 / r00;
        }
        ox = swap ? x_oth : x_piv;
        oy = swap ? x_piv : x_oth;
    }
    P.lm[2 * (int64_t)l] = ox;
    P.lm[2 * (int64_t)l + 1] = oy;
    P.lc[2 * (int64_t)l] = (T)ox;
    P.lc[2 * (int64_t)l + 1] = (T)oy;
}

// lanes q < world of the block poll sender q's flag in this rank's mailbox until it equals the
// iteration's epoch (or mark the step aborted, kStepAbort | kExTimeout, after w.timeout_ticks, or give
// up at once when an exchange wait of this step already timed out: a launch's blocks, and the step's
// later waits, then drain in one timeout; a local solver stall alone does not end the wait, so the
// rank still receives its peers' current headers); then the whole block acquires
__device__ __forceinline__ void p2p_wait_block(const P2PWait& w) {
    const int q = threadIdx.x;
    if (q < w.world) {
        const uint32_t e = *w.epoch;
        const uint32_t* f = reinterpret_cast<const uint32_t*>(w.mailbox + w.flag_off + 64 * (int64_t)q);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t it = 0; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != e; ++it) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > w.timeout_ticks) {
                atomicOr(w.info, kStepAbort | kExTimeout);
                break;
            }
            if ((it & 63) == 63 &&
                (__hip_atomic_load(w.info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kExTimeout))
                break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    __threadfence_system();
}

// one segment per blockIdx.y, its elements grid-strided over blockIdx.x
// (w.mailbox set: every block first waits for the direct exchange's flags, and the stamp marks the
// end of that wait)
template <typename T>
__global__ void seg_copy_kernel(T* val, T* b, T* send, T* recv, T* aux, const ExSeg* segs, unsigned long long* stamp,
                                const P2PWait w) {
    if (w.mailbox) p2p_wait_block(w);
    if (stamp && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();
    const ExSeg g = segs[blockIdx.y];
    T* const base[5] = {val, b, send, recv, aux};
    const T* src = base[g.src_kind] + g.src;
    T* dst = base[g.dst_kind] + g.dst;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g.len; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// the exchange-1 header of a 256-thread block: this rank's chi^2 and robust count, summed in a fixed
// order (valid in thread 0)
__device__ __forceinline__ void header1_block(const double* chi_part, const int32_t* nrob_part, int n, double& chi,
                                              long long& nrob) {
    __shared__ double sc[256];
    __shared__ long long sr[256];
    double c = 0.0;
    long long r = 0;
    sum_partials(chi_part, nrob_part, n, c, r);
    sc[threadIdx.x] = c;
    sr[threadIdx.x] = r;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) { sc[threadIdx.x] += sc[threadIdx.x + o]; sr[threadIdx.x] += sr[threadIdx.x + o]; }
        __syncthreads();
    }
    chi = sc[0];
    nrob = sr[0];
}

__global__ __launch_bounds__(256) void shard_header1_kernel(const double* chi_part, const int32_t* nrob_part, int n,
                                                           double* send1, unsigned long long* stamp) {
    double c;
    long long r;
    header1_block(chi_part, nrob_part, n, c, r);
    if (threadIdx.x == 0) {
        send1[0] = c;
        send1[1] = (double)r;
        if (stamp) *stamp = __builtin_amdgcn_s_memrealtime();
    }
}

// per-block max |x| over the dofs of a node list (poses 3 dofs, landmarks 2)
__global__ __launch_bounds__(256) void node_absmax_kernel(const double* x, const int32_t* nodes, int n,
                                                          const int32_t* node_dof, int NP, double* part) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    double m = 0.0;
    if (t < n) {
        const int u = nodes[t], d = node_dof[u];
        m = nan_max(fabs(x[d]), fabs(x[d + 1]));
        if (u < NP) m = nan_max(m, fabs(x[d + 2]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = nan_max(m, __shfl_xor(m, o));
    __shared__ double sm[4];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = nan_max(nan_max(sm[0], sm[1]), nan_max(sm[2], sm[3]));
}

// block 0: header (max of the partials, reduced by the whole block — one thread walking ~1 200
// partials serially took 109 us at config 3 — and the solver word, which is then zeroed); every
// thread: the boundary payload
__global__ __launch_bounds__(256) void shard_pack2_kernel(const double* x, const double* part, int n_part, int32_t* info,
                                                          const int32_t* bnd, int n_bnd, double* send2,
                                                          unsigned long long* stamp) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0) {   // block-uniform branch
        if (stamp && t == 0) *stamp = __builtin_amdgcn_s_memrealtime();
        double m = 0.0;
        for (int i = threadIdx.x; i < n_part; i += 256) m = nan_max(m, part[i]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = nan_max(m, __shfl_xor(m, o));
        __shared__ double sm[4];
        if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
        __syncthreads();
        if (t == 0) {
            send2[0] = nan_max(nan_max(sm[0], sm[1]), nan_max(sm[2], sm[3]));
            send2[1] = (double)*info;
            *info = 0;
        }
    }
    for (int i = t; i < n_bnd; i += gridDim.x * blockDim.x) send2[2 + i] = x[bnd[i]];
}

__global__ void index_copy_kernel(const double* src, const int32_t* si, double* dst, const int32_t* di, int64_t n,
                                  unsigned long long* stamp, const P2PWait w) {
    if (w.mailbox) p2p_wait_block(w);
    if (stamp && blockIdx.x == 0 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[di ? di[i] : i] = src[si ? si[i] : i];
}

__global__ void shard_combine_kernel(const double* recv1, int64_t c1, const double* recv2, int64_t c2, int world,
                                     double chi_const, int32_t nrob_const, int32_t* local_info, StepStatus* out,
                                     StepStatus* mirror, bool zero_info) {
    if (threadIdx.x != 0) return;
    double chi = 0.0, m = 0.0;
    long long nr = 0, piv = 0;
    int32_t abort_bits = 0;
    if (local_info) {   // an exchange-2 wait that timed out (its abort bit arrived after exchange 2's packing)
        abort_bits |= *local_info & kStepAbort;
        // zero_info: the gathering exchange-2 push sent the whole word without zeroing it (its blocks
        // read it concurrently), so it is zeroed here, after every block has read it
        *local_info = zero_info ? 0 : (*local_info & ~(kStepAbort | kExTimeout));
    }
    for (int q = 0; q < world; ++q) {
        chi += recv1[q * c1];
        nr += (long long)recv1[q * c1 + 1];
        m = nan_max(m, recv2[q * c2]);
        const int32_t inf = (int32_t)recv2[q * c2 + 1];
        piv += inf & ~(kStepAbort | kExTimeout);
        abort_bits |= inf & kStepAbort;
    }
    out->chi2 = chi + chi_const;
    out->n_robust = (int32_t)nr + nrob_const;
    out->max_dx = m;
    out->info = (int32_t)min(piv, (long long)(kExTimeout - 1)) | abort_bits;
    out->aborted |= abort_bits;
    out->stamp[3] = __builtin_amdgcn_s_memrealtime();
    out->seq += 1;
    if (mirror) {   // the summary, then (after a system-scope release) its sequence number (read_stats)
        const StepStatus v = *out;
        mirror->chi2 = v.chi2;
        mirror->max_dx = v.max_dx;
        mirror->n_robust = v.n_robust;
        mirror->info = v.info;
        mirror->aborted = v.aborted;
        for (int k = 0; k < 8; ++k) mirror->stamp[k] = v.stamp[k];
        __threadfence_system();
        __hip_atomic_store(&mirror->seq, v.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// a J+H launch with no blocks (a rank with an empty share of the observations partition) still
// stamps its start, so the phase times of that rank read 0 rather than a stale stamp
__global__ void stamp_kernel(unsigned long long* t) { *t = __builtin_amdgcn_s_memrealtime(); }

// Direct peer exchange (launch_p2p_push, P2PWait). The mailboxes are uncached device memory, so
// remote stores land in the receiver's HBM and its reads never see a stale cached line; the pushing
// block drains its payload stores (vmcnt) and releases at system scope before its flag.
__global__ __launch_bounds__(256) void p2p_push_kernel(const double* send, int64_t count, double* const* peers,
                                                       int64_t data_off, int64_t flag_off, int rank,
                                                       const uint32_t* epoch, const double* chi_part,
                                                       const int32_t* nrob_part, int n_parts,
                                                       unsigned long long* stamp) {
    if (stamp && blockIdx.x == 0 && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();
    char* base = reinterpret_cast<char*>(peers[blockIdx.x]);
    double* dst = reinterpret_cast<double*>(base + data_off) + (int64_t)rank * count;
    int64_t i0 = 0;
    if (chi_part) {   // exchange 1: the header computed here (every block the same sums), then the payload
        double c;
        long long r;
        header1_block(chi_part, nrob_part, n_parts, c, r);
        if (threadIdx.x == 0) { dst[0] = c; dst[1] = (double)r; }
        i0 = kExHeader;
    }
    for (int64_t i = i0 + threadIdx.x; i < count; i += 256) dst[i] = send[i];
    const uint32_t e = *epoch;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<uint32_t*>(base + flag_off + 64 * (int64_t)rank), e, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// launch_p2p_push_gather: one block per receiving rank, the payload read from its sources
__global__ __launch_bounds__(256) void p2p_push_gather_kernel(const P2PPush p) {
    if (p.stamp && blockIdx.x == 0 && threadIdx.x == 0) *p.stamp = __builtin_amdgcn_s_memrealtime();
    char* base = reinterpret_cast<char*>(p.peers[blockIdx.x]);
    double* dst = reinterpret_cast<double*>(base + p.data_off) + (int64_t)p.rank * p.count;
    if (p.which == 1) {   // exchange 1: header, then the pack segments
        double c;
        long long r;
        header1_block(p.chi_part, p.nrob_part, p.n_parts, c, r);
        if (threadIdx.x == 0) { dst[0] = c; dst[1] = (double)r; }
        for (int g = 0; g < p.nseg; ++g) {
            const ExSeg e = p.segs[g];
            const double* src = (e.src_kind == 0 ? p.U : p.u) + e.src;
            for (int64_t i = threadIdx.x; i < e.len; i += 256) dst[e.dst + i] = src[i];
        }
    } else {        // exchange 2: header [max |x|, solver word], then the boundary solution
        double m = 0.0;
        for (int i = threadIdx.x; i < p.n_abs; i += 256) m = nan_max(m, p.abs_part[i]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = nan_max(m, __shfl_xor(m, o));
        __shared__ double sm[4];
        if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            dst[0] = nan_max(nan_max(sm[0], sm[1]), nan_max(sm[2], sm[3]));
            dst[1] = (double)*p.info;
        }
        for (int i = threadIdx.x; i < p.n_bnd; i += 256) dst[2 + i] = p.x[p.bnd[i]];
    }
    const uint32_t e = *p.epoch;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<uint32_t*>(base + p.flag_off + 64 * (int64_t)p.rank), e, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void p2p_wait_kernel(const P2PWait w, unsigned long long* stamp) {
    p2p_wait_block(w);
    if (stamp && threadIdx.x == 0) *stamp = __builtin_amdgcn_s_memrealtime();
}

__global__ __launch_bounds__(256) void cache_scrub_kernel(const double* buf, int64_t n, double* sink) {
    double acc = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc += buf[i];
    if (acc == -1.0) sink[0] = acc;   // never true for the zeroed buffer: keeps the loads alive
}

template <typename T> __global__ void to_f64_kernel(const T* in, double* out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (double)in[i];
}

template <typename T> __global__ void from_f64_kernel(const double* in, T* out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (T)in[i];
}

template <typename T>
__global__ void gather_f64_kernel(const T* in, const int32_t* idx, double* out, int64_t n, unsigned long long* stamp,
                                  uint32_t* epoch, const T* cin, double* cout, int64_t cn) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (stamp) *stamp = __builtin_amdgcn_s_memrealtime();
        if (epoch) *epoch += 1u;
    }
    // items [0, n): the gather; then the copy, four values per item (16-byte fp32 loads, two 16-byte
    // fp64 stores; both arrays are allocation-aligned), then its last cn % 4 values one per item
    const int64_t step = (int64_t)gridDim.x * blockDim.x, cv = cn >> 2;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n + cv + (cn & 3); i += step) {
        if (i < n) {
            out[i] = (double)in[idx[i]];
        } else if (i < n + cv) {
            const int64_t j = i - n;
            const V4<T> v = load4(cin + 4 * j);
            V2<double>* o = (V2<double>*)(cout + 4 * j);
            o[0] = V2<double>{(double)v.x, (double)v.y};
            o[1] = V2<double>{(double)v.z, (double)v.w};
        } else {
            const int64_t j = 4 * cv + (i - n - cv);
            cout[j] = (double)cin[j];
        }
    }
}

// gather_f64_kernel when the folds read the fp32 block array's pose-landmark and landmark-diagonal
// region [lo, hi) themselves (multifrontal.hpp mf_set_fold_source): items [0, n) the right-hand side
// gather, then the block array outside the region, in pairs of values (lo and hi even)
__global__ void gather_f64_ranges_kernel(const float* in, const int32_t* idx, double* out, int64_t n,
                                         unsigned long long* stamp, uint32_t* epoch, const float* cin, double* cout,
                                         int64_t cn, int64_t lo, int64_t hi) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (stamp) *stamp = __builtin_amdgcn_s_memrealtime();
        if (epoch) *epoch += 1u;
    }
    const int64_t pa = lo >> 1, pb = (cn - hi + 1) >> 1;
    const int64_t step = (int64_t)gridDim.x * blockDim.x, items = n + pa + pb;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < items; i += step) {
        if (i < n) {
            out[i] = (double)in[idx[i]];
        } else {
            const int64_t j = i < n + pa ? 2 * (i - n) : hi + 2 * (i - n - pa);
            cout[j] = (double)cin[j];
            if (j + 1 < cn) cout[j + 1] = (double)cin[j + 1];
        }
    }
}

// gather_f64_kernel with a factored pose-landmark region (LinParams::pl_factored): items [0, n) the
// right-hand side gather, then the block array in pairs of values outside the region and one slot
// per item inside it (3 fp32 values in, 6 fp64 values out: the block J_p^T J_l, J_p = (-J_lx, -J_ly,
// J_theta), each product rounded in fp32 as the unfactored kernel rounds it)
__global__ void gather_f64_factored_kernel(const float* in, const int32_t* idx, double* out, int64_t n,
                                           unsigned long long* stamp, uint32_t* epoch, const float* cin, double* cout,
                                           int64_t cn, int64_t pl_off, int64_t pl_slots) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (stamp) *stamp = __builtin_amdgcn_s_memrealtime();
        if (epoch) *epoch += 1u;
    }
    const int64_t pa = pl_off >> 1;                          // value pairs before the region (pl_off even)
    const int64_t pend = pl_off + 6 * pl_slots;              // even
    const int64_t pb = (cn - pend + 1) >> 1;                 // value pairs after it (the last may be single)
    const int64_t step = (int64_t)gridDim.x * blockDim.x, items = n + pa + pl_slots + pb;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < items; i += step) {
        if (i < n) {
            out[i] = (double)in[idx[i]];
        } else if (i < n + pa + pl_slots && i >= n + pa) {
            const int64_t sl = i - n - pa;
            const float* f = cin + pl_off + 3 * sl;
            const float jt = f[0], jx = f[1], jy = f[2];
            const float px = -jx, py = -jy;
            V2<double>* o = (V2<double>*)(cout + pl_off + 6 * sl);
            o[0] = V2<double>{(double)(px * jx), (double)(px * jy)};
            o[1] = V2<double>{(double)(py * jx), (double)(py * jy)};
            o[2] = V2<double>{(double)(jt * jx), (double)(jt * jy)};
        } else {
            const int64_t j = i < n + pa ? 2 * (i - n) : pend + 2 * (i - n - pa - pl_slots);
            cout[j] = (double)cin[j];
            if (j + 1 < cn) cout[j + 1] = (double)cin[j + 1];
        }
    }
}

__global__ void scatter_dense_kernel(const int32_t* rowptr, const int32_t* colind, const double* val, int n,
                                     double* dense) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    for (int e = rowptr[r]; e < rowptr[r + 1]; ++e) dense[(int64_t)colind[e] * n + r] = val[e];  // col-major lower
}

}  // namespace

template <typename T, bool W, bool D, int LPP, int MINW>
hipError_t launch_lin_k(LinParams<T> p, hipStream_t s) {
    const int lm_blocks = (p.n_lm_lanes + kBlock - 1) / kBlock;
    if (p.pose_b0 < 0 || p.n_pose_run < 0 || p.pose_b0 + p.n_pose_run > p.pose_blocks || p.lm_b0 < 0 || p.n_lm_run < 0 ||
        p.lm_b0 + p.n_lm_run > lm_blocks)
        return hipErrorInvalidValue;   // a block range outside the build (checked before any launch)
    const int grid = (p.n_pose_run + p.n_lm_run) * kJhSub;
    if (grid == 0) {
        if (p.t_start) hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(1), 0, s, p.t_start);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((linearize_kernel<T, W, D, LPP, MINW>), dim3(grid), dim3(kJhWg), 0, s, p);
    return hipGetLastError();
}

template <typename T, bool W, bool D, int MINW>
hipError_t launch_lin_lpp(const LinParams<T>& p, int lpp, hipStream_t s) {
    switch (lpp) {
        case 1: return launch_lin_k<T, W, D, 1, MINW>(p, s);
        case 2: return launch_lin_k<T, W, D, 2, MINW>(p, s);
        case 4: return launch_lin_k<T, W, D, 4, MINW>(p, s);
        default: return hipErrorInvalidValue;
    }
}

// Minimum waves per SIMD the kernel is compiled for (register budget): 4 (<= 128 VGPRs); 5 (<= 102)
// makes the fp64 variant spill, measured slower (36 vs 31 us on config 3), and 80 VGPRs for every
// variant (all two-lane waves resident) spill in fp32 too.
template <typename T, bool W, bool D>
hipError_t launch_lin_w(const LinParams<T>& p, int lpp, hipStream_t s) {
    return launch_lin_lpp<T, W, D, 4>(p, lpp, s);
}

template <typename T>
hipError_t launch_linearize(const LinParams<T>& p, int lpp, bool has_w, bool has_dups, hipStream_t s) {
    if (has_w) return has_dups ? launch_lin_w<T, true, true>(p, lpp, s) : launch_lin_w<T, true, false>(p, lpp, s);
    return has_dups ? launch_lin_w<T, false, true>(p, lpp, s) : launch_lin_w<T, false, false>(p, lpp, s);
}

template <typename T> hipError_t launch_boxplus(const UpdateParams<T>& p, hipStream_t s) {
    const int n = p.nodes ? p.n_nodes : p.NP + p.NL;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL((boxplus_kernel<T>), dim3((n + kUpdateBlock - 1) / kUpdateBlock), dim3(kUpdateBlock), 0, s, p);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_seg_copy(T* val, T* b, T* send, T* recv, T* aux, const ExSeg* segs, int nseg, int64_t max_len,
                           hipStream_t s, unsigned long long* stamp, const P2PWait& w) {
    if (w.mailbox && (w.world <= 0 || w.world > 64)) return hipErrorInvalidValue;
    if (nseg == 0 || max_len == 0) {
        if (w.mailbox) hipLaunchKernelGGL(p2p_wait_kernel, dim3(1), dim3(64), 0, s, w, stamp);
        else if (stamp) hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(1), 0, s, stamp);
        return hipGetLastError();
    }
    const int64_t bx = std::min<int64_t>((max_len + 255) / 256, 256);
    hipLaunchKernelGGL((seg_copy_kernel<T>), dim3((unsigned)bx, (unsigned)nseg), dim3(256), 0, s, val, b, send, recv, aux,
                       segs, stamp, w);
    return hipGetLastError();
}

template <typename T> hipError_t launch_triangulate(const TriParams<T>& p, hipStream_t s) {
    if (p.NL == 0) return hipSuccess;
    hipLaunchKernelGGL((triangulate_kernel<T>), dim3((p.NL + 255) / 256), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_reduce_stats(const double* chi_part, const int32_t* nrob_part, int n, double chi_const,
                               int32_t nrob_const, const double* max_part, int n_max, int32_t* info,
                               StepStatus* out, StepStatus* mirror, hipStream_t s) {
    hipLaunchKernelGGL(reduce_stats_kernel, dim3(1), dim3(256), 0, s, chi_part, nrob_part, n, chi_const, nrob_const,
                       max_part, n_max, info, out, mirror);
    return hipGetLastError();
}

hipError_t launch_shard_header1(const double* chi_part, const int32_t* nrob_part, int n_parts, double* send1,
                                hipStream_t s, unsigned long long* stamp) {
    hipLaunchKernelGGL(shard_header1_kernel, dim3(1), dim3(256), 0, s, chi_part, nrob_part, n_parts, send1, stamp);
    return hipGetLastError();
}

hipError_t launch_shard_pack2(const double* x, const int32_t* nodes, int n_nodes, const int32_t* node_dof, int NP,
                              int32_t* info, const int32_t* bnd, int n_bnd, double* part, double* send2,
                              hipStream_t s, unsigned long long* stamp) {
    const int nb = std::max(1, (n_nodes + 255) / 256);
    hipLaunchKernelGGL(node_absmax_kernel, dim3(nb), dim3(256), 0, s, x, nodes, n_nodes, node_dof, NP, part);
    const int pb = std::max(1, std::min(256, (n_bnd + 255) / 256));
    hipLaunchKernelGGL(shard_pack2_kernel, dim3(pb), dim3(256), 0, s, x, part, nb, info, bnd, n_bnd, send2, stamp);
    return hipGetLastError();
}

int launch_node_absmax(const double* x, const int32_t* nodes, int n_nodes, const int32_t* node_dof, int NP, double* part,
                       hipStream_t s, hipError_t* err) {
    const int nb = std::max(1, (n_nodes + 255) / 256);
    hipLaunchKernelGGL(node_absmax_kernel, dim3(nb), dim3(256), 0, s, x, nodes, n_nodes, node_dof, NP, part);
    *err = hipGetLastError();
    return nb;
}

hipError_t launch_index_copy(const double* src, const int32_t* src_idx, double* dst, const int32_t* dst_idx, int64_t n,
                             hipStream_t s, unsigned long long* stamp, const P2PWait& w) {
    if (w.mailbox && (w.world <= 0 || w.world > 64)) return hipErrorInvalidValue;
    if (n == 0) {
        if (w.mailbox) hipLaunchKernelGGL(p2p_wait_kernel, dim3(1), dim3(64), 0, s, w, stamp);
        else if (stamp) hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(1), 0, s, stamp);
        return hipGetLastError();
    }
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(index_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, src_idx, dst, dst_idx, n, stamp, w);
    return hipGetLastError();
}

hipError_t launch_shard_combine(const double* recv1, int64_t c1, const double* recv2, int64_t c2, int world,
                                double chi_const, int32_t nrob_const, int32_t* local_info, StepStatus* out,
                                StepStatus* mirror, hipStream_t s, bool zero_info) {
    hipLaunchKernelGGL(shard_combine_kernel, dim3(1), dim3(64), 0, s, recv1, c1, recv2, c2, world, chi_const, nrob_const,
                       local_info, out, mirror, zero_info);
    return hipGetLastError();
}

hipError_t launch_p2p_push(const double* send, int64_t count, double* const* peers, int64_t data_off, int64_t flag_off,
                           int rank, int world, const uint32_t* epoch, const double* chi_part, const int32_t* nrob_part,
                           int n_parts, unsigned long long* stamp, hipStream_t s) {
    if (world <= 0 || (chi_part && count < kExHeader)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(p2p_push_kernel, dim3(world), dim3(256), 0, s, send, count, peers, data_off, flag_off, rank, epoch,
                       chi_part, nrob_part, n_parts, stamp);
    return hipGetLastError();
}

hipError_t launch_p2p_push_gather(const P2PPush& p, hipStream_t s) {
    const bool bad1 = p.which == 1 && (!p.chi_part || (p.nseg > 0 && (!p.segs || !p.U || !p.u)));
    const bool bad2 = p.which == 2 && (!p.info || !p.x || (p.n_abs > 0 && !p.abs_part) || (p.n_bnd > 0 && !p.bnd) ||
                                       p.count < 2 + (int64_t)p.n_bnd);
    if (p.world <= 0 || (p.which != 1 && p.which != 2) || p.count < kExHeader || bad1 || bad2)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(p2p_push_gather_kernel, dim3(p.world), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_cache_scrub(const double* buf, int64_t n, double* sink, hipStream_t s) {
    hipLaunchKernelGGL(cache_scrub_kernel, dim3(4096), dim3(256), 0, s, buf, n, sink);
    return hipGetLastError();
}

template <typename T> hipError_t launch_to_f64(const T* in, double* out, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL((to_f64_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}

template <typename T> hipError_t launch_from_f64(const double* in, T* out, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL((from_f64_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_gather_f64(const T* in, const int32_t* idx, double* out, int64_t n, hipStream_t s,
                             unsigned long long* stamp, uint32_t* epoch, const T* cin, double* cout, int64_t cn) {
    if (n + cn == 0 && !stamp && !epoch) return hipSuccess;
    const int64_t items = n + (cn >> 2) + (cn & 3);
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((items + 255) / 256, 8192));
    hipLaunchKernelGGL((gather_f64_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, in, idx, out, n, stamp, epoch,
                       cin, cout, cn);
    return hipGetLastError();
}

hipError_t launch_gather_f64_factored(const float* in, const int32_t* idx, double* out, int64_t n, hipStream_t s,
                                      unsigned long long* stamp, uint32_t* epoch, const float* cin, double* cout,
                                      int64_t cn, int64_t pl_off, int64_t pl_slots) {
    if ((pl_off & 1) || pl_off + 6 * pl_slots > cn) return hipErrorInvalidValue;   // checked before launching
    const int64_t items = n + (pl_off >> 1) + pl_slots + ((cn - pl_off - 6 * pl_slots + 1) >> 1);
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((items + 255) / 256, 8192));
    hipLaunchKernelGGL(gather_f64_factored_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, idx, out, n, stamp, epoch,
                       cin, cout, cn, pl_off, pl_slots);
    return hipGetLastError();
}

hipError_t launch_gather_f64_ranges(const float* in, const int32_t* idx, double* out, int64_t n, hipStream_t s,
                                    unsigned long long* stamp, uint32_t* epoch, const float* cin, double* cout,
                                    int64_t cn, int64_t lo, int64_t hi) {
    if ((lo & 1) || (hi & 1) || lo > hi || hi > cn) return hipErrorInvalidValue;   // checked before launching
    const int64_t items = n + (lo >> 1) + ((cn - hi + 1) >> 1);
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((items + 255) / 256, 8192));
    hipLaunchKernelGGL(gather_f64_ranges_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, idx, out, n, stamp, epoch,
                       cin, cout, cn, lo, hi);
    return hipGetLastError();
}

void expand_factored_host(const float* in, double* out, int64_t n, int64_t pl_off, int64_t pl_slots) {
    for (int64_t i = 0; i < n; ++i) out[i] = in[i];
    for (int64_t sl = 0; sl < pl_slots; ++sl) {
        const float* f = in + pl_off + 3 * sl;
        const float jt = f[0], jx = f[1], jy = f[2], px = -jx, py = -jy;
        double* o = out + pl_off + 6 * sl;
        o[0] = (double)(px * jx); o[1] = (double)(px * jy);
        o[2] = (double)(py * jx); o[3] = (double)(py * jy);
        o[4] = (double)(jt * jx); o[5] = (double)(jt * jy);
    }
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
template hipError_t launch_triangulate<double>(const TriParams<double>&, hipStream_t);
template hipError_t launch_seg_copy<double>(double*, double*, double*, double*, double*, const ExSeg*, int, int64_t,
                                            hipStream_t, unsigned long long*, const P2PWait&);
template hipError_t launch_seg_copy<float>(float*, float*, float*, float*, float*, const ExSeg*, int, int64_t,
                                           hipStream_t, unsigned long long*, const P2PWait&);
template hipError_t launch_triangulate<float>(const TriParams<float>&, hipStream_t);
template hipError_t launch_to_f64<double>(const double*, double*, int64_t, hipStream_t);
template hipError_t launch_to_f64<float>(const float*, double*, int64_t, hipStream_t);
template hipError_t launch_from_f64<double>(const double*, double*, int64_t, hipStream_t);
template hipError_t launch_from_f64<float>(const double*, float*, int64_t, hipStream_t);
template hipError_t launch_gather_f64<double>(const double*, const int32_t*, double*, int64_t, hipStream_t,
                                              unsigned long long*, uint32_t*, const double*, double*, int64_t);
template hipError_t launch_gather_f64<float>(const float*, const int32_t*, double*, int64_t, hipStream_t,
                                             unsigned long long*, uint32_t*, const float*, double*, int64_t);

}  // namespace dev
}  // namespace bos
