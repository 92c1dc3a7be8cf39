// GPU supernodal multifrontal Cholesky for the GN normal system (replaces the reference's
// Eigen SimplicialLDLT, slam/solver.cpp:75-85; pattern analysed once like analyzePattern at
// :77-80 — here the symbolic analysis is host/plan.cpp build_multifrontal).
//
// P^T H_nf P = L L^T, H read from the J+H kernel's block array through the assembly map. The
// assembly tree is processed level by level (leaves first). Each level has two launches:
//  * fronts with m = k + r <= kMfWaveMaxM (the many small ones near the leaves), binned by m into
//    classes 16 / 32 / 48 / 64: one wavefront per front, assembled packed in LDS, then factored in
//    registers (lane i holds row i; each pivot column broadcast through a 2 x MAXM LDS buffer);
//  * larger fronts: one 256-thread workgroup, full m x m front in LDS (m <= 90) or global scratch.
// A front is
//   1. zeroed, then receives its entries of H (precomputed map) and the extend-add of its
//      children's update matrices (children sequentially, entries in parallel: deterministic),
//   2. partially factored (right-looking Cholesky of its k own columns),
//   3. written out: the m x k panel of L and the packed r x r update matrix for its parent.
// Forward (bottom-up) and backward (top-down) substitutions use the same tree and levels; the
// wave variants stage the L panel in LDS so no global load sits on the sequential dependency chain.
// Everything is fp64 and deterministic (no atomics on values).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <string>
#include <type_traits>
#include <vector>

#include "../host/plan.hpp"
#include "multifrontal.hpp"

namespace bos {
namespace dev {

namespace {

constexpr int kMfBlock = 256;
#ifdef BOS_MF_PIVOT_CYCLES
__device__ unsigned long long* g_pivot_bwd;   // diagnostic build: the stamp buffer's backward half
#endif
constexpr int kLdsCapM = 90;   // larger fronts up to 90 x 90 doubles (64.8 KB) are factored in LDS

__device__ __forceinline__ int64_t pk(int64_t i, int64_t j, int64_t m) { return j * m - j * (j - 1) / 2 + (i - j); }
__device__ __forceinline__ int pk32(int i, int j, int m) { return j * m - j * (j - 1) / 2 + (i - j); }   // LDS fronts

// L panel traffic (written by the factorization, read once by the backward substitution): the
// stores are non-temporal, so the solve's ~300 MB of L stream past the caches instead of evicting the
// next J+H build's inputs (in-step J+H 16.0-16.5 -> 13.2-14.5 us, solve -14 us; plain stores and
// loads: profiles/r05_ntl_lds_ab.txt). The backward launches' panel loads are non-temporal too (plain
// loads measured slower), except the folded landmarks' backward launch, which reads its L columns
// with plain loads (non-temporal there: solve +13 us, profiles/r05_fold_l_policy_ab.txt).
#define ST_L(p, i, v) __builtin_nontemporal_store((v), (p) + (i))
#define LD_L(p, i) __builtin_nontemporal_load((p) + (i))
#define ST_LF(p, i, v) ST_L(p, i, v)
#define LD_LF(p, i) ((p)[i])

// Copy n doubles global -> LDS by one wavefront, 8 independent loads in flight per lane.
template <int U = 8, bool NTL = false> __device__ __forceinline__ void stage_lds(double* dst, const double* src, int n, int lane) {
    for (int e0 = 0; e0 < n; e0 += 64 * U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = e0 + 64 * u + lane;
            v[u] = e < n ? (NTL ? LD_L(src, e) : src[e]) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = e0 + 64 * u + lane;
            if (e < n) dst[e] = v[u];
        }
    }
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Hand-off data between fronts processed in one dataflow launch (update matrices, forward
// u-vectors, backward x rows) is written and read with relaxed agent-scope atomics (coherent sc1
// accesses) so no L2-wide release/acquire fence is needed per front; COH = false is plain access.
template <bool COH> __device__ __forceinline__ double ldc(const double* p) {
    if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <bool COH> __device__ __forceinline__ void stc(double* p, double v) {
    if constexpr (COH) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

// Tagged granules (cdna_hip_programming.md §6 Guideline 16, R2: the data is the flag). A double
// travels as two 8-byte granules {epoch, 32 bits of it}, each written by one relaxed agent-scope
// atomic store (sc1, write-through) and read by relaxed agent-scope atomic loads (sc1): a consumer
// that sees the step's epoch in both tags holds the value, with no flag, no drain of the producer's
// stores and no second load round trip. The epoch is the GN step's (never 0, bumped per step), so
// granules of earlier steps never match.
__device__ __forceinline__ void tag_pair(unsigned long long* g, double v, uint32_t epoch) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v), t = (unsigned long long)epoch << 32;
    __hip_atomic_store(g, t | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(g + 1, t | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one read of a tagged pair: *ok &= both tags current; the value assembled from the halves
__device__ __forceinline__ double untag_pair(const unsigned long long* g, uint32_t epoch, bool& ok) {
    const unsigned long long lo = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long hi = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ok = ok && (uint32_t)(lo >> 32) == epoch && (uint32_t)(hi >> 32) == epoch;
    return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
}

struct MfArgs {
    const int32_t* level;        // supernode ids of this level
    int count;
    const int32_t* col0;
    const int32_t* k;
    const int32_t* r;
    const int64_t* L_off;
    const int64_t* U_off;
    const int64_t* u_off;
    const int64_t* scratch_off;  // -1 => LDS
    const int32_t* child_ptr;
    const int32_t* child;
    const int64_t* rmap_off;
    const int32_t* rmap;
    const int32_t* amap_ptr;
    const int32_t* amap_src;
    const int32_t* amap_dst;
    const int64_t* findex_off;
    const int32_t* findex;
    const double* A;             // CSR values of H (fp64)
    const float* A32;            // fp32 block array the fold reads instead of A (see mf_set_fold_source),
    int64_t pl_lo;               // and where its factored pose-landmark region starts; A32 null otherwise
    double* L;
    double* U;
    double* u;
    double* scratch;
    double* x;                   // rhs in, solution out (permuted order)
    int32_t* info;               // count of non-positive pivots
    const int32_t* fold_cnt;     // folded landmark children (Schur ordering, see plan.hpp)
    const int32_t* fold_cptr;
    const int32_t* fold_chunk;
    const int32_t* fold_rec;
    const int16_t* emap;            // extend-add positions: entry e of child c's packed update matrix goes to
    const int64_t* emap_off;        // packed position emap[emap_off[c] + e] of its parent's front (wave fronts)
    unsigned long long* stamps_f;   // diagnostics (mf_debug_set_stamps): factor / backward stamps, or null
    unsigned long long* stamps_b;
    // tagged hand-offs inside a dataflow launch (tag_pair / sweep): a flow front whose parent is in
    // the same flow publishes its update matrix and u-vector as tagged granules at Ug + ug_off[s]
    // (-1: plain U / u); every backward front publishes its solved x as tagged granules xg[2 dof]
    unsigned long long* Ug;
    const int64_t* ug_off;
    unsigned long long* xg;
    const int8_t* xtag;             // per supernode: its x is read by a backward flow front (write xg)
    const uint32_t* epoch;          // the GN step's epoch (device word, mf_epoch_ptr)
};

// LDS of one wave's fold chunk: the y (forward-step) values of its landmarks, two per landmark
struct FoldBuf {
    double y[2 * fold_chunk_landmarks(kMfWaveMaxM)];
};

typedef double dbl4 __attribute__((ext_vector_type(4)));

// The folded landmarks' contribution to the front, lower 16 x 16 blocks of W W^T (f64 MFMA
// accumulators: lane l holds rows (l >> 4) + 4 v, column l & 15 of each block) and, per
// position lane, the u-vector part -W y.
template <int MAXM>
struct FoldAcc {
    static constexpr int NB = (MAXM + 15) / 16, NP = NB * (NB + 1) / 2;
    dbl4 d[NP];
    double w;
};

// Assembly of H entries into a front by one wavefront (F[dst] = A[src], or += when the front
// already holds the folded landmarks' part), 4 entries per lane in flight: index loads, then value
// gathers, then LDS stores. Loads past the front's range are clamped to its last entry instead of
// predicated: a predicated load becomes a branch with the load's wait inside it, which serialises
// the four loads (one memory latency each instead of one for all four).
__device__ __forceinline__ void assemble_wave(const MfArgs& a, int q0_, int q1, double* F, int lane, bool add) {
    for (int q0 = q0_; q0 < q1; q0 += 256) {
        int src[4], dst[4];
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = min(q0 + 64 * u + lane, q1 - 1);
            src[u] = a.amap_src[q];
            dst[u] = a.amap_dst[q];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = a.A[src[u]];
        if (add) {   // (uniform) the four front entries read at once, as in extend_child
            double f[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) f[u] = F[dst[u]];
            asm volatile("" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] += f[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (q0 + 64 * u + lane < q1) F[dst[u]] = v[u];
    }
}

// lane l's double, broadcast to the wave (l uniform)
__device__ __forceinline__ double readlane_d(double x, int l) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__global__ __launch_bounds__(kMfBlock) void mf_factor_level(const MfArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int s = a.level[blockIdx.x];
    const int k = a.k[s], r = a.r[s], m = k + r;
    const int tid = threadIdx.x;
    const int64_t so = a.scratch_off[s];
    double* F = so < 0 ? lds : a.scratch + so;
    const int64_t mm = (int64_t)m * m;
    for (int64_t e = tid; e < mm; e += kMfBlock) F[e] = 0.0;
    __syncthreads();
    // scatter H entries (each front position receives at most one entry)
    for (int q = a.amap_ptr[s] + tid; q < a.amap_ptr[s + 1]; q += kMfBlock) F[a.amap_dst[q]] = a.A[a.amap_src[q]];
    __syncthreads();
    // extend-add children's update matrices, one child at a time (lower triangle)
    for (int ci = a.child_ptr[s]; ci < a.child_ptr[s + 1]; ++ci) {
        const int c = a.child[ci];
        const int rc = a.r[c];
        const int32_t* map = a.rmap + a.rmap_off[c];
        const double* Uc = a.U + a.U_off[c];
        for (int j = tid >> 6; j < rc; j += kMfBlock / 64) {
            const int64_t pj = (int64_t)map[j] * m;
            const double* uj = Uc + pk(j, j, rc) - j;
            for (int i = j + (tid & 63); i < rc; i += 64) F[map[i] + pj] += uj[i];
        }
        __syncthreads();
    }
    // right-looking partial Cholesky of the first k columns
    const int wave = tid >> 6, lane = tid & 63;
    for (int j = 0; j < k; ++j) {
        double d = F[j + (int64_t)j * m];
        if (!(d > 0.0)) {
            if (tid == 0) atomicAdd(a.info, 1);
            d = 1e-300;
        }
        const double ljj = sqrt(d);
        const double inv = 1.0 / ljj;
        __syncthreads();
        if (tid == 0) F[j + (int64_t)j * m] = ljj;
        for (int i = j + 1 + tid; i < m; i += kMfBlock) F[i + (int64_t)j * m] *= inv;
        __syncthreads();
        for (int l = j + 1 + wave; l < m; l += kMfBlock / 64) {
            const double flj = F[l + (int64_t)j * m];
            double* col = F + (int64_t)l * m;
            const double* cj = F + (int64_t)j * m;
            for (int i = l + lane; i < m; i += 64) col[i] -= cj[i] * flj;
        }
        __syncthreads();
    }
    // write the L panel (m x k) and the update matrix (r x r)
    double* Ls = a.L + a.L_off[s];
    const int64_t nL = (int64_t)m * k;
    for (int64_t e = tid; e < nL; e += kMfBlock) Ls[e] = F[e];
    double* Us = a.U + a.U_off[s];
    for (int j = wave; j < r; j += kMfBlock / 64) {
        double* uj = Us + pk(j, j, r) - j;
        const double* fj = F + (k + (int64_t)(k + j) * m);
        for (int i = j + lane; i < r; i += 64) uj[i] = fj[i];
    }
}

// forward substitution L y = b for one level (bottom-up); x holds b on entry, y on exit for the
// supernode's own dofs; u receives the r-vector passed to the parent
__global__ __launch_bounds__(kMfBlock) void mf_forward_level(const MfArgs a) {
    extern __shared__ __attribute__((aligned(16))) double w[];
    const int s = a.level[blockIdx.x];
    const int k = a.k[s], r = a.r[s], m = k + r;
    const int tid = threadIdx.x;
    const int c0 = a.col0[s];
    for (int i = tid; i < m; i += kMfBlock) w[i] = i < k ? a.x[c0 + i] : 0.0;
    __syncthreads();
    for (int ci = a.child_ptr[s]; ci < a.child_ptr[s + 1]; ++ci) {
        const int c = a.child[ci];
        const int rc = a.r[c];
        const int32_t* map = a.rmap + a.rmap_off[c];
        const double* uc = a.u + a.u_off[c];
        for (int t = tid; t < rc; t += kMfBlock) w[map[t]] += uc[t];
        __syncthreads();
    }
    const double* Ls = a.L + a.L_off[s];
    for (int j = 0; j < k; ++j) {
        const double yj = w[j] / Ls[j + (int64_t)j * m];
        __syncthreads();
        if (tid == 0) w[j] = yj;
        for (int i = j + 1 + tid; i < m; i += kMfBlock) w[i] -= Ls[i + (int64_t)j * m] * yj;
        __syncthreads();
    }
    for (int i = tid; i < m; i += kMfBlock) {
        if (i < k) a.x[c0 + i] = w[i];
        else a.u[a.u_off[s] + (i - k)] = w[i];
    }
}

// backward substitution L^T x = y for one level (top-down): the rows below the supernode are
// ancestors' dofs whose solution is already final in x
__global__ __launch_bounds__(kMfBlock) void mf_backward_level(const MfArgs a) {
    extern __shared__ __attribute__((aligned(16))) double w[];   // [0,k): y / x,  [k,2k): t
    const int s = a.level[blockIdx.x];
    const int k = a.k[s], r = a.r[s], m = k + r;
    const int tid = threadIdx.x;
    const int c0 = a.col0[s];
    const double* Ls = a.L + a.L_off[s];
    const int32_t* fi = a.findex + a.findex_off[s];
    double* t = w + k;
    // t_j = sum_{i >= k} L[i, j] x[findex[i]]
    const int wave = tid >> 6, lane = tid & 63;
    for (int j = wave; j < k; j += kMfBlock / 64) {
        double acc = 0.0;
        for (int i = k + lane; i < m; i += 64) acc += Ls[i + (int64_t)j * m] * a.x[fi[i]];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) t[j] = acc;
    }
    if (k <= 64) {
        // L11 staged in LDS (column i at stride k + 1) by all waves, then the triangular solve on
        // wave 0 alone, lane i holding t_i: no barrier and no global load in the sequential chain
        // (config 2's separators: k = 20-40, 16-21 us per launch with a barrier pair and a global
        // diagonal load per column). Same operations in the same order: bit-identical x.
        double* S = t + k;
        for (int e = tid; e < k * k; e += kMfBlock) {
            const int i = e / k, j = e - i * k;
            if (j >= i) S[j + i * (k + 1)] = Ls[j + (int64_t)i * m];
        }
        __syncthreads();
        if (wave) return;
        const bool on = lane < k;
        double ti = on ? t[lane] : 0.0;
        const double wi = on ? a.x[c0 + lane] : 0.0;
        const double di = on ? S[lane * (k + 2)] : 1.0;
        double xi = 0.0;
        for (int j = k - 1; j >= 0; --j) {
            const double xj = readlane_d(wi - ti, j) / readlane_d(di, j);
            if (lane == j) xi = xj;
            if (lane < j) ti += S[j + lane * (k + 1)] * xj;
        }
        if (on) {
            a.x[c0 + lane] = xi;
            if (a.xtag[s]) tag_pair(a.xg + 2 * (int64_t)(c0 + lane), xi, *a.epoch);
        }
        return;
    }
    for (int j = tid; j < k; j += kMfBlock) w[j] = a.x[c0 + j];
    __syncthreads();
    for (int j = k - 1; j >= 0; --j) {
        const double xj = (w[j] - t[j]) / Ls[j + (int64_t)j * m];
        __syncthreads();
        if (tid == 0) w[j] = xj;
        for (int i = tid; i < j; i += kMfBlock) t[i] += Ls[j + (int64_t)i * m] * xj;
        __syncthreads();
    }
    for (int j = tid; j < k; j += kMfBlock) a.x[c0 + j] = w[j];
    if (a.xtag[s]) {
        const uint32_t ep = *a.epoch;
        for (int j = tid; j < k; j += kMfBlock) tag_pair(a.xg + 2 * (int64_t)(c0 + j), w[j], ep);
    }
}

// One wavefront per front with m <= MAXM, the factorization in registers: lane i holds row i of
// the (lower) front in a compile-time-indexed array; each column step broadcasts the pivot column
// through a small LDS buffer (one store per lane, broadcast reads). LDS otherwise only stages the
// assembly. F: packed front (MAXM (MAXM + 1) / 2), colbuf: 2 MAXM.

// 1 / sqrt(d) for d > 0 in the normal range: hardware estimate refined by two Newton steps
// (quadratic convergence: full double precision, within an ulp or two of 1.0 / sqrt(d)).
__device__ __forceinline__ double rsqrt_nr(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

// phase stamp k of front s (lane 0; the product launches pass no stamp buffer)
__device__ __forceinline__ void fstamp(unsigned long long* stp, int s, int k) {
#ifdef BOS_MF_PIVOT_CYCLES
    if (stp && stp == g_pivot_bwd) return;   // the backward half holds the pivot-loop cycle stamps
#endif
    if (stp && (threadIdx.x & 63) == 0) stp[8 * (int64_t)s + k] = __builtin_amdgcn_s_memrealtime();
}
#ifdef BOS_MF_PIVOT_CYCLES
// Diagnostic build only (tools/pivot_cycles.py): core-clock stamps of every front in the backward
// half of the stamp buffer: [1] children ready, [2] their values loaded, [3] extend-added, [0] pivot
// loop start (rows in registers), [4..6] after two-pivot steps 1-3, [7] pivot loop end.
__device__ __forceinline__ void cstamp(unsigned long long* stpb, int s, int k) {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (stpb && (threadIdx.x & 63) == 0) stpb[8 * (int64_t)s + k] = t;
}
#endif

// Folded landmark children (Schur ordering) of front s, eliminated by its wave: per chunk (whole
// children, <= 64 row groups, <= fold_chunk_landmarks(m) landmarks) lane q takes one observing pose
// of landmark c — its 3 rows t, t + 1, t + 2 (one 32-byte record: sources of the pose-landmark
// block and of the landmark's 2 x 2 block, the landmark's col0 / r / L offset, the rows' first
// position in this front and c's index in the chunk), factors the 2 x 2 block, forms L[t + g,
// 0..1], the landmark's forward step y, and writes the landmark's L panel and y. The rows also form
// the chunk's W (front position x 2 columns per landmark, in LDS that the front's F uses later) and
// its y; W W^T accumulates in f64 MFMA registers (the landmarks' update matrices -L21 L21^T,
// summed) and -W y in the position lanes (their u-vectors). The caller subtracts both once the
// front is assembled. Nothing goes through global memory and the result is deterministic.
__device__ __forceinline__ int4 fold_rec_load(const MfArgs& a, int q, int half) {
    return reinterpret_cast<const int4*>(a.fold_rec + (int64_t)kFoldRec * q)[half];
}

// The values one chunk's row groups need (the pose-landmark block, 3 x 2, the landmark's 2 x 2
// block and right-hand side), gathered for chunk c + 1 while chunk c is processed.
struct FoldVals {
    double h[6];   // (row g, column j) at 2 g + j
    double a00, a10, a11, x0, x1;
};
// The same from the fp32 build (F32: mf_set_fold_source): the bearing's factored block (J_theta,
// J_lx, J_ly) and the landmark's 2 x 2 block as loaded, and the entries' presence in flags;
// fold_decode forms the doubles the fp64 copy would hold (products in fp32, as
// gather_f64_factored_kernel expands them), so the result is bit-identical.
struct FoldVals32 {
    float jt, jx, jy, a00, a10, a11;
    int flags;   // block present << 0 | a00, a10, a11 present << 2, 3, 4
    double x0, x1;
};
// The fp64 build's values as loaded and their presence in flags (as FoldVals32): the selects are
// applied by fold_decode when the chunk is processed, so the loads stay in flight until then (a
// select right after the loads made the wave wait for them in the chunk that issued them, one
// memory latency per chunk: config 2's blocked-front folds, 33 us at level 0)
struct FoldVals64 {
    double h[6], a00, a10, a11, x0, x1;
    int flags;   // block present << 0 | a00, a10, a11 present << 2, 3, 4
};
template <bool F32> using FoldValsT = typename std::conditional<F32, FoldVals32, FoldVals64>::type;

__device__ __forceinline__ FoldVals fold_decode(const FoldVals64& v) {
    FoldVals d;
    const bool blk = v.flags & 1;
#pragma unroll
    for (int e = 0; e < 6; ++e) d.h[e] = blk ? v.h[e] : 0.0;
    d.a00 = (v.flags & 4) ? v.a00 : 0.0;
    d.a10 = (v.flags & 8) ? v.a10 : 0.0;
    d.a11 = (v.flags & 16) ? v.a11 : 0.0;
    d.x0 = v.x0;
    d.x1 = v.x1;
    return d;
}
__device__ __forceinline__ FoldVals fold_decode(const FoldVals32& v) {
    FoldVals d;
    const bool blk = v.flags & 1;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        const float p = g == 0 ? -v.jx : g == 1 ? -v.jy : v.jt;   // J_p = (-J_lx, -J_ly, J_theta)
        d.h[2 * g] = blk ? (double)(p * v.jx) : 0.0;
        d.h[2 * g + 1] = blk ? (double)(p * v.jy) : 0.0;
    }
    d.a00 = (v.flags & 4) ? (double)v.a00 : 0.0;
    d.a10 = (v.flags & 8) ? (double)v.a10 : 0.0;
    d.a11 = (v.flags & 16) ? (double)v.a11 : 0.0;
    d.x0 = v.x0;
    d.x1 = v.x1;
    return d;
}

template <bool F32>
__device__ __forceinline__ FoldValsT<F32> fold_vals(const MfArgs& a, const int4& r0, const int4& r1, bool mine) {
    if constexpr (F32) {
        // records index the fp64 layout: the block of slot q at pl_lo + 6 q, held factored at
        // pl_lo + 3 q of the fp32 array (mf_set_fold_source checked the records)
        const int q = max(r0.x - (int)a.pl_lo, 0) / 6;
        const float* f = a.A32 + a.pl_lo + 3 * (int64_t)q;
        FoldVals32 v;
        v.jt = f[0];
        v.jx = f[1];
        v.jy = f[2];
        v.a00 = a.A32[max(r0.z, 0)];
        v.a10 = a.A32[max(r0.w, 0)];
        v.a11 = a.A32[max(r1.x, 0)];
        v.x0 = a.x[r1.y];   // (a lane past the chunk's groups reads its last group's: see fold_chunk)
        v.x1 = a.x[r1.y + 1];
        v.flags = (r0.x >= 0 ? 1 : 0) | (r0.z >= 0 ? 4 : 0) | (r0.w >= 0 ? 8 : 0) | (r1.x >= 0 ? 16 : 0);
        return v;
    } else {
    // every load unconditional (indices clamped to valid ones), the value selected afterwards: a
    // predicated load would be a branch with its wait inside, and the next chunk's values must stay
    // in flight while the current chunk is processed
    // (selected by fold_decode, see FoldVals64)
    const int b = max(r0.x, 0);
    FoldVals64 v;
#pragma unroll
    for (int e = 0; e < 6; ++e) v.h[e] = a.A[b + e];
    v.a00 = a.A[max(r0.z, 0)];
    v.a10 = a.A[max(r0.w, 0)];
    v.a11 = a.A[max(r1.x, 0)];
    v.x0 = a.x[r1.y];   // (lanes past the groups: their last group's)
    v.x1 = a.x[r1.y + 1];
    v.flags = (r0.x >= 0 ? 1 : 0) | (r0.z >= 0 ? 4 : 0) | (r0.w >= 0 ? 8 : 0) | (r1.x >= 0 ? 16 : 0);
    return v;
    }
}

// The chunk boundaries of a front (fold_chunk[c], c uniform) from one register holding 64 of them
// (lane i: fold_chunk[base + i]), re-read only when a front has more chunks than that: the loop then
// needs no dependent load per chunk (a vector load whose value decides the next loads would make
// the wave wait for every load issued before it, the prefetched values included).
struct ChunkTable {
    int base, v;
    __device__ __forceinline__ void load(const MfArgs& a, int b, int lane) {
        base = b;
        v = a.fold_chunk[b + lane];   // padded array (up()): in bounds
    }
    // the same inside the chunk loop, waited for on the spot: a load left pending on this rarely taken
    // path would make the compiler wait for every outstanding load at the loop's top on every path
    __device__ __forceinline__ void reload(const MfArgs& a, int b, int lane) {
        load(a, b, lane);
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) (expcnt, lgkmcnt: no wait)
    }
    // fold_chunk[c] for c in [base, base + 64)
    __device__ __forceinline__ int at(int c) const { return __builtin_amdgcn_readlane(v, c - base); }
};

// One fold chunk's elimination (values v, records' meta q1, n rows): the landmarks' 2 x 2 factors, L
// panels and forward steps, the chunk's W in LDS, and W W^T / -W y accumulated.
template <int MAXM, typename VALS>
__device__ __forceinline__ void fold_chunk(const MfArgs& a, double* W, FoldBuf* fb, int m, int lane,
                                           FoldAcc<MAXM>& acc, const VALS& vraw, const int4& q1, int n,
                                           bool first, int s, int& nbad) {
    const FoldVals v = fold_decode(vraw);
    constexpr int NB = FoldAcc<MAXM>::NB;
    constexpr int WS = 2 * fold_chunk_landmarks(MAXM) + 1;   // W row stride (odd: no bank conflicts)
    const int nbm = (m + 15) >> 4;
    const int t = q1.z & 63, rc = (q1.z >> 6) & 63, pos = (q1.z >> kFoldPosShift) & kFoldPosMask,
              lml = (q1.z >> kFoldLmShift) & 63;
    const bool mine = lane < n;
    const int nl = __builtin_amdgcn_readlane(lml, n - 1) + 1;   // landmarks of this chunk
    const int col0 = q1.y;
    const int64_t loff = q1.w;
    // Every lane issues the same global stores: a store under a divergent branch leaves the number of
    // memory operations after the next chunk's loads unknown to the compiler, which then waits for
    // all of them (vmcnt(0)) at the top of every chunk instead of for the loads alone. A lane past
    // the chunk's rows holds the record and values of its last row, and every row of a landmark the
    // landmark's values, so the extra stores write the owners' values, bit for bit, to the owners'
    // addresses (a shared sink instead was measured 17 us slower: every wave of the GPU wrote the
    // same lines).
    {
        double d0 = v.a00;
        const bool bad0 = !(d0 > 0.0);
        d0 = bad0 ? 1e-300 : d0;
        const double i0 = rsqrt_nr(d0), l00 = d0 * i0;
        const double l10 = v.a10 * i0;
        double d1 = v.a11 - l10 * l10;
        const bool bad1 = !(d1 > 0.0);
        d1 = bad1 ? 1e-300 : d1;
        const double i1 = rsqrt_nr(d1), l11 = d1 * i1;
        const double y0 = v.x0 * i0, y1 = (v.x1 - l10 * y0) * i1;
        const int mc = 2 + rc;
        double* Lc = a.L + loff;
        const bool head = mine && t == 0;
        double lt0[3], lt1[3];
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            lt0[g] = v.h[2 * g] * i0;
            lt1[g] = (v.h[2 * g + 1] - lt0[g] * l10) * i1;
            ST_LF(Lc, 2 + t + g, lt0[g]);
            ST_LF(Lc, mc + 2 + t + g, lt1[g]);
        }
        ST_LF(Lc, 0, l00);
        ST_LF(Lc, 1, l10);
        ST_LF(Lc, mc + 1, l11);
        a.x[col0] = y0;
        a.x[col0 + 1] = y1;
        nbad += head ? (int)bad0 + (int)bad1 : 0;
        if (head) {
            fb->y[2 * lml] = y0;
            fb->y[2 * lml + 1] = y1;
        }
        if (mine) {
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                W[(pos + g) * WS + 2 * lml] = lt0[g];
                W[(pos + g) * WS + 2 * lml + 1] = lt1[g];
            }
        }
    }
    wave_sync();
    const int kc = 2 * nl;
    if (lane < m) {   // u-vector part: -(W y) at this lane's position
        double w = 0.0;
        for (int q = 0; q < kc; ++q) w += W[lane * WS + q] * fb->y[q];
        acc.w -= w;
    }
    // W W^T, 4 columns per MFMA step; lane l feeds row 16 b + (l & 15), column 4 st + (l >> 4)
    // of W to the blocks of row b (as A) and of column b (as B, the same values)
    for (int st = 0; 4 * st < kc; ++st) {
        double av[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) av[b] = b < nbm ? W[(16 * b + (lane & 15)) * WS + 4 * st + (lane >> 4)] : 0.0;
        int q = 0;
#pragma unroll
        for (int bi = 0; bi < NB; ++bi)
#pragma unroll
            for (int bj = 0; bj <= bi; ++bj, ++q)
                if (bi < nbm) acc.d[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[bi], av[bj], acc.d[q], 0, 0, 0);
    }
    wave_sync();
    if (mine) {   // clear this chunk's W entries for the next chunk
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            W[(pos + g) * WS + 2 * lml] = 0.0;
            W[(pos + g) * WS + 2 * lml + 1] = 0.0;
        }
    }
    wave_sync();
}

template <int MAXM, bool F32>
__device__ __forceinline__ void fold_children(const MfArgs& a, int s, double* W, FoldBuf* fb, int m, int lane,
                                              FoldAcc<MAXM>& acc) {
    constexpr int WS = 2 * fold_chunk_landmarks(MAXM) + 1;
    static_assert(MAXM * WS <= MAXM * (MAXM + 1) / 2, "W fits the front's LDS triangle");
    static_assert(fold_chunk_landmarks(MAXM) % 2 == 0, "the W W^T steps (4 columns) stay inside W's rows");
#pragma unroll
    for (int q = 0; q < FoldAcc<MAXM>::NP; ++q) acc.d[q] = dbl4{0.0, 0.0, 0.0, 0.0};
    acc.w = 0.0;
    for (int e = lane; e < MAXM * WS; e += 64) W[e] = 0.0;
    const int ch0 = a.fold_cptr[s], ch1 = a.fold_cptr[s + 1];
    int nbad = 0;   // non-positive 2 x 2 pivots of the folded landmarks (head lanes)
    ChunkTable tb;
    tb.load(a, ch0, lane);
    // chunk c: rows [at(c), at(c + 1)); records of a lane past the chunk's rows (or of a chunk past
    // the front's last) are read at a valid index and never used
    auto rec = [&](int c, int n, int4& q0, int4& q1) {
        const int q = tb.at(c) + min(lane, max(n - 1, 0));
        q0 = fold_rec_load(a, q, 0);
        q1 = fold_rec_load(a, q, 1);
    };
    auto len = [&](int c) { return c < ch1 ? tb.at(c + 1) - tb.at(c) : 0; };
    int n = len(ch0);
    int4 r0, r1;
    rec(ch0, n, r0, r1);
    FoldValsT<F32> v = fold_vals<F32>(a, r0, r1, lane < n);
    // next chunk's records, then (inside the loop) its values, both one chunk ahead
    int nn = len(ch0 + 1);
    int4 n0, n1;
    rec(ch0 + 1, nn, n0, n1);
    // Wait for the prologue's loads here: the loop's top then needs no wait on either path (from the
    // back edge, the next chunk's records precede only the last chunk's stores). Left to the
    // compiler, the top waits for every outstanding load and store (vmcnt(0)) because on the entry
    // path the records are the last loads issued.
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    for (int ch = ch0; ch < ch1; ++ch) {
        if (ch + 3 - tb.base > 63) tb.reload(a, ch, lane);   // (uniform; fronts with > 60 chunks only)
        const FoldValsT<F32> cur = v;
        const int4 q1 = r1;
        const int ncur = n;
        // chunk ch + 1: values now (its records arrived during chunk ch - 1), records of ch + 2
        v = fold_vals<F32>(a, n0, n1, lane < nn);
        r0 = n0;
        r1 = n1;
        const int n2 = len(ch + 2);
        rec(ch + 2, n2, n0, n1);
        fold_chunk<MAXM>(a, W, fb, m, lane, acc, cur, q1, ncur, ch == ch0, s, nbad);
        n = nn;
        nn = n2;
    }
    if (nbad) atomicAdd(a.info, nbad);
}

// The front before its assembly: every lower entry of F and of wv set to minus the folded
// landmarks' contribution (each entry once).
template <int MAXM>
__device__ __forceinline__ void fold_store(const FoldAcc<MAXM>& acc, double* F, double* wv, int m, int lane) {
    constexpr int NB = FoldAcc<MAXM>::NB;
    const int nbm = (m + 15) >> 4;
    int q = 0;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int bj = 0; bj <= bi; ++bj, ++q) {
            if (bi < nbm) {
                const int j = 16 * bj + (lane & 15);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int i = 16 * bi + (lane >> 4) + 4 * e;
                    if (i < m && j <= i) F[pk32(i, j, m)] = -acc.d[q][e];
                }
            }
        }
    if (lane < m) wv[lane] = acc.w;
}

// Larger fronts (kMfWaveMaxM < m <= kBlkMaxM: config 2's separators, m ~ 60-100): one 256-thread
// workgroup per front, the whole m x m front in LDS (column-major, leading dimension m, as the plan's
// amap_dst), a blocked right-looking partial Cholesky of its k columns fused with the forward step.
// Per panel of kBlkNb columns: wave 0 factors the panel with its rows in registers (two rows per lane,
// pivots broadcast by v_readlane, no barrier inside the panel) and carries the forward elimination
// along; then all four waves update the trailing lower triangle, A22 -= L21 L21^T, in 16 x 16 tiles
// on f64 MFMA (v_mfma_f64_16x16x4f64, the fold's W W^T pattern). The children's u-vectors are
// extend-added with their update matrices (no separate forward launch). mf_factor_level (with
// mf_forward_level) kept the front in global scratch above 90 rows and took ~140 us per level launch
// at config 2; it remains for m > kBlkMaxM (fallback plans).
#ifndef BOS_MF_BLK_NB   // (A/B builds: the blocked kernel's panel width, a multiple of 4)
#define BOS_MF_BLK_NB 16
#endif
constexpr int kBlkMaxM = kMfBlkMaxM, kBlkNb = BOS_MF_BLK_NB;
static_assert(kBlkNb % 4 == 0 && kBlkNb <= 64, "panel width: MFMA steps of 4 columns, one pair per lane");
constexpr int kBlkTiles = 9;   // 16 x 16 lower tiles per wave: (8 * 9 / 2 = 36 for 128 rows) / 4 waves
// dynamic LDS of a front of m rows: F (m x m), w (kBlkMaxM), the fold's chunk y and landmark count,
// the panel's column broadcast (kBlkNb)
inline int blk_lds_bytes(int m) { return (m * m + kBlkMaxM + 2 * fold_chunk_landmarks(kBlkMaxM) + 2 + 2 * kBlkNb) * 8; }
// children whose update matrices the blocked kernel prefetches (values and front positions, kBlkXU per
// thread: r <= 63), issued before the fold; more (or larger) children take the plain loop
constexpr int kBlkXCh = 2, kBlkXU = 8;

// The folded landmark children of a workgroup front (Schur ordering), the workgroup form of
// fold_children: per chunk (<= kFoldChunk observing poses, <= fold_chunk_landmarks(m) landmarks)
// wave 0's lanes take the chunk's records — the landmarks' 2 x 2 factors, L panels and forward steps,
// the chunk's W (front position x 2 columns per landmark, LDS aliasing F) and y — with the next
// chunk's records and values in flight; then every wave accumulates its 16 x 16 tiles of W W^T on f64
// MFMA (registers, acc[u]: tile wave + 4 u) and each row's thread -W y (wacc). The caller stores
// minus both into the front before its assembly.
template <bool F32>
__device__ __forceinline__ void fold_children_wg(const MfArgs& a, int s, double* W, double* ybuf, int* nlb, int m,
                                                 int tid, dbl4 acc[kBlkTiles], double& wacc) {
    constexpr int cap = fold_chunk_landmarks(kBlkMaxM);
    constexpr int WS = 2 * cap + 1;   // W row stride (odd: no bank conflicts)
    // the wave index as a scalar: branches on it are uniform, so a value loaded on wave 0's path lands in
    // its loop-carried register (a divergent branch merged the paths with copies that waited for the loads)
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int nbt = (m + 15) >> 4, ntiles = nbt * (nbt + 1) / 2;
#pragma unroll
    for (int u = 0; u < kBlkTiles; ++u) acc[u] = dbl4{0.0, 0.0, 0.0, 0.0};
    wacc = 0.0;
    for (int e = tid; e < m * WS; e += kMfBlock) W[e] = 0.0;
    if (tid < 2 * cap) ybuf[tid] = 0.0;
    const int ch0 = a.fold_cptr[s], ch1 = a.fold_cptr[s + 1];
    int nbad = 0;
    ChunkTable tb;
    auto rec = [&](int c, int cnt, int4& q0, int4& q1) {
        const int q = tb.at(c) + min(lane, max(cnt - 1, 0));
        q0 = fold_rec_load(a, q, 0);
        q1 = fold_rec_load(a, q, 1);
    };
    auto len = [&](int c) { return c < ch1 ? tb.at(c + 1) - tb.at(c) : 0; };
    // Wave 0 alone walks the records (the other waves wait at the barrier), so no other wave hides its
    // memory latency: the values are loaded two chunks ahead and the records three, in two register
    // sets that alternate by chunk (the loop is unrolled by two, so a set keeps its registers: a
    // rotation of loop-carried registers made the compiler copy the freshly loaded values at the
    // chunk's end, a copy that waits for the loads).
    struct Set {
        FoldValsT<F32> v;   // values of the chunk this set holds
        int4 m;             // its records' second half (meta)
        int n;              // its rows
        int4 p0, p1;        // records of the chunk that refills the set next
        int np;
    } A, B;
    // (every wave issues the record and value loads, wave 0 alone uses them: loads under a branch on
    // the wave left the registers to be merged with the other waves' path at the branch's end — copies
    // that waited for the loads)
    tb.load(a, ch0, lane);
    {
        int4 q0;
        A.n = len(ch0);
        rec(ch0, A.n, q0, A.m);
        A.v = fold_vals<F32>(a, q0, A.m, lane < A.n);
        B.n = len(ch0 + 1);
        rec(ch0 + 1, B.n, q0, B.m);
        B.v = fold_vals<F32>(a, q0, B.m, lane < B.n);
        A.np = len(ch0 + 2);
        rec(ch0 + 2, A.np, A.p0, A.p1);
    }
    // the prologue's loads waited for here: the loop's top is then reached only from its back edge with
    // loads pending, and waits there for the values of two chunks ago alone (see fold_children)
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    __syncthreads();   // (W cleared)
    // chunk ch from set X; X is refilled with chunk ch + 2's values, Y's records with chunk ch + 3's
#ifdef BOS_MF_BLK_FOLD_CYCLES   // (diagnostics: wave 0's cycles per chunk phase, tools/blk_fold_cycles.py)
    unsigned long long cyc[5] = {0, 0, 0, 0, 0};
    auto now = [&]() {
        unsigned long long t;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
        __builtin_amdgcn_sched_barrier(0);
        return t;
    };
#define BLK_CYC(i, t) cyc[i] += (t)
#else
#define BLK_CYC(i, t)
#endif
    auto chunk = [&](int ch, Set& X, Set& Y) {
        int pos = 0, lml = 0, ncur = 0;
#ifdef BOS_MF_BLK_FOLD_CYCLES
        const unsigned long long c0 = now();
#endif
        if (ch + 4 - tb.base > 63) tb.reload(a, ch, lane);
        FoldVals d = fold_decode(X.v);
        // the decoded values formed here, before the loads into X's registers are issued (left to
        // the compiler, the selects sank to their uses and X.v stayed live past the new loads)
        asm volatile("" : "+v"(d.h[0]), "+v"(d.h[1]), "+v"(d.h[2]), "+v"(d.h[3]), "+v"(d.h[4]), "+v"(d.h[5]),
                     "+v"(d.a00), "+v"(d.a10), "+v"(d.a11), "+v"(d.x0), "+v"(d.x1));
        const int4 q1 = X.m;
        ncur = X.n;
        // the records first, then the values: the memory counter retires in order, so the next
        // chunk's wait for these records must not include these values
        Y.np = len(ch + 3);
        rec(ch + 3, Y.np, Y.p0, Y.p1);
        X.v = fold_vals<F32>(a, X.p0, X.p1, lane < X.np);
        X.m = X.p1;
        X.n = X.np;
        if (wave == 0) {
            const int t = q1.z & 63, rc = (q1.z >> 6) & 63;
            pos = (q1.z >> kFoldPosShift) & kFoldPosMask;
            lml = (q1.z >> kFoldLmShift) & 63;
            const bool mine = lane < ncur;
            // as fold_chunk: every lane issues the same stores (a lane past the chunk's rows holds its
            // last row's record and values: the owners' bits to the owners' addresses)
            double d0 = d.a00;
            const bool bad0 = !(d0 > 0.0);
            d0 = bad0 ? 1e-300 : d0;
            const double i0 = rsqrt_nr(d0), l00 = d0 * i0;
            const double l10 = d.a10 * i0;
            double d1 = d.a11 - l10 * l10;
            const bool bad1 = !(d1 > 0.0);
            d1 = bad1 ? 1e-300 : d1;
            const double i1 = rsqrt_nr(d1), l11 = d1 * i1;
            const double y0 = d.x0 * i0, y1 = (d.x1 - l10 * y0) * i1;
            const int mc = 2 + rc;
            double* Lc = a.L + q1.w;
            const bool head = mine && t == 0;
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                const double lt0 = d.h[2 * g] * i0;
                const double lt1 = (d.h[2 * g + 1] - lt0 * l10) * i1;
                ST_LF(Lc, 2 + t + g, lt0);
                ST_LF(Lc, mc + 2 + t + g, lt1);
                if (mine) {
                    W[(pos + g) * WS + 2 * lml] = lt0;
                    W[(pos + g) * WS + 2 * lml + 1] = lt1;
                }
            }
            ST_LF(Lc, 0, l00);
            ST_LF(Lc, 1, l10);
            ST_LF(Lc, mc + 1, l11);
            a.x[q1.y] = y0;
            a.x[q1.y + 1] = y1;
            nbad += head ? (int)bad0 + (int)bad1 : 0;
            if (head) {
                ybuf[2 * lml] = y0;
                ybuf[2 * lml + 1] = y1;
            }
            const int nl = __builtin_amdgcn_readlane(lml, ncur - 1) + 1;   // landmarks of this chunk
            // the 16-row blocks the chunk's W rows span (its poses are a band of the front's rows):
            // W W^T is zero outside them
            int lo = mine ? pos : 1 << 20, hi = mine ? pos + 2 : -1;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                lo = min(lo, __shfl_xor(lo, o));
                hi = max(hi, __shfl_xor(hi, o));
            }
            if (lane == 0) {
                nlb[0] = nl;
                nlb[1] = lo >> 4;
                nlb[2] = hi >> 4;
            }
        }
#ifdef BOS_MF_BLK_FOLD_CYCLES
        const unsigned long long c1 = now();
#endif
        __syncthreads();
#ifdef BOS_MF_BLK_FOLD_CYCLES
        const unsigned long long c2 = now();
#endif
        const int kc = 2 * nlb[0], blo = nlb[1], bhi = nlb[2];
        // The chunk's W columns past kc are zero (never written in this chunk, cleared after the last)
        // and y is finite there (zeroed before the first chunk), so both loops run over all 2 cap
        // columns with every LDS read issued up front: the same sums in the same order (the extra
        // terms add exact zeros), one LDS latency instead of one per column.
        if (tid < m && (tid >> 4) >= blo && (tid >> 4) <= bhi) {   // u-vector part: -(W y) at this thread's row
            // (in two halves: all 4 cap reads at once held 112 registers at the kernel's peak)
            double wsum = 0.0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                double wr[cap], yr[cap];
#pragma unroll
                for (int q = 0; q < cap; ++q) {
                    wr[q] = W[tid * WS + h * cap + q];
                    yr[q] = ybuf[h * cap + q];
                }
#pragma unroll
                for (int q = 0; q < cap; ++q) wsum += wr[q] * yr[q];
            }
            wacc -= wsum;
        }
        // W W^T, 4 columns per MFMA step: tile (bi, bj) of wave + 4 u; lane l feeds row 16 b + (l & 15),
        // column 4 st + (l >> 4) of W as A (block row bi) and as B (block row bj)
#pragma unroll
        for (int u = 0; u < kBlkTiles; ++u) {
            const int q = wave + 4 * u;
            int bi = 0;
            while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
            const int bj = q - bi * (bi + 1) / 2;
            if (q < ntiles && bi <= bhi && bj >= blo) {   // (uniform) tiles the chunk's W rows reach
                const int ra = min(16 * bi + (lane & 15), m - 1), rb = min(16 * bj + (lane & 15), m - 1);
                const bool oka = 16 * bi + (lane & 15) < m, okb = 16 * bj + (lane & 15) < m;
                double av[cap / 2], bv[cap / 2];
#pragma unroll
                for (int st = 0; st < cap / 2; ++st) {
                    const int cc = 4 * st + (lane >> 4);
                    av[st] = W[ra * WS + cc];
                    bv[st] = W[rb * WS + cc];
                }
#pragma unroll
                for (int st = 0; st < cap / 2; ++st)
                    if (4 * st < kc)   // (uniform)
                        acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(oka ? av[st] : 0.0, okb ? bv[st] : 0.0, acc[u], 0, 0, 0);
            }
        }
#ifdef BOS_MF_BLK_FOLD_CYCLES
        const unsigned long long c3 = now();
#endif
        __syncthreads();
#ifdef BOS_MF_BLK_FOLD_CYCLES
        const unsigned long long c4 = now();
        BLK_CYC(0, c1 - c0); BLK_CYC(1, c2 - c1); BLK_CYC(2, c3 - c2); BLK_CYC(3, c4 - c3); BLK_CYC(4, 1);
#endif
        if (wave == 0 && lane < ncur) {   // clear this chunk's W entries (wave 0 writes the next chunk's after)
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                W[(pos + g) * WS + 2 * lml] = 0.0;
                W[(pos + g) * WS + 2 * lml + 1] = 0.0;
            }
        }
    };
    for (int ch = ch0; ch < ch1; ch += 2) {   // (uniform over the workgroup)
        chunk(ch, A, B);
        if (ch + 1 >= ch1) break;   // (a break: the loop's back edge always follows chunk ch + 1)
        chunk(ch + 1, B, A);
    }
#ifdef BOS_MF_BLK_FOLD_CYCLES
    if (tid == 0 && g_pivot_bwd)
        for (int i = 0; i < 5; ++i) g_pivot_bwd[8 * (int64_t)s + i] = cyc[i];
#endif
#undef BLK_CYC
    if (wave == 0 && nbad) atomicAdd(a.info, nbad);
}

template <bool F32>
__device__ __forceinline__ void factor_front_blk(const MfArgs& a, const int s, double* lds) {
    const int k = a.k[s], r = a.r[s], m = k + r;   // m <= kBlkMaxM (mf_create / the launch check it)
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    // LDS: the small buffers first (fixed, 16-byte aligned offsets), then the front
    double* colbuf = lds;                                             // panel pair broadcast (kBlkNb pairs)
    double* ybuf = colbuf + 2 * kBlkNb;                               // the fold's y of one chunk
    int* nlb = reinterpret_cast<int*>(ybuf + 2 * fold_chunk_landmarks(kBlkMaxM));   // chunk: landmarks, row blocks
    double* w = ybuf + 2 * fold_chunk_landmarks(kBlkMaxM) + 2;        // right-hand side, then the forward results
    double* F = w + kBlkMaxM;                                         // m x m, column-major
    static_assert((2 * kBlkNb + 2 * fold_chunk_landmarks(kBlkMaxM) + 2 + kBlkMaxM) % 2 == 0, "F 16-byte aligned");
    const int c0 = a.col0[s];
    const int nfold = a.fold_cnt[s];
    // the non-folded children (pose separators, typically 2): their update matrices and u-vectors,
    // with their positions in this front (emap), loaded now and in flight during the fold
    const int cb = a.child_ptr[s] + nfold, ce = a.child_ptr[s + 1];
    const int nx = min(ce - cb, kBlkXCh);
    double xv[kBlkXCh][kBlkXU], xuv[kBlkXCh];
    int xp[kBlkXCh][kBlkXU], xum[kBlkXCh], xne[kBlkXCh];
#pragma unroll
    for (int i = 0; i < kBlkXCh; ++i) {
        xne[i] = 0;
        if (i < nx) {   // uniform
            const int c = a.child[cb + i];
            const int rc = a.r[c], ne = rc * (rc + 1) / 2;
            xne[i] = ne;
            const double* Uc = a.U + a.U_off[c];
            const int16_t* ec = a.emap + a.emap_off[c];
#pragma unroll
            for (int u = 0; u < kBlkXU; ++u) {
                const int e = min(tid + kMfBlock * u, ne - 1);   // clamped (see assemble_wave)
                xv[i][u] = Uc[e];
                xp[i][u] = ec[e];
            }
            const int t = min(tid, rc - 1);
            xuv[i] = a.u[a.u_off[c] + t];
            xum[i] = tid < rc ? a.rmap[a.rmap_off[c] + t] : -1;
        }
    }
    // diagnostics (bos_debug_solver_stamps): the per-front phases of tools/solver_stamps.py
    auto stamp = [&](int q) {
        if (a.stamps_f && tid == 0) a.stamps_f[8 * (int64_t)s + q] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    double wacc = 0.0;
    if (nfold > 0) {
        // the folded landmarks first (their W uses F's LDS); F and w then start from minus their
        // contribution, each lower entry written once by the wave holding its tile
        dbl4 acc[kBlkTiles];
        fold_children_wg<F32>(a, s, F, ybuf, nlb, m, tid, acc, wacc);
        for (int e = tid; e < m * m; e += kMfBlock) F[e] = 0.0;
        __syncthreads();
        const int nbt = (m + 15) >> 4, ntiles = nbt * (nbt + 1) / 2;
#pragma unroll
        for (int u = 0; u < kBlkTiles; ++u) {
            const int q = wave + 4 * u;
            if (q < ntiles) {
                int bi = 0;
                while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
                const int bj = q - bi * (bi + 1) / 2;
                const int j = 16 * bj + (lane & 15);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int i = 16 * bi + (lane >> 4) + 4 * e;
                    if (i < m && j <= i) F[i + j * m] = -acc[u][e];
                }
            }
        }
    } else {
        for (int e = tid; e < m * m; e += kMfBlock) F[e] = 0.0;
    }
    if (tid < m) w[tid] = (tid < k ? a.x[c0 + tid] : 0.0) + wacc;   // (m <= kBlkMaxM < kMfBlock)
    __syncthreads();
    stamp(1);
    for (int q = a.amap_ptr[s] + tid; q < a.amap_ptr[s + 1]; q += kMfBlock) F[a.amap_dst[q]] += a.A[a.amap_src[q]];
    __syncthreads();
    stamp(2);
    stamp(3);
    // the other children one at a time (deterministic): update matrix into F, u-vector into w
#pragma unroll
    for (int i = 0; i < kBlkXCh; ++i) {
        if (i < nx) {   // uniform
#pragma unroll
            for (int u = 0; u < kBlkXU; ++u)
                if (tid + kMfBlock * u < xne[i]) F[xp[i][u]] += xv[i][u];
            if (xum[i] >= 0) w[xum[i]] += xuv[i];
            if (xne[i] > kMfBlock * kBlkXU) {   // entries past the prefetched ones (r > 63)
                const int c = a.child[cb + i];
                const double* Uc = a.U + a.U_off[c];
                const int16_t* ec = a.emap + a.emap_off[c];
                for (int e = kMfBlock * kBlkXU + tid; e < xne[i]; e += kMfBlock) F[ec[e]] += Uc[e];
            }
            __syncthreads();
        }
    }
    for (int ci = cb + nx; ci < ce; ++ci) {
        const int c = a.child[ci];
        const int rc = a.r[c];
        const int32_t* map = a.rmap + a.rmap_off[c];
        const double* Uc = a.U + a.U_off[c];
        for (int j = wave; j < rc; j += kMfBlock / 64) {
            const int pj = map[j] * m;
            const double* uj = Uc + pk(j, j, rc) - j;
            for (int i = j + lane; i < rc; i += 64) F[map[i] + pj] += uj[i];
        }
        const double* uc = a.u + a.u_off[c];
        for (int t = tid; t < rc; t += kMfBlock) w[map[t]] += uc[t];
        __syncthreads();
    }
    stamp(4);
    double* Ls = a.L + a.L_off[s];
    int nbad = 0;
    for (int p0 = 0; p0 < k; p0 += kBlkNb) {
        const int nb = min(kBlkNb, k - p0);
        if (wave == 0) {
            // lane l holds rows p0 + l and p0 + 64 + l of the panel's columns (m - p0 <= 128 rows); the
            // reads are clamped to valid positions (one wait for all), the values past the front zero.
            // Columns past nb hold copies of column nb - 1: updated like the others, never a pivot,
            // never stored.
            const int ia = p0 + lane, ib = p0 + 64 + lane;
            const bool va = ia < m, vb = ib < m;
            const int ra = min(ia, m - 1), rb = min(ib, m - 1);
            double pa[kBlkNb], pb[kBlkNb];
#pragma unroll
            for (int c = 0; c < kBlkNb; ++c) {
                const int cc = p0 + min(c, nb - 1);
                pa[c] = F[ra + cc * m];
                pb[c] = F[rb + cc * m];
            }
            asm volatile("" : "+v"(pa[0]), "+v"(pb[0]));
#pragma unroll
            for (int c = 0; c < kBlkNb; ++c) {
                pa[c] = va ? pa[c] : 0.0;
                pb[c] = vb ? pb[c] : 0.0;
            }
            double wa = va ? w[ia] : 0.0, wb = vb ? w[ib] : 0.0;
            // two pivots per step (as factor_front_reg): column j + 1 brought up to date in registers,
            // both columns' panel rows through ONE LDS broadcast as pairs, then a rank-2 update
#pragma unroll
            for (int j = 0; j < kBlkNb; j += 2) {
                if (j + 1 < nb) {   // uniform
                    double d0 = readlane_d(pa[j], j);
                    const bool bad0 = !(d0 > 0.0);
                    nbad += bad0;
                    d0 = bad0 ? 1e-300 : d0;
                    const double inv0 = rsqrt_nr(d0), l00 = d0 * inv0;
                    const double la0 = lane < j ? 0.0 : lane == j ? l00 : pa[j] * inv0;   // L[i, p0 + j]
                    const double lb0 = pb[j] * inv0;
                    const double lj1 = readlane_d(la0, j + 1);                           // L[p0 + j + 1, p0 + j]
                    const double fa = fma(-la0, lj1, pa[j + 1]), fb = fma(-lb0, lj1, pb[j + 1]);
                    double d1 = readlane_d(fa, j + 1);
                    const bool bad1 = !(d1 > 0.0);
                    nbad += bad1;
                    d1 = bad1 ? 1e-300 : d1;
                    const double inv1 = rsqrt_nr(d1), l11 = d1 * inv1;
                    const double la1 = lane < j + 1 ? 0.0 : lane == j + 1 ? l11 : fa * inv1;
                    const double lb1 = fb * inv1;
                    pa[j] = la0;
                    pb[j] = lb0;
                    pa[j + 1] = la1;
                    pb[j + 1] = lb1;
                    if (lane < kBlkNb) reinterpret_cast<double2*>(colbuf)[lane] = make_double2(la0, la1);
                    const double y0 = readlane_d(wa, j) * inv0;   // forward steps
                    wa = lane == j ? y0 : lane > j ? fma(-la0, y0, wa) : wa;
                    wb = fma(-lb0, y0, wb);
                    const double y1 = readlane_d(wa, j + 1) * inv1;
                    wa = lane == j + 1 ? y1 : lane > j + 1 ? fma(-la1, y1, wa) : wa;
                    wb = fma(-lb1, y1, wb);
                    wave_sync();
                    double2 cbv[kBlkNb];
#pragma unroll
                    for (int c = j + 2; c < kBlkNb; ++c) cbv[c] = reinterpret_cast<const double2*>(colbuf)[c];
#pragma unroll
                    for (int c = j + 2; c < kBlkNb; ++c) {
                        pa[c] = fma(-la1, cbv[c].y, fma(-la0, cbv[c].x, pa[c]));
                        pb[c] = fma(-lb1, cbv[c].y, fma(-lb0, cbv[c].x, pb[c]));
                    }
                    __builtin_amdgcn_wave_barrier();   // the next step's broadcast stays after these reads
                } else if (j < nb) {   // the panel's last column (odd nb): nothing left to update
                    double d = readlane_d(pa[j], j);
                    const bool bad = !(d > 0.0);
                    nbad += bad;
                    d = bad ? 1e-300 : d;
                    const double inv = rsqrt_nr(d), ljj = d * inv;
                    const double la = lane < j ? 0.0 : lane == j ? ljj : pa[j] * inv;
                    const double lb = pb[j] * inv;
                    pa[j] = la;
                    pb[j] = lb;
                    const double y = readlane_d(wa, j) * inv;
                    wa = lane == j ? y : lane > j ? fma(-la, y, wa) : wa;
                    wb = fma(-lb, y, wb);
                }
            }
#pragma unroll
            for (int c = 0; c < kBlkNb; ++c) {
                if (c < nb) {
                    if (va) {
                        F[ia + (p0 + c) * m] = pa[c];
                        ST_L(Ls, ia + (p0 + c) * m, pa[c]);
                    }
                    if (vb) {
                        F[ib + (p0 + c) * m] = pb[c];
                        ST_L(Ls, ib + (p0 + c) * m, pb[c]);
                    }
                }
            }
            if (va) w[ia] = wa;
            if (vb) w[ib] = wb;
        }
        __syncthreads();
        // trailing lower triangle, rows / columns [t0, m): 16 x 16 tiles (bi >= bj) over the waves
        const int t0 = p0 + nb, nbt = (m - t0 + 15) >> 4, ntiles = nbt * (nbt + 1) / 2;
        for (int q = wave; q < ntiles; q += kMfBlock / 64) {
            int bi = 0;
            while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
            const int bj = q - bi * (bi + 1) / 2;
            const int ra = t0 + 16 * bi + (lane & 15), rb = t0 + 16 * bj + (lane & 15);
            dbl4 acc = {0.0, 0.0, 0.0, 0.0};
            // every operand read issued up front (clamped positions, masked values), then the MFMAs
            double av[kBlkNb / 4], bv[kBlkNb / 4];
#pragma unroll
            for (int st = 0; st < kBlkNb / 4; ++st) {
                const int cc = min(4 * st + (lane >> 4), nb - 1);
                av[st] = F[min(ra, m - 1) + (p0 + cc) * m];
                bv[st] = F[min(rb, m - 1) + (p0 + cc) * m];
            }
#pragma unroll
            for (int st = 0; st < kBlkNb / 4; ++st) {
                if (4 * st < nb) {   // (uniform)
                    const bool okc = 4 * st + (lane >> 4) < nb;
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(okc && ra < m ? av[st] : 0.0, okc && rb < m ? bv[st] : 0.0,
                                                               acc, 0, 0, 0);
                }
            }
            const int col = t0 + 16 * bj + (lane & 15);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = t0 + 16 * bi + (lane >> 4) + 4 * e;
                if (row < m && row >= col) F[row + col * m] -= acc[e];
            }
        }
        __syncthreads();
    }
    stamp(5);
    if (tid == 0 && nbad) atomicAdd(a.info, nbad);
    // the update matrix (packed lower r x r), the forward results: own dofs to x, the rest to u
    double* Us = a.U + a.U_off[s];
    for (int j = wave; j < r; j += kMfBlock / 64) {
        double* uj = Us + pk(j, j, r) - j;
        const double* fj = F + (k + (k + j) * m);
        for (int i = j + lane; i < r; i += 64) uj[i] = fj[i];
    }
    for (int i = tid; i < m; i += kMfBlock) {
        if (i < k) a.x[c0 + i] = w[i];
        else a.u[a.u_off[s] + (i - k)] = w[i];
    }
    stamp(6);
}

template <bool F32>
__global__ __launch_bounds__(kMfBlock) void mf_factor_blk(const MfArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    factor_front_blk<F32>(a, a.level[blockIdx.x], lds);
}

// ---- dataflow (work-queue) kernels: one launch walks a whole tree range. A wavefront takes the
// next front from an atomic ticket (fronts listed in topological order), prepares what does not
// depend on other fronts (the fold and the assembly of H), waits for the fronts it depends on
// (children bottom-up, the parent top-down) by polling their tagged hand-off data (tag_pair /
// untag_pair: the data is the flag), processes the front and writes its own hand-off data tagged.
// A wave only ever waits for tickets already taken by running waves, so any grid size is
// deadlock-free. Every wait is bounded in time: a dependency that has not arrived within 50 ms marks
// the launch stalled (kStall in info), and from then on every wait of every wave returns at once, so
// a stalled launch drains in about one timeout and is reported as an error (bos_step returns
// BOS_ERR_SOLVER and the box-plus is skipped), never a hang.
// The ticket is reset by the launch itself: the last wave to leave zeroes it (and its exit
// counter), so no host-side reset is needed between launches and no error path can leave a
// partly consumed ticket behind (a launch that never started never took one).
struct Flow {
    const int32_t* order;   // fronts in processing order
    int n;
    int* ticket;            // zero at launch; zeroed again by the launch's last wave
    int* exits;             // waves that have left the launch (same life cycle)
    const uint32_t* epoch_src;   // device word: this step's epoch (bumped once per GN step by the
                                 // step_mark kernel before the first flow launch, mf_epoch_ptr)
    uint32_t epoch;              // *epoch_src, read by the launch itself (graph-replayable)
    const int8_t* fid;      // per supernode: the flow launch (id) that processes it, 0 = none; a front
                            // waits only for fronts of its own launch (the others finished earlier:
                            // per-level launches, the other program, or another rank's exchange)
    int id;
    unsigned long long* stamps;   // diagnostics (bos_debug_solver_stamps): 8 realtime stamps per front, or null
};

// Front-processing modes: per-level launch (no waits), dataflow launch (flags in global memory,
// coherent hand-off). (A third, the tree's top as one workgroup with flags in LDS, measured slower
// than the flows: DESIGN.md §4.)
constexpr int kModeLevel = 0, kModeFlow = 1;

constexpr int kStall = kMfStall;               // or-ed into info when a dependency wait times out
constexpr uint64_t kWaitTicks = 5000000;        // 50 ms of the 100 MHz realtime clock

__device__ __forceinline__ int next_ticket(int* ticket) {
    int t = 0;
    if (threadIdx.x == 0) t = atomicAdd(ticket, 1);
    return __builtin_amdgcn_readfirstlane(t);
}

// Memory ordering of the in-launch hand-off (the form cdna_hip_programming.md §6 Guideline 16 and
// MI355X_MICROARCH.md § visibility allow without an agent-scope acquire; gfx950 has 8 XCDs with
// private L2s and per-CU L1s that other CUs' stores never refresh): every handed-off double (update
// matrices and u-vectors of a child in the same flow, x of a backward front whose children wait for
// it) is written as a tagged pair by relaxed agent-scope atomic stores (global_store ... sc1,
// write-through to the memory-side coherence point) and read by relaxed agent-scope atomic loads
// (global_load ... sc1, which bypass the CU's L1 and the XCD's L2 copy); a consumer accepts a value
// only when both of its halves carry this step's epoch, so it can never take a stale or torn value,
// and no drain, flag or fence is needed on either side. Data from earlier launches (kernel boundary)
// is read with plain loads. Checked in the disassembly: the granule loads and stores are
// global_load/store_dwordx2 sc1, no flat_ access, no scalar load of handed-off data.
// Called by every wave once it has taken its last ticket.
__device__ __forceinline__ void leave_flow(const Flow& f) {
    if (threadIdx.x == 0 && atomicAdd(f.exits, 1) == (int)gridDim.x - 1) {
        __hip_atomic_store(f.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(f.exits, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// A child's extend-add inputs: its r, row map entry (lane < rc) and where its update matrix and
// u-vector live, and the parent-front positions of the first 256 entries of its packed update
// matrix (4 per lane) — static structure, loaded before the child has finished — then its values:
// the u-vector entry and those 256 entries.
struct ChildPre {
    int rc, smap_v;
    double uval;
    double v[4];
    int pos[4];
    const double* Uc;
    const double* uc;
    const int16_t* ec;
    const unsigned long long* G;    // tagged update matrix + u-vector (a child in the same flow), or null
};

// (Every structure and value array is padded by kMfPad elements, so the clamped reads below stay in
// bounds even for an empty child range; see up().)
__device__ __forceinline__ void child_meta(const MfArgs& a, int c, int lane, ChildPre& p) {
    const int rc = a.r[c];   // rc < m <= MAXM
    const int roff = a.rmap_off[c];
    p.rc = rc;
    p.Uc = a.U + a.U_off[c];
    p.uc = a.u + a.u_off[c];
    p.ec = a.emap + a.emap_off[c];
    const int64_t go = a.ug_off[c];
    p.G = go >= 0 ? a.Ug + go : nullptr;
    const int sv = a.rmap[roff + min(lane, max(rc - 1, 0))];
    p.smap_v = lane < rc ? sv : 0;
    const int ne = rc * (rc + 1) / 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = 64 * u + lane;
        const int pv = p.ec[min(e, max(ne - 1, 0))];
        p.pos[u] = e < ne ? pv : 0;
    }
}

template <bool COH>
__device__ __forceinline__ void child_vals(int lane, ChildPre& p) {
    const int rc = p.rc;
    const double uv = ldc<COH>(p.uc + min(lane, max(rc - 1, 0)));
    p.uval = lane < rc ? uv : 0.0;
    const int ne = rc * (rc + 1) / 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = 64 * u + lane;
        const double v = ldc<COH>(p.Uc + min(e, max(ne - 1, 0)));
        p.v[u] = e < ne ? v : 0.0;
    }
}

// A child of the same flow (p.G): poll its tagged update matrix and u-vector until every granule
// carries this step's epoch (the data is the flag: no completion flag, no second load round trip),
// keeping the u-vector entry and the first 256 entries. Bounded (kWaitTicks): a stall marks info
// and returns (the launch then drains, the step fails).
// Waiting is done by ONE lane probing ONE granule (the child's last u-vector entry, its last store),
// the full sweep follows once it matches: a wave sweeping all its granules on every poll multiplied
// the polling traffic by ~600 loads per poll.
__device__ __forceinline__ bool probe_granule(const unsigned long long* g, uint32_t epoch, uint64_t t0, int32_t* info) {
    if (threadIdx.x % 64 == 0) {
        for (uint32_t it = 0;; ++it) {
            if ((uint32_t)(__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) == epoch) break;
            if ((it & 15) == 15) {
                const bool stalled = (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kMfStall) != 0;
                if (stalled || __builtin_amdgcn_s_memrealtime() - t0 > kWaitTicks) break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __builtin_amdgcn_wave_barrier();
    return true;
}

__device__ __forceinline__ void child_sweep(ChildPre& p, uint32_t epoch, int lane, int32_t* info) {
    const int rc = p.rc, ne = rc * (rc + 1) / 2;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    probe_granule(p.G + 2 * (int64_t)(ne + max(rc - 1, 0)) + 1, epoch, t0, info);
    for (uint32_t it = 0;; ++it) {
        bool ok = true;
        const double uv = untag_pair(p.G + 2 * (int64_t)(ne + min(lane, max(rc - 1, 0))), epoch, ok);
        p.uval = lane < rc ? uv : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = 64 * u + lane;
            const double v = untag_pair(p.G + 2 * (int64_t)min(e, max(ne - 1, 0)), epoch, ok);
            p.v[u] = e < ne ? v : 0.0;
        }
        for (int e0 = 256; e0 < ne; e0 += 256)   // later entries: checked here, read in extend_child
#pragma unroll
            for (int u = 0; u < 4; ++u) (void)untag_pair(p.G + 2 * (int64_t)min(e0 + 64 * u + lane, ne - 1), epoch, ok);
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) return;
        if ((it & 15) == 15) {
            const bool stalled = (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kMfStall) != 0;
            if (stalled || __builtin_amdgcn_s_memrealtime() - t0 > kWaitTicks) {
                if (lane == 0) atomicOr(info, kMfStall);
                return;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Extend-add of one child: every entry of its packed update matrix added at its precomputed position
// in the parent's packed front (positions of one child are distinct), then its u-vector.
template <bool COH>
__device__ __forceinline__ void extend_child(const MfArgs& a, const ChildPre& p, double* F, double* wv, int m, int lane,
                                             uint32_t epoch = 0) {
    const int rc = p.rc;
    const int ne = rc * (rc + 1) / 2;
    for (int e0 = 0; e0 < ne; e0 += 256) {
        double v[4];
        int pos[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = min(e0 + 64 * u + lane, ne - 1);   // clamped (see assemble_wave)
            bool ok = true;   // (tagged: child_sweep has seen every tag current)
            v[u] = e0 == 0 ? p.v[u] : p.G ? untag_pair(p.G + 2 * (int64_t)e, epoch, ok) : ldc<COH>(p.Uc + e);
            pos[u] = e0 == 0 ? p.pos[u] : p.ec[e];
        }
        // the four front entries read at once (positions of one child are distinct; a lane past the
        // child's entries reads a valid position and writes nothing), then added and written back: a
        // read-modify-write per entry under its own branch waited for each read separately
        double f[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) f[u] = F[pos[u]];
        asm volatile("" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (e0 + 64 * u + lane < ne) F[pos[u]] = f[u] + v[u];
    }
    if (lane < rc) wv[p.smap_v] += p.uval;
    wave_sync();
}

// Factorization of one front fused with its forward elimination: w (LDS, m doubles) receives the
// front's right-hand side (x of its own dofs) plus the children's u-vectors, extend-added with
// their update matrices; after the partial Cholesky, lane i eliminates with its row of L (still in
// registers): y_j = w_j / L_jj, w_i -= L_ij y_j. y goes to x, the remaining w (rows >= k) to the
// front's u-vector for its parent.
template <int MAXM, int MODE, bool F32>
__device__ __forceinline__ void factor_front_reg(const MfArgs& a, int s, double* F, double* colbuf,
                                                 double* wv, FoldBuf* fb, int lane, const Flow* f) {
    constexpr bool COH = MODE == kModeFlow;
    const int k = a.k[s], r = a.r[s], m = k + r;
    const int nfold = a.fold_cnt[s];
    const int c0 = a.col0[s];
    const int aq0 = a.amap_ptr[s], aq1 = a.amap_ptr[s + 1];   // the assembly's range, loaded up front
    const int np = m * (m + 1) / 2;
    double xo = a.x[c0 + min(lane, k - 1)];   // right-hand side of the own dofs (k < 64; unconditional read)
    // output offsets up front: their loads complete during the assembly instead of before the pivots
    double* Ls = a.L + a.L_off[s];
    double* Us = a.U + a.U_off[s];
    double* us = a.u + a.u_off[s];
    // The first two (non-folded) children's structure is loaded up front, in flight during the
    // assembly and the fold. Everything up to the extend-add depends on H only, so the flow kernel
    // waits for the children after it: on the critical path a front's assembly and fold overlap
    // its children's work.
    const int cb = a.child_ptr[s] + nfold, ce = a.child_ptr[s + 1];
    ChildPre p0, p1;
    if (cb < ce) child_meta(a, a.child[cb], lane, p0);
    if (cb + 1 < ce) child_meta(a, a.child[cb + 1], lane, p1);
    // the folded landmarks first (their W uses F's LDS): F and the u-vector accumulator wv start
    // from minus their contribution, the assembly then adds H
    const bool fold = nfold > 0;
    unsigned long long* const stp = f ? f->stamps : a.stamps_f;
    fstamp(stp, s, 0);
    if (fold) {
        FoldAcc<MAXM> facc;
        fold_children<MAXM, F32>(a, s, F, fb, m, lane, facc);
        wave_sync();
        fold_store<MAXM>(facc, F, wv, m, lane);
    } else {
        for (int e = lane; e < np; e += 64) F[e] = 0.0;
        for (int i = lane; i < m; i += 64) wv[i] = 0.0;    // children's u-vectors accumulate here
    }
    wave_sync();
    fstamp(stp, s, 1);
    assemble_wave(a, aq0, aq1, F, lane, fold);
    wave_sync();
    // the own right-hand side has arrived by now (the assembly waited for its loads): pin it here,
    // so that the compiler does not leave its wait (one memory latency) in front of the pivots
    asm volatile("" : "+v"(xo));
    xo = lane < k ? xo : 0.0;
    fstamp(stp, s, 2);
    // children of this flow hand over tagged granules (child_sweep polls the data itself); children of
    // earlier launches are final (kernel boundary): plain reads
    uint32_t ep = 0;
    if constexpr (MODE == kModeFlow) ep = f->epoch;
    fstamp(stp, s, 3);
#ifdef BOS_MF_PIVOT_CYCLES
    unsigned long long* const cst = stp ? g_pivot_bwd : nullptr;
    cstamp(cst, s, 1);
#endif
    // extend-add, children in list order (deterministic)
    if (cb < ce) {
        if (MODE == kModeFlow && p0.G) child_sweep(p0, ep, lane, a.info);
        else child_vals<COH>(lane, p0);
    }
    if (cb + 1 < ce) {
        if (MODE == kModeFlow && p1.G) child_sweep(p1, ep, lane, a.info);
        else child_vals<COH>(lane, p1);
    }
#ifdef BOS_MF_PIVOT_CYCLES
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the children's values have arrived
    cstamp(cst, s, 2);
#endif
    if (cb < ce) extend_child<COH>(a, p0, F, wv, m, lane, ep);
    if (cb + 1 < ce) extend_child<COH>(a, p1, F, wv, m, lane, ep);
    for (int ci = cb + 2; ci < ce; ++ci) {
        ChildPre pq;
        child_meta(a, a.child[ci], lane, pq);
        if (MODE == kModeFlow && pq.G) child_sweep(pq, ep, lane, a.info);
        else child_vals<COH>(lane, pq);
        extend_child<COH>(a, pq, F, wv, m, lane, ep);
    }
#ifdef BOS_MF_PIVOT_CYCLES
    cstamp(cst, s, 3);
#endif
    const bool live = lane < m;
    const int lrow = min(lane, m - 1);
    double row[MAXM];
#if defined(BOS_MF_PIVOT_CYCLES) && defined(BOS_MF_ROWS_STAMPS)
    cstamp(cst, s, 5);   // (diagnostic: slots 5 / 6 split the row loads instead of timing pivot steps)
#endif
#pragma unroll
    for (int c0 = 0; c0 < MAXM; c0 += 8) {   // whole groups of 8 past m skipped by a scalar branch
#if defined(BOS_MF_PIVOT_CYCLES) && defined(BOS_MF_ROWS_STAMPS)
        if (c0 == 8) cstamp(cst, s, 6);
#endif
        if (c0 < m) {
            // branch-free: every lane reads a position of the LDS front (the column clamped to m - 1:
            // for a row i < m and a column c' < m, 0 <= pk32(i, c', m) < np, also above the diagonal;
            // unclamped, m <= 3 would give negative positions), the group's eight reads
            // under one wait. A predicated read per
            // entry compiled to an exec-mask branch with its own wait each (~2 500 cycles for the rows
            // of a 24-row front); the empty asm keeps the reads out of such branches. Entries above
            // the diagonal, of rows >= m (copies of row m - 1) and of columns >= m are scratch that no
            // stored or broadcast value ever reads, so they are taken as read: selecting zeros there
            // held 48 loop-invariant lane masks that the compiler spilled to VGPR lanes and read back
            // per column. (All columns read at once, without the groups' waits and zero fills: rows
            // 1 500 -> 1 260 cycles at the top, 3 430 -> 2 830 at level 0, solve unchanged,
            // profiles/r05_rows_all_at_once_ab.txt.)
            double v[8];
#pragma unroll
            for (int c = c0; c < c0 + 8; ++c) v[c - c0] = c < MAXM ? F[pk32(lrow, min(c, m - 1), m)] : 0.0;
            asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                         "+v"(v[7]));
#pragma unroll
            for (int c = c0; c < c0 + 8 && c < MAXM; ++c) row[c] = v[c - c0];
        } else {
#pragma unroll
            for (int c = c0; c < c0 + 8 && c < MAXM; ++c) row[c] = 0.0;
        }
    }
    fstamp(stp, s, 4);
    double wi = live ? wv[lane] + xo : 0.0;   // forward elimination, fused into the pivot loop
    // Right-looking, with a rotating register window: before step j, row[t] holds column j + t of
    // this lane's row, so the pivot column is always row[0] and the update of column j + 1 + t is
    // written to row[t] (the shift costs nothing). The pivot loop is a real loop — one copy of its
    // body instead of MAXM unrolled ones keeps the kernel inside the instruction cache. Column j
    // (rows > j) is broadcast through a double-buffered LDS column indexed by t; entries above the
    // diagonal, rows >= m and columns >= m are scratch, so the updates need no predicates.
    const int kf = k;
    int nbad = 0;   // non-positive pivots (uniform), reported once per front
    double* Lj = Ls + lane;
    int j = 0;
#ifdef BOS_MF_PIVOT_CYCLES
    cstamp(cst, s, 0);
#endif
    // Two pivots per step: column j + 1 is brought up to date in registers (L(j+1, j) by readlane),
    // both columns go through ONE LDS broadcast as pairs, and the trailing columns take a rank-2
    // update; the window rotates by two.
    {
#pragma nounroll
        for (; j + 1 < kf; j += 2) {
            double d0 = readlane_d(row[0], j);
            const bool bad0 = !(d0 > 0.0);
            nbad += bad0;
            d0 = bad0 ? 1e-300 : d0;
            const double inv0 = rsqrt_nr(d0), l00 = d0 * inv0;
            const double l0 = lane == j ? l00 : row[0] * inv0;   // L[i, j]
            const double lj1 = readlane_d(l0, j + 1);            // L[j+1, j]
            const double f1 = fma(-l0, lj1, row[1]);             // column j+1 after pivot j
            double d1 = readlane_d(f1, j + 1);
            const bool bad1 = !(d1 > 0.0);
            nbad += bad1;
            d1 = bad1 ? 1e-300 : d1;
            const double inv1 = rsqrt_nr(d1), l11 = d1 * inv1;
            const double l1 = lane == j + 1 ? l11 : f1 * inv1;   // L[i, j+1]
            double2* cp = reinterpret_cast<double2*>(colbuf);   // (L[l, j], L[l, j+1]), l = j + 2 + t
            if (lane > j + 1 && lane < m) cp[lane - j - 2] = make_double2(l0, l1);
            if (live) {
                if (lane >= j) ST_L(Lj, 0, l0);
                if (lane >= j + 1) ST_L(Lj, m, l1);
            }
            Lj += 2 * m;
            const double y0 = readlane_d(wi, j) * inv0;          // forward steps j, j + 1
            if (lane == j) wi = y0;
            else if (lane > j) wi -= l0 * y0;
            const double y1 = readlane_d(wi, j + 1) * inv1;
            if (lane == j + 1) wi = y1;
            else if (lane > j + 1) wi -= l1 * y1;
            wave_sync();
            const int nt = m - j - 2;                            // live columns after this step
#pragma unroll
            for (int t0 = 0; t0 < MAXM - 2; t0 += 8) {
                if (t0 < nt) {
                    // the group's eight pairs read at once (one LDS latency per group; pairs past the
                    // live columns are scratch), the empty asm keeps the compiler from interleaving a
                    // wait per pair: two-pivot step 1 269 -> 1 037 cycles at m = 18, 1 818 -> 1 554 at
                    // m = 42 (tools/pivot_probe2.hip, profiles/r05_pivot_step_anatomy.txt)
                    double2 c[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) c[u] = t0 + u < MAXM - 2 ? cp[t0 + u] : make_double2(0.0, 0.0);
#pragma unroll
                    for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(c[u].x), "+v"(c[u].y));
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (t0 + u < MAXM - 2) row[t0 + u] = fma(-l1, c[u].y, fma(-l0, c[u].x, row[t0 + u + 2]));
                }
            }
            __builtin_amdgcn_wave_barrier();   // the next step's pair stores stay after these reads
#ifdef BOS_MF_PIVOT_CYCLES
#ifdef BOS_MF_ROWS_STAMPS
            if (j / 2 < 1) cstamp(cst, s, 4 + j / 2);
#else
            if (j / 2 < 3) cstamp(cst, s, 4 + j / 2);
#endif
#endif
        }
    }
#pragma nounroll
    for (; j < kf; ++j) {
        double* col = colbuf + (j & 1) * MAXM;
        if (lane > j && lane < m) col[lane - j - 1] = row[0];
        // the pivot straight from lane j's register (no LDS round trip on the critical path; the
        // column's LDS broadcast lands meanwhile), 1 / sqrt(d) by v_rsq_f64 + two Newton steps
        double d = readlane_d(row[0], j);
        wave_sync();
        // the first 8 column entries are read before the pivot arithmetic (no branch between), so
        // their LDS latency overlaps it
        double c0v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c0v[u] = u < MAXM ? col[u] : 0.0;
        const bool bad = !(d > 0.0);
        nbad += bad;
        d = bad ? 1e-300 : d;
        const double inv = rsqrt_nr(d), ljj = d * inv;
        const double lij = lane == j ? ljj : row[0] * inv;   // L[i, j]
        if (live && lane >= j) ST_L(Lj, 0, lij);
        Lj += m;
        // forward step: y_j = w_j / L_jj, w_i -= L_ij y_j
        const double yj = readlane_d(wi, j) * inv;
        if (lane == j) wi = yj;
        else if (lane > j) wi -= lij * yj;
        const double g = lij * inv;                          // L[i, j] / L[j, j]
        const int nt = m - j - 1;                            // live columns after this step (uniform)

#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (u < MAXM - 1) row[u] = fma(-g, c0v[u], row[u + 1]);   // -= L[i,j] L[l,j], l = j + 1 + t
#pragma unroll
        for (int t0 = 8; t0 < MAXM - 1; t0 += 8) {
            if (t0 < nt) {
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int t = t0 + u;
                    if (t < MAXM - 1) row[t] = fma(-g, col[t], row[t + 1]);
                }
            }
        }
    }
#ifdef BOS_MF_PIVOT_CYCLES
    cstamp(cst, s, 7);
#endif
    if (nbad && lane == 0) atomicAdd(a.info, nbad);
    fstamp(stp, s, 5);
    // the update matrix: row[t] holds column k + t; for a parent in this flow as tagged granules
    // (update matrix, then u-vector), else plain (coherent) stores
    unsigned long long* const G = (MODE == kModeFlow && a.ug_off[s] >= 0) ? a.Ug + a.ug_off[s] : nullptr;
    if (G) {
#pragma unroll
        for (int t0 = 0; t0 < MAXM; t0 += 8) {
            if (t0 < r) {
#pragma unroll
                for (int t = t0; t < t0 + 8 && t < MAXM; ++t)
                    if (live && lane >= k && t <= lane - k) tag_pair(G + 2 * pk(lane - k, t, r), row[t], ep);
            }
        }
    } else {
#pragma unroll
        for (int t0 = 0; t0 < MAXM; t0 += 8) {
            if (t0 < r) {
#pragma unroll
                for (int t = t0; t < t0 + 8 && t < MAXM; ++t)
                    if (live && lane >= k && t <= lane - k) stc<COH>(Us + pk(lane - k, t, r), row[t]);
            }
        }
    }
    if (live) {
        if (lane < k) a.x[c0 + lane] = wi;
        else if (G) tag_pair(G + 2 * ((int64_t)r * (r + 1) / 2 + (lane - k)), wi, ep);
        else stc<COH>(us + (lane - k), wi);
    }
    wave_sync();
}

// (class 48 bounded to 4 waves per SIMD spills and measured slower)
template <int MAXM, bool F32>
__global__ __launch_bounds__(64, 1) void mf_factor_reg(const MfArgs a) {
    __shared__ __attribute__((aligned(16))) double F[MAXM * (MAXM + 1) / 2];
    __shared__ __attribute__((aligned(16))) double colbuf[2 * MAXM];
    __shared__ __attribute__((aligned(16))) double wv[MAXM];
    __shared__ FoldBuf fb;
    factor_front_reg<MAXM, kModeLevel, F32>(a, a.level[blockIdx.x], F, colbuf, wv, &fb, threadIdx.x, nullptr);
}

// Level-launch wave fronts with the pivots on register panels and the trailing update on f64 MFMA
// (VERDICT r05 next 1). factor_front_reg holds a lane's whole front row in registers (row[MAXM]): at
// class 48 that is 96 of the kernel's 147 VGPRs and caps level 0 (10 350 fronts, k ~ 18, m ~ 42) at 3
// waves per SIMD. Here a lane holds only the KP columns of the current panel: the pivot loop (the
// same two-pivot steps, LDS pair broadcast) runs over the panel's columns, the L columns go to global
// memory as before and into the front's LDS triangle in place of the columns they replace, and the
// rest of the front, still in LDS, takes A22 -= L21 L21^T in 16 x 16 tiles on v_mfma_f64_16x16x4f64
// (the fold's W W^T pattern); the last panel's tiles go straight to the update matrix. The prologue
// (fold, assembly, children) is factor_front_reg's, with the children's structure read after the
// fold instead of before it (its registers would be live across the fold).
template <int MAXM, int KP, bool F32>
__device__ __forceinline__ void factor_front_pan(const MfArgs& a, int s, double* F, double* colbuf, double* wv,
                                                 FoldBuf* fb, int lane) {
    const int k = a.k[s], r = a.r[s], m = k + r;
    const int nfold = a.fold_cnt[s];
    const int c0 = a.col0[s];
    const int aq0 = a.amap_ptr[s], aq1 = a.amap_ptr[s + 1];
    const int np = m * (m + 1) / 2;
    double xo = a.x[c0 + min(lane, k - 1)];
    double* Ls = a.L + a.L_off[s];
    double* Us = a.U + a.U_off[s];
    double* us = a.u + a.u_off[s];
    const int cb = a.child_ptr[s] + nfold, ce = a.child_ptr[s + 1];
    unsigned long long* const stp = a.stamps_f;
    fstamp(stp, s, 0);
    if (nfold > 0) {
        FoldAcc<MAXM> facc;
        fold_children<MAXM, F32>(a, s, F, fb, m, lane, facc);
        wave_sync();
        fold_store<MAXM>(facc, F, wv, m, lane);
    } else {
        for (int e = lane; e < np; e += 64) F[e] = 0.0;
        for (int i = lane; i < m; i += 64) wv[i] = 0.0;
    }
    wave_sync();
    fstamp(stp, s, 1);
    ChildPre p0c, p1c;   // (structure in flight during the assembly)
    if (cb < ce) child_meta(a, a.child[cb], lane, p0c);
    if (cb + 1 < ce) child_meta(a, a.child[cb + 1], lane, p1c);
    assemble_wave(a, aq0, aq1, F, lane, nfold > 0);
    wave_sync();
    asm volatile("" : "+v"(xo));
    xo = lane < k ? xo : 0.0;
    fstamp(stp, s, 2);
    fstamp(stp, s, 3);
    if (cb < ce) child_vals<false>(lane, p0c);
    if (cb + 1 < ce) child_vals<false>(lane, p1c);
    if (cb < ce) extend_child<false>(a, p0c, F, wv, m, lane);
    if (cb + 1 < ce) extend_child<false>(a, p1c, F, wv, m, lane);
    for (int ci = cb + 2; ci < ce; ++ci) {
        ChildPre pq;
        child_meta(a, a.child[ci], lane, pq);
        child_vals<false>(lane, pq);
        extend_child<false>(a, pq, F, wv, m, lane);
    }
    fstamp(stp, s, 4);
    const bool live = lane < m;
    const int lrow = min(lane, m - 1);
    double wi = live ? wv[lane] + xo : 0.0;   // forward elimination, fused into the pivot loop
    int nbad = 0;
    double2* cp = reinterpret_cast<double2*>(colbuf);
    for (int p0 = 0; p0 < k; p0 += KP) {
        const int nb = min(KP, k - p0);
        // row[t] = F(lane, p0 + t) (column clamped to m - 1: branch-free reads, one wait; entries
        // above the diagonal, of rows >= m and columns past the panel are scratch)
        double row[KP];
#pragma unroll
        for (int t0 = 0; t0 < KP; t0 += 8) {
            double v[8];
#pragma unroll
            for (int t = t0; t < t0 + 8; ++t) v[t - t0] = F[pk32(lrow, min(p0 + t, m - 1), m)];
            asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                         "+v"(v[7]));
#pragma unroll
            for (int t = t0; t < t0 + 8; ++t) row[t] = v[t - t0];
        }
        double* Lj = Ls + lane + (int64_t)p0 * m;
        int j = 0;   // pivot p0 + j; before step j, row[t] holds column p0 + j + t
#pragma nounroll
        for (; j + 1 < nb; j += 2) {
            const int J = p0 + j;
            double d0 = readlane_d(row[0], J);
            const bool bad0 = !(d0 > 0.0);
            nbad += bad0;
            d0 = bad0 ? 1e-300 : d0;
            const double inv0 = rsqrt_nr(d0), l00 = d0 * inv0;
            const double l0 = lane == J ? l00 : row[0] * inv0;   // L[i, J]
            const double lj1 = readlane_d(l0, J + 1);
            const double f1 = fma(-l0, lj1, row[1]);
            double d1 = readlane_d(f1, J + 1);
            const bool bad1 = !(d1 > 0.0);
            nbad += bad1;
            d1 = bad1 ? 1e-300 : d1;
            const double inv1 = rsqrt_nr(d1), l11 = d1 * inv1;
            const double l1 = lane == J + 1 ? l11 : f1 * inv1;   // L[i, J + 1]
            // pairs of the panel's later rows (the rank-2 update of its remaining columns)
            if (lane > J + 1 && lane < p0 + nb) cp[lane - J - 2] = make_double2(l0, l1);
            if (live) {
                if (lane >= J) {
                    ST_L(Lj, 0, l0);
                    F[pk32(lane, J, m)] = l0;   // L21 for the trailing update (column J is consumed)
                }
                if (lane >= J + 1) {
                    ST_L(Lj, m, l1);
                    F[pk32(lane, J + 1, m)] = l1;
                }
            }
            Lj += 2 * m;
            const double y0 = readlane_d(wi, J) * inv0;          // forward steps J, J + 1
            if (lane == J) wi = y0;
            else if (lane > J) wi -= l0 * y0;
            const double y1 = readlane_d(wi, J + 1) * inv1;
            if (lane == J + 1) wi = y1;
            else if (lane > J + 1) wi -= l1 * y1;
            wave_sync();
            const int nt = nb - j - 2;                           // panel columns left after this step
#pragma unroll
            for (int t0 = 0; t0 < KP - 2; t0 += 8) {
                if (t0 < nt) {
                    double2 c[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) c[u] = t0 + u < KP - 2 ? cp[t0 + u] : make_double2(0.0, 0.0);
#pragma unroll
                    for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(c[u].x), "+v"(c[u].y));
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (t0 + u < KP - 2) row[t0 + u] = fma(-l1, c[u].y, fma(-l0, c[u].x, row[t0 + u + 2]));
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (j < nb) {   // the panel's last column (odd nb)
            const int J = p0 + j;
            double d = readlane_d(row[0], J);
            const bool bad = !(d > 0.0);
            nbad += bad;
            d = bad ? 1e-300 : d;
            const double inv = rsqrt_nr(d), ljj = d * inv;
            const double lij = lane == J ? ljj : row[0] * inv;
            if (live && lane >= J) {
                ST_L(Lj, 0, lij);
                F[pk32(lane, J, m)] = lij;
            }
            const double yj = readlane_d(wi, J) * inv;
            if (lane == J) wi = yj;
            else if (lane > J) wi -= lij * yj;
        }
        wave_sync();
        // trailing block, rows / columns [t0, m): A22 -= L21 L21^T (L21 = rows >= t0 of the panel's L
        // columns, now in F) in 16 x 16 tiles; the last panel's result is the update matrix
        const int t0 = p0 + nb, T = m - t0;
        if (T > 0) {
            const bool last = t0 == k;
            const int nbt = (T + 15) >> 4;
            for (int bi = 0; bi < nbt; ++bi)
                for (int bj = 0; bj <= bi; ++bj) {
                    const int ra = t0 + 16 * bi + (lane & 15), rb = t0 + 16 * bj + (lane & 15);
                    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
                    for (int kk = 0; kk < nb; kk += 4) {
                        const int cc = kk + (lane >> 4);
                        const int col = p0 + min(cc, nb - 1);
                        const double av = F[pk32(min(ra, m - 1), col, m)];
                        const double bv = F[pk32(min(rb, m - 1), col, m)];
                        const bool ok = cc < nb;
                        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ok && ra < m ? av : 0.0, ok && rb < m ? bv : 0.0,
                                                                   acc, 0, 0, 0);
                    }
                    const int jj = t0 + 16 * bj + (lane & 15);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int ii = t0 + 16 * bi + (lane >> 4) + 4 * e;
                        if (ii < m && jj <= ii) {
                            const double v = F[pk32(ii, jj, m)] - acc[e];
                            if (last) Us[pk(ii - k, jj - k, r)] = v;
                            else F[pk32(ii, jj, m)] = v;
                        }
                    }
                }
            wave_sync();
        }
    }
    if (nbad && lane == 0) atomicAdd(a.info, nbad);
    fstamp(stp, s, 5);
    if (live) {
        if (lane < k) a.x[c0 + lane] = wi;
        else us[lane - k] = wi;
    }
    wave_sync();
}

// the class-48 level launches take the panel kernel (A/B builds: -DBOS_MF_PAN=0 keeps mf_factor_reg)
#ifndef BOS_MF_PAN
#define BOS_MF_PAN 1
#endif
constexpr bool kPanel48 = BOS_MF_PAN != 0;
// the class-64 level launches too (config 2's separators of 49-64 rows; config 3's side-stream class)
#ifndef BOS_MF_PAN64
#define BOS_MF_PAN64 1
#endif
constexpr bool kPanel64 = BOS_MF_PAN64 != 0;
#ifndef BOS_MF_PAN_KP
#define BOS_MF_PAN_KP 24
#endif
constexpr int kPanelKP = BOS_MF_PAN_KP;
// waves per SIMD the panel kernel is compiled for. Its register peak is the fold (the panel's rows
// alone take 92 VGPRs, the fold 132), so it stays at mf_factor_reg<48>'s 3 waves per SIMD; bounded to 4
// it spills 3 registers (14 in fp64) and measured no faster. Measured (config 3, tools/gn_ab.py, two
// rounds, profiles/r06_panel_ab.txt): solve 439.6 / 442.8 us with mf_factor_reg, 439.0 / 439.8 with
// 16-column panels at 4 waves, 433.7 / 432.0 with 24 columns at 3 waves (one panel for most level-0
// fronts, k ~ 18), 433.6 / 434.4 with 32.
#ifndef BOS_MF_PAN_WAVES
#define BOS_MF_PAN_WAVES 3
#endif

template <int MAXM, int KP> struct WaveLds {
    double F[MAXM * (MAXM + 1) / 2];
    double colbuf[2 * (KP > 0 ? KP : MAXM)];
    double wv[MAXM];
    FoldBuf fb;
};
template <int MAXM, int KP, bool F32>
__global__ __launch_bounds__(64, MAXM > 48 ? 2 : BOS_MF_PAN_WAVES) void mf_factor_pan(const MfArgs a) {
    __shared__ __attribute__((aligned(16))) double F[MAXM * (MAXM + 1) / 2];
    __shared__ __attribute__((aligned(16))) double colbuf[2 * KP];
    __shared__ __attribute__((aligned(16))) double wv[MAXM];
    __shared__ FoldBuf fb;
    factor_front_pan<MAXM, KP, F32>(a, a.level[blockIdx.x], F, colbuf, wv, &fb, threadIdx.x);
}

// One wave front of class 3, 2, 1 or 0 with its LDS at slot (mf_factor_mixb)
template <int MAXM, int KP, bool F32>
__device__ __forceinline__ void wave_front(const MfArgs& a, int s, char* slot, int lane) {
    auto* L = reinterpret_cast<WaveLds<MAXM, KP>*>(slot);
    if constexpr (KP > 0)
        factor_front_pan<MAXM, KP, F32>(a, s, L->F, L->colbuf, L->wv, &L->fb, lane);
    else
        factor_front_reg<MAXM, kModeLevel, F32>(a, s, L->F, L->colbuf, L->wv, &L->fb, lane, nullptr);
}

#ifndef BOS_MF_MIXB   // (A/B builds: -DBOS_MF_MIXB=0 keeps the blocked fronts on the second side stream)
#define BOS_MF_MIXB 1
#endif
constexpr bool kMixB = BOS_MF_MIXB != 0;

// A level with blocked fronts (65-128 rows, config 2's separators) and few fronts in all: ONE launch
// of four-wave workgroups instead of the blocked launch on a second side stream beside the wave
// fronts (each level then paid a fork and a join, ~10 us per level at config 2). The first n4
// workgroups each factor one blocked front (factor_front_blk, the whole dynamic LDS), each of the
// others one wave front of class 3, 2, 1 or 0 on its first wave (the other three leave at once; two
// wave fronts in one workgroup computed wrong factors). Registers are the blocked
// path's (1 wave per SIMD), so the host uses it only when the level fits the GPU in one round (one
// workgroup per CU); dynamic LDS max(blocked front, one class-64 front).
template <bool F32>
__global__ __launch_bounds__(kMfBlock) void mf_factor_mixb(const MfArgs a, const int32_t* blk_list, int n4, int4 n, int4 o) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int b = blockIdx.x;
    if (b < n4) {   // (uniform per workgroup)
        factor_front_blk<F32>(a, blk_list[b], lds);
        return;
    }
#ifdef BOS_DIAG_PAIR   // (diagnostics: class-2 fronts two per workgroup, on waves 0 and BOS_DIAG_PAIR)
    {
        const int wv = threadIdx.x >> 6;
        int i = b - n4;
        if (i >= n.w && i - n.w < (n.z + 1) / 2) {
            const int j = 2 * (i - n.w) + (wv == BOS_DIAG_PAIR ? 1 : 0);
            if ((wv == 0 || wv == BOS_DIAG_PAIR) && j < n.z)
                wave_front<48, kPanel48 ? kPanelKP : 0, F32>(a, a.level[o.z + j],
                                                             reinterpret_cast<char*>(lds) + wv * 10400 * 1, threadIdx.x & 63);
            return;
        }
    }
#endif
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    char* slot = reinterpret_cast<char*>(lds);
    const int32_t* lst = a.level;
    int i = b - n4;
    if (i < n.w) { wave_front<64, kPanel64 ? kPanelKP : 0, F32>(a, lst[o.w + i], slot, lane); return; }
    i -= n.w;
#ifdef BOS_DIAG_PAIR
    i -= (n.z + 1) / 2;
#else
    if (i < n.z) { wave_front<48, kPanel48 ? kPanelKP : 0, F32>(a, lst[o.z + i], slot, lane); return; }
    i -= n.z;
#endif
    if (i < n.y) { wave_front<32, 0, F32>(a, lst[o.y + i], slot, lane); return; }
    i -= n.y;
    if (i < n.x) wave_front<16, 0, F32>(a, lst[o.x + i], slot, lane);
}
#ifdef BOS_DIAG_PAIR
constexpr int kMixbWaveLds = 4 * 10400;
static_assert(sizeof(WaveLds<48, kPanel48 ? kPanelKP : 0>) <= 10400, "diagnostic slot");
#else
constexpr int kMixbWaveLds = (int)sizeof(WaveLds<64, kPanel64 ? kPanelKP : 0>);
#endif


// Backward substitution of one front by one wavefront (any m); LDS: x_own[k] | t[k] | x_rows[r] |
// L panel (m x k). The rows below the supernode are ancestors' dofs, already final in x.
// The L panel and the front's own forward results do not depend on the ancestors, so the flow
// kernel stages them before it waits for the parent (FLOW: f and parent set).
constexpr int kBwdRegK = 32;   // fronts with k <= this solve their triangle from registers

template <int MODE>
__device__ __forceinline__ void backward_front(const MfArgs& a, int s, double* w, int lane, const Flow* f,
                                               const int32_t* parent) {
    constexpr bool COH = MODE == kModeFlow;
    const int k = a.k[s], r = a.r[s], m = k + r;
    const int c0 = a.col0[s];
    const int32_t* fi = a.findex + a.findex_off[s];
    double* t = w + k;
    double* xs = w + 2 * k;
    double* Lw = w + 2 * k + r;
    // where the first 64 rows' x live (static); clamped, branch-free reads (see assemble_wave)
    const int xi0 = fi[k + min(lane, max(r - 1, 0))];
    unsigned long long* const stp = f ? f->stamps : a.stamps_b;
    fstamp(stp, s, 0);
    if constexpr (MODE == kModeLevel) {
        // per-level launch: the parents' x are final (earlier launches), so the front's own
        // right-hand side and the first 64 rows' x are loaded beside the panel, all in flight at once
        const double y0v = a.x[c0 + min(lane, k - 1)], xr0v = a.x[xi0];
        const double y0 = lane < k ? y0v : 0.0;
        const double xr0 = lane < r ? xr0v : 0.0;
        stage_lds<16, true>(Lw, a.L + a.L_off[s], m * k, lane);
        if (lane < k) w[lane] = y0;
        for (int j = 64 + lane; j < k; j += 64) w[j] = a.x[c0 + j];
        fstamp(stp, s, 1);
        fstamp(stp, s, 2);
        if (lane < r) xs[lane] = xr0;
        for (int i = 64 + lane; i < r; i += 64) xs[i] = a.x[fi[k + i]];
    } else {
        stage_lds<8, true>(Lw, a.L + a.L_off[s], m * k, lane);
        for (int j = lane; j < k; j += 64) w[j] = a.x[c0 + j];
        fstamp(stp, s, 1);
        if (parent[s] >= 0 && f->fid[parent[s]] == f->id) {
            // the rows are dofs of ancestors, whose x every backward front publishes as tagged
            // granules (xg): one lane probes the parent's first dof, then the rows are swept until
            // every tag is this step's epoch (no completion flag)
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            probe_granule(a.xg + 2 * (int64_t)a.col0[parent[s]] + 1, f->epoch, t0, a.info);
            for (uint32_t it = 0;; ++it) {
                bool ok = true;
                const double v0 = untag_pair(a.xg + 2 * (int64_t)xi0, f->epoch, ok);
                if (lane < r) xs[lane] = v0;
                for (int i = 64 + lane; i < r; i += 64) xs[i] = untag_pair(a.xg + 2 * (int64_t)fi[k + i], f->epoch, ok);
                if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
                if ((it & 15) == 15) {
                    const bool stalled = (__hip_atomic_load(a.info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kStall) != 0;
                    if (stalled || __builtin_amdgcn_s_memrealtime() - t0 > kWaitTicks) {
                        if (lane == 0) atomicOr(a.info, kStall);
                        break;
                    }
                }
                __builtin_amdgcn_s_sleep(1);
            }
        } else {   // the parent finished in an earlier launch (or none): final x
            if (lane < r) xs[lane] = ldc<COH>(a.x + xi0);
            for (int i = 64 + lane; i < r; i += 64) xs[i] = ldc<COH>(a.x + fi[k + i]);
        }
        fstamp(stp, s, 2);
    }
    wave_sync();
    if (k <= 64) {
        // lane j < k: t_j = sum_i L[k + i, j] x[fi[k + i]] in row order, then the triangular
        // solve in registers: x_j = (y_j - t_j) / L_jj broadcast from lane j, t_i += L[j, i] x_j
        const bool own = lane < k;
        double tj = 0.0;
        if (own)
            for (int i = 0; i < r; ++i) tj += Lw[k + i + lane * m] * xs[i];
        // 1 / L_jj by every lane at once, off the sequential chain below
        const double yv = own ? w[lane] : 0.0, rjj = own ? 1.0 / Lw[lane + lane * m] : 1.0;
        double xv = 0.0;
        // per-level launches only: in the backward flow the register form measured slower (solve +6 us,
        // profiles/r05_backward_flow_registers_ab.txt)
        if (MODE == kModeLevel && k <= kBwdRegK) {
            // the lane's column of the k x k block in registers, read from LDS before the chain, so
            // each step of the sequential chain is arithmetic and a lane read only
            double lr[kBwdRegK];
#pragma unroll
            for (int j = 0; j < kBwdRegK; ++j) lr[j] = own && j < k ? Lw[j + lane * m] : 0.0;
#pragma unroll
            for (int j = kBwdRegK - 1; j >= 0; --j) {
                if (j < k) {   // uniform
                    const double xj = readlane_d((yv - tj) * rjj, j);
                    if (lane == j) xv = xj;
                    else if (lane < j) tj += lr[j] * xj;
                }
            }
        } else {
            for (int j = k - 1; j >= 0; --j) {
                const double xj = readlane_d((yv - tj) * rjj, j);
                if (lane == j) xv = xj;
                else if (lane < j) tj += Lw[j + lane * m] * xj;
            }
        }
        if (own) stc<COH>(a.x + c0 + lane, xv);
        if (a.xtag[s] && own) tag_pair(a.xg + 2 * (int64_t)(c0 + lane), xv, *a.epoch);
        wave_sync();
        fstamp(stp, s, 3);
        return;
    }
    // t_j = sum_i L[k + i, j] x[fi[k + i]]: fixed-order wave reduction per column
    for (int j = 0; j < k; ++j) {
        double v = 0.0;
        for (int i = lane; i < r; i += 64) v += Lw[k + i + j * m] * xs[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) t[j] = v;
    }
    wave_sync();
    for (int j = k - 1; j >= 0; --j) {
        const double xj = (w[j] - t[j]) / Lw[j + j * m];
        wave_sync();
        if (lane == 0) w[j] = xj;
        for (int i = lane; i < j; i += 64) t[i] += Lw[j + i * m] * xj;
        wave_sync();
    }
    for (int j = lane; j < k; j += 64) stc<COH>(a.x + c0 + j, w[j]);
    if (a.xtag[s]) {
        const uint32_t ep = *a.epoch;
        for (int j = lane; j < k; j += 64) tag_pair(a.xg + 2 * (int64_t)(c0 + j), w[j], ep);
    }
    wave_sync();
}

__global__ __launch_bounds__(64) void mf_backward_wave(const MfArgs a) {
    extern __shared__ __attribute__((aligned(16))) double w[];
    backward_front<kModeLevel>(a, a.level[blockIdx.x], w, threadIdx.x, nullptr, nullptr);
}

// Backward substitution of the folded landmarks (k = 2), kFoldLanes lanes each (rows of the
// landmark's two L columns across the lanes, coalesced): t = L21^T x_rows reduced over the lanes,
// then x1 = (y1 - t1) / L11, x0 = (y0 - t0 - L10 x1) / L00. A lane takes up to four rows per pass
// with every load of the pass issued at once (row indices and L values, then the x gathers), and
// the landmark's own values are loaded before them: the launch is latency bound (few dependent
// hops per landmark, 200k landmarks), so fewer lanes per landmark with more loads in flight each
// beat one row per lane.
// (one lane per landmark from a packed record measured slower: DESIGN.md §4)
#ifndef BOS_MF_FOLD_LANES
#define BOS_MF_FOLD_LANES 4
#endif
// measured: 22 us at 4 lanes, 23 at 8, 34 at 16 (config 3); round 5: 2 / 8 lanes +10 / +3 us of solve
constexpr int kFoldLanes = BOS_MF_FOLD_LANES;
__global__ __launch_bounds__(kMfBlock) void mf_backward_fold(const MfArgs a) {
    const int g = (blockIdx.x * kMfBlock + threadIdx.x) / kFoldLanes;
    const int q0 = threadIdx.x % kFoldLanes;
    const bool valid = g < a.count;
    const int s = valid ? a.level[g] : 0;
    const int r = valid ? a.r[s] : 0, m = 2 + r;
    const double* Ls = a.L + (valid ? a.L_off[s] : 0);
    const int32_t* fi = a.findex + (valid ? a.findex_off[s] : 0) + 2;
    const int c0 = valid ? a.col0[s] : 0;
    const bool head = valid && q0 == 0;
    // the landmark's own values, read by all its lanes (one address: no extra traffic) so no branch
    // holds a wait; only the head lane uses them
    const double y0v = a.x[c0], y1v = a.x[c0 + 1], L00v = LD_LF(Ls, 0), L10v = LD_LF(Ls, 1), L11v = LD_LF(Ls, m + 1);
    const double y0 = head ? y0v : 0.0, y1 = head ? y1v : 0.0;
    const double L00 = head ? L00v : 1.0, L10 = head ? L10v : 0.0, L11 = head ? L11v : 1.0;
    double t0 = 0.0, t1 = 0.0;
    const int rl = r > 0 ? r - 1 : 0;   // reads of rows past r are clamped (and their products dropped)
    for (int q = q0; q < r; q += 4 * kFoldLanes) {
        int idx[4];
        double la[4], lb[4], xv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int qq = min(q + u * kFoldLanes, rl);
            idx[u] = fi[qq];
            la[u] = LD_LF(Ls, 2 + qq);
            lb[u] = LD_LF(Ls, m + 2 + qq);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) xv[u] = a.x[idx[u]];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool ok = q + u * kFoldLanes < r;
            t0 += ok ? la[u] * xv[u] : 0.0;
            t1 += ok ? lb[u] * xv[u] : 0.0;
        }
    }
#pragma unroll
    for (int o = kFoldLanes / 2; o > 0; o >>= 1) {
        t0 += __shfl_xor(t0, o, kFoldLanes);
        t1 += __shfl_xor(t1, o, kFoldLanes);
    }
    if (head) {
        const double x1 = (y1 - t1) / L11;
        t0 += L10 * x1;
        a.x[c0] = (y0 - t0) / L00;
        a.x[c0 + 1] = x1;
    }
}

// The flow kernel instantiates one register class only: inlining all four merged their register
// demands (256 VGPRs + AGPRs, 1 wave per SIMD), out-of-line calls spilled, and forcing 4 waves per
// SIMD spilled too (all measured slower); 2 waves per SIMD (no spills) measured faster than 3 (a
// few spilled registers). Fronts of the flow range are <= kFlowMaxM (mf_create picks the range
// accordingly).
constexpr int kFlowMaxM = kMfFlowMaxM;

template <bool F32>
__device__ __forceinline__ void factor_flow_body(const MfArgs& a, const Flow& f) {
    __shared__ __attribute__((aligned(16))) double F[kFlowMaxM * (kFlowMaxM + 1) / 2];
    __shared__ __attribute__((aligned(16))) double colbuf[2 * kFlowMaxM];
    __shared__ __attribute__((aligned(16))) double wv[kFlowMaxM];
    __shared__ FoldBuf fb;
    const int lane = threadIdx.x;
    // a wave takes at most n + 1 tickets: the loop is bounded (an unbounded for (;;) version of
    // this kernel never terminated on gfx950 / ROCm 7.2)
    for (int it = 0; it <= f.n; ++it) {
        const int t = next_ticket(f.ticket);
        if (t >= f.n) break;
        const int s = f.order[t];
        factor_front_reg<kFlowMaxM, kModeFlow, F32>(a, s, F, colbuf, wv, &fb, lane, &f);   // m <= kFlowMaxM
        // (no completion flag: a parent in this flow polls the tagged granules themselves)
        fstamp(f.stamps, s, 6);
        fstamp(f.stamps, s, 7);
    }
    leave_flow(f);
}

template <bool F32>
__global__ __launch_bounds__(64, 2) void mf_factor_flow(const MfArgs a, const Flow f_in) {
    Flow f = f_in;
    f.epoch = *f_in.epoch_src;
    factor_flow_body<F32>(a, f);
}

__global__ __launch_bounds__(64) void mf_backward_flow(const MfArgs a, const Flow f_in, const int32_t* parent) {
    extern __shared__ __attribute__((aligned(16))) double w[];
    Flow f = f_in;
    f.epoch = *f_in.epoch_src;
    for (int it = 0; it <= f.n; ++it) {
        const int t = next_ticket(f.ticket);
        if (t >= f.n) break;
        const int s = f.order[t];
        backward_front<kModeFlow>(a, s, w, threadIdx.x, &f, parent);
        // (no completion flag: the children poll the tagged x granules themselves)
        fstamp(f.stamps, s, 4);
    }
    leave_flow(f);
}

// Structure arrays carry kMfPad zeroed elements after their end: the kernels read clamped indices
// unconditionally (branch-free loads, see assemble_wave) and may touch up to one chunk / 64 lanes past
// a range's last element.
constexpr int64_t kMfPad = 64;
template <typename X> int up(X** p, const std::vector<X>& v, std::string& err) {
    *p = nullptr;
    if (v.empty()) return 0;
    const size_t bytes = v.size() * sizeof(X), padded = bytes + kMfPad * sizeof(X);
    if (hipMalloc((void**)p, padded) != hipSuccess) { err = "hipMalloc failed (multifrontal)"; return -2; }
    if (hipMemcpy(*p, v.data(), bytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset((char*)*p + bytes, 0, padded - bytes) != hipSuccess) {
        err = "hipMemcpy failed (multifrontal)";
        return -2;
    }
    return 0;
}

}  // namespace

// front size classes: m <= 16, 32, 48, 64 (one wavefront, registers / LDS), m <= kBlkMaxM (workgroup,
// blocked, folds landmarks: mf_factor_blk) and larger (workgroup, global scratch: mf_factor_level)
constexpr int kClasses = 6;
inline int front_class(int m) { return m <= kMfWaveMaxM ? (m - 1) / 16 : m <= kBlkMaxM ? 4 : 5; }
// The launch a front goes to: fronts with 16 < m <= 32 run in the class-48 launch of their level (one
// launch packs the level's waves better than two in a row on one stream: solve 589 -> 564 us on
// config 3; moving the m <= 16 fronts too measured 570)
inline int launch_class(int m) {
    const int c = front_class(m);
    return c == 1 ? 2 : c;
}

// The fronts one launch sequence processes: every front on one GPU; a rank's own subtrees or the
// replicated top when sharded (plan.hpp Shard). Levels below flow_lev0 run per level (binned by
// front class), the rest of the factorization as one dataflow launch; the backward solve as one
// dataflow launch over levels >= solve_lev0 (top-down), then per level, then the folded landmarks.
struct Prog {
    int id = 0;                     // flow id (1: own / everything, 2: top)
    std::vector<int32_t> ptr;       // (level l, class c) = list[ptr[l * kClasses + c], ...)
    std::vector<int> lds_factor, lds_fwd, lds_bwd;   // per (level, class): dynamic LDS bytes
    std::vector<int> lds_blk;       // per level: mf_factor_blk's LDS for its class-4 fronts
    int32_t* list = nullptr;
    int flow_lev0 = 0, n_flow_factor = 0;
    bool first_waited = false;      // the factor flow's first front has its parent in the same flow
    int32_t* order_factor = nullptr;
    bool flow_solve = false;
    int solve_lev0 = 0, n_flow_solve = 0, lds_bwd_flow = 0;
    int32_t* order_bwd = nullptr;
    int32_t* fold_list = nullptr;   // folded landmarks whose parent is in this program
    int n_fold = 0;
    // per-level backward launches of the wave fronts (classes 0-3, one launch per level, the LDS of
    // the level's largest panel): level l's fronts are blist[bptr[l] .. bptr[l + 1]), blds[l] bytes each
    std::vector<int32_t> bptr;
    std::vector<int> blds;
    int32_t* blist = nullptr;
    int count(int lev, int c0, int c1) const { return ptr[lev * kClasses + c1] - ptr[lev * kClasses + c0]; }
    int count(int lev, int c) const { return count(lev, c, c + 1); }
    int lds_max(const std::vector<int>& v, int lev, int c0, int c1) const {
        int b = 0;
        for (int c = c0; c < c1; ++c) b = std::max(b, v[lev * kClasses + c]);
        return b;
    }
};

// Dataflow launch geometry (config 3, measured with tools/solver_stamps.py and variant builds): a
// wave waiting on a dependency polls its flag, and waiting waves slow the ones working, so the flows
// run few waves: 6 per CU for the factorization (solve 593 us at 6 against 599 at 8, 602 at 4, 682
// at 12) and 4 per CU for the backward substitution (582 us at 4, 617 at 6, 636 at 8, 706 at 16).
// The flows take only the narrow top of the tree; wide levels (independent fronts, throughput
// bound) run as per-level launches: the backward substitution of levels with >= kSolveWideLevel
// fronts before the flow reaches them (config 3: levels 0-5, solve 659 -> 582 us), the
// factorization of levels with >= kFactorWideLevel fronts before its flow starts (config 3: levels
// 0-2, 564 -> 556 us; also level 3: 567).
#ifndef BOS_MF_FLOW_WAVES_F   // (A/B builds may override the flow geometry)
#define BOS_MF_FLOW_WAVES_F 6
#endif
constexpr int kFlowWavesFactor = BOS_MF_FLOW_WAVES_F;
// The per-level backward launch of a level's wave fronts gives every wave the LDS of the level's
// largest panel (m k doubles): class-64 fronts (up to ~16 KB) then hold a level-0 launch to 8-10
// waves per CU; splitting the big panels into a launch of their own measured no faster.
#ifndef BOS_MF_FLOW_WAVES_B
#define BOS_MF_FLOW_WAVES_B 4
#endif
constexpr int kFlowWavesBackward = BOS_MF_FLOW_WAVES_B;
#ifndef BOS_MF_SOLVE_WIDE   // (A/B builds may override the two thresholds)
#define BOS_MF_SOLVE_WIDE 256
#endif
#ifndef BOS_MF_FACTOR_WIDE
#define BOS_MF_FACTOR_WIDE 2048
#endif
constexpr int kSolveWideLevel = BOS_MF_SOLVE_WIDE;
constexpr int kFactorWideLevel = BOS_MF_FACTOR_WIDE;
struct MfDevice {
    int nlevels = 0, nsuper = 0, ncu = 256;
    bool mixb = false;            // mf_factor_mixb too (a level's blocked and wave fronts in one launch)
    bool blk = false;             // mf_factor_blk may take its (up to 132 KB of) dynamic LDS
    // a level's largest fronts (class 64: few, one latency-bound round) run on a side stream beside
    // the level's other classes
    hipStream_t side = nullptr, side2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_join2 = nullptr;
    static constexpr int tiny16 = 256;   // class-16 launches of at most this many fronts go to the side stream too
    Prog prog[2];                 // [0]: own (or every front), [1]: the replicated top (sharded only)
    int8_t *fid_f = nullptr, *fid_b = nullptr;   // flow membership: factor, backward
    int32_t* parent = nullptr;
    int* tickets = nullptr;       // [2 * kMfTickets]: work-queue tickets, then the launches' exit counters
    uint32_t* epoch = nullptr;    // device word, 1 at creation (granule tags start at 0), bumped per GN step
    unsigned long long* stamps = nullptr;   // diagnostics: [2][nsuper][8] flow stamps (factor, backward), or null
    int32_t *fold_cnt = nullptr, *fold_cptr = nullptr, *fold_chunk = nullptr, *fold_rec = nullptr;
    int16_t* emap = nullptr;
    int64_t* emap_off = nullptr;
    int32_t *col0 = nullptr, *k = nullptr, *r = nullptr, *child_ptr = nullptr, *child = nullptr,
            *rmap = nullptr, *amap_ptr = nullptr, *amap_src = nullptr, *amap_dst = nullptr, *findex = nullptr,
            *info = nullptr;
    int64_t *L_off = nullptr, *U_off = nullptr, *u_off = nullptr, *scratch_off = nullptr, *rmap_off = nullptr,
            *findex_off = nullptr;
    double *L = nullptr, *U = nullptr, *u = nullptr, *scratch = nullptr;
    const float* A32 = nullptr;   // mf_set_fold_source
    int64_t pl_lo = 0;
    // tagged hand-offs (MfArgs): update-matrix granules of flow fronts whose parent is in the same
    // flow, their offsets, x granules per dof and the fronts whose x a backward flow reads
    unsigned long long *Ug = nullptr, *xg = nullptr;
    int64_t* ug_off = nullptr;
    int8_t* xtag = nullptr;

    MfArgs args(const Prog& P, int lev, int c, const double* A, double* x) const {
        MfArgs g;
        g.level = P.list + (P.ptr.empty() ? 0 : P.ptr[lev * kClasses + c]);
        g.count = P.ptr.empty() ? 0 : P.count(lev, c);
        g.col0 = col0; g.k = k; g.r = r; g.L_off = L_off; g.U_off = U_off; g.u_off = u_off;
        g.scratch_off = scratch_off; g.child_ptr = child_ptr; g.child = child; g.rmap_off = rmap_off; g.rmap = rmap;
        g.amap_ptr = amap_ptr; g.amap_src = amap_src; g.amap_dst = amap_dst; g.findex_off = findex_off;
        g.findex = findex; g.A = A; g.A32 = A32; g.pl_lo = pl_lo; g.L = L; g.U = U; g.u = u; g.scratch = scratch; g.x = x; g.info = info;
        g.fold_cnt = fold_cnt; g.fold_cptr = fold_cptr; g.fold_chunk = fold_chunk; g.fold_rec = fold_rec;
        g.emap = emap; g.emap_off = emap_off;
        g.Ug = Ug; g.ug_off = ug_off; g.xg = xg; g.xtag = xtag; g.epoch = epoch;
        g.stamps_f = stamps;
        g.stamps_b = stamps ? stamps + 8 * (int64_t)nsuper : nullptr;
        return g;
    }
};

namespace {

int build_prog(const Multifrontal& F, const std::vector<int8_t>& sel, int id, Prog& P, std::vector<int8_t>& fid_f,
               std::vector<int8_t>& fid_b, std::string& err) {
    P.id = id;
    const int L = F.nlevels;
    P.lds_factor.assign(L * kClasses, 0); P.lds_fwd.assign(L * kClasses, 0); P.lds_bwd.assign(L * kClasses, 0);
    P.ptr.assign(L * kClasses + 1, 0);
    P.lds_blk.assign(L, 0);
    auto mine = [&](int s) { return sel[s] == id; };
    std::vector<int32_t> lst;
    for (int l = 0; l < L; ++l)
        for (int c = 0; c < kClasses; ++c) {
            const int lc = l * kClasses + c;
            for (int q = F.level_ptr[l]; q < F.level_ptr[l + 1]; ++q) {
                const int s = F.level[q], k = F.k[s], m = k + F.r[s];
                if (!mine(s) || launch_class(m) != c) continue;
                lst.push_back(s);
                if (c < 4) {
                    P.lds_fwd[lc] = std::max(P.lds_fwd[lc], (m + m * k) * 8);
                    P.lds_bwd[lc] = std::max(P.lds_bwd[lc], (2 * k + (m - k) + m * k) * 8);
                } else {
                    if (m <= kLdsCapM) P.lds_factor[lc] = std::max(P.lds_factor[lc], m * m * 8);
                    if (c == 4) P.lds_blk[l] = std::max(P.lds_blk[l], blk_lds_bytes(m));
                    P.lds_fwd[lc] = std::max(P.lds_fwd[lc], m * 8);
                    P.lds_bwd[lc] = std::max(P.lds_bwd[lc], (2 * k + (k <= 64 ? k * (k + 1) : 0)) * 8);
                }
            }
            // longest fronts first (estimated by flops plus folded rows): the launch's tail is
            // then made of short fronts
            auto cost = [&](int s2) {
                const double k = F.k[s2], r = F.r[s2];
                double cc = k * k * k / 3 + k * k * r + k * r * r;
                if (!F.fold_cnt.empty())
                    for (int ci = F.child_ptr[s2]; ci < F.child_ptr[s2] + F.fold_cnt[s2]; ++ci)
                        cc += 4.0 * F.r[F.child[ci]] * F.r[F.child[ci]];
                return cc;
            };
            std::stable_sort(lst.begin() + P.ptr[lc], lst.end(), [&](int x, int y) { return cost(x) > cost(y); });
            P.ptr[lc + 1] = (int32_t)lst.size();
        }
    auto mine_in_level = [&](int l) {
        int c = 0;
        for (int q = F.level_ptr[l]; q < F.level_ptr[l + 1]; ++q) c += mine(F.level[q]);
        return c;
    };
    std::vector<int32_t> blst;
    P.bptr.assign(L + 1, 0);
    P.blds.assign(L, 0);
    for (int l = 0; l < L; ++l) {
        // the level's wave fronts (classes 0-3, in list order: longest first)
        const int q0 = P.ptr[l * kClasses], q1 = P.ptr[l * kClasses + 4];
        for (int q = q0; q < q1; ++q) {
            const int s2 = lst[q], k = F.k[s2], m = k + F.r[s2];
            P.blds[l] = std::max(P.blds[l], (2 * k + (m - k) + m * k) * 8);
            blst.push_back(s2);
        }
        P.bptr[l + 1] = (int32_t)blst.size();
    }
    // dataflow ranges: the factor flow starts at the lowest level (>= 2) from which every front is
    // <= kFlowMaxM, and above the wide levels. Both decided on the whole tree, not on this program's
    // fronts: a front is then factored by the same kernel (per-level or flow) whatever the partition,
    // and the per-level class-48 kernel (mf_factor_pan: trailing update on MFMA) and the flow's
    // rounding differ, so a sharded step equals the one-GPU step bit for bit only this way.
    P.flow_lev0 = L;
    while (P.flow_lev0 > 2) {
        bool small = true;
        for (int q = F.level_ptr[P.flow_lev0 - 1]; q < F.level_ptr[P.flow_lev0] && small; ++q)
            small = F.k[F.level[q]] + F.r[F.level[q]] <= kFlowMaxM;
        if (!small) break;
        --P.flow_lev0;
    }
    {
        int wide = std::min(2, L);
        while (wide < L && F.level_ptr[wide + 1] - F.level_ptr[wide] >= kFactorWideLevel) ++wide;
        P.flow_lev0 = std::max(P.flow_lev0, wide);
    }
    std::vector<int32_t> ofac, ofwd;
    for (int q = F.level_ptr[std::min(P.flow_lev0, L)]; q < F.level_ptr[L]; ++q) {
        const int s = F.level[q];
        if (!mine(s)) continue;
        ofac.push_back(s);
        fid_f[s] = (int8_t)id;
    }
    P.n_flow_factor = (int)ofac.size();
    P.first_waited = !ofac.empty() && F.parent[ofac[0]] >= 0 && fid_f[F.parent[ofac[0]]] == id;
    P.solve_lev0 = std::min(2, L);
    while (P.solve_lev0 < L && mine_in_level(P.solve_lev0) >= kSolveWideLevel) ++P.solve_lev0;
    for (int q = F.level_ptr[P.solve_lev0]; q < F.level_ptr[L]; ++q) {
        const int s = F.level[q], k = F.k[s], m = k + F.r[s];
        if (!mine(s)) continue;
        ofwd.push_back(s);
        P.lds_bwd_flow = std::max(P.lds_bwd_flow, (2 * k + (m - k) + m * k) * 8);
    }
    std::vector<int32_t> obwd(ofwd.rbegin(), ofwd.rend());
    P.n_flow_solve = (int)ofwd.size();
    P.flow_solve = P.n_flow_solve > 0 && P.lds_bwd_flow <= 48 * 1024;
    if (!P.flow_solve) P.solve_lev0 = L;
    else
        for (int s : obwd) fid_b[s] = (int8_t)id;
    std::vector<int32_t> folds;
    for (int s : F.fold_list)
        if (mine(F.parent[s])) folds.push_back(s);
    P.n_fold = (int)folds.size();
    int rc;
    if ((rc = up(&P.list, lst, err)) || (rc = up(&P.order_factor, ofac, err)) || (rc = up(&P.order_bwd, obwd, err)) ||
        (rc = up(&P.fold_list, folds, err)) || (rc = up(&P.blist, blst, err)))
        return rc;
    return 0;
}

void free_prog(Prog& P) {
    void* bufs[] = {P.list, P.order_factor, P.order_bwd, P.fold_list, P.blist};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
}

}  // namespace

int mf_create(const Multifrontal& F, const int8_t* owner, int rank, MfDevice** out, std::string& err) {
    MfDevice* d = new MfDevice();
    *out = d;
    d->nlevels = F.nlevels;
    d->nsuper = F.nsuper;
    std::vector<int64_t> scr(F.nsuper, -1);
    int64_t scratch_size = 0;
    for (int s = 0; s < F.nsuper; ++s) {
        const int m = F.k[s] + F.r[s];
        if (m > kLdsCapM) { scr[s] = scratch_size; scratch_size += (int64_t)m * m; }
    }
    {
        int dev = 0, ncu = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
            d->ncu = ncu;
        // a front of kBlkMaxM rows takes 129 KB of LDS (160 KB per CU on gfx950)
        const int blk_lds = blk_lds_bytes(kBlkMaxM);
        d->blk = hipFuncSetAttribute((const void*)mf_factor_blk<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     blk_lds) == hipSuccess &&
                 hipFuncSetAttribute((const void*)mf_factor_blk<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     blk_lds) == hipSuccess;
        d->mixb = d->blk &&
                  hipFuncSetAttribute((const void*)mf_factor_mixb<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      blk_lds) == hipSuccess &&
                  hipFuncSetAttribute((const void*)mf_factor_mixb<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      blk_lds) == hipSuccess;
        (void)hipGetLastError();
        if (!d->blk) {
            // the plan folds landmarks into fronts of up to kMfBlkMaxM rows, which only mf_factor_blk eliminates
            for (int s = 0; s < F.nsuper; ++s)
                if (F.k[s] + F.r[s] > kMfWaveMaxM && !F.fold_cnt.empty() && F.fold_cnt[s] > 0) {
                    err = "multifrontal: the blocked front kernel cannot get its LDS (needed by this plan's folds)";
                    return -2;
                }
        }
    }
    // program of every supernode: 1 = own (everything on one GPU), 2 = top, 0 = another rank's
    std::vector<int8_t> sel(F.nsuper, 1), fid_f(F.nsuper, 0), fid_b(F.nsuper, 0);
    if (owner)
        for (int s = 0; s < F.nsuper; ++s) sel[s] = owner[s] == rank ? 1 : owner[s] == -1 ? 2 : 0;
    int rc;
    if ((rc = build_prog(F, sel, 1, d->prog[0], fid_f, fid_b, err)) ||
        (owner && (rc = build_prog(F, sel, 2, d->prog[1], fid_f, fid_b, err))))
        return rc;
    if ((rc = up(&d->fid_f, fid_f, err)) || (rc = up(&d->fid_b, fid_b, err)) || (rc = up(&d->parent, F.parent, err)))
        return rc;
    {   // tagged hand-offs: a flow front whose parent is in the same flow publishes its update matrix
        // and u-vector as granule pairs; every ancestor of a backward-flow front publishes its x so
        std::vector<int64_t> ugo(F.nsuper, -1);
        int64_t ug_size = 0, ndof = 0;
        for (int c = 0; c < F.nsuper; ++c) {
            ndof = std::max<int64_t>(ndof, (int64_t)F.col0[c] + F.k[c]);
            const int p = F.parent[c];
            if (p < 0 || fid_f[c] == 0 || fid_f[p] != fid_f[c]) continue;
            const int64_t rc2 = F.r[c];
            ugo[c] = ug_size;
            ug_size += 2 * (rc2 * (rc2 + 1) / 2 + rc2);
        }
        std::vector<int8_t> xt(F.nsuper, 0);
        for (int c = 0; c < F.nsuper; ++c)
            if (fid_b[c] != 0)
                for (int q = c; q >= 0 && !xt[q]; q = F.parent[q]) xt[q] = 1;
        if ((rc = up(&d->ug_off, ugo, err)) || (rc = up(&d->xtag, xt, err))) return rc;
        auto alloc0 = [&](unsigned long long** p, int64_t n) -> int {
            n = std::max<int64_t>(n, 1) + 2 * kMfPad;
            if (hipMalloc((void**)p, n * sizeof(unsigned long long)) != hipSuccess ||
                hipMemset(*p, 0, n * sizeof(unsigned long long)) != hipSuccess) {
                err = "hipMalloc failed (multifrontal granules)";
                return -2;
            }
            return 0;
        };
        if ((rc = alloc0(&d->Ug, ug_size)) || (rc = alloc0(&d->xg, 2 * ndof))) return rc;
    }
    if (hipMalloc((void**)&d->tickets, 2 * kMfTickets * sizeof(int)) != hipSuccess ||
        hipMemset(d->tickets, 0, 2 * kMfTickets * sizeof(int)) != hipSuccess ||
        hipMalloc((void**)&d->epoch, sizeof(uint32_t)) != hipSuccess) {
        err = "hipMalloc failed (multifrontal flow)";
        return -2;
    }
    {
        const uint32_t one = 1;
        if (hipMemcpy(d->epoch, &one, sizeof(one), hipMemcpyHostToDevice) != hipSuccess) {
            err = "hipMemcpy failed (multifrontal epoch)";
            return -2;
        }
    }
    {   // extend-add positions of every child whose parent is a wave or blocked front (m <= kBlkMaxM)
        std::vector<int64_t> eoff(F.nsuper, 0);
        std::vector<int16_t> em;
        for (int c = 0; c < F.nsuper; ++c) {
            const int p = F.parent[c];
            if (p < 0) continue;
            const int mp = F.k[p] + F.r[p], rc = F.r[c];
            if (mp > kBlkMaxM || rc == 0) continue;
            bool folded = false;
            for (int ci = F.child_ptr[p]; ci < F.child_ptr[p] + (F.fold_cnt.empty() ? 0 : F.fold_cnt[p]); ++ci)
                folded = folded || F.child[ci] == c;
            if (folded) continue;
            eoff[c] = (int64_t)em.size();
            const int32_t* rm = F.rmap.data() + F.rmap_off[c];
            for (int j = 0; j < rc; ++j)
                for (int i = j; i < rc; ++i) {
                    const int I = rm[i], J = rm[j];
                    if (I < J || I >= mp) { err = "multifrontal: child row map not increasing"; return -1; }
                    // wave fronts: packed lower column-major; blocked fronts: full m x m column-major
                    em.push_back((int16_t)(mp <= kMfWaveMaxM ? J * mp - J * (J - 1) / 2 + (I - J) : I + J * mp));
                }
        }
        if ((rc = up(&d->emap, em, err)) || (rc = up(&d->emap_off, eoff, err))) return rc;
    }
    if ((rc = up(&d->col0, F.col0, err)) || (rc = up(&d->k, F.k, err)) ||
        (rc = up(&d->r, F.r, err)) || (rc = up(&d->child_ptr, F.child_ptr, err)) || (rc = up(&d->child, F.child, err)) ||
        (rc = up(&d->rmap, F.rmap, err)) || (rc = up(&d->amap_ptr, F.amap_ptr, err)) ||
        (rc = up(&d->amap_src, F.amap_src, err)) || (rc = up(&d->amap_dst, F.amap_dst, err)) ||
        (rc = up(&d->findex, F.findex, err)) || (rc = up(&d->L_off, F.L_off, err)) || (rc = up(&d->U_off, F.U_off, err)) ||
        (rc = up(&d->u_off, F.u_off, err)) || (rc = up(&d->scratch_off, scr, err)) ||
        (rc = up(&d->rmap_off, F.rmap_off, err)) || (rc = up(&d->findex_off, F.findex_off, err)) ||
        (rc = up(&d->fold_cnt, F.fold_cnt, err)) || (rc = up(&d->fold_cptr, F.fold_cptr, err)) ||
        (rc = up(&d->fold_chunk, F.fold_chunk, err)) || (rc = up(&d->fold_rec, F.fold_rec, err)))
        return rc;
    if (hipStreamCreateWithFlags(&d->side, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&d->side2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_join2, hipEventDisableTiming) != hipSuccess) {
        err = "side stream creation failed (multifrontal)";
        return -2;
    }
    auto alloc = [&](double** p, int64_t n) -> int {   // + kMfPad: clamped reads (up())
        if (n <= 0) n = 1;
        if (hipMalloc((void**)p, (n + kMfPad) * sizeof(double)) != hipSuccess) { err = "hipMalloc failed (multifrontal buffers)"; return -2; }
        if (hipMemset(*p, 0, (n + kMfPad) * sizeof(double)) != hipSuccess) { err = "hipMemset failed (multifrontal buffers)"; return -2; }
        return 0;
    };
    if ((rc = alloc(&d->L, F.L_size)) || (rc = alloc(&d->U, F.U_size)) || (rc = alloc(&d->u, F.u_size)) ||
        (rc = alloc(&d->scratch, scratch_size)))
        return rc;
    if (hipMalloc((void**)&d->info, sizeof(int32_t)) != hipSuccess) { err = "hipMalloc failed (info)"; return -2; }
    if (hipMemset(d->info, 0, sizeof(int32_t)) != hipSuccess) { err = "hipMemset failed"; return -2; }
    return 0;
}

void mf_destroy(MfDevice* d) {
    if (!d) return;
    free_prog(d->prog[0]);
    free_prog(d->prog[1]);
    void* bufs[] = {d->emap, d->emap_off, d->epoch, d->fid_f, d->fid_b, d->fold_cnt, d->fold_cptr, d->fold_chunk, d->fold_rec, d->parent,
                    d->tickets, d->col0, d->k, d->r, d->child_ptr, d->child, d->rmap, d->amap_ptr, d->amap_src,
                    d->amap_dst, d->findex, d->info, d->L_off, d->U_off, d->u_off, d->scratch_off, d->rmap_off,
                    d->findex_off, d->L, d->U, d->u, d->scratch, d->Ug, d->xg, d->ug_off, d->xtag};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (d->ev_fork) (void)hipEventDestroy(d->ev_fork);
    if (d->ev_join) (void)hipEventDestroy(d->ev_join);
    if (d->ev_join2) (void)hipEventDestroy(d->ev_join2);
    if (d->side) (void)hipStreamDestroy(d->side);
    if (d->side2) (void)hipStreamDestroy(d->side2);
    delete d;
}

// info is zero on entry: zeroed at creation and, after every iteration, by the end-of-step
// reduce_stats launch (mf_info_ptr). The work-queue tickets reset themselves (leave_flow). Every
// launch argument is fixed (the flows read the step's epoch from the device), so the sequence can be
// captured once into a hipGraph and replayed.
template <bool F32>
hipError_t mf_factor_t(MfDevice* d, int which, const double* A, double* x, hipStream_t s) {
    hipError_t e;
    const Prog& P = d->prog[which];
    if (P.ptr.empty()) return hipSuccess;
    for (int l = 0; l < std::min(P.flow_lev0, d->nlevels); ++l) {
        int n;
        // a level with blocked fronts and few fronts in all (config 2): one launch for all of them
#ifdef BOS_DIAG_PAIR
        const int n4 = P.count(l, 4), nwf = P.count(l, 0, 4) - P.count(l, 2) + (P.count(l, 2) + 1) / 2;
#else
        const int n4 = P.count(l, 4), nwf = P.count(l, 0, 4);
#endif
        if (kMixB && d->mixb && n4 > 0 && n4 + nwf <= d->ncu) {
            const int4 nw = make_int4(P.count(l, 0), P.count(l, 1), P.count(l, 2), P.count(l, 3));
            const int4 ow = make_int4(0, P.count(l, 0), P.count(l, 0, 2), P.count(l, 0, 3));
            hipLaunchKernelGGL((mf_factor_mixb<F32>), dim3(n4 + nwf), dim3(kMfBlock), std::max(P.lds_blk[l], kMixbWaveLds),
                               s, d->args(P, l, 0, A, x), d->args(P, l, 4, A, x).level, n4, nw, ow);
            if ((n = P.count(l, 5))) {   // fronts above kBlkMaxM rows (fallback plans)
                hipLaunchKernelGGL(mf_factor_level, dim3(n), dim3(kMfBlock), P.lds_factor[l * kClasses + 5], s,
                                   d->args(P, l, 5, A, x));
                hipLaunchKernelGGL(mf_forward_level, dim3(n), dim3(kMfBlock), P.lds_fwd[l * kClasses + 5], s,
                                   d->args(P, l, 5, A, x));
            }
            if ((e = hipGetLastError()) != hipSuccess) return e;
            continue;
        }
        const bool fork = d->side && P.count(l, 3) > 0;
        // the level's blocked fronts (config 2's separators: a few workgroups, each one latency-bound
        // front) on a second side stream, beside the wave fronts instead of after them
        const bool fork2 = d->side2 && d->blk && P.count(l, 4) > 0;
        // a handful of class-16 fronts (one latency-bound round, negligible load) follow them there
        const bool tiny16 = fork && P.count(l, 0) <= d->tiny16;
        if (fork || fork2) {
            if ((e = hipEventRecord(d->ev_fork, s)) != hipSuccess) return e;
        }
        if (fork2) {
            if ((e = hipStreamWaitEvent(d->side2, d->ev_fork, 0)) != hipSuccess) return e;
            hipLaunchKernelGGL((mf_factor_blk<F32>), dim3(P.count(l, 4)), dim3(kMfBlock), P.lds_blk[l], d->side2,
                               d->args(P, l, 4, A, x));
            if ((e = hipEventRecord(d->ev_join2, d->side2)) != hipSuccess) return e;
        }
        if (fork) {
            if ((e = hipStreamWaitEvent(d->side, d->ev_fork, 0)) != hipSuccess) return e;
            if (kPanel64)
                hipLaunchKernelGGL((mf_factor_pan<64, kPanelKP, F32>), dim3(P.count(l, 3)), dim3(64), 0, d->side,
                                   d->args(P, l, 3, A, x));
            else
                hipLaunchKernelGGL((mf_factor_reg<64, F32>), dim3(P.count(l, 3)), dim3(64), 0, d->side, d->args(P, l, 3, A, x));
            if (tiny16 && (n = P.count(l, 0)))
                hipLaunchKernelGGL((mf_factor_reg<16, F32>), dim3(n), dim3(64), 0, d->side, d->args(P, l, 0, A, x));
            if ((e = hipEventRecord(d->ev_join, d->side)) != hipSuccess) return e;
        }
        if ((n = P.count(l, 0)) && !tiny16)
            hipLaunchKernelGGL((mf_factor_reg<16, F32>), dim3(n), dim3(64), 0, s, d->args(P, l, 0, A, x));
        if ((n = P.count(l, 1))) hipLaunchKernelGGL((mf_factor_reg<32, F32>), dim3(n), dim3(64), 0, s, d->args(P, l, 1, A, x));
        if ((n = P.count(l, 2))) {
            if (kPanel48)
                hipLaunchKernelGGL((mf_factor_pan<48, kPanelKP, F32>), dim3(n), dim3(64), 0, s, d->args(P, l, 2, A, x));
            else
                hipLaunchKernelGGL((mf_factor_reg<48, F32>), dim3(n), dim3(64), 0, s, d->args(P, l, 2, A, x));
        }
        if ((n = P.count(l, 3)) && !fork) {
            if (kPanel64)
                hipLaunchKernelGGL((mf_factor_pan<64, kPanelKP, F32>), dim3(n), dim3(64), 0, s, d->args(P, l, 3, A, x));
            else
                hipLaunchKernelGGL((mf_factor_reg<64, F32>), dim3(n), dim3(64), 0, s, d->args(P, l, 3, A, x));
        }
        if (fork && (e = hipStreamWaitEvent(s, d->ev_join, 0)) != hipSuccess) return e;
        if (fork2 && (e = hipStreamWaitEvent(s, d->ev_join2, 0)) != hipSuccess) return e;
        // larger fronts: up to kBlkMaxM rows the blocked workgroup kernel (MFMA; folds; forward step fused),
        // above it (fallback plans) the unblocked workgroup kernel in global scratch and its forward step
        for (int c = fork2 ? 5 : 4; c < kClasses; ++c) {
            if (!(n = P.count(l, c))) continue;
            if (c == 4 && d->blk) {
                hipLaunchKernelGGL((mf_factor_blk<F32>), dim3(n), dim3(kMfBlock), P.lds_blk[l], s, d->args(P, l, 4, A, x));
            } else {
                hipLaunchKernelGGL(mf_factor_level, dim3(n), dim3(kMfBlock), P.lds_factor[l * kClasses + c], s,
                                   d->args(P, l, c, A, x));
                hipLaunchKernelGGL(mf_forward_level, dim3(n), dim3(kMfBlock), P.lds_fwd[l * kClasses + c], s,
                                   d->args(P, l, c, A, x));
            }
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (P.n_flow_factor > 0) {
        const Flow f{P.order_factor, P.n_flow_factor, d->tickets, d->tickets + kMfTickets, d->epoch, 0u,
                     d->fid_f, P.id, d->stamps};
        const int grid = std::min(P.n_flow_factor, d->ncu * kFlowWavesFactor);
        hipLaunchKernelGGL((mf_factor_flow<F32>), dim3(grid), dim3(64), 0, s, d->args(P, 0, 0, A, x), f);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t mf_factor(MfDevice* d, int which, const double* A, double* x, hipStream_t s) {
    return d->A32 ? mf_factor_t<true>(d, which, A, x, s) : mf_factor_t<false>(d, which, A, x, s);
}

void mf_set_fold_source(MfDevice* d, const float* A32, int64_t pl_lo) {
    d->A32 = A32;
    d->pl_lo = pl_lo;
}

hipError_t mf_solve(MfDevice* d, int which, double* x, hipStream_t s) {
    // backward substitution (the forward one ran inside mf_factor): one flow launch over the levels
    // >= solve_lev0 (top-down), then per-level launches below it
    hipError_t e;
    const Prog& P = d->prog[which];
    if (P.ptr.empty()) return hipSuccess;
    if (P.flow_solve) {
        const Flow fb{P.order_bwd, P.n_flow_solve, d->tickets + 1, d->tickets + kMfTickets + 1,
                      d->epoch, 0u, d->fid_b, P.id, d->stamps ? d->stamps + 8 * (int64_t)d->nsuper : nullptr};
        const int grid = std::min(P.n_flow_solve, d->ncu * kFlowWavesBackward);
        hipLaunchKernelGGL(mf_backward_flow, dim3(grid), dim3(64), P.lds_bwd_flow, s, d->args(P, 0, 0, nullptr, x), fb,
                           (const int32_t*)d->parent);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    for (int l = std::min(P.solve_lev0, d->nlevels) - 1; l >= 0; --l) {
        int n;
        if (P.bptr[l + 1] > P.bptr[l]) {
            MfArgs g = d->args(P, l, 0, nullptr, x);
            g.level = P.blist + P.bptr[l];
            g.count = P.bptr[l + 1] - P.bptr[l];
            hipLaunchKernelGGL(mf_backward_wave, dim3(g.count), dim3(64), P.blds[l], s, g);
        }
        if ((n = P.count(l, 4, kClasses))) {   // the workgroup fronts (classes 4 and 5, one list)
            MfArgs g = d->args(P, l, 4, nullptr, x);
            g.count = n;
            hipLaunchKernelGGL(mf_backward_level, dim3(n), dim3(kMfBlock), P.lds_max(P.lds_bwd, l, 4, kClasses), s, g);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (P.n_fold > 0) {   // folded landmarks last: their rows are poses, final by now
        MfArgs g = d->args(P, 0, 0, nullptr, x);
        g.level = P.fold_list;
        g.count = P.n_fold;
        hipLaunchKernelGGL(mf_backward_fold, dim3(((int64_t)P.n_fold * kFoldLanes + kMfBlock - 1) / kMfBlock), dim3(kMfBlock), 0, s, g);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

int32_t* mf_info_ptr(const MfDevice* d) { return d->info; }
uint32_t* mf_epoch_ptr(const MfDevice* d) { return d->epoch; }
void mf_debug_set_stamps(MfDevice* d, unsigned long long* stamps) {
    d->stamps = stamps;
#ifdef BOS_MF_PIVOT_CYCLES
    unsigned long long* b = stamps ? stamps + 8 * (int64_t)d->nsuper : nullptr;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pivot_bwd), &b, sizeof(b));
#endif
}
int32_t* mf_tickets_ptr(const MfDevice* d) { return d->tickets; }
double* mf_update_ptr(const MfDevice* d) { return d->U; }
double* mf_uvec_ptr(const MfDevice* d) { return d->u; }

hipError_t mf_debug_skip_next_front(MfDevice* d, hipStream_t s) {
    // only where a front of the same launch waits for the skipped one (otherwise nothing would notice
    // the skip and the step would use the front's previous outputs)
    if (d->prog[0].n_flow_factor == 0 || !d->prog[0].first_waited) return hipErrorInvalidValue;
    static const int one = 1;
    return hipMemcpyAsync(d->tickets, &one, sizeof(int), hipMemcpyHostToDevice, s);
}

}  // namespace dev
}  // namespace bos
