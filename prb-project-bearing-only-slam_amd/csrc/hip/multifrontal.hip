// GPU supernodal multifrontal Cholesky for the GN normal system (replaces the reference's
// Eigen SimplicialLDLT, slam/solver.cpp:75-85; pattern analysed once like analyzePattern at
// :77-80 — here the symbolic analysis is host/plan.cpp build_multifrontal).
//
// H_nf (already in nested-dissection order, lower CSR) = L L^T. The assembly tree is processed
// level by level (leaves first): one launch per level, one workgroup per supernode. A workgroup
//   1. zeroes its dense front F (m x m, column-major, in LDS when it fits, else global scratch),
//   2. scatters its entries of H (precomputed map) and extend-adds its children's update
//      matrices (children sequentially, entries in parallel: deterministic),
//   3. runs a right-looking partial Cholesky of its k own columns,
//   4. writes the m x k panel of L and the r x r update matrix for its parent.
// Forward (bottom-up) and backward (top-down) substitutions use the same tree and levels.
// Everything is fp64 and deterministic (no atomics on values).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "../host/plan.hpp"
#include "multifrontal.hpp"

namespace bos {
namespace dev {

namespace {

constexpr int kMfBlock = 256;
constexpr int kLdsCapM = 90;   // fronts up to 90 x 90 doubles (64.8 KB) are factored in LDS

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
    double* L;
    double* U;
    double* u;
    double* scratch;
    double* x;                   // rhs in, solution out (permuted order)
    int32_t* info;               // count of non-positive pivots
};

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
        const int64_t n2 = (int64_t)rc * rc;
        for (int64_t e = tid; e < n2; e += kMfBlock) {
            const int i = (int)(e % rc), j = (int)(e / rc);
            if (i >= j) F[map[i] + (int64_t)map[j] * m] += Uc[e];
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
    const int64_t nU = (int64_t)r * r;
    for (int64_t e = tid; e < nU; e += kMfBlock) {
        const int i = (int)(e % r), j = (int)(e / r);
        Us[e] = F[(k + i) + (int64_t)(k + j) * m];
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
}

template <typename X> int up(X** p, const std::vector<X>& v, std::string& err) {
    *p = nullptr;
    if (v.empty()) return 0;
    if (hipMalloc((void**)p, v.size() * sizeof(X)) != hipSuccess) { err = "hipMalloc failed (multifrontal)"; return -2; }
    if (hipMemcpy(*p, v.data(), v.size() * sizeof(X), hipMemcpyHostToDevice) != hipSuccess) {
        err = "hipMemcpy failed (multifrontal)";
        return -2;
    }
    return 0;
}

}  // namespace

struct MfDevice {
    int nlevels = 0;
    std::vector<int32_t> level_ptr;
    std::vector<int> level_lds_factor, level_lds_fwd, level_lds_bwd;
    int32_t *level = nullptr, *col0 = nullptr, *k = nullptr, *r = nullptr, *child_ptr = nullptr, *child = nullptr,
            *rmap = nullptr, *amap_ptr = nullptr, *amap_src = nullptr, *amap_dst = nullptr, *findex = nullptr,
            *info = nullptr;
    int64_t *L_off = nullptr, *U_off = nullptr, *u_off = nullptr, *scratch_off = nullptr, *rmap_off = nullptr,
            *findex_off = nullptr;
    double *L = nullptr, *U = nullptr, *u = nullptr, *scratch = nullptr;

    MfArgs args(int lev, const double* A, double* x) const {
        MfArgs g;
        g.level = level + level_ptr[lev];
        g.count = level_ptr[lev + 1] - level_ptr[lev];
        g.col0 = col0; g.k = k; g.r = r; g.L_off = L_off; g.U_off = U_off; g.u_off = u_off;
        g.scratch_off = scratch_off; g.child_ptr = child_ptr; g.child = child; g.rmap_off = rmap_off; g.rmap = rmap;
        g.amap_ptr = amap_ptr; g.amap_src = amap_src; g.amap_dst = amap_dst; g.findex_off = findex_off;
        g.findex = findex; g.A = A; g.L = L; g.U = U; g.u = u; g.scratch = scratch; g.x = x; g.info = info;
        return g;
    }
};

int mf_create(const Multifrontal& F, MfDevice** out, std::string& err) {
    MfDevice* d = new MfDevice();
    *out = d;
    d->nlevels = F.nlevels;
    d->level_ptr = F.level_ptr;
    std::vector<int64_t> scr(F.nsuper, -1);
    int64_t scratch_size = 0;
    for (int s = 0; s < F.nsuper; ++s) {
        const int m = F.k[s] + F.r[s];
        if (m > kLdsCapM) { scr[s] = scratch_size; scratch_size += (int64_t)m * m; }
    }
    d->level_lds_factor.assign(F.nlevels, 0);
    d->level_lds_fwd.assign(F.nlevels, 0);
    d->level_lds_bwd.assign(F.nlevels, 0);
    for (int l = 0; l < F.nlevels; ++l)
        for (int q = F.level_ptr[l]; q < F.level_ptr[l + 1]; ++q) {
            const int s = F.level[q];
            const int m = F.k[s] + F.r[s];
            if (m <= kLdsCapM) d->level_lds_factor[l] = std::max(d->level_lds_factor[l], m * m * 8);
            d->level_lds_fwd[l] = std::max(d->level_lds_fwd[l], m * 8);
            d->level_lds_bwd[l] = std::max(d->level_lds_bwd[l], 2 * F.k[s] * 8);
        }
    int rc = 0;
    if ((rc = up(&d->level, F.level, err)) || (rc = up(&d->col0, F.col0, err)) || (rc = up(&d->k, F.k, err)) ||
        (rc = up(&d->r, F.r, err)) || (rc = up(&d->child_ptr, F.child_ptr, err)) || (rc = up(&d->child, F.child, err)) ||
        (rc = up(&d->rmap, F.rmap, err)) || (rc = up(&d->amap_ptr, F.amap_ptr, err)) ||
        (rc = up(&d->amap_src, F.amap_src, err)) || (rc = up(&d->amap_dst, F.amap_dst, err)) ||
        (rc = up(&d->findex, F.findex, err)) || (rc = up(&d->L_off, F.L_off, err)) || (rc = up(&d->U_off, F.U_off, err)) ||
        (rc = up(&d->u_off, F.u_off, err)) || (rc = up(&d->scratch_off, scr, err)) ||
        (rc = up(&d->rmap_off, F.rmap_off, err)) || (rc = up(&d->findex_off, F.findex_off, err)))
        return rc;
    auto alloc = [&](double** p, int64_t n) -> int {
        if (n <= 0) n = 1;
        if (hipMalloc((void**)p, n * sizeof(double)) != hipSuccess) { err = "hipMalloc failed (multifrontal buffers)"; return -2; }
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
    void* bufs[] = {d->level, d->col0, d->k, d->r, d->child_ptr, d->child, d->rmap, d->amap_ptr, d->amap_src,
                    d->amap_dst, d->findex, d->info, d->L_off, d->U_off, d->u_off, d->scratch_off, d->rmap_off,
                    d->findex_off, d->L, d->U, d->u, d->scratch};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    delete d;
}

hipError_t mf_factor(MfDevice* d, const double* A, hipStream_t s) {
    hipError_t e = hipMemsetAsync(d->info, 0, sizeof(int32_t), s);
    if (e != hipSuccess) return e;
    for (int l = 0; l < d->nlevels; ++l) {
        const int n = d->level_ptr[l + 1] - d->level_ptr[l];
        if (!n) continue;
        hipLaunchKernelGGL(mf_factor_level, dim3(n), dim3(kMfBlock), d->level_lds_factor[l], s, d->args(l, A, nullptr));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t mf_solve(MfDevice* d, double* x, hipStream_t s) {
    hipError_t e;
    for (int l = 0; l < d->nlevels; ++l) {
        const int n = d->level_ptr[l + 1] - d->level_ptr[l];
        if (!n) continue;
        hipLaunchKernelGGL(mf_forward_level, dim3(n), dim3(kMfBlock), d->level_lds_fwd[l], s, d->args(l, nullptr, x));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    for (int l = d->nlevels - 1; l >= 0; --l) {
        const int n = d->level_ptr[l + 1] - d->level_ptr[l];
        if (!n) continue;
        hipLaunchKernelGGL(mf_backward_level, dim3(n), dim3(kMfBlock), d->level_lds_bwd[l], s, d->args(l, nullptr, x));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

const int32_t* mf_info_ptr(const MfDevice* d) { return d->info; }

}  // namespace dev
}  // namespace bos
