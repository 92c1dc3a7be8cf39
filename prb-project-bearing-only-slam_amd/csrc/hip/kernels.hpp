// Device-side parameter blocks and launch wrappers of the GN kernels (hip/kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace bos {
namespace dev {

// One wavefront processes one task of a work list (host/plan.hpp WorkList).
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = 64 * kWavesPerBlock;

template <typename T> struct LinParams {
    // state caches (T precision), refreshed by the box-plus kernel
    const T* pc;          // [NP][4] x, y, cos(theta), sin(theta)
    const T* pth;         // [NP] theta
    const T* lc;          // [NL][2]
    // pose-centric work list
    int ntask_pose, nblk_pose;
    const int32_t* a_task;
    const int32_t* a_seg_item;
    const int32_t* a_seg_node;
    const int32_t* a_other;
    const int32_t* a_slot;
    const int32_t* a_grp;     // may be null when the list has no groups
    const T* a_z;
    const T* a_w;             // null => omega = 1
    // landmark-centric work list
    int ntask_lm;
    const int32_t* b_task;
    const int32_t* b_seg_item;
    const int32_t* b_seg_node;
    const int32_t* b_other;
    const int32_t* b_slot;
    const int32_t* b_grp;
    const T* b_z;
    const T* b_w;
    // odometry edges
    const int32_t* o_src;
    const int32_t* o_dst;
    const T* o_z;             // [M_o][3]
    const T* o_om;            // [M_o][6] upper triangle (00, 01, 02, 11, 12, 22)
    // node layout
    const int32_t* p_row0;
    const int32_t* p_base;
    const int32_t* p_bpos;
    const int32_t* l_row0;
    const int32_t* l_base;
    const int32_t* l_bpos;
    // outputs
    T* val;                   // lower triangle of P^T H_nf P (CSR value array)
    T* b;                     // [n + 3], permuted dof order, fixed pose last
    double* chi2_part;        // [ntask_pose]
    int32_t* nrob_part;       // [ntask_pose]
    T kt;                     // robust kernel threshold
    T lambda;                 // damping
};

template <typename T> struct UpdateParams {
    int NP, NL, fixed;
    const int32_t* node_dof;  // [NP + NL]
    const double* x;          // solution of H_nf x = b_nf (dx = -x)
    double* pose;             // [NP][3] master state, fp64
    double* lm;               // [NL][2]
    T* pc;
    T* pth;
    T* lc;
    unsigned long long* max_dx_bits;   // max |dx| as ordered bits of a non-negative double
};

template <typename T>
hipError_t launch_linearize(const LinParams<T>& p, bool has_w, bool has_groups, hipStream_t s);
template <typename T> hipError_t launch_refresh_cache(const UpdateParams<T>& p, hipStream_t s);
template <typename T> hipError_t launch_boxplus(const UpdateParams<T>& p, hipStream_t s);
hipError_t launch_reduce_stats(const double* chi_part, const int32_t* nrob_part, int n, double* chi_out,
                               int32_t* nrob_out, hipStream_t s);
template <typename T> hipError_t launch_to_f64(const T* in, double* out, int64_t n, hipStream_t s);
hipError_t launch_scatter_dense(const int32_t* rowptr, const int32_t* colind, const double* val, int n, double* dense,
                                hipStream_t s);

}  // namespace dev
}  // namespace bos
