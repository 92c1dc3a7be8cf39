// Device-side parameter blocks and launch wrappers of the GN kernels (hip/kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace bos {
namespace dev {

// One wavefront processes one task of a work list (host/plan.hpp WorkList).
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = 64 * kWavesPerBlock;

// LDS staging capacities of one wavefront (must match host/plan.cpp kStageCap / kMaxTaskNodes)
constexpr int kStageCap = 1024;      // CSR values of a task's rows
constexpr int kBCap = 144;           // b entries of a task (<= kMaxTaskNodes x 3)
constexpr int kSlots = 128;          // contribution slots: 2 sides x 64 entries
constexpr int kMaxTaskNodes = 48;    // nodes of one multi-node task (host/plan.cpp kMaxTaskNodes)

template <typename T> struct LinParams {
    // state caches (T precision), refreshed by the box-plus kernel
    const T* pc;          // [NP][4] x, y, cos(theta), sin(theta)
    const T* pth;         // [NP] theta
    const T* lc;          // [NL][2]
    int NP;
    // node-range tasks (host/plan.hpp RangeTasks)
    int ntask;
    const int32_t* task_q;
    const int32_t* task_be;
    const int32_t* task_oe;
    const uint8_t* task_flags;
    const int32_t* be_pose;
    const int32_t* be_lm;
    const int32_t* be_meta;
    const T* be_z;
    const T* be_w;        // null => omega = 1
    const T* be_woff;     // duplicate groups only
    const int32_t* oe_edge;
    const int32_t* oe_meta;
    const T* oe_omoff;    // duplicate groups only
    const int32_t* o_src;
    const int32_t* o_dst;
    const T* o_z;         // [M_o][3]
    const T* o_om;        // [M_o][6] upper triangle (00, 01, 02, 11, 12, 22)
    const int32_t* pos_node;
    const int32_t* pos_row0;
    const int32_t* pos_base;
    const int32_t* pos_dof;
    const int32_t* node_base;   // per node id (pose stix, NP + landmark stix)
    const int32_t* cl_ptr;
    const uint16_t* cl;
    // outputs
    T* val;               // lower triangle of P^T H_nf P (CSR value array)
    T* b;                 // [n + 3], permuted dof order, fixed pose last (not written)
    double* chi2_part;    // [ntask]
    int32_t* nrob_part;   // [ntask]
    T kt;                 // robust kernel threshold
    T lambda;             // damping
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
hipError_t launch_linearize(const LinParams<T>& p, bool has_w, bool has_dups, hipStream_t s);
template <typename T> hipError_t launch_refresh_cache(const UpdateParams<T>& p, hipStream_t s);
template <typename T> hipError_t launch_boxplus(const UpdateParams<T>& p, hipStream_t s);
hipError_t launch_reduce_stats(const double* chi_part, const int32_t* nrob_part, int n, double* chi_out,
                               int32_t* nrob_out, hipStream_t s);
template <typename T> hipError_t launch_to_f64(const T* in, double* out, int64_t n, hipStream_t s);
hipError_t launch_scatter_dense(const int32_t* rowptr, const int32_t* colind, const double* val, int n, double* dense,
                                hipStream_t s);

}  // namespace dev
}  // namespace bos
