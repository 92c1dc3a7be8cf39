// Static structure of the GN normal system, built once per solver handle (bos_create).
//
// The reference rebuilds H from scratch every iteration with Eigen sparse additions
// (slam/solver.cpp:28-69) and runs SimplicialLDLT::analyzePattern once (:77-80). Here the
// pattern is fixed up front: H_nf (the fixed pose's rows/cols removed, solver.cpp:71-73) is laid
// out as the lower triangle of P^T H_nf P in CSR, where P is a fill-reducing node ordering, so
// the J+H kernels scatter straight into the array the sparse Cholesky consumes (no per-step
// permutation pass), and every observation knows its destination slots in advance.
//
// Nodes: pose stix u in [0, NP) (3 dofs), landmark stix l as node NP + l (2 dofs).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace bos {

struct ProblemIndex {
    int NP = 0, NL = 0, Mb = 0, Mo = 0, fixed = -1;
    const int32_t* b_pose = nullptr;
    const int32_t* b_lm = nullptr;
    const int32_t* o_src = nullptr;
    const int32_t* o_dst = nullptr;
    const double* b_omega = nullptr;   // [Mb] or null (= 1)
    const double* o_omega = nullptr;   // [Mo * 9]
};

// Work of the J+H kernel (hip/kernels.hip). A task is one wavefront and owns a contiguous
// range of elimination positions [task_q[t], task_q[t + 1]): its CSR rows are the contiguous
// value range [pos_row0[q0], pos_row0[q1]) and its b entries [pos_dof[q0], pos_dof[q1]), which
// the wavefront assembles in LDS and stores with coalesced writes. Entries are the observations
// incident to the task's nodes (an observation whose two endpoints lie in different tasks
// appears in both). meta bits: 0 = first endpoint (pose / src) inside, 1 = second endpoint
// (landmark / dst) inside, 2 = count this observation in chi^2, 3 = write the off-diagonal
// block, 4 = the owner (row side) of that block is the second endpoint; bits 8.. = offset of
// the block's first entry relative to the task's first value.
struct RangeTasks {
    std::vector<int32_t> task_q;        // [ntask + 1] position ranges
    std::vector<int32_t> task_be;       // [ntask + 1] bearing-entry ranges
    std::vector<int32_t> task_oe;       // [ntask + 1] odometry-entry ranges
    std::vector<uint8_t> task_flags;    // bit 0: rows staged in LDS; bit 1: single node (chunked)
    std::vector<int32_t> be_pose, be_lm, be_meta, be_obs;
    std::vector<double> be_woff;        // off-block weight (sum over duplicate group; 0 = no write)
    std::vector<int32_t> oe_edge, oe_meta;
    std::vector<double> oe_omoff;       // [6 per entry] off-block information (duplicate groups)
    std::vector<int32_t> cl_ptr;        // [m + 1] per position: range into cl
    std::vector<uint16_t> cl;           // contribution slots (2 * entry + side, entry local to the task)
    bool has_dups = false;
    int max_entries = 0;
    int ntask() const { return task_q.empty() ? 0 : (int)task_q.size() - 1; }
    int nentries() const { return (int)be_pose.size() + (int)oe_edge.size(); }
};

struct OrderingReport {
    std::string chosen;                // "temporal" or "nested-dissection"
    double flops_temporal = 0, flops_nd = 0;
    int64_t nnz_temporal = 0, nnz_nd = 0;
};

// Supernodal multifrontal Cholesky structure (GPU solver, hip/multifrontal.hip). Supernodes are
// the blocks of the nested-dissection ordering (contiguous position ranges); the assembly tree
// links each supernode to the one holding the first row of its update matrix. Fronts are dense,
// column-major, index list = [k own dofs | r update rows].
struct Multifrontal {
    int nsuper = 0, nlevels = 0, max_m = 0;
    std::vector<int32_t> col0, k, r;        // per supernode: first dof, #own dofs, #update rows
    std::vector<int64_t> findex_off;        // into findex (m = k + r entries; first k = col0..col0+k-1)
    std::vector<int32_t> findex;
    std::vector<int64_t> L_off;             // dense m x k panel (col-major) in the factor buffer
    std::vector<int64_t> U_off;             // dense r x r update matrix (col-major)
    std::vector<int64_t> u_off;             // r-vector (forward solve update)
    std::vector<int32_t> parent;            // -1 for roots
    std::vector<int32_t> child_ptr, child;  // children CSR
    std::vector<int64_t> rmap_off;          // per supernode: r positions of its rows in the parent's front
    std::vector<int32_t> rmap;
    std::vector<int32_t> amap_ptr;          // per supernode: range into amap_src / amap_dst
    std::vector<int32_t> amap_src, amap_dst;// value index in the CSR of H -> column-major front position
    std::vector<int32_t> level_ptr, level;  // supernodes grouped by tree level (leaves first)
    int64_t L_size = 0, U_size = 0, u_size = 0;
    double flops = 0;
};

struct Plan {
    int NP = 0, NL = 0, Mb = 0, Mo = 0, fixed = -1;
    int64_t n = 0;                         // system size N - 3
    std::vector<int32_t> node_pos;         // elimination position; -1 for the fixed pose
    std::vector<int32_t> node_dof;         // first dof in the permuted system; fixed pose -> n
    std::vector<int32_t> node_row0;        // CSR position of the node's first row start; -1 fixed
    std::vector<int32_t> node_base;        // entries before the diagonal block in each of its rows
    std::vector<int32_t> rowptr, colind;   // lower triangle of P^T H_nf P, n rows
    std::vector<int32_t> Lptr, Lind;       // symbolic Cholesky factor (lower, with diagonal)
    Multifrontal mf;                       // built when factor_mode == kFactorMultifrontal
    RangeTasks tasks;
    std::vector<int32_t> pos_node, pos_row0, pos_base, pos_dof;   // per elimination position
    OrderingReport ordering;
    // ownership for observation sharding: this rank writes rows [row_begin, row_end)
    int32_t row_begin = 0, row_end = 0;
    int64_t val_begin = 0, val_end = 0;
    std::vector<int32_t> rank_row_begin;   // [world + 1] row split of every rank
    int64_t nnzA() const { return rowptr.empty() ? 0 : rowptr.back(); }
    int64_t nnzL() const { return Lptr.empty() ? 0 : Lptr.back(); }
};

enum FactorMode {
    kFactorNone = 0,          // dense solver: pattern only
    kFactorScalar = 1,        // scalar CSR Cholesky pattern (rocSOLVER csrrf), cheapest-flops ordering
    kFactorMultifrontal = 2,  // nested dissection + supernodal multifrontal structure (GPU solver)
};

// Builds the plan. Returns 0 or a negative BOS_ERR_* code with a message in err.
int build_plan(const ProblemIndex& pi, int rank, int world, int factor_mode, Plan& out, std::string& err);

// Node ordering only (positions) and its symbolic cost. nd_only: force nested dissection and
// return its blocks (contiguous position ranges: leaves and separators) in `blocks`.
int order_nodes(const ProblemIndex& pi, bool nd_only, std::vector<int32_t>& node_pos,
                std::vector<std::pair<int32_t, int32_t>>* blocks, OrderingReport& rep, std::string& err);

}  // namespace bos
