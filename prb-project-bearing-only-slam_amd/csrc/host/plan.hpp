// Static structure of the GN normal system, built once per solver handle (bos_create).
//
// The reference rebuilds H from scratch every iteration with Eigen sparse additions
// (slam/solver.cpp:28-69) and runs SimplicialLDLT::analyzePattern once (:77-80). Here the
// structure is fixed up front: the J+H kernel writes H block-sparse in observation order
// (BlockLayout), every value exactly once; the solver sees H_nf (the fixed pose's rows/cols
// removed, solver.cpp:71-73) as the lower triangle of P^T H_nf P, P a fill-reducing node ordering,
// through index maps into the block array (no per-step assembly or permutation pass).
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
    // planning options (bos_options): J+H lanes per pose (0 = by the bearings per pose) and poses per
    // nested-dissection leaf of the Schur ordering (0 = kSchurLeaf)
    int lpp = 0;
    int schur_leaf = 0;
};

// J+H launch geometry shared by the host plan and the kernel (hip/kernels.hpp kBlock)
constexpr int kJhBlock = 256;
// some (pose, landmark) bearing pair or (pose, pose) odometry pair occurs twice (plan.cpp)
bool duplicate_pairs(const ProblemIndex& pi);
// J+H lanes per pose: bos_options.lanes_per_pose when set, else 2 from 32 bearings per pose on, 2 on
// a sharded rank (world > 1) when there are no duplicate pairs, and 1 otherwise. Without duplicate
// pairs two or four lanes per pose interleave a pose's bearings and compute H and b bit for bit as
// one lane does (kernels.hip pose_lanes); a rank's share leaves the GPU with few waves, where two
// lanes halve each pose's chain (config 3, per rank in-step J+H: W = 2 15 -> 13 us, W = 8 14 -> 11
// us), while on one GPU one lane is fastest (17 against 20 and 25 us with two and four). build_layout
// and build_shard both use this.
inline int plan_lanes_per_pose(const ProblemIndex& pi, int world) {
    const double avg = pi.NP ? (double)pi.Mb / pi.NP : 0.0;
    if (pi.lpp > 0) return pi.lpp;
    if (avg >= 32) return 2;
    return world > 1 && !duplicate_pairs(pi) ? 2 : 1;
}
// Contiguous share [a, b) of n items for rank r of W (BOS_PARTITION_OBSERVATIONS: each rank runs a
// range of the J+H's pose blocks and one of its landmark blocks, i.e. of the observations in
// measurement order)
inline void split_range(int64_t n, int r, int W, int64_t& a, int64_t& b) {
    a = n * r / W;
    b = n * (r + 1) / W;
}

// Block-sparse storage of H that the J+H kernel (hip/kernels.hip) writes, in observation order
// rather than in the solver's order (the solver reads it through index maps: Multifrontal::amap_src
// and csr_src). One array of T:
//   [0, off_ldiag)        pose diagonal blocks, 6 per pose, lower triangle (00, 10, 11, 20, 21, 22)
//   [off_ldiag, off_pl)   landmark diagonal blocks, 3 per landmark (00, 10, 11)
//   [off_pl, off_pp)      pose-landmark blocks H_pl (3 x 2 row-major), 6 values per bearing slot
//                         (below); a pair observed more than once uses the slot of its last bearing
//   [off_pp, size)        pose-pose blocks, one per unordered pair {p < q} joined by odometry edges
//                         (either direction), ordered by p then q: the sum of the edges' H_sd =
//                         -J_s^T Omega J_s, symmetric (J_d = -J_s), so 6 values like a diagonal block
// b stays in the reference dof numbering (3 per pose, then 2 per landmark; the fixed pose's entries
// are computed but not used). Diagonal blocks and b include all nodes, the fixed pose too.
//
// Work: lpp lanes per pose (lane g = pose * lpp + sub), one lane per landmark; lanes form waves of
// 64. A lane walks a list of bearings (pose lanes: a segment of the pose's bearings sorted by
// landmark, so duplicates of one pair are adjacent and merged by one lane; lane 0 of a pose also
// walks its odometry entries). The lists are stored wave-interleaved: item j of lane t of wave w
// sits in slot w_base[w] + w_stride[w] j + t, so each step of a wave reads 64 consecutive records
// and writes 64 consecutive blocks (whole cache lines). Consecutive waves with the same list length
// form a group stored step-major (w_stride = 64 x the group's waves): the waves of a group, which run
// their steps side by side, then read and write one contiguous stretch per step (HBM page locality)
// instead of one stretch per wave.
struct LaneLists {
    std::vector<int32_t> w_base;    // [waves + 1] slot of item 0 of lane 0 of each wave; [waves] = slots
    std::vector<int32_t> w_stride;  // [waves] slots between items j and j + 1 of a lane
    std::vector<int32_t> w_len;     // [waves] items per lane in the wave (max over its lanes)
    std::vector<int32_t> cnt;       // [lanes] items of each lane
    std::vector<int32_t> obs;       // [slots] bearing in each slot, -1 = padding
    int64_t slots() const { return w_base.empty() ? 0 : w_base.back(); }
    int32_t slot(int g, int j) const { return w_base[g / 64] + w_stride[g / 64] * j + (g & 63); }
};

constexpr int kLmWindow = 256;   // landmark lanes are permuted only inside aligned windows of this size

struct BlockLayout {
    int64_t off_ldiag = 0, off_pl = 0, off_pp = 0, size = 0;
    int lpp = 1;                        // lanes per pose: 1, 2 or 4
    bool interleaved = false;           // lpp > 1 without duplicate pairs: items dealt round robin
    bool has_dups = false;              // some (pose, landmark) or (src, dst) pair repeats
    // pose lane groups: group i (lanes i * lpp ... + lpp - 1) runs pose lane_pose[i] (-1: padding);
    // one rank runs the poses of Shard::lane_poses (all poses in stix order on one GPU)
    std::vector<int32_t> lane_pose;
    LaneLists pose_lanes;               // lanes = lane_pose.size() * lpp
    LaneLists lm_lanes;                 // lane g -> landmark lm_lane_lm[g]
    // landmark of each landmark lane (Shard::lane_lms): inside each window of kLmWindow lanes the
    // window's landmarks sorted by consecutive-pose lanes first, then degree (descending), so the
    // lanes of a wave take one path and walk lists of similar length
    std::vector<int32_t> lm_lane_lm;
    // [lanes] the landmark lane's first pose when its poses are consecutive stix (p0, p0 + 1, ...,
    // no repeated pose), else -1 (LinParams::ll_run)
    std::vector<int32_t> lm_lane_run;
    std::vector<int32_t> ub_ptr;        // [NP + 1] pose-landmark blocks of each pose
    std::vector<int32_t> ub_lm;         // [nub] landmark of each pose-landmark block (ascending per pose)
    std::vector<int32_t> ub_slot;       // [nub] bearing slot holding the block
    std::vector<int32_t> po_ptr;        // [NP + 1] odometry entries of each pose (self-loops have none)
    std::vector<int32_t> po_ent;        // edge << 1 | 1 when the pose is the destination; per pose
                                        // sorted by (other pose, edge)
    std::vector<int32_t> po_blk;        // pose-pose block an entry adds to when the other pose is the
                                        // higher one (this pose stores it), else -1
    // [NP] 1: the pose's odometry entries are exactly edge p - 1 = (p - 1, p) seen from its
    // destination and edge p = (p, p + 1) from its source (a chain pose: the J+H derives them from p)
    std::vector<uint8_t> po_chain;
    std::vector<int32_t> uo_ptr;        // [NP + 1] pose-pose blocks stored by each pose (the lower one)
    std::vector<int32_t> uo_dst;        // [nuo] the higher pose of each pose-pose block
    std::vector<int32_t> csr_src;       // [nnzA] block value of each stored entry of P^T H_nf P; -2 when
                                        // this rank's J+H does not compute it (sharded plans)
    int nub() const { return ub_ptr.empty() ? 0 : ub_ptr.back(); }
    int nuo() const { return uo_ptr.empty() ? 0 : uo_ptr.back(); }
    int poses_per_wave() const { return 64 / lpp; }
    int64_t pose_blocks() const { return ((int64_t)lane_pose.size() * lpp + kJhBlock - 1) / kJhBlock; }
    int64_t lm_blocks() const { return ((int64_t)lm_lane_lm.size() + kJhBlock - 1) / kJhBlock; }
};


struct OrderingReport {
    std::string chosen;                // "temporal" or "nested-dissection"
    double flops_temporal = 0, flops_nd = 0;
    int64_t nnz_temporal = 0, nnz_nd = 0;
};

// Supernodal multifrontal Cholesky structure (GPU solver, hip/multifrontal.hip). Supernodes are
// the blocks of the nested-dissection ordering (contiguous position ranges); the assembly tree
// links each supernode to the one holding the first row of its update matrix. Fronts are dense,
// index list = [k own dofs | r update rows]. Storage conventions:
//  - fronts with m = k + r <= kMfWaveMaxM are factored by one wavefront, packed lower-triangular
//    column-major (mf_packed); their amap_dst are packed indices. Larger fronts are full m x m
//    column-major and their amap_dst are i + j m.
//  - update matrices U are packed lower-triangular column-major (r (r + 1) / 2 values) for all.
//  - L panels are m x k column-major (entries above the diagonal unused).
constexpr int kMfWaveMaxM = 64;
constexpr int kMfFlowMaxM = 48;   // fronts of the dataflow factor launch (hip/multifrontal.hip kFlowMaxM)
constexpr int kMfBlkMaxM = 128;   // fronts of 65-128 rows: one workgroup, the front in LDS, blocked on MFMA
                                  // (hip/multifrontal.hip mf_factor_blk); landmarks fold into them too
constexpr int kFoldChunk = 64;   // folded row groups per chunk (one per lane)
constexpr int kFoldRec = 8;      // ints per folded row group (the 3 rows of one observing pose)
// fold record word 6: t (row of the landmark's update rows, 6 bits) | r[c] << 6 (6 bits) | the row's
// position in the parent front << kFoldPosShift (7 bits: parents up to kMfBlkMaxM rows) | the
// landmark's index in its chunk << kFoldLmShift (6 bits)
constexpr int kFoldPosShift = 12, kFoldPosMask = 127, kFoldLmShift = 19;
// landmarks per fold chunk for a parent front of size m: the device forms the chunk's W (m x 2
// landmarks, row stride 2 cap + 1, aliasing the front's packed LDS triangle of m (m + 1) / 2
// values) whose W W^T it accumulates with f64 MFMA, 4 columns per step (cap even: the steps read
// no column past 2 cap)
constexpr int fold_chunk_landmarks(int m) { return m <= 16 ? 2 : m <= 32 ? 6 : m <= 48 ? 10 : 14; }
inline int64_t mf_packed(int64_t i, int64_t j, int64_t m) { return j * m - j * (j - 1) / 2 + (i - j); }   // i >= j

struct Multifrontal {
    int nsuper = 0, nlevels = 0, max_m = 0;
    std::vector<int32_t> col0, k, r;        // per supernode: first dof, #own dofs, #update rows
    std::vector<int64_t> findex_off;        // into findex (m = k + r entries; first k = col0..col0+k-1)
    std::vector<int32_t> findex;
    std::vector<int64_t> L_off;             // dense m x k panel (col-major) in the factor buffer
    std::vector<int64_t> U_off;             // packed lower r x r update matrix
    std::vector<int64_t> u_off;             // r-vector (forward solve update)
    std::vector<int32_t> parent;            // -1 for roots
    std::vector<int32_t> child_ptr, child;  // children CSR
    std::vector<int64_t> rmap_off;          // per supernode: r positions of its rows in the parent's front
    std::vector<int32_t> rmap;
    std::vector<int32_t> amap_ptr;          // per supernode: range into amap_src / amap_dst
    std::vector<int32_t> amap_src, amap_dst;// block-array value (BlockLayout) -> front position (see above)
    std::vector<int32_t> level_ptr, level;  // supernodes grouped by tree level (leaves first)
    // Schur ordering: landmark supernodes (k = 2, leaves) are folded into their parent's front when
    // the parent is factored by one wavefront (m <= kMfWaveMaxM) or one blocked workgroup
    // (m <= kMfBlkMaxM): the parent's wave(s) eliminate them
    // itself (no launch, no update matrix). Folded supernodes are in no level list (the parent's
    // level ignores them); fold_list holds them for the backward substitution.
    std::vector<int32_t> fold_cnt;          // per supernode: #folded children (the first of its child list)
    std::vector<int32_t> fold_cptr;         // per supernode: its chunks [fold_cptr[s], fold_cptr[s + 1])
    std::vector<int32_t> fold_chunk;        // chunk c = folded row groups [fold_chunk[c], fold_chunk[c + 1]):
                                            // whole children, <= kFoldChunk groups
    std::vector<int32_t> fold_rec;          // kFoldRec ints per folded row group (layout: build_multifrontal)
    std::vector<int32_t> fold_list;         // folded supernodes
    int64_t L_size = 0, U_size = 0, u_size = 0;
    double flops = 0;
    // Schur plans (build_plan): whether every front fits the fast kernels (m <= kMfWaveMaxM, and
    // m <= kMfFlowMaxM from level 2 up), the largest front from level 2 up, and the separator balance
    // (percent) of the plan kept
    bool fits = true;
    int max_m_upper = 0;
    int balance_pct = 40;
};

// Multi-GPU sharding of the multifrontal solve. The assembly tree is cut into
// subtrees, each owned by one rank, below a replicated top (the separators above the cut, factored
// and solved by every rank). A rank's J+H runs the lanes of its own and of the top nodes, which is
// everything its fronts read (validate_plan proves it); no part of H crosses between ranks. Two
// exchanges per GN iteration: the subtree roots' update matrices and u-vectors before the top is
// factored, and the solution of the boundary nodes (subtree nodes a top lane reads) after the
// backward solve. One GPU: world 1, every node owned by rank 0, no top, no exchange.
constexpr int kExHeader = 2;   // doubles at the head of each rank's exchange buffer (stats partials)
struct Shard {
    int rank = 0, world = 1;
    std::vector<int8_t> sn_owner;      // per supernode: owning rank, -1 = top (every rank)
    std::vector<int32_t> node_owner;   // per node: owning rank, -1 = top, -2 = the fixed pose (no supernode;
                                       // its lane runs as a top lane: chi^2 only)
    std::vector<int32_t> lane_poses;   // J+H pose lanes: own poses, padding (-1) to a J+H block, top poses
    int own_pose_lanes = 0;            // lane_poses[0, own_pose_lanes): own poses (and padding)
    std::vector<int32_t> lane_lms;     // J+H landmark lanes: own landmarks, then top landmarks
    // exchange 1: subtree roots (with a parent) of rank q = roots[root_ptr[q], root_ptr[q + 1])
    std::vector<int32_t> root_ptr, roots;
    int64_t ex1_count = 0;             // doubles per rank: header + the largest rank's U / u payload
    // exchange 2: boundary dofs (permuted numbering) of rank q = bnd_dof[bnd_ptr[q], bnd_ptr[q + 1])
    std::vector<int32_t> bnd_ptr, bnd_dof;
    int64_t ex2_count = 0;
    // nodes this rank's box-plus updates: own + top (the first n_upd_local), then the boundary nodes
    // of the other ranks (their solution arrives with exchange 2)
    std::vector<int32_t> upd_nodes;
    int n_upd_local = 0;
    int n_top_fronts = 0, n_own_fronts = 0;
};

struct Plan {
    int NP = 0, NL = 0, Mb = 0, Mo = 0, fixed = -1;
    int64_t n = 0;                         // system size N - 3
    std::vector<int32_t> node_pos;         // elimination position; -1 for the fixed pose
    std::vector<int32_t> node_dof;         // first dof in the permuted system; fixed pose -> n
    std::vector<int32_t> rowptr, colind;   // lower triangle of P^T H_nf P, n rows
    std::vector<int32_t> Lptr, Lind;       // symbolic Cholesky factor (lower, with diagonal)
    Multifrontal mf;                       // built when factor_mode == kFactorMultifrontal
    BlockLayout blk;
    OrderingReport ordering;
    Shard shard;
    int64_t nnzA() const { return rowptr.empty() ? 0 : rowptr.back(); }
    int64_t nnzL() const { return Lptr.empty() ? 0 : Lptr.back(); }
};

enum FactorMode {
    kFactorNone = 0,          // dense solver: pattern only
    kFactorScalar = 1,        // scalar CSR Cholesky pattern (rocSOLVER csrrf), cheapest-flops ordering
    kFactorMultifrontal = 2,  // nested dissection + supernodal multifrontal structure (GPU solver)
    kFactorSchur = 3,         // multifrontal with every landmark eliminated first (its own leaf
                              // supernode), then nested dissection of the poses on the graph of the
                              // Schur complement S = H_pp - H_pl H_ll^-1 H_lp
};

// Builds the plan. Returns 0 or a negative BOS_ERR_* code with a message in err.
int build_plan(const ProblemIndex& pi, int rank, int world, int factor_mode, Plan& out, std::string& err);

// BOS_PARTITION_OBSERVATIONS on a one-GPU plan: the J+H block ranges of rank r of W (pose blocks
// [pb0, pb1), landmark blocks [lb0, lb1)), and which nodes' lanes they run (lane_node[u] = 1)
void observation_lanes(const Plan& P, int rank, int world, int64_t& pb0, int64_t& pb1, int64_t& lb0, int64_t& lb1,
                       std::vector<char>* lane_node);
// The block value of every stored entry of the lower triangle whose J+H lane is in lane_node (the
// rule of build_csr_src: a diagonal block by its node, a pose-landmark block by its pose, a pose-pose
// block by the lower pose): owned[e] = 1
void owned_entries(const Plan& P, const std::vector<char>& lane_node, std::vector<uint8_t>& owned);

// True when the multifrontal plan reads the pose-landmark and landmark-diagonal entries of the block
// array [off_ldiag, off_pp) only through fold records, each record's pose-landmark pair (t, 0), (t, 1)
// of one slot and its landmark block inside the landmark-diagonal region: the folds can then read the
// fp32 build's factored blocks directly (mf_set_fold_source) and the fp64 copy can skip the region.
bool mf_fold_reads_fp32(const Plan& P);

// Segments of exchange 1 for rank `rank` (hip/solver_capi.hip): pack = this rank's roots' U / u into
// its send buffer, unpack = every other rank's roots from the receive buffer (kinds: 0 U, 1 u, 2 send,
// 3 receive; offsets in doubles).
struct ExchangeSeg {
    int64_t src, dst, len;
    int32_t src_kind, dst_kind;
};
void exchange1_segments(const Plan& P, std::vector<ExchangeSeg>& pack, std::vector<ExchangeSeg>& unpack);

// Node ordering only (positions) and its symbolic cost. mode kFactorScalar / kFactorNone: the
// cheapest of temporal, landmarks-first and nested dissection; kFactorMultifrontal: nested
// dissection; kFactorSchur: landmarks first, then nested dissection of the poses on the graph of S.
// The multifrontal modes return their supernode blocks (contiguous position ranges) in `blocks`.
int order_nodes(const ProblemIndex& pi, int mode, std::vector<int32_t>& node_pos,
                std::vector<std::pair<int32_t, int32_t>>* blocks, OrderingReport& rep, std::string& err);

}  // namespace bos
