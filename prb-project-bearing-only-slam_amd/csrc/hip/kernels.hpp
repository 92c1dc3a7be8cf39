// Device-side parameter blocks and launch wrappers of the GN kernels (hip/kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace bos {
namespace dev {

constexpr int kBlock = 256;   // J+H block of lanes (host/plan.hpp kJhBlock)
// J+H launch: workgroups of kJhWg threads, kJhSub of them per block of lanes (linearize_kernel,
// jh_unit); chi^2 partials: one per pose workgroup
constexpr int kJhWg = 256;
constexpr int kJhSub = kBlock / kJhWg;
static_assert(kJhSub * kJhWg == kBlock && kJhWg % 64 == 0, "J+H workgroup");
// padding records after each lane-list array: the J+H kernel reads records up to five items past a
// lane's last one, unguarded
constexpr int kRecPad = 512;

// Pose-list records whose next item observes the same landmark (a run of duplicate observations,
// summed into the run's last slot) carry kRunCont in their index.
constexpr int32_t kRunCont = (int32_t)0x80000000u;
constexpr int32_t kIdxMask = 0x7fffffff;
// A pose lane count (pl_cnt, the group's first lane) with kOdoChain set: the pose is an odometry
// chain pose (BlockLayout::po_chain; never with duplicate pairs), its entries derived from p
constexpr int32_t kOdoChain = 0x40000000;

// A lane list item is the other endpoint (landmark for the pose lists, pose for the landmark lists)
// and the measured bearing, stored as two arrays (index, z) so each is read exactly once.

// J+H build (host/plan.hpp BlockLayout). Blocks [0, pose_blocks) run lane groups of lpp lanes, group
// i for pose lane_pose[i] (-1: padding), the rest one lane per landmark lane (landmark ll_lm[g]).
// Lane lists are wave-interleaved: item j of lane t of wave w is slot w_base[w] + w_stride[w] j + t
// (plan.hpp LaneLists: groups of equal-length waves stored step-major).
template <typename T> struct LinParams {
    // state caches (T precision): host-computed at create / set_state, then kept by the box-plus kernel
    const T* pc;          // [NP][4] x, y, cos(theta), sin(theta)
    const T* pth;         // [NP] theta
    const T* lc;          // [NL][2]
    int NP;
    const int32_t* lane_pose;  // [n_groups] pose of each lane group, -1 = padding; null: group i = pose i
    int n_groups, n_lm_lanes, pose_blocks;
    // the blocks this launch runs: pose blocks [pose_b0, pose_b0 + n_pose_run), landmark blocks
    // [lm_b0, lm_b0 + n_lm_run) (everything on one GPU; a range of each with BOS_PARTITION_OBSERVATIONS)
    int pose_b0, n_pose_run, lm_b0, n_lm_run;
    // pose lanes
    const int32_t* pw_base;   // [waves + 1]
    const int32_t* pw_stride; // [waves]
    const int32_t* pl_cnt;    // [NP * lpp] items per lane (| kOdoChain)
    const int32_t* pb_idx;    // [slots] landmark (| kRunCont); the pose-landmark block of a slot is at off_pl + 6 slot
    const T* pb_z;            // [slots] measured bearing
    const T* pb_w;            // [slots] information, null => 1
    const int32_t* po_ptr;    // [NP + 1]
    const int32_t* po_ent;    // edge << 1 | destination side
    const int32_t* po_oth;    // the other pose of the entry's edge
    const int32_t* po_blk;    // pose-pose block the entry adds to (other pose higher), else -1
    const int32_t* o_src;
    const int32_t* o_dst;
    const T* o_z;             // [M_o][3]
    const T* o_om;            // [M_o][6] upper triangle (00, 01, 02, 11, 12, 22), edge k's at om_stride k
    int om_stride;            // 6, or 0 when every edge carries the same information (one row, read by all:
                              // the reference dataset's and the synthetic worlds' diag(500, 500, 5000))
    // landmark lanes
    const int32_t* lw_base;   // [waves + 1]
    const int32_t* lw_stride; // [waves]
    const int32_t* ll_cnt;    // [NL] per lane
    const int32_t* ll_lm;     // [NL] landmark of each lane (degree-sorted inside 256-lane windows)
    const int32_t* lb_idx;    // [slots] pose
    // [NL] per lane: the first pose when the lane's poses are consecutive (p0, p0 + 1, ..., no
    // repeats; BlockLayout::lm_lane_run), else -1. Such a lane reads no index records: its pose
    // gathers depend on no load. Null: every lane reads its records.
    const int32_t* ll_run;
    // [NL] per lane {landmark | count << 20, ll_run's value}: the three headers in one load (set when
    // they fit; ll_lm / ll_cnt / ll_run are then null)
    const int2* ll_hdr;
    const T* lb_z;            // [slots] measured bearing
    const T* lb_w;
    // outputs
    T* hval;                  // block array (BlockLayout)
    T* b;                     // [3 NP + 2 NL], reference dof numbering
    int off_ldiag, off_pl, off_pp;
    // factored pose-landmark blocks (fp32 build, unit bearing weights, no duplicate pairs): slot s
    // holds (J_theta, J_lx, J_ly) at off_pl + 3 s instead of the 6 block values at off_pl + 6 s; the
    // block is J_p^T J_l with J_p = (-J_lx, -J_ly, J_theta) exactly (solver_jacobians.cpp:51-64:
    // the translation columns of the bearing Jacobian are minus its landmark columns), expanded by
    // the solver's fp64 conversion (launch_gather_f64)
    int pl_factored;
    double* chi2_part;        // [pose_blocks * kJhSub]: one per pose workgroup
    int32_t* nrob_part;       // [pose_blocks * kJhSub]
    T kt;                     // robust kernel threshold
    T lambda;                 // damping
    unsigned long long* diag_stamps;   // timeline diagnostics only (8 x u64 per wave), null otherwise
    unsigned long long* t_start;       // phase timing: block 0 writes the realtime clock at its start, or null
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
    double* max_part;         // [update blocks] max |dx| of each block (reduced by reduce_stats)
    const int32_t* info;      // solver status word or null; | kStepAbort => the update is skipped
    // sharded step: every rank's exchange-2 header [max |x|, solver word] (ex_hdr[q * ex_stride],
    // q < ex_world; null otherwise): any rank's abort bit skips the update
    const double* ex_hdr;
    int64_t ex_stride;
    int ex_world;
    const int32_t* nodes;     // nodes to update (sharded: own, top, boundary), null = all NP + NL
    int n_nodes;
    unsigned long long* t_start;   // phase timing: block 0 writes the realtime clock at its start, or null
};

// Solver status bit: the factorization's results are invalid (a dataflow launch timed out,
// multifrontal.hpp kMfStall); the box-plus then leaves the state untouched and bos_step fails.
constexpr int32_t kStepAbort = 1 << 30;
// Set with kStepAbort by a direct-exchange wait that timed out (a peer's data never arrived): the
// step's later exchange waits then give up at once. A local solver stall (kStepAbort alone) does not
// shorten them: the rank still waits (bounded) for its peers' exchange 2, so every rank combines the
// same, current headers and reports the failed step alike.
constexpr int32_t kExTimeout = 1 << 29;

// End-of-iteration summary, read back by the host in one copy.
struct StepStatus {
    double chi2;
    double max_dx;
    int32_t n_robust;
    int32_t info;     // solver status: count of non-positive pivots, | kStepAbort (see above)
    int32_t aborted;  // sticky: kStepAbort once any step aborted; the host clears it when it reports it
    int32_t seq;      // steps summarised so far (reduce_stats); written to the host mirror last
    // phase boundaries of the last step, realtime clock (100 MHz), written by the step's own kernels
    // (no events in the step): [0] J+H start, [1] J+H end / solve start, [2] solve end / update
    // start, [3] step end. BOS_PARTITION_OBSERVATIONS: [1] = J+H end (before the all-reduce), [4] =
    // solve start (after it). BOS_PARTITION_SUBTREE: [4] exchange 1 start (phase 0 done), [5]
    // exchange 1 end (phase 1 starts), [6] exchange 2 start, [7] exchange 2 end (phase 2 starts).
    unsigned long long stamp[8];
};
constexpr double kStampMs = 1e-5;   // one realtime tick in ms

constexpr int kUpdateBlock = 256;

// Landmark triangulation (slam/triangulation.cpp:21-74) on the device: one lane per landmark over its
// bearings (CSR in file order, as the reference groups them by landmark id).
template <typename T> struct TriParams {
    int NL;
    const int32_t* lm_ptr;    // [NL + 1]
    const int32_t* lm_obs;    // [M_b] bearing indices grouped by landmark
    const int32_t* b_pose;    // [M_b]
    const double* b_z;        // [M_b]
    const double* pose;       // [NP][3] master state
    double* scratch;          // [M_b][3] the least-squares rows (a0, a1, r) in CSR order
    double* lm;               // [NL][2] out: master state
    T* lc;                    // [NL][2] out: T-precision cache
};

// Exchange of the sharded J+H results (hip/solver_capi.hip enqueue_exchange): copies of contiguous
// segments between the block array (kind 0), b (1), the packed send buffer (2) and the all-gather
// receive buffer (3).
struct ExSeg {
    int64_t src, dst, len;   // element offsets and count
    int32_t src_kind, dst_kind;
};

// A wait for the direct exchange's flags (bos_exchange_p2p_connect), fused into the launch that
// reads the received data: in every block, lanes q < world poll sender q's flag (mailbox + flag_off
// + 64 q) until it equals the iteration's epoch (*epoch), or mark the step aborted (*info |=
// kStepAbort) after timeout_ticks of the 100 MHz realtime clock (bos_set_exchange_timeout, 2 s by
// default), or stop at once when another block already did; then the block reads. mailbox null:
// no wait.
struct P2PWait {
    const char* mailbox = nullptr;
    int64_t flag_off = 0;
    int world = 0;
    const uint32_t* epoch = nullptr;
    int32_t* info = nullptr;
    uint64_t timeout_ticks = 200000000ull;
};

// Segment kinds (ExSeg src_kind / dst_kind): 0 val, 1 b, 2 send, 3 recv, 4 aux (the received
// exchange-1 headers' local copy). *stamp (if set) gets the realtime clock at the launch's start
// (after the wait, with one); with nothing to copy, a wait (or the stamp) still runs
template <typename T>
hipError_t launch_seg_copy(T* val, T* b, T* send, T* recv, T* aux, const ExSeg* segs, int nseg, int64_t max_len,
                           hipStream_t s, unsigned long long* stamp = nullptr, const P2PWait& w = P2PWait());

template <typename T>
hipError_t launch_linearize(const LinParams<T>& p, int lpp, bool has_w, bool has_dups, hipStream_t s);
template <typename T> hipError_t launch_boxplus(const UpdateParams<T>& p, hipStream_t s);

// Sharded GN step (host/plan.hpp Shard, hip/solver_capi.hip). Exchange buffers are doubles with a
// kExHeader-double header per rank.
constexpr int kExHeader = 2;   // = bos::kExHeader (host/plan.hpp)
// Exchange 1 header: this rank's chi^2 and robust count (sums of the J+H partials [0, n_parts));
// *stamp (if set) gets the realtime clock at its end.
hipError_t launch_shard_header1(const double* chi_part, const int32_t* nrob_part, int n_parts, double* send1,
                                hipStream_t s, unsigned long long* stamp = nullptr);
// out[i] = (T)in[i]: the all-reduced exchange buffer (fp64 on the host side of the external exchange)
// back into the system's precision (exact: the values are T values summed with zeros)
template <typename T> hipError_t launch_from_f64(const double* in, T* out, int64_t n, hipStream_t s);
// Exchange 2: header = max |x| over the dofs of nodes[0, n_nodes) (the rank's own and top nodes)
// and the solver word *info (then zeroed for the next iteration); payload = x[bnd[i]].
hipError_t launch_shard_pack2(const double* x, const int32_t* nodes, int n_nodes, const int32_t* node_dof, int NP,
                              int32_t* info, const int32_t* bnd, int n_bnd, double* part, double* send2,
                              hipStream_t s, unsigned long long* stamp = nullptr);
// the first launch of launch_shard_pack2 alone: per-block max |x| partials into part; returns the
// number of partials (for launch_p2p_push_gather's exchange 2)
int launch_node_absmax(const double* x, const int32_t* nodes, int n_nodes, const int32_t* node_dof, int NP, double* part,
                       hipStream_t s, hipError_t* err);
// dst[dst_idx[i]] = src[src_idx[i]], i < n; *stamp (if set) gets the realtime clock at the start
// (after the wait, with one)
hipError_t launch_index_copy(const double* src, const int32_t* src_idx, double* dst, const int32_t* dst_idx, int64_t n,
                             hipStream_t s, unsigned long long* stamp = nullptr, const P2PWait& w = P2PWait());
// All ranks' headers -> *out (chi^2 and robust count summed in rank order plus the self-loop
// terms, max |dx| the max, info: non-positive pivots summed, abort bits or-ed; `aborted` sticky
// sticky), identical on every rank.
hipError_t launch_shard_combine(const double* recv1, int64_t c1, const double* recv2, int64_t c2, int world,
                                double chi_const, int32_t nrob_const, int32_t* local_info, StepStatus* out,
                                StepStatus* mirror, hipStream_t s, bool zero_info = false);
template <typename T> hipError_t launch_triangulate(const TriParams<T>& p, hipStream_t s);
// Direct peer exchange (bos_exchange_p2p_connect): one block per receiving rank q copies the
// `count` doubles of `send` to peers[q] + data_off (bytes) + rank * count doubles, drains its stores,
// releases at system scope and stores the iteration's epoch (*epoch) into its flag slot there
// (peers[q] + flag_off + 64 * rank); the receiver waits with a P2PWait. chi_part set (exchange 1):
// the first kExHeader doubles are the header of launch_shard_header1, computed by the push itself
// (no header launch). *stamp (if set) gets the realtime clock at the start.
hipError_t launch_p2p_push(const double* send, int64_t count, double* const* peers, int64_t data_off, int64_t flag_off,
                           int rank, int world, const uint32_t* epoch, const double* chi_part, const int32_t* nrob_part,
                           int n_parts, unsigned long long* stamp, hipStream_t s);
// The direct exchange's push with the payload gathered from where it lives instead of from a packed
// send buffer (one launch less per exchange). Exchange 1: the header of
// launch_shard_header1, then every pack segment (src_kind 0: U, 1: u; dst: offset in the slot).
// Exchange 2: the header [max of abs_part, *info] (launch_shard_pack2's, without zeroing
// *info: the combine launch zeroes it after the step, zero_info), then x[bnd[i]] at 2 + i.
struct P2PPush {
    int which = 1;                      // exchange 1 or 2
    double* const* peers = nullptr;
    int64_t data_off = 0, flag_off = 0, count = 0;
    int rank = 0, world = 0;
    const uint32_t* epoch = nullptr;
    unsigned long long* stamp = nullptr;
    const double* chi_part = nullptr;   // exchange 1
    const int32_t* nrob_part = nullptr;
    int n_parts = 0;
    const double* U = nullptr;
    const double* u = nullptr;
    const ExSeg* segs = nullptr;
    int nseg = 0;
    const double* x = nullptr;          // exchange 2
    const double* abs_part = nullptr;
    int n_abs = 0;
    const int32_t* info = nullptr;
    const int32_t* bnd = nullptr;
    int n_bnd = 0;
};
hipError_t launch_p2p_push_gather(const P2PPush& p, hipStream_t s);
// Reduces the J+H kernel's chi^2 / robust-count partials (nrob_part null: chi_part is an
// all-reduced header [chi^2, robust count], n ignored) (plus the constant terms of odometry
// self-loops, chi_const / nrob_const) and the box-plus max |dx| partials (when max_part is set; a NaN
// propagates) into *out, moves *info into out->info and zeroes *info for the next iteration: one
// launch replaces the per-step memsets and read-backs. out->aborted is sticky; out->stamp[3] gets the
// realtime clock at the end. The finished summary is also copied to *mirror (host-mapped memory the
// host reads after synchronising: no copy launch per step), if set.
hipError_t launch_reduce_stats(const double* chi_part, const int32_t* nrob_part, int n, double chi_const,
                               int32_t nrob_const, const double* max_part, int n_max, int32_t* info,
                               StepStatus* out, StepStatus* mirror, hipStream_t s);
// Reads n doubles (all of them: the sum is compared with an impossible value), so L2 and the
// Infinity Cache hold clean lines of this buffer afterwards (cold-cache timing, bos_time_linearize).
hipError_t launch_cache_scrub(const double* buf, int64_t n, double* sink, hipStream_t s);
template <typename T> hipError_t launch_to_f64(const T* in, double* out, int64_t n, hipStream_t s);
// out[i] = (double)in[idx[i]], i < n, and (when cn > 0) cout[i] = (double)cin[i], i < cn, in one
// launch. Block 0 also writes the realtime clock to *stamp and bumps *epoch (the multifrontal flows'
// step epoch, multifrontal.hpp mf_epoch_ptr) when those are set: the right-hand side gather (with
// the fp64 copy of an fp32 block array) opens the solve of a GN step, so the step needs no marker
// launches.
template <typename T>
hipError_t launch_gather_f64(const T* in, const int32_t* idx, double* out, int64_t n, hipStream_t s,
                             unsigned long long* stamp = nullptr, uint32_t* epoch = nullptr, const T* cin = nullptr,
                             double* cout = nullptr, int64_t cn = 0);
// The same with a block array whose pose-landmark region [pl_off, pl_off + 6 pl_slots) is stored
// factored (LinParams::pl_factored): that region is expanded to the 6 block values per slot in fp64
// (the products rounded in T, so the values equal those of an unfactored build), the rest copied.
hipError_t launch_gather_f64_factored(const float* in, const int32_t* idx, double* out, int64_t n, hipStream_t s,
                                      unsigned long long* stamp, uint32_t* epoch, const float* cin, double* cout,
                                      int64_t cn, int64_t pl_off, int64_t pl_slots);
// the right-hand side gather and the fp64 copy of the block array outside [lo, hi) (the region the
// folds read from the fp32 array themselves, mf_set_fold_source)
hipError_t launch_gather_f64_ranges(const float* in, const int32_t* idx, double* out, int64_t n, hipStream_t s,
                                    unsigned long long* stamp, uint32_t* epoch, const float* cin, double* cout,
                                    int64_t cn, int64_t lo, int64_t hi);
// Host-side expansion of a factored block array (bos_export_system): region as above, in place on a
// copy of the fp32 array converted to double
void expand_factored_host(const float* in, double* out, int64_t n, int64_t pl_off, int64_t pl_slots);
hipError_t launch_scatter_dense(const int32_t* rowptr, const int32_t* colind, const double* val, int n, double* dense,
                                hipStream_t s);

}  // namespace dev
}  // namespace bos
