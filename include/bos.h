/*
 * bos.h — C ABI of the MI355X-native Gauss-Newton solver for 2-D bearing-only SLAM.
 *
 * Drop-in boundary for the reference's `proj02::Solver` (torchipeppo/prb-project-bearing-only-slam,
 * slam/solver.hpp:21-92). Plain pointers and sizes only, no exceptions across the boundary,
 * status 0 = OK, < 0 = error with a message from bos_last_error().
 *
 * Ownership and semantics follow the reference:
 *  - bos_create COPIES the problem (the reference's Solver ctor copies State and observation
 *    vectors, slam/solver.cpp:5-8); the caller's arrays are not referenced afterwards.
 *  - bos_step is synchronous: on return the state held by the handle has been updated
 *    (Solver::step, slam/solver.cpp:27-97).
 *  - one handle = one host thread; concurrent calls on one handle are undefined (the reference
 *    mutates its members H, b and the LDLT object in step(), slam/solver.hpp:58-82).
 *
 * Reference-side binding: see INTEGRATION.md.
 */
#ifndef BOS_H_
#define BOS_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BOS_ABI_VERSION 3

/* status codes */
#define BOS_OK 0
#define BOS_ERR_INVALID -1      /* bad argument / malformed problem                         */
#define BOS_ERR_DEVICE -2       /* HIP runtime error or no device                            */
#define BOS_ERR_SOLVER -3       /* rocSOLVER / rocBLAS failure                               */
#define BOS_ERR_IO -4           /* file not found / parse error                              */
#define BOS_ERR_UNSUPPORTED -5  /* input the build does not handle (see bos_last_error)     */
#define BOS_ERR_COMM -6         /* RCCL failure                                              */

/* arithmetic of the J+H build (the solve is always fp64) */
#define BOS_FP64 64
#define BOS_FP32 32

/* linear solver for H_nf dx = -b_nf (the reference: Eigen SimplicialLDLT, slam/solver.hpp:71-72) */
#define BOS_SOLVER_SUPERNODAL 0   /* GPU multifrontal supernodal Cholesky, nested dissection          */
#define BOS_SOLVER_DENSE_CHOL 1   /* rocSOLVER potrf/potrs on a dense copy (small problems)          */
#define BOS_SOLVER_ROCSOLVER_RF 2 /* rocSOLVER csrrf analysis/refactchol/solve (level-scheduled)      */
#define BOS_SOLVER_SCHUR 3        /* same GPU engine, landmarks eliminated first (default): the pose fronts
                                     factor the Schur complement S = H_pp - H_pl H_ll^-1 H_lp (config 5) */
#define BOS_SOLVER_SPARSE_CHOL BOS_SOLVER_SCHUR

/* how a world_size > 1 step is split over the ranks */
#define BOS_PARTITION_SUBTREE 0       /* default: per-rank subtrees of the Schur assembly tree below a
                                         replicated top; a rank builds only the H its fronts read, two
                                         all-gathers per iteration (subtree roots' updates, boundary x) */
#define BOS_PARTITION_OBSERVATIONS 1  /* BASELINE north star: the J+H lanes (observations in measurement
                                         order) split into contiguous ranges, one all-reduce (sum) of the
                                         whole (H, b) per iteration, the solve and update replicated */

/*
 * Problem in stix order (framework/state.hpp:47-53): poses in file order, landmarks in
 * ascending-id order (slam/triangulation.cpp:68-73). Replaces the (State, BearingObservationVector,
 * OdometryObservationVector, fixed_pose_id) arguments of Solver::Solver (slam/solver.hpp:30);
 * ids are resolved to stix once here instead of std::map::at per observation per iteration
 * (framework/state.cpp:43-63).
 */
typedef struct bos_problem {
    int32_t num_poses;              /* NP                                                        */
    int32_t num_landmarks;          /* NL                                                        */
    int32_t num_bearings;           /* M_b                                                       */
    int32_t num_odometry;           /* M_o                                                       */
    const double* pose_xyt;         /* [NP*3] x, y, theta                                        */
    const double* landmark_xy;      /* [NL*2], or NULL: triangulated on the device (bos_triangulate) */
    const int32_t* bearing_pose;    /* [M_b] pose stix                                           */
    const int32_t* bearing_landmark;/* [M_b] landmark stix                                       */
    const double* bearing_z;        /* [M_b] bearing, already smallestAngle-wrapped              */
    const double* bearing_omega;    /* [M_b] information, or NULL for 1 (observation.hpp:16,22)  */
    const int32_t* odom_src;        /* [M_o] pose stix                                           */
    const int32_t* odom_dst;        /* [M_o] pose stix                                           */
    const double* odom_z;           /* [M_o*3] x, y, theta in the source frame                   */
    const double* odom_omega;       /* [M_o*9] row-major symmetric information matrix            */
    int32_t fixed_pose;             /* stix of the pose held fixed (solver.cpp:99-125)           */
} bos_problem;

typedef struct bos_options {
    int32_t precision;              /* BOS_FP64 (default) or BOS_FP32                            */
    int32_t solver;                 /* BOS_SOLVER_SCHUR (default) / _SUPERNODAL / _DENSE_CHOL / _ROCSOLVER_RF */
    int32_t device;                 /* HIP device ordinal, -1 = current                          */
    int32_t rank;                   /* shard index (0 for one GPU)                               */
    int32_t world_size;             /* number of shards (1 for one GPU)                          */
    const void* nccl_unique_id;     /* 128-byte ncclUniqueId: bos_step runs the sharded step's two
                                       exchanges as RCCL all-gathers. NULL with world_size > 1:
                                       external exchange, the caller drives bos_step_phase and moves
                                       the buffers (bos_exchange_*). Given with world_size 1 it runs
                                       the sharded phases and RCCL with one rank (one-GPU test)      */
    double kernel_threshold;        /* robust kernel threshold, reference default 1.0 (:16)      */
    double damping;                 /* damping factor, reference default 0.01 (:17)              */
    void* stream;                   /* hipStream_t to launch on, NULL = the handle's own stream  */
    int32_t partition;              /* BOS_PARTITION_SUBTREE (default) / _OBSERVATIONS (world_size > 1) */
    int32_t lanes_per_pose;         /* J+H lanes per pose: 0 = the plan's choice, else 1, 2 or 4   */
    int32_t schur_leaf;             /* poses per nested-dissection leaf of the Schur ordering: 0 = the
                                       default (10); larger leaves give fronts over 64 rows, which run
                                       on the workgroup kernels (a planning option: the arithmetic of
                                       a front is the same)                                         */
} bos_options;

/* Per-iteration statistics (the reference prints nothing; step() returns void). */
typedef struct bos_step_stats {
    double chi2;                    /* sum e^T Omega e over all edges before the robust kernel   */
    int32_t n_robust;               /* observations scaled by the robust kernel                  */
    int32_t solver_info;            /* 0 ok, >0 number of non-positive pivots the factorization met
                                       (reported and continued, like the reference's NumericalIssue
                                       message, slam/solver.cpp:82-84)                            */
    double max_abs_dx;              /* max |dx| of the applied update (NaN if the update was not finite) */
    double t_linearize_ms;          /* J+H build only (the exchange is t_exchange_ms), timed on the
                                       device by the step's own kernels (realtime clock stamps)     */
    double t_exchange_ms;           /* RCCL exchange part (0 on one GPU)                         */
    double t_solve_ms;              /* factorization + triangular solves                         */
    double t_update_ms;             /* box-plus                                                  */
} bos_step_stats;

/* Static sizes of the linear system built by bos_create (for export buffers / roofline). */
typedef struct bos_system_info {
    int64_t n;                      /* N - 3 (fixed pose removed)                                */
    int64_t nnz_lower;              /* stored entries of the lower triangle of H_nf              */
    int64_t nnz_factor;             /* entries of the Cholesky factor (sparse solver)            */
    int64_t algorithmic_bytes;      /* SURVEY §8(d) J+H bytes for this problem and precision      */
    int64_t num_block_values;       /* size of the block array of H the J+H kernel writes        */
    int32_t lanes_per_pose;         /* J+H work split: lanes per pose (1 or 2)                   */
    int32_t pose_lane_groups;       /* J+H pose lane groups this rank runs (own, padding, top)   */
    int32_t landmark_lanes;         /* J+H landmark lanes this rank runs                         */
    int32_t own_fronts;             /* multifrontal fronts of this rank's subtrees               */
    int32_t top_fronts;             /* fronts of the replicated top (0 on one GPU)               */
    int32_t comm_ranks;             /* ranks the RCCL communicator holds (ncclCommCount), 0 without one */
    int32_t partition;              /* BOS_PARTITION_* of a sharded handle                       */
    int32_t pl_factored;            /* 1: pose-landmark blocks stored factored (3 floats, fp32 J+H) */
    int32_t fold_fp32;              /* 1: the solver's landmark folds read the fp32 block array (the fp64
                                       copy skips the pose-landmark and landmark-diagonal region)  */
    int64_t layout_bytes;           /* algorithmic_bytes with this layout's output: 12 B less per
                                       pose-landmark block when pl_factored                       */
} bos_system_info;

void bos_default_options(bos_options* opt);
const char* bos_last_error(void);
int bos_abi_version(void);
int bos_device_count(void);
/* Peer access between the visible devices (no reference counterpart: the multi-GPU bench records it
 * beside its exchange decision). out[i * n + j] = 1 if device i can access device j's memory
 * (hipDeviceCanAccessPeer; 1 on the diagonal), for n = min(capacity, bos_device_count()) devices;
 * *n_out = that n. */
int bos_device_peer_access(int32_t capacity, int32_t* out, int32_t* n_out);
/* ncclGetUniqueId for world_size > 1: rank 0 creates it, the caller distributes the bytes */
int bos_nccl_unique_id(void* out, int64_t len);

/* Solver::Solver (slam/solver.hpp:30, slam/solver.cpp:5-18) */
int bos_create(const bos_problem* problem, const bos_options* options, struct bos_solver** out);
/* ~Solver */
int bos_destroy(struct bos_solver* s);
/* Solver::set_kernel_threshold / set_damping_factor (slam/solver.hpp:33-34) */
int bos_set_kernel_threshold(struct bos_solver* s, double kt);
int bos_set_damping_factor(struct bos_solver* s, double df);
/* Solver::step (slam/solver.hpp:36, slam/solver.cpp:27-97): one synchronous GN iteration.
 * BOS_ERR_SOLVER (state untouched by the failed iteration) if the GPU factorization could not
 * complete (a dataflow dependency wait timed out); a non-positive pivot is only reported in
 * stats->solver_info, as the reference reports and continues. */
int bos_step(struct bos_solver* s, bos_step_stats* stats);
/* bos_step repeated n times with one host synchronisation at the end (UI batch of 50,
 * executables/bearing_only_slam.cpp:95-98); stats of the last iteration */
int bos_step_n(struct bos_solver* s, int n, bos_step_stats* last);
/* The J+H build alone (slam/solver.cpp:28-69) — H and b stay on the device */
int bos_linearize(struct bos_solver* s, bos_step_stats* stats);
/* Enqueue the J+H build on the handle's stream without synchronising (benchmarking) */
int bos_linearize_async(struct bos_solver* s);
int bos_synchronize(struct bos_solver* s);
/* triangulate_landmarks (slam/triangulation.cpp:65-74, per landmark triangulate_one_landmark
 * :21-62): every landmark re-estimated on the device from the current poses and its bearings
 * (column-pivoted least squares, the basic solution for single-observation landmarks), synchronous.
 * bos_create does the same when bos_problem.landmark_xy is NULL (the reference triangulates before
 * constructing the Solver, executables/bearing_only_slam.cpp). The _async form only enqueues it. */
int bos_triangulate(struct bos_solver* s);
int bos_triangulate_async(struct bos_solver* s);
int bos_system_info_get(const struct bos_solver* s, bos_system_info* info);
/*
 * Export the last linearization in the reference's dof order (poses 3*stix, landmarks
 * 3*NP + 2*stix, slam/solver_jacobians.cpp:70-71): the lower triangle of H with the fixed pose's
 * rows/cols removed (H_nofixed, slam/solver.cpp:72, indices still in full N numbering) as COO
 * (capacity = nnz_lower), and the full b[N] (slam/solver.cpp:45,61).
 */
int bos_export_system(const struct bos_solver* s, int64_t capacity, int32_t* rows, int32_t* cols, double* vals,
                      double* b);
/* On sharded handles (world_size > 1, or a communicator) bos_linearize is BOS_ERR_UNSUPPORTED (a
 * rank builds only part of H); bos_export_system and bos_get_last_dx are supported with
 * BOS_PARTITION_OBSERVATIONS after a step (every rank holds the all-reduced system and the whole
 * dx) and BOS_ERR_UNSUPPORTED with BOS_PARTITION_SUBTREE (a rank holds H and x of its own, top and
 * boundary nodes only). */
/*
 * Multi-GPU (one process per GPU, world_size > 1, BOS_SOLVER_SCHUR / _SUPERNODAL). The sparse
 * Cholesky's assembly tree is cut into per-rank subtrees below a replicated top; each rank builds
 * the part of H its fronts read (its own and the top nodes' J+H lanes), factors its subtrees, and
 * two all-gathers per iteration move the subtree roots' update matrices (exchange 1) and the
 * boundary solution (exchange 2). With a communicator bos_step does everything. Without one
 * (external exchange) the caller runs, per iteration:
 *   bos_step_phase(s, 0); all-gather of every rank's exchange-1 buffer (bos_exchange_download /
 *   bos_exchange_upload, rank order); bos_step_phase(s, 1); the same for exchange 2;
 *   bos_step_phase(s, 2, stats)   (synchronous, like bos_step).
 * After a step a rank's state is current on the nodes it owns, the top and the boundary nodes
 * (bos_node_owner: owning rank per node, -1 top, -2 fixed pose); merge per owner for the full state.
 *
 * BOS_PARTITION_OBSERVATIONS (the north star's form): phase 0 is rank r's range of J+H lanes, the one
 * exchange is an all-reduce (sum) of every rank's exchange-1 buffer (its chi^2 partials and its
 * (H, b) values, zero outside its range; bos_exchange_upload then takes the element-wise SUM, one
 * rank's size, not the concatenation), phase 1 runs the solve and the box-plus of every node and
 * returns the stats (phase 2 does not exist). Every rank then holds the whole state.
 */
int bos_step_phase(struct bos_solver* s, int32_t phase, bos_step_stats* stats);
int bos_exchange_size(const struct bos_solver* s, int32_t which, int64_t* doubles_per_rank);
int bos_exchange_download(struct bos_solver* s, int32_t which, double* send);
int bos_exchange_upload(struct bos_solver* s, int32_t which, const double* recv_all_ranks);
int bos_node_owner(const struct bos_solver* s, int32_t* owner);
/*
 * Direct peer exchange (BOS_PARTITION_SUBTREE, round 4): instead of the two ncclAllGather calls,
 * every rank writes its exchange buffers straight into every rank's receive mailbox (uncached device
 * memory, mapped into the other ranks' processes by HIP IPC: over xGMI between GPUs) and raises a
 * per-sender flag there; the receiving rank's next kernel waits for every sender's flag of the
 * current iteration (bounded: a missing peer aborts the step with BOS_ERR_SOLVER instead of
 * hanging). Two small launches per exchange, no collective library, and the whole iteration stays
 * one graph. bos_exchange_p2p_handle writes this rank's mailbox handle (BOS_P2P_HANDLE_BYTES bytes);
 * the caller gathers every rank's (rank order, e.g. torch.distributed.all_gather_object) and passes
 * them to bos_exchange_p2p_connect, after which bos_step uses the direct exchange (a communicator
 * is then not needed; world_size 1 exchanges with itself). All ranks must step in lockstep (each
 * bos_step / bos_step_n iteration on every rank). BOS_ERR_UNSUPPORTED if the mailbox cannot be
 * exported (no uncached IPC memory) or on other partitions; callers then keep RCCL.
 */
#define BOS_P2P_HANDLE_BYTES 64
int bos_exchange_p2p_handle(struct bos_solver* s, void* handle);
int bos_exchange_p2p_connect(struct bos_solver* s, const void* handles);
/* Timing contract of the direct exchange. A rank's step waits on the device for the other ranks'
 * pushes (two waits per iteration); a wait gives up after `seconds` (default 2 s, so host-side gaps
 * of one rank between its bos_step calls — the first step's graph captures, logging, a pause —
 * stay far inside it) and then marks the step aborted: every later exchange wait of that step
 * returns at once, the box-plus is skipped and bos_step returns BOS_ERR_SOLVER. A local solver
 * stall (a dataflow dependency wait that timed out) aborts the step too but does not shorten the
 * exchange waits, so that rank still receives its peers' current exchange 2. An abort raised before
 * exchange 2 travels in exchange 2's header, so every rank skips that update together and reports
 * BOS_ERR_SOLVER for the same step; a wait on exchange 2 itself that times out skips the update on
 * the ranks that timed out only, so after any BOS_ERR_SOLVER from a sharded step the caller must
 * bring all ranks back to one state (bos_set_state on every rank) or destroy the handles. Once connected, bos_step_phase and
 * bos_exchange_download / _upload return BOS_ERR_INVALID (the exchange is the handle's own). Every
 * rank must finish stepping (its last bos_step returned on every rank, e.g. a barrier) before any
 * rank calls bos_destroy: the peers' pushes write into this rank's mailbox. */
int bos_set_exchange_timeout(struct bos_solver* s, double seconds);

/* State read/write in stix order (State::poses / landmarks, framework/state.hpp:47-48) */
int bos_get_state(const struct bos_solver* s, double* pose_xyt, double* landmark_xy);
int bos_set_state(struct bos_solver* s, const double* pose_xyt, const double* landmark_xy);
/* The dx of the last bos_step in the reference's dof order (slam/solver.cpp:88-94) */
int bos_get_last_dx(const struct bos_solver* s, double* dx);
/* Diagnostics: the phase boundaries of the last completed step, realtime clock (100 MHz ticks),
 * as the step's own kernels stamped them: [0] J+H start, [1] J+H end / solve start, [2] solve end,
 * [3] step end; subtree-sharded handles: [4] phase 0 done (own subtrees factored, exchange 1
 * starts), [5] exchange 1 received (replicated top starts), [6] phase 1 done (top factored and
 * solved, own subtrees solved backward; exchange 2 starts), [7] exchange 2 received (box-plus
 * starts). bench.py reports them per rank. */
int bos_last_step_stamps(const struct bos_solver* s, uint64_t stamps[8]);

#ifdef __cplusplus
}
#endif
#endif /* BOS_H_ */
