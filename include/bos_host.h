/*
 * bos_host.h — host-side utilities of libbos.so (no GPU needed): the reference's g2o loader and
 * landmark triangulation, the synthetic world generator, and plan inspection for tests.
 *
 *   bos_dataset_load_g2o   <- parse_g2o           (utils/g2o_utils.hpp:29, g2o_utils.cpp:10-146)
 *                            + default fixed pose (executables/bearing_only_slam.cpp:63-65)
 *                            + triangulate_landmarks (slam/triangulation.hpp:8, triangulation.cpp:65-74)
 *   bos_dataset_write_g2o  <- (no reference counterpart: the checkpoint artefact of SURVEY.md §5)
 */
#ifndef BOS_HOST_H_
#define BOS_HOST_H_

#include "bos.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bos_dataset bos_dataset;

/* Parse a g2o file, default the fixed pose to the first pose and (if triangulate) append the
 * triangulated landmarks in ascending-id order. verbose prints the reference's warnings. */
int bos_dataset_load_g2o(const char* path, int triangulate, int verbose, bos_dataset** out);
/* Synthetic world: initial guess = dead-reckoned odometry chain, landmarks
 * triangulated from it; ground truth available through bos_dataset_ground_truth. */
int bos_dataset_synthetic(int32_t num_poses, int32_t num_landmarks, int32_t bearings_per_pose, uint64_t seed,
                          bos_dataset** out);
/* Problem view (pointers owned by the dataset, valid until bos_dataset_free). */
int bos_dataset_problem(const bos_dataset* ds, bos_problem* view);
const int32_t* bos_dataset_pose_ids(const bos_dataset* ds);
const int32_t* bos_dataset_landmark_ids(const bos_dataset* ds);
int32_t bos_dataset_fixed_pose_id(const bos_dataset* ds);
float bos_dataset_bound(const bos_dataset* ds);
/* Ground truth of a synthetic dataset in stix order; BOS_ERR_INVALID for loaded files. */
int bos_dataset_ground_truth(const bos_dataset* ds, const double** pose_xyt, const double** landmark_xy);
/* Write the dataset as g2o; pose_xyt / landmark_xy override the state (NULL = dataset state). */
int bos_dataset_write_g2o(const bos_dataset* ds, const char* path, const double* pose_xyt, const double* landmark_xy,
                          int with_landmarks);
void bos_dataset_free(bos_dataset* ds);

/* Solver::normalized_angle (slam/solver.hpp:50, slam/solver_jacobians.cpp:325-333): the wrap into
 * [-pi, pi) the kernels use (bos_math.hpp), compared in double as the reference does. An |a| past
 * ~1e15 (or an infinite one), on which the reference's loops never end, gives NaN. */
double bos_normalized_angle_f64(double a);
float bos_normalized_angle_f32(float a);

typedef struct bos_plan_info {
    int64_t n;
    int64_t nnz_lower;
    int64_t nnz_factor;
    int64_t num_block_values;       /* block array of H (J+H kernel layout)                      */
    int64_t lanes_per_pose;
    double flops_temporal;
    double flops_nested_dissection;
    char ordering[32];
    int64_t mf_supernodes;          /* multifrontal: supernodes / tree levels / largest front */
    int64_t mf_levels;
    int64_t mf_max_front;
    double mf_flops;
    int64_t mf_update_bytes;
    int64_t mf_fits;                /* Schur: every front fits the fast kernels (m <= 64, m <= 48 from level 2 up) */
    int64_t mf_max_front_upper;     /* Schur: largest front from tree level 2 up                  */
    int64_t mf_balance_pct;         /* Schur: separator balance of the plan kept (40 = first try)   */
    /* multi-GPU shard of rank `rank` (multifrontal solvers; one GPU: everything own, no top) */
    int64_t shard_own_fronts;       /* fronts of this rank's subtrees                             */
    int64_t shard_top_fronts;       /* fronts of the replicated top                               */
    int64_t shard_roots;            /* this rank's subtree roots below the top (exchange 1)       */
    int64_t shard_ex1_doubles;      /* exchange 1 buffer per rank (doubles)                        */
    int64_t shard_ex2_doubles;      /* exchange 2 buffer per rank (doubles)                        */
    int64_t shard_pose_lanes;       /* J+H pose lane groups (own, padding, top)                    */
    int64_t shard_own_pose_lanes;
    int64_t shard_lm_lanes;
    int64_t shard_update_nodes;     /* nodes the box-plus updates (own, top, boundary)             */
    int64_t mf_fold_fp32;           /* the folds alone read the pose-landmark / landmark-diagonal
                                       region (mf_fold_reads_fp32): an fp32 build's folds read it
                                       from the fp32 array (bos_system_info.fold_fp32)             */
    int64_t lm_lanes_consecutive;   /* J+H landmark lanes whose poses are consecutive (p0, p0 + 1,
                                       ...): they read no pose-index records                      */
    int64_t pose_odometry_chain;    /* poses whose odometry entries are exactly edges p - 1 = (p - 1,
                                       p) and p = (p, p + 1): the J+H derives them from p          */
} bos_plan_info;

/* Build the static plan on the host (what bos_create does before touching the GPU) with the
 * planning fields of `options` (NULL = bos_default_options): solver (BOS_SOLVER_*: it selects the
 * ordering), partition, lanes_per_pose, schur_leaf; its rank / world_size are ignored (the
 * arguments below give them).
 * If ref_rows/ref_cols/owned are given (capacity >= nnz_lower) they receive, for every stored
 * entry of the lower triangle of H_nf, its (row, col) in the reference dof numbering
 * (row >= col) and whether rank `rank` of `world` computes it (its J+H lanes write the block);
 * b_owned (n + 3 entries, indexed by reference dof) marks the b entries its lanes write;
 * perm_to_ref (n + 3 entries) maps the permuted dof order used on the device to reference dofs. */
int bos_plan_inspect(const bos_problem* problem, const bos_options* options, int32_t rank, int32_t world, int64_t capacity, int32_t* ref_rows,
                     int32_t* ref_cols, uint8_t* owned, uint8_t* b_owned, int32_t* perm_to_ref, bos_plan_info* info);

/* Test hook: the GPU multifrontal algorithm re-run on the host with the plan's tree and maps
 * (options->solver BOS_SOLVER_SUPERNODAL or _SCHUR; vals in the plan's CSR order, rhs/x in its permuted
 * dof order). Not used by any solve. */
int bos_plan_mf_selftest(const bos_problem* problem, const bos_options* options, const double* vals, const double* rhs, double* x);

/* Owner of every node (NP poses, then NL landmarks) when the multifrontal solve is sharded over
 * `world` ranks: the rank, -1 for the replicated top, -2 for the fixed pose. */
int bos_plan_node_owner(const bos_problem* problem, const bos_options* options, int32_t world, int32_t* owner);

/* Test hook: the sharded GN solve (plan.hpp Shard) simulated on the host for all `world` ranks,
 * both exchanges included: per-rank plans, each rank's J+H outputs only, subtree factorization,
 * exchange 1, replicated top, backward, exchange 2. BOS_OK when the merged solution x (permuted
 * order, n) equals the one-rank solution bit for bit, the ranks agree on the top, every observation's
 * chi^2 is counted by one rank and every node a rank's J+H reads is kept current by its box-plus.
 * vals / rhs as for bos_plan_mf_selftest. */
int bos_plan_shard_selftest(const bos_problem* problem, const bos_options* options, int32_t world, const double* vals,
                            const double* rhs, double* x);

/* CPU baseline of bench.py (the build's own C++ CPU backend on the host's cores):
 * one GN iteration per bos_cpu_gn_step — J+H over the plan's lanes (fp64), the multifrontal
 * factorization and solves of the plan's tree with each level's fronts in parallel, box-plus — on
 * `threads` threads. A separate object: bos_create / bos_step never use it (no CPU fallback). */
typedef struct bos_cpu_gn bos_cpu_gn;
int bos_cpu_gn_create(const bos_problem* problem, int32_t solver, int32_t threads, bos_cpu_gn** out);
int bos_cpu_gn_step(bos_cpu_gn* c, double* chi2);
int bos_cpu_gn_get_state(const bos_cpu_gn* c, double* pose_xyt, double* landmark_xy);
void bos_cpu_gn_destroy(bos_cpu_gn* c);

/* Benchmark helpers (bench.py; HIP events on the handle's stream, no torch):
 * bos_time_linearize: n J+H builds. flush_caches = 0: back to back, the average per build;
 * flush_caches = 1: 512 MiB (of two alternating buffers) are read before each build so its inputs
 * come from HBM (as inside a GN step); each build timed alone by its own pair of events.
 * bos_time_triangulate: n device triangulations back to back (re-estimates the landmarks).
 * bos_time_steps: n GN iterations, each exactly a bos_step call (launch, wait, status read and
 * checked), timed on the host clock in a C loop: the synchronous rate a C++ caller of the drop-in
 * (the reference's driver, executables/bearing_only_slam.cpp:95-98) sees, without a binding's
 * per-call overhead. */
int bos_time_linearize(struct bos_solver* s, int32_t n, int32_t flush_caches, double* ms_per_build);
int bos_time_triangulate(struct bos_solver* s, int32_t n, double* ms_per_call);
int bos_time_steps(struct bos_solver* s, int32_t n, double* ms_per_step);

/* The C++ façade proj02::Solver (prb-project-bearing-only-slam_amd/csrc/host/solver.hpp, the
 * reference's class API, slam/solver.hpp:21-92) driven as the reference's executable drives it
 * (executables/bearing_only_slam.cpp:93-99: solver.step() in a loop, then one read of solver.state
 * to draw it). The façade is built from `problem` (ids = stix); one untimed step, then n
 * Solver::step() calls timed on the host clock: *ms_per_step. *ms_state_read: the one read of
 * solver.state after them (its lazy download of the device state). *mismatches: doubles of
 * solver.state whose bits differ from bos_get_state of the façade's handle. *ms_per_step_capi: n
 * bos_step calls on the same handle right after (bos_time_steps). Optional outputs may be NULL. */
int bos_time_facade_steps(const bos_problem* problem, const bos_options* options, int32_t n, double* ms_per_step,
                          double* ms_state_read, double* ms_per_step_capi, int64_t* mismatches);
/* Test hook: n steps of the façade beside n bos_step calls of a second handle created from the same
 * problem, solver.state read every 7 steps and written once (a landmark moved, a pose turned:
 * through the façade's public state, by bos_get_state / bos_set_state on the other handle) at n / 2.
 * *mismatches = doubles of solver.state that differ in their bits from the device states at the
 * reads and at the end (0 expected). */
int bos_debug_facade_selftest(const bos_problem* problem, const bos_options* options, int32_t n, int64_t* mismatches);

/* Test hook (process-wide, default 0 = product behaviour; not part of the drop-in boundary): the
 * line-by-line g2o parser instead of the chunked one (the tests prove them identical). */
void bos_debug_set_g2o_parser(int32_t line_by_line);
/* Test hook: the next bos_step's factor dataflow launch skips its first front, so a dependency
 * wait times out — bos_step must then fail with BOS_ERR_SOLVER and leave the state untouched.
 * BOS_ERR_UNSUPPORTED when the handle's solver has no dataflow launch. */
int bos_debug_inject_stall(struct bos_solver* s);
/* Test hook: run the one-GPU GN step as individual launches (enable = 0) instead of the captured
 * hipGraph replay (1, default). The same kernels in the same order either way. */
int bos_debug_set_step_graph(struct bos_solver* s, int32_t enable);
/* Diagnostics: one GN step (individual launches) whose multifrontal dataflow launches stamp every
 * front they process: stamps[16 * nsuper] = factor stamps [nsuper][8] (start, folded, assembled,
 * children ready, extend-added, factored, written, published), then backward stamps [nsuper][8]
 * (start, staged, parent ready, solved, published; 0 = not in a flow launch); realtime clock,
 * 100 MHz. meta[4 * nsuper] = tree level (-1 folded), k, r, folded children. */
int bos_debug_solver_stamps(struct bos_solver* s, int64_t capacity, uint64_t* stamps, int32_t* meta);

/* Diagnostics: one J+H launch with per-wave timeline stamps, 8 x uint64 per wave: block, wave in
 * block, kind (0 pose lanes / 1 landmark lanes), t_start, t_loop, t_loop_end, t_end (realtime clock,
 * 100 MHz ticks), hw_id | xcc_id << 32. capacity in waves; *n_waves = waves of the launch;
 * flush_caches = 1: 512 MiB read before the launch (inputs from HBM, as in a GN step). Not part
 * of the drop-in boundary; the product launches never carry stamps. */
int bos_debug_linearize_timeline(struct bos_solver* s, int64_t capacity, uint64_t* stamps, int64_t* n_waves,
                                 int32_t flush_caches);

#ifdef __cplusplus
}
#endif
#endif /* BOS_HOST_H_ */
