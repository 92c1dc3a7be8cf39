// C ABI implementation (include/bos.h): the handle owns every device buffer, the static plan
// (host/plan.hpp), the rocSOLVER refactorization state and the RCCL communicator.
//
// One GN iteration (reference Solver::step, slam/solver.cpp:27-97):
//   1. linearize_kernel          J+H build into the block array of H and b (+ damping)
//   2. sparse Cholesky factorization + solve: the GPU supernodal multifrontal solver (default;
//      structure analysed once, like SimplicialLDLT::analyzePattern at solver.cpp:77-80), or
//      rocSOLVER csrrf / dense potrf-potrs on a gathered CSR copy
//   3. boxplus_kernel            left-multiplicative box-plus with dx = -x (state.cpp:69-80)
// Sharded over world > 1 ranks, BOS_PARTITION_SUBTREE (host/plan.hpp Shard, host/shard.cpp): the
// J+H runs this rank's own and the top nodes' lanes, the multifrontal solve its subtrees, then
// (exchange 1, all-gather of the subtree roots' U / u) the replicated top, the backward solves, then
// (exchange 2, all-gather of the boundary solution) the box-plus of its own, top and boundary nodes.
// BOS_PARTITION_OBSERVATIONS (the north star's form): the J+H runs a contiguous range of the
// one-GPU plan's lanes, one all-reduce (sum) of (H, b) and the chi^2 header, then the one-GPU solve
// and box-plus on every rank. The exchanges run on RCCL, or — external mode, no communicator — the
// caller moves the buffers between the phases (bos_step_phase; tests on one GPU, gloo).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/bos.h"
#include "../../../include/bos_host.h"
#include "../host/bos_math.hpp"
#include "../host/error.hpp"
#include "../host/plan.hpp"
#include "kernels.hpp"
#include "multifrontal.hpp"

namespace {

int fail(int code, const std::string& msg) { return bos::set_error(code, msg); }

#define HIP_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) return fail(BOS_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define RB_TRY(expr)                                                                                   \
    do {                                                                                               \
        rocblas_status s_ = (expr);                                                                    \
        if (s_ != rocblas_status_success)                                                              \
            return fail(BOS_ERR_SOLVER, std::string(#expr) + ": " + rocblas_status_to_string(s_));     \
    } while (0)
#define NC_TRY(expr)                                                                                   \
    do {                                                                                               \
        ncclResult_t r_ = (expr);                                                                      \
        if (r_ != ncclSuccess) return fail(BOS_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

template <typename X> int dalloc(X** p, size_t count) {
    *p = nullptr;
    if (count == 0) return BOS_OK;
    HIP_TRY(hipMalloc((void**)p, count * sizeof(X)));
    return BOS_OK;
}
template <typename X> int upload(X** p, const std::vector<X>& v) {
    int rc = dalloc(p, v.size());
    if (rc) return rc;
    if (!v.empty()) HIP_TRY(hipMemcpy(*p, v.data(), v.size() * sizeof(X), hipMemcpyHostToDevice));
    return BOS_OK;
}

}  // namespace

struct bos_solver {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int precision = BOS_FP64;
    int solver_kind = BOS_SOLVER_SUPERNODAL;
    int rank = 0, world = 1;
    double kt = 1.0, damping = 0.01;
    bos::Plan plan;
    int NP = 0, NL = 0, Mb = 0, Mo = 0;
    bool has_w = false, has_dups = false;
    // fp32 build with a multifrontal solve, unit weights, no duplicate pairs: the J+H writes the
    // pose-landmark blocks factored (LinParams::pl_factored), the solver's fp64 conversion expands them
    bool pl_factored = false;
    // ... and the folds read them (and the landmark diagonal blocks) from the fp32 array themselves, so
    // the fp64 copy skips that region (bos::mf_fold_reads_fp32, mf_set_fold_source)
    bool fold32 = false;
    size_t tsize = 8;   // sizeof(T)
    // state
    double* d_pose = nullptr;
    double* d_lm = nullptr;
    void* d_pc = nullptr;
    void* d_pth = nullptr;
    void* d_lc = nullptr;
    // J+H work lists (host/plan.hpp BlockLayout)
    int32_t *pw_base = nullptr, *pw_stride = nullptr, *pl_cnt = nullptr, *lw_base = nullptr, *lw_stride = nullptr, *ll_cnt = nullptr, *ll_lm = nullptr, *po_ptr = nullptr, *po_ent = nullptr, *po_oth = nullptr, *po_blk = nullptr, *csr_src = nullptr,
            *elim_ref = nullptr;
    int32_t *pb_idx = nullptr, *lb_idx = nullptr, *ll_run = nullptr, *ll_hdr = nullptr;
    void *pb_z = nullptr, *pb_w = nullptr, *lb_z = nullptr, *lb_w = nullptr;
    int pose_blocks = 0;
    // odometry
    int32_t *o_src = nullptr, *o_dst = nullptr;
    void *o_z = nullptr, *o_om = nullptr;
    int om_stride = 6;                         // 0: every edge has the same information (LinParams)
    // node layout
    int32_t* node_dof = nullptr;
    // system
    void* d_val = nullptr;      // T, block array of H (BlockLayout)
    void* d_b = nullptr;        // T, 3 NP + 2 NL, reference dof numbering
    double* d_val64 = nullptr;  // fp32 build: fp64 copy of the block array for the solver
    double* d_csr64 = nullptr;  // dense / csrrf solvers: CSR values of P^T H_nf P (fp64)
    double* d_rhs = nullptr;    // n, permuted order; solution in place
    int32_t *d_rowptr = nullptr, *d_colind = nullptr;
    int32_t *d_Lptr = nullptr, *d_Lind = nullptr, *d_pivQ = nullptr;
    double* d_Lval = nullptr;
    double* d_dense = nullptr;
    int32_t* d_info = nullptr;
    double* d_chi_part = nullptr;
    int32_t* d_nrob_part = nullptr;
    bos::dev::StepStatus* d_status = nullptr;   // end-of-iteration summary (device)
    bos::dev::StepStatus* h_status = nullptr;   // its host-mapped mirror, written by the step's last kernel
    bos::dev::StepStatus* m_status = nullptr;   // device address of h_status
    // sharded step (world > 1): BOS_PARTITION_SUBTREE (sharded) or _OBSERVATIONS (obs)
    bool sharded = false, external = false;
    int partition = BOS_PARTITION_SUBTREE;
    bool obs = false;
    int64_t pose_b0 = 0, n_pose_run = 0, lm_b0 = 0, n_lm_run = 0;   // J+H blocks this rank runs
    void* d_sys = nullptr;        // obs: the all-reduced [H values | b] (T) the solve reads
    void* sys_val = nullptr;      // the block array and b the solve reads (d_val / d_b, or d_sys)
    void* sys_b = nullptr;
    int64_t vb_count = 0;         // obs: T values of [block array (even length) | b]
    int solve_stamp = 1;          // StepStatus stamp slot the solve's first launch writes
    int32_t* lane_pose = nullptr;            // J+H pose lane groups (Shard::lane_poses)
    bool lane_identity = false;              // group i runs pose i (one GPU): the kernel skips the table
    int chi_parts = 0;                       // J+H chi^2 partial blocks this rank counts
    double *ex1_send = nullptr, *ex1_recv = nullptr, *ex2_send = nullptr, *ex2_recv = nullptr;
    // every rank's exchange-1 header (chi^2, robust count), copied out of the mailbox by phase 1's
    // unpack right after its wait: a faster rank may push the next iteration's exchange 1 into the
    // mailbox before this rank's phase 2 combines the headers
    double* hdr1 = nullptr;
    uint64_t ex_timeout_ticks = 200000000ull;  // direct-exchange flag waits: 2 s (bos_set_exchange_timeout)
    // sharded: the receive buffers of both exchanges and the direct exchange's flags live in one
    // mailbox, uncached device memory (bos_exchange_p2p_connect maps every rank's into the others)
    char* mailbox = nullptr;
    bool mailbox_uncached = false;
    int64_t mb_ex1 = 0, mb_ex2 = 0, mb_flag1 = 0, mb_flag2 = 0;   // byte offsets
    bool p2p = false;                          // direct peer exchange connected
    double** d_peers = nullptr;                // [world] every rank's mailbox (own included)
    std::vector<void*> peer_maps;              // opened IPC mappings (closed at destroy)
    int64_t ex1_count = 0, ex2_count = 0;
    bos::dev::ExSeg *ex1_pack = nullptr, *ex1_unpack = nullptr;
    int n_abs = 1;                          // max |x| partials of exchange 2 (direct exchange)
    int n1p = 0, n1u = 0;
    int64_t maxlen1p = 0, maxlen1u = 0;
    int32_t *ex2_bnd = nullptr, *ex2_usrc = nullptr, *ex2_udst = nullptr;   // pack / unpack index lists
    int n_bnd = 0, n_bnd_remote = 0;
    int32_t* upd_nodes = nullptr;
    int n_upd = 0, n_upd_local = 0;
    double* abs_part = nullptr;
    int phase = 0;                           // next bos_step_phase expected (external mode)
    bool phase_first = true;
    // triangulation inputs: bearings grouped by landmark (file order), their pose and z (fp64)
    int32_t *tri_ptr = nullptr, *tri_obs = nullptr, *tri_pose = nullptr;
    double *tri_z = nullptr, *tri_scr = nullptr;
    double* d_maxpart = nullptr;                 // box-plus max |dx| per update block
    // the J+H build's static inputs (work lists, records, odometry) carved from one allocation
    // (JhStage): the fields below point into it and are not freed one by one
    char* jh_arena = nullptr;
    std::vector<void**> jh_fields;
    rocblas_handle rb = nullptr;
    rocsolver_rfinfo rf = nullptr;
    bos::dev::MfDevice* mf = nullptr;
    bool analyzed = false;
    ncclComm_t comm = nullptr;
    hipEvent_t ev[8] = {};
    std::vector<int32_t> ref_dof;   // permuted dof -> reference dof (size n + 3)
    bool have_dx = false;
    // odometry self-loops: z[3] and Omega upper triangle [6] each (constant chi^2 terms)
    std::vector<double> loop_z, loop_om;
    double* scrub = nullptr;   // bos_time_linearize(flush_caches): 2 x 512 MiB, one read between launches
    int scrub_turn = 0;
    // one-GPU multifrontal GN step captured once into a graph (every launch argument is fixed:
    // kernel threshold and damping are baked in, so setting them drops the graph)
    hipGraph_t graph = nullptr;          // the step after its J+H build (synchronous steps)
    hipGraphExec_t graph_exec = nullptr;
    hipGraph_t graph_full = nullptr;     // the whole step (the steps of a batch before its last)
    hipGraphExec_t exec_full = nullptr;
    hipGraph_t pgraph[3] = {};          // sharded step, external exchanges: one graph per phase
    hipGraphExec_t pexec[3] = {};
    // sharded step with a communicator: the whole iteration (phases and their RCCL collectives) as
    // one graph; rccl_capture_failed: RCCL could not be captured, the phase graphs run instead
    hipGraph_t sgraph = nullptr, stail = nullptr;   // the whole iteration; the iteration after its J+H build
    hipGraphExec_t sexec = nullptr, stail_exec = nullptr;
    bool rccl_capture_failed = false;
    bool graph_failed = false;   // capture not possible on this stream (e.g. the legacy null stream)
    // one GPU: the status sequence number last seen, and the status launches enqueued since (each
    // bumps the device counter once; wait_status polls for seq_seen + seq_pending)
    int32_t seq_seen = 0, seq_pending = 0;
};

static_assert(bos::dev::kStepAbort == bos::dev::kMfStall, "solver abort bit");
static_assert(bos::dev::kExHeader == bos::kExHeader, "exchange header size");

namespace {
// both multifrontal orderings (nested dissection / landmarks-first Schur) share the GPU engine
bool uses_mf(const bos_solver* s) {
    return s->solver_kind == BOS_SOLVER_SUPERNODAL || s->solver_kind == BOS_SOLVER_SCHUR;
}
}  // namespace

namespace {

template <typename T> bos::dev::LinParams<T> lin_params(const bos_solver* s) {
    bos::dev::LinParams<T> p;
    p.pc = (const T*)s->d_pc;
    p.pth = (const T*)s->d_pth;
    p.lc = (const T*)s->d_lc;
    const bos::Plan& P = s->plan;
    p.NP = s->NP;
    p.lane_pose = s->lane_identity ? nullptr : s->lane_pose;
    p.n_groups = (int)P.blk.lane_pose.size();
    p.n_lm_lanes = (int)P.blk.lm_lane_lm.size();
    p.pose_blocks = s->pose_blocks;
    p.pose_b0 = (int)s->pose_b0;
    p.n_pose_run = (int)s->n_pose_run;
    p.lm_b0 = (int)s->lm_b0;
    p.n_lm_run = (int)s->n_lm_run;
    p.pw_base = s->pw_base; p.pw_stride = s->pw_stride; p.pl_cnt = s->pl_cnt;
    p.pb_idx = s->pb_idx; p.pb_z = (const T*)s->pb_z; p.pb_w = (const T*)s->pb_w;
    p.po_ptr = s->po_ptr; p.po_ent = s->po_ent; p.po_oth = s->po_oth; p.po_blk = s->po_blk;
    p.o_src = s->o_src; p.o_dst = s->o_dst; p.o_z = (const T*)s->o_z; p.o_om = (const T*)s->o_om;
    p.om_stride = s->om_stride;
    p.lw_base = s->lw_base; p.lw_stride = s->lw_stride; p.ll_cnt = s->ll_cnt; p.ll_lm = s->ll_lm;
    p.lb_idx = s->lb_idx; p.lb_z = (const T*)s->lb_z; p.lb_w = (const T*)s->lb_w; p.ll_run = s->ll_run;
    p.ll_hdr = reinterpret_cast<const int2*>(s->ll_hdr);
    p.hval = (T*)s->d_val;
    p.b = (T*)s->d_b;
    p.off_ldiag = (int)P.blk.off_ldiag; p.off_pl = (int)P.blk.off_pl; p.off_pp = (int)P.blk.off_pp;
    p.chi2_part = s->d_chi_part;
    p.nrob_part = s->d_nrob_part;
    p.pl_factored = s->pl_factored ? 1 : 0;
    p.kt = (T)s->kt;
    p.lambda = (T)s->damping;
    p.diag_stamps = nullptr;
    p.t_start = nullptr;
    return p;
}

template <typename T> bos::dev::UpdateParams<T> upd_params(const bos_solver* s) {
    bos::dev::UpdateParams<T> u;
    u.NP = s->NP; u.NL = s->NL; u.fixed = s->plan.fixed;
    u.node_dof = s->node_dof;
    u.x = s->d_rhs;
    u.pose = s->d_pose; u.lm = s->d_lm;
    u.pc = (T*)s->d_pc; u.pth = (T*)s->d_pth; u.lc = (T*)s->d_lc;
    u.max_part = s->d_maxpart;
    // sharded: the abort bits of every rank's exchange-2 header (the local word was moved into it)
    // (sharded: the local word is zeroed by exchange 2's packing; it can then only carry the abort bit
    // of a direct-exchange wait that timed out)
    u.info = uses_mf(s) ? bos::dev::mf_info_ptr(s->mf) : nullptr;
    u.ex_hdr = s->sharded ? s->ex2_recv + 1 : nullptr;
    u.ex_stride = s->ex2_count;
    u.ex_world = s->world;
    u.nodes = s->sharded ? s->upd_nodes : nullptr;
    u.n_nodes = s->n_upd;
    u.t_start = nullptr;
    return u;
}

// Host staging of device arrays that are uploaded together into one allocation (each at a 256-byte
// aligned offset; an empty array stays null, as with upload)
struct JhStage {
    std::vector<char> host;
    std::vector<std::pair<void**, size_t>> fields;
    template <typename X> void add(X** p, const std::vector<X>& v) {
        *p = nullptr;
        if (v.empty()) return;
        const size_t off = (host.size() + 255) & ~(size_t)255;
        host.resize(off + v.size() * sizeof(X));
        std::memcpy(host.data() + off, v.data(), v.size() * sizeof(X));
        fields.push_back({reinterpret_cast<void**>(p), off});
    }
    template <typename T> void add_T(void** p, const std::vector<double>& v) {
        std::vector<T> t(v.begin(), v.end());
        add(reinterpret_cast<T**>(p), t);
    }
};

int flush_stage(bos_solver* s, JhStage& st) {
    if (st.host.empty()) return BOS_OK;
    HIP_TRY(hipMalloc((void**)&s->jh_arena, st.host.size()));
    HIP_TRY(hipMemcpy(s->jh_arena, st.host.data(), st.host.size(), hipMemcpyHostToDevice));
    for (auto& f : st.fields) {
        *f.first = s->jh_arena + f.second;
        s->jh_fields.push_back(f.first);
    }
    st = JhStage{};
    return BOS_OK;
}

int enqueue_linearize(bos_solver* s, unsigned long long* t_start = nullptr) {
    hipError_t e;
    const int lpp = s->plan.blk.lpp;
    if (s->precision == BOS_FP32) {
        bos::dev::LinParams<float> p = lin_params<float>(s);
        p.t_start = t_start;
        e = bos::dev::launch_linearize<float>(p, lpp, s->has_w, s->has_dups, s->stream);
    } else {
        bos::dev::LinParams<double> p = lin_params<double>(s);
        p.t_start = t_start;
        e = bos::dev::launch_linearize<double>(p, lpp, s->has_w, s->has_dups, s->stream);
    }
    if (e != hipSuccess) return fail(BOS_ERR_DEVICE, std::string("linearize launch: ") + hipGetErrorString(e));
    return BOS_OK;
}

// Exchange tables and buffers of the sharded step (host/shard.cpp): exchange 1 by segments of the
// update-matrix / u-vector arrays, exchange 2 by dof index lists.
int setup_shard(bos_solver* s) {
    const bos::Shard& S = s->plan.shard;
    const int W = s->world;
    int rc;
    s->ex1_count = S.ex1_count;
    s->ex2_count = S.ex2_count;
    std::vector<bos::ExchangeSeg> hp, hu;
    bos::exchange1_segments(s->plan, hp, hu);
    auto conv = [](const std::vector<bos::ExchangeSeg>& v, int64_t& maxlen) {
        std::vector<bos::dev::ExSeg> o(v.size());
        for (size_t i = 0; i < v.size(); ++i) {
            o[i] = {v[i].src, v[i].dst, v[i].len, v[i].src_kind, v[i].dst_kind};
            maxlen = std::max(maxlen, v[i].len);
        }
        return o;
    };
    const std::vector<bos::dev::ExSeg> pack = conv(hp, s->maxlen1p);
    std::vector<bos::dev::ExSeg> unpack = conv(hu, s->maxlen1u);
    for (int q = 0; q < W; ++q)   // rank q's header -> hdr1[q * kExHeader] (kind 4), after the wait
        unpack.push_back({(int64_t)q * S.ex1_count, (int64_t)q * bos::kExHeader, bos::kExHeader, 3, 4});
    s->maxlen1u = std::max<int64_t>(s->maxlen1u, bos::kExHeader);
    s->n1p = (int)pack.size();
    s->n1u = (int)unpack.size();
    std::vector<int32_t> bnd(S.bnd_dof.begin() + S.bnd_ptr[s->rank], S.bnd_dof.begin() + S.bnd_ptr[s->rank + 1]);
    std::vector<int32_t> usrc, udst;
    for (int q = 0; q < W; ++q) {
        if (q == s->rank) continue;
        for (int i = S.bnd_ptr[q]; i < S.bnd_ptr[q + 1]; ++i) {
            usrc.push_back((int32_t)((int64_t)q * S.ex2_count + bos::kExHeader + (i - S.bnd_ptr[q])));
            udst.push_back(S.bnd_dof[i]);
        }
    }
    s->n_bnd = (int)bnd.size();
    s->n_bnd_remote = (int)usrc.size();
    s->n_upd = (int)S.upd_nodes.size();
    s->n_upd_local = S.n_upd_local;
    if ((rc = upload(&s->ex1_pack, pack)) || (rc = upload(&s->ex1_unpack, unpack)) || (rc = upload(&s->ex2_bnd, bnd)) ||
        (rc = upload(&s->ex2_usrc, usrc)) || (rc = upload(&s->ex2_udst, udst)) || (rc = upload(&s->upd_nodes, S.upd_nodes)) ||
        (rc = dalloc(&s->ex1_send, (size_t)s->ex1_count)) || (rc = dalloc(&s->ex2_send, (size_t)s->ex2_count)) ||
        (rc = dalloc(&s->hdr1, (size_t)W * bos::kExHeader)) ||
        (rc = dalloc(&s->abs_part, (size_t)std::max(1, (S.n_upd_local + 255) / 256))))
        return rc;
    {   // the mailbox: [exchange 1: W x ex1_count][exchange 2: W x ex2_count][flags: 2 x W x 64 B]
        auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
        s->mb_ex1 = 0;
        s->mb_ex2 = al((int64_t)W * s->ex1_count * (int64_t)sizeof(double));
        s->mb_flag1 = s->mb_ex2 + al((int64_t)W * s->ex2_count * (int64_t)sizeof(double));
        s->mb_flag2 = s->mb_flag1 + 64 * (int64_t)W;
        const size_t bytes = (size_t)(s->mb_flag2 + 64 * (int64_t)W);
        if (hipExtMallocWithFlags((void**)&s->mailbox, bytes, hipDeviceMallocUncached) == hipSuccess) {
            s->mailbox_uncached = true;
        } else {
            (void)hipGetLastError();
            HIP_TRY(hipMalloc((void**)&s->mailbox, bytes));
        }
        HIP_TRY(hipMemset(s->mailbox, 0, bytes));
        s->ex1_recv = reinterpret_cast<double*>(s->mailbox + s->mb_ex1);
        s->ex2_recv = reinterpret_cast<double*>(s->mailbox + s->mb_ex2);
    }
    HIP_TRY(hipMemset(s->ex1_send, 0, s->ex1_count * sizeof(double)));
    HIP_TRY(hipMemset(s->ex2_send, 0, s->ex2_count * sizeof(double)));
    HIP_TRY(hipMemset(s->hdr1, 0, (size_t)W * bos::kExHeader * sizeof(double)));
    return BOS_OK;
}

// chi^2 and robust count of the odometry self-loops: constant (e = -z whatever the state, their
// Jacobian is zero, see host/plan.cpp build_layout), evaluated in T like the kernel. No J+H lane
// counts them, so every rank adds them once to the step's combined (summed over ranks) chi^2.
template <typename T> void self_loop_terms(const bos_solver* s, double& chi, int32_t& nrob) {
    chi = 0.0;
    nrob = 0;
    const T kt = (T)s->kt;
    for (size_t i = 0; i < s->loop_z.size() / 3; ++i) {
        const T* z = nullptr;
        T zz[3], u[6];
        for (int v = 0; v < 3; ++v) zz[v] = (T)s->loop_z[3 * i + v];
        for (int v = 0; v < 6; ++v) u[v] = (T)s->loop_om[6 * i + v];
        z = zz;
        const T e0 = (T)0 - z[0], e1 = (T)0 - z[1];
        const T e2 = bos::normalized_angle<T>(bos::normalized_angle<T>((T)0) - z[2]);
        const T Oe0 = u[0] * e0 + u[1] * e1 + u[2] * e2;
        const T Oe1 = u[1] * e0 + u[3] * e1 + u[4] * e2;
        const T Oe2 = u[2] * e0 + u[4] * e1 + u[5] * e2;
        const T rho = e0 * Oe0 + e1 * Oe1 + e2 * Oe2;
        chi += (double)rho;
        if (rho > kt) ++nrob;
    }
}

int enqueue_stats(bos_solver* s, bool with_update) {
    int32_t* info = uses_mf(s) ? bos::dev::mf_info_ptr(s->mf) : (s->solver_kind == BOS_SOLVER_DENSE_CHOL ? s->d_info : nullptr);
    const int nupd = (s->NP + s->NL + bos::dev::kUpdateBlock - 1) / bos::dev::kUpdateBlock;
    double chi_c = 0.0;
    int32_t nrob_c = 0;
    if (s->precision == BOS_FP32) self_loop_terms<float>(s, chi_c, nrob_c);
    else self_loop_terms<double>(s, chi_c, nrob_c);
    // observations partition: the all-reduced header [chi^2, robust count] instead of the partials
    HIP_TRY(bos::dev::launch_reduce_stats(s->obs ? s->ex1_recv : s->d_chi_part, s->obs ? nullptr : s->d_nrob_part,
                                          s->chi_parts, chi_c, nrob_c, with_update ? s->d_maxpart : nullptr, nupd, info,
                                          s->d_status, s->m_status, s->stream));
    return BOS_OK;
}

double self_loop_chi(const bos_solver* s, int32_t& nrob) {
    double c = 0.0;
    if (s->precision == BOS_FP32) self_loop_terms<float>(s, c, nrob);
    else self_loop_terms<double>(s, c, nrob);
    return c;
}

// the block array as the multifrontal solver reads it (fp64)
const double* mf_matrix(const bos_solver* s) {
    return s->precision == BOS_FP32 ? s->d_val64 : (const double*)s->sys_val;
}

// right-hand side in elimination order, and the fp64 copy of an fp32 block array. The gather also
// stamps the solve's start and opens the step's flow epoch (the first solver launch of a GN step).
int enqueue_solver_inputs(bos_solver* s) {
    const int64_t n = s->plan.n;
    const bool f32 = s->precision == BOS_FP32;
    unsigned long long* stamp = s->d_status->stamp + s->solve_stamp;
    uint32_t* epoch = uses_mf(s) ? bos::dev::mf_epoch_ptr(s->mf) : nullptr;
    const bool conv = f32 && uses_mf(s);   // the fp64 copy of the block array, in the same launch
    if (s->fold32) {   // the copy skips what the folds read from the fp32 array
        HIP_TRY(bos::dev::launch_gather_f64_ranges((const float*)s->sys_b, s->elim_ref, s->d_rhs, n, s->stream, stamp,
                                                   epoch, (const float*)s->sys_val, s->d_val64, s->plan.blk.size,
                                                   s->plan.blk.off_ldiag, s->plan.blk.off_pp));
        return BOS_OK;
    }
    if (s->pl_factored) {   // the copy expands the factored pose-landmark blocks
        HIP_TRY(bos::dev::launch_gather_f64_factored((const float*)s->sys_b, s->elim_ref, s->d_rhs, n, s->stream, stamp,
                                                     epoch, (const float*)s->sys_val, s->d_val64, s->plan.blk.size,
                                                     s->plan.blk.off_pl, s->plan.blk.pose_lanes.slots()));
        return BOS_OK;
    }
    HIP_TRY(f32 ? bos::dev::launch_gather_f64<float>((const float*)s->sys_b, s->elim_ref, s->d_rhs, n, s->stream, stamp, epoch,
                                                     conv ? (const float*)s->sys_val : nullptr, conv ? s->d_val64 : nullptr,
                                                     conv ? s->plan.blk.size : 0)
                : bos::dev::launch_gather_f64<double>((const double*)s->sys_b, s->elim_ref, s->d_rhs, n, s->stream, stamp, epoch));
    return BOS_OK;
}

int enqueue_solve(bos_solver* s, bool& ran_analysis) {
    const int64_t n = s->plan.n;
    ran_analysis = false;
    if (n == 0) return BOS_OK;
    const bool f32 = s->precision == BOS_FP32;
    int rc;
    if ((rc = enqueue_solver_inputs(s))) return rc;
    const rocblas_int nn = (rocblas_int)n;
    if (uses_mf(s)) {   // reads the block array through its assembly map
        HIP_TRY(bos::dev::mf_factor(s->mf, 0, mf_matrix(s), s->d_rhs, s->stream));
        HIP_TRY(bos::dev::mf_solve(s->mf, 0, s->d_rhs, s->stream));
        return BOS_OK;
    }
    double* A = s->d_csr64;
    HIP_TRY(f32 ? bos::dev::launch_gather_f64<float>((const float*)s->sys_val, s->csr_src, A, s->plan.nnzA(), s->stream)
                : bos::dev::launch_gather_f64<double>((const double*)s->sys_val, s->csr_src, A, s->plan.nnzA(), s->stream));
    if (s->solver_kind == BOS_SOLVER_DENSE_CHOL) {
        HIP_TRY(hipMemsetAsync(s->d_dense, 0, (size_t)n * n * sizeof(double), s->stream));
        HIP_TRY(bos::dev::launch_scatter_dense(s->d_rowptr, s->d_colind, A, nn, s->d_dense, s->stream));
        RB_TRY(rocsolver_dpotrf(s->rb, rocblas_fill_lower, nn, s->d_dense, nn, s->d_info));
        RB_TRY(rocsolver_dpotrs(s->rb, rocblas_fill_lower, nn, 1, s->d_dense, nn, s->d_rhs, nn));
        return BOS_OK;
    }
    const rocblas_int nnzA = (rocblas_int)s->plan.nnzA(), nnzT = (rocblas_int)s->plan.nnzL();
    if (!s->analyzed) {
        RB_TRY(rocsolver_dcsrrf_analysis(s->rb, nn, 1, nnzA, s->d_rowptr, s->d_colind, A, nnzT, s->d_Lptr, s->d_Lind,
                                         s->d_Lval, nullptr, s->d_pivQ, s->d_rhs, nn, s->rf));
        s->analyzed = true;
        ran_analysis = true;
    }
    RB_TRY(rocsolver_dcsrrf_refactchol(s->rb, nn, nnzA, s->d_rowptr, s->d_colind, A, nnzT, s->d_Lptr, s->d_Lind,
                                       s->d_Lval, s->d_pivQ, s->rf));
    RB_TRY(rocsolver_dcsrrf_solve(s->rb, nn, 1, nnzT, s->d_Lptr, s->d_Lind, s->d_Lval, nullptr, s->d_pivQ, s->d_rhs,
                                  nn, s->rf));
    return BOS_OK;
}

int enqueue_update(bos_solver* s) {
    hipError_t e;
    if (s->precision == BOS_FP32) {
        bos::dev::UpdateParams<float> u = upd_params<float>(s);
        u.t_start = s->d_status->stamp + 2;
        e = bos::dev::launch_boxplus<float>(u, s->stream);
    } else {
        bos::dev::UpdateParams<double> u = upd_params<double>(s);
        u.t_start = s->d_status->stamp + 2;
        e = bos::dev::launch_boxplus<double>(u, s->stream);
    }
    if (e != hipSuccess) return fail(BOS_ERR_DEVICE, std::string("boxplus launch: ") + hipGetErrorString(e));
    return BOS_OK;
}

// State caches in T precision (x, y, cos, sin per pose; theta; landmark x, y) computed on the host
// from the master state with the host libm, exactly as the CPU oracle evaluates them, so that
// iteration 0 is bit-reproducible against it (see host/det_atan2.hpp); the box-plus kernel keeps
// them current afterwards.
template <typename T> int upload_cache_T(bos_solver* s) {
    const int NP = s->NP, NL = s->NL;
    std::vector<double> pose(3 * (size_t)NP), lm(2 * (size_t)NL);
    HIP_TRY(hipMemcpy(pose.data(), s->d_pose, pose.size() * sizeof(double), hipMemcpyDeviceToHost));
    if (NL) HIP_TRY(hipMemcpy(lm.data(), s->d_lm, lm.size() * sizeof(double), hipMemcpyDeviceToHost));
    std::vector<T> pc(4 * (size_t)NP), pth(NP), lc(2 * (size_t)NL);
    for (int i = 0; i < NP; ++i) {
        const T th = (T)pose[3 * (size_t)i + 2];
        pc[4 * (size_t)i] = (T)pose[3 * (size_t)i];
        pc[4 * (size_t)i + 1] = (T)pose[3 * (size_t)i + 1];
        pc[4 * (size_t)i + 2] = std::cos(th);
        pc[4 * (size_t)i + 3] = std::sin(th);
        pth[i] = th;
    }
    for (size_t j = 0; j < lc.size(); ++j) lc[j] = (T)lm[j];
    HIP_TRY(hipMemcpy(s->d_pc, pc.data(), pc.size() * sizeof(T), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s->d_pth, pth.data(), pth.size() * sizeof(T), hipMemcpyHostToDevice));
    if (NL) HIP_TRY(hipMemcpy(s->d_lc, lc.data(), lc.size() * sizeof(T), hipMemcpyHostToDevice));
    return BOS_OK;
}

int upload_cache(bos_solver* s) { return s->precision == BOS_FP32 ? upload_cache_T<float>(s) : upload_cache_T<double>(s); }

float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.f;
    return ms;
}

template <typename T> bos::dev::TriParams<T> tri_params(const bos_solver* s) {
    bos::dev::TriParams<T> p;
    p.NL = s->NL;
    p.lm_ptr = s->tri_ptr; p.lm_obs = s->tri_obs; p.b_pose = s->tri_pose; p.b_z = s->tri_z;
    p.pose = s->d_pose; p.scratch = s->tri_scr; p.lm = s->d_lm; p.lc = (T*)s->d_lc;
    return p;
}

int enqueue_triangulate(bos_solver* s) {
    const hipError_t e = s->precision == BOS_FP32 ? bos::dev::launch_triangulate<float>(tri_params<float>(s), s->stream)
                                                  : bos::dev::launch_triangulate<double>(tri_params<double>(s), s->stream);
    if (e != hipSuccess) return fail(BOS_ERR_DEVICE, std::string("triangulate launch: ") + hipGetErrorString(e));
    return BOS_OK;
}

// The step status (one copy). The sticky abort flag is cleared here once reported, so every
// bos_step / bos_step_n batch starts with it clear.
// Waits for the status of the last enqueued step. One GPU: the host polls the sequence number the
// step's last kernel writes to the host-mapped mirror after the summary (a system-scope release in
// between), which it sees ~10 us before a stream synchronisation returns (tools/sync_step_trace.py);
// the stream is not synchronised (every later call that reads device memory synchronises it, and
// launches are stream ordered). A fault or an unexpected state falls back to the stream wait.
int wait_status(bos_solver* s, bool sync) {
    if (!sync && s->seq_pending > 0) {
        const int32_t target = s->seq_seen + s->seq_pending;
        s->seq_seen = target;
        s->seq_pending = 0;
        const volatile int32_t* q = &s->h_status->seq;
        for (uint64_t it = 1;; ++it) {
            if (*q == target) {
                std::atomic_thread_fence(std::memory_order_acquire);
                return BOS_OK;
            }
            if ((it & 4095) == 0) {   // the stream done (or failed) without the number: report it
                const hipError_t e = hipStreamQuery(s->stream);
                if (e != hipErrorNotReady) {
                    if (*q == target) break;
                    s->seq_seen = *q;   // what the device actually wrote: the next step waits for its own number
                    if (e != hipSuccess) HIP_TRY(e);
                    return fail(BOS_ERR_DEVICE, "step status sequence number not written");
                }
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        return BOS_OK;
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->seq_seen = s->h_status->seq;   // the device counter, whatever ran
    s->seq_pending = 0;
    return BOS_OK;
}

// sync: wait for the stream (callers that read events or device memory next), not only the status
int read_stats(bos_solver* s, bos_step_stats* st, int32_t* aborted = nullptr, bool sync = false) {
    int rc;
    if ((rc = wait_status(s, sync))) return rc;
    bos::dev::StepStatus h;
    std::memcpy(&h, (const void*)s->h_status, sizeof(h));   // written by the step's last kernel
    if (h.aborted) {
        HIP_TRY(hipMemsetAsync(&s->d_status->aborted, 0, sizeof(int32_t), s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
    }
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->chi2 = h.chi2;
        st->n_robust = h.n_robust;
        st->solver_info = h.info & ~bos::dev::kStepAbort;
        st->max_abs_dx = h.max_dx;
        if (!s->sharded) {   // phase boundaries stamped by the step's kernels
            auto d = [](unsigned long long a, unsigned long long b) { return b > a ? (double)(b - a) * bos::dev::kStampMs : 0.0; };
            st->t_linearize_ms = d(h.stamp[0], h.stamp[1]);
            // observations partition: J+H end [1], the all-reduce, solve start [4]
            st->t_exchange_ms = s->obs ? d(h.stamp[1], h.stamp[4]) : 0.0;
            st->t_solve_ms = d(h.stamp[s->solve_stamp], h.stamp[2]);
            st->t_update_ms = d(h.stamp[2], h.stamp[3]);
        }
    }
    if (aborted) *aborted = h.aborted;
    return BOS_OK;
}

// ---- sharded GN iteration in three phases (exchanges between them). With a communicator the
// whole iteration — the phases and the two ncclAllGather calls between them — is captured once into
// one graph and replayed (do_step_sharded); in external mode (the caller moves the buffers) each
// phase is a graph of its own. Phase boundaries are stamped by the phases' own kernels (StepStatus
// stamp slots 0-7), not by events.
// phase 0: J+H (own + top lanes), solver inputs, own subtrees factored (and forward-solved),
// exchange-1 buffer packed (roots' U / u, this rank's chi^2 partials)
// phase 1: the other ranks' roots in place, the top factored and solved, own subtrees solved
// backward, exchange-2 buffer packed (max |x| of own + top, solver word, boundary solution)
// phase 2: boundary solution in place, box-plus of own + top + boundary nodes (skipped when any
// rank's factorization aborted: every rank's header), step status combined from every rank's headers
// the wait for exchange `which` of the direct exchange, fused into the launch that reads it (none
// without the direct exchange)
bos::dev::P2PWait p2p_wait(const bos_solver* s, int which) {
    bos::dev::P2PWait w;
    if (!s->p2p) return w;
    w.mailbox = s->mailbox;
    w.flag_off = which == 1 ? s->mb_flag1 : s->mb_flag2;
    w.world = s->world;
    w.epoch = bos::dev::mf_epoch_ptr(s->mf);
    w.info = bos::dev::mf_info_ptr(s->mf);
    w.timeout_ticks = s->ex_timeout_ticks;
    return w;
}

int shard_enqueue(bos_solver* s, int phase, bool with_jh = true) {
    int rc;
    double* U = bos::dev::mf_update_ptr(s->mf);
    double* u = bos::dev::mf_uvec_ptr(s->mf);
    if (phase == 0) {
        if (with_jh && (rc = enqueue_linearize(s, s->d_status->stamp))) return rc;
        if ((rc = enqueue_solver_inputs(s))) return rc;   // opens this step's flow epoch
        HIP_TRY(bos::dev::mf_factor(s->mf, 0, mf_matrix(s), s->d_rhs, s->stream));
        if (!s->p2p) {   // (the direct exchange's push gathers the payload and computes the header itself)
            HIP_TRY(bos::dev::launch_seg_copy<double>(U, u, s->ex1_send, s->ex1_recv, s->hdr1, s->ex1_pack, s->n1p,
                                                      s->maxlen1p, s->stream));
            HIP_TRY(bos::dev::launch_shard_header1(s->d_chi_part, s->d_nrob_part, s->chi_parts, s->ex1_send, s->stream,
                                                   s->d_status->stamp + 4));
        }
    } else if (phase == 1) {
        HIP_TRY(bos::dev::launch_seg_copy<double>(U, u, s->ex1_send, s->ex1_recv, s->hdr1, s->ex1_unpack, s->n1u, s->maxlen1u,
                                                  s->stream, s->d_status->stamp + 5, p2p_wait(s, 1)));
        HIP_TRY(bos::dev::mf_factor(s->mf, 1, mf_matrix(s), s->d_rhs, s->stream));
        HIP_TRY(bos::dev::mf_solve(s->mf, 1, s->d_rhs, s->stream));
        HIP_TRY(bos::dev::mf_solve(s->mf, 0, s->d_rhs, s->stream));
        if (s->p2p) {   // the push packs exchange 2 itself (exchange()); the max |x| partials first
            hipError_t e = hipSuccess;
            s->n_abs = bos::dev::launch_node_absmax(s->d_rhs, s->upd_nodes, s->n_upd_local, s->node_dof, s->NP,
                                                    s->abs_part, s->stream, &e);
            HIP_TRY(e);
        } else {
            HIP_TRY(bos::dev::launch_shard_pack2(s->d_rhs, s->upd_nodes, s->n_upd_local, s->node_dof, s->NP,
                                                 bos::dev::mf_info_ptr(s->mf), s->ex2_bnd, s->n_bnd, s->abs_part,
                                                 s->ex2_send, s->stream, s->d_status->stamp + 6));
        }
    } else {
        HIP_TRY(bos::dev::launch_index_copy(s->ex2_recv, s->ex2_usrc, s->d_rhs, s->ex2_udst, s->n_bnd_remote, s->stream,
                                            s->d_status->stamp + 7, p2p_wait(s, 2)));
        if ((rc = enqueue_update(s))) return rc;
        int32_t nrob_c = 0;
        const double chi_c = self_loop_chi(s, nrob_c);
        // exchange-1 headers from phase 1's local copy (the mailbox may already hold the next
        // iteration's); exchange 2's are still current (no rank pushes again before this rank does)
        HIP_TRY(bos::dev::launch_shard_combine(s->hdr1, bos::kExHeader, s->ex2_recv, s->ex2_count, s->world, chi_c,
                                               nrob_c, bos::dev::mf_info_ptr(s->mf), s->d_status, s->m_status, s->stream,
                                               s->p2p));
    }
    return BOS_OK;
}

int capture(bos_solver* s, int phase, hipGraph_t* graph, hipGraphExec_t* exec);
int enqueue_step_tail(bos_solver* s);

// ---- BOS_PARTITION_OBSERVATIONS step (the north star's form): phase 0 = this rank's range of J+H
// lanes and its chi^2 / robust-count header (external mode: the whole [header | H values | b] in
// fp64 into the exchange buffer); one all-reduce (sum) over the ranks; phase 1 = (external: the
// summed buffer back into T) the one-GPU solve, box-plus of every node and stats. Every value of H and
// b is written by exactly one rank's lanes and is zero on the others, so the sum is exact and every
// rank solves the one-GPU system bit for bit.
int obs_enqueue(bos_solver* s, int phase, bool with_jh = true) {
    int rc;
    const bool f32 = s->precision == BOS_FP32;
    if (phase == 0) {
        if (with_jh && (rc = enqueue_linearize(s, s->d_status->stamp))) return rc;
        HIP_TRY(bos::dev::launch_shard_header1(s->d_chi_part, s->d_nrob_part, s->chi_parts, s->ex1_send, s->stream,
                                               s->d_status->stamp + 1));
        if (s->external)
            HIP_TRY(f32 ? bos::dev::launch_to_f64<float>((const float*)s->d_val, s->ex1_send + bos::kExHeader, s->vb_count, s->stream)
                        : bos::dev::launch_to_f64<double>((const double*)s->d_val, s->ex1_send + bos::kExHeader, s->vb_count, s->stream));
        return BOS_OK;
    }
    if (s->external)
        HIP_TRY(f32 ? bos::dev::launch_from_f64<float>(s->ex1_recv + bos::kExHeader, (float*)s->d_sys, s->vb_count, s->stream)
                    : bos::dev::launch_from_f64<double>(s->ex1_recv + bos::kExHeader, (double*)s->d_sys, s->vb_count, s->stream));
    return enqueue_step_tail(s);
}

int rccl_allreduce_obs(bos_solver* s);

int obs_phase(bos_solver* s, int phase) {
    int rc;
    if (!s->pexec[phase] && !s->graph_failed && (rc = capture(s, 10 + phase, &s->pgraph[phase], &s->pexec[phase]))) return rc;
    if (s->pexec[phase]) HIP_TRY(hipGraphLaunch(s->pexec[phase], s->stream));
    else if ((rc = obs_enqueue(s, phase))) return rc;
    return BOS_OK;
}

// the one exchange: (H values | b) in T and the header, summed over the ranks (one RCCL group)
int rccl_allreduce_obs(bos_solver* s) {
    const ncclDataType_t t = s->precision == BOS_FP32 ? ncclFloat : ncclDouble;
    NC_TRY(ncclGroupStart());
    const ncclResult_t r1 = ncclAllReduce(s->d_val, s->d_sys, (size_t)s->vb_count, t, ncclSum, s->comm, s->stream);
    const ncclResult_t r2 = ncclAllReduce(s->ex1_send, s->ex1_recv, bos::kExHeader, ncclDouble, ncclSum, s->comm, s->stream);
    NC_TRY(ncclGroupEnd());
    NC_TRY(r1);
    NC_TRY(r2);
    return BOS_OK;
}

// one phase: its graph (captured on first use)
int shard_phase(bos_solver* s, int phase) {
    int rc;
    if (!s->pexec[phase] && !s->graph_failed && (rc = capture(s, phase, &s->pgraph[phase], &s->pexec[phase]))) return rc;
    if (s->pexec[phase]) HIP_TRY(hipGraphLaunch(s->pexec[phase], s->stream));
    else if ((rc = shard_enqueue(s, phase))) return rc;
    return BOS_OK;
}
int shard_phase0(bos_solver* s) { return shard_phase(s, 0); }
int shard_phase1(bos_solver* s) { return shard_phase(s, 1); }
int shard_phase2(bos_solver* s) { return shard_phase(s, 2); }

int rccl_allgather(bos_solver* s, const double* send, double* recv, int64_t count) {
    NC_TRY(ncclAllGather(send, recv, (size_t)count, ncclDouble, s->comm, s->stream));
    return BOS_OK;
}

int finish_step(bos_solver* s, bos_step_stats* st);

// one all-gather of the sharded step: RCCL, or the direct peer exchange's push to every rank's
// mailbox (the push gathers its payload and computes the header; the receiving side's wait is fused
// into the launch that reads the data, p2p_wait)
int exchange(bos_solver* s, int which) {
    const double* send = which == 1 ? s->ex1_send : s->ex2_send;
    double* recv = which == 1 ? s->ex1_recv : s->ex2_recv;
    const int64_t count = which == 1 ? s->ex1_count : s->ex2_count;
    if (!s->p2p) return rccl_allgather(s, send, recv, count);
    const int64_t data = which == 1 ? s->mb_ex1 : s->mb_ex2, flag = which == 1 ? s->mb_flag1 : s->mb_flag2;
    // the push gathers its payload where it lives (exchange 1: the subtree roots' U / u by the pack
    // segments, with the chi^2 header; exchange 2: the boundary solution with the max |x| / solver-word
    // header): no pack launch before it
    bos::dev::P2PPush p;
    p.which = which;
    p.peers = s->d_peers;
    p.data_off = data;
    p.flag_off = flag;
    p.count = count;
    p.rank = s->rank;
    p.world = s->world;
    p.epoch = bos::dev::mf_epoch_ptr(s->mf);
    if (which == 1) {
        p.stamp = s->d_status->stamp + 4;
        p.chi_part = s->d_chi_part;
        p.nrob_part = s->d_nrob_part;
        p.n_parts = s->chi_parts;
        p.U = bos::dev::mf_update_ptr(s->mf);
        p.u = bos::dev::mf_uvec_ptr(s->mf);
        p.segs = s->ex1_pack;
        p.nseg = s->n1p;
    } else {
        p.stamp = s->d_status->stamp + 6;
        p.x = s->d_rhs;
        p.abs_part = s->abs_part;
        p.n_abs = s->n_abs;
        p.info = bos::dev::mf_info_ptr(s->mf);
        p.bnd = s->ex2_bnd;
        p.n_bnd = s->n_bnd;
    }
    HIP_TRY(bos::dev::launch_p2p_push_gather(p, s->stream));
    return BOS_OK;
}

// the whole sharded iteration with its exchanges (on the handle's stream); with_jh false:
// everything after the J+H build
int enqueue_sharded_step(bos_solver* s, bool with_jh = true) {
    int rc;
    if ((rc = shard_enqueue(s, 0, with_jh)) || (rc = exchange(s, 1)) || (rc = shard_enqueue(s, 1)) ||
        (rc = exchange(s, 2)))
        return rc;
    return shard_enqueue(s, 2);
}

// the whole observations-partition iteration with its all-reduce (with_jh false: after the J+H build)
int enqueue_obs_step(bos_solver* s, bool with_jh = true) {
    int rc;
    if ((rc = obs_enqueue(s, 0, with_jh)) || (rc = rccl_allreduce_obs(s))) return rc;
    return obs_enqueue(s, 1);
}

// One graph for a multi-rank iteration with its RCCL collectives, and one of the iteration after
// its J+H build (captured on first use). If the collectives cannot be captured,
// rccl_capture_failed is set and the caller runs the phase graphs with the collectives between them
// instead (the same launches in the same order).
int capture_rccl_graph(bos_solver* s, bool with_jh, hipGraph_t* graph, hipGraphExec_t* exec) {
    if (hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        s->graph_failed = true;
        return BOS_OK;
    }
    const int rc = s->obs ? enqueue_obs_step(s, with_jh) : enqueue_sharded_step(s, with_jh);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s->stream, &g);
    if (rc || e != hipSuccess || !g) {
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        s->rccl_capture_failed = true;   // (a launch error reappears on the eager path)
        return BOS_OK;
    }
    if (hipGraphInstantiate(exec, g, nullptr, nullptr, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipGraphDestroy(g);
        *exec = nullptr;
        s->rccl_capture_failed = true;
        return BOS_OK;
    }
    *graph = g;
    return BOS_OK;
}

int capture_rccl_step(bos_solver* s) {
    int rc;
    if (s->graph_failed || s->rccl_capture_failed) return BOS_OK;
    if (!s->sexec && (rc = capture_rccl_graph(s, true, &s->sgraph, &s->sexec))) return rc;
    if (s->sexec && !s->stail_exec && (rc = capture_rccl_graph(s, false, &s->stail, &s->stail_exec))) return rc;
    return BOS_OK;
}

// A multi-rank iteration on RCCL (sharded or observations partition): a batch's steps before its
// last replay the whole iteration's graph; a synchronous step launches its J+H build directly and
// the rest as a graph submitted while the build runs (as the one-GPU step, launch_step).
int launch_rccl_step(bos_solver* s, bool sync) {
    int rc;
    if ((rc = capture_rccl_step(s))) return rc;
    if (!sync && s->sexec) {
        HIP_TRY(hipGraphLaunch(s->sexec, s->stream));
    } else if (s->stail_exec) {
        if ((rc = enqueue_linearize(s, s->d_status->stamp))) return rc;
        HIP_TRY(hipGraphLaunch(s->stail_exec, s->stream));
    } else if (s->obs) {
        if ((rc = obs_phase(s, 0)) || (rc = rccl_allreduce_obs(s)) || (rc = obs_phase(s, 1))) return rc;
    } else if ((rc = shard_phase0(s)) || (rc = exchange(s, 1)) || (rc = shard_phase1(s)) || (rc = exchange(s, 2)) ||
               (rc = shard_phase2(s))) {
        return rc;
    }
    ++s->seq_pending;   // the iteration's status launch bumps the device counter once
    return BOS_OK;
}

int do_step_sharded(bos_solver* s, bos_step_stats* st, bool sync) {
    if (!s->comm && !s->p2p)
        return fail(BOS_ERR_INVALID, "sharded handle without a communicator or direct exchange: drive bos_step_phase");
    int rc;
    if ((rc = launch_rccl_step(s, sync))) return rc;
    s->have_dx = true;
    if (!sync) return BOS_OK;
    return finish_step(s, st);
}

// reads the status of the step just enqueued (sharded: phases 0-2), fails an aborted one
int finish_step(bos_solver* s, bos_step_stats* st) {
    int rc;
    int32_t aborted = 0;
    if ((rc = read_stats(s, st, &aborted))) return rc;
    if (aborted) {
        s->have_dx = false;
        return fail(BOS_ERR_SOLVER, "sparse factorization aborted: a dataflow dependency wait timed out (state "
                                    "left unchanged by the failed iteration)");
    }
    if (st && s->sharded) {   // phase boundaries stamped by the phases' kernels (StepStatus::stamp)
        bos::dev::StepStatus h;
        std::memcpy(&h, (const void*)s->h_status, sizeof(h));
        auto d = [](unsigned long long a, unsigned long long b) { return b > a ? (double)(b - a) * bos::dev::kStampMs : 0.0; };
        st->t_linearize_ms = d(h.stamp[0], h.stamp[1]);
        st->t_solve_ms = d(h.stamp[1], h.stamp[4]) + d(h.stamp[5], h.stamp[6]);
        st->t_exchange_ms = d(h.stamp[4], h.stamp[5]) + d(h.stamp[6], h.stamp[7]);
        st->t_update_ms = d(h.stamp[7], h.stamp[3]);
    }
    return BOS_OK;
}

// The device work of one GN iteration on one GPU: J+H (stamp 0 at its start), solve (its first
// launch stamps 1 and opens the flows' epoch), box-plus (stamp 2), status (stamp 3 at its end, then
// the host-mapped copy). No events, no marker launches, no host synchronisation: the sequence after
// the J+H build is captured once into a hipGraph and replayed (do_step).
// the step after the J+H build (the captured graph: see do_step)
int enqueue_step_tail(bos_solver* s) {
    int rc;
    bool analysed_now = false;
    if ((rc = enqueue_solve(s, analysed_now))) return rc;
    if ((rc = enqueue_update(s))) return rc;
    return enqueue_stats(s, true);
}

int enqueue_step(bos_solver* s) {
    int rc;
    if ((rc = enqueue_linearize(s, s->d_status->stamp))) return rc;
    return enqueue_step_tail(s);
}

void drop_graph(bos_solver* s) {
    // bos_step returns on the status sequence number, before the stream has drained: a graph may
    // still be running
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->graph_exec) (void)hipGraphExecDestroy(s->graph_exec);
    if (s->graph) (void)hipGraphDestroy(s->graph);
    s->graph_exec = nullptr;
    s->graph = nullptr;
    if (s->exec_full) (void)hipGraphExecDestroy(s->exec_full);
    if (s->graph_full) (void)hipGraphDestroy(s->graph_full);
    s->exec_full = nullptr;
    s->graph_full = nullptr;
    for (int i = 0; i < 3; ++i) {
        if (s->pexec[i]) (void)hipGraphExecDestroy(s->pexec[i]);
        if (s->pgraph[i]) (void)hipGraphDestroy(s->pgraph[i]);
        s->pexec[i] = nullptr;
        s->pgraph[i] = nullptr;
    }
    if (s->sexec) (void)hipGraphExecDestroy(s->sexec);
    if (s->sgraph) (void)hipGraphDestroy(s->sgraph);
    if (s->stail_exec) (void)hipGraphExecDestroy(s->stail_exec);
    if (s->stail) (void)hipGraphDestroy(s->stail);
    s->sexec = s->stail_exec = nullptr;
    s->sgraph = s->stail = nullptr;
}

// Capture the launches of one GN step (phase -1: the one-GPU step after its J+H build,
// enqueue_step_tail; -2: the whole one-GPU step; 0-2: a subtree-sharded phase; 10-11: an
// observations-partition phase) into *exec (multifrontal
// solvers: rocSOLVER's paths are not captured). A stream that cannot be captured leaves
// graph_failed set and the launches run eagerly, the same ones in the same order.
int capture(bos_solver* s, int phase, hipGraph_t* graph, hipGraphExec_t* exec) {
    if (hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        s->graph_failed = true;
        return BOS_OK;
    }
    const int rc = phase == -1   ? enqueue_step_tail(s)
                   : phase == -2 ? enqueue_step(s)
                   : phase >= 10 ? obs_enqueue(s, phase - 10)
                                 : shard_enqueue(s, phase);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(s->stream, &g);
    if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    if (e != hipSuccess || !g) return fail(BOS_ERR_DEVICE, std::string("step graph capture: ") + hipGetErrorString(e));
    *graph = g;
    HIP_TRY(hipGraphInstantiate(exec, g, nullptr, nullptr, 0));
    return BOS_OK;
}

int launch_step(bos_solver* s, bool sync);

// One GN iteration. sync: read the status back (the last step of a bos_step_n batch). A
// factorization whose dataflow launch timed out leaves the state untouched (the box-plus kernel
// checks the solver word) and fails the call.
int do_step(bos_solver* s, bos_step_stats* st, bool sync) {
    if (s->sharded) return do_step_sharded(s, st, sync);
    int rc;
    if (s->obs) {
        if (!s->comm) return fail(BOS_ERR_INVALID, "observations-partition handle without a communicator: drive bos_step_phase");
        if ((rc = launch_rccl_step(s, sync))) return rc;
    } else if ((rc = launch_step(s, sync))) {
        return rc;
    } else {
        ++s->seq_pending;   // the step's status launch (now enqueued) bumps the device counter once
    }
    s->have_dx = true;
    if (!sync) return BOS_OK;
    int32_t aborted = 0;
    if ((rc = read_stats(s, st, &aborted))) return rc;
    if (aborted) {
        s->have_dx = false;
        return fail(BOS_ERR_SOLVER, "sparse factorization aborted: a dataflow dependency wait timed out (state "
                                    "left unchanged by the failed iteration)");
    }
    return BOS_OK;
}

// The launches of one one-GPU GN iteration (see do_step)
int launch_step(bos_solver* s, bool sync) {
    int rc;
    if (uses_mf(s) && !s->graph_exec && !s->graph_failed && (rc = capture(s, -1, &s->graph, &s->graph_exec))) return rc;
    if (uses_mf(s) && !s->exec_full && !s->graph_failed && (rc = capture(s, -2, &s->graph_full, &s->exec_full)))
        return rc;   // both graphs at the first step, so neither kind of call pays a capture later
    if (!sync && s->exec_full) {
        // a batch's step before its last: the host is ahead of the device, one graph per step
        HIP_TRY(hipGraphLaunch(s->exec_full, s->stream));
    } else if (s->graph_exec) {
        // synchronous: the J+H build launched directly (it starts a few us after the call), the
        // rest of the step as the graph, submitted while the build runs (a graph's first kernel
        // starts 13-25 us after hipGraphLaunch, tools/sync_step_trace.py; launching the input
        // gather directly too measured slower: 1 760 against 1 790 it/s)
        if ((rc = enqueue_linearize(s, s->d_status->stamp))) return rc;
        HIP_TRY(hipGraphLaunch(s->graph_exec, s->stream));
    } else if ((rc = enqueue_step(s))) {
        return rc;
    }
    return BOS_OK;
}

// 512 MiB read (2x the Infinity Cache) from one of two buffers, alternately: afterwards L2 and the
// Infinity Cache hold none of the build's inputs, and no scrub finds the previous scrub's lines there
// (so the time of a scrub does not depend on what ran before it)
int scrub_caches(bos_solver* s) {
    constexpr int64_t kScrub = (int64_t)1 << 26;   // doubles per buffer
    int rc;
    if (!s->scrub) {
        if ((rc = dalloc(&s->scrub, 2 * kScrub + 1))) return rc;
        HIP_TRY(hipMemset(s->scrub, 0, (2 * kScrub + 1) * sizeof(double)));
    }
    const double* buf = s->scrub + (s->scrub_turn++ & 1) * kScrub;
    HIP_TRY(bos::dev::launch_cache_scrub(buf, kScrub, s->scrub + 2 * kScrub, s->stream));
    return BOS_OK;
}

}  // namespace

extern "C" {

int bos_abi_version(void) { return BOS_ABI_VERSION; }

int bos_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int bos_device_peer_access(int32_t capacity, int32_t* out, int32_t* n_out) {
    if (!out || !n_out || capacity < 0) return fail(BOS_ERR_INVALID, "bad argument");
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess) {
        (void)hipGetLastError();
        nd = 0;
    }
    const int n = std::min<int>(nd, capacity);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            int ok = i == j;
            if (i != j && hipDeviceCanAccessPeer(&ok, i, j) != hipSuccess) {
                (void)hipGetLastError();
                ok = 0;
            }
            out[(int64_t)i * n + j] = ok ? 1 : 0;
        }
    *n_out = n;
    return BOS_OK;
}

void bos_default_options(bos_options* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->precision = BOS_FP64;
    o->solver = BOS_SOLVER_SPARSE_CHOL;
    o->device = -1;
    o->rank = 0;
    o->world_size = 1;
    o->kernel_threshold = 1.0;
    o->damping = 0.01;
}

int bos_nccl_unique_id(void* out, int64_t len) {
    if (!out || len < (int64_t)sizeof(ncclUniqueId)) return fail(BOS_ERR_INVALID, "bos_nccl_unique_id: buffer too small");
    ncclUniqueId id;
    NC_TRY(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof(id));
    return BOS_OK;
}

int bos_destroy(bos_solver* s) {
    if (!s) return BOS_OK;
    if (s->device >= 0) (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    drop_graph(s);
    for (void** f : s->jh_fields) *f = nullptr;   // inside jh_arena
    void* bufs[] = {s->d_pose, s->d_lm, s->d_pc, s->d_pth, s->d_lc, s->pw_base, s->pw_stride, s->pl_cnt, s->lw_base, s->lw_stride, s->ll_cnt, s->ll_lm,
                    s->po_ptr, s->po_ent, s->po_oth, s->po_blk, s->csr_src, s->elim_ref, s->pb_idx, s->pb_z, s->pb_w, s->lb_idx, s->lb_z, s->lb_w, s->ll_run, s->ll_hdr,
                    s->o_src, s->o_dst, s->o_z, s->o_om, s->node_dof, s->d_val, s->obs ? nullptr : s->d_b, s->d_sys,
                    s->d_val64, s->d_csr64,
                    s->d_rhs, s->d_rowptr, s->d_colind, s->d_Lptr, s->d_Lind, s->d_pivQ,
                    s->d_Lval, s->d_dense, s->d_info, s->d_chi_part, s->d_nrob_part, s->d_status,
                    s->d_maxpart, s->tri_ptr, s->tri_obs, s->tri_pose, s->tri_z, s->tri_scr,
                    s->scrub, s->lane_pose, s->ex1_send, s->obs ? s->ex1_recv : nullptr, s->ex2_send, s->mailbox,
                    s->d_peers, s->ex1_pack, s->hdr1,
                    s->ex1_unpack, s->ex2_bnd, s->ex2_usrc, s->ex2_udst, s->upd_nodes, s->abs_part, s->jh_arena};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (s->h_status) (void)hipHostFree(s->h_status);
    for (void* m : s->peer_maps) (void)hipIpcCloseMemHandle(m);
    if (s->rf) rocsolver_destroy_rfinfo(s->rf);
    if (s->mf) bos::dev::mf_destroy(s->mf);
    if (s->rb) rocblas_destroy_handle(s->rb);
    if (s->comm) ncclCommDestroy(s->comm);
    for (hipEvent_t& e : s->ev)
        if (e) (void)hipEventDestroy(e);
    if (s->own_stream && s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return BOS_OK;
}

int bos_create(const bos_problem* pb, const bos_options* opt_in, bos_solver** out) {
    if (!pb || !out) return fail(BOS_ERR_INVALID, "bos_create: null argument");
    *out = nullptr;
    bos_options opt;
    bos_default_options(&opt);
    if (opt_in) opt = *opt_in;
    if (opt.precision != BOS_FP64 && opt.precision != BOS_FP32) return fail(BOS_ERR_INVALID, "precision must be 32 or 64");
    if (opt.solver != BOS_SOLVER_SUPERNODAL && opt.solver != BOS_SOLVER_DENSE_CHOL &&
        opt.solver != BOS_SOLVER_ROCSOLVER_RF && opt.solver != BOS_SOLVER_SCHUR)
        return fail(BOS_ERR_INVALID, "unknown solver");
    if (opt.partition != BOS_PARTITION_SUBTREE && opt.partition != BOS_PARTITION_OBSERVATIONS)
        return fail(BOS_ERR_INVALID, "unknown partition");
    if (pb->num_poses <= 0 || pb->num_landmarks < 0 || pb->num_bearings < 0 || pb->num_odometry < 0)
        return fail(BOS_ERR_INVALID, "bad problem sizes");
    if (!pb->pose_xyt ||
        (pb->num_bearings && (!pb->bearing_pose || !pb->bearing_landmark || !pb->bearing_z)) ||
        (pb->num_odometry && (!pb->odom_src || !pb->odom_dst || !pb->odom_z || !pb->odom_omega)))
        return fail(BOS_ERR_INVALID, "null problem array");
    int ndev = 0;
    // host waits spin instead of sleeping (bos_step is synchronous: its wait is on the critical path
    // of every iteration); only possible before the process's first device use, ignored afterwards
    (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
    (void)hipGetLastError();
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(BOS_ERR_DEVICE, "no HIP device visible (the HIP path has no CPU fallback)");
    if (opt.world_size < 1 || opt.rank < 0 || opt.rank >= opt.world_size) return fail(BOS_ERR_INVALID, "bad rank / world_size");

    bos_solver* s = new bos_solver();
    auto bail = [&](int rc) { bos_destroy(s); return rc; };
    s->precision = opt.precision;
    s->tsize = opt.precision == BOS_FP32 ? 4 : 8;
    s->solver_kind = opt.solver;
    s->rank = opt.rank;
    s->world = opt.world_size;
    s->kt = opt.kernel_threshold;
    s->damping = opt.damping;
    s->NP = pb->num_poses; s->NL = pb->num_landmarks; s->Mb = pb->num_bearings; s->Mo = pb->num_odometry;
    if (opt.device >= 0) {
        if (opt.device >= ndev) return bail(fail(BOS_ERR_DEVICE, "device ordinal out of range"));
        if (hipSetDevice(opt.device) != hipSuccess) return bail(fail(BOS_ERR_DEVICE, "hipSetDevice failed"));
        s->device = opt.device;
    } else {
        if (hipGetDevice(&s->device) != hipSuccess) return bail(fail(BOS_ERR_DEVICE, "hipGetDevice failed"));
    }

    // ---- static plan (host)
    bos::ProblemIndex pi;
    pi.NP = s->NP; pi.NL = s->NL; pi.Mb = s->Mb; pi.Mo = s->Mo; pi.fixed = pb->fixed_pose;
    pi.b_pose = pb->bearing_pose; pi.b_lm = pb->bearing_landmark; pi.o_src = pb->odom_src; pi.o_dst = pb->odom_dst;
    pi.b_omega = pb->bearing_omega; pi.o_omega = pb->odom_omega;
    pi.lpp = opt.lanes_per_pose;
    pi.schur_leaf = opt.schur_leaf;
    // multi-rank (world > 1, or a communicator given with world 1: a one-GPU test of the path)
    const bool multi = s->world > 1 || opt.nccl_unique_id;
    s->partition = opt.partition;
    s->obs = multi && opt.partition == BOS_PARTITION_OBSERVATIONS;
    s->sharded = multi && opt.partition == BOS_PARTITION_SUBTREE;
    s->external = multi && !opt.nccl_unique_id;
    std::string err;
    const int fmode = s->solver_kind == BOS_SOLVER_SUPERNODAL    ? bos::kFactorMultifrontal
                      : s->solver_kind == BOS_SOLVER_SCHUR        ? bos::kFactorSchur
                      : s->solver_kind == BOS_SOLVER_ROCSOLVER_RF ? bos::kFactorScalar
                                                                  : bos::kFactorNone;
    // the observations partition runs a range of the one-GPU plan's lanes
    int rc = s->obs ? bos::build_plan(pi, 0, 1, fmode, s->plan, err) : bos::build_plan(pi, s->rank, s->world, fmode, s->plan, err);
    if (rc) return bail(fail(rc, "plan: " + err));
    const bos::Plan& P = s->plan;
    if (s->solver_kind == BOS_SOLVER_DENSE_CHOL && P.n > 40000)
        return bail(fail(BOS_ERR_UNSUPPORTED, "dense solver limited to n <= 40000"));
    s->has_dups = P.blk.has_dups;
    s->has_w = false;
    if (pb->bearing_omega)
        for (int k = 0; k < s->Mb; ++k)
            if (pb->bearing_omega[k] != 1.0) { s->has_w = true; break; }
    s->pl_factored = s->precision == BOS_FP32 && uses_mf(s) && !s->has_w && !s->has_dups;

    // ---- streams / events / libraries
    if (opt.stream) {
        s->stream = (hipStream_t)opt.stream;
    } else {
        if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess)
            return bail(fail(BOS_ERR_DEVICE, "hipStreamCreate failed"));
        s->own_stream = true;
    }
    for (hipEvent_t& e : s->ev)
        if (hipEventCreate(&e) != hipSuccess) return bail(fail(BOS_ERR_DEVICE, "hipEventCreate failed"));
    if (rocblas_create_handle(&s->rb) != rocblas_status_success) return bail(fail(BOS_ERR_SOLVER, "rocblas_create_handle"));
    if (rocblas_set_stream(s->rb, s->stream) != rocblas_status_success) return bail(fail(BOS_ERR_SOLVER, "rocblas_set_stream"));
    if (s->solver_kind == BOS_SOLVER_ROCSOLVER_RF) {
        const rocblas_status st = rocsolver_create_rfinfo(&s->rf, s->rb);
        if (st != rocblas_status_success) {
            size_t fr = 0, tot = 0;
            (void)hipMemGetInfo(&fr, &tot);
            return bail(fail(BOS_ERR_SOLVER, "rocsolver_create_rfinfo: status " + std::to_string((int)st) +
                                                 ", device memory free " + std::to_string(fr >> 20) + " MiB"));
        }
        if (rocsolver_set_rfinfo_mode(s->rf, rocsolver_rfinfo_mode_cholesky) != rocblas_status_success)
            return bail(fail(BOS_ERR_SOLVER, "set_rfinfo_mode"));
    }
    if (multi && !uses_mf(s)) return bail(fail(BOS_ERR_UNSUPPORTED, "sharding needs a multifrontal solver"));
    if (opt.nccl_unique_id) {
        ncclUniqueId id;
        std::memcpy(&id, opt.nccl_unique_id, sizeof(id));
        ncclResult_t r = ncclCommInitRank(&s->comm, s->world, id, s->rank);
        if (r != ncclSuccess) return bail(fail(BOS_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)));
        int count = 0;   // the ranks the communicator actually holds
        r = ncclCommCount(s->comm, &count);
        if (r != ncclSuccess) return bail(fail(BOS_ERR_COMM, std::string("ncclCommCount: ") + ncclGetErrorString(r)));
        if (count != s->world)
            return bail(fail(BOS_ERR_COMM, "communicator holds " + std::to_string(count) + " ranks, world_size " +
                                               std::to_string(s->world)));
    }
    if (s->sharded && (rc = setup_shard(s))) return bail(rc);

    // ---- upload
    const int NP = s->NP, NL = s->NL;
    std::vector<double> pose(pb->pose_xyt, pb->pose_xyt + 3 * (size_t)NP);
    for (int i = 0; i < NP; ++i) pose[3 * i + 2] = bos::normalized_angle<double>(bos::smallest_angle<double>(pose[3 * i + 2]));
    // landmark_xy == NULL: the landmarks are triangulated on the device below (the reference's
    // triangulate_landmarks before the Solver ctor, bearing_only_slam.cpp / slam/triangulation.cpp)
    std::vector<double> lm(2 * (size_t)NL, 0.0);
    if (pb->landmark_xy) lm.assign(pb->landmark_xy, pb->landmark_xy + 2 * (size_t)NL);
    if ((rc = upload(&s->d_pose, pose)) || (rc = upload(&s->d_lm, lm))) return bail(rc);
    const bool f32 = s->precision == BOS_FP32;
    auto alloc_T = [&](void** p, size_t count) -> int {
        if (f32) return dalloc((float**)p, count);
        return dalloc((double**)p, count);
    };
    // the J+H's inputs: the state caches (filled by upload_cache, then by the box-plus) and the
    // static work lists, records and odometry, in one allocation (flush_stage)
    JhStage stage;
    auto stage_Tv = [&](void** p, const std::vector<double>& v) {
        if (f32) stage.add_T<float>(p, v);
        else stage.add_T<double>(p, v);
    };
    stage_Tv(&s->d_pc, std::vector<double>(4 * (size_t)NP, 0.0));
    stage_Tv(&s->d_pth, std::vector<double>((size_t)NP, 0.0));
    stage_Tv(&s->d_lc, std::vector<double>(2 * (size_t)NL, 0.0));

    {
        const bos::BlockLayout& B = P.blk;
        // slot records (padding slots: index 0, z 0). The arrays carry kRecPad extra padding records
        // so the kernel's two-ahead prefetch never leaves them; a prefetched padding record is
        // never evaluated.
        const std::vector<int32_t>& po = B.pose_lanes.obs;
        const std::vector<int32_t>& lo = B.lm_lanes.obs;
        const size_t pad = bos::dev::kRecPad;
        std::vector<double> pbz(po.size() + pad, 0.0), lbz(lo.size() + pad, 0.0), pbw, lbw;
        std::vector<int32_t> pbi(po.size() + pad, 0), lbi(lo.size() + pad, 0);
        for (size_t i = 0; i < po.size(); ++i)
            if (po[i] >= 0) { pbi[i] = pb->bearing_landmark[po[i]]; pbz[i] = pb->bearing_z[po[i]]; }
        for (size_t i = 0; i < lo.size(); ++i)
            if (lo[i] >= 0) { lbi[i] = pb->bearing_pose[lo[i]]; lbz[i] = pb->bearing_z[lo[i]]; }
        {   // runs of duplicate (pose, landmark) observations: every record but the run's last is flagged
            const bos::LaneLists& PLn = B.pose_lanes;
            for (size_t g = 0; g < PLn.cnt.size(); ++g)
                for (int j = 0; j + 1 < PLn.cnt[g]; ++j) {
                    const int64_t sl = PLn.slot((int)g, j), sn = PLn.slot((int)g, j + 1);
                    if (pbi[sl] == pbi[sn]) pbi[sl] |= bos::dev::kRunCont;
                }
        }
        // odometry entries, padded (entry 0 / other pose 0 / no block): the J+H reads a pose's first
        // two entries unconditionally, in bounds even for the last pose without entries
        std::vector<int32_t> po_oth(B.po_ent.size() + pad, 0), po_ent(B.po_ent), po_blk(B.po_blk);
        po_ent.resize(B.po_ent.size() + pad, 0);
        po_blk.resize(B.po_blk.size() + pad, -1);
        for (size_t x = 0; x < B.po_ent.size(); ++x) {
            const int32_t e = B.po_ent[x];
            po_oth[x] = (e & 1) ? pb->odom_src[e >> 1] : pb->odom_dst[e >> 1];
        }
        // chain poses flagged in their first lane's count; interleaved groups: each lane's count with
        // the group's round count (its first lane's) in bits 16-29 (kernels.hip pose_lanes)
        std::vector<int32_t> plc(B.pose_lanes.cnt);
        if (B.interleaved)
            for (size_t g = 0; g < plc.size(); ++g) plc[g] |= B.pose_lanes.cnt[g - g % B.lpp] << 16;
        if (!B.has_dups)
            for (size_t i = 0; i < B.lane_pose.size(); ++i)
                if (B.lane_pose[i] >= 0 && B.po_chain[B.lane_pose[i]]) plc[i * B.lpp] |= bos::dev::kOdoChain;
        stage.add(&s->pw_base, B.pose_lanes.w_base); stage.add(&s->pl_cnt, plc);
        stage.add(&s->pw_stride, B.pose_lanes.w_stride); stage.add(&s->lw_stride, B.lm_lanes.w_stride);
        stage.add(&s->lw_base, B.lm_lanes.w_base);
        {   // a landmark lane's header in one 8-byte record {landmark | count << 20, first pose of the
            // lane's consecutive run or -1} when they fit (one load instead of three; LinParams::ll_hdr)
            const size_t nl = B.lm_lane_lm.size();
            bool fits = nl < ((size_t)1 << 20);
            for (size_t g = 0; g < nl && fits; ++g)
                fits = B.lm_lane_lm[g] >= 0 && B.lm_lane_lm[g] < (1 << 20) && B.lm_lanes.cnt[g] >= 0 && B.lm_lanes.cnt[g] < (1 << 12);
            if (fits && nl > 0) {
                std::vector<int32_t> hdr(2 * nl);
                for (size_t g = 0; g < nl; ++g) {
                    hdr[2 * g] = (int32_t)((uint32_t)B.lm_lane_lm[g] | ((uint32_t)B.lm_lanes.cnt[g] << 20));
                    hdr[2 * g + 1] = B.lm_lane_run.empty() ? -1 : B.lm_lane_run[g];
                }
                stage.add(&s->ll_hdr, hdr);
            } else {
                stage.add(&s->ll_cnt, B.lm_lanes.cnt);
                stage.add(&s->ll_lm, B.lm_lane_lm); stage.add(&s->ll_run, B.lm_lane_run);
            }
        }
        stage.add(&s->po_ptr, B.po_ptr); stage.add(&s->po_ent, po_ent); stage.add(&s->po_oth, po_oth);
        stage.add(&s->po_blk, po_blk); stage.add(&s->pb_idx, pbi); stage_Tv(&s->pb_z, pbz);
        stage.add(&s->lb_idx, lbi); stage_Tv(&s->lb_z, lbz);
        if (s->has_w) {
            pbw.assign(po.size() + pad, 0.0); lbw.assign(lo.size() + pad, 0.0);
            for (size_t i = 0; i < po.size(); ++i) if (po[i] >= 0) pbw[i] = pb->bearing_omega[po[i]];
            for (size_t i = 0; i < lo.size(); ++i) if (lo[i] >= 0) lbw[i] = pb->bearing_omega[lo[i]];
            stage_Tv(&s->pb_w, pbw); stage_Tv(&s->lb_w, lbw);
        }
        static_assert(bos::kJhBlock == bos::dev::kBlock, "J+H block size");
        s->pose_blocks = (int)B.pose_blocks();
        // J+H blocks this rank runs: all of them, or (observations partition) its ranges
        if (s->obs) {
            int64_t pb1 = 0, lb1 = 0;
            bos::observation_lanes(P, s->rank, s->world, s->pose_b0, pb1, s->lm_b0, lb1, nullptr);
            s->n_pose_run = pb1 - s->pose_b0;
            s->n_lm_run = lb1 - s->lm_b0;
        } else {
            s->n_pose_run = s->pose_blocks;
            s->n_lm_run = B.lm_blocks();
        }
        // chi^2 partials: own lanes (a whole number of blocks when sharded), the top lanes on rank 0;
        // observations partition: every block (the others' partials stay 0)
        s->chi_parts = bos::dev::kJhSub *
                       (s->rank == 0 || s->obs ? s->pose_blocks : (int)((int64_t)P.shard.own_pose_lanes * B.lpp / bos::dev::kBlock));
        stage.add(&s->lane_pose, B.lane_pose);
        s->lane_identity = true;
        for (size_t i = 0; i < B.lane_pose.size() && s->lane_identity; ++i) s->lane_identity = B.lane_pose[i] == (int32_t)i;
    }
    for (int k = 0; k < s->Mo; ++k)
        if (pb->odom_src[k] == pb->odom_dst[k]) {
            const double* m = pb->odom_omega + 9 * (size_t)k;
            for (int v = 0; v < 3; ++v) s->loop_z.push_back(pb->odom_z[3 * (size_t)k + v]);
            for (double v : {m[0], m[1], m[2], m[4], m[5], m[8]}) s->loop_om.push_back(v);
        }
    {
        std::vector<int32_t> os(pb->odom_src, pb->odom_src + s->Mo), od(pb->odom_dst, pb->odom_dst + s->Mo);
        // one zero edge of padding (the J+H's unconditional reads of entry 0 when there is none)
        std::vector<double> oz(pb->odom_z, pb->odom_z + 3 * (size_t)s->Mo), om(6 * (size_t)s->Mo + 6, 0.0);
        oz.resize(3 * (size_t)s->Mo + 3, 0.0);
        bool same = true;   // every edge's information equal (bit for bit): one row, om_stride 0
        for (int k = 0; k < s->Mo; ++k) {
            const double* m = pb->odom_omega + 9 * (size_t)k;
            const double u[6] = {m[0], m[1], m[2], m[4], m[5], m[8]};
            for (int q = 0; q < 6; ++q) {
                om[6 * (size_t)k + q] = u[q];
                same = same && std::memcmp(&om[6 * (size_t)k + q], &om[q], sizeof(double)) == 0;
            }
        }
        s->om_stride = 6;
        if (same && s->Mo > 0) {   // the J+H then reads 24 (fp32) / 48 bytes of information in all, not per edge
            om.resize(12);
            s->om_stride = 0;
        }
        stage.add(&s->o_src, os); stage.add(&s->o_dst, od); stage_Tv(&s->o_z, oz); stage_Tv(&s->o_om, om);
    }
    if ((rc = flush_stage(s, stage))) return bail(rc);
    // permuted dof -> reference dof
    s->ref_dof.assign(P.n + 3, 0);
    for (int u = 0; u < NP + NL; ++u) {
        const int sz = u < NP ? 3 : 2;
        const int ref0 = u < NP ? 3 * u : 3 * NP + 2 * (u - NP);
        for (int d = 0; d < sz; ++d) s->ref_dof[P.node_dof[u] + d] = ref0 + d;
    }
    const int64_t nval = std::max<int64_t>(P.blk.size, 1), nb = 3 * (int64_t)NP + 2 * (int64_t)NL;
    if ((rc = upload(&s->node_dof, P.node_dof))) return bail(rc);
    if (s->obs) {
        // [block array (even length) | b] in one buffer, all-reduced in one call into d_sys; the
        // values outside this rank's lanes stay 0
        const int64_t nv2 = (nval + 1) & ~(int64_t)1;
        s->vb_count = nv2 + nb;
        if ((rc = alloc_T(&s->d_val, s->vb_count)) || (rc = alloc_T(&s->d_sys, s->vb_count))) return bail(rc);
        s->d_b = (char*)s->d_val + nv2 * s->tsize;
        s->sys_val = s->d_sys;
        s->sys_b = (char*)s->d_sys + nv2 * s->tsize;
        HIP_TRY(hipMemset(s->d_val, 0, s->vb_count * s->tsize));
        HIP_TRY(hipMemset(s->d_sys, 0, s->vb_count * s->tsize));
        s->ex1_count = bos::kExHeader + (s->external ? s->vb_count : 0);
        if ((rc = dalloc(&s->ex1_send, (size_t)s->ex1_count)) || (rc = dalloc(&s->ex1_recv, (size_t)s->ex1_count))) return bail(rc);
        HIP_TRY(hipMemset(s->ex1_send, 0, s->ex1_count * sizeof(double)));
        HIP_TRY(hipMemset(s->ex1_recv, 0, s->ex1_count * sizeof(double)));
        s->solve_stamp = 4;
    } else {
        if ((rc = alloc_T(&s->d_val, nval)) || (rc = alloc_T(&s->d_b, nb))) return bail(rc);
        s->sys_val = s->d_val;
        s->sys_b = s->d_b;
        HIP_TRY(hipMemset(s->d_val, 0, nval * s->tsize));
        HIP_TRY(hipMemset(s->d_b, 0, nb * s->tsize));
    }
    if ((rc = dalloc(&s->d_rhs, std::max<int64_t>(P.n, 1)))) return bail(rc);
    if (f32 && uses_mf(s) && (rc = dalloc(&s->d_val64, nval))) return bail(rc);
    {
        std::vector<int32_t> er(s->ref_dof.begin(), s->ref_dof.begin() + P.n);
        if ((rc = upload(&s->elim_ref, er))) return bail(rc);
    }
    if (!uses_mf(s) &&
        ((rc = upload(&s->d_rowptr, P.rowptr)) || (rc = upload(&s->d_colind, P.colind)) ||
         (rc = upload(&s->csr_src, P.blk.csr_src)) || (rc = dalloc(&s->d_csr64, std::max<int64_t>(P.nnzA(), 1)))))
        return bail(rc);
    if (uses_mf(s)) {
        std::string merr;
        if (bos::dev::mf_create(P.mf, s->sharded ? P.shard.sn_owner.data() : nullptr, s->rank, &s->mf, merr))
            return bail(fail(BOS_ERR_DEVICE, merr));
        s->fold32 = s->pl_factored && bos::mf_fold_reads_fp32(P);
        if (s->fold32) bos::dev::mf_set_fold_source(s->mf, (const float*)s->sys_val, P.blk.off_pl);
    } else if (s->solver_kind == BOS_SOLVER_ROCSOLVER_RF) {
        std::vector<int32_t> piv(P.n);
        for (int64_t i = 0; i < P.n; ++i) piv[i] = (int32_t)i;   // ordering already applied in the layout
        if ((rc = upload(&s->d_Lptr, P.Lptr)) || (rc = upload(&s->d_Lind, P.Lind)) || (rc = upload(&s->d_pivQ, piv)) ||
            (rc = dalloc(&s->d_Lval, std::max<int64_t>(P.nnzL(), 1))))
            return bail(rc);
        HIP_TRY(hipMemset(s->d_Lval, 0, std::max<int64_t>(P.nnzL(), 1) * sizeof(double)));
    } else {
        if ((rc = dalloc(&s->d_dense, (size_t)P.n * P.n))) return bail(rc);
    }
    const int nt = std::max(1, s->pose_blocks * bos::dev::kJhSub);   // chi^2 partials: one per pose workgroup
    if ((rc = dalloc(&s->d_info, 1)) || (rc = dalloc(&s->d_chi_part, nt)) || (rc = dalloc(&s->d_nrob_part, nt)) ||
        (rc = dalloc(&s->d_status, 1)) ||
        (rc = dalloc(&s->d_maxpart, (size_t)std::max(1, (s->NP + s->NL + bos::dev::kUpdateBlock - 1) / bos::dev::kUpdateBlock))))
        return bail(rc);
    HIP_TRY(hipMemset(s->d_chi_part, 0, nt * sizeof(double)));
    HIP_TRY(hipMemset(s->d_nrob_part, 0, nt * sizeof(int32_t)));
    HIP_TRY(hipMemset(s->d_info, 0, sizeof(int32_t)));
    HIP_TRY(hipMemset(s->d_status, 0, sizeof(bos::dev::StepStatus)));   // the abort flag is sticky
    if (hipHostMalloc((void**)&s->h_status, sizeof(bos::dev::StepStatus), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&s->m_status, s->h_status, 0) != hipSuccess)
        return bail(fail(BOS_ERR_DEVICE, "host-mapped status allocation failed"));
    std::memset(s->h_status, 0, sizeof(bos::dev::StepStatus));
    {   // triangulation inputs (kept for bos_triangulate)
        std::vector<int32_t> tptr(NL + 1, 0), tobs(s->Mb), tpose(pb->bearing_pose, pb->bearing_pose + s->Mb);
        for (int k = 0; k < s->Mb; ++k) ++tptr[pb->bearing_landmark[k] + 1];
        for (int l = 0; l < NL; ++l) tptr[l + 1] += tptr[l];
        std::vector<int32_t> w(tptr.begin(), tptr.end() - 1);
        for (int k = 0; k < s->Mb; ++k) tobs[w[pb->bearing_landmark[k]]++] = k;
        std::vector<double> tz(pb->bearing_z, pb->bearing_z + s->Mb);
        if ((rc = upload(&s->tri_ptr, tptr)) || (rc = upload(&s->tri_obs, tobs)) || (rc = upload(&s->tri_pose, tpose)) ||
            (rc = upload(&s->tri_z, tz)) || (rc = dalloc(&s->tri_scr, 3 * (size_t)std::max(1, s->Mb))))
            return bail(rc);
    }
    if (!pb->landmark_xy && NL) {
        if ((rc = enqueue_triangulate(s))) return bail(rc);
        HIP_TRY(hipStreamSynchronize(s->stream));   // upload_cache reads the landmarks back
    }
    if ((rc = upload_cache(s))) return bail(rc);
    HIP_TRY(hipStreamSynchronize(s->stream));
    *out = s;
    return BOS_OK;
}

int bos_set_kernel_threshold(bos_solver* s, double kt) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    if (kt != s->kt) drop_graph(s);
    s->kt = kt;
    return BOS_OK;
}

int bos_set_damping_factor(bos_solver* s, double df) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    if (df != s->damping) drop_graph(s);
    s->damping = df;
    return BOS_OK;
}

int bos_step(bos_solver* s, bos_step_stats* st) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    HIP_TRY(hipSetDevice(s->device));
    return do_step(s, st, true);
}

int bos_step_n(bos_solver* s, int n, bos_step_stats* last) {
    if (!s || n < 0) return fail(BOS_ERR_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(s->device));
    for (int i = 0; i < n; ++i) {
        int rc = do_step(s, last, i + 1 == n);
        if (rc) return rc;
    }
    return BOS_OK;
}

int bos_linearize_async(bos_solver* s) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    return enqueue_linearize(s);
}

int bos_debug_linearize_timeline(bos_solver* s, int64_t capacity, uint64_t* stamps, int64_t* n_waves, int32_t flush_caches) {
    if (!s || !n_waves) return fail(BOS_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(s->device));
    const bos::Plan& P = s->plan;
    const int64_t grid = s->pose_blocks + ((int64_t)P.blk.lm_lane_lm.size() + bos::dev::kBlock - 1) / bos::dev::kBlock;
    const int64_t waves = grid * (bos::dev::kBlock / 64);
    *n_waves = waves;
    if (!stamps || capacity < waves) return BOS_OK;
    unsigned long long* d = nullptr;
    int rc = dalloc(&d, 8 * (size_t)waves);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(d, 0, 8 * (size_t)waves * sizeof(unsigned long long), s->stream));
    if (flush_caches && (rc = scrub_caches(s))) { (void)hipFree(d); return rc; }
    hipError_t e;
    const int lpp = P.blk.lpp;
    if (s->precision == BOS_FP32) {
        bos::dev::LinParams<float> p = lin_params<float>(s);
        p.diag_stamps = d;
        e = bos::dev::launch_linearize<float>(p, lpp, s->has_w, s->has_dups, s->stream);
    } else {
        bos::dev::LinParams<double> p = lin_params<double>(s);
        p.diag_stamps = d;
        e = bos::dev::launch_linearize<double>(p, lpp, s->has_w, s->has_dups, s->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e == hipSuccess) e = hipMemcpy(stamps, d, 8 * (size_t)waves * sizeof(uint64_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(BOS_ERR_DEVICE, std::string("timeline: ") + hipGetErrorString(e));
    return BOS_OK;
}

int bos_time_linearize(bos_solver* s, int32_t n, int32_t flush_caches, double* ms_per_build) {
    if (!s || n <= 0 || !ms_per_build) return fail(BOS_ERR_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(s->device));
    int rc;
    if (!flush_caches) {   // back to back: the block array and lists stay in L2 / Infinity Cache
        HIP_TRY(hipEventRecord(s->ev[0], s->stream));
        for (int i = 0; i < n; ++i)
            if ((rc = enqueue_linearize(s))) return rc;
        HIP_TRY(hipEventRecord(s->ev[1], s->stream));
        HIP_TRY(hipEventSynchronize(s->ev[1]));
        *ms_per_build = elapsed(s->ev[0], s->ev[1]) / n;
        return BOS_OK;
    }
    // cold: before every build, 512 MiB are read (scrub_caches) so the build's inputs come from HBM,
    // as inside a GN step where the solver streams its factor between two builds; each build is
    // bracketed by its own events (their cost included: conservative)
    double total = 0.0;
    for (int i = 0; i < n; ++i) {
        if ((rc = scrub_caches(s))) return rc;
        HIP_TRY(hipEventRecord(s->ev[0], s->stream));
        if ((rc = enqueue_linearize(s))) return rc;
        HIP_TRY(hipEventRecord(s->ev[1], s->stream));
        HIP_TRY(hipEventSynchronize(s->ev[1]));
        total += elapsed(s->ev[0], s->ev[1]);
    }
    *ms_per_build = total / n;
    return BOS_OK;
}

int bos_time_triangulate(bos_solver* s, int32_t n, double* ms_per_call) {
    if (!s || n <= 0 || !ms_per_call) return fail(BOS_ERR_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(s->device));
    int rc;
    HIP_TRY(hipEventRecord(s->ev[0], s->stream));
    for (int i = 0; i < n; ++i)
        if ((rc = enqueue_triangulate(s))) return rc;
    HIP_TRY(hipEventRecord(s->ev[1], s->stream));
    HIP_TRY(hipEventSynchronize(s->ev[1]));
    *ms_per_call = elapsed(s->ev[0], s->ev[1]) / n;
    s->have_dx = false;
    return BOS_OK;
}

int bos_time_steps(bos_solver* s, int32_t n, double* ms_per_step) {
    if (!s || n <= 0 || !ms_per_step) return fail(BOS_ERR_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(s->device));
    bos_step_stats st;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {   // exactly bos_step: launch, wait, status read and checked
        const int rc = do_step(s, &st, true);
        if (rc) return rc;
    }
    const auto t1 = std::chrono::steady_clock::now();
    *ms_per_step = std::chrono::duration<double, std::milli>(t1 - t0).count() / n;
    return BOS_OK;
}

int bos_step_phase(bos_solver* s, int32_t phase, bos_step_stats* st) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    if (s->obs) {   // observations partition: phases 0 and 1, the all-reduce between them
        if (phase != s->phase) return fail(BOS_ERR_INVALID, "bos_step_phase: phases run 0, 1 in order");
        HIP_TRY(hipSetDevice(s->device));
        const int rc = obs_phase(s, phase);
        if (rc) { s->phase = 0; return rc; }
        s->phase = (phase + 1) % 2;
        if (phase == 0) return BOS_OK;
        ++s->seq_pending;
        s->have_dx = true;
        return finish_step(s, st);
    }
    if (!s->sharded) return fail(BOS_ERR_INVALID, "bos_step_phase needs a sharded handle (world_size > 1)");
    if (s->p2p) return fail(BOS_ERR_INVALID, "bos_step_phase: the handle exchanges directly (bos_exchange_p2p_connect); use bos_step");
    if (phase != s->phase) return fail(BOS_ERR_INVALID, "bos_step_phase: phases run 0, 1, 2 in order");
    HIP_TRY(hipSetDevice(s->device));
    int rc = phase == 0 ? shard_phase0(s) : phase == 1 ? shard_phase1(s) : shard_phase2(s);
    if (rc) { s->phase = 0; return rc; }
    s->phase = (phase + 1) % 3;
    if (phase < 2) return BOS_OK;
    ++s->seq_pending;   // phase 2's status launch bumps the device counter
    s->have_dx = true;
    return finish_step(s, st);
}

int bos_exchange_size(const bos_solver* s, int32_t which, int64_t* doubles_per_rank) {
    if (!s || !doubles_per_rank || (which != 1 && which != 2)) return fail(BOS_ERR_INVALID, "bad argument");
    if (!s->sharded && !(s->obs && which == 1)) return fail(BOS_ERR_INVALID, "not a sharded handle / no such exchange");
    *doubles_per_rank = which == 1 ? s->ex1_count : s->ex2_count;
    return BOS_OK;
}

int bos_exchange_download(bos_solver* s, int32_t which, double* send) {
    if (!s || !send || (which != 1 && which != 2)) return fail(BOS_ERR_INVALID, "bad argument");
    if (s->p2p) return fail(BOS_ERR_INVALID, "bos_exchange_download: the handle exchanges directly (bos_exchange_p2p_connect)");
    if (!s->sharded && !(s->obs && which == 1)) return fail(BOS_ERR_INVALID, "not a sharded handle / no such exchange");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    const int64_t c = which == 1 ? s->ex1_count : s->ex2_count;
    HIP_TRY(hipMemcpy(send, which == 1 ? s->ex1_send : s->ex2_send, c * sizeof(double), hipMemcpyDeviceToHost));
    return BOS_OK;
}

int bos_exchange_upload(bos_solver* s, int32_t which, const double* recv_all) {
    if (!s || !recv_all || (which != 1 && which != 2)) return fail(BOS_ERR_INVALID, "bad argument");
    if (s->p2p) return fail(BOS_ERR_INVALID, "bos_exchange_upload: the handle exchanges directly (bos_exchange_p2p_connect)");
    if (!s->sharded && !(s->obs && which == 1)) return fail(BOS_ERR_INVALID, "not a sharded handle / no such exchange");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    // subtree partition: every rank's buffer (all-gather); observations partition: their sum
    const int64_t c = s->obs ? s->ex1_count : (which == 1 ? s->ex1_count : s->ex2_count) * s->world;
    HIP_TRY(hipMemcpy(which == 1 ? s->ex1_recv : s->ex2_recv, recv_all, c * sizeof(double), hipMemcpyHostToDevice));
    return BOS_OK;
}

int bos_set_exchange_timeout(bos_solver* s, double seconds) {
    if (!s || !(seconds > 0.0) || seconds > 3600.0) return fail(BOS_ERR_INVALID, "bad argument");
    const uint64_t t = (uint64_t)(seconds * 1e8);   // 100 MHz realtime clock
    if (t != s->ex_timeout_ticks) drop_graph(s);     // a launch argument of the captured step
    s->ex_timeout_ticks = t;
    return BOS_OK;
}

int bos_exchange_p2p_handle(bos_solver* s, void* handle) {
    if (!s || !handle) return fail(BOS_ERR_INVALID, "null argument");
    if (!s->sharded) return fail(BOS_ERR_UNSUPPORTED, "direct exchange: subtree-sharded handles only");
    if (!s->mailbox_uncached) return fail(BOS_ERR_UNSUPPORTED, "direct exchange: no uncached device memory for the mailbox");
    HIP_TRY(hipSetDevice(s->device));
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, s->mailbox);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(BOS_ERR_UNSUPPORTED, std::string("direct exchange: hipIpcGetMemHandle: ") + hipGetErrorString(e));
    }
    static_assert(sizeof(h) == BOS_P2P_HANDLE_BYTES, "IPC handle size");
    std::memcpy(handle, &h, sizeof(h));
    return BOS_OK;
}

int bos_exchange_p2p_connect(bos_solver* s, const void* handles) {
    if (!s || !handles) return fail(BOS_ERR_INVALID, "null argument");
    if (!s->sharded || !s->mailbox_uncached) return fail(BOS_ERR_UNSUPPORTED, "direct exchange: not available on this handle");
    if (s->p2p) return fail(BOS_ERR_INVALID, "direct exchange: already connected");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    // the peers' mailboxes are written by this device's kernels: every other visible device must be
    // reachable (xGMI), or the caller keeps the RCCL exchange
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    for (int d = 0; d < ndev; ++d) {
        int ok = 0;
        if (d != s->device && (hipDeviceCanAccessPeer(&ok, s->device, d) != hipSuccess || !ok)) {
            (void)hipGetLastError();
            return fail(BOS_ERR_UNSUPPORTED, "direct exchange: device " + std::to_string(s->device) +
                                                 " has no peer access to device " + std::to_string(d));
        }
    }
    std::vector<double*> peers(s->world, nullptr);
    for (int q = 0; q < s->world; ++q) {
        if (q == s->rank) { peers[q] = reinterpret_cast<double*>(s->mailbox); continue; }
        hipIpcMemHandle_t h;
        std::memcpy(&h, static_cast<const char*>(handles) + (size_t)q * BOS_P2P_HANDLE_BYTES, sizeof(h));
        void* p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess || !p) {
            (void)hipGetLastError();
            for (void* m : s->peer_maps) (void)hipIpcCloseMemHandle(m);
            s->peer_maps.clear();
            return fail(BOS_ERR_UNSUPPORTED, std::string("direct exchange: hipIpcOpenMemHandle (rank ") + std::to_string(q) +
                                                 "): " + hipGetErrorString(e));
        }
        s->peer_maps.push_back(p);
        peers[q] = reinterpret_cast<double*>(p);
    }
    int rc;
    if ((rc = upload(&s->d_peers, peers))) return rc;
    drop_graph(s);   // the next step captures the iteration with the direct exchange
    s->rccl_capture_failed = false;
    s->p2p = true;
    return BOS_OK;
}

int bos_node_owner(const bos_solver* s, int32_t* owner) {
    if (!s || !owner) return fail(BOS_ERR_INVALID, "null argument");
    if (s->obs) return fail(BOS_ERR_UNSUPPORTED, "observations partition: every rank holds every node");
    const std::vector<int32_t>& o = s->plan.shard.node_owner;
    if (o.empty()) return fail(BOS_ERR_UNSUPPORTED, "no shard (not a multifrontal solver)");
    std::copy(o.begin(), o.end(), owner);
    return BOS_OK;
}

int bos_debug_inject_stall(bos_solver* s) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    if (!uses_mf(s)) return fail(BOS_ERR_UNSUPPORTED, "no dataflow launch in this solver");
    HIP_TRY(hipSetDevice(s->device));
    const hipError_t e = bos::dev::mf_debug_skip_next_front(s->mf, s->stream);
    if (e == hipErrorInvalidValue)
        return fail(BOS_ERR_UNSUPPORTED, "no dataflow launch in this plan whose first front another front of it waits for");
    HIP_TRY(e);
    return BOS_OK;
}

int bos_debug_solver_stamps(bos_solver* s, int64_t capacity, uint64_t* stamps, int32_t* meta) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    if (!uses_mf(s) || s->sharded || s->obs) return fail(BOS_ERR_UNSUPPORTED, "one-GPU multifrontal handles only");
    const bos::Multifrontal& F = s->plan.mf;
    const int64_t need = 16 * (int64_t)F.nsuper;
    if (!stamps || !meta || capacity < need) return fail(BOS_ERR_INVALID, "stamps: capacity 16 * supernodes");
    HIP_TRY(hipSetDevice(s->device));
    unsigned long long* d = nullptr;
    int rc = dalloc(&d, (size_t)need);
    if (rc) return rc;
    HIP_TRY(hipMemset(d, 0, need * sizeof(unsigned long long)));
    drop_graph(s);
    const bool gf = s->graph_failed;
    s->graph_failed = true;   // one eager step with the stamps
    bos::dev::mf_debug_set_stamps(s->mf, d);
    rc = do_step(s, nullptr, true);
    if (!rc && hipStreamSynchronize(s->stream) != hipSuccess) rc = fail(BOS_ERR_DEVICE, "stamps step");
    bos::dev::mf_debug_set_stamps(s->mf, nullptr);
    s->graph_failed = gf;
    if (!rc && hipMemcpy(stamps, d, need * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail(BOS_ERR_DEVICE, "stamps copy");
    (void)hipFree(d);
    if (rc) return rc;
    std::vector<int32_t> lev(F.nsuper, -1);
    for (int l = 0; l < F.nlevels; ++l)
        for (int q = F.level_ptr[l]; q < F.level_ptr[l + 1]; ++q) lev[F.level[q]] = l;
    for (int x = 0; x < F.nsuper; ++x) {
        meta[4 * x] = lev[x];
        meta[4 * x + 1] = F.k[x];
        meta[4 * x + 2] = F.r[x];
        meta[4 * x + 3] = F.fold_cnt.empty() ? 0 : F.fold_cnt[x];
    }
    return BOS_OK;
}

int bos_debug_set_step_graph(bos_solver* s, int32_t enable) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    drop_graph(s);
    s->graph_failed = !enable;
    return BOS_OK;
}

int bos_triangulate(bos_solver* s) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    HIP_TRY(hipSetDevice(s->device));
    int rc = enqueue_triangulate(s);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->have_dx = false;
    return BOS_OK;
}

int bos_triangulate_async(bos_solver* s) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    return enqueue_triangulate(s);
}

int bos_synchronize(bos_solver* s) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    HIP_TRY(hipStreamSynchronize(s->stream));
    return BOS_OK;
}

int bos_linearize(bos_solver* s, bos_step_stats* st) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    if (s->sharded || s->obs) return fail(BOS_ERR_UNSUPPORTED, "bos_linearize on a sharded handle (a rank builds part of H)");
    HIP_TRY(hipSetDevice(s->device));
    int rc;
    HIP_TRY(hipEventRecord(s->ev[0], s->stream));
    if ((rc = enqueue_linearize(s))) return rc;
    HIP_TRY(hipEventRecord(s->ev[1], s->stream));
    HIP_TRY(hipEventRecord(s->ev[2], s->stream));
    if ((rc = enqueue_stats(s, false))) return rc;
    if ((rc = read_stats(s, st, nullptr, true))) return rc;   // the events are read next
    if (st) {
        st->t_linearize_ms = elapsed(s->ev[0], s->ev[1]);
        st->t_exchange_ms = elapsed(s->ev[1], s->ev[2]);
        st->t_solve_ms = st->t_update_ms = 0.0;
    }
    return BOS_OK;
}

int bos_system_info_get(const bos_solver* s, bos_system_info* info) {
    if (!s || !info) return fail(BOS_ERR_INVALID, "null argument");
    std::memset(info, 0, sizeof(*info));
    const bos::Plan& P = s->plan;
    info->n = P.n;
    info->nnz_lower = P.nnzA();
    info->nnz_factor = uses_mf(s) ? P.mf.L_size : P.nnzL();
    const int64_t Mb = s->Mb, Mo = s->Mo, NP = s->NP, NL = s->NL;
    // compulsory reads of inputs + state, one write of every output block
    info->algorithmic_bytes = s->precision == BOS_FP32 ? 36 * Mb + 80 * Mo + 60 * NP + 32 * NL
                                                       : 64 * Mb + 152 * Mo + 120 * NP + 64 * NL;
    info->pl_factored = s->pl_factored ? 1 : 0;
    info->fold_fp32 = s->fold32 ? 1 : 0;
    info->layout_bytes = info->algorithmic_bytes - (s->pl_factored ? 12 * Mb : 0);
    info->num_block_values = P.blk.size;
    info->lanes_per_pose = P.blk.lpp;
    info->pose_lane_groups = (int32_t)P.blk.lane_pose.size();
    info->landmark_lanes = (int32_t)P.blk.lm_lane_lm.size();
    info->own_fronts = P.shard.n_own_fronts;
    info->top_fronts = P.shard.n_top_fronts;
    info->partition = s->partition;
    info->comm_ranks = 0;
    if (s->comm) {
        int count = 0;
        NC_TRY(ncclCommCount(s->comm, &count));
        info->comm_ranks = count;
    }
    return BOS_OK;
}

int bos_export_system(const bos_solver* s, int64_t capacity, int32_t* rows, int32_t* cols, double* vals, double* b) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    if (s->sharded) return fail(BOS_ERR_UNSUPPORTED, "bos_export_system on a subtree-sharded handle (a rank holds part of H)");
    const bos::Plan& P = s->plan;
    const int64_t nnz = P.nnzA();
    if ((rows || cols || vals) && capacity < nnz) return fail(BOS_ERR_INVALID, "export capacity < nnz_lower");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (vals) {
        const int64_t nv = P.blk.size;
        std::vector<double> v(nv);
        if (s->precision == BOS_FP32) {
            std::vector<float> f(nv);
            if (nv) HIP_TRY(hipMemcpy(f.data(), s->sys_val, nv * sizeof(float), hipMemcpyDeviceToHost));
            if (s->pl_factored) bos::dev::expand_factored_host(f.data(), v.data(), nv, P.blk.off_pl, P.blk.pose_lanes.slots());
            else for (int64_t i = 0; i < nv; ++i) v[i] = f[i];
        } else if (nv) {
            HIP_TRY(hipMemcpy(v.data(), s->sys_val, nv * sizeof(double), hipMemcpyDeviceToHost));
        }
        for (int64_t e = 0; e < nnz; ++e) vals[e] = v[P.blk.csr_src[e]];
    }
    if (rows || cols) {
        for (int64_t r = 0; r < P.n; ++r)
            for (int64_t e = P.rowptr[r]; e < P.rowptr[r + 1]; ++e) {
                const int32_t a = s->ref_dof[r], c = s->ref_dof[P.colind[e]];
                if (rows) rows[e] = std::max(a, c);
                if (cols) cols[e] = std::min(a, c);
            }
    }
    if (b) {   // b is kept in the reference numbering; the fixed pose's entries are not part of H_nf
        const int64_t nb = 3 * (int64_t)s->NP + 2 * (int64_t)s->NL;
        if (s->precision == BOS_FP32) {
            std::vector<float> v(nb);
            HIP_TRY(hipMemcpy(v.data(), s->sys_b, nb * sizeof(float), hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < nb; ++i) b[i] = v[i];
        } else {
            HIP_TRY(hipMemcpy(b, s->sys_b, nb * sizeof(double), hipMemcpyDeviceToHost));
        }
        for (int d = 0; d < 3; ++d) b[3 * (int64_t)P.fixed + d] = 0.0;
    }
    return BOS_OK;
}

int bos_get_state(const bos_solver* s, double* pose_xyt, double* landmark_xy) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (pose_xyt) HIP_TRY(hipMemcpy(pose_xyt, s->d_pose, 3 * (size_t)s->NP * sizeof(double), hipMemcpyDeviceToHost));
    if (landmark_xy && s->NL)
        HIP_TRY(hipMemcpy(landmark_xy, s->d_lm, 2 * (size_t)s->NL * sizeof(double), hipMemcpyDeviceToHost));
    return BOS_OK;
}

int bos_set_state(bos_solver* s, const double* pose_xyt, const double* landmark_xy) {
    if (!s) return fail(BOS_ERR_INVALID, "null handle");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (pose_xyt) {
        std::vector<double> p(pose_xyt, pose_xyt + 3 * (size_t)s->NP);
        for (int i = 0; i < s->NP; ++i) p[3 * i + 2] = bos::normalized_angle<double>(bos::smallest_angle<double>(p[3 * i + 2]));
        HIP_TRY(hipMemcpy(s->d_pose, p.data(), p.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    if (landmark_xy && s->NL)
        HIP_TRY(hipMemcpy(s->d_lm, landmark_xy, 2 * (size_t)s->NL * sizeof(double), hipMemcpyHostToDevice));
    int rc = upload_cache(s);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
    return BOS_OK;
}

int bos_last_step_stamps(const bos_solver* s, uint64_t stamps[8]) {
    if (!s || !stamps) return fail(BOS_ERR_INVALID, "null argument");
    bos::dev::StepStatus h;
    std::memcpy(&h, (const void*)s->h_status, sizeof(h));   // the last step's summary (host-mapped)
    for (int i = 0; i < 8; ++i) stamps[i] = h.stamp[i];
    return BOS_OK;
}

int bos_get_last_dx(const bos_solver* s, double* dx) {
    if (!s || !dx) return fail(BOS_ERR_INVALID, "null argument");
    if (s->sharded) return fail(BOS_ERR_UNSUPPORTED, "bos_get_last_dx on a subtree-sharded handle (a rank holds part of x)");
    if (!s->have_dx) return fail(BOS_ERR_INVALID, "no step has been run");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    const int64_t n = s->plan.n;
    std::vector<double> x(n);
    if (n) HIP_TRY(hipMemcpy(x.data(), s->d_rhs, n * sizeof(double), hipMemcpyDeviceToHost));
    const int64_t N = n + 3;
    for (int64_t i = 0; i < N; ++i) dx[i] = 0.0;
    for (int64_t i = 0; i < n; ++i) dx[s->ref_dof[i]] = -x[i];
    return BOS_OK;
}

}  // extern "C"
