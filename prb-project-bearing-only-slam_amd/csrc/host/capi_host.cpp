// Host-side C ABI (include/bos_host.h): datasets (g2o / synthetic) and plan inspection.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/bos_host.h"
#include "g2o_utils.hpp"
#include "host_mf.hpp"
#include "plan.hpp"
#include "synthetic.hpp"
#include "triangulation.hpp"

#include "error.hpp"

namespace {
int hfail(int code, const std::string& m) { return bos::set_error(code, m); }
}  // namespace

struct bos_dataset {
    proj02::State state;
    proj02::BearingObservationVector bearings;
    proj02::OdometryObservationVector odometry;
    int fixed_pose_id = -1;
    float bound = 0;
    // SoA problem view
    std::vector<double> pose_xyt, lm_xy, b_z, o_z, o_om;
    std::vector<int32_t> b_pose, b_lm, o_src, o_dst, pose_ids, lm_ids;
    int32_t fixed_stix = 0;
    bool has_gt = false;
    std::vector<double> gt_pose, gt_lm;

    int finalize() {
        const proj02::NEPoseVector& P = state.poses_vec();
        const proj02::LMPosVector& L = state.landmarks_vec();
        pose_xyt.resize(3 * P.size());
        for (size_t i = 0; i < P.size(); ++i) {
            pose_xyt[3 * i] = P[i].x; pose_xyt[3 * i + 1] = P[i].y; pose_xyt[3 * i + 2] = P[i].theta;
        }
        lm_xy.resize(2 * L.size());
        for (size_t j = 0; j < L.size(); ++j) { lm_xy[2 * j] = L[j].x; lm_xy[2 * j + 1] = L[j].y; }
        pose_ids.assign(state.pose_ids().begin(), state.pose_ids().end());
        lm_ids.assign(state.landmark_ids().begin(), state.landmark_ids().end());
        // id -> stix as flat tables when the ids are dense enough (else the State's maps); a repeated
        // id maps to its last stix, as the State's map does (state.cpp:23)
        auto flat = [](const std::vector<int32_t>& ids, std::vector<int32_t>& tab, int32_t& lo) {
            tab.clear();
            lo = 0;
            if (ids.empty()) return false;
            const auto mm = std::minmax_element(ids.begin(), ids.end());
            lo = *mm.first;
            const int64_t span = (int64_t)*mm.second - lo + 1;
            if (span > 4 * (int64_t)ids.size() + 1024) return false;
            tab.assign((size_t)span, -1);
            for (size_t i = 0; i < ids.size(); ++i) tab[(size_t)(ids[i] - lo)] = (int32_t)i;
            return true;
        };
        std::vector<int32_t> ptab, ltab;
        int32_t plo = 0, llo = 0;
        const bool pf = flat(pose_ids, ptab, plo), lf = flat(lm_ids, ltab, llo);
        auto pstix = [&](int id) -> int32_t {
            if (!pf) return state.pose_stix(id);
            const int64_t q = (int64_t)id - plo;
            if (q < 0 || q >= (int64_t)ptab.size() || ptab[(size_t)q] < 0) throw std::out_of_range("pose id");
            return ptab[(size_t)q];
        };
        auto lstix = [&](int id) -> int32_t {
            if (!lf) return state.landmark_stix(id);
            const int64_t q = (int64_t)id - llo;
            if (q < 0 || q >= (int64_t)ltab.size() || ltab[(size_t)q] < 0) throw std::out_of_range("landmark id");
            return ltab[(size_t)q];
        };
        try {
            b_pose.resize(bearings.size()); b_lm.resize(bearings.size()); b_z.resize(bearings.size());
            for (size_t k = 0; k < bearings.size(); ++k) {
                b_pose[k] = pstix(bearings[k].get_pose_id());
                b_lm[k] = lstix(bearings[k].get_lm_id());
                b_z[k] = bearings[k].get_bearing_angle();
            }
            o_src.resize(odometry.size()); o_dst.resize(odometry.size());
            o_z.resize(3 * odometry.size()); o_om.resize(9 * odometry.size());
            for (size_t k = 0; k < odometry.size(); ++k) {
                o_src[k] = pstix(odometry[k].get_source_id());
                o_dst[k] = pstix(odometry[k].get_dest_id());
                const proj02::EPose z = odometry[k].get_transformation();
                o_z[3 * k] = z.x; o_z[3 * k + 1] = z.y; o_z[3 * k + 2] = z.z;
                const proj02::Mat3 m = odometry[k].get_omega();
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) o_om[9 * k + 3 * r + c] = m(r, c);
            }
            fixed_stix = pstix(fixed_pose_id);
        } catch (const std::out_of_range&) {
            return hfail(BOS_ERR_INVALID, "an observation or FIX references an unknown id");
        }
        return BOS_OK;
    }
};

namespace {

bos::ProblemIndex index_of(const bos_problem* pb) {
    bos::ProblemIndex pi;
    pi.NP = pb->num_poses; pi.NL = pb->num_landmarks; pi.Mb = pb->num_bearings; pi.Mo = pb->num_odometry;
    pi.fixed = pb->fixed_pose;
    pi.b_pose = pb->bearing_pose; pi.b_lm = pb->bearing_landmark; pi.o_src = pb->odom_src; pi.o_dst = pb->odom_dst;
    pi.b_omega = pb->bearing_omega; pi.o_omega = pb->odom_omega;
    return pi;
}

}  // namespace

extern "C" {

int bos_dataset_load_g2o(const char* path, int triangulate, int verbose, bos_dataset** out) {
    if (!path || !out) return hfail(BOS_ERR_INVALID, "null argument");
    *out = nullptr;
    bos_dataset* d = new bos_dataset();
    const int rc = proj02::parse_g2o(path, d->state, d->bearings, d->odometry, d->fixed_pose_id, d->bound);
    if (rc) { delete d; return hfail(BOS_ERR_IO, rc == -1 ? "cannot open g2o file" : "malformed g2o line"); }
    if (d->state.number_of_poses() == 0) { delete d; return hfail(BOS_ERR_INVALID, "no poses"); }
    if (d->fixed_pose_id < 0) d->fixed_pose_id = d->state.default_pose_id();   // bearing_only_slam.cpp:63-65
    if (triangulate) proj02::triangulate_landmarks(d->state, d->bearings, verbose != 0);
    const int r2 = d->finalize();
    if (r2) { delete d; return r2; }
    *out = d;
    return BOS_OK;
}

double bos_normalized_angle_f64(double a) { return bos::normalized_angle<double>(a); }
float bos_normalized_angle_f32(float a) { return bos::normalized_angle<float>(a); }

int bos_dataset_synthetic(int32_t num_poses, int32_t num_landmarks, int32_t bearings_per_pose, uint64_t seed,
                          bos_dataset** out) {
    if (!out) return hfail(BOS_ERR_INVALID, "null argument");
    *out = nullptr;
    proj02::SyntheticParams p;
    p.num_poses = num_poses;
    p.num_landmarks = num_landmarks;
    p.bearings_per_pose = bearings_per_pose;
    p.seed = seed;
    proj02::SyntheticWorld w;
    if (!proj02::make_synthetic(p, w)) return hfail(BOS_ERR_INVALID, "infeasible synthetic sizes");
    bos_dataset* d = new bos_dataset();
    d->state = w.initial_guess;
    d->bearings = std::move(w.bearings);
    d->odometry = std::move(w.odometry);
    d->fixed_pose_id = w.fixed_pose_id;
    proj02::triangulate_landmarks(d->state, d->bearings, false);
    const int rc = d->finalize();
    if (rc) { delete d; return rc; }
    // ground truth in the same stix order (landmark ids ascending in both states)
    d->has_gt = true;
    for (const proj02::NEPose& q : w.ground_truth.poses_vec()) {
        d->gt_pose.push_back(q.x); d->gt_pose.push_back(q.y); d->gt_pose.push_back(q.theta);
    }
    d->gt_lm.resize(2 * d->lm_ids.size());
    for (size_t j = 0; j < d->lm_ids.size(); ++j) {
        const proj02::LMPos l = w.ground_truth.get_landmark_by_id(d->lm_ids[j]);
        d->gt_lm[2 * j] = l.x; d->gt_lm[2 * j + 1] = l.y;
    }
    double b = 0;
    for (double v : d->gt_pose) b = std::max(b, std::fabs(v));
    d->bound = (float)b + 3.0f;
    *out = d;
    return BOS_OK;
}

int bos_dataset_problem(const bos_dataset* d, bos_problem* v) {
    if (!d || !v) return hfail(BOS_ERR_INVALID, "null argument");
    std::memset(v, 0, sizeof(*v));
    v->num_poses = (int32_t)d->pose_ids.size();
    v->num_landmarks = (int32_t)d->lm_ids.size();
    v->num_bearings = (int32_t)d->b_pose.size();
    v->num_odometry = (int32_t)d->o_src.size();
    v->pose_xyt = d->pose_xyt.data();
    v->landmark_xy = d->lm_xy.empty() ? nullptr : d->lm_xy.data();
    v->bearing_pose = d->b_pose.data();
    v->bearing_landmark = d->b_lm.data();
    v->bearing_z = d->b_z.data();
    v->bearing_omega = nullptr;
    v->odom_src = d->o_src.data();
    v->odom_dst = d->o_dst.data();
    v->odom_z = d->o_z.data();
    v->odom_omega = d->o_om.data();
    v->fixed_pose = d->fixed_stix;
    return BOS_OK;
}

const int32_t* bos_dataset_pose_ids(const bos_dataset* d) { return d ? d->pose_ids.data() : nullptr; }
const int32_t* bos_dataset_landmark_ids(const bos_dataset* d) { return d ? d->lm_ids.data() : nullptr; }
int32_t bos_dataset_fixed_pose_id(const bos_dataset* d) { return d ? d->fixed_pose_id : -1; }
float bos_dataset_bound(const bos_dataset* d) { return d ? d->bound : 0.f; }

int bos_dataset_ground_truth(const bos_dataset* d, const double** pose_xyt, const double** landmark_xy) {
    if (!d || !d->has_gt) return hfail(BOS_ERR_INVALID, "no ground truth");
    if (pose_xyt) *pose_xyt = d->gt_pose.data();
    if (landmark_xy) *landmark_xy = d->gt_lm.data();
    return BOS_OK;
}

int bos_dataset_write_g2o(const bos_dataset* d, const char* path, const double* pose_xyt, const double* landmark_xy,
                          int with_landmarks) {
    if (!d || !path) return hfail(BOS_ERR_INVALID, "null argument");
    proj02::State st((int)d->pose_ids.size(), (int)d->lm_ids.size());
    const double* P = pose_xyt ? pose_xyt : d->pose_xyt.data();
    const double* L = landmark_xy ? landmark_xy : d->lm_xy.data();
    for (size_t i = 0; i < d->pose_ids.size(); ++i) st.add_pose(P[3 * i], P[3 * i + 1], P[3 * i + 2], d->pose_ids[i]);
    for (size_t j = 0; j < d->lm_ids.size(); ++j) st.add_landmark(L[2 * j], L[2 * j + 1], d->lm_ids[j]);
    if (proj02::write_g2o(path, st, d->bearings, d->odometry, d->fixed_pose_id, with_landmarks != 0))
        return hfail(BOS_ERR_IO, "cannot write g2o file");
    return BOS_OK;
}

void bos_dataset_free(bos_dataset* d) { delete d; }

namespace {
int factor_mode_of(int32_t solver) {
    switch (solver) {
        case BOS_SOLVER_SUPERNODAL: return bos::kFactorMultifrontal;
        case BOS_SOLVER_SCHUR: return bos::kFactorSchur;
        case BOS_SOLVER_ROCSOLVER_RF: return bos::kFactorScalar;
        case BOS_SOLVER_DENSE_CHOL: return bos::kFactorNone;
        default: return -1;
    }
}

// The planning fields of an options struct (NULL = defaults): the problem index with the plan
// options, the factor mode, and the options themselves
int plan_args(const bos_problem* pb, const bos_options* in, bos::ProblemIndex& pi, int& fmode, bos_options& opt) {
    bos_default_options(&opt);
    if (in) opt = *in;
    fmode = factor_mode_of(opt.solver);
    if (fmode < 0) return hfail(BOS_ERR_INVALID, "unknown solver");
    if (opt.partition != BOS_PARTITION_SUBTREE && opt.partition != BOS_PARTITION_OBSERVATIONS)
        return hfail(BOS_ERR_INVALID, "unknown partition");
    pi = index_of(pb);
    pi.lpp = opt.lanes_per_pose;
    pi.schur_leaf = opt.schur_leaf;
    return BOS_OK;
}

// The plan of rank `rank` of `world`: BOS_PARTITION_OBSERVATIONS plans are one-GPU plans (every rank
// holds the whole structure and runs a range of its lanes)
int plan_for(const bos::ProblemIndex& pi, const bos_options& opt, int fmode, int rank, int world, bos::Plan& P,
             std::string& err) {
    if (opt.partition == BOS_PARTITION_OBSERVATIONS) return bos::build_plan(pi, 0, 1, fmode, P, err);
    return bos::build_plan(pi, rank, world, fmode, P, err);
}
}  // namespace

void bos_debug_set_g2o_parser(int32_t line_by_line) { proj02::g_g2o_line_parser = line_by_line != 0; }

int bos_plan_inspect(const bos_problem* pb, const bos_options* options, int32_t rank, int32_t world, int64_t capacity,
                     int32_t* ref_rows, int32_t* ref_cols, uint8_t* owned, uint8_t* b_owned, int32_t* perm_to_ref,
                     bos_plan_info* info) {
    if (!pb) return hfail(BOS_ERR_INVALID, "null problem");
    if (world < 1 || rank < 0 || rank >= world) return hfail(BOS_ERR_INVALID, "bad rank/world");
    bos::ProblemIndex pi;
    bos_options opt;
    int fmode = 0;
    int rc = plan_args(pb, options, pi, fmode, opt);
    if (rc) return rc;
    bos::Plan P;
    std::string err;
    rc = plan_for(pi, opt, fmode, rank, world, P, err);
    if (rc) return hfail(rc, err);
    // observations partition: this rank's share of the one-GPU plan's lanes
    const bool obs = opt.partition == BOS_PARTITION_OBSERVATIONS && world > 1;
    std::vector<char> lane_node;
    std::vector<uint8_t> own_e;
    if (obs) {
        int64_t pb0, pb1, lb0, lb1;
        bos::observation_lanes(P, rank, world, pb0, pb1, lb0, lb1, &lane_node);
        bos::owned_entries(P, lane_node, own_e);
    }
    const int NP = pi.NP;
    std::vector<int32_t> ref(P.n + 3);
    for (int u = 0; u < pi.NP + pi.NL; ++u) {
        const int sz = u < NP ? 3 : 2;
        const int r0 = u < NP ? 3 * u : 3 * NP + 2 * (u - NP);
        for (int d = 0; d < sz; ++d) ref[P.node_dof[u] + d] = r0 + d;
    }
    if (info) {
        std::memset(info, 0, sizeof(*info));
        info->n = P.n;
        info->nnz_lower = P.nnzA();
        info->nnz_factor = P.mf.nsuper ? P.mf.L_size : P.nnzL();
        info->num_block_values = P.blk.size;
        info->lanes_per_pose = P.blk.lpp;
        info->flops_temporal = P.ordering.flops_temporal;
        info->flops_nested_dissection = P.ordering.flops_nd;
        info->mf_supernodes = P.mf.nsuper;
        info->mf_fold_fp32 = bos::mf_fold_reads_fp32(P) ? 1 : 0;
        for (int32_t p0 : P.blk.lm_lane_run) info->lm_lanes_consecutive += p0 >= 0;
        for (uint8_t c : P.blk.po_chain) info->pose_odometry_chain += c;
        info->mf_levels = P.mf.nlevels;
        info->mf_max_front = P.mf.max_m;
        info->mf_flops = P.mf.flops;
        info->mf_update_bytes = P.mf.U_size * 8;
        info->mf_fits = P.mf.fits;
        info->mf_max_front_upper = P.mf.max_m_upper;
        info->mf_balance_pct = P.mf.balance_pct;
        const bos::Shard& S = P.shard;
        info->shard_own_fronts = S.n_own_fronts;
        info->shard_top_fronts = S.n_top_fronts;
        info->shard_roots = S.root_ptr.empty() ? 0 : S.root_ptr[rank + 1] - S.root_ptr[rank];
        info->shard_ex1_doubles = S.ex1_count;
        info->shard_ex2_doubles = S.ex2_count;
        info->shard_pose_lanes = (int64_t)S.lane_poses.size();
        info->shard_own_pose_lanes = S.own_pose_lanes;
        info->shard_lm_lanes = (int64_t)S.lane_lms.size();
        info->shard_update_nodes = (int64_t)S.upd_nodes.size();
        std::strncpy(info->ordering, P.ordering.chosen.c_str(), sizeof(info->ordering) - 1);
    }
    if (ref_rows || ref_cols || owned) {
        if (capacity < P.nnzA()) return hfail(BOS_ERR_INVALID, "capacity < nnz_lower");
        for (int64_t r = 0; r < P.n; ++r)
            for (int64_t e = P.rowptr[r]; e < P.rowptr[r + 1]; ++e) {
                const int32_t a = ref[r], c = ref[P.colind[e]];
                if (ref_rows) ref_rows[e] = std::max(a, c);
                if (ref_cols) ref_cols[e] = std::min(a, c);
                if (owned) owned[e] = obs ? own_e[e] : P.blk.csr_src[e] >= 0 ? 1 : 0;
            }
    }
    if (perm_to_ref)
        for (int64_t i = 0; i < P.n + 3; ++i) perm_to_ref[i] = ref[i];
    if (b_owned) {   // b lives in the reference numbering; a lane writes its node's entries
        for (int64_t i = 0; i < P.n + 3; ++i) b_owned[i] = 0;
        for (int32_t p : P.blk.lane_pose)
            if (p >= 0 && (!obs || lane_node[p]))
                for (int d = 0; d < 3; ++d) b_owned[3 * (int64_t)p + d] = 1;
        for (int32_t l : P.blk.lm_lane_lm)
            if (!obs || lane_node[NP + l])
                for (int d = 0; d < 2; ++d) b_owned[3 * (int64_t)NP + 2 * (int64_t)l + d] = 1;
    }
    return BOS_OK;
}

int bos_plan_node_owner(const bos_problem* pb, const bos_options* options, int32_t world, int32_t* owner) {
    if (!pb || !owner || world < 1) return hfail(BOS_ERR_INVALID, "bad argument");
    bos::ProblemIndex pi;
    bos_options opt;
    int fmode = 0;
    int rc = plan_args(pb, options, pi, fmode, opt);
    if (rc) return rc;
    if (opt.partition == BOS_PARTITION_OBSERVATIONS)
        return hfail(BOS_ERR_UNSUPPORTED, "observations partition: every rank holds every node");
    bos::Plan P;
    std::string err;
    rc = bos::build_plan(pi, 0, world, fmode, P, err);
    if (rc) return hfail(rc, err);
    if (P.shard.node_owner.empty()) return hfail(BOS_ERR_UNSUPPORTED, "no shard (not a multifrontal solver)");
    std::copy(P.shard.node_owner.begin(), P.shard.node_owner.end(), owner);
    return BOS_OK;
}

// Test hook: runs the multifrontal algorithm of hip/multifrontal.hip on the host with the plan's
// tree and maps (validates the symbolic structure without a GPU). vals: values of the stored
// entries of H_nf in bos_plan_inspect's order (scattered into the block array here), rhs / x:
// permuted order of length n. Not used by any solve path.
int bos_plan_mf_selftest(const bos_problem* pb, const bos_options* options, const double* vals, const double* rhs,
                         double* x) {
    if (!pb || !vals || !rhs || !x) return hfail(BOS_ERR_INVALID, "null argument");
    bos::ProblemIndex pi;
    bos_options opt;
    int fmode = 0;
    int rc = plan_args(pb, options, pi, fmode, opt);
    if (rc) return rc;
    if (opt.solver != BOS_SOLVER_SUPERNODAL && opt.solver != BOS_SOLVER_SCHUR)
        return hfail(BOS_ERR_INVALID, "selftest needs a multifrontal solver");
    bos::Plan P;
    std::string err;
    rc = bos::build_plan(pi, 0, 1, fmode, P, err);
    if (rc) return hfail(rc, err);
    bos::HostMf M(P, vals, rhs);
    auto all = [](int) { return true; };
    M.factor(all);
    M.forward(all);
    M.backward(all);
    std::copy(M.x.begin(), M.x.end(), x);
    return BOS_OK;
}

// The sharded solve (plan.hpp Shard) simulated on the host for all `world` ranks, exchanges
// included (the all-gathers become concatenations of the per-rank send buffers). Every rank builds
// its own plan, holds only the block values its J+H computes (vals scattered through its
// csr_src), factors and forward-solves its subtrees, packs its roots' U / u (exchange1_segments),
// unpacks the others', factors and solves the top, solves its subtrees backward and packs its
// boundary solution (exchange 2). Checks: the ranks agree on the top bit for bit; the merged x
// (each node from its owner) equals the one-rank run bit for bit; every observation's chi^2 is
// counted by exactly one rank; every node a rank's J+H lanes read is in its box-plus set.
int bos_plan_shard_selftest(const bos_problem* pb, const bos_options* options, int32_t world, const double* vals,
                            const double* rhs, double* x) {
    if (!pb || !vals || !rhs || !x || world < 1) return hfail(BOS_ERR_INVALID, "bad argument");
    bos::ProblemIndex pi;
    bos_options opt;
    int fmode = 0;
    const int arc = plan_args(pb, options, pi, fmode, opt);
    if (arc) return arc;
    if (opt.solver != BOS_SOLVER_SUPERNODAL && opt.solver != BOS_SOLVER_SCHUR)
        return hfail(BOS_ERR_INVALID, "selftest needs a multifrontal solver");
    if (opt.partition != BOS_PARTITION_SUBTREE) return hfail(BOS_ERR_INVALID, "selftest of the subtree partition");
    const int NP = pi.NP, NL = pi.NL;
    std::vector<bos::Plan> plans(world);
    for (int r = 0; r < world; ++r) {
        std::string err;
        const int rc = bos::build_plan(pi, r, world, fmode, plans[r], err);
        if (rc) return hfail(rc, err);
    }
    bos::Plan one;
    {
        std::string err;
        const int rc = bos::build_plan(pi, 0, 1, fmode, one, err);
        if (rc) return hfail(rc, err);
    }
    const int64_t n = one.n;
    // the one-rank run: the values each rank's J+H computes are the one-rank values of those entries
    bos::HostMf ref(one, vals, rhs);
    auto all = [](int) { return true; };
    ref.factor(all);
    ref.forward(all);
    ref.backward(all);
    std::vector<bos::HostMf> M;
    M.reserve(world);
    for (int r = 0; r < world; ++r) {
        const bos::Plan& P = plans[r];
        if (P.n != n || P.mf.nsuper != one.mf.nsuper || P.mf.L_size != one.mf.L_size)
            return hfail(BOS_ERR_INVALID, "ranks disagree on the tree");
        M.emplace_back(P, vals, rhs);
    }
    // phase 1: own subtrees
    std::vector<std::vector<double>> send1(world);
    for (int r = 0; r < world; ++r) {
        const bos::Shard& S = plans[r].shard;
        auto own = [&](int s) { return S.sn_owner[s] == r; };
        M[r].factor(own);
        M[r].forward(own);
        std::vector<bos::ExchangeSeg> pk, un;
        bos::exchange1_segments(plans[r], pk, un);
        send1[r].assign(S.ex1_count, 0.0);
        for (const bos::ExchangeSeg& g : pk) {
            const std::vector<double>& src = g.src_kind == 0 ? M[r].U : M[r].u;
            if (g.dst_kind != 2 || g.dst + g.len > S.ex1_count) return hfail(BOS_ERR_INVALID, "exchange 1 pack out of range");
            std::copy(src.begin() + g.src, src.begin() + g.src + g.len, send1[r].begin() + g.dst);
        }
    }
    for (int r = 0; r < world; ++r) {   // the all-gather + unpack
        const bos::Shard& S = plans[r].shard;
        std::vector<double> recv;
        for (int q = 0; q < world; ++q) {
            if (plans[q].shard.ex1_count != S.ex1_count) return hfail(BOS_ERR_INVALID, "ranks disagree on exchange 1");
            recv.insert(recv.end(), send1[q].begin(), send1[q].end());
        }
        std::vector<bos::ExchangeSeg> pk, un;
        bos::exchange1_segments(plans[r], pk, un);
        for (const bos::ExchangeSeg& g : un) {
            std::vector<double>& dst = g.dst_kind == 0 ? M[r].U : M[r].u;
            if (g.src_kind != 3 || g.src + g.len > (int64_t)recv.size()) return hfail(BOS_ERR_INVALID, "exchange 1 unpack out of range");
            std::copy(recv.begin() + g.src, recv.begin() + g.src + g.len, dst.begin() + g.dst);
        }
        auto topf = [&](int s) { return S.sn_owner[s] == -1; };
        auto own = [&](int s) { return S.sn_owner[s] == r; };
        M[r].factor(topf);
        M[r].forward(topf);
        M[r].backward(topf);
        M[r].backward(own);
    }
    // exchange 2: boundary solution from its owner
    for (int r = 0; r < world; ++r) {
        const bos::Shard& S = plans[r].shard;
        for (int q = 0; q < world; ++q) {
            if (q == r) continue;
            for (int i = S.bnd_ptr[q]; i < S.bnd_ptr[q + 1]; ++i) M[r].x[S.bnd_dof[i]] = M[q].x[S.bnd_dof[i]];
        }
    }
    // checks
    const bos::Shard& S0 = plans[0].shard;
    std::vector<int> owner_of_dof(n, -3);
    for (int u = 0; u < NP + NL; ++u) {
        if (S0.node_owner[u] == -2) continue;
        const int sz = u < NP ? 3 : 2;
        for (int d = 0; d < sz; ++d) owner_of_dof[one.node_dof[u] + d] = S0.node_owner[u];
    }
    for (int64_t i = 0; i < n; ++i) {
        const int o = owner_of_dof[i];
        if (o == -3) return hfail(BOS_ERR_INVALID, "dof without an owner");
        const double v = M[o < 0 ? 0 : o].x[i];
        if (o < 0)
            for (int r = 1; r < world; ++r)
                if (M[r].x[i] != v) return hfail(BOS_ERR_INVALID, "ranks disagree on a top dof");
        if (v != ref.x[i]) return hfail(BOS_ERR_INVALID, "sharded solution differs from the one-rank solution");
        x[i] = v;
    }
    std::vector<int> chi(pi.Mb + pi.Mo, 0);
    for (int r = 0; r < world; ++r) {
        const bos::Plan& P = plans[r];
        const bos::Shard& S = P.shard;
        if (S.node_owner != S0.node_owner) return hfail(BOS_ERR_INVALID, "ranks disagree on node ownership");
        std::vector<char> fresh(NP + NL, 0);
        for (int u : S.upd_nodes) fresh[u] = 1;
        fresh[pi.fixed] = 1;
        std::vector<char> lane(NP + NL, 0);
        for (size_t i = 0; i < S.lane_poses.size(); ++i) {
            const int p = S.lane_poses[i];
            if (p < 0) continue;
            lane[p] = 1;
            if ((int)i < S.own_pose_lanes || r == 0) {
                for (int k = 0; k < pi.Mb; ++k) if (pi.b_pose[k] == p) ++chi[k];
                for (int k = 0; k < pi.Mo; ++k) if (pi.o_src[k] == p && pi.o_src[k] != pi.o_dst[k]) ++chi[pi.Mb + k];
            }
        }
        for (int l : S.lane_lms) lane[NP + l] = 1;
        for (int k = 0; k < pi.Mb; ++k) {
            const int p = pi.b_pose[k], l = NP + pi.b_lm[k];
            if ((lane[p] || lane[l]) && !(fresh[p] && fresh[l])) return hfail(BOS_ERR_INVALID, "a J+H lane reads a stale node");
        }
        for (int k = 0; k < pi.Mo; ++k) {
            const int a = pi.o_src[k], b = pi.o_dst[k];
            if ((lane[a] || lane[b]) && !(fresh[a] && fresh[b])) return hfail(BOS_ERR_INVALID, "a J+H lane reads a stale node");
        }
    }
    for (int k = 0; k < pi.Mb + pi.Mo; ++k) {
        const bool loop = k >= pi.Mb && pi.o_src[k - pi.Mb] == pi.o_dst[k - pi.Mb];
        if (chi[k] != (loop ? 0 : 1)) return hfail(BOS_ERR_INVALID, "chi^2 of an observation not counted exactly once");
    }
    return BOS_OK;
}

}  // extern "C"
