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

// The multifrontal algorithm of hip/multifrontal.hip on the host (test hooks only): factor, forward
// and backward over the fronts a predicate selects, in level order, with the plan's maps. The block
// array holds what this plan's J+H writes: vals (stored entries of H_nf, one-rank order) through
// its csr_src.
struct HostMf {
    const bos::Plan& P;
    const bos::Multifrontal& F;
    std::vector<double> hval, L, U, u, x;
    std::vector<std::vector<double>> fwv;
    HostMf(const bos::Plan& plan, const double* vals, const double* rhs)
        : P(plan), F(plan.mf), hval(plan.blk.size, 0.0), L(plan.mf.L_size), U(plan.mf.U_size), u(plan.mf.u_size),
          x(rhs, rhs + plan.n), fwv(plan.mf.nsuper) {
        for (int64_t e = 0; e < P.nnzA(); ++e)
            if (P.blk.csr_src[e] >= 0) hval[P.blk.csr_src[e]] = vals[e];
    }
    // folded landmark children (Schur ordering): the fold records, as fold_children reads them;
    // their u entries accumulate per parent in fwv
    void fold(int s, std::vector<double>& W, int m) {
        fwv[s].assign(m, 0.0);
        for (int ch = F.fold_cptr[s]; ch < F.fold_cptr[s + 1]; ++ch) {
            const int q0 = F.fold_chunk[ch], nq = F.fold_chunk[ch + 1] - q0;
            std::vector<double> l0(nq), l1(nq);
            std::vector<int> pos(nq), rcs(nq);
            for (int q = 0; q < nq; ++q) {
                const int32_t* rec = F.fold_rec.data() + (size_t)bos::kFoldRec * (q0 + q);
                auto v = [&](int32_t src) { return src >= 0 ? hval[src] : 0.0; };
                const int col0 = rec[5], t = rec[6] & 63, rc = (rec[6] >> 6) & 63;
                const double l00 = std::sqrt(std::max(v(rec[2]), 1e-300)), l10 = v(rec[3]) / l00;
                const double l11 = std::sqrt(std::max(v(rec[4]) - l10 * l10, 1e-300));
                l0[q] = v(rec[0]) / l00;
                l1[q] = (v(rec[1]) - l0[q] * l10) / l11;
                const double y0 = x[col0] / l00, y1 = (x[col0 + 1] - l10 * y0) / l11;
                double* Lc = L.data() + rec[7];
                const int mc = 2 + rc;
                Lc[2 + t] = l0[q];
                Lc[mc + 2 + t] = l1[q];
                if (t == 0) { Lc[0] = l00; Lc[1] = l10; Lc[mc + 1] = l11; }
                pos[q] = (rec[6] >> 12) & 63;
                rcs[q] = rc;
                fwv[s][pos[q]] -= l0[q] * y0 + l1[q] * y1;
            }
            for (int q = 0; q < nq; ++q) {   // the landmarks' forward results, after every row used them
                const int32_t* rec = F.fold_rec.data() + (size_t)bos::kFoldRec * (q0 + q);
                if ((rec[6] & 63) == 0) {
                    const int col0 = rec[5];
                    const double* Lc = L.data() + rec[7];
                    const double y0 = x[col0] / Lc[0];
                    x[col0 + 1] = (x[col0 + 1] - Lc[1] * y0) / Lc[2 + ((rec[6] >> 6) & 63) + 1];
                    x[col0] = y0;
                }
            }
            for (int c0 = 0; c0 < nq; c0 += rcs[c0])
                for (int j = c0; j < c0 + rcs[c0]; ++j)
                    for (int i = j; i < c0 + rcs[c0]; ++i)
                        W[pos[i] + (size_t)pos[j] * m] -= l0[i] * l0[j] + l1[i] * l1[j];
        }
    }
    template <typename Pred> void factor(Pred sel) {
        for (int lv = 0; lv < F.nlevels; ++lv)
            for (int q = F.level_ptr[lv]; q < F.level_ptr[lv + 1]; ++q) {
                const int s = F.level[q], k = F.k[s], r = F.r[s], m = k + r;
                if (!sel(s)) continue;
                std::vector<double> W((size_t)m * m, 0.0);
                for (int a = F.amap_ptr[s]; a < F.amap_ptr[s + 1]; ++a) {
                    int64_t d = F.amap_dst[a];
                    if (m <= bos::kMfWaveMaxM) {   // packed lower column-major -> (i, j)
                        int64_t j = 0;
                        while (d >= m - j) { d -= m - j; ++j; }
                        d = (j + d) + j * m;
                    }
                    W[d] = hval[F.amap_src[a]];
                }
                fold(s, W, m);
                for (int ci = F.child_ptr[s] + F.fold_cnt[s]; ci < F.child_ptr[s + 1]; ++ci) {
                    const int c = F.child[ci], rc2 = F.r[c];
                    const int32_t* map = F.rmap.data() + F.rmap_off[c];
                    for (int j = 0; j < rc2; ++j)
                        for (int i = j; i < rc2; ++i) W[map[i] + (size_t)map[j] * m] += U[F.U_off[c] + bos::mf_packed(i, j, rc2)];
                }
                for (int j = 0; j < k; ++j) {
                    const double d = std::sqrt(std::max(W[j + (size_t)j * m], 1e-300));
                    W[j + (size_t)j * m] = d;
                    for (int i = j + 1; i < m; ++i) W[i + (size_t)j * m] /= d;
                    for (int l = j + 1; l < m; ++l)
                        for (int i = l; i < m; ++i) W[i + (size_t)l * m] -= W[i + (size_t)j * m] * W[l + (size_t)j * m];
                }
                for (int j = 0; j < k; ++j)
                    for (int i = 0; i < m; ++i) L[F.L_off[s] + i + (size_t)j * m] = W[i + (size_t)j * m];
                for (int j = 0; j < r; ++j)
                    for (int i = j; i < r; ++i) U[F.U_off[s] + bos::mf_packed(i, j, r)] = W[(k + i) + (size_t)(k + j) * m];
            }
    }
    template <typename Pred> void forward(Pred sel) {
        for (int lv = 0; lv < F.nlevels; ++lv)
            for (int q = F.level_ptr[lv]; q < F.level_ptr[lv + 1]; ++q) {
                const int s = F.level[q], k = F.k[s], r = F.r[s], m = k + r;
                if (!sel(s)) continue;
                std::vector<double> w(m, 0.0);
                for (int i = 0; i < k; ++i) w[i] = x[F.col0[s] + i];
                for (size_t i = 0; i < fwv[s].size(); ++i) w[i] += fwv[s][i];
                for (int ci = F.child_ptr[s] + F.fold_cnt[s]; ci < F.child_ptr[s + 1]; ++ci) {
                    const int c = F.child[ci];
                    for (int t = 0; t < F.r[c]; ++t) w[F.rmap[F.rmap_off[c] + t]] += u[F.u_off[c] + t];
                }
                const double* Ls = L.data() + F.L_off[s];
                for (int j = 0; j < k; ++j) {
                    w[j] /= Ls[j + (size_t)j * m];
                    for (int i = j + 1; i < m; ++i) w[i] -= Ls[i + (size_t)j * m] * w[j];
                }
                for (int i = 0; i < k; ++i) x[F.col0[s] + i] = w[i];
                for (int t = 0; t < r; ++t) u[F.u_off[s] + t] = w[k + t];
            }
    }
    // top-down over the selected fronts, then their folded landmarks
    template <typename Pred> void backward(Pred sel) {
        std::vector<int32_t> bwd;
        for (auto it = F.level.rbegin(); it != F.level.rend(); ++it)
            if (sel(*it)) bwd.push_back(*it);
        for (int s : F.fold_list)
            if (sel(F.parent[s])) bwd.push_back(s);
        for (int s : bwd) {
            const int k = F.k[s], m = k + F.r[s];
            const double* Ls = L.data() + F.L_off[s];
            const int32_t* fi = F.findex.data() + F.findex_off[s];
            for (int j = k - 1; j >= 0; --j) {
                double acc = x[F.col0[s] + j];
                for (int i = j + 1; i < m; ++i) acc -= Ls[i + (size_t)j * m] * x[fi[i]];
                x[F.col0[s] + j] = acc / Ls[j + (size_t)j * m];
            }
        }
    }
};

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
}  // namespace

void bos_debug_set_schur_leaf(int32_t poses) { bos::g_schur_leaf = poses > 0 ? poses : 0; }
void bos_debug_set_g2o_parser(int32_t line_by_line) { proj02::g_g2o_line_parser = line_by_line != 0; }

int bos_plan_inspect(const bos_problem* pb, int32_t solver, int32_t rank, int32_t world, int64_t capacity, int32_t* ref_rows,
                     int32_t* ref_cols, uint8_t* owned, uint8_t* b_owned, int32_t* perm_to_ref,
                     bos_plan_info* info) {
    if (!pb) return hfail(BOS_ERR_INVALID, "null problem");
    const int fmode = factor_mode_of(solver);
    if (fmode < 0) return hfail(BOS_ERR_INVALID, "unknown solver");
    const bos::ProblemIndex pi = index_of(pb);
    bos::Plan P;
    std::string err;
    const int rc = bos::build_plan(pi, rank, world, fmode, P, err);
    if (rc) return hfail(rc, err);
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
                if (owned) owned[e] = P.blk.csr_src[e] >= 0 ? 1 : 0;
            }
    }
    if (perm_to_ref)
        for (int64_t i = 0; i < P.n + 3; ++i) perm_to_ref[i] = ref[i];
    if (b_owned) {   // b lives in the reference numbering; a lane writes its node's entries
        for (int64_t i = 0; i < P.n + 3; ++i) b_owned[i] = 0;
        for (int32_t p : P.blk.lane_pose)
            if (p >= 0)
                for (int d = 0; d < 3; ++d) b_owned[3 * (int64_t)p + d] = 1;
        for (int32_t l : P.blk.lm_lane_lm)
            for (int d = 0; d < 2; ++d) b_owned[3 * (int64_t)NP + 2 * (int64_t)l + d] = 1;
    }
    return BOS_OK;
}

int bos_plan_node_owner(const bos_problem* pb, int32_t solver, int32_t world, int32_t* owner) {
    if (!pb || !owner) return hfail(BOS_ERR_INVALID, "null argument");
    const int fmode = factor_mode_of(solver);
    if (fmode < 0) return hfail(BOS_ERR_INVALID, "unknown solver");
    bos::Plan P;
    std::string err;
    const int rc = bos::build_plan(index_of(pb), 0, world, fmode, P, err);
    if (rc) return hfail(rc, err);
    if (P.shard.node_owner.empty()) return hfail(BOS_ERR_UNSUPPORTED, "no shard (not a multifrontal solver)");
    std::copy(P.shard.node_owner.begin(), P.shard.node_owner.end(), owner);
    return BOS_OK;
}

// Test hook: runs the multifrontal algorithm of hip/multifrontal.hip on the host with the plan's
// tree and maps (validates the symbolic structure without a GPU). vals: values of the stored
// entries of H_nf in bos_plan_inspect's order (scattered into the block array here), rhs / x:
// permuted order of length n. Not used by any solve path.
int bos_plan_mf_selftest(const bos_problem* pb, int32_t solver, const double* vals, const double* rhs, double* x) {
    if (!pb || !vals || !rhs || !x) return hfail(BOS_ERR_INVALID, "null argument");
    if (solver != BOS_SOLVER_SUPERNODAL && solver != BOS_SOLVER_SCHUR)
        return hfail(BOS_ERR_INVALID, "selftest needs a multifrontal solver");
    bos::Plan P;
    std::string err;
    const int rc = bos::build_plan(index_of(pb), 0, 1, factor_mode_of(solver), P, err);
    if (rc) return hfail(rc, err);
    HostMf M(P, vals, rhs);
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
int bos_plan_shard_selftest(const bos_problem* pb, int32_t solver, int32_t world, const double* vals, const double* rhs,
                            double* x) {
    if (!pb || !vals || !rhs || !x || world < 1) return hfail(BOS_ERR_INVALID, "bad argument");
    if (solver != BOS_SOLVER_SUPERNODAL && solver != BOS_SOLVER_SCHUR)
        return hfail(BOS_ERR_INVALID, "selftest needs a multifrontal solver");
    const bos::ProblemIndex pi = index_of(pb);
    const int NP = pi.NP, NL = pi.NL;
    std::vector<bos::Plan> plans(world);
    for (int r = 0; r < world; ++r) {
        std::string err;
        const int rc = bos::build_plan(pi, r, world, factor_mode_of(solver), plans[r], err);
        if (rc) return hfail(rc, err);
    }
    bos::Plan one;
    {
        std::string err;
        const int rc = bos::build_plan(pi, 0, 1, factor_mode_of(solver), one, err);
        if (rc) return hfail(rc, err);
    }
    const int64_t n = one.n;
    // the one-rank run: the values each rank's J+H computes are the one-rank values of those entries
    HostMf ref(one, vals, rhs);
    auto all = [](int) { return true; };
    ref.factor(all);
    ref.forward(all);
    ref.backward(all);
    std::vector<HostMf> M;
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
