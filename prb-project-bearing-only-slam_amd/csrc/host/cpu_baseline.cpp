// CPU baseline of bench.py ("the build's own C++ CPU backend"):
// one Gauss-Newton iteration of the reference's Solver::step (slam/solver.cpp:27-97) on the host's
// cores, with the same static plan as the GPU path —
//   * J+H: every pose lane and landmark lane of the plan (host/plan.hpp BlockLayout) evaluated in
//     parallel over poses / landmarks, written into the same block array (fp64),
//   * sparse Cholesky: the multifrontal algorithm of hip/multifrontal.hip on the host (host/host_mf.hpp),
//     the fronts of each tree level in parallel,
//   * box-plus in parallel.
// Timed by bench.py only; bos_create / bos_step never use it (the product has no CPU fallback).
#include <cmath>
#include <cstring>
#include <memory>
#include <string>

#include "../../../include/bos_host.h"
#include "bos_math.hpp"
#include "error.hpp"
#include "host_mf.hpp"
#include "plan.hpp"

struct bos_cpu_gn {
    bos::Plan plan;
    std::unique_ptr<bos::Pool> pool;
    std::unique_ptr<bos::HostMf> mf;
    int NP = 0, NL = 0;
    std::vector<double> pose, lm, b;
    std::vector<int32_t> b_pose, b_lm, o_src, o_dst;
    std::vector<double> b_z, b_w, o_z, o_om;   // o_om: upper triangle (00, 01, 02, 11, 12, 22)
    double kt = 1.0, damping = 0.01;
};

namespace {

int cfail(int code, const std::string& m) { return bos::set_error(code, m); }

// J+H of one pose lane group (all of its lanes) and of one landmark lane, as hip/kernels.hip
// pose_lanes / landmark_lane compute them (fp64)
void jh_pose(bos_cpu_gn* c, int grp, double& chi) {
    const bos::Plan& P = c->plan;
    const bos::BlockLayout& B = P.blk;
    const int p = B.lane_pose[grp];
    if (p < 0) return;
    const double X = c->pose[3 * p], Y = c->pose[3 * p + 1], th = c->pose[3 * p + 2];
    const double cs = std::cos(th), ss = std::sin(th);
    double h[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
    double* hv = c->mf->hval.data();
    for (int sub = 0; sub < B.lpp; ++sub) {
        const int lane = grp * B.lpp + sub;
        const int n = B.pose_lanes.cnt[lane];
        double acc[6] = {0, 0, 0, 0, 0, 0};
        for (int j = 0; j < n; ++j) {
            const int32_t sl = B.pose_lanes.slot(lane, j);
            const int k = B.pose_lanes.obs[sl];
            const int l = c->b_lm[k];
            double J[5];
            double e = bos::bearing_error_jacobian<double>(X, Y, cs, ss, c->lm[2 * l], c->lm[2 * l + 1], c->b_z[k], J);
            const double w = c->b_w.empty() ? 1.0 : c->b_w[k];
            const double rho = e * w * e;
            chi += rho;
            if (rho > c->kt) e *= std::sqrt(c->kt / rho);
            const double w0 = J[0] * w, w1 = J[1] * w, w2 = J[2] * w;
            h[0] += w0 * J[0]; h[1] += w1 * J[0]; h[2] += w1 * J[1];
            h[3] += w2 * J[0]; h[4] += w2 * J[1]; h[5] += w2 * J[2];
            g[0] += w0 * e; g[1] += w1 * e; g[2] += w2 * e;
            const double o[6] = {w0 * J[3], w0 * J[4], w1 * J[3], w1 * J[4], w2 * J[3], w2 * J[4]};
            for (int q = 0; q < 6; ++q) acc[q] += o[q];
            const bool last = j + 1 == n ||
                              c->b_lm[B.pose_lanes.obs[B.pose_lanes.slot(lane, j + 1)]] != l;
            if (last) {
                double* dst = hv + B.off_pl + 6 * (int64_t)sl;
                for (int q = 0; q < 6; ++q) { dst[q] = acc[q]; acc[q] = 0.0; }
            }
        }
    }
    double acc6[6] = {0, 0, 0, 0, 0, 0};
    for (int x = B.po_ptr[p]; x < B.po_ptr[p + 1]; ++x) {
        const int e = B.po_ent[x], k = e >> 1;
        const bool dst = e & 1;
        const int s = c->o_src[k], d = c->o_dst[k];
        const double* zs = c->o_z.data() + 3 * (size_t)k;
        const double* u = c->o_om.data() + 6 * (size_t)k;
        double E[3], J[18];
        bos::odometry_error_jacobian<double>(c->pose[3 * s], c->pose[3 * s + 1], c->pose[3 * s + 2],
                                             std::cos(c->pose[3 * s + 2]), std::sin(c->pose[3 * s + 2]), c->pose[3 * d],
                                             c->pose[3 * d + 1], c->pose[3 * d + 2], zs[0], zs[1], zs[2], E, J);
        const double Om[3][3] = {{u[0], u[1], u[2]}, {u[1], u[3], u[4]}, {u[2], u[4], u[5]}};
        double Oe[3];
        for (int i = 0; i < 3; ++i) Oe[i] = Om[i][0] * E[0] + Om[i][1] * E[1] + Om[i][2] * E[2];
        const double rho = E[0] * Oe[0] + E[1] * Oe[1] + E[2] * Oe[2];
        if (rho > c->kt) {
            const double sc = std::sqrt(c->kt / rho);
            for (int i = 0; i < 3; ++i) Oe[i] *= sc;
        }
        if (!dst) chi += rho;
        // H_ss = J_s^T Omega J_s (J_d = -J_s), b_s = J_s^T Omega e
        double Hs[3][3], bs[3];
        for (int a = 0; a < 3; ++a) {
            for (int b2 = 0; b2 < 3; ++b2) {
                double v = 0.0;
                for (int i = 0; i < 3; ++i)
                    for (int jj = 0; jj < 3; ++jj) v += J[6 * i + a] * Om[i][jj] * J[6 * jj + b2];
                Hs[a][b2] = v;
            }
            bs[a] = J[a] * Oe[0] + J[6 + a] * Oe[1] + J[12 + a] * Oe[2];
        }
        const double hl[6] = {Hs[0][0], Hs[1][0], Hs[1][1], Hs[2][0], Hs[2][1], Hs[2][2]};
        for (int q = 0; q < 6; ++q) h[q] += hl[q];
        for (int q = 0; q < 3; ++q) g[q] += dst ? -bs[q] : bs[q];
        const int blk = B.po_blk[x];
        if (blk >= 0) {
            for (int q = 0; q < 6; ++q) acc6[q] -= hl[q];
            if (x + 1 == B.po_ptr[p + 1] || B.po_blk[x + 1] != blk) {
                double* dstp = hv + B.off_pp + 6 * (int64_t)blk;
                for (int q = 0; q < 6; ++q) { dstp[q] = acc6[q]; acc6[q] = 0.0; }
            }
        }
    }
    double* hp = hv + 6 * (int64_t)p;
    const double lam = c->damping;
    hp[0] = h[0] + lam; hp[1] = h[1]; hp[2] = h[2] + lam; hp[3] = h[3]; hp[4] = h[4]; hp[5] = h[5] + lam;
    for (int q = 0; q < 3; ++q) c->b[3 * (size_t)p + q] = g[q];
}

void jh_landmark(bos_cpu_gn* c, int lane) {
    const bos::BlockLayout& B = c->plan.blk;
    const int l = B.lm_lane_lm[lane];
    const double lx = c->lm[2 * l], ly = c->lm[2 * l + 1];
    double h[3] = {0, 0, 0}, g[2] = {0, 0};
    for (int j = 0; j < B.lm_lanes.cnt[lane]; ++j) {
        const int k = B.lm_lanes.obs[B.lm_lanes.slot(lane, j)];
        const int p = c->b_pose[k];
        const double th = c->pose[3 * p + 2];
        double J[5];
        double e = bos::bearing_error_jacobian<double>(c->pose[3 * p], c->pose[3 * p + 1], std::cos(th), std::sin(th), lx,
                                                       ly, c->b_z[k], J);
        const double w = c->b_w.empty() ? 1.0 : c->b_w[k];
        const double rho = e * w * e;
        if (rho > c->kt) e *= std::sqrt(c->kt / rho);
        const double w3 = J[3] * w, w4 = J[4] * w;
        h[0] += w3 * J[3]; h[1] += w4 * J[3]; h[2] += w4 * J[4];
        g[0] += w3 * e; g[1] += w4 * e;
    }
    double* hp = c->mf->hval.data() + B.off_ldiag + 3 * (int64_t)l;
    hp[0] = h[0] + c->damping; hp[1] = h[1]; hp[2] = h[2] + c->damping;
    c->b[3 * (size_t)c->NP + 2 * (size_t)l] = g[0];
    c->b[3 * (size_t)c->NP + 2 * (size_t)l + 1] = g[1];
}

}  // namespace

extern "C" {

int bos_cpu_gn_create(const bos_problem* pb, int32_t solver, int32_t threads, bos_cpu_gn** out) {
    if (!pb || !out) return cfail(BOS_ERR_INVALID, "null argument");
    if (solver != BOS_SOLVER_SCHUR && solver != BOS_SOLVER_SUPERNODAL)
        return cfail(BOS_ERR_INVALID, "the CPU baseline runs the multifrontal solvers");
    *out = nullptr;
    std::unique_ptr<bos_cpu_gn> c(new bos_cpu_gn());
    bos::ProblemIndex pi;
    pi.NP = pb->num_poses; pi.NL = pb->num_landmarks; pi.Mb = pb->num_bearings; pi.Mo = pb->num_odometry;
    pi.fixed = pb->fixed_pose;
    pi.b_pose = pb->bearing_pose; pi.b_lm = pb->bearing_landmark; pi.o_src = pb->odom_src; pi.o_dst = pb->odom_dst;
    pi.b_omega = pb->bearing_omega; pi.o_omega = pb->odom_omega;
    std::string err;
    const int rc = bos::build_plan(pi, 0, 1, solver == BOS_SOLVER_SCHUR ? bos::kFactorSchur : bos::kFactorMultifrontal,
                                   c->plan, err);
    if (rc) return cfail(rc, err);
    c->NP = pi.NP;
    c->NL = pi.NL;
    c->pose.assign(pb->pose_xyt, pb->pose_xyt + 3 * (size_t)pi.NP);
    for (int i = 0; i < pi.NP; ++i) c->pose[3 * i + 2] = bos::normalized_angle<double>(bos::smallest_angle<double>(c->pose[3 * i + 2]));
    if (!pb->landmark_xy && pi.NL) return cfail(BOS_ERR_INVALID, "the CPU baseline needs landmark positions");
    c->lm.assign(pb->landmark_xy, pb->landmark_xy + 2 * (size_t)pi.NL);
    c->b.assign(3 * (size_t)pi.NP + 2 * (size_t)pi.NL, 0.0);
    c->b_pose.assign(pi.b_pose, pi.b_pose + pi.Mb);
    c->b_lm.assign(pi.b_lm, pi.b_lm + pi.Mb);
    c->b_z.assign(pb->bearing_z, pb->bearing_z + pi.Mb);
    if (pb->bearing_omega) c->b_w.assign(pb->bearing_omega, pb->bearing_omega + pi.Mb);
    c->o_src.assign(pi.o_src, pi.o_src + pi.Mo);
    c->o_dst.assign(pi.o_dst, pi.o_dst + pi.Mo);
    c->o_z.assign(pb->odom_z, pb->odom_z + 3 * (size_t)pi.Mo);
    c->o_om.resize(6 * (size_t)pi.Mo);
    for (int k = 0; k < pi.Mo; ++k) {
        const double* m = pb->odom_omega + 9 * (size_t)k;
        const double u[6] = {m[0], m[1], m[2], m[4], m[5], m[8]};
        std::memcpy(&c->o_om[6 * (size_t)k], u, sizeof(u));
    }
    c->pool.reset(new bos::Pool(std::max(1, threads)));
    c->mf.reset(new bos::HostMf(c->plan, c->pool.get()));
    *out = c.release();
    return BOS_OK;
}

int bos_cpu_gn_step(bos_cpu_gn* c, double* chi2) {
    if (!c) return cfail(BOS_ERR_INVALID, "null handle");
    const bos::Plan& P = c->plan;
    bos::Pool& pool = *c->pool;
    const int G = (int)P.blk.lane_pose.size(), NLL = (int)P.blk.lm_lane_lm.size();
    // J+H (self-loops: chi^2 only, their Jacobian is zero; see host/plan.cpp build_layout)
    std::vector<double> chi_part(G, 0.0);
    pool.parallel_for(G, [&](int64_t i) { jh_pose(c, (int)i, chi_part[i]); });
    pool.parallel_for(NLL, [&](int64_t i) { jh_landmark(c, (int)i); });
    double chi = 0.0;
    for (double v : chi_part) chi += v;
    for (int k = 0; k < (int)c->o_src.size(); ++k)
        if (c->o_src[k] == c->o_dst[k]) {
            const double* z = &c->o_z[3 * (size_t)k];
            const double* u = &c->o_om[6 * (size_t)k];
            const double e[3] = {-z[0], -z[1], bos::normalized_angle<double>(-z[2])};
            const double Oe[3] = {u[0] * e[0] + u[1] * e[1] + u[2] * e[2], u[1] * e[0] + u[3] * e[1] + u[4] * e[2],
                                  u[2] * e[0] + u[4] * e[1] + u[5] * e[2]};
            chi += e[0] * Oe[0] + e[1] * Oe[1] + e[2] * Oe[2];
        }
    if (chi2) *chi2 = chi;
    // solve H_nf x = b_nf (rhs in elimination order), dx = -x
    bos::HostMf& M = *c->mf;
    const int64_t n = P.n;
    std::vector<int32_t> ref(n);
    for (int u = 0; u < c->NP + c->NL; ++u) {
        if (u == P.fixed) continue;
        const int sz = u < c->NP ? 3 : 2;
        const int r0 = u < c->NP ? 3 * u : 3 * c->NP + 2 * (u - c->NP);
        for (int d = 0; d < sz; ++d) ref[P.node_dof[u] + d] = r0 + d;
    }
    for (int64_t i = 0; i < n; ++i) M.x[i] = c->b[ref[i]];
    auto all = [](int) { return true; };
    M.factor(all);
    M.forward(all);
    M.backward(all);
    // box-plus (framework/state.cpp:69-80)
    pool.parallel_for(c->NP + c->NL, [&](int64_t u) {
        if (u == P.fixed) return;
        const int d = P.node_dof[u];
        if (u < c->NP) {
            double* p = &c->pose[3 * u];
            bos::boxplus_pose<double>(p[0], p[1], p[2], -M.x[d], -M.x[d + 1], -M.x[d + 2]);
        } else {
            double* l = &c->lm[2 * (u - c->NP)];
            l[0] += -M.x[d];
            l[1] += -M.x[d + 1];
        }
    });
    return BOS_OK;
}

int bos_cpu_gn_get_state(const bos_cpu_gn* c, double* pose_xyt, double* landmark_xy) {
    if (!c) return cfail(BOS_ERR_INVALID, "null handle");
    if (pose_xyt) std::memcpy(pose_xyt, c->pose.data(), c->pose.size() * sizeof(double));
    if (landmark_xy) std::memcpy(landmark_xy, c->lm.data(), c->lm.size() * sizeof(double));
    return BOS_OK;
}

void bos_cpu_gn_destroy(bos_cpu_gn* c) { delete c; }

}  // extern "C"
