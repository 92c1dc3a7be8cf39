#include "synthetic.hpp"

#include <algorithm>
#include <cmath>
#include <random>

namespace proj02 {

namespace {

struct Rng {
    std::mt19937_64 g;
    explicit Rng(uint64_t s) : g(s) {}
    double uniform() { return (double)(g() >> 11) * (1.0 / 9007199254740992.0); }   // [0, 1)
    double uniform(double a, double b) { return a + (b - a) * uniform(); }
    double normal() {   // Box-Muller, deterministic across standard libraries
        double u1 = uniform();
        while (u1 <= 1e-300) u1 = uniform();
        const double u2 = uniform();
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * bos::kPi * u2);
    }
    uint64_t below(uint64_t n) { return n ? g() % n : 0; }
};

}  // namespace

bool make_synthetic(const SyntheticParams& p, SyntheticWorld& out) {
    const int NP = p.num_poses, NL = p.num_landmarks, K = p.bearings_per_pose;
    if (NP < 2 || K < 1 || NL < K || (long long)NP * K < 2LL * NL) return false;
    Rng rng(p.seed);
    const double W = p.world_extent > 0 ? p.world_extent : std::min(1000.0, std::max(40.0, 3.0 * std::sqrt((double)NP)));
    const double half = 0.5 * W, margin = std::min(20.0, 0.15 * W);

    // ---- ground-truth trajectory and noisy odometry
    std::vector<double> gx(NP), gy(NP), gth(NP);
    gx[0] = 0; gy[0] = 0; gth[0] = 0;
    std::vector<double> zx(NP), zy(NP), zt(NP);
    double turn = 0;
    for (int i = 0; i + 1 < NP; ++i) {
        const double u = rng.uniform(0.75, 1.0);
        turn = 0.8 * turn + 0.02 * rng.normal();
        // steer towards the centre when close to the border
        const double nx = gx[i] + std::cos(gth[i]) * 4.0, ny = gy[i] + std::sin(gth[i]) * 4.0;
        if (std::fabs(nx) > half - margin || std::fabs(ny) > half - margin) {
            const double want = std::atan2(-gy[i], -gx[i]);
            const double d = bos::normalized_angle<double>(want - gth[i]);
            turn = std::max(-0.12, std::min(0.12, 0.25 * d));
        }
        const double dth = std::max(-0.15, std::min(0.15, turn));
        gx[i + 1] = gx[i] + std::cos(gth[i]) * u;
        gy[i + 1] = gy[i] + std::sin(gth[i]) * u;
        gth[i + 1] = bos::normalized_angle<double>(gth[i] + dth);
        // measurement in the source frame: R_s^T (t_d - t_s), theta_d - theta_s (+ noise)
        zx[i] = u + rng.normal() / std::sqrt(p.odom_info_xy);
        zy[i] = 0.0 + rng.normal() / std::sqrt(p.odom_info_xy);
        zt[i] = dth + rng.normal() / std::sqrt(p.odom_info_theta);
    }

    // ---- landmark windows: K lanes, each a composition of [0, NP) into windows of length >= 2
    std::vector<int> per_lane(K, NL / K);
    for (int k = 0; k < NL % K; ++k) per_lane[k] += 1;
    struct Win { int lane, first, last; };
    std::vector<Win> wins;
    wins.reserve(NL);
    for (int k = 0; k < K; ++k) {
        // balanced composition of NP poses into n windows (lengths within ~[base/2, 3*base/2],
        // every length >= 2) so that ranges stay sensor-like (the dataset's max range is 5 m)
        const int n = per_lane[k];
        const int base = NP / n;
        std::vector<int> len(n);
        // stagger the lanes: a random first window, the rest balanced
        len[0] = n > 1 ? std::max(2, std::min(NP - 2 * (n - 1), 2 + (int)rng.below((uint64_t)std::max(1, base))))
                       : NP;
        if (n > 1) {
            const int rem = NP - len[0], m = n - 1;
            for (int j = 1; j < n; ++j) len[j] = rem / m + ((j - 1) < rem % m ? 1 : 0);
            const int b2 = rem / m;
            const int lo = std::max(2, b2 - b2 / 2), hi = b2 + b2 / 2 + 1;
            for (int t = 0; t < 2 * m; ++t) {   // random neighbour transfers add jitter, keep the sum
                const int a = 1 + (int)rng.below((uint64_t)m), b = a + 1 < n ? a + 1 : 1;
                if (a != b && len[a] > lo && len[b] < hi) { --len[a]; ++len[b]; }
            }
        }
        int st = 0;
        for (int j = 0; j < n; ++j) {
            wins.push_back({k, st, st + len[j] - 1});
            st += len[j];
        }
    }
    // deterministic landmark order: by window start, then lane
    std::stable_sort(wins.begin(), wins.end(), [](const Win& a, const Win& b) {
        return a.first != b.first ? a.first < b.first : a.lane < b.lane;
    });

    // ---- landmark placement with parallax (">= 2 observations per landmark with
    // parallax"). A candidate is drawn from the window's last pose (bearing 20-82 deg to the window's
    // side, range 0.7-4.5 m; wider after 128 attempts) and kept if every pose of the window sees it in
    // front (|bearing| < 85 deg, range > 0.5 m and <= max(5.5 m, window span + 2 m)) and the rays
    // from the window's poses span >= kMinParallax. With information 1 per bearing and the
    // reference's constant damping 0.01 (slam/solver.cpp:16-17), a landmark's along-ray curvature is
    // about (1 - cos parallax) / range^2: at 4 deg and 7 m (the old generator's tail) it is 1e-4, a
    // hundredth of the damping, and such landmarks crept along their rays for hundreds of GN
    // iterations and crossed poses (bearing errors of pi); at >= 20 deg and <= 5 m it is >= 2.4e-3.
    // If no candidate qualifies, the one with the widest parallax among the visible ones is kept
    // (`min_parallax` of the world reports the minimum reached).
    constexpr double kMinParallax = 20.0 * bos::kPi / 180.0;
    const double cos_front = std::cos(85.0 * bos::kPi / 180.0);
    std::vector<double> lx(NL), ly(NL);
    std::vector<std::vector<int>> seen_by(NP);
    double min_par = 1e300;
    for (int j = 0; j < NL; ++j) {
        const Win& w = wins[j];
        const int L = w.last;
        const double side = (w.lane % 2) ? 1.0 : -1.0;
        const double span = std::hypot(gx[L] - gx[w.first], gy[L] - gy[w.first]);
        const double r_cap = std::max(5.5, span + 2.0);
        double best_x = 0, best_y = 0, best_par = -1;
        bool have_visible = false;
        for (int attempt = 0; attempt < 256; ++attempt) {
            const bool wide = attempt >= 128;
            const double beta = side * rng.uniform(20.0, 82.0) * (bos::kPi / 180.0);
            const double rho = rng.uniform(0.7, wide ? 7.0 : 4.5);
            const double bx = gx[L] + rho * std::cos(gth[L] + beta);
            const double by = gy[L] + rho * std::sin(gth[L] + beta);
            bool ok = true;
            double a0 = 0, amin = 0, amax = 0;
            for (int i = w.first; i <= L && ok; ++i) {
                const double dx = bx - gx[i], dy = by - gy[i];
                const double c = std::cos(gth[i]), s = std::sin(gth[i]);
                const double qx = c * dx + s * dy;
                const double r = std::hypot(dx, dy);
                ok = r > 0.5 && r <= r_cap && qx > cos_front * r;
                const double a = std::atan2(dy, dx);
                if (i == w.first) a0 = a;
                const double d = bos::normalized_angle<double>(a - a0);
                amin = std::min(amin, d);
                amax = std::max(amax, d);
            }
            if (!ok) continue;
            const double par = amax - amin;
            if (!have_visible || par > best_par) { best_x = bx; best_y = by; best_par = par; have_visible = true; }
            if (par >= kMinParallax) break;
        }
        if (!have_visible) return false;
        lx[j] = best_x;
        ly[j] = best_y;
        min_par = std::min(min_par, best_par);
        for (int i = w.first; i <= L; ++i) seen_by[i].push_back(j);
    }

    // ---- assemble the two states and the measurements (bearings listed per pose, like the dataset)
    out = SyntheticWorld();
    out.fixed_pose_id = 0;
    out.min_parallax = min_par;
    const int lm_id0 = NP;   // ids unique across poses and landmarks (g2o convention)
    double ix = gx[0], iy = gy[0], ith = gth[0];
    for (int i = 0; i < NP; ++i) {
        out.ground_truth.add_pose(gx[i], gy[i], gth[i], i);
        out.initial_guess.add_pose(ix, iy, ith, i);
        if (i + 1 < NP) {   // dead reckoning with the noisy odometry (predict_odometry inverted)
            const double c = std::cos(ith), s = std::sin(ith);
            ix += c * zx[i] - s * zy[i];
            iy += s * zx[i] + c * zy[i];
            ith = bos::normalized_angle<double>(ith + zt[i]);
        }
    }
    for (int j = 0; j < NL; ++j) out.ground_truth.add_landmark(lx[j], ly[j], lm_id0 + j);
    Mat3 om;
    om(0, 0) = p.odom_info_xy; om(1, 1) = p.odom_info_xy; om(2, 2) = p.odom_info_theta;
    om(0, 1) = om(0, 2) = om(1, 0) = om(1, 2) = om(2, 0) = om(2, 1) = 0;
    out.bearings.reserve((size_t)NP * K);
    for (int i = 0; i < NP; ++i) {
        std::vector<int>& v = seen_by[i];
        std::sort(v.begin(), v.end());
        const double c = std::cos(gth[i]), s = std::sin(gth[i]);
        for (int j : v) {
            const double qx = c * (lx[j] - gx[i]) + s * (ly[j] - gy[i]);
            const double qy = -s * (lx[j] - gx[i]) + c * (ly[j] - gy[i]);
            const double z = bos::normalized_angle<double>(std::atan2(qy, qx) + p.sigma_bearing * rng.normal());
            out.bearings.emplace_back(i, lm_id0 + j, z);
        }
        if (i + 1 < NP) out.odometry.emplace_back(i, i + 1, zx[i], zy[i], zt[i], om);
    }
    return true;
}

}  // namespace proj02
