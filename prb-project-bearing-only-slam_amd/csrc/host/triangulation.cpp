#include "triangulation.hpp"

#include <algorithm>
#include <cmath>
#include <iostream>
#include <limits>
#include <thread>
#include <vector>

namespace proj02 {

BearingObservationsByLandmarkId subdivide_bearings_by_landmark_id(const BearingObservationVector& all) {
    BearingObservationsByLandmarkId m;
    for (const BearingObservation& o : all) m[o.get_lm_id()].push_back(o);
    return m;
}

// Two-column least squares by column-pivoted modified Gram-Schmidt (with one re-orthogonalisation).
// Pivot = the column of larger norm (Eigen ColPivHouseholderQR takes the first maximal norm);
// number of pivots follows Eigen's nonzeroPivots() rule, so a 1-row or exactly rank-deficient
// system returns the basic solution: pivot component solved, the other component 0.
LMPos triangulate_one_landmark(const State& state, const BearingObservationVector& obs, bool verbose) {
    const size_t M = obs.size();
    if (M == 1 && verbose) {
        std::cout << "Landmark no. " << obs[0].get_lm_id() << " only has one observation.\n";
        std::cout << "  Bearing-only SLAM won't be able to locate it properly." << std::endl;
    }
    std::vector<double> a0(M), a1(M), r(M);
    double n0 = 0, n1 = 0;
    for (size_t i = 0; i < M; ++i) {
        const EPose p = t2v(state.get_pose_by_id(obs[i].get_pose_id()));
        const double ang = p.z + obs[i].get_bearing_angle();
        const double s = std::sin(ang), c = std::cos(ang);
        a0[i] = s;
        a1[i] = -c;
        r[i] = s * p.x - c * p.y;
        n0 += a0[i] * a0[i];
        n1 += a1[i] * a1[i];
    }
    const bool swap = n1 > n0;
    const std::vector<double>& c0 = swap ? a1 : a0;
    std::vector<double> c1 = swap ? a0 : a1;
    const double r00 = std::sqrt(std::max(n0, n1));
    if (r00 == 0.0) return LMPos(0, 0);
    std::vector<double> q0(M);
    for (size_t i = 0; i < M; ++i) q0[i] = c0[i] / r00;
    double qb0 = 0;
    for (size_t i = 0; i < M; ++i) qb0 += q0[i] * r[i];
    double x_piv = 0, x_oth = 0;
    bool rank2 = false;
    double r01 = 0, r11 = 0, qb1 = 0;
    if (M >= 2) {
        for (int pass = 0; pass < 2; ++pass) {       // MGS + one re-orthogonalisation
            double d = 0;
            for (size_t i = 0; i < M; ++i) d += q0[i] * c1[i];
            for (size_t i = 0; i < M; ++i) c1[i] -= d * q0[i];
            r01 += d;
        }
        double rem = 0;
        for (size_t i = 0; i < M; ++i) rem += c1[i] * c1[i];
        const double eps = std::numeric_limits<double>::epsilon();
        const double thr = (r00 * eps) * (r00 * eps) / (double)M * (double)(M - 1);
        if (!(rem < thr)) {
            rank2 = true;
            r11 = std::sqrt(rem);
            for (size_t i = 0; i < M; ++i) qb1 += (c1[i] / r11) * r[i];
        }
    }
    if (rank2) {
        x_oth = qb1 / r11;
        x_piv = (qb0 - r01 * x_oth) / r00;
    } else {
        x_piv = qb0 / r00;
        x_oth = 0;
    }
    return swap ? LMPos(x_oth, x_piv) : LMPos(x_piv, x_oth);
}

// Groups in ascending id order with the bearings of a group in file order (the std::map of
// subdivide_bearings_by_landmark_id), solved in parallel, added to the state in id order.
void triangulate_landmarks(State& state, const BearingObservationVector& observations, bool verbose) {
    std::vector<int32_t> order(observations.size());
    for (size_t k = 0; k < order.size(); ++k) order[k] = (int32_t)k;
    std::stable_sort(order.begin(), order.end(),
                     [&](int32_t a, int32_t b) { return observations[a].get_lm_id() < observations[b].get_lm_id(); });
    std::vector<size_t> gptr;
    for (size_t i = 0; i < order.size(); ++i)
        if (i == 0 || observations[order[i]].get_lm_id() != observations[order[i - 1]].get_lm_id()) gptr.push_back(i);
    gptr.push_back(order.size());
    const size_t ng = gptr.size() - 1;
    std::vector<LMPos> out(ng);
    auto solve = [&](size_t g0, size_t g1) {
        BearingObservationVector grp;
        for (size_t g = g0; g < g1; ++g) {
            grp.clear();
            for (size_t i = gptr[g]; i < gptr[g + 1]; ++i) grp.push_back(observations[order[i]]);
            out[g] = triangulate_one_landmark(state, grp, verbose);
        }
    };
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = verbose ? 1 : std::min<size_t>(std::min(16u, hw), std::max<size_t>(1, ng / 4096));
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; ++t) th.emplace_back(solve, ng * t / nt, ng * (t + 1) / nt);
    solve(0, ng / nt);
    for (std::thread& t : th) t.join();
    for (size_t g = 0; g < ng; ++g) state.add_landmark(out[g], observations[order[gptr[g]]].get_lm_id());
}

}  // namespace proj02
