// The reference's numeric harness (tests/solver_stuff.cpp:17-163) run through the proj02::Solver
// façade (csrc/host/solver.hpp): predict_bearing known answers (:17-38), predict_odometry of the
// initial guess against each edge's measurement (:92-114, every edge instead of 8), and the
// analytic-vs-numerical Jacobian statistics for bearings on the ground truth (:41-89) and odometry
// on the initial guess (:117-163). No GPU: the façade creates its device handle only on step().
//
// Usage: jacobian_harness <initial_guess.g2o> <ground_truth.g2o> [--eps E]
// Prints one "key value" pair per line (parsed by tests/test_host.py).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../host/g2o_utils.hpp"
#include "../host/solver.hpp"
#include "../host/triangulation.hpp"

using namespace proj02;

int main(int argc, char** argv) {
    if (argc < 3) {
        std::printf("usage: jacobian_harness <initial_guess.g2o> <ground_truth.g2o> [--eps E]\n");
        return 1;
    }
    double eps = 1e-6;
    for (int i = 3; i + 1 < argc; ++i)
        if (!std::strcmp(argv[i], "--eps")) eps = std::atof(argv[++i]);
    State state_ig(300, 200), state_gt(300, 200);
    BearingObservationVector beobs_ig, beobs_gt;
    OdometryObservationVector odobs_ig, odobs_gt;
    int fixed_pose_id = -1, unused = -1;
    float b1 = 0, b2 = 0;
    if (parse_g2o(argv[1], state_ig, beobs_ig, odobs_ig, fixed_pose_id, b1) ||
        parse_g2o(argv[2], state_gt, beobs_gt, odobs_gt, unused, b2)) {
        std::printf("error cannot-read\n");
        return 1;
    }
    if (fixed_pose_id < 0) fixed_pose_id = state_ig.default_pose_id();   // solver_stuff.cpp:201-203
    triangulate_landmarks(state_ig, beobs_ig, false);                    // :206

    // predict_trust_check (:17-38), on the ground truth
    {
        const double PI = 3.14159265358979323846;
        OdometryObservationVector none;
        Solver s(state_gt, beobs_gt, none, fixed_pose_id);
        const struct { double th, lx, ly; } q[7] = {{0, 1, 0}, {0, 0, 1}, {0, -1, 0}, {0, 0, -1},
                                                     {0, 1, 1}, {PI / 2, 1, 1}, {PI, 1, 0}};
        for (int i = 0; i < 7; ++i)
            std::printf("kat%d %.17g\n", i, s.predict_bearing(v2t(EPose(0, 0, q[i].th)), LMPos(q[i].lx, q[i].ly)));
    }
    // jacobian_correctness_test (:41-89), bearings on the ground truth
    {
        OdometryObservationVector none;
        Solver s(state_gt, beobs_gt, none, fixed_pose_id);
        double hs = 0, hm = 0, ts = 0, tm = 0;
        for (const BearingObservation& obs : beobs_gt) {
            double e1, e2;
            JacobianRow a, n;
            s.error_and_jacobian(state_gt, obs, e1, a);
            s.error_and_numerical_jacobian(state_gt, obs, e2, n, eps);
            double sum = 0, mx = 0;
            for (int k = 0; k < 5; ++k) {
                const double d = std::fabs(a.values[k] - n.values[k]);
                sum += d;
                mx = std::max(mx, d);
            }
            hs = std::max(hs, sum);
            hm = std::max(hm, mx);
            ts += sum;
            tm += mx;
        }
        std::printf("bearing_highest_sum %.9g\nbearing_highest_max %.9g\nbearing_average_sum %.9g\n"
                    "bearing_average_max %.9g\nbearing_count %zu\n",
                    hs, hm, ts / beobs_gt.size(), tm / beobs_gt.size(), beobs_gt.size());
    }
    // predict_trust_check_odom (:92-114) on every edge of the initial guess, and
    // jacobian_correctness_test_odom (:117-163)
    {
        Solver s(state_ig, beobs_ig, odobs_ig, fixed_pose_id);
        double pmax = 0;
        for (const OdometryObservation& obs : odobs_ig) {
            const EPose p = s.predict_odometry(state_ig.get_pose_by_id(obs.get_source_id()),
                                               state_ig.get_pose_by_id(obs.get_dest_id()));
            const EPose z = obs.get_transformation();
            pmax = std::max({pmax, std::fabs(p.x - z.x), std::fabs(p.y - z.y),
                             std::fabs(s.normalized_angle(p.z - z.z))});
        }
        std::printf("odometry_predict_max_diff %.9g\nodometry_count %zu\n", pmax, odobs_ig.size());
        double hs = 0, hm = 0, ts = 0, tm = 0;
        for (const OdometryObservation& obs : odobs_ig) {
            EPose e1, e2;
            Jacobian3 a, n;
            s.error_and_jacobian(state_ig, obs, e1, a);
            s.error_and_numerical_jacobian(state_ig, obs, e2, n, eps);
            double sum = 0, mx = 0;
            for (int r = 0; r < 3; ++r)
                for (int k = 0; k < 6; ++k) {
                    const double d = std::fabs(a.values[r][k] - n.values[r][k]);
                    sum += d;
                    mx = std::max(mx, d);
                }
            hs = std::max(hs, sum);
            hm = std::max(hm, mx);
            ts += sum;
            tm += mx;
        }
        std::printf("odometry_highest_sum %.9g\nodometry_highest_max %.9g\nodometry_average_sum %.9g\n"
                    "odometry_average_max %.9g\n",
                    hs, hm, ts / odobs_ig.size(), tm / odobs_ig.size());
    }
    return 0;
}
