// The C++ façade proj02::Solver (solver.hpp) driven the way the reference's executable drives
// proj02::Solver (executables/bearing_only_slam.cpp:93-99: solver.step() 50 times, then
// draw(solver.state)), for bench.py and the tests (include/bos_host.h).
#include <chrono>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "../../../include/bos_host.h"
#include "error.hpp"
#include "solver.hpp"

namespace {

int ffail(int code, const std::string& m) { return bos::set_error(code, m); }

// The reference's inputs from a C ABI problem: ids are the stix (every lookup still goes through
// the State's id maps, as in the reference).
struct FacadeInputs {
    proj02::State state;
    proj02::BearingObservationVector bearings;
    proj02::OdometryObservationVector odometry;
    int fixed_pose_id = 0;

    explicit FacadeInputs(const bos_problem* pb) : state(pb->num_poses, pb->num_landmarks) {
        for (int i = 0; i < pb->num_poses; ++i)
            state.add_pose(proj02::NEPose(pb->pose_xyt[3 * i], pb->pose_xyt[3 * i + 1], pb->pose_xyt[3 * i + 2]), i);
        for (int j = 0; j < pb->num_landmarks; ++j)
            state.add_landmark(pb->landmark_xy[2 * j], pb->landmark_xy[2 * j + 1], j);
        bearings.reserve((size_t)pb->num_bearings);
        for (int k = 0; k < pb->num_bearings; ++k)
            bearings.emplace_back(pb->bearing_pose[k], pb->bearing_landmark[k], pb->bearing_z[k],
                                  pb->bearing_omega ? pb->bearing_omega[k] : 1.0);
        odometry.reserve((size_t)pb->num_odometry);
        for (int k = 0; k < pb->num_odometry; ++k) {
            proj02::Mat3 om;
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) om(r, c) = pb->odom_omega[9 * k + 3 * r + c];
            odometry.emplace_back(pb->odom_src[k], pb->odom_dst[k], pb->odom_z[3 * k], pb->odom_z[3 * k + 1],
                                  pb->odom_z[3 * k + 2], om);
        }
        fixed_pose_id = pb->fixed_pose;
    }
};

// doubles of `st` that differ in their bits from (pose, lm)
int64_t count_mismatches(const proj02::State& st, const std::vector<double>& pose, const std::vector<double>& lm) {
    int64_t bad = 0;
    const proj02::NEPoseVector& P = st.poses_vec();
    const proj02::LMPosVector& L = st.landmarks_vec();
    auto diff = [](double a, double b) { return std::memcmp(&a, &b, sizeof(double)) != 0; };
    for (size_t i = 0; i < P.size(); ++i)
        bad += diff(P[i].x, pose[3 * i]) + diff(P[i].y, pose[3 * i + 1]) + diff(P[i].theta, pose[3 * i + 2]);
    for (size_t j = 0; j < L.size(); ++j) bad += diff(L[j].x, lm[2 * j]) + diff(L[j].y, lm[2 * j + 1]);
    return bad;
}

// the façade's state as read (a copy: a later solver.handle() marks the state stale and the next
// read would download it again)
void snapshot(const proj02::State& st, std::vector<double>& pose, std::vector<double>& lm) {
    const proj02::NEPoseVector& P = st.poses_vec();
    const proj02::LMPosVector& L = st.landmarks_vec();
    pose.resize(3 * P.size());
    lm.resize(2 * L.size());
    for (size_t i = 0; i < P.size(); ++i) {
        pose[3 * i] = P[i].x;
        pose[3 * i + 1] = P[i].y;
        pose[3 * i + 2] = P[i].theta;
    }
    for (size_t j = 0; j < L.size(); ++j) {
        lm[2 * j] = L[j].x;
        lm[2 * j + 1] = L[j].y;
    }
}

bool valid(const bos_problem* pb) {
    return pb && pb->num_poses > 0 && pb->num_landmarks > 0 && pb->pose_xyt && pb->landmark_xy &&
           (pb->num_bearings == 0 || (pb->bearing_pose && pb->bearing_landmark && pb->bearing_z)) &&
           (pb->num_odometry == 0 || (pb->odom_src && pb->odom_dst && pb->odom_z && pb->odom_omega));
}

}  // namespace

extern "C" {

int bos_time_facade_steps(const bos_problem* pb, const bos_options* options, int32_t n, double* ms_per_step,
                          double* ms_state_read, double* ms_per_step_capi, int64_t* mismatches) {
    if (!valid(pb) || n < 1 || !ms_per_step) return ffail(BOS_ERR_INVALID, "bad argument");
    try {
        FacadeInputs in(pb);
        proj02::Solver solver(in.state, in.bearings, in.odometry, in.fixed_pose_id, options);
        solver.step();                                  // handle, plan and the step's graphs: untimed
        (void)solver.state.get_pose_by_id(0);
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        for (int i = 0; i < n; ++i) solver.step();      // bearing_only_slam.cpp:95-98
        const auto t1 = clk::now();
        double sum = 0;                                 // draw(solver.state): one read of the state
        const proj02::State& shown = solver.state;
        for (const proj02::NEPose& p : shown.poses_vec()) sum += p.x;
        const auto t2 = clk::now();
        *ms_per_step = std::chrono::duration<double, std::milli>(t1 - t0).count() / n;
        if (ms_state_read) *ms_state_read = std::chrono::duration<double, std::milli>(t2 - t1).count() + 0 * sum;
        if (mismatches) {
            // the values that timed read produced, copied before solver.handle() (which marks the
            // façade's state stale, so reading it afterwards would download the device state again and
            // compare it with itself), against the device state
            std::vector<double> fpose, flm;
            snapshot(shown, fpose, flm);
            const size_t NP = (size_t)pb->num_poses, NL = (size_t)pb->num_landmarks;
            std::vector<double> pose(3 * NP), lm(2 * NL);
            if (fpose.size() != pose.size() || flm.size() != lm.size()) return ffail(BOS_ERR_INVALID, "facade state size");
            bos_solver* h = solver.handle();
            if (bos_get_state(h, pose.data(), lm.data()) != BOS_OK) return BOS_ERR_DEVICE;
            int64_t bad = 0;
            for (size_t i = 0; i < pose.size(); ++i) bad += std::memcmp(&fpose[i], &pose[i], sizeof(double)) != 0;
            for (size_t i = 0; i < lm.size(); ++i) bad += std::memcmp(&flm[i], &lm[i], sizeof(double)) != 0;
            *mismatches = bad;
        }
        if (ms_per_step_capi) {                         // the same handle, bos_step in a C loop
            const int rc = bos_time_steps(solver.handle(), n, ms_per_step_capi);
            if (rc != BOS_OK) return rc;
        }
    } catch (const std::exception& e) {
        return ffail(BOS_ERR_DEVICE, std::string("facade: ") + e.what());
    }
    return BOS_OK;
}

int bos_debug_facade_selftest(const bos_problem* pb, const bos_options* options, int32_t n, int64_t* mismatches) {
    if (!valid(pb) || n < 2 || !mismatches) return ffail(BOS_ERR_INVALID, "bad argument");
    bos_solver* r = nullptr;
    try {
        const size_t NP = (size_t)pb->num_poses, NL = (size_t)pb->num_landmarks;
        FacadeInputs in(pb);
        proj02::Solver solver(in.state, in.bearings, in.odometry, in.fixed_pose_id, options);
        bos_options opt;
        bos_default_options(&opt);
        if (options) opt = *options;
        if (bos_create(pb, &opt, &r) != BOS_OK) return BOS_ERR_DEVICE;
        std::vector<double> pose(3 * NP), lm(2 * NL);
        int64_t bad = 0;
        const int edit_at = n / 2;
        const int lm_id = (int)(NL / 3), pose_id = (int)(NP / 2);
        for (int i = 0; i < n; ++i) {
            if (i == edit_at) {
                // a caller's write between steps (the reference's next step() reads it): through the
                // façade's public state, and by hand on the C ABI handle
                solver.state.landmarks_vec()[(size_t)lm_id].x += 0.25;
                proj02::NEPose& q = solver.state.poses_vec()[(size_t)pose_id];
                q.theta = bos::normalized_angle<double>(q.theta + 0.01);
                if (bos_get_state(r, pose.data(), lm.data()) != BOS_OK) throw std::runtime_error(bos_last_error());
                lm[2 * (size_t)lm_id] += 0.25;
                pose[3 * (size_t)pose_id + 2] = bos::normalized_angle<double>(pose[3 * (size_t)pose_id + 2] + 0.01);
                if (bos_set_state(r, pose.data(), lm.data()) != BOS_OK) throw std::runtime_error(bos_last_error());
            }
            solver.step();
            if (bos_step(r, nullptr) != BOS_OK) throw std::runtime_error(bos_last_error());
            if (i % 7 == 3) {   // reads between steps (each after a step downloads the device state)
                const proj02::State& st = solver.state;
                if (bos_get_state(r, pose.data(), lm.data()) != BOS_OK) throw std::runtime_error(bos_last_error());
                bad += count_mismatches(st, pose, lm);
            }
        }
        const proj02::State& st = solver.state;
        // the façade's state against its own device state, then against the plain handle's
        if (bos_get_state(solver.handle(), pose.data(), lm.data()) != BOS_OK) throw std::runtime_error(bos_last_error());
        bad += count_mismatches(st, pose, lm);
        if (bos_get_state(r, pose.data(), lm.data()) != BOS_OK) throw std::runtime_error(bos_last_error());
        bad += count_mismatches(st, pose, lm);
        *mismatches = bad;
    } catch (const std::exception& e) {
        bos_destroy(r);
        return ffail(BOS_ERR_DEVICE, std::string("facade selftest: ") + e.what());
    }
    bos_destroy(r);
    return BOS_OK;
}

}  // extern "C"
