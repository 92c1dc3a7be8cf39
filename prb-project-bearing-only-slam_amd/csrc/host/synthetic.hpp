// Deterministic synthetic bearing-only SLAM worlds (SURVEY.md §8(d) generator spec).
#pragma once

#include <cstdint>
#include <vector>

#include "observation.hpp"
#include "state.hpp"

namespace proj02 {

struct SyntheticParams {
    int num_poses = 1000;
    int num_landmarks = 2000;
    int bearings_per_pose = 20;      // K: every pose observes exactly K landmarks
    uint64_t seed = 0xB05EED01ull;
    double world_extent = 0;         // side of the square world in m; 0 = auto (<= 1 km)
    double sigma_bearing = 0.003;    // rad (GT residual std of the shipped dataset)
    double odom_info_xy = 500.0;     // information, as EDGE_SE2 in the dataset
    double odom_info_theta = 5000.0;
};

struct SyntheticWorld {
    State ground_truth;               // GT poses + landmarks (VERTEX_XY)
    State initial_guess;              // dead-reckoned poses, no landmarks (triangulate them)
    BearingObservationVector bearings;
    OdometryObservationVector odometry;
    int fixed_pose_id = 0;
    double min_parallax = 0;          // smallest ray spread of any landmark (rad, ground truth)
};

// Trajectory: a bounded random walk (step 0.75-1 m, smooth heading changes, steered back inside
// the world). Landmarks: K "lanes"; lane k cuts the pose sequence into windows of >= 2 consecutive
// poses, one landmark per window, placed beside the window's last pose so every pose of the
// window sees it in front (|bearing| < 85 deg) and the window's rays span >= 20 deg wherever the
// geometry allows it (min_parallax reports what was reached). Each pose therefore observes exactly
// K landmarks, each landmark is observed >= 2 times with parallax, and (pose, landmark) pairs are
// unique.
// Returns false if the counts are infeasible (num_poses * K < 2 * num_landmarks, or
// num_landmarks < K).
bool make_synthetic(const SyntheticParams& p, SyntheticWorld& out);

}  // namespace proj02
