#include "state.hpp"

#include <cstdio>
#include <iostream>
#include <stdexcept>

namespace proj02 {

State::State(int expected_states, int expected_landmarks) {
    poses.reserve(expected_states > 0 ? expected_states : 0);
    landmarks.reserve(expected_landmarks > 0 ? expected_landmarks : 0);
    pose_stix_to_id.reserve(expected_states > 0 ? expected_states : 0);
    lm_stix_to_id.reserve(expected_landmarks > 0 ? expected_landmarks : 0);
}

State::State(const State& o)
    : poses(o.poses_vec()), landmarks(o.landmarks_vec()), pose_id_to_stix(o.pose_id_to_stix),
      pose_stix_to_id(o.pose_stix_to_id), lm_id_to_stix(o.lm_id_to_stix), lm_stix_to_id(o.lm_stix_to_id) {}

State& State::operator=(const State& o) {
    if (this == &o) return *this;
    touch();   // replaced on the host: a source's next step uploads it
    poses = o.poses_vec();
    landmarks = o.landmarks_vec();
    pose_id_to_stix = o.pose_id_to_stix;
    pose_stix_to_id = o.pose_stix_to_id;
    lm_id_to_stix = o.lm_id_to_stix;
    lm_stix_to_id = o.lm_stix_to_id;
    return *this;
}

void State::add_pose(const NEPose& pose, const int& id) {
    touch();
    poses.push_back(pose);
    pose_id_to_stix[id] = (int)poses.size() - 1;   // a repeated id re-points the map (state.cpp:23)
    pose_stix_to_id.push_back(id);
}

void State::add_pose(const double& x, const double& y, const double& theta, const int& id) {
    add_pose(v2t(EPose(x, y, theta)), id);
}

void State::add_landmark(const LMPos& lm, const int& id) {
    touch();
    landmarks.push_back(lm);
    lm_id_to_stix[id] = (int)landmarks.size() - 1;
    lm_stix_to_id.push_back(id);
}

void State::add_landmark(const double& x, const double& y, const int& id) { add_landmark(LMPos(x, y), id); }

NEPose State::get_pose_by_id(const int& id) const { return poses_vec()[pose_id_to_stix.at(id)]; }
LMPos State::get_landmark_by_id(const int& id) const { return landmarks_vec()[lm_id_to_stix.at(id)]; }

int State::number_of_poses() const { return (int)poses.size(); }
int State::number_of_landmarks() const { return (int)landmarks.size(); }

int State::pose_stix(const int& id) const { return pose_id_to_stix.at(id); }
int State::landmark_stix(const int& id) const { return lm_id_to_stix.at(id); }

int State::default_pose_id() {
    if (pose_stix_to_id.empty()) throw std::out_of_range("State::default_pose_id: no poses");
    return pose_stix_to_id[0];
}

void State::apply_boxplus(const std::vector<double>& dx) {
    touch();
    const size_t NP = poses.size(), NL = landmarks.size();
    if (dx.size() < 3 * NP + 2 * NL) throw std::invalid_argument("State::apply_boxplus: dx too short");
    for (size_t i = 0; i < NP; ++i) poses[i] = boxplus(poses[i], EPose(dx[3 * i], dx[3 * i + 1], dx[3 * i + 2]));
    for (size_t j = 0; j < NL; ++j) landmarks[j] += LMPos(dx[3 * NP + 2 * j], dx[3 * NP + 2 * j + 1]);
}

void State::print_full_vector() {
    materialize();
    std::cout << "State:";
    for (const NEPose& p : poses) {
        const EPose e = t2v(p);
        std::cout << ' ' << e.x << ' ' << e.y << ' ' << e.z;
    }
    for (const LMPos& l : landmarks) std::cout << ' ' << l.x << ' ' << l.y;
    std::cout << std::endl;
}

}  // namespace proj02
