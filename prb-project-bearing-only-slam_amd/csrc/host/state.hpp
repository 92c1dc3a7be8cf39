// proj02::State — mirror of framework/state.hpp:15-54 (no drawing; OpenCV is out of scope).
#pragma once

#include <string>
#include <vector>

#include "definitions.hpp"

namespace proj02 {

// boxplus (framework/state.hpp:11-13): v2t(dx) * X
inline NEPose boxplus(const NEPose& X, const EPose& dx) {
    NEPose r = X;
    bos::boxplus_pose<double>(r.x, r.y, r.theta, dx.x, dx.y, dx.z);
    return r;
}

class State {
  public:
    State(int expected_states = 300, int expected_landmarks = 200);

    void add_pose(const NEPose& pose, const int& id);                          // state.cpp:20-25
    void add_pose(const double& x, const double& y, const double& theta, const int& id);  // :27-30
    void add_landmark(const LMPos& lm, const int& id);                          // :32-37
    void add_landmark(const double& x, const double& y, const int& id);         // :39-41

    // std::out_of_range on an unknown id, like std::map::at (state.cpp:43-49)
    NEPose get_pose_by_id(const int& id) const;
    LMPos get_landmark_by_id(const int& id) const;

    int number_of_poses() const;
    int number_of_landmarks() const;

    int pose_stix(const int& id) const;                                         // state.cpp:58-60
    int landmark_stix(const int& id) const;                                     // :61-63
    int default_pose_id();                                                      // :65-67

    // state.cpp:69-80, dx in the reference dof order (poses 3*stix, landmarks 3*NP + 2*stix)
    void apply_boxplus(const std::vector<double>& delta_x);
    void print_full_vector();                                                   // :82-93

    // direct stix-order access (the reference keeps these private; the C ABI needs them)
    const NEPoseVector& poses_vec() const { return poses; }
    const LMPosVector& landmarks_vec() const { return landmarks; }
    NEPoseVector& poses_vec() { return poses; }
    LMPosVector& landmarks_vec() { return landmarks; }
    const AssociationVec& pose_ids() const { return pose_stix_to_id; }
    const AssociationVec& landmark_ids() const { return lm_stix_to_id; }

  private:
    NEPoseVector poses;
    LMPosVector landmarks;
    AssociationMap pose_id_to_stix;
    AssociationVec pose_stix_to_id;
    AssociationMap lm_id_to_stix;
    AssociationVec lm_stix_to_id;
};

}  // namespace proj02
