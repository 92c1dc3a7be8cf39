// proj02::State — mirror of framework/state.hpp:15-54 (no drawing; OpenCV is out of scope).
#pragma once

#include <atomic>
#include <mutex>
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

class State;

// Where a State's current values live when it is not the host vectors: proj02::Solver registers
// itself for its public `state` member, whose values after a step are on the device. The State
// then refreshes its vectors from the source on the first read after a step (lazy: a caller that
// steps 50 times and reads once pays one download, not 50), and remembers a write through a
// non-const accessor so that the next step uploads the host values first (the reference's step()
// reads its member state, slam/solver.cpp:27-97).
class StateSource {
  public:
    virtual void pull_state(NEPoseVector& poses, LMPosVector& landmarks) = 0;

  protected:
    ~StateSource() = default;
};

class State {
  public:
    State(int expected_states = 300, int expected_landmarks = 200);
    // A copy is a plain host State: the source's current values, no source attached.
    State(const State& o);
    State& operator=(const State& o);

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

    // direct stix-order access (the reference keeps these private; the C ABI needs them). A
    // reference from the non-const overloads counts as a write and is valid until the next step.
    const NEPoseVector& poses_vec() const { materialize(); return poses; }
    const LMPosVector& landmarks_vec() const { materialize(); return landmarks; }
    NEPoseVector& poses_vec() { touch(); return poses; }
    LMPosVector& landmarks_vec() { touch(); return landmarks; }
    const AssociationVec& pose_ids() const { return pose_stix_to_id; }
    const AssociationVec& landmark_ids() const { return lm_stix_to_id; }

    // Source protocol (proj02::Solver): attach once; mark_stale after every step; take_host_writes
    // before a step returns (and clears) whether the host values were written since.
    void attach_source(StateSource* src) { source_ = src; stale_ = false; host_written_ = false; }
    void mark_stale() { stale_ = source_ != nullptr; }
    bool take_host_writes() { const bool w = host_written_; host_written_ = false; return w; }

  private:
    // The first read after a step downloads the values. Const reads from several threads are safe
    // (one of them downloads under the lock; the others wait for it), and stale_ is cleared only
    // once the download succeeded, so a read whose download throws leaves the next read to retry
    // instead of returning the pre-step values. A write (non-const accessor) while
    // another thread reads is a data race, as on any std::vector.
    void materialize() const {
        if (!stale_) return;
        std::lock_guard<std::mutex> g(pull_lock_.m);
        if (stale_) {
            source_->pull_state(poses, landmarks);
            stale_ = false;
        }
    }
    void touch() { materialize(); host_written_ = true; }

    // a mutex that copies and assigns as a fresh one (State itself is copyable, as the reference's)
    struct PullLock {
        std::mutex m;
        PullLock() = default;
        PullLock(const PullLock&) {}
        PullLock& operator=(const PullLock&) { return *this; }
    };
    mutable PullLock pull_lock_;
    StateSource* source_ = nullptr;
    mutable std::atomic<bool> stale_{false};
    bool host_written_ = false;
    // mutable: a const read may refresh them from the source
    mutable NEPoseVector poses;
    mutable LMPosVector landmarks;
    AssociationMap pose_id_to_stix;
    AssociationVec pose_stix_to_id;
    AssociationMap lm_id_to_stix;
    AssociationVec lm_stix_to_id;
};

}  // namespace proj02
