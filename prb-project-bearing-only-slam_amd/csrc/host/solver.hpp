// proj02::Solver — C++ façade with the reference's API (slam/solver.hpp:21-92) over the C ABI
// (include/bos.h). step() runs on the GPU (HIP kernels + GPU sparse Cholesky); there is no CPU path.
// Like the reference's ctor (slam/solver.cpp:5-18) the constructor only copies and resolves ids
// (an unknown id throws std::out_of_range); the device handle is created by the first call that
// needs it (step, step_n, handle), so the per-observation API (predict_*, error_and_*jacobian) —
// what the reference's harness tests/solver_stuff.cpp calls — works on a host without a GPU.
//
// Differences to the reference, all documented in INTEGRATION.md:
//  - SparseMatrixXf Jacobians (Eigen) become small dense blocks with their column indices
//    (JacobianRow / Jacobian3), because Eigen is not available.
//  - values are double; precision of the GPU J+H build is chosen with bos_options::precision.
//  - errors are reported with std::runtime_error (the reference has no error path; an unknown id
//    still throws std::out_of_range from State).
#pragma once

#include <stdexcept>
#include <vector>

#include "../../../include/bos.h"
#include "observation.hpp"
#include "state.hpp"

namespace proj02 {

// 1 x N bearing Jacobian: 5 non-zeros at columns [3*pose_stix + 0..2, 3*NP + 2*lm_stix + 0..1]
struct JacobianRow {
    int cols[5] = {0, 0, 0, 0, 0};
    double values[5] = {0, 0, 0, 0, 0};
    double coeff(int col) const;
};

// 3 x N odometry Jacobian: columns [3*src + 0..2, 3*dst + 0..2]
struct Jacobian3 {
    int cols[6] = {0, 0, 0, 0, 0, 0};
    double values[3][6] = {};
    double coeff(int row, int col) const;
};

// The public `state` follows the device lazily (State / StateSource, state.hpp): step() leaves the
// new values on the device and the first read of `state` afterwards downloads them (fp64, bit for
// bit bos_get_state); a write to `state` between steps (non-const accessor, assignment,
// apply_boxplus) is uploaded before the next step, as the reference's step() reads its member.
class Solver final : private StateSource {
  public:
    State state;
    BearingObservationVector bearing_observations;
    OdometryObservationVector odometry_observations;

    // slam/solver.hpp:30. options == nullptr -> bos_default_options (fp64, sparse Cholesky)
    Solver(const State& state, const BearingObservationVector& bear_obs, const OdometryObservationVector& odom_obs,
           const int& fixed_pose_id, const bos_options* options = nullptr);
    ~Solver();
    Solver(const Solver&) = delete;
    Solver& operator=(const Solver&) = delete;

    void set_kernel_threshold(float kt);   // :33
    void set_damping_factor(float df);     // :34
    void step();                           // :36 — one GN iteration, state updated on return
    void step_n(int n);                    // n iterations, one state download at the end
    const bos_step_stats& last_stats() const { return stats_; }
    // The device handle (created on first use). The caller may step it directly: the public state
    // re-reads the device afterwards (host writes pending at this call are uploaded first).
    bos_solver* handle();

    // :38-44
    void error_and_jacobian(const State& state, const BearingObservation& obs, double& error, JacobianRow& J);
    void error_and_jacobian(const State& state, const OdometryObservation& obs, EPose& error, Jacobian3& J);
    void error_and_numerical_jacobian(const State& state, const BearingObservation& obs, double& error,
                                      JacobianRow& J, double epsilon = 1e-6);
    void error_and_numerical_jacobian(const State& state, const OdometryObservation& obs, EPose& error, Jacobian3& J,
                                      double epsilon = 1e-6);
    // :46-50
    double predict_bearing(const NEPose& pose, const LMPos& lm);
    EPose predict_odometry(const NEPose& src, const NEPose& dst);
    double normalized_angle(double angle);

  private:
    void pull_state(NEPoseVector& poses, LMPosVector& landmarks) override;
    void push_state();
    void before_step();
    bos_solver* ensure();   // creates the device handle on first use
    bos_solver* h_ = nullptr;
    int fixed_pose_id_;
    bos_step_stats stats_ = {};
    // the problem in the C ABI's SoA form (bos_create copies it)
    std::vector<double> pose_, lm_, bz_, bw_, oz_, om_;   // pose_ / lm_ also stage state transfers
    std::vector<int32_t> bp_, bl_, os_, od_;
    bool w1_ = true;
    bos_options opt_;
};

}  // namespace proj02
