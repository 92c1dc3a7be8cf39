#include "solver.hpp"

#include <string>

#include "bos_math.hpp"

namespace proj02 {

namespace {
void check(int rc, const char* what) {
    if (rc != BOS_OK) throw std::runtime_error(std::string(what) + ": " + bos_last_error());
}
}  // namespace

double JacobianRow::coeff(int col) const {
    double v = 0;
    for (int k = 0; k < 5; ++k)
        if (cols[k] == col) v += values[k];
    return v;
}

double Jacobian3::coeff(int row, int col) const {
    double v = 0;
    for (int k = 0; k < 6; ++k)
        if (cols[k] == col) v += values[row][k];
    return v;
}

Solver::Solver(const State& st, const BearingObservationVector& bear_obs, const OdometryObservationVector& odom_obs,
               const int& fixed_pose_id, const bos_options* options)
    : state(st), bearing_observations(bear_obs), odometry_observations(odom_obs), fixed_pose_id_(fixed_pose_id) {
    // SoA problem in stix order; ids resolved once (std::map::at throws on unknown ids like the reference)
    const int NP = state.number_of_poses(), NL = state.number_of_landmarks();
    pose_.resize(3 * (size_t)NP);
    lm_.resize(2 * (size_t)NL);
    const size_t Mb = bearing_observations.size(), Mo = odometry_observations.size();
    bp_.resize(Mb); bl_.resize(Mb); os_.resize(Mo); od_.resize(Mo);
    bz_.resize(Mb); bw_.resize(Mb); oz_.resize(3 * Mo); om_.resize(9 * Mo);
    for (size_t k = 0; k < Mb; ++k) {
        const BearingObservation& o = bearing_observations[k];
        bp_[k] = state.pose_stix(o.get_pose_id());
        bl_[k] = state.landmark_stix(o.get_lm_id());
        bz_[k] = o.get_bearing_angle();
        bw_[k] = o.get_omega();
        w1_ = w1_ && bw_[k] == 1.0;
    }
    for (size_t k = 0; k < Mo; ++k) {
        const OdometryObservation& o = odometry_observations[k];
        os_[k] = state.pose_stix(o.get_source_id());
        od_[k] = state.pose_stix(o.get_dest_id());
        const EPose z = o.get_transformation();
        oz_[3 * k] = z.x; oz_[3 * k + 1] = z.y; oz_[3 * k + 2] = z.z;
        const Mat3 m = o.get_omega();
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) om_[9 * k + 3 * r + c] = m(r, c);
    }
    (void)state.pose_stix(fixed_pose_id);   // unknown fixed pose id: std::out_of_range now, like the reference
    bos_default_options(&opt_);
    if (options) opt_ = *options;
}

namespace {
// the host state in the C ABI's SoA form (const accessors: reading is not a write)
void stage_state(const State& st, std::vector<double>& pose, std::vector<double>& lm) {
    const NEPoseVector& P = st.poses_vec();
    const LMPosVector& L = st.landmarks_vec();
    if (pose.size() != 3 * P.size() || lm.size() != 2 * L.size())
        throw std::runtime_error("proj02::Solver: poses or landmarks were added to solver.state after construction");
    for (size_t i = 0; i < P.size(); ++i) { pose[3 * i] = P[i].x; pose[3 * i + 1] = P[i].y; pose[3 * i + 2] = P[i].theta; }
    for (size_t j = 0; j < L.size(); ++j) { lm[2 * j] = L[j].x; lm[2 * j + 1] = L[j].y; }
}
}  // namespace

bos_solver* Solver::ensure() {
    if (h_) return h_;
    // the public state as it is now (the reference's step() reads its member state)
    stage_state(state, pose_, lm_);
    bos_problem pb;
    pb.num_poses = state.number_of_poses(); pb.num_landmarks = state.number_of_landmarks();
    pb.num_bearings = (int32_t)bz_.size(); pb.num_odometry = (int32_t)os_.size();
    pb.pose_xyt = pose_.data(); pb.landmark_xy = lm_.data();
    pb.bearing_pose = bp_.data(); pb.bearing_landmark = bl_.data(); pb.bearing_z = bz_.data();
    pb.bearing_omega = w1_ ? nullptr : bw_.data();
    pb.odom_src = os_.data(); pb.odom_dst = od_.data(); pb.odom_z = oz_.data(); pb.odom_omega = om_.data();
    pb.fixed_pose = state.pose_stix(fixed_pose_id_);
    check(bos_create(&pb, &opt_, &h_), "bos_create");
    state.attach_source(this);   // from here on the device holds the current values
    return h_;
}

Solver::~Solver() { bos_destroy(h_); }

void Solver::set_kernel_threshold(float kt) {
    opt_.kernel_threshold = kt;
    if (h_) check(bos_set_kernel_threshold(h_, kt), "set_kernel_threshold");
}
void Solver::set_damping_factor(float df) {
    opt_.damping = df;
    if (h_) check(bos_set_damping_factor(h_, df), "set_damping_factor");
}

// StateSource: the device's fp64 state, copied as is (bit for bit bos_get_state)
void Solver::pull_state(NEPoseVector& poses, LMPosVector& landmarks) {
    check(bos_get_state(h_, pose_.data(), lm_.data()), "bos_get_state");
    for (size_t i = 0; i < poses.size(); ++i) poses[i] = NEPose(pose_[3 * i], pose_[3 * i + 1], pose_[3 * i + 2]);
    for (size_t j = 0; j < landmarks.size(); ++j) landmarks[j] = LMPos(lm_[2 * j], lm_[2 * j + 1]);
}

void Solver::push_state() {
    stage_state(state, pose_, lm_);
    check(bos_set_state(h_, pose_.data(), lm_.data()), "bos_set_state");
}

void Solver::before_step() {
    const bool fresh = h_ == nullptr;
    ensure();
    // a write to `state` since the last step (or, for a fresh handle, since bos_create copied it)
    if (state.take_host_writes() && !fresh) push_state();
}

bos_solver* Solver::handle() {
    before_step();
    state.mark_stale();
    return h_;
}

void Solver::step() {
    before_step();
    const int rc = bos_step(h_, &stats_);
    state.mark_stale();   // even a failed step may have moved nothing or everything: re-read
    check(rc, "bos_step");
}

void Solver::step_n(int n) {
    before_step();
    const int rc = bos_step_n(h_, n, &stats_);
    state.mark_stale();
    check(rc, "bos_step_n");
}

double Solver::normalized_angle(double a) { return bos::normalized_angle<double>(a); }

double Solver::predict_bearing(const NEPose& pose, const LMPos& lm) {
    const Vec2 g = pose.inverse_apply(lm);
    return std::atan2(g.y, g.x);
}

EPose Solver::predict_odometry(const NEPose& src, const NEPose& dst) {
    const EPose es = t2v(src), ed = t2v(dst);
    const double c = std::cos(src.theta), s = std::sin(src.theta);
    const double tx = ed.x - es.x, ty = ed.y - es.y;
    return EPose(c * tx + s * ty, -s * tx + c * ty, normalized_angle(ed.z - es.z));
}

void Solver::error_and_jacobian(const State& st, const BearingObservation& obs, double& error, JacobianRow& J) {
    const NEPose p = st.get_pose_by_id(obs.get_pose_id());
    const LMPos l = st.get_landmark_by_id(obs.get_lm_id());
    error = bos::bearing_error_jacobian<double>(p.x, p.y, std::cos(p.theta), std::sin(p.theta), l.x, l.y,
                                                obs.get_bearing_angle(), J.values);
    const int pc = 3 * st.pose_stix(obs.get_pose_id());
    const int lc = 3 * st.number_of_poses() + 2 * st.landmark_stix(obs.get_lm_id());
    const int cols[5] = {pc, pc + 1, pc + 2, lc, lc + 1};
    for (int k = 0; k < 5; ++k) J.cols[k] = cols[k];
}

void Solver::error_and_jacobian(const State& st, const OdometryObservation& obs, EPose& error, Jacobian3& J) {
    const NEPose s = st.get_pose_by_id(obs.get_source_id());
    const NEPose d = st.get_pose_by_id(obs.get_dest_id());
    const EPose z = obs.get_transformation();
    double e[3], JJ[18];
    bos::odometry_error_jacobian<double>(s.x, s.y, s.theta, std::cos(s.theta), std::sin(s.theta), d.x, d.y, d.theta,
                                         z.x, z.y, z.z, e, JJ);
    error = EPose(e[0], e[1], e[2]);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 6; ++c) J.values[r][c] = JJ[6 * r + c];
    const int sc = 3 * st.pose_stix(obs.get_source_id()), dc = 3 * st.pose_stix(obs.get_dest_id());
    const int cols[6] = {sc, sc + 1, sc + 2, dc, dc + 1, dc + 2};
    for (int k = 0; k < 6; ++k) J.cols[k] = cols[k];
}

// slam/solver_jacobians.cpp:170-222 (central differences through boxplus)
void Solver::error_and_numerical_jacobian(const State& st, const BearingObservation& obs, double& error,
                                          JacobianRow& J, double eps) {
    const NEPose p = st.get_pose_by_id(obs.get_pose_id());
    const LMPos l = st.get_landmark_by_id(obs.get_lm_id());
    const double z = obs.get_bearing_angle();
    auto err = [&](const EPose& dp, const LMPos& dl) {
        const NEPose q = boxplus(p, dp);
        return normalized_angle(predict_bearing(q, l + dl) - z);
    };
    error = err(EPose(0, 0, 0), LMPos(0, 0));
    const EPose sel_p[3] = {EPose(1, 0, 0), EPose(0, 1, 0), EPose(0, 0, 1)};
    for (int k = 0; k < 3; ++k) {
        const EPose d(eps * sel_p[k].x, eps * sel_p[k].y, eps * sel_p[k].z), m(-d.x, -d.y, -d.z);
        J.values[k] = (err(d, LMPos(0, 0)) - err(m, LMPos(0, 0))) / (2 * eps);
    }
    J.values[3] = (err(EPose(0, 0, 0), LMPos(eps, 0)) - err(EPose(0, 0, 0), LMPos(-eps, 0))) / (2 * eps);
    J.values[4] = (err(EPose(0, 0, 0), LMPos(0, eps)) - err(EPose(0, 0, 0), LMPos(0, -eps))) / (2 * eps);
    const int pc = 3 * st.pose_stix(obs.get_pose_id());
    const int lc = 3 * st.number_of_poses() + 2 * st.landmark_stix(obs.get_lm_id());
    const int cols[5] = {pc, pc + 1, pc + 2, lc, lc + 1};
    for (int k = 0; k < 5; ++k) J.cols[k] = cols[k];
}

// slam/solver_jacobians.cpp:224-299
void Solver::error_and_numerical_jacobian(const State& st, const OdometryObservation& obs, EPose& error, Jacobian3& J,
                                          double eps) {
    const NEPose s = st.get_pose_by_id(obs.get_source_id());
    const NEPose d = st.get_pose_by_id(obs.get_dest_id());
    const EPose z = obs.get_transformation();
    auto err = [&](const EPose& ds, const EPose& dd) {
        const EPose pr = predict_odometry(boxplus(s, ds), boxplus(d, dd));
        return EPose(pr.x - z.x, pr.y - z.y, normalized_angle(pr.z - z.z));
    };
    error = err(EPose(0, 0, 0), EPose(0, 0, 0));
    for (int k = 0; k < 6; ++k) {
        double v[3] = {0, 0, 0};
        v[k % 3] = eps;
        const EPose dp(v[0], v[1], v[2]), dm(-v[0], -v[1], -v[2]), zero(0, 0, 0);
        const EPose a = k < 3 ? err(dp, zero) : err(zero, dp);
        const EPose b = k < 3 ? err(dm, zero) : err(zero, dm);
        J.values[0][k] = (a.x - b.x) / (2 * eps);
        J.values[1][k] = (a.y - b.y) / (2 * eps);
        J.values[2][k] = (a.z - b.z) / (2 * eps);
    }
    const int sc = 3 * st.pose_stix(obs.get_source_id()), dc = 3 * st.pose_stix(obs.get_dest_id());
    const int cols[6] = {sc, sc + 1, sc + 2, dc, dc + 1, dc + 2};
    for (int k = 0; k < 6; ++k) J.cols[k] = cols[k];
}

}  // namespace proj02
