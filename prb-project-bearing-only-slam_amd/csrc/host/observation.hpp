// Measurement records — mirror of framework/observation.hpp:12-81.
#pragma once

#include <vector>

#include "definitions.hpp"

namespace proj02 {

// Bearing-only pose-landmark observation (observation.hpp:12-40). The bearing is stored as the
// angle of the reference's Rotation2f; get_bearing_angle() is its smallestAngle().
class BearingObservation {
  public:
    BearingObservation(const int& pose_id, const int& lm_id, const double& bearing, const double& omega = 1)
        : pose_id(pose_id), lm_id(lm_id), bearing(bearing), omega(omega) {}
    int get_pose_id() const { return pose_id; }
    int get_lm_id() const { return lm_id; }
    double get_bearing() const { return bearing; }
    double get_bearing_angle() const { return bos::smallest_angle<double>(bearing); }
    double get_omega() const { return omega; }

  private:
    int pose_id;
    int lm_id;
    double bearing;
    double omega;
};

// Odometry in the source pose's chart (observation.hpp:48-81): t_d = t_s + R_s z_t,
// theta_d = theta_s + z_theta (NOT an SE(2) composition, observation.hpp:43-47).
class OdometryObservation {
  public:
    OdometryObservation(const int& source_id, const int& dest_id, EPose transformation, Mat3 omega)
        : source_id(source_id), dest_id(dest_id), transformation(transformation), omega(omega) {}
    OdometryObservation(const int& source_id, const int& dest_id, double x, double y, double theta, Mat3 omega)
        : source_id(source_id), dest_id(dest_id), transformation(x, y, theta), omega(omega) {}
    int get_source_id() const { return source_id; }
    int get_dest_id() const { return dest_id; }
    EPose get_transformation() const { return transformation; }
    Mat3 get_omega() const { return omega; }

  private:
    int source_id;
    int dest_id;
    EPose transformation;
    Mat3 omega;
};

typedef std::vector<BearingObservation> BearingObservationVector;
typedef std::vector<OdometryObservation> OdometryObservationVector;
typedef std::map<int, BearingObservationVector> BearingObservationsByLandmarkId;  // observation.hpp:81

}  // namespace proj02
