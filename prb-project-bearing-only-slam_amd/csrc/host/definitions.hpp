// Host-side types mirroring framework/definitions.hpp of the reference without Eigen/OpenCV.
// NEPose (reference: Eigen::Isometry2f, definitions.hpp:17) is stored as (x, y, theta): the
// reference only ever reads the rotation through R itself or t2v's angle, and R <- dR R is
// theta <- theta + dtheta, so the explicit angle is an exact re-parametrisation.
#pragma once

#include <cmath>
#include <map>
#include <vector>

#include "bos_math.hpp"

namespace proj02 {

struct Vec2 {
    double x = 0, y = 0;
    Vec2() = default;
    Vec2(double x_, double y_) : x(x_), y(y_) {}
    Vec2 operator+(const Vec2& o) const { return {x + o.x, y + o.y}; }
    Vec2 operator-(const Vec2& o) const { return {x - o.x, y - o.y}; }
    Vec2& operator+=(const Vec2& o) { x += o.x; y += o.y; return *this; }
};

struct Vec3 {
    double x = 0, y = 0, z = 0;
    Vec3() = default;
    Vec3(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
    double operator()(int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};

struct Mat2 {
    double m[2][2] = {{1, 0}, {0, 1}};
    double operator()(int r, int c) const { return m[r][c]; }
    Mat2 transpose() const { Mat2 t; t.m[0][0] = m[0][0]; t.m[0][1] = m[1][0]; t.m[1][0] = m[0][1]; t.m[1][1] = m[1][1]; return t; }
    Vec2 operator*(const Vec2& v) const { return {m[0][0] * v.x + m[0][1] * v.y, m[1][0] * v.x + m[1][1] * v.y}; }
};

struct Mat3 {
    double m[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    double operator()(int r, int c) const { return m[r][c]; }
    double& operator()(int r, int c) { return m[r][c]; }
};

typedef Vec3 EPose;   // Euclidean pose (definitions.hpp:18)
typedef Vec2 LMPos;   // landmark position (definitions.hpp:20)

// Non-Euclidean pose (definitions.hpp:17), stored as translation + angle.
struct NEPose {
    double x = 0, y = 0, theta = 0;
    NEPose() = default;
    NEPose(double x_, double y_, double th_) : x(x_), y(y_), theta(th_) {}
    Mat2 rotation() const {
        Mat2 r;
        const double c = std::cos(theta), s = std::sin(theta);
        r.m[0][0] = c; r.m[0][1] = -s; r.m[1][0] = s; r.m[1][1] = c;
        return r;
    }
    Vec2 translation() const { return {x, y}; }
    // Isometry inverse: (R^T, -R^T t)
    Vec2 inverse_apply(const Vec2& p) const {
        const double c = std::cos(theta), s = std::sin(theta);
        const double itx = -(c * x + s * y), ity = -(-s * x + c * y);
        return {(c * p.x + s * p.y) + itx, (-s * p.x + c * p.y) + ity};
    }
};

typedef std::vector<NEPose> NEPoseVector;
typedef std::vector<LMPos> LMPosVector;
typedef std::map<int, int> AssociationMap;   // id -> stix (definitions.hpp:27)
typedef std::vector<int> AssociationVec;     // stix -> id (definitions.hpp:28)

// t2v (definitions.hpp:39-43)
inline EPose t2v(const NEPose& p) { return EPose(p.x, p.y, bos::smallest_angle<double>(p.theta)); }
// v2t (definitions.hpp:45-53)
inline NEPose v2t(const EPose& e) {
    return NEPose(e.x, e.y, bos::normalized_angle<double>(bos::smallest_angle<double>(e.z)));
}

}  // namespace proj02
