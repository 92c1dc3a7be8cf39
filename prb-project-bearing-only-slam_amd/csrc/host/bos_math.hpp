// Per-observation math of the GN hot path, shared by the HIP kernels (hip/linearize.hip) and the
// host façade (proj02::Solver::error_and_jacobian). Header-only, __host__ __device__.
//
// Conventions (reference torchipeppo/prb-project-bearing-only-slam):
//  - pose (x, y, theta) with R = [[c, -s], [s, c]], c = cos(theta), s = sin(theta); theta is the
//    angle t2v() would return (framework/definitions.hpp:39-43), kept wrapped to [-pi, pi).
//  - perturbation is left-multiplicative: X' = v2t(dx) * X (framework/state.hpp:11-13).
#pragma once

#include <cmath>

#include "det_atan2.hpp"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define BOS_HD __host__ __device__ __forceinline__
#else
#define BOS_HD inline
#endif

namespace bos {

// CV_PI / CV_2PI are double constants in the reference (slam/solver_jacobians.cpp:325-333).
constexpr double kPi = 3.1415926535897932384626433832795;
constexpr double k2Pi = 6.283185307179586476925286766559;

// Solver::normalized_angle (slam/solver_jacobians.cpp:325-333): [-pi, pi), compared in double.
// For a float, (double)a < -pi <=> a <= -(float)pi and (double)a >= pi <=> a >= (float)pi
// ((float)pi > pi), so the common in-range case skips the double arithmetic exactly.
template <typename T> BOS_HD T normalized_angle(T a) {
    if (sizeof(T) == 4 && a > -(T)3.14159274101257324 && a < (T)3.14159274101257324) return a;
    // Beyond |a| = 1e6, or not finite, the reference's loops below would run for ages or forever (an
    // infinite a; a float whose ulp exceeds 2 pi) — on the GPU a hung wave. Such an a (only ever seen
    // from a diverged iteration) is first brought near [-pi, pi) by subtracting the nearest multiple
    // of 2 pi (a few instructions, unlike fmod, which costs registers in every kernel that inlines
    // this); a non-finite one becomes NaN. Every |a| <= 1e6 takes exactly the reference's path.
    // Past |a| ~ 1e15 the quotient a / 2 pi is no longer exact and the remainder can be anything
    // (and a float of that size does not move by +-2 pi), so a remainder outside [-4 pi, 4 pi]
    // carries no angle: NaN, which the loops below pass through unchanged.
    if (!(std::fabs((double)a) <= 1e6)) {
        a = (T)((double)a - k2Pi * std::rint((double)a / k2Pi));
        if (!(std::fabs((double)a) <= 2.0 * k2Pi)) return (T)__builtin_nan("");
    }
    while ((double)a < -kPi) a = (T)((double)a + k2Pi);
    while ((double)a >= kPi) a = (T)((double)a - k2Pi);
    return a;
}

// Rotation2D::smallestAngle (framework/definitions.hpp:42; slam/solver_jacobians.cpp:18).
template <typename T> BOS_HD T smallest_angle(T a) {
    const T two_pi = (T)k2Pi, pi = (T)kPi;
    T t = std::fmod(a, two_pi);
    if (t > pi) t -= two_pi;
    else if (t < -pi) t += two_pi;
    return t;
}

// Bearing error only (slam/solver_jacobians.cpp:15-18, :301-305), with g = X^-1 l. Evaluated with
// plain IEEE operations (no FP contraction) and the portable atan2, so that the GPU lanes and the
// CPU oracle round identically: an error on the +-pi wrap flips sign on a last-ulp difference
// (det_atan2.hpp).
template <typename T> BOS_HD T bearing_error(T px, T py, T c, T s, T lx, T ly, T z, T& gx, T& gy) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    // g = X^-1 l = R^T l + (-R^T t), Isometry inverse (R^T, -R^T t) (:32, :302); explicit fma
    // (correctly rounded on both targets), the oracle evaluates the same expressions
    using std::fma;
    const T itx = -fma(c, px, s * py);
    const T ity = -fma(-s, px, c * py);
    gx = fma(c, lx, s * ly) + itx;
    gy = fma(-s, lx, c * ly) + ity;
    return normalized_angle<T>(det_atan2<T>(gy, gx) - z);                // :15, :18
}

// 1/x for the Jacobian's 1/|g|^2 (slam/solver_jacobians.cpp:35). Host: IEEE division. Device: the
// hardware reciprocal (fp32: v_rcp_f32, 1 ulp) or its Newton-refined fp64 form. The Jacobian
// tolerates an ulp; the error's atan2 (det_atan2.hpp) keeps its correctly rounded division.
template <typename T> BOS_HD T jac_recip(T x) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (sizeof(T) == 4) {
        return __builtin_amdgcn_rcpf(x);
    } else {
        T r = __builtin_amdgcn_rcp(x);
        r = fma(fma(-x, r, (T)1), r, r);
        return fma(fma(-x, r, (T)1), r, r);
    }
#else
    return (T)1 / x;
#endif
}

// Bearing error and analytic Jacobian (slam/solver_jacobians.cpp:9-95).
// Inputs: pose translation (px, py), cached c = cos(theta), s = sin(theta); landmark (lx, ly);
// measured z (smallestAngle-wrapped). Outputs: e = normalized(atan2(g) - z) and
// J = [dJ/dt_x, dJ/dt_y, dJ/dtheta, dJ/dl_x, dJ/dl_y]. Returns e.
template <typename T>
BOS_HD T bearing_error_jacobian(T px, T py, T c, T s, T lx, T ly, T z, T J[5]) {
    T gx, gy;
    const T e = bearing_error<T>(px, py, c, s, lx, ly, z, gx, gy);
    const T f = jac_recip<T>(gx * gx + gy * gy);                         // :35
    const T a0 = f * (-gy), a1 = f * gx;                                 // :47-48
    const T gth_x = c * ly + s * (-lx);                                  // R^T [[0,1],[-1,0]] l (:60)
    const T gth_y = -s * ly + c * (-lx);
    J[3] = a0 * c + a1 * (-s);                                           // R^T (:64)
    J[4] = a0 * s + a1 * c;
    J[0] = -J[3];                                                        // -R^T (:59): exactly minus
    J[1] = -J[4];                                                        // the landmark columns
    J[2] = a0 * gth_x + a1 * gth_y;
    return e;
}

// Odometry error and Jacobian (slam/solver_jacobians.cpp:97-168), J row-major 3x6 with columns
// [dx_s, dy_s, dth_s, dx_d, dy_d, dth_d]. The prediction is predict_odometry (:307-323).
template <typename T>
BOS_HD void odometry_error_jacobian(T xs, T ys, T ths, T cs, T ss, T xd, T yd, T thd, T z0, T z1, T z2,
                                    T e[3], T J[18]) {
    const T tx = xd - xs, ty = yd - ys;
    const T p0 = cs * tx + ss * ty;                                      // R_s^T (t_d - t_s) (:319)
    const T p1 = -ss * tx + cs * ty;
    const T p2 = normalized_angle<T>(thd - ths);                         // :321
    e[0] = p0 - z0;                                                      // :106
    e[1] = p1 - z1;
    e[2] = normalized_angle<T>(p2 - z2);                                 // :107
    J[0] = -cs; J[1] = -ss; J[2] = -ss * xd + cs * yd;                   // :137, :139
    J[3] = cs;  J[4] = ss;  J[5] = ss * xd - cs * yd;                    // :143, :145
    J[6] = ss;  J[7] = -cs; J[8] = -cs * xd - ss * yd;
    J[9] = -ss; J[10] = cs; J[11] = ss * yd + cs * xd;
    J[12] = 0;  J[13] = 0;  J[14] = (T)-1;                               // :140
    J[15] = 0;  J[16] = 0;  J[17] = (T)1;                                // :146
}

// Left-multiplicative box-plus (framework/state.hpp:11-13 + definitions.hpp:45-53):
// R <- dR R, t <- dR t + dt; theta kept wrapped.
template <typename T> BOS_HD void boxplus_pose(T& x, T& y, T& th, T dx, T dy, T dth) {
    const T c = cos(dth), s = sin(dth);
    const T nx = c * x - s * y + dx;
    const T ny = s * x + c * y + dy;
    x = nx;
    y = ny;
    th = normalized_angle<T>(th + dth);
}

}  // namespace bos
