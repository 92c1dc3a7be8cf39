// =====================================================================================
//  ORACLE — TEST INFRASTRUCTURE ONLY.
//
//  CPU restatement of the reference's Gauss-Newton hot path for 2-D bearing-only SLAM
//  (torchipeppo/prb-project-bearing-only-slam). Only tests/, __graft_entry__.smoke() and
//  bench.py's cpu_baseline leg may load this library, and only as the checker / the
//  timed CPU baseline. The product (libbos.so, HIP) never links or calls it.
//
//  Parity pinning (see oracle/README and DESIGN.md §Oracle): the reference cannot be
//  built here (Eigen3 / OpenCV absent), so this restatement is pinned by the reference's
//  own known-answer checks (tests/solver_stuff.cpp:25-38 predict_bearing KATs, :93-114
//  predict_odometry on the IG), its Jacobian-check harness (:42-89, :117-163), the README
//  convergence claim (README.md:22-24) and by an independent NumPy restatement committed
//  as tests/golden/make_golden.py.
//
//  Every function below cites the reference file:line it restates. Scalar type T is
//  float (reference semantics: every Eigen type in framework/definitions.hpp:17-37 is
//  float) or double (the build's fp64 parity mode).
// =====================================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>
#include <map>
#include <limits>
#ifdef _OPENMP
#include <omp.h>
#endif

// The one libm substitute shared with the product: a portable atan2 (fdlibm-style reduction,
// plain IEEE operations; <= 1 ulp vs glibc, tests/test_oracle.py). Bearings whose error sits on
// the +-pi wrap (the reference's single-observation landmarks) flip sign on a last-ulp difference
// of atan2, so for the reference dataset the oracle and the GPU path must round identically. It is
// used only in the bit-reproducing form (bearing_g below); the literal form (oracle_set_literal)
// uses libm's atan2 and Eigen's product sums and shares no code with the product — the synthetic
// worlds' parity tests run in it. This file is compiled with -ffp-contract=off.
#include "../prb-project-bearing-only-slam_amd/csrc/host/det_atan2.hpp"

namespace {

// OpenCV's CV_PI / CV_2PI are double constants; the reference compares a float against them
// (slam/solver_jacobians.cpp:325-333), so the comparison and the add happen in double.
constexpr double CV_PI_D = 3.1415926535897932384626433832795;
constexpr double CV_2PI_D = 6.283185307179586476925286766559;

// Solver::normalized_angle — slam/solver_jacobians.cpp:325-333. Half-open [-pi, pi).
// The reference's loops, run as written whenever they end: a step that leaves the angle unchanged
// (its ulp is past 4 pi) is where the reference never ends, and gives NaN, as does a non-finite
// angle. One bound for the oracle's own running time: an fp64 |angle| > 1e9 (the loops would take
// more than 1.6e8 steps) is reduced by the nearest multiple of 2 pi first, the product's rule
// (bos_math.hpp) — that range is parity-unpinned (tests/test_oracle.py). Between 1e6 and that bound
// the product reduces in one step where the reference rounds every step, and they differ by the
// loop's accumulated rounding.
template <typename T> inline T normalized_angle(T angle) {
    if (!std::isfinite((double)angle)) return std::numeric_limits<T>::quiet_NaN();
    if (sizeof(T) == 8 && std::fabs((double)angle) > 1e9) {
        const double r = (double)angle - CV_2PI_D * std::nearbyint((double)angle / CV_2PI_D);
        if (!(std::fabs(r) <= 2.0 * CV_2PI_D)) return std::numeric_limits<T>::quiet_NaN();
        angle = (T)r;
    }
    while ((double)angle < -CV_PI_D) {
        const T next = (T)((double)angle + CV_2PI_D);
        if (next == angle) return std::numeric_limits<T>::quiet_NaN();
        angle = next;
    }
    while ((double)angle >= CV_PI_D) {
        const T next = (T)((double)angle - CV_2PI_D);
        if (next == angle) return std::numeric_limits<T>::quiet_NaN();
        angle = next;
    }
    return angle;
}

// Eigen::Rotation2D<T>::smallestAngle() as used at slam/solver_jacobians.cpp:18 and
// framework/definitions.hpp:42: fmod by 2pi, then one correction into [-pi, pi].
template <typename T> inline T smallest_angle(T a) {
    const T two_pi = (T)(2.0 * CV_PI_D);
    const T pi = (T)CV_PI_D;
    T tmp = std::fmod(a, two_pi);
    if (tmp > pi) tmp -= two_pi;
    else if (tmp < -pi) tmp += two_pi;
    return tmp;
}

template <typename T> struct PoseT { T x, y, th; };

// Two evaluations of the bearing prediction g = X^-1 l and its atan2:
//  * literal (oracle_set_literal(1)): Eigen's `pose.inverse() * lm` as the reference writes it
//    (slam/solver_jacobians.cpp:32, :302): Isometry inverse (R^T, -R^T t), each row a plain
//    product sum (this file is compiled without FP contraction), and libm atan2 (:15, :304). It
//    shares nothing with the product's code, so the C2/C3 parity tests use it: their bearings are
//    all in front of their poses (|bearing| < 85 deg), far from the +-pi wrap.
//  * bit-reproducing (default): the rounding sequence of the GPU kernels (bos_math.hpp
//    bearing_error, products summed with one explicit fma each) and the portable atan2 shared with
//    them. The reference dataset's single-observation landmarks sit exactly on the +-pi wrap after
//    triangulation, where the sign of e (and so b) flips on the last ulp of atan2: C1 and the mini
//    dataset are compared in this mode.
int g_literal = 0;

template <typename T> inline void bearing_g(const PoseT<T>& p, T lx, T ly, T& gx, T& gy) {
    const T c = std::cos(p.th), s = std::sin(p.th);
    if (g_literal) {
        const T itx = -(c * p.x + s * p.y), ity = -(-s * p.x + c * p.y);   // -R^T t
        gx = (c * lx + s * ly) + itx;                                          // R^T l + (-R^T t)
        gy = (-s * lx + c * ly) + ity;
        return;
    }
    const T itx = -std::fma(c, p.x, s * p.y);
    const T ity = -std::fma(-s, p.x, c * p.y);
    gx = std::fma(c, lx, s * ly) + itx;
    gy = std::fma(-s, lx, c * ly) + ity;
}

// Knife-edge bearings: an error exactly on the +-pi wrap (pred - z = +-pi up to the last ulp) is
// +pi or -pi depending on the last bit of atan2 and of g, so two correct evaluations may disagree
// in its sign (the reference dataset's landmark 112 after triangulation: -pi in the bit-reproducing
// form, +pi in the literal one). oracle_set_wrap_signs fixes that sign per bearing (from what the
// GPU path chose, read off its exported b by the tests), for errors within 1e-9 (fp64) / 1e-6
// (fp32) of pi only; every other bearing keeps its computed error.
std::vector<signed char> g_wrap_sign;

template <typename T> inline T knife_edge(int k, T e) {
    if (g_wrap_sign.empty() || g_wrap_sign[(size_t)k] == 0) return e;
    const double tol = sizeof(T) == 4 ? 1e-6 : 1e-9;
    if (!(std::fabs((double)e) >= CV_PI_D - tol)) return e;
    return g_wrap_sign[(size_t)k] > 0 ? (T)std::fabs(e) : (T)-std::fabs(e);
}

template <typename T> inline T bearing_atan2(T gy, T gx) {
    return g_literal ? std::atan2(gy, gx) : bos::det_atan2(gy, gx);
}

template <typename T> inline T predict_bearing(const PoseT<T>& p, T lx, T ly) {
    T gx, gy;
    bearing_g(p, lx, ly, gx, gy);
    return bearing_atan2(gy, gx);
}

// Bearing error_and_jacobian — slam/solver_jacobians.cpp:9-95.
// J (1x5) = [J_t(2) | J_theta | J_l(2)] at column bases 3*pose_stix and 3*NP+2*lm_stix (:70-71).
template <typename T> inline T bearing_error_and_jacobian(const PoseT<T>& p, T lx, T ly, T z, T J[5]) {
    const T c = std::cos(p.th), s = std::sin(p.th);
    T gx, gy;
    bearing_g(p, lx, ly, gx, gy);
    const T pred = bearing_atan2(gy, gx);                              // :15, :301-305
    const T e = normalized_angle<T>(pred - z);                         // :18 (z already smallestAngle)
    const T f = (T)1 / (gx * gx + gy * gy);                            // :35
    const T a0 = f * (-gy), a1 = f * gx;                               // :47-48
    // R^T = [[c, s], [-s, c]]; jac_of_g_wrt_Dt = -R^T (:59);
    // jac_of_g_wrt_Dtheta = R^T * [[0,1],[-1,0]] * l = R^T (ly, -lx) (:52-60);
    // jac_of_g_wrt_Dxl = R^T (:64). J = jac_atan2 (1x2) * jac_g (2xN) (:92).
    const T gth_x = c * ly + s * (-lx);
    const T gth_y = -s * ly + c * (-lx);
    J[0] = a0 * (-c) + a1 * (s);
    J[1] = a0 * (-s) + a1 * (-c);
    J[2] = a0 * gth_x + a1 * gth_y;
    J[3] = a0 * c + a1 * (-s);
    J[4] = a0 * s + a1 * c;
    return e;
}

// Solver::predict_odometry — slam/solver_jacobians.cpp:307-323 (with t2v, definitions.hpp:39-43).
template <typename T> inline void predict_odometry(const PoseT<T>& s, const PoseT<T>& d, T out[3]) {
    const T cs = std::cos(s.th), ss = std::sin(s.th);
    const T tx = d.x - s.x, ty = d.y - s.y;                             // :318
    out[0] = cs * tx + ss * ty;                                         // :319 R_s^T t
    out[1] = -ss * tx + cs * ty;
    out[2] = normalized_angle<T>(d.th - s.th);                          // :321
}

// Odometry error_and_jacobian — slam/solver_jacobians.cpp:97-168. J is 3x6, row-major,
// columns [dx_s, dy_s, dth_s, dx_d, dy_d, dth_d].
template <typename T> inline void odometry_error_and_jacobian(const PoseT<T>& s, const PoseT<T>& d,
                                                              const T z[3], T e[3], T J[18]) {
    T pred[3];
    predict_odometry<T>(s, d, pred);
    e[0] = pred[0] - z[0];                                              // :106
    e[1] = pred[1] - z[1];
    e[2] = normalized_angle<T>(pred[2] - z[2]);                         // :107
    const T cs = std::cos(s.th), ss = std::sin(s.th);
    const T xd = d.x, yd = d.y;
    // jac_wrt_Dt_s = -R_s^T (:137); jac_wrt_Dtheta_s = (DR' R_s)^T t_d, -1 (:139-140);
    // jac_wrt_Dt_d = R_s^T (:143); jac_wrt_Dtheta_d = R_s^T DR' t_d, +1 (:145-146).
    const T ths0 = -ss * xd + cs * yd, ths1 = -cs * xd - ss * yd;
    const T thd0 = ss * xd - cs * yd, thd1 = ss * yd + cs * xd;
    const T Jr[18] = {
        -cs, -ss, ths0,  cs, ss, thd0,
         ss, -cs, ths1, -ss, cs, thd1,
         0,    0, (T)-1,  0,  0, (T)1,
    };
    std::memcpy(J, Jr, sizeof(Jr));
}

template <typename T> struct ProblemView {
    int NP, NL, Mb, Mo, fixed;
    const double *pose_xyt, *lm_xy;
    const int32_t *b_pose, *b_lm;
    const double *b_z, *b_omega;
    const int32_t *o_src, *o_dst;
    const double *o_z, *o_omega;
};

template <typename T> inline PoseT<T> load_pose(const double* xyt, int i) {
    return PoseT<T>{(T)xyt[3 * i], (T)xyt[3 * i + 1], (T)xyt[3 * i + 2]};
}

int num_threads_or(int t) {
#ifdef _OPENMP
    return t > 0 ? t : omp_get_max_threads();
#else
    (void)t;
    return 1;
#endif
}

// One linearization = the accumulation loops of Solver::step (slam/solver.cpp:28-69):
// bearings in file order (:31-46), odometry (:48-62), robust kernel scaling e only
// (:37-41, :54-58), damping on all N (:64-69). Output is block-structured (no permutation).
//   pose_diag [NP][3][3], lm_diag [NL][2][2]     accumulated diagonal blocks (+damping)
//   hpl       [Mb][3][2]  H(pose dofs, lm dofs) contribution of bearing k
//   hoff      [Mo][3][3]  H(src dofs, dst dofs) contribution of odometry edge k
//   b         [3NP + 2NL] reference dof order
template <typename T>
int linearize(const ProblemView<T>& P, double kernel_threshold, double damping, double* pose_diag,
              double* lm_diag, double* hpl, double* hoff, double* b, double* chi2_out, int* nrobust_out,
              int threads) {
    const int NP = P.NP, NL = P.NL;
    const int N = 3 * NP + 2 * NL;
    const T kt = (T)kernel_threshold;
    const int nt = num_threads_or(threads);
    std::vector<std::vector<T>> pd(nt, std::vector<T>(9 * (size_t)NP, (T)0));
    std::vector<std::vector<T>> ld(nt, std::vector<T>(4 * (size_t)NL, (T)0));
    std::vector<std::vector<T>> bb(nt, std::vector<T>((size_t)N, (T)0));
    std::vector<double> chi(nt, 0.0);
    std::vector<int> nrob(nt, 0);

#ifdef _OPENMP
#pragma omp parallel num_threads(nt)
#endif
    {
#ifdef _OPENMP
        const int tid = omp_get_thread_num();
#else
        const int tid = 0;
#endif
        T* PD = pd[tid].data();
        T* LD = ld[tid].data();
        T* B = bb[tid].data();
        double lchi = 0.0;
        int lrob = 0;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int k = 0; k < P.Mb; ++k) {
            const int ip = P.b_pose[k], il = P.b_lm[k];
            const PoseT<T> p = load_pose<T>(P.pose_xyt, ip);
            const T lx = (T)P.lm_xy[2 * il], ly = (T)P.lm_xy[2 * il + 1];
            T J[5];
            T e = knife_edge<T>(k, bearing_error_and_jacobian<T>(p, lx, ly, (T)P.b_z[k], J));
            const T w = P.b_omega ? (T)P.b_omega[k] : (T)1;             // observation.hpp:16,22 (omega=1)
            const T rho = e * w * e;                                     // solver.cpp:37
            lchi += (double)rho;
            if (rho > kt) { e *= std::sqrt(kt / rho); ++lrob; }          // solver.cpp:38-40
            // H += J^T w J (:44); b += J^T w e (:45)
            T* pdk = PD + 9 * (size_t)ip;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) pdk[3 * i + j] += J[i] * w * J[j];
            T* ldk = LD + 4 * (size_t)il;
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) ldk[2 * i + j] += J[3 + i] * w * J[3 + j];
            double* hk = hpl + 6 * (size_t)k;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 2; ++j) hk[2 * i + j] = (double)(J[i] * w * J[3 + j]);
            for (int i = 0; i < 3; ++i) B[3 * ip + i] += J[i] * w * e;
            for (int i = 0; i < 2; ++i) B[3 * NP + 2 * il + i] += J[3 + i] * w * e;
        }
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int k = 0; k < P.Mo; ++k) {
            const int is = P.o_src[k], id = P.o_dst[k];
            const PoseT<T> s = load_pose<T>(P.pose_xyt, is);
            const PoseT<T> d = load_pose<T>(P.pose_xyt, id);
            T z[3] = {(T)P.o_z[3 * k], (T)P.o_z[3 * k + 1], (T)P.o_z[3 * k + 2]};
            T Om[9];
            for (int i = 0; i < 9; ++i) Om[i] = (T)P.o_omega[9 * k + i];
            T e[3], J[18];
            odometry_error_and_jacobian<T>(s, d, z, e, J);
            T Oe[3];
            for (int i = 0; i < 3; ++i) Oe[i] = Om[3 * i] * e[0] + Om[3 * i + 1] * e[1] + Om[3 * i + 2] * e[2];
            T rho = e[0] * Oe[0] + e[1] * Oe[1] + e[2] * Oe[2];          // solver.cpp:54
            lchi += (double)rho;
            if (rho > kt) {                                              // solver.cpp:55-57
                const T sc = std::sqrt(kt / rho);
                for (int i = 0; i < 3; ++i) { e[i] *= sc; Oe[i] *= sc; }
                ++lrob;
            }
            if (is == id) {
                // self-loop: the source and destination triplets share columns and setFromTriplets
                // sums them (solver_jacobians.cpp:126-165): J = J_s + J_d = 0 exactly (the two blocks
                // are exact negations), so H and b receive nothing (solver.cpp:60-61)
                for (int i = 0; i < 9; ++i) hoff[9 * (size_t)k + i] = 0.0;
                continue;
            }
            // OJ = Omega * J (3x6)
            T OJ[18];
            for (int i = 0; i < 3; ++i)
                for (int c = 0; c < 6; ++c)
                    OJ[6 * i + c] = Om[3 * i] * J[c] + Om[3 * i + 1] * J[6 + c] + Om[3 * i + 2] * J[12 + c];
            // H6 = J^T OJ ; b6 = J^T Oe  (solver.cpp:60-61)
            T H6[36], b6[6];
            for (int r = 0; r < 6; ++r) {
                for (int c = 0; c < 6; ++c)
                    H6[6 * r + c] = J[r] * OJ[c] + J[6 + r] * OJ[6 + c] + J[12 + r] * OJ[12 + c];
                b6[r] = J[r] * Oe[0] + J[6 + r] * Oe[1] + J[12 + r] * Oe[2];
            }
            T* ps = PD + 9 * (size_t)is;
            T* pdd = PD + 9 * (size_t)id;
            double* hk = hoff + 9 * (size_t)k;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    ps[3 * i + j] += H6[6 * i + j];
                    pdd[3 * i + j] += H6[6 * (3 + i) + 3 + j];
                    hk[3 * i + j] = (double)H6[6 * i + 3 + j];
                }
            for (int i = 0; i < 3; ++i) {
                B[3 * is + i] += b6[i];
                B[3 * id + i] += b6[3 + i];
            }
        }
        chi[tid] = lchi;
        nrob[tid] = lrob;
    }
    // deterministic reduction in thread order
    double chi2 = 0.0;
    int nr = 0;
    for (int t = 0; t < nt; ++t) { chi2 += chi[t]; nr += nrob[t]; }
    for (size_t i = 0; i < 9 * (size_t)NP; ++i) {
        T acc = (T)0;
        for (int t = 0; t < nt; ++t) acc += pd[t][i];
        pose_diag[i] = (double)acc;
    }
    for (size_t i = 0; i < 4 * (size_t)NL; ++i) {
        T acc = (T)0;
        for (int t = 0; t < nt; ++t) acc += ld[t][i];
        lm_diag[i] = (double)acc;
    }
    for (size_t i = 0; i < (size_t)N; ++i) {
        T acc = (T)0;
        for (int t = 0; t < nt; ++t) acc += bb[t][i];
        b[i] = (double)acc;
    }
    // damping on all N (solver.cpp:64-69), in the scalar type of the reference accumulation
    const T lam = (T)damping;
    for (int i = 0; i < NP; ++i)
        for (int d = 0; d < 3; ++d) pose_diag[9 * (size_t)i + 4 * d] = (double)((T)pose_diag[9 * (size_t)i + 4 * d] + lam);
    for (int j = 0; j < NL; ++j)
        for (int d = 0; d < 2; ++d) lm_diag[4 * (size_t)j + 3 * d] = (double)((T)lm_diag[4 * (size_t)j + 3 * d] + lam);
    if (chi2_out) *chi2_out = chi2;
    if (nrobust_out) *nrobust_out = nr;
    return 0;
}

// The same accumulation, parallel without per-thread copies of H and b ("owner computes", the
// CPU baseline of bench.py): each pose owns its diagonal block, its b entries and the pose-landmark
// blocks of its bearings; each landmark owns its diagonal block and b entries. A bearing is
// evaluated twice (once by its pose, once by its landmark), an odometry edge by both endpoints
// (the source also writes the off-diagonal block and counts chi^2). Only the summation order of
// the diagonal blocks and b differs from linearize() (rounding-level differences).
//   pb_ptr/pb_obs: bearings grouped by pose; lb_ptr/lb_obs: by landmark;
//   po_ptr/po_ent: odometry entries of each pose, edge << 1 | (pose is the destination).
template <typename T>
int linearize_owner(const ProblemView<T>& P, const int32_t* pb_ptr, const int32_t* pb_obs, const int32_t* lb_ptr,
                    const int32_t* lb_obs, const int32_t* po_ptr, const int32_t* po_ent, double kernel_threshold,
                    double damping, double* pose_diag, double* lm_diag, double* hpl, double* hoff, double* b,
                    double* chi2_out, int* nrobust_out, int threads) {
    const int NP = P.NP, NL = P.NL;
    const T kt = (T)kernel_threshold, lam = (T)damping;
    const int nt = num_threads_or(threads);
    double chi2 = 0.0;
    long long nr = 0;
#ifdef _OPENMP
#pragma omp parallel for num_threads(nt) schedule(dynamic, 256) reduction(+ : chi2, nr)
#endif
    for (int ip = 0; ip < NP; ++ip) {
        const PoseT<T> p = load_pose<T>(P.pose_xyt, ip);
        T H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, B[3] = {0, 0, 0};
        for (int x = pb_ptr[ip]; x < pb_ptr[ip + 1]; ++x) {
            const int k = pb_obs[x], il = P.b_lm[k];
            T J[5];
            T e = knife_edge<T>(k, bearing_error_and_jacobian<T>(p, (T)P.lm_xy[2 * il], (T)P.lm_xy[2 * il + 1], (T)P.b_z[k], J));
            const T w = P.b_omega ? (T)P.b_omega[k] : (T)1;
            const T rho = e * w * e;
            chi2 += (double)rho;
            if (rho > kt) { e *= std::sqrt(kt / rho); ++nr; }
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) H[3 * i + j] += J[i] * w * J[j];
            double* hk = hpl + 6 * (size_t)k;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 2; ++j) hk[2 * i + j] = (double)(J[i] * w * J[3 + j]);
            for (int i = 0; i < 3; ++i) B[i] += J[i] * w * e;
        }
        for (int x = po_ptr[ip]; x < po_ptr[ip + 1]; ++x) {
            const int k = po_ent[x] >> 1;
            const bool dst = po_ent[x] & 1;
            const int is = P.o_src[k], id = P.o_dst[k];
            const PoseT<T> s = load_pose<T>(P.pose_xyt, is), d = load_pose<T>(P.pose_xyt, id);
            T z[3] = {(T)P.o_z[3 * k], (T)P.o_z[3 * k + 1], (T)P.o_z[3 * k + 2]};
            T Om[9];
            for (int i = 0; i < 9; ++i) Om[i] = (T)P.o_omega[9 * k + i];
            T e[3], J[18];
            odometry_error_and_jacobian<T>(s, d, z, e, J);
            T Oe[3];
            for (int i = 0; i < 3; ++i) Oe[i] = Om[3 * i] * e[0] + Om[3 * i + 1] * e[1] + Om[3 * i + 2] * e[2];
            const T rho = e[0] * Oe[0] + e[1] * Oe[1] + e[2] * Oe[2];
            if (rho > kt) {
                const T sc = std::sqrt(kt / rho);
                for (int i = 0; i < 3; ++i) Oe[i] *= sc;
            }
            if (is == id) {   // self-loop: J = J_s + J_d = 0 (see linearize), chi^2 only
                if (!dst) {
                    chi2 += (double)rho;
                    if (rho > kt) ++nr;
                    for (int i = 0; i < 9; ++i) hoff[9 * (size_t)k + i] = 0.0;
                }
                continue;
            }
            const int c0 = dst ? 3 : 0;   // this pose's columns of J
            T OJ[18];
            for (int i = 0; i < 3; ++i)
                for (int c = 0; c < 6; ++c)
                    OJ[6 * i + c] = Om[3 * i] * J[c] + Om[3 * i + 1] * J[6 + c] + Om[3 * i + 2] * J[12 + c];
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c)
                    H[3 * r + c] += J[c0 + r] * OJ[c0 + c] + J[6 + c0 + r] * OJ[6 + c0 + c] + J[12 + c0 + r] * OJ[12 + c0 + c];
                B[r] += J[c0 + r] * Oe[0] + J[6 + c0 + r] * Oe[1] + J[12 + c0 + r] * Oe[2];
            }
            if (!dst) {
                chi2 += (double)rho;
                if (rho > kt) ++nr;
                double* hk = hoff + 9 * (size_t)k;
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c)
                        hk[3 * r + c] = (double)(J[r] * OJ[3 + c] + J[6 + r] * OJ[9 + c] + J[12 + r] * OJ[15 + c]);
            }
        }
        for (int d = 0; d < 3; ++d) H[4 * d] += lam;
        for (int i = 0; i < 9; ++i) pose_diag[9 * (size_t)ip + i] = (double)H[i];
        for (int i = 0; i < 3; ++i) b[3 * (size_t)ip + i] = (double)B[i];
    }
#ifdef _OPENMP
#pragma omp parallel for num_threads(nt) schedule(dynamic, 512)
#endif
    for (int il = 0; il < NL; ++il) {
        const T lx = (T)P.lm_xy[2 * il], ly = (T)P.lm_xy[2 * il + 1];
        T H[4] = {0, 0, 0, 0}, B[2] = {0, 0};
        for (int x = lb_ptr[il]; x < lb_ptr[il + 1]; ++x) {
            const int k = lb_obs[x];
            T J[5];
            T e = knife_edge<T>(k, bearing_error_and_jacobian<T>(load_pose<T>(P.pose_xyt, P.b_pose[k]), lx, ly, (T)P.b_z[k], J));
            const T w = P.b_omega ? (T)P.b_omega[k] : (T)1;
            const T rho = e * w * e;
            if (rho > kt) e *= std::sqrt(kt / rho);
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) H[2 * i + j] += J[3 + i] * w * J[3 + j];
            for (int i = 0; i < 2; ++i) B[i] += J[3 + i] * w * e;
        }
        H[0] += lam;
        H[3] += lam;
        for (int i = 0; i < 4; ++i) lm_diag[4 * (size_t)il + i] = (double)H[i];
        for (int i = 0; i < 2; ++i) b[3 * (size_t)NP + 2 * (size_t)il + i] = (double)B[i];
    }
    if (chi2_out) *chi2_out = chi2;
    if (nrobust_out) *nrobust_out = (int)nr;
    return 0;
}

// State::apply_boxplus — framework/state.cpp:69-80 with boxplus = v2t(dx) * X
// (framework/state.hpp:11-13, definitions.hpp:45-53): R <- dR R, t <- dR t + dt.
// theta is stored explicitly and kept wrapped by normalized_angle (t2v(X) then equals it).
template <typename T> void apply_boxplus(int NP, int NL, double* pose_xyt, double* lm_xy, const double* dx) {
    for (int i = 0; i < NP; ++i) {
        const T dxx = (T)dx[3 * i], dyy = (T)dx[3 * i + 1], dth = (T)dx[3 * i + 2];
        const T c = std::cos(dth), s = std::sin(dth);
        const T x = (T)pose_xyt[3 * i], y = (T)pose_xyt[3 * i + 1], th = (T)pose_xyt[3 * i + 2];
        pose_xyt[3 * i] = (double)(c * x - s * y + dxx);
        pose_xyt[3 * i + 1] = (double)(s * x + c * y + dyy);
        pose_xyt[3 * i + 2] = (double)normalized_angle<T>(th + dth);
    }
    for (int j = 0; j < NL; ++j) {
        lm_xy[2 * j] = (double)((T)lm_xy[2 * j] + (T)dx[3 * NP + 2 * j]);
        lm_xy[2 * j + 1] = (double)((T)lm_xy[2 * j + 1] + (T)dx[3 * NP + 2 * j + 1]);
    }
}

// triangulate_one_landmark — slam/triangulation.cpp:21-62: rows [sin(th+a), -cos(th+a)],
// rhs sin*px - cos*py, solved by Eigen colPivHouseholderQr (:59). Restated for 2 columns:
// column-pivoted Householder QR; the number of pivots follows Eigen's nonzeroPivots()
// rule; a rank-1 system gets the basic solution (pivot component solved, the other 0).
template <typename T> void triangulate_one(int M, const T* a0, const T* a1, const T* rhs, T out[2]) {
    std::vector<T> A0(a0, a0 + M), A1(a1, a1 + M), bv(rhs, rhs + M);
    T n0 = 0, n1 = 0;
    for (int i = 0; i < M; ++i) { n0 += A0[i] * A0[i]; n1 += A1[i] * A1[i]; }
    const bool swap = n1 > n0;                       // Eigen picks the first maximal norm
    std::vector<T>& C0 = swap ? A1 : A0;
    std::vector<T>& C1 = swap ? A0 : A1;
    auto householder = [&](int k, std::vector<T>& col, std::vector<std::vector<T>*> others) -> T {
        // Householder on col[k:], apply to others[k:]; returns r_kk.
        T sig = 0;
        for (int i = k + 1; i < M; ++i) sig += col[i] * col[i];
        const T x0 = col[k];
        if (sig == (T)0) return x0;
        const T mu = std::sqrt(x0 * x0 + sig);
        const T beta = x0 >= (T)0 ? -mu : mu;          // Eigen makeHouseholder: c0 >= 0 -> -norm
        const T v0 = x0 - beta;
        const T tau = (beta - x0) / beta;
        // essential part v[i] = col[i]/v0
        for (auto* o : others) {
            std::vector<T>& y = *o;
            T dot = y[k];
            for (int i = k + 1; i < M; ++i) dot += (col[i] / v0) * y[i];
            y[k] -= tau * dot;
            for (int i = k + 1; i < M; ++i) y[i] -= tau * dot * (col[i] / v0);
        }
        col[k] = beta;
        return beta;
    };
    const T r00 = householder(0, C0, {&C1, &bv});
    // Eigen ColPivHouseholderQR::_solve_impl uses nonzeroPivots(): the factorization stops at
    // step k when the largest remaining column norm^2 < (maxColNorm*eps)^2 * (rows-k)/rows.
    // A 1-row system has min(rows, cols) = 1 pivot (basic solution).
    const T max_col_norm = std::sqrt(std::max(n0, n1));
    const T eps = std::numeric_limits<T>::epsilon();
    const T thr_helper = (max_col_norm * eps) * (max_col_norm * eps) / (T)M;
    T r11 = (T)0;
    int rank = 1;
    if (M >= 2) {
        T rem = 0;
        for (int i = 1; i < M; ++i) rem += C1[i] * C1[i];
        if (!(rem < thr_helper * (T)(M - 1))) {
            r11 = householder(1, C1, {&bv});
            rank = 2;
        }
    }
    if (n0 == (T)0 && n1 == (T)0) rank = 0;
    T x0 = 0, x1 = 0;
    if (rank == 2) {
        x1 = bv[1] / r11;
        x0 = (bv[0] - C1[0] * x1) / r00;
    } else if (rank == 1) {
        x0 = bv[0] / r00;
        x1 = 0;
    }
    if (swap) { out[0] = x1; out[1] = x0; }
    else { out[0] = x0; out[1] = x1; }
}

}  // namespace

extern "C" {

// ABI version of this oracle, checked by oracle/oracle.py.
int oracle_version(void) { return 5; }

void oracle_set_literal(int on) { g_literal = on != 0; }
int oracle_get_literal() { return g_literal; }
// n = 0 clears; else signs[k] in {-1, 0, +1} for every bearing k < n (0 = no override)
void oracle_set_wrap_signs(int n, const signed char* signs) {
    if (n <= 0 || !signs) g_wrap_sign.clear();
    else g_wrap_sign.assign(signs, signs + n);
}
double oracle_normalized_angle_f64(double a) { return normalized_angle<double>(a); }
float oracle_normalized_angle_f32(float a) { return normalized_angle<float>(a); }
double oracle_smallest_angle_f64(double a) { return smallest_angle<double>(a); }
float oracle_smallest_angle_f32(float a) { return smallest_angle<float>(a); }

double oracle_predict_bearing_f64(const double* pose, double lx, double ly) {
    return predict_bearing<double>(PoseT<double>{pose[0], pose[1], pose[2]}, lx, ly);
}
float oracle_predict_bearing_f32(const float* pose, float lx, float ly) {
    return predict_bearing<float>(PoseT<float>{pose[0], pose[1], pose[2]}, lx, ly);
}
void oracle_predict_odometry_f64(const double* s, const double* d, double* out) {
    predict_odometry<double>(PoseT<double>{s[0], s[1], s[2]}, PoseT<double>{d[0], d[1], d[2]}, out);
}

// Per-observation error + analytic Jacobian (slam/solver_jacobians.cpp:9-95, :97-168).
double oracle_atan2_f64(double y, double x) { return bos::det_atan2<double>(y, x); }
float oracle_atan2_f32(float y, float x) { return bos::det_atan2<float>(y, x); }

double oracle_bearing_ej_f64(const double* pose, const double* lm, double z, double* J5) {
    return bearing_error_and_jacobian<double>(PoseT<double>{pose[0], pose[1], pose[2]}, lm[0], lm[1], z, J5);
}
float oracle_bearing_ej_f32(const float* pose, const float* lm, float z, float* J5) {
    return bearing_error_and_jacobian<float>(PoseT<float>{pose[0], pose[1], pose[2]}, lm[0], lm[1], z, J5);
}
// Every bearing's error e_k (fp64, the current form; no knife-edge override): the tests find the
// bearings on the +-pi wrap with it.
void oracle_bearing_errors(int Mb, const double* pose_xyt, const double* lm_xy, const int32_t* b_pose,
                           const int32_t* b_lm, const double* b_z, double* e_out) {
    for (int k = 0; k < Mb; ++k) {
        double J[5];
        e_out[k] = bearing_error_and_jacobian<double>(load_pose<double>(pose_xyt, b_pose[k]), lm_xy[2 * b_lm[k]],
                                                      lm_xy[2 * b_lm[k] + 1], b_z[k], J);
    }
}

void oracle_odometry_ej_f64(const double* s, const double* d, const double* z, double* e3, double* J18) {
    odometry_error_and_jacobian<double>(PoseT<double>{s[0], s[1], s[2]}, PoseT<double>{d[0], d[1], d[2]}, z, e3, J18);
}
void oracle_odometry_ej_f32(const float* s, const float* d, const float* z, float* e3, float* J18) {
    odometry_error_and_jacobian<float>(PoseT<float>{s[0], s[1], s[2]}, PoseT<float>{d[0], d[1], d[2]}, z, e3, J18);
}

int oracle_linearize(int precision, int NP, int NL, int Mb, int Mo, const double* pose_xyt, const double* lm_xy,
                     const int32_t* b_pose, const int32_t* b_lm, const double* b_z, const double* b_omega,
                     const int32_t* o_src, const int32_t* o_dst, const double* o_z, const double* o_omega,
                     double kernel_threshold, double damping, double* pose_diag, double* lm_diag, double* hpl,
                     double* hoff, double* b, double* chi2, int* nrobust, int threads) {
    if (precision == 32) {
        ProblemView<float> P{NP, NL, Mb, Mo, -1, pose_xyt, lm_xy, b_pose, b_lm, b_z, b_omega, o_src, o_dst, o_z, o_omega};
        return linearize<float>(P, kernel_threshold, damping, pose_diag, lm_diag, hpl, hoff, b, chi2, nrobust, threads);
    }
    ProblemView<double> P{NP, NL, Mb, Mo, -1, pose_xyt, lm_xy, b_pose, b_lm, b_z, b_omega, o_src, o_dst, o_z, o_omega};
    return linearize<double>(P, kernel_threshold, damping, pose_diag, lm_diag, hpl, hoff, b, chi2, nrobust, threads);
}

int oracle_linearize_owner(int precision, int NP, int NL, int Mb, int Mo, const double* pose_xyt, const double* lm_xy,
                           const int32_t* b_pose, const int32_t* b_lm, const double* b_z, const double* b_omega,
                           const int32_t* o_src, const int32_t* o_dst, const double* o_z, const double* o_omega,
                           const int32_t* pb_ptr, const int32_t* pb_obs, const int32_t* lb_ptr, const int32_t* lb_obs,
                           const int32_t* po_ptr, const int32_t* po_ent, double kernel_threshold, double damping,
                           double* pose_diag, double* lm_diag, double* hpl, double* hoff, double* b, double* chi2,
                           int* nrobust, int threads) {
    if (precision == 32) {
        ProblemView<float> P{NP, NL, Mb, Mo, -1, pose_xyt, lm_xy, b_pose, b_lm, b_z, b_omega, o_src, o_dst, o_z, o_omega};
        return linearize_owner<float>(P, pb_ptr, pb_obs, lb_ptr, lb_obs, po_ptr, po_ent, kernel_threshold, damping,
                                      pose_diag, lm_diag, hpl, hoff, b, chi2, nrobust, threads);
    }
    ProblemView<double> P{NP, NL, Mb, Mo, -1, pose_xyt, lm_xy, b_pose, b_lm, b_z, b_omega, o_src, o_dst, o_z, o_omega};
    return linearize_owner<double>(P, pb_ptr, pb_obs, lb_ptr, lb_obs, po_ptr, po_ent, kernel_threshold, damping,
                                   pose_diag, lm_diag, hpl, hoff, b, chi2, nrobust, threads);
}

void oracle_apply_boxplus(int precision, int NP, int NL, double* pose_xyt, double* lm_xy, const double* dx) {
    if (precision == 32) apply_boxplus<float>(NP, NL, pose_xyt, lm_xy, dx);
    else apply_boxplus<double>(NP, NL, pose_xyt, lm_xy, dx);
}

// triangulate_landmarks — slam/triangulation.cpp:65-74: bearings grouped by landmark id in
// ascending id order (std::map, :5-19); each group solved by triangulate_one_landmark (:21-62).
// Inputs: bearings given as (pose stix, landmark id, z = smallestAngle(bearing)).
// Output: lm_ids_out[nl] ascending, lm_xy_out[2*nl]; returns nl (or <0 on error).
int oracle_triangulate(int precision, int NP, const double* pose_xyt, int Mb, const int32_t* b_pose,
                       const int32_t* b_lmid, const double* b_z, int max_out, int32_t* lm_ids_out,
                       double* lm_xy_out) {
    std::map<int, std::vector<int>> groups;
    for (int k = 0; k < Mb; ++k) groups[b_lmid[k]].push_back(k);
    if ((int)groups.size() > max_out) return -1;
    int n = 0;
    for (auto& kv : groups) {
        const std::vector<int>& ks = kv.second;
        const int M = (int)ks.size();
        if (precision == 32) {
            std::vector<float> a0(M), a1(M), r(M);
            for (int i = 0; i < M; ++i) {
                const int ip = b_pose[ks[i]];
                if (ip < 0 || ip >= NP) return -2;
                const float th = normalized_angle<float>((float)pose_xyt[3 * ip + 2]);
                const float bz = (float)b_z[ks[i]];
                const float s = std::sin(th + bz), c = std::cos(th + bz);    // :50-51
                a0[i] = s; a1[i] = -c;                                         // :53
                r[i] = s * (float)pose_xyt[3 * ip] - c * (float)pose_xyt[3 * ip + 1];  // :54
            }
            float out[2];
            triangulate_one<float>(M, a0.data(), a1.data(), r.data(), out);
            lm_xy_out[2 * n] = out[0];
            lm_xy_out[2 * n + 1] = out[1];
        } else {
            std::vector<double> a0(M), a1(M), r(M);
            for (int i = 0; i < M; ++i) {
                const int ip = b_pose[ks[i]];
                if (ip < 0 || ip >= NP) return -2;
                const double th = pose_xyt[3 * ip + 2];
                const double bz = b_z[ks[i]];
                const double s = std::sin(th + bz), c = std::cos(th + bz);
                a0[i] = s; a1[i] = -c;
                r[i] = s * pose_xyt[3 * ip] - c * pose_xyt[3 * ip + 1];
            }
            double out[2];
            triangulate_one<double>(M, a0.data(), a1.data(), r.data(), out);
            lm_xy_out[2 * n] = out[0];
            lm_xy_out[2 * n + 1] = out[1];
        }
        lm_ids_out[n] = kv.first;
        ++n;
    }
    return n;
}

}  // extern "C"
