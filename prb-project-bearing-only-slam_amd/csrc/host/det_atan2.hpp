// Portable atan2 with identical results on the host (g++, x86-64) and on gfx950 (hipcc).
//
// Why: a bearing whose predicted and measured angles differ by almost exactly pi (the reference's
// single-observation landmarks, placed by the rank-1 basic solution of slam/triangulation.cpp,
// land there) has an error e = normalized_angle(atan2(g) - z) on the wrap discontinuity, so the
// last ulp of atan2 decides the sign of e and of its whole b contribution. libm atan2 (glibc) and
// the ROCm device library differ in the last ulp, so the GPU path and the CPU oracle both use this
// routine, evaluated with plain IEEE operations (no FP contraction: callers compile it with
// -ffp-contract=off or inside `#pragma clang fp contract(off)`), and round identically.
//
// Algorithm: the classic argument reduction of fdlibm's atan (breakpoints 7/16, 11/16, 19/16,
// 39/16; atan(c) split into hi + lo) written branch-free with one division, an odd minimax
// polynomial on |u| <= 7/16, then the atan2 quadrant fix with pi split into hi + lo.
// Accuracy is checked against libm in tests/test_oracle.py (<= 1 ulp double, <= 1 ulp float).
#pragma once

#include <cmath>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define BOS_DET_HD __host__ __device__ __forceinline__
#else
#define BOS_DET_HD inline
#endif

namespace bos {

template <typename T> struct AtanConsts;

template <> struct AtanConsts<double> {
    static constexpr double hi[5] = {0.0, 4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                     9.82793723247329054082e-01, 1.57079632679489655800e+00};
    static constexpr double lo[5] = {0.0, 2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                     1.39033110312309984516e-17, 6.12323399573676603587e-17};
    static constexpr double aT[11] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01,
                                      1.42857142725034663711e-01,  -1.11111104054623557880e-01,
                                      9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                                      6.66107313738753120669e-02,  -5.83357013379057348645e-02,
                                      4.97687799461593236017e-02,  -3.65315727442169155270e-02,
                                      1.62858201153657823623e-02};
    static constexpr double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    static constexpr double pi_o_2 = 1.5707963267948965580e+00;
};

template <> struct AtanConsts<float> {
    static constexpr float hi[5] = {0.0f, 4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    static constexpr float lo[5] = {0.0f, 5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    static constexpr float aT[11] = {3.3333334327e-01f,  -2.0000000298e-01f, 1.4285714924e-01f,  -1.1111110449e-01f,
                                     9.0908870101e-02f,  -7.6918758452e-02f, 6.6610731184e-02f,  -5.8335702866e-02f,
                                     4.9768779427e-02f,  -3.6531571299e-02f, 1.6285819933e-02f};
    static constexpr float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    static constexpr float pi_o_2 = 1.5707963705e+00f;
};

// atan(ay / ax) for ay, ax > 0, with a single division: the reduced argument
// u = (t - c) / (1 + c t) is formed as (ay - c ax) / (ax + c ay) (u = -ax / ay beyond 39/16; the
// numerator is exact for c = 1/2 and 1 by Sterbenz). Horner chains use explicit fma, which is
// correctly rounded on both targets.
template <typename T> BOS_DET_HD T det_atan_ratio(T ay, T ax) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    using C = AtanConsts<T>;
    // reduction interval: 0: t < 7/16, 1: < 11/16, 2: < 19/16, 3: < 39/16, 4: beyond. The tests
    // are nested (k ax is monotone in k), so the interval is the last one that holds; written as
    // selects (no branches on the GPU)
    const bool b1 = ay >= (T)0.4375 * ax, b2 = ay >= (T)0.6875 * ax, b3 = ay >= (T)1.1875 * ax,
               b4 = ay >= (T)2.4375 * ax;
    const T c = b3 ? (T)1.5 : b2 ? (T)1 : b1 ? (T)0.5 : (T)0;
    const T num = b4 ? -ax : ay - c * ax;
    const T den = b4 ? ay : ax + c * ay;
    const T u = num / den;
    const T z = u * u, w = z * z;
    using std::fma;
    const T s1 = z * fma(w, fma(w, fma(w, fma(w, fma(w, C::aT[10], C::aT[8]), C::aT[6]), C::aT[4]), C::aT[2]), C::aT[0]);
    const T s2 = w * fma(w, fma(w, fma(w, fma(w, C::aT[9], C::aT[7]), C::aT[5]), C::aT[3]), C::aT[1]);
    // atan(c) = hi + lo, selected without memory indexing
    const T hi = b4 ? C::hi[4] : b3 ? C::hi[3] : b2 ? C::hi[2] : b1 ? C::hi[1] : (T)0;
    const T lo = b4 ? C::lo[4] : b3 ? C::lo[3] : b2 ? C::lo[2] : b1 ? C::lo[1] : (T)0;
    return hi - (fma(u, s1 + s2, -lo) - u);
}

template <typename T> BOS_DET_HD T det_atan2(T y, T x) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    using C = AtanConsts<T>;
    const T ax = std::fabs(x), ay = std::fabs(y);
    // the ratio is evaluated unconditionally and discarded on the axes (0/0 there), so the GPU
    // runs this as selects
    const T a = det_atan_ratio<T>(ay, ax);
    const bool neg_x = std::signbit(x);
    const T r = ay == (T)0 ? (neg_x ? C::pi : (T)0) : ax == (T)0 ? C::pi_o_2 : neg_x ? C::pi - (a - C::pi_lo) : a;
    return std::signbit(y) ? -r : r;
}

}  // namespace bos
