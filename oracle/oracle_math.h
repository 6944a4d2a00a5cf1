// oracle_math.h -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Deterministic scalar math used by the CPU restatement of the B-SHOT hot path.
// PARITY UNPINNED vs. PCL/Eigen/FLANN: the reference (TingKaiChen/B-SHOT-SLAM) delegates this
// arithmetic to PCL >= 1.7.2 / Eigen3 / FLANN, none of which exist in this container and none of
// which the reference pins by a test or golden vector. What follows restates the
// published algorithms with ONE documented operation order, using only
// IEEE-754 +,-,*,/,sqrt (correctly rounded on x86-64 SSE2 and on gfx950), so that the product's
// HIP kernels can reproduce the oracle bit-for-bit:
//   * transcendentals: acos/atan/atan2 in double = fdlibm algorithms; sin/cos in double = Taylor
//     series valid on |x| <= 1.2; float variants = (float) of the double result,
//   * symmetric 3x3 eigen-decomposition: cyclic Jacobi in double (stands in for Eigen's
//     SelfAdjointEigenSolver; eigenvector signs are disambiguated by the callers exactly as PCL),
//   * PCL's closed-form float eigen33/computeRoots (pcl/common/impl/eigen.hpp),
//   * 3x3 SVD: one-sided (Hestenes) Jacobi (stands in for Eigen::JacobiSVD inside umeyama).
// Compiled with -ffp-contract=off: no FMA contraction anywhere.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

namespace orc {

// ------------------------------------------------------------------ fdlibm-style atan / acos
inline double o_atan(double x) {
    static const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                     9.82793723247329054082e-01, 1.57079632679489655800e+00};
    static const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                     1.39033110312309984516e-17, 6.12323399573676603587e-17};
    static const double aT[11] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01,
                                  1.42857142725034663711e-01,  -1.11111104054623557880e-01,
                                  9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                                  6.66107313738753120669e-02,  -5.83357013379057348645e-02,
                                  4.97687799461593236017e-02,  -3.65315727442169155270e-02,
                                  1.62858201153657823623e-02};
    if (x != x) return x;
    const bool neg = x < 0.0;
    double ax = neg ? -x : x;
    if (ax >= 3.6893488147419103e+19) {  // 2^65: atan -> +-pi/2
        const double r = atanhi[3] + atanlo[3];
        return neg ? -r : r;
    }
    int id;
    if (ax < 0.4375) {
        if (ax < 1.862645149230957e-09) return x;  // 2^-29
        id = -1;
    } else if (ax < 1.1875) {
        if (ax < 0.6875) { id = 0; ax = (2.0 * ax - 1.0) / (2.0 + ax); }
        else             { id = 1; ax = (ax - 1.0) / (ax + 1.0); }
    } else {
        if (ax < 2.4375) { id = 2; ax = (ax - 1.5) / (1.0 + 1.5 * ax); }
        else             { id = 3; ax = -1.0 / ax; }
    }
    const double z = ax * ax;
    const double w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) {
        const double r = ax - ax * (s1 + s2);
        return neg ? -r : r;
    }
    const double r = atanhi[id] - ((ax * (s1 + s2) - atanlo[id]) - ax);
    return neg ? -r : r;
}

inline double o_atan2(double y, double x) {
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    const double pio2 = 1.57079632679489655800e+00;
    if (x != x || y != y) return x + y;
    if (y == 0.0) {
        if (std::signbit(x)) return std::signbit(y) ? -pi : pi;
        return y;
    }
    if (x == 0.0) return y < 0.0 ? -pio2 : pio2;
    if (std::isinf(x)) {
        if (std::isinf(y)) {
            const double r = x > 0 ? pio2 * 0.5 : 3.0 * pio2 * 0.5;
            return y < 0 ? -r : r;
        }
        const double r = x > 0 ? 0.0 : pi;
        return y < 0 ? -r : r;
    }
    if (std::isinf(y)) return y < 0 ? -pio2 : pio2;
    double z = o_atan(std::fabs(y / x));
    if (x > 0.0) return y < 0 ? -z : z;
    z = pi - (z - pi_lo);
    return y < 0 ? -z : z;
}

inline double o_acos_R(double z) {
    const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
                 qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    return p / q;
}

inline double o_acos(double x) {
    const double pi = 3.14159265358979311600e+00;
    const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
    if (x != x) return x;
    const double ax = std::fabs(x);
    if (ax >= 1.0) {
        if (ax == 1.0) return x > 0.0 ? 0.0 : pi + 2.0 * pio2_lo;
        return std::nan("");
    }
    if (ax < 0.5) {
        if (ax <= 6.938893903907228e-18) return pio2_hi + pio2_lo;  // 2^-57
        const double r = o_acos_R(x * x);
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if (x < 0.0) {
        const double z = (1.0 + x) * 0.5;
        const double s = std::sqrt(z);
        const double w = o_acos_R(z) * s - pio2_lo;
        return pi - 2.0 * (s + w);
    }
    const double z = (1.0 - x) * 0.5;
    const double s = std::sqrt(z);
    uint64_t bits;
    std::memcpy(&bits, &s, 8);
    bits &= 0xFFFFFFFF00000000ull;
    double df;
    std::memcpy(&df, &bits, 8);
    const double c = (z - df * df) / (s + df);
    const double w = o_acos_R(z) * s + c;
    return 2.0 * (df + w);
}

// cos / sin for |x| <= 1.2 (the only range on the path: theta = atan2(.)/3 in [0, pi/3]).
// Horner in z = x^2, highest order first, terms through 1/24! (truncation < 1e-25 on that range).
inline double o_cos_series(double x) {
    const double z = x * x;
    double r = 1.0 / 620448401733239439360000.0;    // 1/24!
    r = r * z - 1.0 / 1124000727777607680000.0;     // 1/22!
    r = r * z + 1.0 / 2432902008176640000.0;        // 1/20!
    r = r * z - 1.0 / 6402373705728000.0;           // 1/18!
    r = r * z + 1.0 / 20922789888000.0;             // 1/16!
    r = r * z - 1.0 / 87178291200.0;                // 1/14!
    r = r * z + 1.0 / 479001600.0;                  // 1/12!
    r = r * z - 1.0 / 3628800.0;                    // 1/10!
    r = r * z + 1.0 / 40320.0;                      // 1/8!
    r = r * z - 1.0 / 720.0;                        // 1/6!
    r = r * z + 1.0 / 24.0;                         // 1/4!
    r = r * z - 0.5;                                // 1/2!
    r = r * z + 1.0;
    return r;
}

inline double o_sin(double x) {  // |x| <= 1.2
    const double z = x * x;
    double r = 1.0 / 25852016738884976640000.0;     // 1/23!
    r = r * z - 1.0 / 51090942171709440000.0;       // 1/21!
    r = r * z + 1.0 / 121645100408832000.0;         // 1/19!
    r = r * z - 1.0 / 355687428096000.0;            // 1/17!
    r = r * z + 1.0 / 1307674368000.0;              // 1/15!
    r = r * z - 1.0 / 6227020800.0;                 // 1/13!
    r = r * z + 1.0 / 39916800.0;                   // 1/11!
    r = r * z - 1.0 / 362880.0;                     // 1/9!
    r = r * z + 1.0 / 5040.0;                       // 1/7!
    r = r * z - 1.0 / 120.0;                        // 1/5!
    r = r * z + 1.0 / 6.0;                          // 1/3!
    // sin x = x - x*z*(1/3! - z/5! + ...)
    return x - x * (z * r);
}

inline float o_atan2f(float y, float x) { return (float)o_atan2((double)y, (double)x); }
inline float o_cosf(float x) { return (float)o_cos_series((double)x); }
inline float o_sinf(float x) { return (float)o_sin((double)x); }

// ------------------------------------------------------------------ PCL eigen33 (float)
// Restates pcl::computeRoots2 / computeRoots / eigen33 (pcl/common/impl/eigen.hpp, PCL 1.8)
// with the C++ evaluation order of the source expressions. m is row-major 3x3.
inline void o_computeRoots2(float b, float c, float roots[3]) {
    roots[0] = 0.0f;
    float d = (float)((double)(b * b) - 4.0 * (double)c);
    if (d < 0.0f) d = 0.0f;
    const float sd = std::sqrt(d);
    roots[2] = 0.5f * (b + sd);
    roots[1] = 0.5f * (b - sd);
}

inline void o_computeRoots(const float m[9], float roots[3]) {
    const float m00 = m[0], m01 = m[1], m02 = m[2], m11 = m[4], m12 = m[5], m22 = m[8];
    const float c0 = ((((m00 * m11) * m22 + ((2.0f * m01) * m02) * m12) - (m00 * m12) * m12) -
                      (m11 * m02) * m02) - (m22 * m01) * m01;
    const float c1 = ((((m00 * m11 - m01 * m01) + m00 * m22) - m02 * m02) + m11 * m22) - m12 * m12;
    const float c2 = (m00 + m11) + m22;
    if (std::fabs(c0) < 1.19209290e-07f) {
        o_computeRoots2(c2, c1, roots);
        return;
    }
    const float s_inv3 = (float)(1.0 / 3.0);
    const float s_sqrt3 = std::sqrt(3.0f);
    const float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > 0.0f) a_over_3 = 0.0f;
    const float half_b = 0.5f * (c0 + c2_over_3 * (((2.0f * c2_over_3) * c2_over_3) - c1));
    float q = half_b * half_b + (a_over_3 * a_over_3) * a_over_3;
    if (q > 0.0f) q = 0.0f;
    const float rho = std::sqrt(-a_over_3);
    const float theta = o_atan2f(std::sqrt(-q), half_b) * s_inv3;
    const float cos_theta = o_cosf(theta);
    const float sin_theta = o_sinf(theta);
    roots[0] = c2_over_3 + (2.0f * rho) * cos_theta;
    roots[1] = c2_over_3 - rho * (cos_theta + s_sqrt3 * sin_theta);
    roots[2] = c2_over_3 - rho * (cos_theta - s_sqrt3 * sin_theta);
    float t;
    if (roots[0] >= roots[1]) { t = roots[0]; roots[0] = roots[1]; roots[1] = t; }
    if (roots[1] >= roots[2]) {
        t = roots[1]; roots[1] = roots[2]; roots[2] = t;
        if (roots[0] >= roots[1]) { t = roots[0]; roots[0] = roots[1]; roots[1] = t; }
    }
    if (roots[0] <= 0.0f) o_computeRoots2(c2, c1, roots);
}

inline float o_scale_of(const float m[9]) {
    float s = std::fabs(m[0]);
    for (int i = 1; i < 9; ++i) {
        const float a = std::fabs(m[i]);
        if (a > s) s = a;
    }
    if (s <= 1.17549435e-38f) s = 1.0f;
    return s;
}

// eigen33(mat, eigenvalue, eigenvector): smallest eigenvalue and its eigenvector.
inline void o_eigen33_min(const float mat[9], float* eigenvalue, float vec[3]) {
    const float scale = o_scale_of(mat);
    float sm[9];
    for (int i = 0; i < 9; ++i) sm[i] = mat[i] / scale;
    float ev[3];
    o_computeRoots(sm, ev);
    *eigenvalue = ev[0] * scale;
    sm[0] -= ev[0]; sm[4] -= ev[0]; sm[8] -= ev[0];
    const float* r0 = sm;
    const float* r1 = sm + 3;
    const float* r2 = sm + 6;
    float v1[3] = {r0[1] * r1[2] - r0[2] * r1[1], r0[2] * r1[0] - r0[0] * r1[2], r0[0] * r1[1] - r0[1] * r1[0]};
    float v2[3] = {r0[1] * r2[2] - r0[2] * r2[1], r0[2] * r2[0] - r0[0] * r2[2], r0[0] * r2[1] - r0[1] * r2[0]};
    float v3[3] = {r1[1] * r2[2] - r1[2] * r2[1], r1[2] * r2[0] - r1[0] * r2[2], r1[0] * r2[1] - r1[1] * r2[0]};
    const float len1 = (v1[0] * v1[0] + v1[1] * v1[1]) + v1[2] * v1[2];
    const float len2 = (v2[0] * v2[0] + v2[1] * v2[1]) + v2[2] * v2[2];
    const float len3 = (v3[0] * v3[0] + v3[1] * v3[1]) + v3[2] * v3[2];
    const float* v;
    float len;
    if (len1 >= len2 && len1 >= len3) { v = v1; len = len1; }
    else if (len2 >= len1 && len2 >= len3) { v = v2; len = len2; }
    else { v = v3; len = len3; }
    const float sl = std::sqrt(len);
    vec[0] = v[0] / sl; vec[1] = v[1] / sl; vec[2] = v[2] / sl;
}

// eigen33(mat, evals): all three eigenvalues, ascending.
inline void o_eigen33_vals(const float mat[9], float evals[3]) {
    const float scale = o_scale_of(mat);
    float sm[9];
    for (int i = 0; i < 9; ++i) sm[i] = mat[i] / scale;
    o_computeRoots(sm, evals);
    evals[0] *= scale; evals[1] *= scale; evals[2] *= scale;
}

// ------------------------------------------------------------------ Jacobi eigen (double)
// Cyclic Jacobi on a symmetric 3x3 (row-major a[9]); returns eigenvalues ascending in w[3] and
// the matching unit eigenvectors as COLUMNS of v[9] (row-major). Stands in for
// Eigen::SelfAdjointEigenSolver<Matrix3d> (used by PCL's SHOT LRF and ISS).
inline void o_jacobi3(const double ain[9], double w[3], double v[9]) {
    double a[9];
    for (int i = 0; i < 9; ++i) a[i] = ain[i];
    for (int i = 0; i < 9; ++i) v[i] = (i % 4 == 0) ? 1.0 : 0.0;
    static const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};
    for (int sweep = 0; sweep < 32; ++sweep) {
        const double off = std::fabs(a[1]) + std::fabs(a[2]) + std::fabs(a[5]);
        if (off == 0.0) break;
        for (int k = 0; k < 3; ++k) {
            const int p = P[k], q = Q[k];
            const double apq = a[p * 3 + q];
            if (apq == 0.0) continue;
            const double app = a[p * 3 + p], aqq = a[q * 3 + q];
            const double g = 100.0 * std::fabs(apq);
            if (sweep > 3 && std::fabs(app) + g == std::fabs(app) && std::fabs(aqq) + g == std::fabs(aqq)) {
                a[p * 3 + q] = 0.0;
                a[q * 3 + p] = 0.0;
                continue;
            }
            const double theta = (aqq - app) / (2.0 * apq);
            double t;
            if (std::fabs(theta) > 1e150) {
                t = 0.5 / theta;
            } else {
                t = 1.0 / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                if (theta < 0.0) t = -t;
            }
            const double c = 1.0 / std::sqrt(t * t + 1.0);
            const double s = t * c;
            const double tau = s / (1.0 + c);
            a[p * 3 + p] = app - t * apq;
            a[q * 3 + q] = aqq + t * apq;
            a[p * 3 + q] = 0.0;
            a[q * 3 + p] = 0.0;
            const int r = 3 - p - q;
            const double arp = a[r * 3 + p], arq = a[r * 3 + q];
            const double nrp = arp - s * (arq + tau * arp);
            const double nrq = arq + s * (arp - tau * arq);
            a[r * 3 + p] = nrp; a[p * 3 + r] = nrp;
            a[r * 3 + q] = nrq; a[q * 3 + r] = nrq;
            for (int i = 0; i < 3; ++i) {
                const double vip = v[i * 3 + p], viq = v[i * 3 + q];
                v[i * 3 + p] = vip - s * (viq + tau * vip);
                v[i * 3 + q] = viq + s * (vip - tau * viq);
            }
        }
    }
    double d[3] = {a[0], a[4], a[8]};
    int idx[3] = {0, 1, 2};
    // stable ascending sort of 3 (insertion)
    for (int i = 1; i < 3; ++i) {
        int j = i;
        while (j > 0 && d[idx[j]] < d[idx[j - 1]]) { int t = idx[j]; idx[j] = idx[j - 1]; idx[j - 1] = t; --j; }
    }
    double vv[9];
    for (int c = 0; c < 3; ++c) {
        w[c] = d[idx[c]];
        for (int i = 0; i < 3; ++i) vv[i * 3 + c] = v[i * 3 + idx[c]];
    }
    for (int i = 0; i < 9; ++i) v[i] = vv[i];
}

// ------------------------------------------------------------------ one-sided Jacobi SVD
// A = U diag(s) V^T for a 3x3 (row-major) in precision T; s descending. U completed by a cross
// product when the smallest singular value vanishes. Stands in for Eigen::JacobiSVD.
template <typename T>
inline void o_svd3(const T ain[9], T U[9], T s[3], T V[9]) {
    T a[9];
    for (int i = 0; i < 9; ++i) a[i] = ain[i];
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? T(1) : T(0);
    const T eps = sizeof(T) == 8 ? T(2.220446049250313e-16) : T(1.1920929e-07f);
    static const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};
    for (int sweep = 0; sweep < 40; ++sweep) {
        bool rotated = false;
        for (int k = 0; k < 3; ++k) {
            const int p = P[k], q = Q[k];
            T alpha = T(0), beta = T(0), gamma = T(0);
            for (int i = 0; i < 3; ++i) {
                const T ap = a[i * 3 + p], aq = a[i * 3 + q];
                alpha = alpha + ap * ap;
                beta = beta + aq * aq;
                gamma = gamma + ap * aq;
            }
            if (gamma == T(0)) continue;
            if (std::fabs(gamma) <= eps * std::sqrt(alpha * beta)) continue;
            rotated = true;
            const T zeta = (beta - alpha) / (T(2) * gamma);
            T t = T(1) / (std::fabs(zeta) + std::sqrt(T(1) + zeta * zeta));
            if (zeta < T(0)) t = -t;
            const T c = T(1) / std::sqrt(T(1) + t * t);
            const T sn = c * t;
            for (int i = 0; i < 3; ++i) {
                const T ap = a[i * 3 + p], aq = a[i * 3 + q];
                a[i * 3 + p] = c * ap - sn * aq;
                a[i * 3 + q] = sn * ap + c * aq;
                const T vp = V[i * 3 + p], vq = V[i * 3 + q];
                V[i * 3 + p] = c * vp - sn * vq;
                V[i * 3 + q] = sn * vp + c * vq;
            }
        }
        if (!rotated) break;
    }
    T nrm[3];
    for (int j = 0; j < 3; ++j) {
        T ss = T(0);
        for (int i = 0; i < 3; ++i) ss = ss + a[i * 3 + j] * a[i * 3 + j];
        nrm[j] = std::sqrt(ss);
    }
    int idx[3] = {0, 1, 2};
    for (int i = 1; i < 3; ++i) {
        int j = i;
        while (j > 0 && nrm[idx[j]] > nrm[idx[j - 1]]) { int t = idx[j]; idx[j] = idx[j - 1]; idx[j - 1] = t; --j; }
    }
    T Vs[9];
    for (int c = 0; c < 3; ++c) {
        s[c] = nrm[idx[c]];
        for (int i = 0; i < 3; ++i) {
            Vs[i * 3 + c] = V[i * 3 + idx[c]];
            U[i * 3 + c] = (s[c] > T(0)) ? a[i * 3 + idx[c]] / s[c] : T(0);
        }
    }
    for (int i = 0; i < 9; ++i) V[i] = Vs[i];
    const T tiny = s[0] * eps * T(8);
    if (!(s[1] > tiny)) {
        // rank <= 1: complete U with an orthonormal basis around column 0
        T u0[3] = {U[0], U[3], U[6]};
        if (!(s[0] > T(0))) { u0[0] = T(1); u0[1] = T(0); u0[2] = T(0); U[0] = T(1); U[3] = T(0); U[6] = T(0); }
        T e[3] = {T(1), T(0), T(0)};
        if (std::fabs(u0[0]) > std::fabs(u0[1])) { e[0] = T(0); e[1] = T(1); }
        T u1[3] = {u0[1] * e[2] - u0[2] * e[1], u0[2] * e[0] - u0[0] * e[2], u0[0] * e[1] - u0[1] * e[0]};
        const T l = std::sqrt((u1[0] * u1[0] + u1[1] * u1[1]) + u1[2] * u1[2]);
        U[1] = u1[0] / l; U[4] = u1[1] / l; U[7] = u1[2] / l;
    }
    if (!(s[2] > tiny)) {
        const T x0 = U[0], y0 = U[3], z0 = U[6], x1 = U[1], y1 = U[4], z1 = U[7];
        U[2] = y0 * z1 - z0 * y1;
        U[5] = z0 * x1 - x0 * z1;
        U[8] = x0 * y1 - y0 * x1;
    }
}

template <typename T>
inline T o_det3(const T m[9]) {
    return (m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6])) +
           m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// Eigen::umeyama(src, dst, with_scaling=false) in precision T for n 3-D points (AoS, T).
// Output: row-major 4x4 rigid transform (last row 0 0 0 1).
template <typename T>
inline void o_umeyama(const T* src, const T* dst, int n, T out[16]) {
    const T one_over_n = T(1) / T(n);
    T sm[3] = {T(0), T(0), T(0)}, dm[3] = {T(0), T(0), T(0)};
    for (int d = 0; d < 3; ++d) {
        T ss = src[d], ds = dst[d];
        for (int i = 1; i < n; ++i) { ss = ss + src[i * 3 + d]; ds = ds + dst[i * 3 + d]; }
        sm[d] = ss * one_over_n;
        dm[d] = ds * one_over_n;
    }
    T sigma[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            T acc = (dst[r] - dm[r]) * (src[c] - sm[c]);
            for (int i = 1; i < n; ++i) acc = acc + (dst[i * 3 + r] - dm[r]) * (src[i * 3 + c] - sm[c]);
            sigma[r * 3 + c] = acc * one_over_n;
        }
    T U[9], S[3], V[9];
    o_svd3<T>(sigma, U, S, V);
    T d3 = T(1);
    if (o_det3<T>(U) * o_det3<T>(V) < T(0)) d3 = T(-1);
    T R[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            R[r * 3 + c] = (U[r * 3 + 0] * V[c * 3 + 0] + U[r * 3 + 1] * V[c * 3 + 1]) + (U[r * 3 + 2] * d3) * V[c * 3 + 2];
    for (int r = 0; r < 3; ++r) {
        out[r * 4 + 0] = R[r * 3 + 0];
        out[r * 4 + 1] = R[r * 3 + 1];
        out[r * 4 + 2] = R[r * 3 + 2];
        out[r * 4 + 3] = dm[r] - ((R[r * 3 + 0] * sm[0] + R[r * 3 + 1] * sm[1]) + R[r * 3 + 2] * sm[2]);
    }
    out[12] = T(0); out[13] = T(0); out[14] = T(0); out[15] = T(1);
}

}  // namespace orc
