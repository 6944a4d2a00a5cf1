// bshot_math.h -- scalar math shared by the gfx950 kernels and the host-side stages of libbshot_amd.
//
// Every routine uses only IEEE-754 +,-,*,/,sqrt (correctly rounded on gfx950 with
// -fhip-fp32-correctly-rounded-divide-sqrt and on x86-64 SSE2) and a fixed operation order;
// libbshot_amd is compiled with -ffp-contract=off, so device and host produce identical bits.
// What each routine stands in for (the reference delegates this arithmetic to PCL/Eigen, which
// are not available here -- DESIGN.md "Numerics conventions"):
//   bm_acos / bm_atan2        acos/atan2 in PCL SHOT interpolateSingleChannel (fdlibm algorithms)
//   bm_cos_s / bm_sin_s       cos/sin inside pcl::computeRoots (Taylor, |x| <= 1.2 suffices)
//   bm_eigen33_min / _vals    pcl::eigen33 (closed form, float), pcl/common/impl/eigen.hpp
//   bm_jacobi3                Eigen::SelfAdjointEigenSolver<Matrix3d> (ISS, SHOT LRF)
//   bm_svd3 / bm_umeyama      Eigen::JacobiSVD inside Eigen::umeyama (RANSAC model, ICP step)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BM_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define BM_HD inline
#endif

namespace bm {

BM_HD double dabs(double x) { return __builtin_fabs(x); }
BM_HD float fabs_(float x) { return __builtin_fabsf(x); }
BM_HD double dsqrt(double x) { return __builtin_sqrt(x); }
BM_HD float fsqrt(float x) { return __builtin_sqrtf(x); }
BM_HD bool isfin(double x) { return __builtin_isfinite(x); }
BM_HD bool isfinf(float x) { return __builtin_isfinite(x); }

// ------------------------------------------------------------------ fdlibm atan / atan2 / acos
BM_HD double atan_(double x) {
    if (x != x) return x;
    const bool neg = x < 0.0;
    double ax = neg ? -x : x;
    if (ax >= 3.6893488147419103e+19) {
        const double r = 1.57079632679489655800e+00 + 6.12323399573676603587e-17;
        return neg ? -r : r;
    }
    int id;
    if (ax < 0.4375) {
        if (ax < 1.862645149230957e-09) return x;
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
    const double s1 = z * (3.33333333333329318027e-01 +
                      w * (1.42857142725034663711e-01 +
                      w * (9.09088713343650656196e-02 +
                      w * (6.66107313738753120669e-02 +
                      w * (4.97687799461593236017e-02 +
                      w * 1.62858201153657823623e-02)))));
    const double s2 = w * (-1.99999999998764832476e-01 +
                      w * (-1.11111104054623557880e-01 +
                      w * (-7.69187620504482999495e-02 +
                      w * (-5.83357013379057348645e-02 +
                      w * -3.65315727442169155270e-02))));
    if (id < 0) {
        const double r = ax - ax * (s1 + s2);
        return neg ? -r : r;
    }
    double hi, lo;
    switch (id) {
        case 0: hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17; break;
        case 1: hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17; break;
        case 2: hi = 9.82793723247329054082e-01; lo = 1.39033110312309984516e-17; break;
        default: hi = 1.57079632679489655800e+00; lo = 6.12323399573676603587e-17; break;
    }
    const double r = hi - ((ax * (s1 + s2) - lo) - ax);
    return neg ? -r : r;
}

BM_HD double atan2_(double y, double x) {
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    const double pio2 = 1.57079632679489655800e+00;
    if (x != x || y != y) return x + y;
    if (y == 0.0) {
        if (__builtin_signbit(x)) return __builtin_signbit(y) ? -pi : pi;
        return y;
    }
    if (x == 0.0) return y < 0.0 ? -pio2 : pio2;
    if (__builtin_isinf(x)) {
        if (__builtin_isinf(y)) {
            const double r = x > 0 ? pio2 * 0.5 : 3.0 * pio2 * 0.5;
            return y < 0 ? -r : r;
        }
        const double r = x > 0 ? 0.0 : pi;
        return y < 0 ? -r : r;
    }
    if (__builtin_isinf(y)) return y < 0 ? -pio2 : pio2;
    double z = atan_(dabs(y / x));
    if (x > 0.0) return y < 0 ? -z : z;
    z = pi - (z - pi_lo);
    return y < 0 ? -z : z;
}

BM_HD double acos_R(double z) {
    const double p = z * (1.66666666666666657415e-01 +
                     z * (-3.25565818622400915405e-01 +
                     z * (2.01212532134862925881e-01 +
                     z * (-4.00555345006794114027e-02 +
                     z * (7.91534994289814532176e-04 +
                     z * 3.47933107596021167570e-05)))));
    const double q = 1.0 + z * (-2.40339491173441421878e+00 +
                           z * (2.02094576023350569471e+00 +
                           z * (-6.88283971605453293030e-01 +
                           z * 7.70381505559019352791e-02)));
    return p / q;
}

BM_HD double acos_(double x) {
    const double pi = 3.14159265358979311600e+00;
    const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
    if (x != x) return x;
    const double ax = dabs(x);
    if (ax >= 1.0) {
        if (ax == 1.0) return x > 0.0 ? 0.0 : pi + 2.0 * pio2_lo;
        return __builtin_nan("");
    }
    if (ax < 0.5) {
        if (ax <= 6.938893903907228e-18) return pio2_hi + pio2_lo;
        const double r = acos_R(x * x);
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if (x < 0.0) {
        const double z = (1.0 + x) * 0.5;
        const double s = dsqrt(z);
        const double w = acos_R(z) * s - pio2_lo;
        return pi - 2.0 * (s + w);
    }
    const double z = (1.0 - x) * 0.5;
    const double s = dsqrt(z);
    const double df = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, s) & 0xFFFFFFFF00000000ull);
    const double c = (z - df * df) / (s + df);
    const double w = acos_R(z) * s + c;
    return 2.0 * (df + w);
}

// Select forms of atan_ / atan2_ / acos_ for a wavefront whose lanes take different fdlibm ranges:
// every range's operands are formed by selects and ONE division (one rational polynomial) serves all
// lanes, where the branchy forms run every taken range's division and polynomial in turn. Each lane
// evaluates exactly the expression its branch evaluates (same operands, same operation order), so
// the results are bit-identical to atan_ / atan2_ / acos_ for the arguments they are used with:
// atan_sel and atan2_sel for finite, not-both-zero (y, x), acos_sel for x in [-1, 1] (PCL's SHOT
// clamps the inclination cosine; csrc/describe2.hip shot_records_of).
BM_HD double atan_sel(double x) {
    const bool neg = x < 0.0;
    const double ax = neg ? -x : x;
    const int id = ax < 0.4375 ? -1 : ax < 0.6875 ? 0 : ax < 1.1875 ? 1 : ax < 2.4375 ? 2 : 3;
    // id -1: ax / 1.0 == ax exactly
    const double num = id < 0 ? ax : id == 0 ? 2.0 * ax - 1.0 : id == 1 ? ax - 1.0 : id == 2 ? ax - 1.5 : -1.0;
    const double den = id < 0 ? 1.0 : id == 0 ? 2.0 + ax : id == 1 ? ax + 1.0 : id == 2 ? 1.0 + 1.5 * ax : ax;
    const double t = num / den;
    const double z = t * t;
    const double w = z * z;
    const double s1 = z * (3.33333333333329318027e-01 +
                      w * (1.42857142725034663711e-01 +
                      w * (9.09088713343650656196e-02 +
                      w * (6.66107313738753120669e-02 +
                      w * (4.97687799461593236017e-02 +
                      w * 1.62858201153657823623e-02)))));
    const double s2 = w * (-1.99999999998764832476e-01 +
                      w * (-1.11111104054623557880e-01 +
                      w * (-7.69187620504482999495e-02 +
                      w * (-5.83357013379057348645e-02 +
                      w * -3.65315727442169155270e-02))));
    const double hi = id == 0 ? 4.63647609000806093515e-01 : id == 1 ? 7.85398163397448278999e-01
                    : id == 2 ? 9.82793723247329054082e-01 : 1.57079632679489655800e+00;
    const double lo = id == 0 ? 2.26987774529616870924e-17 : id == 1 ? 3.06161699786838301793e-17
                    : id == 2 ? 1.39033110312309984516e-17 : 6.12323399573676603587e-17;
    double r = id < 0 ? t - t * (s1 + s2) : hi - ((t * (s1 + s2) - lo) - t);
    if (id < 0 && ax < 1.862645149230957e-09) r = ax;
    if (ax >= 3.6893488147419103e+19) r = 1.57079632679489655800e+00 + 6.12323399573676603587e-17;
    return neg ? -r : r;
}

BM_HD double atan2_sel(double y, double x) {
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    const double pio2 = 1.57079632679489655800e+00;
    const double z = atan_sel(dabs(y / x));
    double r = x > 0.0 ? z : pi - (z - pi_lo);
    r = y < 0 ? -r : r;
    if (x == 0.0) r = y < 0.0 ? -pio2 : pio2;
    if (y == 0.0) r = __builtin_signbit(x) ? (__builtin_signbit(y) ? -pi : pi) : y;
    return r;
}

BM_HD double acos_sel(double x) {
    const double pi = 3.14159265358979311600e+00;
    const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
    const double ax = dabs(x);
    const bool small = ax < 0.5, neg = x < 0.0;
    const double z = small ? x * x : neg ? (1.0 + x) * 0.5 : (1.0 - x) * 0.5;
    const double R = acos_R(z);
    const double s = dsqrt(z);
    const double df = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, s) & 0xFFFFFFFF00000000ull);
    const double c = (z - df * df) / (s + df);
    double r = small ? pio2_hi - (x - (pio2_lo - x * R)) : neg ? pi - 2.0 * (s + (R * s - pio2_lo)) : 2.0 * (df + (R * s + c));
    if (ax <= 6.938893903907228e-18) r = pio2_hi + pio2_lo;
    if (ax >= 1.0) r = ax == 1.0 ? (x > 0.0 ? 0.0 : pi + 2.0 * pio2_lo) : __builtin_nan("");
    return r;
}

BM_HD double cos_s(double x) {
    const double z = x * x;
    double r = 1.0 / 620448401733239439360000.0;
    r = r * z - 1.0 / 1124000727777607680000.0;
    r = r * z + 1.0 / 2432902008176640000.0;
    r = r * z - 1.0 / 6402373705728000.0;
    r = r * z + 1.0 / 20922789888000.0;
    r = r * z - 1.0 / 87178291200.0;
    r = r * z + 1.0 / 479001600.0;
    r = r * z - 1.0 / 3628800.0;
    r = r * z + 1.0 / 40320.0;
    r = r * z - 1.0 / 720.0;
    r = r * z + 1.0 / 24.0;
    r = r * z - 0.5;
    r = r * z + 1.0;
    return r;
}

BM_HD double sin_s(double x) {
    const double z = x * x;
    double r = 1.0 / 25852016738884976640000.0;
    r = r * z - 1.0 / 51090942171709440000.0;
    r = r * z + 1.0 / 121645100408832000.0;
    r = r * z - 1.0 / 355687428096000.0;
    r = r * z + 1.0 / 1307674368000.0;
    r = r * z - 1.0 / 6227020800.0;
    r = r * z + 1.0 / 39916800.0;
    r = r * z - 1.0 / 362880.0;
    r = r * z + 1.0 / 5040.0;
    r = r * z - 1.0 / 120.0;
    r = r * z + 1.0 / 6.0;
    return x - x * (z * r);
}

// ------------------------------------------------------------------ pcl::eigen33 (float)
BM_HD void computeRoots2(float b, float c, float roots[3]) {
    roots[0] = 0.0f;
    float d = (float)((double)(b * b) - 4.0 * (double)c);
    if (d < 0.0f) d = 0.0f;
    const float sd = fsqrt(d);
    roots[2] = 0.5f * (b + sd);
    roots[1] = 0.5f * (b - sd);
}

BM_HD void computeRoots(const float m[9], float roots[3]) {
    const float m00 = m[0], m01 = m[1], m02 = m[2], m11 = m[4], m12 = m[5], m22 = m[8];
    const float c0 = ((((m00 * m11) * m22 + ((2.0f * m01) * m02) * m12) - (m00 * m12) * m12) -
                      (m11 * m02) * m02) - (m22 * m01) * m01;
    const float c1 = ((((m00 * m11 - m01 * m01) + m00 * m22) - m02 * m02) + m11 * m22) - m12 * m12;
    const float c2 = (m00 + m11) + m22;
    if (fabs_(c0) < 1.19209290e-07f) {
        computeRoots2(c2, c1, roots);
        return;
    }
    const float s_inv3 = (float)(1.0 / 3.0);
    const float s_sqrt3 = fsqrt(3.0f);
    const float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > 0.0f) a_over_3 = 0.0f;
    const float half_b = 0.5f * (c0 + c2_over_3 * (((2.0f * c2_over_3) * c2_over_3) - c1));
    float q = half_b * half_b + (a_over_3 * a_over_3) * a_over_3;
    if (q > 0.0f) q = 0.0f;
    const float rho = fsqrt(-a_over_3);
    const float theta = (float)atan2_((double)fsqrt(-q), (double)half_b) * s_inv3;
    const float cos_theta = (float)cos_s((double)theta);
    const float sin_theta = (float)sin_s((double)theta);
    roots[0] = c2_over_3 + (2.0f * rho) * cos_theta;
    roots[1] = c2_over_3 - rho * (cos_theta + s_sqrt3 * sin_theta);
    roots[2] = c2_over_3 - rho * (cos_theta - s_sqrt3 * sin_theta);
    float t;
    if (roots[0] >= roots[1]) { t = roots[0]; roots[0] = roots[1]; roots[1] = t; }
    if (roots[1] >= roots[2]) {
        t = roots[1]; roots[1] = roots[2]; roots[2] = t;
        if (roots[0] >= roots[1]) { t = roots[0]; roots[0] = roots[1]; roots[1] = t; }
    }
    if (roots[0] <= 0.0f) computeRoots2(c2, c1, roots);
}

BM_HD float scale_of(const float m[9]) {
    float s = fabs_(m[0]);
    for (int i = 1; i < 9; ++i) {
        const float a = fabs_(m[i]);
        if (a > s) s = a;
    }
    if (s <= 1.17549435e-38f) s = 1.0f;
    return s;
}

BM_HD void eigen33_min(const float mat[9], float* eigenvalue, float vec[3]) {
    const float scale = scale_of(mat);
    float sm[9];
    for (int i = 0; i < 9; ++i) sm[i] = mat[i] / scale;
    float ev[3];
    computeRoots(sm, ev);
    *eigenvalue = ev[0] * scale;
    sm[0] -= ev[0]; sm[4] -= ev[0]; sm[8] -= ev[0];
    const float v1x = sm[1] * sm[5] - sm[2] * sm[4], v1y = sm[2] * sm[3] - sm[0] * sm[5], v1z = sm[0] * sm[4] - sm[1] * sm[3];
    const float v2x = sm[1] * sm[8] - sm[2] * sm[7], v2y = sm[2] * sm[6] - sm[0] * sm[8], v2z = sm[0] * sm[7] - sm[1] * sm[6];
    const float v3x = sm[4] * sm[8] - sm[5] * sm[7], v3y = sm[5] * sm[6] - sm[3] * sm[8], v3z = sm[3] * sm[7] - sm[4] * sm[6];
    const float len1 = (v1x * v1x + v1y * v1y) + v1z * v1z;
    const float len2 = (v2x * v2x + v2y * v2y) + v2z * v2z;
    const float len3 = (v3x * v3x + v3y * v3y) + v3z * v3z;
    float x, y, z, len;
    if (len1 >= len2 && len1 >= len3) { x = v1x; y = v1y; z = v1z; len = len1; }
    else if (len2 >= len1 && len2 >= len3) { x = v2x; y = v2y; z = v2z; len = len2; }
    else { x = v3x; y = v3y; z = v3z; len = len3; }
    const float sl = fsqrt(len);
    vec[0] = x / sl; vec[1] = y / sl; vec[2] = z / sl;
}

BM_HD void eigen33_vals(const float mat[9], float evals[3]) {
    const float scale = scale_of(mat);
    float sm[9];
    for (int i = 0; i < 9; ++i) sm[i] = mat[i] / scale;
    computeRoots(sm, evals);
    evals[0] *= scale; evals[1] *= scale; evals[2] *= scale;
}

// ------------------------------------------------------------------ cyclic Jacobi (double)
// w ascending; eigenvectors as COLUMNS of row-major v[9].
BM_HD void jacobi_rot(double a[9], double v[9], int p, int q, int sweep) {
    const double apq = a[p * 3 + q];
    if (apq == 0.0) return;
    const double app = a[p * 3 + p], aqq = a[q * 3 + q];
    const double g = 100.0 * dabs(apq);
    if (sweep > 3 && dabs(app) + g == dabs(app) && dabs(aqq) + g == dabs(aqq)) {
        a[p * 3 + q] = 0.0;
        a[q * 3 + p] = 0.0;
        return;
    }
    const double theta = (aqq - app) / (2.0 * apq);
    double t;
    if (dabs(theta) > 1e150) {
        t = 0.5 / theta;
    } else {
        t = 1.0 / (dabs(theta) + dsqrt(theta * theta + 1.0));
        if (theta < 0.0) t = -t;
    }
    const double c = 1.0 / dsqrt(t * t + 1.0);
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

BM_HD void jacobi3(const double ain[9], double w[3], double v[9]) {
    double a[9];
    for (int i = 0; i < 9; ++i) a[i] = ain[i];
    for (int i = 0; i < 9; ++i) v[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 32; ++sweep) {
        const double off = dabs(a[1]) + dabs(a[2]) + dabs(a[5]);
        if (off == 0.0) break;
        jacobi_rot(a, v, 0, 1, sweep);
        jacobi_rot(a, v, 0, 2, sweep);
        jacobi_rot(a, v, 1, 2, sweep);
    }
    const double d0 = a[0], d1 = a[4], d2 = a[8];
    // stable ascending order of (d0, d1, d2)
    int i0 = 0, i1 = 1, i2 = 2;
    double e0 = d0, e1 = d1, e2 = d2;
    if (e1 < e0) { double t = e0; e0 = e1; e1 = t; int ti = i0; i0 = i1; i1 = ti; }
    if (e2 < e1) {
        double t = e1; e1 = e2; e2 = t; int ti = i1; i1 = i2; i2 = ti;
        if (e1 < e0) { t = e0; e0 = e1; e1 = t; ti = i0; i0 = i1; i1 = ti; }
    }
    w[0] = e0; w[1] = e1; w[2] = e2;
    double vv[9];
    for (int i = 0; i < 3; ++i) {
        vv[i * 3 + 0] = v[i * 3 + i0];
        vv[i * 3 + 1] = v[i * 3 + i1];
        vv[i * 3 + 2] = v[i * 3 + i2];
    }
    for (int i = 0; i < 9; ++i) v[i] = vv[i];
}

// ------------------------------------------------------------------ one-sided Jacobi SVD
template <typename T> BM_HD T tabs(T x) { return x < T(0) ? -x : x; }
template <typename T> BM_HD T tsqrt(T x);
template <> BM_HD double tsqrt<double>(double x) { return dsqrt(x); }
template <> BM_HD float tsqrt<float>(float x) { return fsqrt(x); }

template <typename T>
BM_HD void svd3(const T ain[9], T U[9], T s[3], T V[9]) {
    T a[9];
    for (int i = 0; i < 9; ++i) a[i] = ain[i];
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? T(1) : T(0);
    const T eps = sizeof(T) == 8 ? T(2.220446049250313e-16) : T(1.1920929e-07f);
    const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};
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
            if (tabs(gamma) <= eps * tsqrt(alpha * beta)) continue;
            rotated = true;
            const T zeta = (beta - alpha) / (T(2) * gamma);
            T t = T(1) / (tabs(zeta) + tsqrt(T(1) + zeta * zeta));
            if (zeta < T(0)) t = -t;
            const T c = T(1) / tsqrt(T(1) + t * t);
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
        nrm[j] = tsqrt(ss);
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
        T u0[3] = {U[0], U[3], U[6]};
        if (!(s[0] > T(0))) { u0[0] = T(1); u0[1] = T(0); u0[2] = T(0); U[0] = T(1); U[3] = T(0); U[6] = T(0); }
        T e[3] = {T(1), T(0), T(0)};
        if (tabs(u0[0]) > tabs(u0[1])) { e[0] = T(0); e[1] = T(1); }
        T u1[3] = {u0[1] * e[2] - u0[2] * e[1], u0[2] * e[0] - u0[0] * e[2], u0[0] * e[1] - u0[1] * e[0]};
        const T l = tsqrt((u1[0] * u1[0] + u1[1] * u1[1]) + u1[2] * u1[2]);
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
BM_HD T det3(const T m[9]) {
    return (m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6])) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// Rotation/translation from the cross-covariance path of Eigen::umeyama (no scaling).
// sigma: (1/n) * sum (dst_i - dm)(src_i - sm)^T, row-major; out row-major 4x4.
template <typename T>
BM_HD void umeyama_finish(const T sigma[9], const T sm[3], const T dm[3], T out[16]) {
    T U[9], S[3], V[9];
    svd3<T>(sigma, U, S, V);
    T d3 = T(1);
    if (det3<T>(U) * det3<T>(V) < T(0)) d3 = T(-1);
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

// Eigen::umeyama(src, dst, false) over n AoS points in precision T (host ICP/RANSAC and the GPU
// RANSAC scorer share it): sequential sums in point order for the means and the
// cross-covariance. The independent accumulators advance together in one loop (instruction-level
// parallelism); each one's own order of additions is the sequential one. out: row-major 4x4.
template <typename T>
BM_HD void umeyama_seq(const T* src, const T* dst, int n, T out[16]) {
    const T one_over_n = T(1) / T(n);
    T ss[3] = {src[0], src[1], src[2]}, ds[3] = {dst[0], dst[1], dst[2]};
    for (int i = 1; i < n; ++i) {
        const T* a = src + 3 * i;
        const T* b = dst + 3 * i;
        ss[0] = ss[0] + a[0]; ss[1] = ss[1] + a[1]; ss[2] = ss[2] + a[2];
        ds[0] = ds[0] + b[0]; ds[1] = ds[1] + b[1]; ds[2] = ds[2] + b[2];
    }
    T sm[3], dm[3];
    for (int d = 0; d < 3; ++d) {
        sm[d] = ss[d] * one_over_n;
        dm[d] = ds[d] * one_over_n;
    }
    T acc[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) acc[r * 3 + c] = (dst[r] - dm[r]) * (src[c] - sm[c]);
    for (int i = 1; i < n; ++i) {
        const T* a = src + 3 * i;
        const T* b = dst + 3 * i;
        const T s0 = a[0] - sm[0], s1 = a[1] - sm[1], s2 = a[2] - sm[2];
        const T d0 = b[0] - dm[0], d1 = b[1] - dm[1], d2 = b[2] - dm[2];
        acc[0] = acc[0] + d0 * s0; acc[1] = acc[1] + d0 * s1; acc[2] = acc[2] + d0 * s2;
        acc[3] = acc[3] + d1 * s0; acc[4] = acc[4] + d1 * s1; acc[5] = acc[5] + d1 * s2;
        acc[6] = acc[6] + d2 * s0; acc[7] = acc[7] + d2 * s1; acc[8] = acc[8] + d2 * s2;
    }
    T sigma[9];
    for (int r = 0; r < 9; ++r) sigma[r] = acc[r] * one_over_n;
    umeyama_finish<T>(sigma, sm, dm, out);
}

}  // namespace bm
