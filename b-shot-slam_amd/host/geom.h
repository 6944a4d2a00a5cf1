// geom.h -- host-side float/double 4x4 helpers with the operation orders of the Eigen/PCL calls
// they replace (DESIGN.md "Numerics conventions"). Row-major storage.
#pragma once
#include <cmath>
#include <cstring>

#include "../csrc/bshot_math.h"

namespace bg {

struct Mat4f {
    float m[16];
    static Mat4f identity() {
        Mat4f r;
        for (int i = 0; i < 16; ++i) r.m[i] = (i % 5 == 0) ? 1.f : 0.f;
        return r;
    }
};

// Eigen Matrix4f * Matrix4f: res(i,j) = ((a_i0 b_0j + a_i1 b_1j) + a_i2 b_2j) + a_i3 b_3j
inline Mat4f mul(const Mat4f& A, const Mat4f& B) {
    Mat4f R;
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            R.m[r * 4 + c] = ((A.m[r * 4] * B.m[c] + A.m[r * 4 + 1] * B.m[4 + c]) + A.m[r * 4 + 2] * B.m[8 + c]) +
                             A.m[r * 4 + 3] * B.m[12 + c];
    return R;
}

// pcl::transformPointCloud (PCL 1.8 scalar path): x' = ((m00 x + m01 y) + m02 z) + m03. out may alias p.
inline void xform(const Mat4f& T, const float* p, float* out) {
    const float x = p[0], y = p[1], z = p[2];
    out[0] = ((T.m[0] * x + T.m[1] * y) + T.m[2] * z) + T.m[3];
    out[1] = ((T.m[4] * x + T.m[5] * y) + T.m[6] * z) + T.m[7];
    out[2] = ((T.m[8] * x + T.m[9] * y) + T.m[10] * z) + T.m[11];
}

// Matrix4f::inverse(): adjugate / determinant evaluated in double, rounded to float.
inline Mat4f inverse(const Mat4f& M) {
    double m[16], v[16];
    for (int i = 0; i < 16; ++i) m[i] = M.m[i];
    v[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    v[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    v[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    v[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    v[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    v[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    v[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    v[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    v[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    v[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    v[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    v[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    v[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    v[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    v[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    v[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    const double det = m[0] * v[0] + m[1] * v[4] + m[2] * v[8] + m[3] * v[12];
    Mat4f R;
    for (int i = 0; i < 16; ++i) R.m[i] = (float)(v[i] / det);
    return R;
}

// Eigen::umeyama(src, dst, false) over n AoS points in precision T: sequential (rank-order) sums
// for the means and the cross-covariance, one-sided Jacobi SVD. Result rounded to float. The
// independent accumulators advance together in one loop (instruction-level parallelism); each
// one's own order of additions is the sequential one.
template <typename T>
inline Mat4f umeyama(const T* src, const T* dst, int n) {
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
    T out[16];
    bm::umeyama_finish<T>(sigma, sm, dm, out);
    Mat4f R;
    for (int i = 0; i < 16; ++i) R.m[i] = (float)out[i];
    return R;
}

}  // namespace bg
