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

// Eigen::umeyama(src, dst, false) over n AoS points in precision T (bm::umeyama_seq), rounded to
// float.
template <typename T>
inline Mat4f umeyama(const T* src, const T* dst, int n) {
    T out[16];
    bm::umeyama_seq<T>(src, dst, n, out);
    Mat4f R;
    for (int i = 0; i < 16; ++i) R.m[i] = (float)out[i];
    return R;
}

}  // namespace bg
