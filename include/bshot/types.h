// types.h -- the small Eigen subset the reference API exposes (include/common_include.h:6-14),
// without Eigen (absent here): Vector3f, Matrix3f, Matrix4f with the operations the B-SHOT path
// uses (topRightCorner<3,1>, block<3,3>, inverse, products, dot, norm, sum, ==). Products follow
// the Eigen fixed-size evaluation order documented in DESIGN.md "Numerics conventions".
#pragma once
#include <cmath>
#include <cstring>
#include <vector>

namespace myslam {

struct Vector3f {
    float v[3];
    Vector3f() : v{0.f, 0.f, 0.f} {}
    Vector3f(float x, float y, float z) : v{x, y, z} {}
    float& operator[](int i) { return v[i]; }
    float operator[](int i) const { return v[i]; }
    float& operator()(int i) { return v[i]; }
    float operator()(int i) const { return v[i]; }
    Vector3f operator+(const Vector3f& o) const { return Vector3f(v[0] + o.v[0], v[1] + o.v[1], v[2] + o.v[2]); }
    Vector3f operator-(const Vector3f& o) const { return Vector3f(v[0] - o.v[0], v[1] - o.v[1], v[2] - o.v[2]); }
    Vector3f operator*(float s) const { return Vector3f(v[0] * s, v[1] * s, v[2] * s); }
    bool operator==(const Vector3f& o) const { return v[0] == o.v[0] && v[1] == o.v[1] && v[2] == o.v[2]; }
    // Eigen 3.2 reductions of a 3-vector (no packet access: DefaultTraversal, CompleteUnrolling)
    // go through redux_novec_unroller, which halves the range: a0 + (a1 + a2).
    float dot(const Vector3f& o) const { return v[0] * o.v[0] + (v[1] * o.v[1] + v[2] * o.v[2]); }
    float squaredNorm() const { return v[0] * v[0] + (v[1] * v[1] + v[2] * v[2]); }
    float norm() const { return std::sqrt(squaredNorm()); }
    float sum() const { return v[0] + (v[1] + v[2]); }
    static Vector3f Zero() { return Vector3f(); }
};

struct Matrix3f {
    float m[9];  // row-major
    Matrix3f() { for (int i = 0; i < 9; ++i) m[i] = (i % 4 == 0) ? 1.f : 0.f; }
    float& operator()(int r, int c) { return m[r * 3 + c]; }
    float operator()(int r, int c) const { return m[r * 3 + c]; }
    Vector3f operator*(const Vector3f& p) const {  // (m_i0 x + m_i1 y) + m_i2 z
        return Vector3f((m[0] * p[0] + m[1] * p[1]) + m[2] * p[2], (m[3] * p[0] + m[4] * p[1]) + m[5] * p[2],
                        (m[6] * p[0] + m[7] * p[1]) + m[8] * p[2]);
    }
    static Matrix3f Identity() { return Matrix3f(); }
};

struct Matrix4f {
    float m[16];  // row-major
    Matrix4f() { for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.f : 0.f; }
    static Matrix4f Identity() { return Matrix4f(); }
    float& operator()(int r, int c) { return m[r * 4 + c]; }
    float operator()(int r, int c) const { return m[r * 4 + c]; }
    Matrix4f operator*(const Matrix4f& B) const {
        Matrix4f R;
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c)
                R.m[r * 4 + c] = ((m[r * 4] * B.m[c] + m[r * 4 + 1] * B.m[4 + c]) + m[r * 4 + 2] * B.m[8 + c]) +
                                 m[r * 4 + 3] * B.m[12 + c];
        return R;
    }
    bool operator==(const Matrix4f& o) const { return std::memcmp(m, o.m, sizeof(m)) == 0; }
    Vector3f topRightCorner() const { return Vector3f(m[3], m[7], m[11]); }
    Matrix3f block33() const {
        Matrix3f R;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) R.m[r * 3 + c] = m[r * 4 + c];
        return R;
    }
    Matrix4f inverse() const;  // adjugate/determinant in double, rounded to float
    // R * p + t with the transformPointCloud order ((m00 x + m01 y) + m02 z) + m03
    Vector3f transformPoint(const Vector3f& p) const {
        return Vector3f(((m[0] * p[0] + m[1] * p[1]) + m[2] * p[2]) + m[3],
                        ((m[4] * p[0] + m[5] * p[1]) + m[6] * p[2]) + m[7],
                        ((m[8] * p[0] + m[9] * p[1]) + m[10] * p[2]) + m[11]);
    }
};

// build-owned replacement of pcl::PointCloud<pcl::PointXYZ> in the public API
typedef std::vector<Vector3f> PointCloudXYZ;

}  // namespace myslam
