// oracle_core.cpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.h). PARITY UNPINNED vs PCL.
// CPU restatement of the per-frame B-SHOT stages.
#include "oracle_core.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <random>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "oracle_api.h"
#include "oracle_math.h"

namespace orc {

static inline int64_t cell_key(int ix, int iy, int iz) {
    return ((int64_t)(ix + (1 << 20)) << 42) | ((int64_t)(iy + (1 << 20)) << 21) | (int64_t)(iz + (1 << 20));
}
static inline bool finite3(const P3& p) { return std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z); }

Grid::Grid(const P3* pts, int n, float cell) : pts_(pts), n_(n), cell_(cell) {
    std::vector<std::pair<int64_t, int>> keys;
    keys.reserve(n);
    for (int i = 0; i < n; ++i) {
        if (!finite3(pts[i])) continue;  // NaN/Inf points can never satisfy d2 < r2
        const int ix = (int)std::floor((double)pts[i].x / cell);
        const int iy = (int)std::floor((double)pts[i].y / cell);
        const int iz = (int)std::floor((double)pts[i].z / cell);
        keys.emplace_back(cell_key(ix, iy, iz), i);
    }
    std::sort(keys.begin(), keys.end());
    order_.resize(keys.size());
    for (size_t i = 0; i < keys.size(); ++i) {
        order_[i] = keys[i].second;
        if (i == 0 || keys[i].first != keys[i - 1].first) cells_[keys[i].first] = {(int)i, 0};
        cells_[keys[i].first].second++;
    }
}

void Grid::collect(const P3& q, float rr, float r2, std::vector<std::pair<float, int>>& out) const {
    // cube of cells covering [q-rr, q+rr] plus one cell margin (exactness does not depend on it)
    const int x0 = (int)std::floor(((double)q.x - rr) / cell_) - 1, x1 = (int)std::floor(((double)q.x + rr) / cell_) + 1;
    const int y0 = (int)std::floor(((double)q.y - rr) / cell_) - 1, y1 = (int)std::floor(((double)q.y + rr) / cell_) + 1;
    const int z0 = (int)std::floor(((double)q.z - rr) / cell_) - 1, z1 = (int)std::floor(((double)q.z + rr) / cell_) + 1;
    for (int ix = x0; ix <= x1; ++ix)
        for (int iy = y0; iy <= y1; ++iy)
            for (int iz = z0; iz <= z1; ++iz) {
                auto it = cells_.find(cell_key(ix, iy, iz));
                if (it == cells_.end()) continue;
                const int s = it->second.first, c = it->second.second;
                for (int j = 0; j < c; ++j) {
                    const int idx = order_[s + j];
                    const float d2 = d2_flann(q, pts_[idx]);
                    if (d2 < r2) out.emplace_back(d2, idx);
                }
            }
}

void Grid::radius_all(const P3& q, float r2, std::vector<std::pair<float, int>>& out) const {
    out.clear();
    if (!finite3(q)) return;
    collect(q, std::sqrt(r2), r2, out);
    std::sort(out.begin(), out.end());
}

void Grid::radius_knn(const P3& q, float r, int max_nn, std::vector<std::pair<float, int>>& out) const {
    out.clear();
    if (!finite3(q)) return;
    const float r2 = (float)((double)r * (double)r);
    // Exact shortcut: if >= max_nn points lie strictly inside a smaller radius rs, the max_nn
    // nearest (under (d2, idx) order) are all inside rs. Tried radii r/4, r/2, then r.
    for (int step = 0; step < 3; ++step) {
        const float rs = step == 0 ? r * 0.25f : (step == 1 ? r * 0.5f : r);
        const float rs2 = step == 2 ? r2 : (float)((double)rs * (double)rs);
        out.clear();
        collect(q, rs, rs2, out);
        if (step < 2 && (int)out.size() < max_nn) continue;
        if ((int)out.size() > max_nn) {
            std::nth_element(out.begin(), out.begin() + max_nn, out.end());
            out.resize(max_nn);
        }
        std::sort(out.begin(), out.end());
        return;
    }
}

// --------------------------------------------------------------------------------------------
// A1 segmentation ratio: src/lidar_odometry.cpp:53-126 (CV :83-97, CVS :98-108, CVSN :109-119)
static float seg_ratio_one(const P3* pts, const P3& sp, const std::vector<std::pair<float, int>>& nn, int sr_type) {
    // pcl::computeCentroid: float accumulation in result order, then / (float)n (:75-76)
    float cx = 0.f, cy = 0.f, cz = 0.f;
    for (const auto& e : nn) { cx += pts[e.second].x; cy += pts[e.second].y; cz += pts[e.second].z; }
    const float fn = (float)nn.size();
    cx = cx / fn; cy = cy / fn; cz = cz / fn;
    const float tx = sp.x - cx, ty = sp.y - cy, tz = sp.z - cz;  // ctvec = sp - ct (:79)
    if (sr_type == 0) {
        float pos = 0.f, neg = 0.f;
        for (const auto& e : nn) {
            const P3& p = pts[e.second];
            const float vx = p.x - sp.x, vy = p.y - sp.y, vz = p.z - sp.z;
            const float dot = tx * vx + (ty * vy + tz * vz);  // Vector3f::dot: Eigen redux a0 + (a1 + a2)
            if (dot > 0) pos += 1.0f;
            else if (dot < 0) neg += 1.0f;
        }
        return 1.0f - std::min(pos, neg) / std::max(pos, neg);
    }
    const float ctn = std::sqrt(tx * tx + (ty * ty + tz * tz));
    float sum = 0.f;
    for (const auto& e : nn) {
        const P3& p = pts[e.second];
        const float vx = p.x - sp.x, vy = p.y - sp.y, vz = p.z - sp.z;
        const float vn = std::sqrt(vx * vx + (vy * vy + vz * vz));
        if (ctn == 0.f || vn == 0.f) continue;
        const float dot = tx * vx + (ty * vy + tz * vz);
        if (sr_type == 1) sum += dot;
        else sum += dot / (ctn * vn);
    }
    return std::fabs(sum) / (float)nn.size();
}

}  // namespace orc

using namespace orc;

extern "C" {

// Threads for the per-point SR / ISS loops. 1 by default: the reference runs them single-threaded
// (src/lidar_odometry.cpp:61, :457), and bench.py's cpu_baseline keeps that. The golden-fixture
// generator raises it; every point is independent and the output is compacted in index order, so
// the results do not depend on the thread count.
static int g_point_threads = 1;

int oracle_seg_ratio(const float* xyz, int n, float radius, int max_nn, int sr_type, int32_t* idx_out,
                     float* ratio_out, int* n_out) {
    const P3* pts = reinterpret_cast<const P3*>(xyz);
    Grid g(pts, n, radius * 0.25f);
    std::vector<float> r_all(n > 0 ? n : 1);
    std::vector<uint8_t> ok(n > 0 ? n : 1, 0);
#pragma omp parallel num_threads(g_point_threads)
    {
        std::vector<std::pair<float, int>> nn;
#pragma omp for schedule(dynamic, 256)
        for (int i = 0; i < n; ++i) {
            const P3& sp = pts[i];
            if (sp.x == 0 && sp.y == 0 && sp.z == 0) continue;  // :63-64
            g.radius_knn(sp, radius, max_nn, nn);
            if (nn.empty()) continue;  // radiusSearch(...) > 0 (:70)
            const float r = seg_ratio_one(pts, sp, nn, sr_type);
            if (std::isnan(r)) continue;  // :121-122
            r_all[i] = r;
            ok[i] = 1;
        }
    }
    int m = 0;
    for (int i = 0; i < n; ++i)
        if (ok[i]) { idx_out[m] = i; ratio_out[m] = r_all[i]; ++m; }
    *n_out = m;
    return 0;
}

// A2: std::sort by ratio (unstable, libstdc++) + tail slice, src/lidar_odometry.cpp:49-50,131-153
int oracle_select_keypoints(const int32_t* idx, const float* ratio, int n, int k, int32_t* kp_idx, float* kp_ratio,
                            int* k_out) {
    std::vector<std::pair<int, float>> v(n);
    for (int i = 0; i < n; ++i) v[i] = {idx[i], ratio[i]};
    std::sort(v.begin(), v.end(), [](const std::pair<int, float>& l, const std::pair<int, float>& r) {
        return l.second < r.second;
    });
    const int start = n >= k ? n - k : 0;
    int m = 0;
    for (int i = start; i < n; ++i, ++m) { kp_idx[m] = v[i].first; kp_ratio[m] = v[i].second; }
    *k_out = m;
    return 0;
}

// A3: ISS (src/lidar_odometry.cpp:447-461 params; PCL ISSKeypoint3D::detectKeypoints, Appendix A.6)
int oracle_iss(const float* xyz, int n, float salient, float nonmax, double g21, double g32, int min_nn,
               int32_t* out_idx, int cap, int* n_out, double* third_eig) {
    const P3* pts = reinterpret_cast<const P3*>(xyz);
    std::vector<double> third(n, 0.0);
    {
        Grid g(pts, n, salient);
        const float r2 = (float)((double)salient * (double)salient);
#pragma omp parallel num_threads(g_point_threads)
        {
            std::vector<std::pair<float, int>> nn;
#pragma omp for schedule(dynamic, 256)
            for (int i = 0; i < n; ++i) {
                const P3& c = pts[i];
                if (!finite3(c)) continue;
                g.radius_all(c, r2, nn);
                if ((int)nn.size() < min_nn) continue;  // zero scatter -> NaN ratios -> rejected
                const double cx = c.x, cy = c.y, cz = c.z;
                double cov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                for (const auto& e : nn) {
                    const double d[3] = {(double)pts[e.second].x - cx, (double)pts[e.second].y - cy,
                                         (double)pts[e.second].z - cz};
                    for (int a = 0; a < 3; ++a)
                        for (int b = 0; b < 3; ++b) cov[a * 3 + b] += d[a] * d[b];
                }
                double w[3], v[9];
                o_jacobi3(cov, w, v);
                const double e1c = w[2], e2c = w[1], e3c = w[0];
                if (!std::isfinite(e1c) || !std::isfinite(e2c) || !std::isfinite(e3c)) continue;
                if (e3c < 0) continue;
                if ((e2c / e1c) < g21 && (e3c / e2c) < g32) third[i] = e3c;
            }
        }
    }
    int m = 0;
    {
        Grid g(pts, n, nonmax);
        const float r2 = (float)((double)nonmax * (double)nonmax);
        std::vector<uint8_t> keep(n > 0 ? n : 1, 0);
#pragma omp parallel num_threads(g_point_threads)
        {
            std::vector<std::pair<float, int>> nn;
#pragma omp for schedule(dynamic, 256)
            for (int i = 0; i < n; ++i) {
                if (!(third[i] > 0.0) || !finite3(pts[i])) continue;
                g.radius_all(pts[i], r2, nn);
                if ((int)nn.size() < min_nn) continue;
                bool is_max = true;
                for (const auto& e : nn)
                    if (third[i] < third[e.second]) { is_max = false; break; }
                keep[i] = is_max;
            }
        }
        for (int i = 0; i < n; ++i)
            if (keep[i]) {
                if (m < cap) out_idx[m] = i;
                ++m;
            }
    }
    if (third_eig)
        for (int i = 0; i < n; ++i) third_eig[i] = third[i];
    *n_out = m;
    return m <= cap ? 0 : -2;
}

// A4: normals, include/bshot_bits.h:43-94 (computePointNormal + flipNormalTowardsViewpoint).
// normals: N x 4 (nx, ny, nz, curvature) persistent array; slot k <- keypoint k (the reference's
// keypoint-index-into-surface-array behaviour, bshot_bits.h:59,65-86).
int oracle_normals(const float* xyz, int n, const float* kps, int k, float radius, int max_nn, float* normals) {
    const P3* pts = reinterpret_cast<const P3*>(xyz);
    const P3* kp = reinterpret_cast<const P3*>(kps);
    Grid g(pts, n, radius * 0.25f);
    const float qn = std::numeric_limits<float>::quiet_NaN();
    // NormalEstimationOMP (include/bshot_bits.h:62): keypoints are independent
#pragma omp parallel for schedule(dynamic, 8)
    for (int i = 0; i < std::min(k, n); ++i) {
        std::vector<std::pair<float, int>> nn;
        float* o = normals + 4 * i;
        if (!finite3(kp[i])) { o[0] = o[1] = o[2] = o[3] = qn; continue; }
        g.radius_knn(kp[i], radius, max_nn, nn);
        if (nn.empty()) { o[0] = o[1] = o[2] = o[3] = qn; continue; }
        float nx, ny, nz, curv;
        if (nn.size() < 3) {
            nx = ny = nz = curv = qn;
        } else {
            // pcl::computeMeanAndCovarianceMatrix (float, single pass, dense path)
            float acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (const auto& e : nn) {
                const P3& p = pts[e.second];
                acc[0] += p.x * p.x; acc[1] += p.x * p.y; acc[2] += p.x * p.z;
                acc[3] += p.y * p.y; acc[4] += p.y * p.z; acc[5] += p.z * p.z;
                acc[6] += p.x; acc[7] += p.y; acc[8] += p.z;
            }
            const float fn = (float)nn.size();
            for (int a = 0; a < 9; ++a) acc[a] = acc[a] / fn;
            float cov[9];
            cov[0] = acc[0] - acc[6] * acc[6];
            cov[1] = acc[1] - acc[6] * acc[7];
            cov[2] = acc[2] - acc[6] * acc[8];
            cov[4] = acc[3] - acc[7] * acc[7];
            cov[5] = acc[4] - acc[7] * acc[8];
            cov[8] = acc[5] - acc[8] * acc[8];
            cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
            float ev, vec[3];
            o_eigen33_min(cov, &ev, vec);
            nx = vec[0]; ny = vec[1]; nz = vec[2];
            const float eig_sum = (cov[0] + cov[4]) + cov[8];
            curv = (eig_sum != 0.f) ? std::fabs(ev / eig_sum) : 0.f;
        }
        // flipNormalTowardsViewpoint(kp, 0, 0, 0, ...)
        const float vx = 0.f - kp[i].x, vy = 0.f - kp[i].y, vz = 0.f - kp[i].z;
        const float cth = (vx * nx + vy * ny) + vz * nz;
        if (cth < 0) { nx *= -1; ny *= -1; nz *= -1; }
        o[0] = nx; o[1] = ny; o[2] = nz; o[3] = curv;
    }
    return 0;
}

}  // extern "C"

namespace orc {

static const double PST_RAD_45 = 0.78539816339744830961566084581988;
static const double PST_RAD_90 = 1.5707963267948966192313216916398;
static const double PST_RAD_135 = 2.3561944901923449288469825374596;
static const double PST_RAD_PI_7_8 = 2.7488935718910690836548129603691;

static inline float dot4f(float a0, float a1, float a2, float b0, float b1, float b2) {
    // Eigen Vector4f dot under SSE: (a0b0 + a2b2) + (a1b1 + a3b3), with a3 = b3 = 0
    return (a0 * b0 + a2 * b2) + (a1 * b1 + 0.0f);
}

// SHOT LRF: PCL SHOTLocalReferenceFrameEstimation::getLocalRF (Appendix A.4). rf row-major
// (x axis, y axis, z axis). Returns false when the LRF is NaN.
static bool lrf_one(const P3* pts, const P3& c, const std::vector<std::pair<float, int>>& nn, double R,
                    float rf[9]) {
    // Weighted covariance (PCL getLocalRF, double). PCL sums in kd-tree (unsorted) order, so the
    // summation order is a free convention; ours (DESIGN.md "Numerics"): neighbours in (d2, idx)
    // rank order, split into chunks of 64 ranks, each chunk reduced by the xor-butterfly tree
    // (offsets 32, 16, ..., 1; excluded ranks contribute 0), chunk sums added in chunk order.
    std::vector<double> vij;
    vij.reserve(nn.size() * 3);
    double tot[7] = {0, 0, 0, 0, 0, 0, 0};
    int valid = 0;
    const size_t nch = (nn.size() + 63) / 64;
    for (size_t ch = 0; ch < nch; ++ch) {
        double lane[64][7];
        for (int l = 0; l < 64; ++l) {
            for (int j = 0; j < 7; ++j) lane[l][j] = 0.0;
            const size_t r = ch * 64 + l;
            if (r >= nn.size()) continue;
            const P3& p = pts[nn[r].second];
            if (p.x == c.x && p.y == c.y && p.z == c.z) continue;
            const double vx = (double)(p.x - c.x), vy = (double)(p.y - c.y), vz = (double)(p.z - c.z);
            const double w = R - std::sqrt((double)nn[r].first);
            lane[l][0] = w * (vx * vx); lane[l][1] = w * (vx * vy); lane[l][2] = w * (vx * vz);
            lane[l][3] = w * (vy * vy); lane[l][4] = w * (vy * vz); lane[l][5] = w * (vz * vz);
            lane[l][6] = w;
            vij.push_back(vx); vij.push_back(vy); vij.push_back(vz);
            ++valid;
        }
        // butterfly: lane l and lane l^off both hold lane[l] + lane[l^off] (IEEE + commutes),
        // so halving in place gives lane 0's final value
        for (int off = 32; off > 0; off >>= 1)
            for (int l = 0; l < off; ++l)
                for (int j = 0; j < 7; ++j) lane[l][j] = lane[l][j] + lane[l + off][j];
        for (int j = 0; j < 7; ++j) tot[j] = tot[j] + lane[0][j];
    }
    const double sum = tot[6];
    double cov[9];
    cov[0] = tot[0]; cov[1] = tot[1]; cov[2] = tot[2];
    cov[4] = tot[3]; cov[5] = tot[4]; cov[8] = tot[5];
    cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
    if (valid < 5) return false;
    for (int a = 0; a < 9; ++a) cov[a] = cov[a] / sum;  // cov[3,6,7] mirror cov[1,2,5] exactly
    double ev[3], evec[9];
    o_jacobi3(cov, ev, evec);
    if (!std::isfinite(ev[0]) || !std::isfinite(ev[1]) || !std::isfinite(ev[2])) return false;
    double v1[3] = {evec[2], evec[5], evec[8]};  // largest -> x
    double v3[3] = {evec[0], evec[3], evec[6]};  // smallest -> z
    int plusT = 0, plusN = 0;
    for (int ne = 0; ne < valid; ++ne) {
        const double* r = &vij[ne * 3];
        if (((r[0] * v1[0] + r[1] * v1[1]) + r[2] * v1[2]) >= 0) plusT++;
        if (((r[0] * v3[0] + r[1] * v3[1]) + r[2] * v3[2]) >= 0) plusN++;
    }
    const int med = valid / 2;
    plusT = 2 * plusT - valid;
    if (plusT == 0) {
        for (int i = -2; i <= 2; ++i) {
            const double* r = &vij[(med - i) * 3];
            if (((r[0] * v1[0] + r[1] * v1[1]) + r[2] * v1[2]) > 0) plusT++;
        }
        if (plusT < 3) { v1[0] = -v1[0]; v1[1] = -v1[1]; v1[2] = -v1[2]; }
    } else if (plusT < 0) {
        v1[0] = -v1[0]; v1[1] = -v1[1]; v1[2] = -v1[2];
    }
    plusN = 2 * plusN - valid;
    if (plusN == 0) {
        for (int i = -2; i <= 2; ++i) {
            const double* r = &vij[(med - i) * 3];
            if (((r[0] * v3[0] + r[1] * v3[1]) + r[2] * v3[2]) > 0) plusN++;
        }
        if (plusN < 3) { v3[0] = -v3[0]; v3[1] = -v3[1]; v3[2] = -v3[2]; }
    } else if (plusN < 0) {
        v3[0] = -v3[0]; v3[1] = -v3[1]; v3[2] = -v3[2];
    }
    const float x0 = (float)v1[0], x1 = (float)v1[1], x2 = (float)v1[2];
    const float z0 = (float)v3[0], z1 = (float)v3[1], z2 = (float)v3[2];
    rf[0] = x0; rf[1] = x1; rf[2] = x2;
    rf[3] = z1 * x2 - z2 * x1; rf[4] = z2 * x0 - z0 * x2; rf[5] = z0 * x1 - z1 * x0;
    rf[6] = z0; rf[7] = z1; rf[8] = z2;
    return true;
}

// SHOT histogram: createBinDistanceShape + interpolateSingleChannel + normalizeHistogram
// (PCL shot.hpp, Appendix A.5); nr_shape_bins = 10, 32 sectors.
static void shot_hist_one(const P3* pts, const float* normals, const P3& c,
                          const std::vector<std::pair<float, int>>& nn, double R, const float rf[9], float* shot) {
    const int nr_bins = 10;
    const double r12 = R / 2, r34 = (R * 3) / 4, r14 = R / 4;
    for (int j = 0; j < 352; ++j) shot[j] = 0.0f;
    for (const auto& e : nn) {
        const float* nv = normals + 4 * e.second;
        if (!std::isfinite(nv[0]) || !std::isfinite(nv[1]) || !std::isfinite(nv[2])) continue;
        double cosd = (double)dot4f(nv[0], nv[1], nv[2], rf[6], rf[7], rf[8]);
        if (cosd > 1.0) cosd = 1.0;
        if (cosd < -1.0) cosd = -1.0;
        double bd = ((1.0 + cosd) * nr_bins) / 2;
        const P3& p = pts[e.second];
        const float dx = p.x - c.x, dy = p.y - c.y, dz = p.z - c.z;
        const double distance = std::sqrt((double)e.first);
        if (std::fabs(distance - 0.0) < 1e-15) continue;
        double xr = (double)dot4f(dx, dy, dz, rf[0], rf[1], rf[2]);
        double yr = (double)dot4f(dx, dy, dz, rf[3], rf[4], rf[5]);
        double zr = (double)dot4f(dx, dy, dz, rf[6], rf[7], rf[8]);
        if (std::fabs(yr) < 1E-30) yr = 0;
        if (std::fabs(xr) < 1E-30) xr = 0;
        if (std::fabs(zr) < 1E-30) zr = 0;
        const unsigned bit4 = ((yr > 0) || ((yr == 0.0) && (xr < 0))) ? 1u : 0u;
        const unsigned bit3 = ((xr > 0) || ((xr == 0.0) && (yr > 0))) ? (bit4 ? 0u : 1u) : bit4;
        int desc = (int)((bit4 << 3) + (bit3 << 2));
        desc = desc << 1;
        if ((xr * yr > 0) || (xr == 0.0)) desc += (std::fabs(xr) >= std::fabs(yr)) ? 0 : 4;
        else desc += (std::fabs(xr) > std::fabs(yr)) ? 4 : 0;
        desc += zr > 0 ? 1 : 0;
        desc += (distance > r12) ? 2 : 0;
        const int step = (int)std::floor(bd + 0.5);
        const int vol = desc * (nr_bins + 1);
        bd -= step;
        double w = (1 - std::fabs(bd));
        if (bd > 0) shot[vol + ((step + 1) % nr_bins)] += (float)bd;
        else shot[vol + ((step - 1 + nr_bins) % nr_bins)] += -(float)bd;
        if (distance > r12) {
            const double rd = (distance - r34) / r12;
            if (distance > r34) w += 1 - rd;
            else { w += 1 + rd; shot[(desc - 2) * (nr_bins + 1) + step] += (float)(-rd); }
        } else {
            const double rd = (distance - r14) / r12;
            if (distance < r14) w += 1 + rd;
            else { w += 1 - rd; shot[(desc + 2) * (nr_bins + 1) + step] += (float)rd; }
        }
        double ic = zr / distance;
        if (ic < -1.0) ic = -1.0;
        if (ic > 1.0) ic = 1.0;
        const double incl = o_acos(ic);
        if (incl > PST_RAD_90 || (std::fabs(incl - PST_RAD_90) < 1e-30 && zr <= 0)) {
            const double id = (incl - PST_RAD_135) / PST_RAD_90;
            if (incl > PST_RAD_135) w += 1 - id;
            else { w += 1 + id; shot[(desc + 1) * (nr_bins + 1) + step] -= (float)id; }
        } else {
            const double id = (incl - PST_RAD_45) / PST_RAD_90;
            if (incl < PST_RAD_45) w += 1 + id;
            else { w += 1 - id; shot[(desc - 1) * (nr_bins + 1) + step] += (float)id; }
        }
        if (yr != 0.0 || xr != 0.0) {
            const double az = o_atan2(yr, xr);
            const int sel = desc >> 2;
            double ad = (az - (-PST_RAD_PI_7_8 + PST_RAD_45 * sel)) / PST_RAD_45;
            ad = std::max(-0.5, std::min(ad, 0.5));
            if (ad > 0) {
                w += 1 - ad;
                shot[((desc + 4) % 32) * (nr_bins + 1) + step] += (float)ad;
            } else {
                w += 1 + ad;
                shot[((desc - 4 + 32) % 32) * (nr_bins + 1) + step] -= (float)ad;
            }
        }
        shot[vol + step] += (float)w;
    }
    double acc = 0;
    for (int j = 0; j < 352; ++j) acc += (double)(shot[j] * shot[j]);
    acc = std::sqrt(acc);
    const float fa = (float)acc;
    for (int j = 0; j < 352; ++j) shot[j] = shot[j] / fa;
}

}  // namespace orc

extern "C" {

// A5+A6: SHOT352 + LRF for K keypoints over surface cloud (include/bshot_bits.h:113-135).
int oracle_shot(const float* xyz, int n, const float* normals, const float* kps, int k, float radius, float* shot,
                float* rf_out) {
    const P3* pts = reinterpret_cast<const P3*>(xyz);
    const P3* kp = reinterpret_cast<const P3*>(kps);
    Grid g(pts, n, radius * 0.25f);
    const float r2 = (float)((double)radius * (double)radius);
    const double R = (double)radius;
    const float qn = std::numeric_limits<float>::quiet_NaN();
#pragma omp parallel
    {
        std::vector<std::pair<float, int>> nn;
#pragma omp for schedule(dynamic, 4)
        for (int i = 0; i < k; ++i) {
            float* s = shot + 352 * (size_t)i;
            float rf[9];
            g.radius_all(kp[i], r2, nn);
            bool ok = finite3(kp[i]) && lrf_one(pts, kp[i], nn, R, rf);
            if (!ok) for (int j = 0; j < 9; ++j) rf[j] = qn;
            if (!ok || nn.empty() || nn.size() < 5) {
                for (int j = 0; j < 352; ++j) s[j] = qn;
            } else {
                shot_hist_one(pts, normals, kp[i], nn, R, rf, s);
            }
            if (rf_out) for (int j = 0; j < 9; ++j) rf_out[9 * (size_t)i + j] = rf[j];
        }
    }
    return 0;
}

// A7: B-SHOT binarisation, include/bshot_bits.h:144-278. bits: K x 11 u32 (bit j -> word j/32).
int oracle_binarize(const float* shot, int k, uint32_t* bits) {
    for (int i = 0; i < k; ++i) {
        uint32_t* w = bits + 11 * (size_t)i;
        for (int q = 0; q < 11; ++q) w[q] = 0;
        for (int j = 0; j < 88; ++j) {
            const float* v = shot + 352 * (size_t)i + 4 * j;
            const float sum = ((v[0] + v[1]) + v[2]) + v[3];
            const double t = 0.9 * (double)sum;
            unsigned b;
            if (v[0] == 0 && v[1] == 0 && v[2] == 0 && v[3] == 0) b = 0;
            else if ((double)v[0] > t) b = 1;
            else if ((double)v[1] > t) b = 2;
            else if ((double)v[2] > t) b = 4;
            else if ((double)v[3] > t) b = 8;
            else if ((double)(v[0] + v[1]) > t) b = 3;
            else if ((double)(v[1] + v[2]) > t) b = 6;
            else if ((double)(v[2] + v[3]) > t) b = 12;
            else if ((double)(v[0] + v[3]) > t) b = 9;
            else if ((double)(v[1] + v[3]) > t) b = 10;
            else if ((double)(v[0] + v[2]) > t) b = 5;
            else if ((double)((v[0] + v[1]) + v[2]) > t) b = 7;
            else if ((double)((v[1] + v[2]) + v[3]) > t) b = 14;
            else if ((double)((v[0] + v[2]) + v[3]) > t) b = 13;
            else if ((double)((v[0] + v[1]) + v[3]) > t) b = 11;
            else b = 15;
            const int bit = 4 * j;
            w[bit / 32] |= b << (bit % 32);
        }
    }
    return 0;
}

// A9: brute-force Hamming matching with first-index argmin (minVect, include/bshot_bits.h:6-20;
// src/lidar_odometry.cpp:210-242).
int oracle_match(const uint32_t* a, int na, const uint32_t* b, int nb, int32_t* left, int32_t* right,
                 int32_t* corr_q, int32_t* corr_m, int* ncorr) {
    if (na <= 0 || nb <= 0) { *ncorr = 0; return na < 0 || nb < 0 ? -1 : 0; }
    auto ham = [](const uint32_t* x, const uint32_t* y) {
        int d = 0;
        for (int q = 0; q < 11; ++q) d += __builtin_popcount(x[q] ^ y[q]);
        return d;
    };
    for (int i = 0; i < na; ++i) {
        int best = ham(a + 11 * (size_t)i, b), bi = 0;
        for (int k = 1; k < nb; ++k) {
            const int d = ham(a + 11 * (size_t)i, b + 11 * (size_t)k);
            if (d < best) { best = d; bi = k; }
        }
        left[i] = bi;
    }
    for (int k = 0; k < nb; ++k) {
        int best = ham(b + 11 * (size_t)k, a), bi = 0;
        for (int i = 1; i < na; ++i) {
            const int d = ham(b + 11 * (size_t)k, a + 11 * (size_t)i);
            if (d < best) { best = d; bi = i; }
        }
        right[k] = bi;
    }
    int m = 0;
    for (int i = 0; i < na; ++i)
        if (right[left[i]] == i) { corr_q[m] = i; corr_m[m] = left[i]; ++m; }
    *ncorr = m;
    return 0;
}

}  // extern "C"

namespace orc {

// float transform of one point, PCL 1.8 transformPointCloud scalar path (Appendix A.9); T row-major
static inline P3 xform(const float T[16], const P3& p) {
    P3 o;
    o.x = ((T[0] * p.x + T[1] * p.y) + T[2] * p.z) + T[3];
    o.y = ((T[4] * p.x + T[5] * p.y) + T[6] * p.z) + T[7];
    o.z = ((T[8] * p.x + T[9] * p.y) + T[10] * p.z) + T[11];
    return o;
}

}  // namespace orc

extern "C" {

// A10: RANSAC correspondence rejection (src/lidar_odometry.cpp:251-261; PCL
// CorrespondenceRejectorSampleConsensus + RandomSampleConsensus + SampleConsensusModelRegistration,
// Appendix A.7). T_out row-major 4x4. Returns 1 if a model was found, 0 on the identity fallback.
int oracle_ransac(const float* src_xyz, int ns, const float* tgt_xyz, int nt, const int32_t* corr_q,
                  const int32_t* corr_m, int ncorr, int max_iter, double thresh, float* T_out, int32_t* inl_q,
                  int32_t* inl_m, int* n_inl) {
    const P3* src = reinterpret_cast<const P3*>(src_xyz);
    const P3* tgt = reinterpret_cast<const P3*>(tgt_xyz);
    (void)nt;
    auto fallback = [&]() {
        for (int i = 0; i < 16; ++i) T_out[i] = (i % 5 == 0) ? 1.f : 0.f;
        for (int i = 0; i < ncorr; ++i) { inl_q[i] = corr_q[i]; inl_m[i] = corr_m[i]; }
        *n_inl = ncorr;
        return 0;
    };
    std::vector<int> indices(corr_q, corr_q + ncorr);
    if ((int)indices.size() > ns) indices.clear();
    std::unordered_map<int, int> tgt_of;  // correspondences_ (source idx -> target idx)
    for (int i = 0; i < ncorr; ++i) tgt_of[corr_q[i]] = corr_m[i];
    // computeSampleDistanceThreshold(cloud, indices)
    double sample_thresh = 0.0;
    {
        float acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int id : indices) {
            const P3& p = src[id];
            acc[0] += p.x * p.x; acc[1] += p.x * p.y; acc[2] += p.x * p.z;
            acc[3] += p.y * p.y; acc[4] += p.y * p.z; acc[5] += p.z * p.z;
            acc[6] += p.x; acc[7] += p.y; acc[8] += p.z;
        }
        const float fn = (float)indices.size();
        for (int a = 0; a < 9; ++a) acc[a] = acc[a] / fn;
        float cov[9];
        cov[0] = acc[0] - acc[6] * acc[6]; cov[1] = acc[1] - acc[6] * acc[7]; cov[2] = acc[2] - acc[6] * acc[8];
        cov[4] = acc[3] - acc[7] * acc[7]; cov[5] = acc[4] - acc[7] * acc[8]; cov[8] = acc[5] - acc[8] * acc[8];
        cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
        float ev[3];
        o_eigen33_vals(cov, ev);
        const float ssum = (std::sqrt(ev[0]) + std::sqrt(ev[1])) + std::sqrt(ev[2]);
        sample_thresh = (double)ssum / 3.0;
        sample_thresh *= sample_thresh;
    }
    const int nidx = (int)indices.size();
    if (nidx < 3) return fallback();
    std::mt19937 rng(12345u);
    std::vector<int> shuffled = indices;
    auto is_good = [&](const int s[3]) {
        const P3 &a = src[s[0]], &b = src[s[1]], &c = src[s[2]];
        const float p10x = b.x - a.x, p10y = b.y - a.y, p10z = b.z - a.z;
        const float p20x = c.x - a.x, p20y = c.y - a.y, p20z = c.z - a.z;
        const float p21x = c.x - b.x, p21y = c.y - b.y, p21z = c.z - b.z;
        return (double)((p10x * p10x + p10y * p10y) + p10z * p10z) > sample_thresh &&
               (double)((p20x * p20x + p20y * p20y) + p20z * p20z) > sample_thresh &&
               (double)((p21x * p21x + p21y * p21y) + p21z * p21z) > sample_thresh;
    };
    const double thr2 = thresh * thresh;
    auto count_within = [&](const float T[16], std::vector<int>* inl) {
        int cnt = 0;
        for (int i = 0; i < nidx; ++i) {
            const P3 pt = xform(T, src[indices[i]]);
            const P3& q = tgt[tgt_of[indices[i]]];
            const float dx = pt.x - q.x, dy = pt.y - q.y, dz = pt.z - q.z;
            // Eigen Vector4f squaredNorm under SSE: (d0^2 + d2^2) + (d1^2 + d3^2), d3 = 0
            const float d2 = (dx * dx + dz * dz) + (dy * dy + 0.0f);
            if ((double)d2 < thr2) { ++cnt; if (inl) inl->push_back(indices[i]); }
        }
        return cnt;
    };
    int iterations = 0, best_cnt = -std::numeric_limits<int>::max();
    double k = 1.0;
    const double log_prob = std::log(1.0 - 0.99);
    const double one_over_indices = 1.0 / (double)nidx;
    unsigned skipped = 0;
    const unsigned max_skip = (unsigned)max_iter * 10;
    float best_T[16];
    bool have_model = false;
    while (iterations < k && skipped < max_skip) {
        int s[3];
        bool got = false;
        for (unsigned it = 0; it < 1000; ++it) {
            for (int i = 0; i < 3; ++i) {
                const unsigned r = rng() >> 1;
                std::swap(shuffled[i], shuffled[i + (int)(r % (unsigned)(nidx - i))]);
            }
            s[0] = shuffled[0]; s[1] = shuffled[1]; s[2] = shuffled[2];
            if (is_good(s)) { got = true; break; }
        }
        if (!got) break;
        double sd[9], td[9];
        for (int i = 0; i < 3; ++i) {
            const P3& a = src[s[i]];
            const P3& b = tgt[tgt_of[s[i]]];
            sd[i * 3] = a.x; sd[i * 3 + 1] = a.y; sd[i * 3 + 2] = a.z;
            td[i * 3] = b.x; td[i * 3 + 1] = b.y; td[i * 3 + 2] = b.z;
        }
        double Td[16];
        o_umeyama<double>(sd, td, 3, Td);
        float T[16];
        for (int i = 0; i < 16; ++i) T[i] = (float)Td[i];
        const int cnt = count_within(T, nullptr);
        if (cnt > best_cnt) {
            best_cnt = cnt;
            std::memcpy(best_T, T, sizeof(T));
            have_model = true;
            const double w = (double)best_cnt * one_over_indices;
            double p_no = 1.0 - std::pow(w, 3.0);
            p_no = std::max(std::numeric_limits<double>::epsilon(), p_no);
            p_no = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no);
            k = log_prob / std::log(p_no);
        }
        ++iterations;
        if (iterations > max_iter) break;
    }
    if (!have_model) return fallback();
    std::vector<int> inl;
    count_within(best_T, &inl);
    if (inl.size() < 3) return fallback();
    std::unordered_map<int, int> pos_of;
    for (int i = 0; i < ncorr; ++i) pos_of[corr_q[i]] = i;
    for (size_t i = 0; i < inl.size(); ++i) {
        const int p = pos_of[inl[i]];
        inl_q[i] = corr_q[p];
        inl_m[i] = corr_m[p];
    }
    *n_inl = (int)inl.size();
    std::memcpy(T_out, best_T, sizeof(best_T));
    return 1;
}

// A11: point-to-point ICP with PCL IterativeClosestPoint defaults (Appendix A.8);
// src already transformed by the initial guess (src/lidar_odometry.cpp:291-297).
int oracle_icp(const float* src_xyz, int ns, const float* tgt_xyz, int nt, int max_iter, float* T_final, int* iters) {
    const P3* tgt = reinterpret_cast<const P3*>(tgt_xyz);
    std::vector<P3> cur(reinterpret_cast<const P3*>(src_xyz), reinterpret_cast<const P3*>(src_xyz) + ns);
    float fin[16];
    for (int i = 0; i < 16; ++i) fin[i] = (i % 5 == 0) ? 1.f : 0.f;
    double prev_mse = std::numeric_limits<double>::max();
    int it = 0;
    std::vector<int> nn(ns);
    std::vector<float> nd(ns);
    std::vector<float> sbuf, tbuf;
    while (true) {
        if (nt <= 0 || ns < 3) break;
        for (int i = 0; i < ns; ++i) {
            float best = d2_flann(cur[i], tgt[0]);
            int bi = 0;
            for (int j = 1; j < nt; ++j) {
                const float d = d2_flann(cur[i], tgt[j]);
                if (d < best) { best = d; bi = j; }
            }
            nn[i] = bi;
            nd[i] = best;
        }
        sbuf.resize(3 * (size_t)ns);
        tbuf.resize(3 * (size_t)ns);
        for (int i = 0; i < ns; ++i) {
            sbuf[3 * i] = cur[i].x; sbuf[3 * i + 1] = cur[i].y; sbuf[3 * i + 2] = cur[i].z;
            tbuf[3 * i] = tgt[nn[i]].x; tbuf[3 * i + 1] = tgt[nn[i]].y; tbuf[3 * i + 2] = tgt[nn[i]].z;
        }
        float T[16];
        o_umeyama<float>(sbuf.data(), tbuf.data(), ns, T);
        for (int i = 0; i < ns; ++i) cur[i] = xform(T, cur[i]);
        float nf[16];
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c)
                nf[r * 4 + c] = ((T[r * 4] * fin[c] + T[r * 4 + 1] * fin[4 + c]) + T[r * 4 + 2] * fin[8 + c]) +
                                T[r * 4 + 3] * fin[12 + c];
        std::memcpy(fin, nf, sizeof(nf));
        ++it;
        // DefaultConvergenceCriteria::hasConverged
        if (it >= max_iter) break;
        const double cos_angle = 0.5 * (double)(((T[0] + T[5]) + T[10]) - 1.0f);
        const double tsq = (double)((T[3] * T[3] + T[7] * T[7]) + T[11] * T[11]);
        if (cos_angle >= 1.0 && tsq <= 0.0) break;
        double mse = 0;
        for (int i = 0; i < ns; ++i) mse += (double)nd[i];
        mse /= (double)ns;
        if (std::fabs(mse - prev_mse) < 1e-12) break;
        prev_mse = mse;
    }
    std::memcpy(T_final, fin, sizeof(fin));
    *iters = it;
    return 0;
}

}  // extern "C"

extern "C" {

int oracle_radius_search(const float* xyz, int n, const float* q, float radius, int max_nn, int32_t* idx, float* d2,
                         int cap) {
    const P3* pts = reinterpret_cast<const P3*>(xyz);
    Grid g(pts, n, radius * 0.25f);
    std::vector<std::pair<float, int>> nn;
    const P3 qq = {q[0], q[1], q[2]};
    if (max_nn > 0) g.radius_knn(qq, radius, max_nn, nn);
    else g.radius_all(qq, (float)((double)radius * (double)radius), nn);
    const int m = (int)nn.size();
    for (int i = 0; i < m && i < cap; ++i) { idx[i] = nn[i].second; d2[i] = nn[i].first; }
    return m;
}

void oracle_set_threads(int n) {
#ifdef _OPENMP
    omp_set_num_threads(n > 0 ? n : 1);
#else
    (void)n;
#endif
}

void oracle_set_point_threads(int n) { g_point_threads = n > 0 ? n : 1; }

int oracle_get_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void oracle_eig3(const double* a9, double* w3, double* v9) { o_jacobi3(a9, w3, v9); }

void oracle_umeyama(const double* src, const double* dst, int n, int use_float, double* T16) {
    if (use_float) {
        std::vector<float> s(3 * (size_t)n), d(3 * (size_t)n);
        for (int i = 0; i < 3 * n; ++i) { s[i] = (float)src[i]; d[i] = (float)dst[i]; }
        float T[16];
        o_umeyama<float>(s.data(), d.data(), n, T);
        for (int i = 0; i < 16; ++i) T16[i] = T[i];
    } else {
        o_umeyama<double>(src, dst, n, T16);
    }
}

}  // extern "C"
