// oracle_core.h -- TEST INFRASTRUCTURE ONLY. CPU restatement of the B-SHOT hot path of
// TingKaiChen/B-SHOT-SLAM (reference @ /root/reference). Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this code, and only as the checker / CPU baseline.
//
// PARITY UNPINNED: the reference cannot be built here (PCL/FLANN/Eigen absent) and
// ships no test, fixture or golden vector for this path. Each function cites the reference
// file:line it restates; the PCL/FLANN/Eigen internals follow SURVEY.md Appendix A with the
// conventions documented in DESIGN.md §"Numerics conventions".
#pragma once
#include <cstdint>
#include <utility>
#include <vector>
#include <unordered_map>

namespace orc {

struct P3 { float x, y, z; };

// Uniform hashed grid over a cloud (exact radius queries; FLANN result semantics:
// d2 = ((dx*dx + dy*dy) + dz*dz) in float, kept iff d2 < r2 (strict), sorted by (d2, index)).
class Grid {
  public:
    Grid(const P3* pts, int n, float cell);
    // all neighbours with d2 < r2 (sorted by (d2, idx))
    void radius_all(const P3& q, float r2, std::vector<std::pair<float, int>>& out) const;
    // the max_nn smallest (d2, idx) with d2 < r2, sorted
    void radius_knn(const P3& q, float r, int max_nn, std::vector<std::pair<float, int>>& out) const;

  private:
    void collect(const P3& q, float rr, float r2, std::vector<std::pair<float, int>>& out) const;
    const P3* pts_;
    int n_;
    float cell_;
    std::vector<int> order_;
    std::unordered_map<int64_t, std::pair<int, int>> cells_;
};

inline float d2_flann(const P3& q, const P3& p) {
    const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
    return (dx * dx + dy * dy) + dz * dz;
}

}  // namespace orc
