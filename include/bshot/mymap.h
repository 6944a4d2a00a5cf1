// mymap.h -- myslam::Map, same containers, hasher and block scheme as the reference
// (include/mymap.h:9-51). Its std::unordered_map iteration order decides the target index order
// of matching, so it stays host C++ with libstdc++ containers.
// pcl::PointCloud<pcl::PointXYZ> in getKeypoints is replaced by PointCloudXYZ.
#pragma once
#include <cmath>
#include <cstdint>
#include <memory>
#include <unordered_map>
#include <vector>

#include "keypoint.h"
#include "types.h"

namespace myslam {

class Map {
  public:
    struct MapHasher {
        unsigned long operator()(const Vector3f& p) const {
            return (unsigned long)std::fabs(std::round(p.sum()));
        }
    };
    typedef std::shared_ptr<Map> Ptr;
    typedef std::unordered_map<Vector3f, Keypoint::Ptr, MapHasher> Block;
    typedef std::unordered_map<unsigned long, Block> BlockMap;
    typedef std::vector<Vector3f> KPointCloud;
    Map() {}

    void addKeypoint(Keypoint::Ptr keypoint);
    void getKeypoints(Vector3f pos, float range, PointCloudXYZ& kpts_pos, std::vector<bshot_descriptor>& descriptors);
    void getAllKeypoints(std::vector<Vector3f>& vec);
    void getBlockKeypoints(std::vector<KPointCloud>& kpc);
    unsigned long getBlockID(Vector3f pos);
    int size();
    // getKeypoints strategy (same output either way): 0 visits the map's blocks when that is
    // cheaper than the reference's 21^3 lookups, 1 always runs the lookup loop (tests)
    void setQueryMode(int mode) { query_mode_ = mode; }

  private:
    BlockMap keypoints_;
    int prec = 10000;  // map grid (mm)
    int query_mode_ = 0;

    // acceleration only (contents and iteration order of keypoints_ are untouched): per block, its
    // keypoints bucketed in 1 m cells for the 800 mm suppression test of addKeypoint, and a flat
    // copy of the block in iteration order for getKeypoints, rebuilt after the block changes
    struct Cand {
        Vector3f p;
        const Keypoint* kp;
    };
    struct BlockAux {
        std::unordered_map<uint64_t, std::vector<Cand>> cells;
        bool dirty = true;
        std::vector<Vector3f> pos;
        std::vector<bshot_descriptor> desc;
    };
    std::unordered_map<unsigned long, BlockAux> aux_;
};

}  // namespace myslam
