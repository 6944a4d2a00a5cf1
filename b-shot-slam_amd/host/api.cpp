// api.cpp -- Frame (src/frame.cpp), Keypoint (src/keypoint.cpp), Map (src/mymap.cpp) of the C++ API.
#include <bitset>
#include <cmath>

#include "../../include/bshot/frame.h"
#include "../../include/bshot/keypoint.h"
#include "../../include/bshot/mymap.h"
#include "geom.h"
#include "../../include/bshot_abi.h"

namespace myslam {

// ---------------------------------------------------------------- Frame (src/frame.cpp:3-64)
Frame::Frame()
    : id_(-1), timestamp_(-1), pointcloud_(nullptr), keypoints_(nullptr), descriptors_(nullptr), is_key_frame_(false) {}

Frame::Frame(long id, double time_stamp, Matrix4f T_c_w, PCPtr pc, PCPtr kps, DCPPtr dcpts, bool isKeyframe)
    : id_(id), timestamp_((long long)time_stamp), T_c_w_(T_c_w), pointcloud_(pc), keypoints_(kps),
      descriptors_(dcpts), is_key_frame_(isKeyframe) {}

Frame::~Frame() {}

Frame::Ptr Frame::createFrame() {
    static long factory_id = 0;
    return Frame::Ptr(new Frame(factory_id++));
}

void Frame::setTimestamp(const long long timestamp) { timestamp_ = timestamp; }
void Frame::setPose(const Matrix4f& T_c_w) { T_c_w_ = T_c_w; }
void Frame::setPointCloud(PCPtr pc) { pointcloud_ = pc; }
void Frame::setKeypoints(PCPtr kps) { keypoints_ = kps; }
void Frame::setDescriptors(DCPPtr dcpts) { descriptors_ = dcpts; }

Matrix4f Matrix4f::inverse() const {
    bg::Mat4f a;
    std::memcpy(a.m, m, sizeof(m));
    const bg::Mat4f r = bg::inverse(a);
    Matrix4f o;
    std::memcpy(o.m, r.m, sizeof(m));
    return o;
}

// ---------------------------------------------------------------- Keypoint (src/keypoint.cpp)
unsigned long Keypoint::factory_id_ = 0;

Keypoint::Keypoint() : id_(-1), pos_(Vector3f(0, 0, 0)) {}

Keypoint::Keypoint(unsigned long id, Vector3f& position, float& seg_ratio, bshot_descriptor& descriptor)
    : id_(id), pos_(position), seg_ratio_(seg_ratio), descriptor_(descriptor) {}

Keypoint::Ptr Keypoint::createKeypoint(Vector3f& pos, float seg_ratio, bshot_descriptor descriptor) {
    const int prec = 10;  // 10 mm grid: int(trunc(p / prec)) * prec (src/keypoint.cpp:25-29)
    Vector3f grid_pos((float)((int)std::trunc(pos[0] / (float)prec) * prec),
                      (float)((int)std::trunc(pos[1] / (float)prec) * prec),
                      (float)((int)std::trunc(pos[2] / (float)prec) * prec));
    return std::make_shared<Keypoint>(factory_id_++, grid_pos, seg_ratio, descriptor);
}

// ---------------------------------------------------------------- Map (src/mymap.cpp)
void Map::addKeypoint(Keypoint::Ptr keypoint) {
    const unsigned long block_id = getBlockID(keypoint->getPosition());
    auto it = keypoints_.find(block_id);
    if (it == keypoints_.end()) {
        Block kp_block;
        kp_block.insert(std::make_pair(keypoint->getPosition(), keypoint));
        keypoints_.insert(std::make_pair(block_id, kp_block));
        return;
    }
    bool isCandidate = true;
    const Vector3f p = keypoint->getPosition();
    for (auto& kp : it->second) {
        if ((p - kp.first).norm() < 800 && keypoint->getSegRatio() <= kp.second->getSegRatio()) isCandidate = false;
    }
    if (isCandidate) it->second[p] = keypoint;
}

void Map::getKeypoints(Vector3f pos, float range, PointCloudXYZ& kpts_pos, std::vector<bshot_descriptor>& descriptors) {
    kpts_pos.clear();
    descriptors.clear();
    const int x_min = (int)std::round((pos[0] - range) / (float)prec) * prec;
    const int x_max = (int)std::round((pos[0] + range) / (float)prec) * prec;
    const int y_min = (int)std::round((pos[1] - range) / (float)prec) * prec;
    const int y_max = (int)std::round((pos[1] + range) / (float)prec) * prec;
    const int z_min = (int)std::round((pos[2] - range) / (float)prec) * prec;
    const int z_max = (int)std::round((pos[2] + range) / (float)prec) * prec;
    for (int x = x_min; x <= x_max; x += prec)
        for (int y = y_min; y <= y_max; y += prec)
            for (int z = z_min; z <= z_max; z += prec) {
                auto it = keypoints_.find(getBlockID(Vector3f((float)x, (float)y, (float)z)));
                if (it == keypoints_.end()) continue;
                kpts_pos.reserve(kpts_pos.size() + it->second.size());
                descriptors.reserve(descriptors.size() + it->second.size());
                for (auto& kp : it->second) {
                    kpts_pos.push_back(kp.first);
                    descriptors.push_back(kp.second->getDescriptor());
                }
            }
}

void Map::getAllKeypoints(std::vector<Vector3f>& vec) {
    vec.clear();
    for (auto& block : keypoints_)
        for (auto& kp : block.second) vec.push_back(kp.first);
}

int Map::size() {
    int count = 0;
    for (auto& block : keypoints_) count += (int)block.second.size();
    return count;
}

unsigned long Map::getBlockID(Vector3f pos) {
    // 64-bit key = low 21 bits of each 10 m grid coordinate (src/mymap.cpp:95-105)
    const int gx = (int)(float)((int)std::round(pos[0] / (float)prec) * prec);
    const int gy = (int)(float)((int)std::round(pos[1] / (float)prec) * prec);
    const int gz = (int)(float)((int)std::round(pos[2] / (float)prec) * prec);
    const uint64_t i = ((uint64_t)(int64_t)gx << 42) & ((uint64_t)0x1FFFFF << 42);
    const uint64_t j = ((uint64_t)(int64_t)gy << 21) & ((uint64_t)0x1FFFFF << 21);
    const uint64_t k = ((uint64_t)(int64_t)gz) & (uint64_t)0x1FFFFF;
    return (unsigned long)(i | j | k);
}

void Map::getBlockKeypoints(std::vector<KPointCloud>& kpc) {
    for (auto& block : keypoints_) {
        KPointCloud temp;
        temp.reserve(block.second.size());
        for (auto& kp : block.second) temp.push_back(kp.first);
        kpc.push_back(temp);
    }
}

}  // namespace myslam

// ---------------------------------------------------------------- host-only Map C ABI
struct bshot_map {
    myslam::Map m;
};

extern "C" {

bshot_map* bshot_map_create(void) { return new bshot_map(); }
void bshot_map_destroy(bshot_map* m) { delete m; }

int bshot_map_add(bshot_map* m, const float* xyz, float ratio, const uint32_t* bits11) {
    if (!m || !xyz || !bits11) return BSHOT_EINVAL;
    myslam::Vector3f p(xyz[0], xyz[1], xyz[2]);
    bshot_descriptor d;
    d.bits = myslam::words_to_bits(bits11);
    m->m.addKeypoint(myslam::Keypoint::createKeypoint(p, ratio, d));
    return BSHOT_OK;
}

int bshot_map_query(bshot_map* m, const float* pos, float range, float* xyz, uint32_t* bits, int cap) {
    if (!m || !pos) return BSHOT_EINVAL;
    myslam::PointCloudXYZ k;
    std::vector<bshot_descriptor> d;
    m->m.getKeypoints(myslam::Vector3f(pos[0], pos[1], pos[2]), range, k, d);
    const int n = (int)k.size();
    if (n > cap) return -n;
    for (int i = 0; i < n; ++i) {
        if (xyz) { xyz[3 * i] = k[i][0]; xyz[3 * i + 1] = k[i][1]; xyz[3 * i + 2] = k[i][2]; }
        if (bits) myslam::bits_to_words(d[i].bits, bits + 11 * (size_t)i);
    }
    return n;
}

int bshot_map_size(bshot_map* m) { return m ? m->m.size() : 0; }

uint64_t bshot_map_block_id(const float* pos) {
    myslam::Map tmp;
    return (uint64_t)tmp.getBlockID(myslam::Vector3f(pos[0], pos[1], pos[2]));
}

}  // extern "C"
