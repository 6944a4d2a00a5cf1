// api.cpp -- Frame (src/frame.cpp), Keypoint (src/keypoint.cpp), Map (src/mymap.cpp) of the C++ API.
#include <algorithm>
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
// 1 m suppression cells: two keypoints closer than 800 mm are in the same or adjacent cells
static inline int sup_cell(float v) { return (int)std::floor(v / 1000.f); }
static inline uint64_t sup_key(int x, int y, int z) {
    return ((uint64_t)(uint32_t)(x + (1 << 20)) << 42) | ((uint64_t)(uint32_t)(y + (1 << 20)) << 21) |
           (uint64_t)(uint32_t)(z + (1 << 20));
}

void Map::addKeypoint(Keypoint::Ptr keypoint) {
    const Vector3f p = keypoint->getPosition();
    const unsigned long block_id = getBlockID(p);
    const int cx = sup_cell(p[0]), cy = sup_cell(p[1]), cz = sup_cell(p[2]);
    auto it = keypoints_.find(block_id);
    BlockAux& ax = aux_[block_id];
    if (it == keypoints_.end()) {
        Block kp_block;
        kp_block.insert(std::make_pair(p, keypoint));
        keypoints_.insert(std::make_pair(block_id, kp_block));
        ax.cells[sup_key(cx, cy, cz)].push_back(Cand{p, keypoint.get()});
        ax.dirty = true;
        return;
    }
    // src/mymap.cpp: rejected when any keypoint of the block lies within 800 mm with a segmentation
    // ratio >= this one's -- the same predicate over the same keypoints, visited by cell
    const float sr = keypoint->getSegRatio();
    // cells meeting the ball (801 mm: margin for the float norm's rounding): <= 2 per axis
    const int x0 = sup_cell(p[0] - 801.f), x1 = sup_cell(p[0] + 801.f);
    const int y0 = sup_cell(p[1] - 801.f), y1 = sup_cell(p[1] + 801.f);
    const int z0 = sup_cell(p[2] - 801.f), z1 = sup_cell(p[2] + 801.f);
    for (int gx = x0; gx <= x1; ++gx)
        for (int gy = y0; gy <= y1; ++gy)
            for (int gz = z0; gz <= z1; ++gz) {
                auto c = ax.cells.find(sup_key(gx, gy, gz));
                if (c == ax.cells.end()) continue;
                for (const Cand& e : c->second)
                    if ((p - e.p).norm() < 800 && sr <= e.kp->getSegRatio()) return;
            }
    std::vector<Cand>& mine = ax.cells[sup_key(cx, cy, cz)];
    const bool existed = it->second.find(p) != it->second.end();
    it->second[p] = keypoint;
    if (existed) {
        for (Cand& e : mine)
            if (e.p[0] == p[0] && e.p[1] == p[1] && e.p[2] == p[2]) e.kp = keypoint.get();
    } else {
        mine.push_back(Cand{p, keypoint.get()});
    }
    ax.dirty = true;
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
    auto append = [&](BlockMap::iterator it) {
        BlockAux& ax = aux_[it->first];
        if (ax.dirty) {
            // the block's iteration order, as the reference loop visits it
            ax.pos.clear();
            ax.desc.clear();
            ax.pos.reserve(it->second.size());
            ax.desc.reserve(it->second.size());
            for (auto& kp : it->second) {
                ax.pos.push_back(kp.first);
                ax.desc.push_back(kp.second->getDescriptor());
            }
            ax.dirty = false;
        }
        kpts_pos.insert(kpts_pos.end(), ax.pos.begin(), ax.pos.end());
        descriptors.insert(descriptors.end(), ax.desc.begin(), ax.desc.end());
    };
    if (x_max < x_min || y_max < y_min || z_max < z_min) return;
    const long long nx = (x_max - x_min) / prec + 1, ny = (y_max - y_min) / prec + 1, nz = (z_max - z_min) / prec + 1;
    const long long M = 0x1FFFFF, span = M + 1;
    if (query_mode_ == 0 && (long long)keypoints_.size() < nx * ny * nz && nx * prec < span && ny * prec < span &&
        nz * prec < span) {
        // Same blocks in the same order as the reference's x/y/z loop of lookups
        // (src/mymap.cpp:28-74), found by visiting the map's blocks instead: a loop position's
        // block id holds the low 21 bits of each coordinate (getBlockID), and with the box
        // narrower than 2^21 mm per axis at most one loop position has a block's 21-bit residues.
        auto slot = [&](long long r, int lo, long long cnt) -> long long {
            const long long d = (r - ((long long)lo & M)) & M;  // i * prec == d, both < 2^21
            if (d % prec) return -1;
            const long long i = d / prec;
            return i < cnt ? i : -1;
        };
        std::vector<std::pair<long long, BlockMap::iterator>> hits;
        for (auto it = keypoints_.begin(); it != keypoints_.end(); ++it) {
            const unsigned long long id = it->first;
            const long long i = slot((long long)((id >> 42) & M), x_min, nx);
            if (i < 0) continue;
            const long long j = slot((long long)((id >> 21) & M), y_min, ny);
            if (j < 0) continue;
            const long long k = slot((long long)(id & M), z_min, nz);
            if (k < 0) continue;
            hits.emplace_back((i * ny + j) * nz + k, it);
        }
        std::sort(hits.begin(), hits.end(),
                  [](const std::pair<long long, BlockMap::iterator>& a,
                     const std::pair<long long, BlockMap::iterator>& b) { return a.first < b.first; });
        for (auto& h : hits) append(h.second);
        return;
    }
    for (int x = x_min; x <= x_max; x += prec)
        for (int y = y_min; y <= y_max; y += prec)
            for (int z = z_min; z <= z_max; z += prec) {
                const unsigned long id = getBlockID(Vector3f((float)x, (float)y, (float)z));
                auto it = keypoints_.find(id);
                if (it == keypoints_.end()) continue;
                append(it);
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

int bshot_map_set_query_mode(bshot_map* m, int mode) {
    if (!m || mode < 0 || mode > 1) return BSHOT_EINVAL;
    m->m.setQueryMode(mode);
    return BSHOT_OK;
}

uint64_t bshot_map_block_id(const float* pos) {
    myslam::Map tmp;
    return (uint64_t)tmp.getBlockID(myslam::Vector3f(pos[0], pos[1], pos[2]));
}

}  // extern "C"
