// oracle_odom.cpp -- TEST INFRASTRUCTURE ONLY. PARITY UNPINNED vs PCL (see oracle_core.h).
// CPU restatement of the per-frame odometry loop: LidarOdometry (src/lidar_odometry.cpp:29-445),
// Keypoint (src/keypoint.cpp:23-32), Map (include/mymap.h:9-51, src/mymap.cpp:4-105) and the
// headless frame loop of test/odometry_test.cpp:159-180 / test/kp_test.cpp:159-181.
#include <algorithm>
#include <bitset>
#include <cmath>
#include <cstring>
#include <limits>
#include <memory>
#include <unordered_map>
#include <vector>

#include "oracle_api.h"
#include "oracle_core.h"
#include "oracle_math.h"

namespace orc {

struct V3 {
    float v[3];
    bool operator==(const V3& o) const { return v[0] == o.v[0] && v[1] == o.v[1] && v[2] == o.v[2]; }
};
struct Desc { uint32_t w[11]; };

struct Kp {
    V3 pos;
    float ratio;
    Desc d;
};

// Map::MapHasher (include/mymap.h:12-25): abs(round(p.sum())) on the float sum
struct MapHasher {
    unsigned long operator()(const V3& p) const {
        const float s = p.v[0] + (p.v[1] + p.v[2]);  // Eigen redux order a0 + (a1 + a2)
        return (unsigned long)std::fabs(std::round(s));
    }
};

class OMap {
  public:
    typedef std::unordered_map<V3, std::shared_ptr<Kp>, MapHasher> Block;
    const int prec = 10000;
    std::unordered_map<unsigned long, Block> blocks;
    // canonical order (the GPU map's mode 2, not the reference's): each block's keys in first-insert order
    bool canonical = false;
    std::unordered_map<unsigned long, std::vector<V3>> first_order;

    unsigned long block_id(const V3& p) const {  // src/mymap.cpp:95-105
        const float gx = (float)((int)std::round(p.v[0] / (float)prec) * prec);
        const float gy = (float)((int)std::round(p.v[1] / (float)prec) * prec);
        const float gz = (float)((int)std::round(p.v[2] / (float)prec) * prec);
        const uint64_t i = ((uint64_t)(int64_t)(int)gx << 42) & ((uint64_t)0x1FFFFF << 42);
        const uint64_t j = ((uint64_t)(int64_t)(int)gy << 21) & ((uint64_t)0x1FFFFF << 21);
        const uint64_t k = ((uint64_t)(int64_t)(int)gz) & (uint64_t)0x1FFFFF;
        return (unsigned long)(i | j | k);
    }
    void add(std::shared_ptr<Kp> kp) {  // src/mymap.cpp:4-26
        const unsigned long id = block_id(kp->pos);
        auto it = blocks.find(id);
        if (it == blocks.end()) {
            Block b;
            b.insert(std::make_pair(kp->pos, kp));
            blocks.insert(std::make_pair(id, b));
            if (canonical) first_order[id].push_back(kp->pos);
            return;
        }
        bool cand = true;
        for (auto& e : blocks[id]) {
            const float dx = kp->pos.v[0] - e.first.v[0], dy = kp->pos.v[1] - e.first.v[1],
                        dz = kp->pos.v[2] - e.first.v[2];
            if (std::sqrt(dx * dx + (dy * dy + dz * dz)) < 800 && kp->ratio <= e.second->ratio) cand = false;
        }
        if (cand) {
            if (canonical && blocks[id].find(kp->pos) == blocks[id].end()) first_order[id].push_back(kp->pos);
            blocks[id][kp->pos] = kp;
        }
    }
    void query(const V3& pos, float range, std::vector<P3>& kps, std::vector<Desc>& ds) {  // :28-74
        kps.clear();
        ds.clear();
        const int x_min = (int)std::round((pos.v[0] - range) / (float)prec) * prec;
        const int x_max = (int)std::round((pos.v[0] + range) / (float)prec) * prec;
        const int y_min = (int)std::round((pos.v[1] - range) / (float)prec) * prec;
        const int y_max = (int)std::round((pos.v[1] + range) / (float)prec) * prec;
        const int z_min = (int)std::round((pos.v[2] - range) / (float)prec) * prec;
        const int z_max = (int)std::round((pos.v[2] + range) / (float)prec) * prec;
        for (int x = x_min; x <= x_max; x += prec)
            for (int y = y_min; y <= y_max; y += prec)
                for (int z = z_min; z <= z_max; z += prec) {
                    const V3 c = {{(float)x, (float)y, (float)z}};
                    auto it = blocks.find(block_id(c));
                    if (it == blocks.end()) continue;
                    if (canonical) {
                        for (const V3& q : first_order[it->first]) {
                            kps.push_back({q.v[0], q.v[1], q.v[2]});
                            ds.push_back(it->second.find(q)->second->d);
                        }
                        continue;
                    }
                    for (auto& e : it->second) {
                        kps.push_back({e.first.v[0], e.first.v[1], e.first.v[2]});
                        ds.push_back(e.second->d);
                    }
                }
    }
    int size() const {
        int c = 0;
        for (auto& b : blocks) c += (int)b.second.size();
        return c;
    }
};

struct OFrame {
    std::vector<P3> pc;
    std::vector<P3> kps;
    std::vector<Desc> desc;
    float pose[16];
    OFrame() { for (int i = 0; i < 16; ++i) pose[i] = (i % 5 == 0) ? 1.f : 0.f; }
};

static void mul44(const float A[16], const float B[16], float C[16]) {  // Eigen Matrix4f product order
    float R[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            R[r * 4 + c] = ((A[r * 4] * B[c] + A[r * 4 + 1] * B[4 + c]) + A[r * 4 + 2] * B[8 + c]) + A[r * 4 + 3] * B[12 + c];
    std::memcpy(C, R, sizeof(R));
}

// general 4x4 inverse: cofactor expansion in double of the float matrix, rounded to float
static void inv44(const float Mf[16], float Out[16]) {
    double m[16], inv[16];
    for (int i = 0; i < 16; ++i) m[i] = Mf[i];
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    const double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    for (int i = 0; i < 16; ++i) Out[i] = (float)(inv[i] / det);
}

static inline P3 xf(const float T[16], const P3& p) {
    P3 o;
    o.x = ((T[0] * p.x + T[1] * p.y) + T[2] * p.z) + T[3];
    o.y = ((T[4] * p.x + T[5] * p.y) + T[6] * p.z) + T[7];
    o.z = ((T[8] * p.x + T[9] * p.y) + T[10] * p.z) + T[11];
    return o;
}

// 1-NN repeatability (kpEvaluation, src/lidar_odometry.cpp:392-445)
static float repeat_rate(const std::vector<P3>& src, const std::vector<P3>& ref) {
    if (src.empty()) return 0.f;
    float hit = 0.f;
    for (const P3& s : src) {
        if (s.x == 0 && s.y == 0 && s.z == 0) continue;
        float best = std::numeric_limits<float>::infinity();
        for (const P3& r : ref) best = std::min(best, d2_flann(s, r));
        if (!ref.empty() && best <= 900.f) hit += 1.f;
    }
    return hit / (float)src.size();
}

class OOdom {
  public:
    oracle_params p;
    bool initial = true;
    std::shared_ptr<OFrame> ref, src;
    std::vector<float> seg_ratios;
    std::vector<float> normals;  // persistent N x 4 (bshot_bits.h:59)
    OMap map;
    std::vector<P3> c2kps;
    std::vector<Desc> c2bits;
    std::vector<int32_t> inl_q, inl_m;
    std::vector<P3> iss_src, iss_ref;
    float ransac_T[16];
    float T_best[16];
#ifdef ORACLE_DIAG
    // diagnostic-only build (oracle/Makefile diag, never the product, never the parity oracle):
    // fix_normals computes the normal of every surface point (the evident intent of
    // include/bshot_bits.h:59-86, whose loop writes keypoint k's normal into surface slot k);
    // pose_override replaces the frame's estimated pose (kept in the stats) by a given one for
    // the pose and the map update, so a sequence can be replayed under ground-truth poses.
    int diag_fix_normals = 0;
    int diag_have_override = 0;
    float diag_override[16];
    std::vector<int32_t> mut_q, mut_m;
#endif

    explicit OOdom(const oracle_params& pp) : p(pp) {
        map.canonical = pp.map_canonical != 0;
        for (int i = 0; i < 16; ++i) ransac_T[i] = T_best[i] = (i % 5 == 0) ? 1.f : 0.f;
    }

    void pass_src2ref() { ref = src; iss_ref = iss_src; }

    void corr_stats(const float T[16], oracle_frame_stats* st) const {
        const size_t n = inl_q.size();
        st->corr_n = (int)n;
        if (n == 0) {
            st->corr_avg = st->corr_sd = st->corr_med = NAN;
            return;
        }
        std::vector<float> dv;
        dv.reserve(n);
        float avg = 0;
        for (size_t i = 0; i < n; ++i) {
            const P3 a = xf(T, src->kps[inl_q[i]]);
            const P3& b = c2kps[inl_m[i]];
            const float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
            dv.push_back(std::sqrt(dx * dx + (dy * dy + dz * dz)));
            avg += dv.back();
        }
        avg = avg / (float)n;
        float sd = 0;
        for (size_t i = 0; i < n; ++i) sd += (dv[i] - avg) * (dv[i] - avg);
        sd = std::sqrt(sd / (float)n);
        std::sort(dv.begin(), dv.end());
        st->corr_avg = avg;
        st->corr_sd = sd;
        st->corr_med = dv[n / 2];
    }

    int process(const float* xyz, int n, oracle_frame_stats* st) {
        std::memset(st, 0, sizeof(*st));
        auto f = std::make_shared<OFrame>();
        f->pc.assign(reinterpret_cast<const P3*>(xyz), reinterpret_cast<const P3*>(xyz) + n);
        if (!initial) pass_src2ref();
        src = f;
        st->n_points = n;
        // ---- extractKeypoints (src/lidar_odometry.cpp:51-171)
        std::vector<int32_t> idx(n), kidx(p.num_keypoints);
        std::vector<float> ratio(n), kr(p.num_keypoints);
        int nv = 0, k = 0;
        oracle_seg_ratio(xyz, n, p.seg_radius, p.seg_max_nn, p.sr_type, idx.data(), ratio.data(), &nv);
        oracle_select_keypoints(idx.data(), ratio.data(), nv, p.num_keypoints, kidx.data(), kr.data(), &k);
        st->n_valid_ratios = nv;
        st->n_keypoints = k;
        src->kps.resize(k);
        for (int i = 0; i < k; ++i) src->kps[i] = f->pc[kidx[i]];
        seg_ratios.assign(kr.begin(), kr.begin() + k);
        if (initial) pass_src2ref();
        iss_src.clear();
        if (p.run_iss) {
            std::vector<int32_t> iss(n > 0 ? n : 1);
            int ni = 0;
            oracle_iss(xyz, n, p.iss_salient, p.iss_nonmax, p.iss_gamma21, p.iss_gamma32, p.iss_min_nn, iss.data(), n,
                       &ni, nullptr);
            for (int i = 0; i < ni; ++i) iss_src.push_back(f->pc[iss[i]]);
        }
        st->n_iss = (int)iss_src.size();
        if (initial) iss_ref = iss_src;
        // ---- computeDescriptors (:173-184)
        normals.resize(4 * (size_t)n, 0.0f);  // std::vector::resize keeps [0, min) (persistent)
#ifdef ORACLE_DIAG
        if (diag_fix_normals)
            oracle_normals(xyz, n, xyz, n, p.normal_radius, p.normal_max_nn, normals.data());
        else
#endif
        oracle_normals(xyz, n, reinterpret_cast<const float*>(src->kps.data()), k, p.normal_radius, p.normal_max_nn,
                       normals.data());
        std::vector<float> shot(352 * (size_t)std::max(k, 1));
        oracle_shot(xyz, n, normals.data(), reinterpret_cast<const float*>(src->kps.data()), k, p.shot_radius,
                    shot.data(), nullptr);
        src->desc.resize(k);
        oracle_binarize(shot.data(), k, reinterpret_cast<uint32_t*>(src->desc.data()));
        // ---- featureMatching (:186-265)
        if (initial) {
            pass_src2ref();
            c2kps = ref->kps;
            c2bits = src->desc;
        } else {
            const V3 pos = {{ref->pose[3], ref->pose[7], ref->pose[11]}};
            map.query(pos, p.map_range, c2kps, c2bits);
            for (const P3& q : ref->kps) c2kps.push_back(xf(ref->pose, q));
            c2bits.insert(c2bits.end(), ref->desc.begin(), ref->desc.end());
        }
        const int m = (int)c2kps.size();
        st->n_target = m;
        std::vector<int32_t> left(std::max(k, 1)), right(std::max(m, 1)), cq(std::max(k, 1)), cm(std::max(k, 1));
        int nc = 0;
        oracle_match(reinterpret_cast<const uint32_t*>(src->desc.data()), k,
                     reinterpret_cast<const uint32_t*>(c2bits.data()), m, left.data(), right.data(), cq.data(),
                     cm.data(), &nc);
        st->n_mutual = nc;
#ifdef ORACLE_DIAG
        mut_q.assign(cq.begin(), cq.begin() + nc);
        mut_m.assign(cm.begin(), cm.begin() + nc);
#endif
        inl_q.assign(std::max(nc, 1), 0);
        inl_m.assign(std::max(nc, 1), 0);
        int ni = 0;
        oracle_ransac(reinterpret_cast<const float*>(src->kps.data()), k, reinterpret_cast<const float*>(c2kps.data()),
                      m, cq.data(), cm.data(), nc, p.ransac_max_iter, p.ransac_thresh, ransac_T, inl_q.data(),
                      inl_m.data(), &ni);
        inl_q.resize(ni);
        inl_m.resize(ni);
        st->n_inliers = ni;
        // ---- evaluateEstimation (:267-331)
        float Ti_inv[16], Tij[16];
        inv44(ref->pose, Ti_inv);
        mul44(Ti_inv, ransac_T, Tij);
        const float h_diff = std::acos(Tij[5]);
        const float t_diff = std::sqrt(Tij[3] * Tij[3] + (Tij[7] * Tij[7] + Tij[11] * Tij[11]));
        st->h_diff = h_diff;
        st->t_diff = t_diff;
        float T_est[16];
        if ((double)(h_diff * 180.f) / M_PI > 10 || t_diff > 1200 || ni < 15) {
            std::memcpy(T_est, ref->pose, sizeof(T_est));
            st->gated = 1;
        } else {
            std::memcpy(T_est, ransac_T, sizeof(T_est));
        }
        std::vector<P3> icp_src(k);
        for (int i = 0; i < k; ++i) icp_src[i] = xf(T_est, src->kps[i]);
        float Ticp[16];
        int iters = 0;
        oracle_icp(reinterpret_cast<const float*>(icp_src.data()), k, reinterpret_cast<const float*>(c2kps.data()), m,
                   p.icp_max_iter, Ticp, &iters);
        st->icp_iters = iters;
        if (p.run_icp) mul44(Ticp, T_est, T_best);
        else std::memcpy(T_best, ransac_T, sizeof(T_best));
        // ---- evaluate_corr_ (:303-330): corr = the RANSAC inliers (:260), corr_cloud = cloud1
        // keypoints under T_best_ (evaluate_icp_) or T_j; pcl::geometry::distance = Eigen norm of the
        // difference (a0 + (a1 + a2), then sqrt); float sums in corr order, divided by (float)size
        corr_stats(p.eval_icp ? T_best : ransac_T, st);
        // ---- kpEvaluation (kp_test only; cheap) (:392-445)
        st->repeat_sr = repeat_rate(src->kps, ref->kps);
        st->repeat_iss = repeat_rate(iss_src, iss_ref);
        // ---- poseEstimation (:333-342)
        std::memcpy(st->pose, T_best, sizeof(T_best));
#ifdef ORACLE_DIAG
        if (diag_have_override) {
            std::memcpy(T_best, diag_override, sizeof(T_best));
            diag_have_override = 0;
        }
#endif
        std::memcpy(src->pose, T_best, sizeof(T_best));
        // ---- updateMap (:344-376) with Keypoint::createKeypoint (src/keypoint.cpp:23-32)
        for (int i = 0; i < k; ++i) {
            const P3 w = xf(T_best, src->kps[i]);
            auto kp = std::make_shared<Kp>();
            kp->pos.v[0] = (float)((int)std::trunc(w.x / 10.f) * 10);
            kp->pos.v[1] = (float)((int)std::trunc(w.y / 10.f) * 10);
            kp->pos.v[2] = (float)((int)std::trunc(w.z / 10.f) * 10);
            kp->ratio = seg_ratios[i];
            kp->d = src->desc[i];
            map.add(kp);
        }
        initial = false;
        std::memcpy(st->T_ransac, ransac_T, sizeof(ransac_T));
        st->map_size = map.size();
        return 0;
    }
};

}  // namespace orc

using namespace orc;

extern "C" {

void oracle_default_params(oracle_params* p) {
    p->seg_radius = 3000.f; p->seg_max_nn = 300; p->sr_type = 0; p->num_keypoints = 600;
    p->iss_salient = 60.f; p->iss_nonmax = 40.f; p->iss_gamma21 = 0.975; p->iss_gamma32 = 0.975; p->iss_min_nn = 5;
    p->normal_radius = 3000.f; p->normal_max_nn = 300; p->shot_radius = 3000.f; p->map_range = 100000.f;
    p->ransac_max_iter = 2000; p->ransac_thresh = 1500.0; p->icp_max_iter = 10; p->run_icp = 1; p->run_iss = 1;
    p->map_canonical = 0; p->eval_icp = 1;
}
void* oracle_odom_create(const oracle_params* p) { return new OOdom(*p); }
void oracle_odom_destroy(void* h) { delete static_cast<OOdom*>(h); }
int oracle_odom_process(void* h, const float* xyz, int n, oracle_frame_stats* st) {
    return static_cast<OOdom*>(h)->process(xyz, n, st);
}
int oracle_odom_get_keypoints(void* h, float* xyz, int cap) {
    auto* o = static_cast<OOdom*>(h);
    const int k = (int)o->src->kps.size();
    if (k > cap) return -k;
    std::memcpy(xyz, o->src->kps.data(), sizeof(P3) * k);
    return k;
}
int oracle_odom_get_ratios(void* h, float* r, int cap) {
    auto* o = static_cast<OOdom*>(h);
    const int k = (int)o->seg_ratios.size();
    if (k > cap) return -k;
    std::memcpy(r, o->seg_ratios.data(), sizeof(float) * k);
    return k;
}
int oracle_odom_get_bits(void* h, uint32_t* bits, int cap) {
    auto* o = static_cast<OOdom*>(h);
    const int k = (int)o->src->desc.size();
    if (k > cap) return -k;
    std::memcpy(bits, o->src->desc.data(), sizeof(Desc) * k);
    return k;
}
int oracle_odom_get_target(void* h, float* xyz, uint32_t* bits, int cap) {
    auto* o = static_cast<OOdom*>(h);
    const int m = (int)o->c2kps.size();
    if (m > cap) return -m;
    if (xyz) std::memcpy(xyz, o->c2kps.data(), sizeof(P3) * m);
    if (bits) std::memcpy(bits, o->c2bits.data(), sizeof(Desc) * m);
    return m;
}
int oracle_odom_get_inliers(void* h, int32_t* q, int32_t* m, int cap) {
    auto* o = static_cast<OOdom*>(h);
    const int c = (int)o->inl_q.size();
    if (c > cap) return -c;
    std::memcpy(q, o->inl_q.data(), sizeof(int32_t) * c);
    std::memcpy(m, o->inl_m.data(), sizeof(int32_t) * c);
    return c;
}
int oracle_odom_get_iss(void* h, float* xyz, int cap) {
    auto* o = static_cast<OOdom*>(h);
    const int c = (int)o->iss_src.size();
    if (c > cap) return -c;
    std::memcpy(xyz, o->iss_src.data(), sizeof(P3) * c);
    return c;
}

#ifdef ORACLE_DIAG
void oracle_diag_fix_normals(void* h, int on) { static_cast<OOdom*>(h)->diag_fix_normals = on; }
void oracle_diag_pose_override(void* h, const float* T16) {
    auto* o = static_cast<OOdom*>(h);
    std::memcpy(o->diag_override, T16, sizeof(o->diag_override));
    o->diag_have_override = 1;
}
int oracle_diag_get_mutual(void* h, int32_t* q, int32_t* m, int cap) {
    auto* o = static_cast<OOdom*>(h);
    const int c = (int)o->mut_q.size();
    if (c > cap) return -c;
    std::memcpy(q, o->mut_q.data(), sizeof(int32_t) * c);
    std::memcpy(m, o->mut_m.data(), sizeof(int32_t) * c);
    return c;
}
#endif

}  // extern "C"
