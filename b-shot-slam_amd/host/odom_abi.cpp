// odom_abi.cpp -- C ABI over myslam::LidarOdometry: the headless odometry_test frame loop
// (test/odometry_test.cpp:159-194, test/kp_test.cpp:159-181) plus the map-delta records used by
// the multi-GPU throughput mode (BASELINE config 4). No exception crosses the ABI.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "../../include/bshot/lidar_odometry.h"
#include "../../include/bshot_abi.h"
#include "../csrc/ctx.h"
#include "../csrc/gmap.h"

int bshot_odom_exchange_ctx(bshot_ctx* c, bshot_xchg* x, int include_self, int sim_peers);  // host/xchg.cpp

struct bshot_odom {
    std::unique_ptr<myslam::LidarOdometry> lo;
    std::string err;
    std::vector<float> delta;  // last frame's map delta, 15 floats per keypoint (built on request)
    bool delta_ready = true;
    myslam::Matrix4f d_pose;                     // what bshot_odom_map_delta builds it from
    myslam::Frame::PCPtr d_kps;
    myslam::Frame::DCPPtr d_ds;
    std::vector<float> d_ratios;
    std::vector<myslam::Map> replicas;
    const float* next_d = nullptr;  // lookahead cloud (bshot_odom_set_next_device)
    int next_n = 0;
    const float* next2_d = nullptr;  // the one after (bshot_odom_set_next2_device)
    int next2_n = 0;
    std::FILE* metrics = nullptr;  // per-sweep JSON lines (bshot_odom_set_metrics_file / BSHOT_METRICS)
    long long sweep = 0;
    // frame-sharded chain owner (bshot_odom_process_record): the sequence's own persistent normals
    // array (include/bshot_bits.h:58-87) -- logical size and slots [0, min(size, K)) (the slots past
    // K are never written, so they stay zero) -- against which every record's stale slots are checked
    bool shard_owner = false;
    int seq_size = 0;
    std::vector<float> seq_nrm;
    ~bshot_odom() {
        if (metrics) std::fclose(metrics);
    }
};

static int guard(bshot_odom* o, const std::function<void()>& f);

namespace {

constexpr int kRec = 15;  // x, y, z, ratio, 11 descriptor words (bit patterns)

// one JSON line per sweep: the counts of every stage, the gate's decision and why
// (src/lidar_odometry.cpp:283-290: heading > 10 deg, |t| > 1200 mm, < 15 inliers), the pose and the
// main thread's wall ms per phase. The reference only prints these (cout, :128,167,244,274-279).
void write_metrics(bshot_odom* o, const bshot_frame_stats& s, double wall_ms) {
    if (!o->metrics) return;
    const double h_deg = (double)s.h_diff * 180.0 / M_PI;
    std::string why;
    if (h_deg > 10) why += "\"heading\",";
    if (s.t_diff > 1200) why += "\"translation\",";
    if (s.n_inliers < 15) why += "\"inliers\",";
    if (!why.empty()) why.pop_back();
    std::fprintf(o->metrics,
                 "{\"sweep\": %lld, \"n_points\": %d, \"n_valid_ratios\": %d, \"n_keypoints\": %d, \"n_iss\": %d, "
                 "\"n_target\": %d, \"n_mutual\": %d, \"n_inliers\": %d, \"icp_iters\": %d, \"gated\": %d, "
                 "\"gate_reasons\": [%s], \"h_diff_deg\": %.6g, \"t_diff_mm\": %.6g, \"map_size\": %d, "
                 "\"wall_ms\": %.4f, \"host_ms\": {\"extract\": %.4f, \"iss\": %.4f, \"describe\": %.4f, "
                 "\"match\": %.4f, \"ransac\": %.4f, \"icp\": %.4f, \"map\": %.4f, \"kp_eval\": %.4f}, \"pose\": [",
                 o->sweep, s.n_points, s.n_valid_ratios, s.n_keypoints, s.n_iss, s.n_target, s.n_mutual, s.n_inliers,
                 s.icp_iters, s.gated, why.c_str(), std::isfinite(h_deg) ? h_deg : -1.0,
                 std::isfinite(s.t_diff) ? (double)s.t_diff : -1.0, s.map_size, wall_ms, s.host_ms[0], s.host_ms[1],
                 s.host_ms[2], s.host_ms[3], s.host_ms[4], s.host_ms[5], s.host_ms[6], s.host_ms[7]);
    for (int i = 0; i < 12; ++i) std::fprintf(o->metrics, i ? ", %.9g" : "%.9g", (double)s.pose[i]);
    std::fprintf(o->metrics, "]");
    if (s.corr_n >= 0) {
        // evaluate_corr_ (src/lidar_odometry.cpp:303-330): "Corr num", "Corr avg dist", "Corr SD dist", "Corr med"
        auto num = [](float v) { return std::isfinite(v) ? (double)v : -1.0; };
        std::fprintf(o->metrics, ", \"corr\": {\"n\": %d, \"avg_mm\": %.9g, \"sd_mm\": %.9g, \"med_mm\": %.9g}", s.corr_n,
                     num(s.corr_avg), num(s.corr_sd), num(s.corr_med));
    }
    std::fprintf(o->metrics, "}\n");
    std::fflush(o->metrics);
}

// the lookahead set by bshot_odom_set_next[2]_device: the next sweep's grids/SR/ISS (side stream)
// and top-K/describe (worker thread) run while this one is matched, RANSAC-gated, ICP-refined and
// merged into the map (or, extracting only, packed)
void start_lookahead(bshot_odom* o) {
    myslam::LidarOdometry& lo = *o->lo;
    if (o->next_d) {
        lo.prefetchFrameDevice(o->next_d, o->next_n);
        o->next_d = nullptr;
        if (o->next2_d) lo.queueFrameDevice(o->next2_d, o->next2_n);
    }
    o->next2_d = nullptr;
}

// ex: another context's extraction of this sweep (bshot_odom_process_record), else the cloud
int run_frame(bshot_odom* o, const float* xyz, const float* d_xyz, int n, bshot_frame_stats* st,
              std::shared_ptr<const myslam::LidarOdometry::Extracted> ex = nullptr) {
    const auto t0 = std::chrono::steady_clock::now();
    myslam::LidarOdometry& lo = *o->lo;
    const int K = lo.params().num_keypoints;
    if (o->shard_owner && !ex) {
        // a sweep the chain owner extracts itself (a record was refused): its describe must start from
        // the sequence's normals state, not from whatever this context last described -- including a
        // lookahead describe the caller's set_next_device started on this context over its own array
        // (joined and dropped first, so it is neither adopted nor still writing the array)
        lo.resetNormalsState(o->seq_size, (int)(o->seq_nrm.size() / 4), o->seq_nrm.data());
    }
    myslam::Frame::Ptr f = myslam::Frame::createFrame();
    if (xyz) {
        auto pc = std::make_shared<std::vector<myslam::Vector3f>>(n);
        if (n > 0) std::memcpy(&(*pc)[0][0], xyz, sizeof(float) * 3 * n);
        f->setPointCloud(pc);
    }
    if (!lo.isInitial()) lo.passSrc2Ref();
    if (ex) lo.setSrcFrameExtracted(f, ex);
    else if (xyz) lo.setSrcFrame(f);
    else lo.setSrcFrameDevice(f, d_xyz, n);
    lo.extractKeypoints();
    lo.computeDescriptors();
    if (o->shard_owner && !ex) {
        const int m = std::max(0, std::min(n, K));
        o->seq_nrm.assign(4 * (size_t)m, 0.f);
        if (m > 0 && bsh::ctx_normals_read(lo.context(), m, o->seq_nrm.data()) < 0)
            throw std::runtime_error(std::string("normals state: ") + bshot_last_error(lo.context()));
        o->seq_size = n;
    }
    start_lookahead(o);
    lo.featureMatching();
    lo.evaluateEstimation();
    lo.poseEstimation();
    if (o->lo->params().run_kp_eval) lo.kpEvaluation();
    lo.updateMap();
    lo.updateCorrespondence();
    if (st) *st = lo.lastStats();
    if (o->metrics)
        write_metrics(o, lo.lastStats(),
                      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    ++o->sweep;
    // map delta inputs (the records are built only when bshot_odom_map_delta asks for them)
    o->d_pose = f->getPose();
    o->d_kps = f->getKeypoints();
    o->d_ds = f->getDescriptors();
    o->d_ratios = lo.segRatios();
    o->delta_ready = false;
    return BSHOT_OK;
}

// the K keypoint records the last frame offered to Map::addKeypoint: world position on the
// 10 mm keypoint grid, ratio, descriptor words
void build_delta(bshot_odom* o) {
    if (o->delta_ready) return;
    const myslam::Matrix3f R = o->d_pose.block33();
    const myslam::Vector3f T = o->d_pose.topRightCorner();
    const size_t k = o->d_kps ? o->d_kps->size() : 0;
    o->delta.assign(k * kRec, 0.f);
    for (size_t i = 0; i < k; ++i) {
        myslam::Vector3f w = R * o->d_kps->at(i) + T;
        bshot_descriptor d;
        d.bits = o->d_ds->at(i);
        auto kp = myslam::Keypoint::createKeypoint(w, o->d_ratios[i], d);
        float* r = &o->delta[i * kRec];
        r[0] = kp->getPosition()[0];
        r[1] = kp->getPosition()[1];
        r[2] = kp->getPosition()[2];
        r[3] = o->d_ratios[i];
        uint32_t words[11];
        myslam::bits_to_words(d.bits, words);
        std::memcpy(r + 4, words, sizeof(words));
    }
    o->delta_ready = true;
}

}  // namespace

static int guard(bshot_odom* o, const std::function<void()>& f) {
    try {
        f();
        return BSHOT_OK;
    } catch (const std::exception& e) {
        o->err = e.what();
        return BSHOT_EHIP;
    }
}

extern "C" {

int bshot_odom_create(bshot_odom** out, int device, const bshot_params* p) {
    if (!out) return BSHOT_EINVAL;
    *out = nullptr;
    bshot_params prm;
    if (p) prm = *p;
    else bshot_default_params(&prm);
    auto* o = new bshot_odom();
    try {
        o->lo.reset(new myslam::LidarOdometry(prm, device));
    } catch (const std::exception& e) {
        delete o;
        return BSHOT_EHIP;
    }
    // the headless loop never reads the host Map: no replay log (host memory stays flat over a run;
    // bshot_odom_set_option(o, "host_map_log", 1) before the first sweep restores it)
    o->lo->context()->opt_host_map_log = 0;
    if (const char* path = std::getenv("BSHOT_METRICS")) o->metrics = std::fopen(path, "a");
    *out = o;
    return BSHOT_OK;
}

int bshot_odom_upload(bshot_odom* o, float* d_dst, const float* h_src, int n) {
    if (!o || n < 0 || (n > 0 && (!d_dst || !h_src))) return BSHOT_EINVAL;
    bshot_ctx* c = o->lo->context();
    (void)hipSetDevice(c->device);
    // 32 workgroups: a full-chip grid would hold every CU while it waits on PCIe reads (8, 32, 1024
    // workgroups and an SDMA copy measured alike, 369-375 sweeps/s, experiments/README.md)
    if (bsh::kcopy(d_dst, h_src, sizeof(float) * 3 * (size_t)n, c->pre, 32) != hipSuccess) {
        o->err = "upload: kernel copy launch";
        return BSHOT_EHIP;
    }
    return BSHOT_OK;
}

int bshot_odom_set_metrics_file(bshot_odom* o, const char* path) {
    if (!o) return BSHOT_EINVAL;
    if (o->metrics) std::fclose(o->metrics);
    o->metrics = nullptr;
    if (!path || !*path) return BSHOT_OK;
    o->metrics = std::fopen(path, "w");
    if (!o->metrics) {
        o->err = std::string("cannot open ") + path;
        return BSHOT_EINVAL;
    }
    return BSHOT_OK;
}

void bshot_odom_destroy(bshot_odom* o) { delete o; }

const char* bshot_odom_last_error(const bshot_odom* o) { return o ? o->err.c_str() : "null"; }

int bshot_odom_set_option(bshot_odom* o, const char* name, int value) {
    if (!o || !name) return BSHOT_EINVAL;
    // the two evaluation switches of the reference's class (include/lidar_odometry.h:48-49,
    // test/odometry_test.cpp:107-108); everything else is a context knob
    if (!std::strcmp(name, "eval_corr")) {
        o->lo->setEvaluateCorr(value != 0);
        return BSHOT_OK;
    }
    if (!std::strcmp(name, "eval_icp")) {
        o->lo->setEvaluateICP(value != 0);
        return BSHOT_OK;
    }
    return bshot_set_option(o->lo->context(), name, value);
}

int bshot_odom_set_next_device(bshot_odom* o, const float* d_next, int n_next) {
    if (!o || n_next < 0 || (n_next > 0 && !d_next)) return BSHOT_EINVAL;
    o->next_d = n_next > 0 ? d_next : nullptr;
    o->next_n = n_next;
    return BSHOT_OK;
}

int bshot_odom_set_next2_device(bshot_odom* o, const float* d_next2, int n_next2) {
    if (!o || n_next2 < 0 || (n_next2 > 0 && !d_next2)) return BSHOT_EINVAL;
    o->next2_d = n_next2 > 0 ? d_next2 : nullptr;
    o->next2_n = n_next2;
    return BSHOT_OK;
}

int bshot_odom_exchange(bshot_odom* o, bshot_xchg* x, int include_self) {
    if (!o || !x) return BSHOT_EINVAL;
    const int rc = bshot_odom_exchange_ctx(o->lo->context(), x, include_self, 0);
    if (rc < 0) o->err = bshot_last_error(o->lo->context());
    return rc;
}

int bshot_odom_exchange_sim(bshot_odom* o, bshot_xchg* x, int peers) {
    if (!o || !x || peers < 0) return BSHOT_EINVAL;
    const int rc = bshot_odom_exchange_ctx(o->lo->context(), x, 0, peers);
    if (rc < 0) o->err = bshot_last_error(o->lo->context());
    return rc;
}

int bshot_odom_gpu_replica_insert(bshot_odom* o, int replica, const float* rec, int n) {
    if (!o || replica < 0 || n < 0 || (n > 0 && !rec)) return BSHOT_EINVAL;
    const int rc = bsh::gmap_insert_host_records(o->lo->context(), replica, rec, n);
    if (rc < 0) o->err = bshot_last_error(o->lo->context());
    return rc;
}

int bshot_odom_gpu_replica_size(bshot_odom* o, int replica) {
    if (!o) return BSHOT_EINVAL;
    return bsh::gmap_replica_size(o->lo->context(), replica);
}

int bshot_odom_gpu_replica_query(bshot_odom* o, int replica, const float pos[3], float range, float* xyz,
                                 uint32_t* bits, int cap) {
    if (!o || !pos || !xyz || !bits) return BSHOT_EINVAL;
    bshot_ctx* c = o->lo->context();
    return bsh::gmap_replica_query(c, replica, pos, range, c->opt_gpu_map == 2, xyz, bits, cap);
}

// frame-sharded single sequence: record layout (floats): [0] magic, [1] n_points, [2] n_valid,
// [3] k, [4] n_iss, [5] K (num_keypoints), [6] m = min(n_points, K) (int bits), [7] 0; k x 3
// keypoints, k ratios, k x 11 descriptor words (bit patterns), n_iss x 3 ISS points, m x 4 normals
// slots (the persistent array as the sweep's SHOT read it: [0, k) its own, [k, m) stale)
static constexpr int kRecMagic = 0x32534852;  // "RHS2"
static constexpr int kRecHdr = 8;

int bshot_odom_extract_device(bshot_odom* o, const float* d_xyz, int n, float* rec, int cap) {
    if (!o || n < 0 || (n > 0 && !d_xyz) || cap < 0 || (cap > 0 && !rec)) return BSHOT_EINVAL;
    int len = 0;
    const int rc = guard(o, [&]() {
        myslam::LidarOdometry& lo = *o->lo;
        myslam::Frame::Ptr f = myslam::Frame::createFrame();
        lo.setSrcFrameDevice(f, d_xyz, n);
        lo.extractKeypoints();
        lo.computeDescriptors();
        // the normals slots are read before the next sweep's lookahead describe can touch them
        const myslam::LidarOdometry::Extracted e = lo.extractedWithNormals();
        start_lookahead(o);
        const int k = (int)e.kps.size(), ni = (int)e.iss.size(), m = (int)(e.normals.size() / 4);
        len = kRecHdr + 15 * k + 3 * ni + 4 * m;
        if (len > cap) return;
        const int hdr[kRecHdr] = {kRecMagic, e.n_points, e.n_valid, k, ni, lo.params().num_keypoints, m, 0};
        std::memcpy(rec, hdr, sizeof(hdr));
        float* p = rec + kRecHdr;
        if (k) std::memcpy(p, e.kps[0].v, sizeof(float) * 3 * k);
        p += 3 * k;
        if (k) std::memcpy(p, e.ratios.data(), sizeof(float) * k);
        p += k;
        if (k) std::memcpy(p, e.words.data(), sizeof(uint32_t) * 11 * k);
        p += 11 * k;
        if (ni) std::memcpy(p, e.iss[0].v, sizeof(float) * 3 * ni);
        p += 3 * ni;
        if (m) std::memcpy(p, e.normals.data(), sizeof(float) * 4 * m);
    });
    if (rc < 0) return rc;
    return len > cap ? -len : len;
}

int bshot_odom_process_record(bshot_odom* o, const float* rec, int len, bshot_frame_stats* st) {
    if (!o || !rec || len < kRecHdr) return BSHOT_EINVAL;
    int hdr[kRecHdr];
    std::memcpy(hdr, rec, sizeof(hdr));
    const int n = hdr[1], k = hdr[3], ni = hdr[4], K = hdr[5], m = hdr[6];
    const int myK = o->lo->params().num_keypoints;
    if (hdr[0] != kRecMagic || n < 0 || k < 0 || ni < 0 || k > n || m != std::min(n, std::max(K, 0)) ||
        (long long)len != kRecHdr + 15ll * k + 3ll * ni + 4ll * m) {
        o->err = "bshot_odom_process_record: not an extraction record";
        return BSHOT_EINVAL;
    }
    if (K != myK || k > K) {
        o->err = "bshot_odom_process_record: record extracted with K = " + std::to_string(K) + ", this context has K = " +
                 std::to_string(myK);
        return BSHOT_EINVAL;
    }
    const float* nrm = rec + kRecHdr + 15 * (size_t)k + 3 * (size_t)ni;
    if (!o->shard_owner) {
        // the sequence's normals state so far: this context's own (empty for a fresh context)
        const int rc0 = guard(o, [&]() {
            o->lo->drainLookahead();
            bshot_ctx* c = o->lo->context();
            const int m0 = std::min(c->normals_size, myK);
            o->seq_nrm.assign(4 * (size_t)std::max(m0, 0), 0.f);
            if (m0 > 0 && bsh::ctx_normals_read(c, m0, o->seq_nrm.data()) < 0)
                throw std::runtime_error(std::string("normals state: ") + bshot_last_error(c));
            o->seq_size = c->normals_size;
        });
        if (rc0 < 0) return rc0;
        o->shard_owner = true;
    }
    // the sequence's state after resize(n) (include/bshot_bits.h:59: slots [0, min(size, n)) kept, new
    // ones zero), against which the record's stale slots [k, m) must match bit for bit: the record's
    // SHOT read them, the sequential reference would have read these
    std::vector<float> next(4 * (size_t)m, 0.f);
    const int keep = std::min(std::min(o->seq_size, n), (int)(o->seq_nrm.size() / 4));
    if (std::min(keep, m) > 0) std::memcpy(next.data(), o->seq_nrm.data(), sizeof(float) * 4 * std::min(keep, m));
    if (m > k && std::memcmp(next.data() + 4 * (size_t)k, nrm + 4 * (size_t)k, sizeof(float) * 4 * (m - k)) != 0) {
        o->err = "bshot_odom_process_record: the record was described over stale normals slots [" + std::to_string(k) +
                 ", " + std::to_string(m) + ") that differ from this sequence's (a sweep with fewer than K keypoints "
                 "after a sweep another context extracted); extract this sweep on the chain owner instead "
                 "(bshot_odom_process_device)";
        return BSHOT_ESTALE;
    }
    if (k) std::memcpy(next.data(), nrm, sizeof(float) * 4 * k);
    auto e = std::make_shared<myslam::LidarOdometry::Extracted>();
    e->n_points = n;
    e->n_valid = hdr[2];
    const float* p = rec + kRecHdr;
    e->kps.resize(k);
    if (k) std::memcpy(&e->kps[0][0], p, sizeof(float) * 3 * k);
    p += 3 * k;
    e->ratios.assign(p, p + k);
    p += k;
    e->words.resize(11 * (size_t)k);
    if (k) std::memcpy(e->words.data(), p, sizeof(uint32_t) * 11 * k);
    p += 11 * k;
    e->iss.resize(ni);
    if (ni) std::memcpy(&e->iss[0][0], p, sizeof(float) * 3 * ni);
    const int rc = guard(o, [&]() { run_frame(o, nullptr, nullptr, e->n_points, st, e); });
    if (rc == BSHOT_OK) {
        o->seq_nrm.swap(next);
        o->seq_size = n;
    }
    return rc;
}

int bshot_odom_drain(bshot_odom* o) {
    if (!o) return BSHOT_EINVAL;
    return guard(o, [&]() { o->lo->drainLookahead(); });
}

int bshot_odom_process(bshot_odom* o, const float* xyz, int n, bshot_frame_stats* st) {
    if (!o || n < 0 || (n > 0 && !xyz)) return BSHOT_EINVAL;
    return guard(o, [&]() { run_frame(o, xyz, nullptr, n, st); });
}

int bshot_odom_process_device(bshot_odom* o, const float* d_xyz, int n, bshot_frame_stats* st) {
    if (!o || n < 0 || (n > 0 && !d_xyz)) return BSHOT_EINVAL;
    return guard(o, [&]() { run_frame(o, nullptr, d_xyz, n, st); });
}

int bshot_odom_get_keypoints(bshot_odom* o, float* xyz, int cap) {
    auto k = o->lo->getSrcFrame() ? o->lo->getSrcFrame()->getKeypoints() : nullptr;
    const int n = k ? (int)k->size() : 0;
    if (n > cap) return -n;
    if (n) std::memcpy(xyz, &(*k)[0][0], sizeof(float) * 3 * n);
    return n;
}

int bshot_odom_get_ratios(bshot_odom* o, float* r, int cap) {
    const auto& v = o->lo->segRatios();
    const int n = (int)v.size();
    if (n > cap) return -n;
    if (n) std::memcpy(r, v.data(), sizeof(float) * n);
    return n;
}

int bshot_odom_get_bits(bshot_odom* o, uint32_t* bits, int cap) {
    auto d = o->lo->getSrcFrame() ? o->lo->getSrcFrame()->getDescriptors() : nullptr;
    const int n = d ? (int)d->size() : 0;
    if (n > cap) return -n;
    for (int i = 0; i < n; ++i) myslam::bits_to_words((*d)[i], bits + 11 * (size_t)i);
    return n;
}

int bshot_odom_get_target(bshot_odom* o, float* xyz, uint32_t* bits, int cap) {
    const auto& k = o->lo->targetKeypoints();
    const auto& d = o->lo->targetDescriptors();
    const int n = (int)k.size();
    if (n > cap) return -n;
    if (xyz && n) std::memcpy(xyz, k.data()->v, sizeof(float) * 3 * n);
    if (bits)
        for (int i = 0; i < n; ++i) myslam::bits_to_words(d[i].bits, bits + 11 * (size_t)i);
    return n;
}

int bshot_odom_get_inliers(bshot_odom* o, int32_t* q, int32_t* m, int cap) {
    const auto& c = o->lo->inlierCorrespondences();
    const int n = (int)c.size();
    if (n > cap) return -n;
    for (int i = 0; i < n; ++i) { q[i] = c[i].first; m[i] = c[i].second; }
    return n;
}

int bshot_odom_get_iss(bshot_odom* o, float* xyz, int cap) {
    auto k = o->lo->getISSKeypoints();
    const int n = (int)k->size();
    if (n > cap) return -n;
    if (n) std::memcpy(xyz, &(*k)[0][0], sizeof(float) * 3 * n);
    return n;
}

bshot_ctx* bshot_odom_ctx(bshot_odom* o) { return o ? o->lo->context() : nullptr; }

int bshot_odom_map_delta(bshot_odom* o, float* rec, int cap) {
    if (!o) return BSHOT_EINVAL;
    build_delta(o);
    const int n = (int)(o->delta.size() / kRec);
    if (n > cap) return -n;
    if (n) std::memcpy(rec, o->delta.data(), sizeof(float) * kRec * n);
    return n;
}

int bshot_odom_replica_insert(bshot_odom* o, int replica, const float* rec, int n) {
    if (!o || replica < 0 || n < 0) return BSHOT_EINVAL;
    if ((int)o->replicas.size() <= replica) o->replicas.resize(replica + 1);
    return guard(o, [&]() {
        for (int i = 0; i < n; ++i) {
            const float* r = rec + (size_t)i * kRec;
            myslam::Vector3f p(r[0], r[1], r[2]);
            uint32_t words[11];
            std::memcpy(words, r + 4, sizeof(words));
            bshot_descriptor d;
            d.bits = myslam::words_to_bits(words);
            // positions are already on the 10 mm grid: createKeypoint is idempotent on them
            o->replicas[replica].addKeypoint(myslam::Keypoint::createKeypoint(p, r[3], d));
        }
    });
}

int bshot_odom_replica_size(bshot_odom* o, int replica) {
    if (!o || replica < 0 || replica >= (int)o->replicas.size()) return 0;
    return o->replicas[replica].size();
}

}  // extern "C"
