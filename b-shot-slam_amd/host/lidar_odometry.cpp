// lidar_odometry.cpp -- myslam::LidarOdometry on MI355X (reference: src/lidar_odometry.cpp:1-525).
// Host C++ keeps the order-defining, data-dependent steps that are cheap and serial (libstdc++
// sort semantics for the top-K, the unordered_map keypoint map, RANSAC, gating); everything
// proportional to N or K x neighbourhood runs in the gfx950 kernels through the context.
#include "../../include/bshot/lidar_odometry.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <mutex>
#include <thread>

#include "../csrc/ctx.h"
#include "../csrc/gmap.h"
#include "geom.h"
#include "../../include/bshot/tic_toc.h"

namespace myslam {

static void zero_stats(bshot_frame_stats& s) {
    std::memset(&s, 0, sizeof(s));
    s.corr_n = -1;
}

// features of one sweep computed ahead of time on a worker thread (prefetchFrameDevice)
// A2 top-K of a queued sweep (two ahead), computed on its own host thread as soon as the sweep's
// SR ratios land in pinned memory, so the lookahead worker starts its describe right away. The
// pinned ratio buffer and SR event it reads belong to the queued cloud state and are not reused
// before the sweep is described (ctx_queue_dev reuses the other slot).
struct LidarOdometry::TopkAhead {
    const float* d_xyz = nullptr;
    int n = 0;
    std::thread th;
    std::string err;
    int nv = 0;
    std::vector<int32_t> kidx;
    std::vector<float> kr;
};

// SR ratios of a cloud (pinned host copy) -> valid (index, ratio) pairs -> top-K (libstdc++ order)
static int select_from_ratios(const float* h_ratio, int n, int k_want, std::vector<int32_t>& kidx,
                              std::vector<float>& kr, int* nv_out) {
    kidx.resize(k_want > 0 ? k_want : 1);
    kr.resize(kidx.size());
    int k = 0;
    const int rc = bsh::topk_from_ratios(h_ratio, n, k_want, kidx.data(), kr.data(), &k, nv_out);
    if (rc < 0) return rc;
    kidx.resize(k);
    kr.resize(k);
    return BSHOT_OK;
}

struct LidarOdometry::Lookahead {
    const float* d_xyz = nullptr;
    int n = 0;
    std::shared_ptr<TopkAhead> topk;  // precomputed top-K (joined by the worker), or null
    std::thread th;
    std::string err;
    int nv = 0;
    std::vector<int32_t> kidx;
    std::vector<float> kr;
    PointCloudXYZ kps, iss;
    std::vector<uint32_t> words;
    float ms[3] = {0.f, 0.f, 0.f};  // extract, iss, describe (worker-thread wall time)
    bool external = false;  // another context's extraction (setSrcFrameExtracted): no normals state here
};

LidarOdometry::LidarOdometry()
    : status_(INITIAL), shouldUpdateMap(true), sr_type_("CV"), evaluate_icp_(true), evaluate_corr_(false),
      run_icp_(true) {
    bshot_default_params(&prm_);
    check(bshot_create(&ctx_, 0, &prm_), "bshot_create");
    zero_stats(stats_);
}

LidarOdometry::LidarOdometry(const bshot_params& p, int device)
    : prm_(p), status_(INITIAL), shouldUpdateMap(true), sr_type_("CV"), evaluate_icp_(true), evaluate_corr_(false),
      run_icp_(p.run_icp != 0) {
    if (prm_.sr_type == 1) sr_type_ = "CVS";
    if (prm_.sr_type == 2) sr_type_ = "CVSN";
    check(bshot_create(&ctx_, device, &prm_), "bshot_create");
    zero_stats(stats_);
}

LidarOdometry::~LidarOdometry() {
    if (ahead_ && ahead_->th.joinable()) ahead_->th.join();
    dropTopkAhead();
    bshot_destroy(ctx_);
}

void LidarOdometry::drainLookahead() {
    joinAhead();
    if (topk_ahead_ && topk_ahead_->th.joinable()) topk_ahead_->th.join();
}

void LidarOdometry::dropTopkAhead() {
    if (topk_ahead_ && topk_ahead_->th.joinable()) topk_ahead_->th.join();
    topk_ahead_.reset();
}

void LidarOdometry::joinAhead() {
    if (!ahead_) return;
    if (ahead_->th.joinable()) ahead_->th.join();
    auto la = ahead_;
    ahead_.reset();
    if (!la->err.empty()) {
        err_ = la->err;
        throw std::runtime_error(err_);
    }
    ready_ = la;
}

// a lookahead result that is not adopted: its describe already advanced the persistent normals
// (include/bshot_bits.h:59) past the state the sweep actually described next must start from
void LidarOdometry::dropReady() {
    if (!ready_) return;
    const bool external = ready_->external;  // another context's record: nothing to restore here
    ready_.reset();
    if (!external) check(bsh::ctx_normals_restore(ctx_), "restore normals");
}

void LidarOdometry::resetNormalsState(int size, int m, const float* slots) {
    // the lookahead's describe (worker thread + side stream) ran over the array being replaced: join
    // it and drop its result (its grids and SR stay valid, they do not read the normals), then write
    joinAhead();
    dropReady();
    check(bsh::ctx_normals_write(ctx_, size, m, slots), "normals state");
}

void LidarOdometry::check(int rc, const char* where) {
    if (rc >= 0) return;
    err_ = std::string(where) + ": " + (ctx_ ? bshot_last_error(ctx_) : "no context");
    throw std::runtime_error(err_);
}

void LidarOdometry::setSRType(std::string sr_type) {
    // a type change takes effect at the next extractKeypoints (as in the reference): sweeps already
    // prefetched or queued with the old type are dropped, after their threads are done
    joinAhead();
    dropReady();
    dropTopkAhead();
    ctx_->pf.prefetched = false;
    ctx_->pf2.prefetched = false;
    sr_type_ = sr_type;
    prm_.sr_type = sr_type == "CVS" ? 1 : (sr_type == "CVSN" ? 2 : 0);
    ctx_->prm.sr_type = prm_.sr_type;
}

void LidarOdometry::setRefFrame(Frame::Ptr ref) {
    ref_ = ref;
    ref_pc_ = *ref_->getPointCloud();
}

void LidarOdometry::setSrcFrame(Frame::Ptr src) {
    joinAhead();
    dropReady();
    src_ = src;
    src_pc_ = *src_->getPointCloud();
    src_dev_ = nullptr;
    src_ext_ = nullptr;
    src_n_ = (int)src_pc_.size();
    check(bshot_set_cloud(ctx_, src_n_ ? &src_pc_[0][0] : nullptr, src_n_), "setSrcFrame");
}

void LidarOdometry::setSrcFrameDevice(Frame::Ptr src, const float* d_xyz, int n) {
    ctx_->hmark("M_frame");
    joinAhead();
    ctx_->hmark("M_joined");
    if (ready_ && !(ready_->d_xyz == d_xyz && ready_->n == n)) dropReady();
    src_ = src;
    src_pc_.clear();
    src_dev_ = d_xyz;
    src_ext_ = nullptr;
    src_n_ = n;
    check(bshot_set_cloud_device(ctx_, d_xyz, n), "setSrcFrameDevice");
}

void LidarOdometry::setSrcFrameExtracted(Frame::Ptr src, std::shared_ptr<const Extracted> ex) {
    if (!ex) throw std::runtime_error("setSrcFrameExtracted: no record");
    joinAhead();
    dropReady();
    auto la = std::make_shared<Lookahead>();
    la->external = true;
    la->d_xyz = reinterpret_cast<const float*>(ex.get());  // the record's identity, matched below
    la->n = ex->n_points;
    la->nv = ex->n_valid;
    la->kidx.resize(ex->kps.size());  // only its size is read (the keypoint count)
    la->kr = ex->ratios;
    la->kps = ex->kps;
    la->iss = ex->iss;
    la->words = ex->words;
    if (la->kr.size() != la->kps.size() || la->words.size() != 11 * la->kps.size())
        throw std::runtime_error("setSrcFrameExtracted: inconsistent record");
    ready_ = la;
    src_ = src;
    src_pc_.clear();
    // the record's address is an identity token only: it is no device cloud (issKpDetection must not
    // restore it) and it dangles once the caller's record is gone
    src_dev_ = nullptr;
    src_ext_ = la->d_xyz;
    src_n_ = la->n;
}

LidarOdometry::Extracted LidarOdometry::extracted() const {
    Extracted e;
    e.n_points = stats_.n_points;
    e.n_valid = stats_.n_valid_ratios;
    e.kps = cloud1_kps_;
    e.iss = isskps_src;
    e.ratios = seg_ratios_;
    e.words.resize(11 * cloud1_bshot_.size());
    for (size_t i = 0; i < cloud1_bshot_.size(); ++i) bits_to_words(cloud1_bshot_[i].bits, &e.words[11 * i]);
    return e;
}

LidarOdometry::Extracted LidarOdometry::extractedWithNormals() {
    Extracted e = extracted();
    const int m = std::min(e.n_points, prm_.num_keypoints);
    e.normals.assign(4 * (size_t)std::max(m, 0), 0.f);
    if (m > 0) check(bsh::ctx_normals_read(ctx_, m, e.normals.data()), "read normals");
    return e;
}

void LidarOdometry::prefetchFrameDevice(const float* d_xyz, int n) {
    joinAhead();
    dropReady();
    // grids + SR + ISS on the side stream (after everything already queued on the main stream,
    // i.e. after this sweep's describe, whose normals the next describe continues from)
    ctx_->hmark("M_prefetch");
    check(bshot_prefetch_cloud_device(ctx_, d_xyz, n), "prefetchFrameDevice");
    auto la = std::make_shared<Lookahead>();
    la->d_xyz = d_xyz;
    la->n = n;
    // the top-K started when this sweep was queued travels with it to the worker
    if (topk_ahead_ && topk_ahead_->d_xyz == d_xyz && topk_ahead_->n == n) la->topk = std::move(topk_ahead_);
    else dropTopkAhead();
    topk_ahead_.reset();
    Lookahead* p = la.get();
    la->th = std::thread([this, p]() {
        try {
            runAhead(*p);
        } catch (const std::exception& e) {
            p->err = e.what();
        }
    });
    ahead_ = la;
    ctx_->hmark("M_prefetched");
}

void LidarOdometry::queueFrameDevice(const float* d_xyz, int n) {
    // issued from the worker (after its describe) it started the sweep after next's SR too late and
    // slowed the describe it then overlapped (measured 260 -> 237 sweeps/s): the main thread issues
    // the launches (a thread of their own only moved the wait, profiles/ab_queue_at.txt)
    dropTopkAhead();
    bshot_ctx* c = ctx_;
    const int kwant = prm_.num_keypoints;
    // top-K of the queued sweep on its own thread once its SR lands (reads only the queue slot's
    // pinned ratios and SR event, which stay with the sweep until it is described)
    auto start_topk = [c, d_xyz, n, kwant]() -> std::shared_ptr<TopkAhead> {
        if (!(c->pf2.d_xyz == d_xyz && c->pf2.n == n && c->pf2.sr_state == 1) || c->opt_topk_thread == 0) return nullptr;
        auto tk = std::make_shared<TopkAhead>();
        tk->d_xyz = d_xyz;
        tk->n = n;
        TopkAhead* p = tk.get();
        const hipEvent_t ev = c->pf2.ev_sr;
        const float* h_ratio = c->pf2.h_ratio.p;
        const int* h_err = c->pf2.h_err.p;
        const int dev = c->device;
        p->th = std::thread([p, c, ev, h_ratio, h_err, dev, kwant, n]() {
            (void)hipSetDevice(dev);
            if (hipEventSynchronize(ev) != hipSuccess) {
                p->err = "lookahead sr";
                return;
            }
            c->hmark("T_sr_ready");
            if (h_err[0]) {
                p->err = sr_error_message(h_err[0]);
                return;
            }
            if (select_from_ratios(h_ratio, n, kwant, p->kidx, p->kr, &p->nv) < 0) p->err = "topk";
            c->hmark("T_done");
        });
        return tk;
    };
    check(bshot_queue_cloud_device(ctx_, d_xyz, n), "queueFrameDevice");
    ctx_->hmark("M_queued");
    topk_ahead_ = start_topk();
}

// worker thread: the extract + describe half of the frame for the prefetched cloud (ctx->pf) on
// the side stream. Same steps as extractKeypoints()/computeDescriptors(), so same results.
void LidarOdometry::runAhead(Lookahead& la) {
    bshot_ctx* c = ctx_;
    (void)hipSetDevice(c->device);
    CloudState& S = c->pf;
    auto fail = [&](const char* what) { throw std::runtime_error(std::string(what) + ": " + c->err); };
    TicToc t_ex;
    c->hmark("W_start");
    if (hipEventSynchronize(S.ev_sr) != hipSuccess) fail("lookahead sr");
    c->hmark("W_sr_ready");
    if (la.topk) {
        // computed on the top-K thread when this sweep was queued
        if (la.topk->th.joinable()) la.topk->th.join();
        if (!la.topk->err.empty()) throw std::runtime_error(la.topk->err);
        la.nv = la.topk->nv;
        la.kidx = std::move(la.topk->kidx);
        la.kr = std::move(la.topk->kr);
        la.topk.reset();
    } else {
        if (S.h_err.p[0]) throw std::runtime_error(sr_error_message(S.h_err.p[0]));
        if (select_from_ratios(S.h_ratio.p, S.n, prm_.num_keypoints, la.kidx, la.kr, &la.nv) < 0) fail("topk");
    }
    const int k = (int)la.kidx.size();
    la.kps.resize(k);
    // queued without a sync: the describe below follows it on the side stream, and the coordinates
    // are copied out after the side stream's final sync
    if (bsh::ctx_gather_kps_async(c, S, c->side, la.kidx.data(), k) != BSHOT_OK) fail("lookahead gather");
    la.ms[0] = (float)t_ex.toc();
    TicToc t_d;
    // describe is queued on the side stream; while it runs, ISS (own stream) is collected
    c->hmark("W_topk_done");
    if (bsh::ctx_normals_snapshot(c, c->side, k, true) != BSHOT_OK) fail("lookahead normals snapshot");
    if (bsh::ctx_describe_on(c, S, c->side, k) != BSHOT_OK) fail("lookahead describe");
    c->hmark("W_describe_queued");
    TicToc t_iss;
    if (prm_.run_iss) {
        if (S.iss_state != 1 || hipEventSynchronize(S.ev_iss) != hipSuccess) fail("lookahead iss");
        if (S.h_err.p[1] & 4) throw std::runtime_error("iss: more than 512 neighbours inside the salient radius");
        std::vector<int32_t> ii;
        ii.reserve(1024);
        const unsigned char* fl = S.h_flag.p;
        for (int i = 0; i < S.n; ++i)
            if (fl[i]) ii.push_back(i);
        la.iss.resize(ii.size());
        if (!ii.empty() &&
            bsh::ctx_gather_host_on(c, S, c->iss, ii.data(), (int)ii.size(), c->gout, &la.iss[0][0]) != BSHOT_OK)
            fail("lookahead iss gather");
    }
    la.ms[1] = (float)t_iss.toc();
    c->hmark("W_iss_done");
    if (c->p_bits.ensure(11 * (size_t)(k > 0 ? k : 1)) != hipSuccess || c->p_err.ensure(4) != hipSuccess)
        fail("alloc pinned");
    for (int attempt = 0; attempt < 3; ++attempt) {
        c->p_err.p[0] = 0;
        if (k > 0 && bsh::kcopy2(c->p_bits.p, c->bits.p, sizeof(uint32_t) * 11 * k, c->p_err.p, c->errw.p,
                                 4 * sizeof(int), c->side) != hipSuccess)
            fail("D2H bits");
        if (hipStreamSynchronize(c->side) != hipSuccess) fail("lookahead sync");
        if (k > 0 && bsh::ctx_describe_replan(c, c->p_err.p)) {
            // the device-side plan ran out of capacity: again, planned on the host
            if (bsh::ctx_describe_on(c, S, c->side, k) != BSHOT_OK) fail("lookahead describe (replan)");
            continue;
        }
        break;
    }
    if (k > 0 && (c->p_err.p[0] & 2)) throw std::runtime_error("normals neighbourhood overflow");
    la.words.assign(c->p_bits.p, c->p_bits.p + 11 * (size_t)k);
    if (k > 0) std::memcpy(&la.kps[0][0], c->p_kps3.p, sizeof(float) * 3 * k);
    c->hmark("W_done");
    la.ms[2] = (float)t_d.toc();

}

void LidarOdometry::passSrc2Ref() {
    ref_ = src_;
    ref_pc_ = src_pc_;
    isskps_ref = isskps_src;
}

// gather xyz of the given cloud indices (device gather; works for host and device clouds)
static PointCloudXYZ gather_points(bshot_ctx* c, const std::vector<int32_t>& idx, DBuf<float>& dst) {
    PointCloudXYZ out(idx.size());
    if (idx.empty()) return out;
    if (bsh::ctx_gather_host(c, idx.data(), (int)idx.size(), dst, &out[0][0]) != BSHOT_OK)
        throw std::runtime_error(std::string("gather: ") + c->err);
    return out;
}

void LidarOdometry::extractKeypoints() {
    zero_stats(stats_);
    TicToc t_ex;
    const int n = src_n_;
    stats_.n_points = n;
    if (ready_ && static_cast<const void*>(ready_->d_xyz) == srcId() && ready_->n == n) {
        // computed ahead by the worker thread (prefetchFrameDevice)
        const Lookahead& la = *ready_;
        stats_.n_valid_ratios = la.nv;
        stats_.n_keypoints = (int)la.kidx.size();
        seg_ratios_ = la.kr;
        src_->setKeypoints(std::make_shared<std::vector<Vector3f>>(la.kps));
        if (isInitial()) {
            passSrc2Ref();
            ref_->setKeypoints(src_->getKeypoints());
        }
        cloud1_kps_ = *src_->getKeypoints();
        cloud2_kps_ = *ref_->getKeypoints();
        isskps_src = la.iss;
        stats_.n_iss = (int)isskps_src.size();
        if (isInitial()) isskps_ref = isskps_src;
        stats_.host_ms[0] = (float)t_ex.toc();
        return;
    }
    if (src_ext_) throw std::runtime_error("extractKeypoints: the external frame's record is gone");
    // A1 + A2 (src/lidar_odometry.cpp:51-153)
    std::vector<int32_t> idx(n > 0 ? n : 1), kidx(prm_.num_keypoints > 0 ? prm_.num_keypoints : 1);
    std::vector<float> ratio(n > 0 ? n : 1), kr(kidx.size());
    int nv = 0, k = 0;
    // ISS is independent of SR: it runs on the side stream while SR, top-K and the gather proceed
    if (prm_.run_iss) check(bsh::ctx_iss_launch(ctx_), "iss launch");
    check(bshot_seg_ratio(ctx_, idx.data(), ratio.data(), &nv), "seg_ratio");
    check(bshot_select_topk(idx.data(), ratio.data(), nv, prm_.num_keypoints, kidx.data(), kr.data(), &k), "topk");
    kidx.resize(k);
    stats_.n_valid_ratios = nv;
    stats_.n_keypoints = k;
    seg_ratios_.assign(kr.begin(), kr.begin() + k);
    src_->setKeypoints(std::make_shared<std::vector<Vector3f>>(gather_points(ctx_, kidx, ctx_->kps)));
    if (isInitial()) {
        passSrc2Ref();
        ref_->setKeypoints(src_->getKeypoints());
    }
    cloud1_kps_ = *src_->getKeypoints();
    cloud2_kps_ = *ref_->getKeypoints();
    stats_.host_ms[0] = (float)t_ex.toc();
    TicToc t_iss;
    // A3 ISS (src/lidar_odometry.cpp:164-170): computed every frame, used by kpEvaluation only
    isskps_src.clear();
    if (prm_.run_iss) {
        std::vector<int32_t> iss(n > 0 ? n : 1);
        int ni = 0;
        check(bshot_iss(ctx_, iss.data(), (int)iss.size(), &ni), "iss");
        iss.resize(ni);
        isskps_src = gather_points(ctx_, iss, ctx_->gout);
    }
    stats_.n_iss = (int)isskps_src.size();
    if (isInitial()) isskps_ref = isskps_src;
    stats_.host_ms[1] = (float)t_iss.toc();
}

void LidarOdometry::computeDescriptors() {
    // A4-A7 (src/lidar_odometry.cpp:173-184); keypoints are already on the device (ctx->kps)
    TicToc t_d;
    const int k = (int)cloud1_kps_.size();
    if (ready_ && static_cast<const void*>(ready_->d_xyz) == srcId() && ready_->n == src_n_) {
        const std::vector<uint32_t>& w = ready_->words;
        cloud1_bshot_.resize(k);
        auto desc = std::make_shared<std::vector<std::bitset<352>>>();
        desc->reserve(k);
        for (int i = 0; i < k; ++i) {
            cloud1_bshot_[i].bits = words_to_bits(&w[11 * (size_t)i]);
            desc->push_back(cloud1_bshot_[i].bits);
        }
        src_->setDescriptors(desc);
        const bool external = ready_->external;
        ready_.reset();
        if (!external) bsh::ctx_normals_discard(ctx_);  // adopted: its normals are the state to continue from
        stats_.host_ms[2] = (float)t_d.toc();
        return;
    }
    if (src_ext_) throw std::runtime_error("computeDescriptors: the external frame's record is gone");
    check(bsh::ctx_describe_dev(ctx_, k), "describe");
    check(ctx_->p_bits.ensure(11 * (size_t)(k > 0 ? k : 1)) == hipSuccess ? BSHOT_OK : BSHOT_EHIP, "alloc pinned bits");
    check(ctx_->p_err.ensure(4) == hipSuccess ? BSHOT_OK : BSHOT_EHIP, "alloc pinned err");
    const uint32_t* words = ctx_->p_bits.p;
    for (int attempt = 0; attempt < 3; ++attempt) {
        ctx_->p_err.p[0] = 0;
        if (k > 0) {
            if (bsh::kcopy2(ctx_->p_bits.p, ctx_->bits.p, sizeof(uint32_t) * 11 * k, ctx_->p_err.p, ctx_->errw.p,
                            4 * sizeof(int), ctx_->stream) != hipSuccess)
                check(BSHOT_EHIP, "D2H bits");
        }
        check(bsh::ctx_sync_main(ctx_), "describe sync");
        ctx_->resolve_events();
        if (k > 0 && bsh::ctx_describe_replan(ctx_, ctx_->p_err.p)) {
            // the device-side plan ran out of capacity: again, planned on the host
            check(bsh::ctx_describe_dev(ctx_, k), "describe (replan)");
            continue;
        }
        break;
    }
    if (k > 0 && (ctx_->p_err.p[0] & 2)) check(BSHOT_ECAP, "normals neighbourhood overflow");
    cloud1_bshot_.resize(k);
    auto desc = std::make_shared<std::vector<std::bitset<352>>>();
    desc->reserve(k);
    for (int i = 0; i < k; ++i) {
        cloud1_bshot_[i].bits = words_to_bits(&words[11 * (size_t)i]);
        desc->push_back(cloud1_bshot_[i].bits);
    }
    src_->setDescriptors(desc);
    stats_.host_ms[2] = (float)t_d.toc();
}

bool LidarOdometry::gpuMap() const { return ctx_->opt_gpu_map != 0; }

void LidarOdometry::syncHostMap() {
    if (map_log_skipped_)
        throw std::runtime_error("host Map view unavailable: sweeps were inserted with context option host_map_log=0 "
                                 "(set it to 1 before the first sweep)");
    // replay updateMap's offers into the host Map (same keypoints, ratios, descriptors, poses, order)
    for (; map_log_done_ < map_log_.size(); ++map_log_done_) {
        MapLogEntry& e = map_log_[map_log_done_];
        const Matrix3f R = e.T.block33();
        const Vector3f T = e.T.topRightCorner();
        for (size_t i = 0; i < e.ratios.size(); ++i) {
            Vector3f kp_pos = R * e.kps->at(i) + T;
            bshot_descriptor d;
            d.bits = e.desc->at(i);
            globalMap_.addKeypoint(Keypoint::createKeypoint(kp_pos, e.ratios[i], d));
        }
        e.kps.reset();
        e.desc.reset();
        e.ratios.clear();
    }
}

const std::vector<bshot_descriptor>& LidarOdometry::targetDescriptors() {
    if (targets_on_device_) {
        const int nb = (int)cloud2_kps_.size();
        std::vector<uint32_t> w(11 * (size_t)(nb > 0 ? nb : 1));
        check(bsh::gmap_target_descriptors(ctx_, last_na_, nb, w.data()), "target descriptors");
        cloud2_bshot_.resize(nb);
        for (int i = 0; i < nb; ++i) cloud2_bshot_[i].bits = words_to_bits(&w[11 * (size_t)i]);
        targets_on_device_ = false;
    }
    return cloud2_bshot_;
}

void LidarOdometry::featureMatching() {
    // src/lidar_odometry.cpp:186-265
    TicToc t_m;
    targets_on_device_ = false;
    if (!isInitial() && gpuMap()) {
        // the targets are assembled in HBM (csrc/gmap.hip): map blocks around the ref position in
        // the reference's loop and libstdc++ order, then the ref keypoints in the world frame
        const Matrix4f rp = ref_->getPose();
        const Vector3f pos = rp.topRightCorner();
        Frame::PCPtr rk = ref_->getKeypoints();
        Frame::DCPPtr rd = ref_->getDescriptors();
        const int kref = rk && rd ? (int)std::min(rk->size(), rd->size()) : 0;
        std::vector<uint32_t> refw(11 * (size_t)(kref > 0 ? kref : 1));
        for (int i = 0; i < kref; ++i) bits_to_words((*rd)[i], &refw[11 * (size_t)i]);
        const int na = (int)cloud1_bshot_.size();
        std::vector<uint32_t> a(11 * (size_t)(na > 0 ? na : 1));
        for (int i = 0; i < na; ++i) bits_to_words(cloud1_bshot_[i].bits, &a[11 * (size_t)i]);
        std::vector<int32_t> left(na > 0 ? na : 1), right, cq(na > 0 ? na : 1), cm(na > 0 ? na : 1);
        std::vector<float> tgt;
        int nb = 0, nc = 0;
        ctx_->hmark("M_match_prep");
        check(bsh::gmap_match(ctx_, a.data(), na, pos.v, prm_.map_range, kref ? &(*rk)[0][0] : nullptr, refw.data(), kref,
                              rp.m, ctx_->opt_gpu_map == 2, &nb, tgt, left.data(), right, cq.data(), cm.data(), &nc),
              "match");
        ctx_->hmark("M_matched");
        cloud2_kps_.resize(nb);
        if (nb > 0) std::memcpy(&cloud2_kps_[0][0], tgt.data(), sizeof(float) * 3 * nb);
        cloud2_bshot_.clear();
        targets_on_device_ = true;
        last_na_ = na;
        stats_.n_target = nb;
        stats_.n_mutual = nc;
        stats_.host_ms[3] = (float)t_m.toc();
        // the ICP targets are these: their grids go on the main stream now, ahead of RANSAC's launch,
        // and build while the host draws RANSAC's hypotheses
        if (nb > 0) check(bsh::ctx_icp_prepare(ctx_, ctx_->gtgt.p, nb), "icp prepare");
        ransacStep(na, nb, cq, cm, nc);
        return;
    }
    if (isInitial()) {
        passSrc2Ref();
        ref_->setKeypoints(src_->getKeypoints());
        cloud2_bshot_ = cloud1_bshot_;
        cloud2_kps_ = *ref_->getKeypoints();
    } else {
        const Matrix4f rp = ref_->getPose();
        globalMap_.getKeypoints(rp.topRightCorner(), prm_.map_range, cloud2_kps_, cloud2_bshot_);
        ctx_->hmark("M_map_query");
        for (const Vector3f& q : *ref_->getKeypoints()) cloud2_kps_.push_back(rp.transformPoint(q));
        std::vector<bshot_descriptor> rb = eigen2dc(ref_->getDescriptors());
        cloud2_bshot_.insert(cloud2_bshot_.end(), rb.begin(), rb.end());
    }
    const int na = (int)cloud1_bshot_.size(), nb = (int)cloud2_bshot_.size();
    stats_.n_target = nb;
    std::vector<uint32_t> a(11 * (size_t)(na > 0 ? na : 1)), b(11 * (size_t)(nb > 0 ? nb : 1));
    for (int i = 0; i < na; ++i) bits_to_words(cloud1_bshot_[i].bits, &a[11 * (size_t)i]);
    for (int i = 0; i < nb; ++i) bits_to_words(cloud2_bshot_[i].bits, &b[11 * (size_t)i]);
    std::vector<int32_t> left(na > 0 ? na : 1), right(nb > 0 ? nb : 1), cq(na > 0 ? na : 1), cm(na > 0 ? na : 1);
    int nc = 0;
    ctx_->hmark("M_match_prep");
    check(bshot_match(ctx_, a.data(), na, b.data(), nb, left.data(), right.data(), cq.data(), cm.data(), &nc), "match");
    ctx_->hmark("M_matched");
    stats_.n_mutual = nc;
    stats_.host_ms[3] = (float)t_m.toc();
    ransacStep(na, nb, cq, cm, nc);
}

void LidarOdometry::ransacStep(int na, int nb, const std::vector<int32_t>& cq, const std::vector<int32_t>& cm, int nc) {
    TicToc t_r;
    // RANSAC rejection (maxIter 2000, threshold 1500 mm)
    std::vector<int32_t> iq(nc > 0 ? nc : 1), im(nc > 0 ? nc : 1);
    int ni = 0;
    float T[16];
    const float* s1 = na ? &cloud1_kps_[0][0] : nullptr;
    const float* s2 = nb ? &cloud2_kps_[0][0] : nullptr;
    if (ctx_->opt_ransac_dev)
        check(bshot_ransac_dev(ctx_, s1, na, s2, nb, cq.data(), cm.data(), nc, prm_.ransac_max_iter,
                               prm_.ransac_thresh, T, iq.data(), im.data(), &ni),
              "ransac");
    else
        check(bshot_ransac(s1, na, s2, nb, cq.data(), cm.data(), nc, prm_.ransac_max_iter, prm_.ransac_thresh, T,
                           iq.data(), im.data(), &ni),
              "ransac");
    std::memcpy(T_ransac_.m, T, sizeof(T));
    ctx_->hmark("M_ransac");
    corr_.resize(ni);
    for (int i = 0; i < ni; ++i) corr_[i] = std::make_pair(iq[i], im[i]);
    stats_.n_inliers = ni;
    stats_.host_ms[4] = (float)t_r.toc();
}

void LidarOdometry::evaluateEstimation() {
    // src/lidar_odometry.cpp:267-331
    const Matrix4f T_j = T_ransac_;
    const Matrix4f T_i = ref_->getPose();
    const Matrix4f T_ij = T_i.inverse() * T_j;
    const float h_diff = std::acos(T_ij(1, 1));  // e_y^T R e_y
    const Vector3f t = T_ij.topRightCorner();
    const float t_diff = t.norm();
    stats_.h_diff = h_diff;
    stats_.t_diff = t_diff;
    Matrix4f T_est;
    if (h_diff * 180 / M_PI > 10 || t_diff > 1200 || corr_.size() < 15) {
        T_est = ref_->getPose();
        shouldUpdateMap = false;
        stats_.gated = 1;
    } else {
        T_est = T_j;
        shouldUpdateMap = true;
    }
    // ICP always runs (:291-297), source = cloud1 keypoints transformed by T_est
    TicToc t_icp;
    const int k = (int)cloud1_kps_.size(), m = (int)cloud2_kps_.size();
    std::vector<float> src(3 * (size_t)(k > 0 ? k : 1));
    for (int i = 0; i < k; ++i) {
        const Vector3f p = T_est.transformPoint(cloud1_kps_[i]);
        src[3 * i] = p[0]; src[3 * i + 1] = p[1]; src[3 * i + 2] = p[2];
    }
    float Ticp[16];
    int iters = 0;
    if (targets_on_device_) {
        // the targets are already in HBM (gmap_match)
        check(bsh::ctx_icp(ctx_, src.data(), k, m ? &cloud2_kps_[0][0] : nullptr, m, prm_.icp_max_iter, Ticp, &iters,
                           ctx_->gtgt.p),
              "icp");
        ctx_->resolve_events();
    } else {
        check(bshot_icp(ctx_, src.data(), k, m ? &cloud2_kps_[0][0] : nullptr, m, prm_.icp_max_iter, Ticp, &iters),
              "icp");
    }
    stats_.icp_iters = iters;
    ctx_->hmark("M_icp");
    check(bsh::ctx_queue_iss(ctx_), "queued iss");  // option iss_defer: the queued sweep's ISS starts now
    stats_.host_ms[5] = (float)t_icp.toc();
    Matrix4f F;
    std::memcpy(F.m, Ticp, sizeof(Ticp));
    T_best_ = run_icp_ ? F * T_est : T_j;
    stats_.corr_n = -1;
    if (evaluate_corr_) {
        // correspondence distance statistics (:303-330) over corr = the RANSAC inliers (:260):
        // corr_cloud = cloud1 keypoints under T_best_ (evaluate_icp_) or T_j, as transformPointCloud
        // does; pcl::geometry::distance = Eigen norm of the difference; float sums in corr order,
        // divided by (float)size; median = sorted[size / 2]. The reference prints them (cout); here
        // they go to bshot_frame_stats and the metrics JSON lines. With no inliers the reference
        // divides 0 / 0 and reads an empty vector: NaN here.
        const Matrix4f& Tc = evaluate_icp_ ? T_best_ : T_j;
        const size_t n = corr_.size();
        stats_.corr_n = (int)n;
        if (n == 0) {
            stats_.corr_avg = stats_.corr_sd = stats_.corr_med = NAN;
        } else {
            std::vector<float> dv;
            dv.reserve(n);
            float avg = 0;
            for (auto& c : corr_) {
                dv.push_back((Tc.transformPoint(cloud1_kps_[c.first]) - cloud2_kps_[c.second]).norm());
                avg += dv.back();
            }
            avg = avg / (float)n;
            float sd = 0;
            for (float d : dv) sd += (d - avg) * (d - avg);
            sd = std::sqrt(sd / (float)n);
            std::sort(dv.begin(), dv.end());
            stats_.corr_avg = avg;
            stats_.corr_sd = sd;
            stats_.corr_med = dv[n / 2];
        }
    }
}

void LidarOdometry::poseEstimation() { src_->setPose(T_best_); }

void LidarOdometry::updateMap() {
    // src/lidar_odometry.cpp:344-376 (shouldUpdateMap is never read by the reference)
    TicToc t_map;
    Frame::PCPtr kps = src_->getKeypoints();
    if (gpuMap()) {
        // csrc/gmap.hip: the same inserts in HBM; the descriptors are the rows featureMatching staged
        const int k = (int)cloud1_bshot_.size();
        // the host view's replay log grows by ~60 B per keypoint per sweep; a caller that never
        // reads the host Map (bshot_odom) turns it off
        if (ctx_->opt_host_map_log)
            map_log_.push_back(MapLogEntry{kps, src_->getDescriptors(),
                                           std::vector<float>(seg_ratios_.begin(), seg_ratios_.begin() + k), T_best_});
        else
            ++map_log_skipped_;
        int msz = 0;
        check(bsh::gmap_insert(ctx_, k ? &(*kps)[0][0] : nullptr, seg_ratios_.data(), ctx_->ma.p, k, T_best_.m, &msz),
              "map update");
        stats_.map_size = msz;
    } else {
        const Matrix3f R = T_best_.block33();
        const Vector3f T = T_best_.topRightCorner();
        for (size_t i = 0; i < cloud1_bshot_.size(); i++) {
            Vector3f kp_pos = R * kps->at(i) + T;
            Keypoint::Ptr kp = Keypoint::createKeypoint(kp_pos, seg_ratios_[i], cloud1_bshot_[i]);
            globalMap_.addKeypoint(kp);
        }
        stats_.map_size = globalMap_.size();
    }
    status_ = RUN;
    std::memcpy(stats_.T_ransac, T_ransac_.m, sizeof(stats_.T_ransac));
    std::memcpy(stats_.pose, T_best_.m, sizeof(stats_.pose));
    stats_.host_ms[6] = (float)t_map.toc();
    ctx_->hmark("M_map");
}

void LidarOdometry::updateCorrespondence() {
    corrs.clear();
    corrs.reserve(corr_.size());
    for (auto& co : corr_) corrs.push_back(std::make_pair(cloud1_kps_[co.first], cloud2_kps_[co.second]));
}

static float repeat_rate(const PointCloudXYZ& src, const PointCloudXYZ& ref) {
    if (src.empty()) return 0.f;
    float hit = 0.f;
    for (const Vector3f& s : src) {
        if (s[0] == 0 && s[1] == 0 && s[2] == 0) continue;
        float best = INFINITY;
        for (const Vector3f& r : ref) {
            const float dx = s[0] - r[0], dy = s[1] - r[1], dz = s[2] - r[2];
            const float d2 = (dx * dx + dy * dy) + dz * dz;
            if (d2 < best) best = d2;
        }
        if (!ref.empty() && best <= 900.f) hit += 1.f;
    }
    return hit / (float)src.size();
}

void LidarOdometry::kpEvaluation() {
    // src/lidar_odometry.cpp:392-445: 1-NN repeatability (<= 30 mm) of SR and ISS keypoints
    TicToc t_kp;
    stats_.repeat_sr = repeat_rate(*src_->getKeypoints(), *ref_->getKeypoints());
    stats_.repeat_iss = repeat_rate(isskps_src, isskps_ref);
    stats_.host_ms[7] = (float)t_kp.toc();
}

PointCloudXYZ LidarOdometry::issKpDetection(const PointCloudXYZ& kps) {
    // standalone ISS over an arbitrary cloud (src/lidar_odometry.cpp:447-461); the lookahead threads
    // finish first (they issue on the context's streams), their prefetched results stay valid
    joinAhead();
    const int n = (int)kps.size();
    check(bshot_set_cloud(ctx_, n ? kps.data()->v : nullptr, n), "iss set cloud");
    std::vector<int32_t> iss(n > 0 ? n : 1);
    int ni = 0;
    check(bshot_iss(ctx_, iss.data(), (int)iss.size(), &ni), "iss");
    PointCloudXYZ out;
    for (int i = 0; i < ni; ++i) out.push_back(kps[iss[i]]);
    // restore the source cloud
    // (an external frame has no cloud on this context: nothing to restore)
    if (src_n_ > 0) {
        if (src_dev_) check(bshot_set_cloud_device(ctx_, src_dev_, src_n_), "restore cloud");
        else if (!src_pc_.empty()) check(bshot_set_cloud(ctx_, &src_pc_[0][0], src_n_), "restore cloud");
    }
    return out;
}

Frame::PCPtr LidarOdometry::getKeypoints() {
    syncHostMap();
    Frame::PCPtr kps = std::make_shared<std::vector<Vector3f>>();
    globalMap_.getAllKeypoints(*kps);
    return kps;
}
Frame::PCPtr LidarOdometry::getSrcKeypoints() { return std::make_shared<std::vector<Vector3f>>(cloud1_kps_); }
Frame::PCPtr LidarOdometry::getRefKeypoints() { return std::make_shared<std::vector<Vector3f>>(cloud2_kps_); }
Frame::PCPtr LidarOdometry::getISSKeypoints() { return std::make_shared<std::vector<Vector3f>>(isskps_src); }

PointCloudXYZ LidarOdometry::eigen2pcl(Frame::PCPtr pcptr) { return pcptr ? *pcptr : PointCloudXYZ(); }

std::vector<bshot_descriptor> LidarOdometry::eigen2dc(Frame::DCPPtr pcptr) {
    std::vector<bshot_descriptor> d;
    if (!pcptr) return d;
    d.reserve(pcptr->size());
    for (auto& b : *pcptr) {
        bshot_descriptor x;
        x.bits = b;
        d.push_back(x);
    }
    return d;
}

std::vector<LidarOdometry::PC> LidarOdometry::getBlockKeypoints() {
    syncHostMap();
    std::vector<PC> kpblock;
    globalMap_.getBlockKeypoints(kpblock);
    return kpblock;
}

}  // namespace myslam
