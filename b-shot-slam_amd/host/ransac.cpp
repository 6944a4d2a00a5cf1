// ransac.cpp -- A10 RANSAC correspondence rejection with PCL semantics
// (src/lidar_odometry.cpp:251-261: CorrespondenceRejectorSampleConsensus, maxIter 2000, inlier
// threshold 1500 mm; RandomSampleConsensus + SampleConsensusModelRegistration).
//
// Structure: the hypothesis stream does not depend on model scores (draws happen only in
// getSamples: mt19937(12345) >> 1, partial Fisher-Yates on the persistent shuffled index vector,
// isSampleGood redraws), so phase 1 generates every sample triplet up front and phase 2 scans the
// hypotheses in order applying PCL's best-model / adaptive-k / max-iteration rules. The scores
// phase 2 reads come either from the host (bshot_ransac: each hypothesis scored when the scan
// reaches it) or from one GPU launch that scores them all (bshot_ransac_dev, csrc/ransac.hip;
// SURVEY.md §8f rank 2). Both compute the same integers, so both give the same result.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

#include "../../include/bshot_abi.h"
#include "../csrc/ctx.h"
#include "geom.h"

namespace {

struct Pt { float x, y, z; };

// computeMeanAndCovarianceMatrix (float, single pass) over src[indices] -> eigen33 values
double sample_threshold(const Pt* src, const std::vector<int>& ind) {
    float acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int id : ind) {
        const Pt& p = src[id];
        acc[0] += p.x * p.x; acc[1] += p.x * p.y; acc[2] += p.x * p.z;
        acc[3] += p.y * p.y; acc[4] += p.y * p.z; acc[5] += p.z * p.z;
        acc[6] += p.x; acc[7] += p.y; acc[8] += p.z;
    }
    const float fn = (float)ind.size();
    for (int a = 0; a < 9; ++a) acc[a] = acc[a] / fn;
    float cov[9];
    cov[0] = acc[0] - acc[6] * acc[6]; cov[1] = acc[1] - acc[6] * acc[7]; cov[2] = acc[2] - acc[6] * acc[8];
    cov[4] = acc[3] - acc[7] * acc[7]; cov[5] = acc[4] - acc[7] * acc[8]; cov[8] = acc[5] - acc[8] * acc[8];
    cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
    float ev[3];
    bm::eigen33_vals(cov, ev);
    const float s = (std::sqrt(ev[0]) + std::sqrt(ev[1])) + std::sqrt(ev[2]);
    double t = (double)s / 3.0;
    return t * t;
}

// ctx == nullptr: host scoring; else the GPU scores every hypothesis in one launch on ctx->stream
int ransac_impl(bshot_ctx* ctx, const float* src_xyz, int ns, const float* tgt_xyz, int nt, const int32_t* corr_q,
                const int32_t* corr_m, int n_corr, int max_iter, double thresh, float* T_out, int32_t* inl_q,
                int32_t* inl_m, int* n_inl) {
    if (!T_out || !n_inl || n_corr < 0 || ns < 0 || nt < 0) return BSHOT_EINVAL;
    const Pt* src = reinterpret_cast<const Pt*>(src_xyz);
    const Pt* tgt = reinterpret_cast<const Pt*>(tgt_xyz);
    auto fallback = [&]() {
        const bg::Mat4f I = bg::Mat4f::identity();
        std::memcpy(T_out, I.m, sizeof(I.m));
        for (int i = 0; i < n_corr; ++i) { inl_q[i] = corr_q[i]; inl_m[i] = corr_m[i]; }
        *n_inl = n_corr;
        return 0;
    };
    std::vector<int> indices(corr_q, corr_q + n_corr);
    if ((int)indices.size() > ns) indices.clear();  // SampleConsensusModel ctor index check
    // source index -> target index (the last correspondence of a source index wins, as PCL's map)
    for (int i = 0; i < n_corr; ++i)
        if (corr_q[i] < 0 || corr_q[i] >= ns || corr_m[i] < 0 || corr_m[i] >= nt) return BSHOT_EINVAL;
    std::vector<int> tgt_of(ns > 0 ? ns : 1, -1);
    for (int i = 0; i < n_corr; ++i) tgt_of[corr_q[i]] = corr_m[i];
    const int nidx = (int)indices.size();
    if (nidx < 3) return fallback();
    const double sample_thresh = sample_threshold(src, indices);

    // ---- phase 1: the hypothesis stream (getSamples for iterations 0..max_iter), drawn lazily:
    // draw_until(h) extends it to h hypotheses (fewer if a draw fails: the stream ends there).
    // `pos` follows the shuffle of index values with their positions in `indices` (what the GPU
    // scorer reads).
    std::mt19937 rng(12345u);
    std::vector<int> shuffled = indices, pos(nidx);
    for (int i = 0; i < nidx; ++i) pos[i] = i;
    std::vector<int> samples, spos;
    samples.reserve(3 * (size_t)(max_iter + 1));
    spos.reserve(3 * (size_t)(max_iter + 1));
    bool stream_end = false;
    auto draw_until = [&](int h) {
        h = std::min(h, max_iter + 1);
        while (!stream_end && (int)samples.size() / 3 < h) {
            bool got = false;
            for (unsigned chk = 0; chk < 1000 && !got; ++chk) {
                for (int i = 0; i < 3; ++i) {
                    const unsigned r = rng() >> 1;
                    const int j = i + (int)(r % (unsigned)(nidx - i));
                    std::swap(shuffled[i], shuffled[j]);
                    std::swap(pos[i], pos[j]);
                }
                const Pt &a = src[shuffled[0]], &b = src[shuffled[1]], &c = src[shuffled[2]];
                const float p10x = b.x - a.x, p10y = b.y - a.y, p10z = b.z - a.z;
                const float p20x = c.x - a.x, p20y = c.y - a.y, p20z = c.z - a.z;
                const float p21x = c.x - b.x, p21y = c.y - b.y, p21z = c.z - b.z;
                got = (double)((p10x * p10x + p10y * p10y) + p10z * p10z) > sample_thresh &&
                      (double)((p20x * p20x + p20y * p20y) + p20z * p20z) > sample_thresh &&
                      (double)((p21x * p21x + p21y * p21y) + p21z * p21z) > sample_thresh;
            }
            if (!got) {
                stream_end = true;
                break;
            }
            for (int i = 0; i < 3; ++i) {
                samples.push_back(shuffled[i]);
                spos.push_back(pos[i]);
            }
        }
        return (int)samples.size() / 3;
    };

    // per-correspondence source / target points in index order (countWithinDistance loop order)
    std::vector<Pt> cs(nidx), ct(nidx);
    for (int i = 0; i < nidx; ++i) { cs[i] = src[indices[i]]; ct[i] = tgt[tgt_of[indices[i]]]; }
    const double thr2 = thresh * thresh;
    auto count_within = [&](const bg::Mat4f& T, std::vector<int>* inl) {
        int cnt = 0;
        for (int i = 0; i < nidx; ++i) {
            float p[3];
            bg::xform(T, &cs[i].x, p);
            const float dx = p[0] - ct[i].x, dy = p[1] - ct[i].y, dz = p[2] - ct[i].z;
            const float d2 = (dx * dx + dz * dz) + (dy * dy + 0.0f);  // Vector4f squaredNorm (SSE)
            if ((double)d2 < thr2) { ++cnt; if (inl) inl->push_back(indices[i]); }
        }
        return cnt;
    };
    auto model_of = [&](int h) {
        double sd[9], td[9];
        for (int i = 0; i < 3; ++i) {
            const Pt& a = src[samples[3 * h + i]];
            const Pt& b = tgt[tgt_of[samples[3 * h + i]]];
            sd[i * 3] = a.x; sd[i * 3 + 1] = a.y; sd[i * 3 + 2] = a.z;
            td[i * 3] = b.x; td[i * 3 + 1] = b.y; td[i * 3 + 2] = b.z;
        }
        return bg::umeyama<double>(sd, td, 3);
    };

    // ---- GPU scores of every hypothesis (sample positions index cs/ct), launched only when PCL's
    // adaptive loop outlasts the host's share: the host scores the first host_max hypotheses
    // itself (PCL usually stops within a few dozen), then the rest of the stream is drawn and the
    // GPU scores it in one launch (identical counts: same float expression,
    // tests/test_parity_gpu.py::test_ransac_dev_matches_host)
    // The GPU launch goes out first (asynchronously) and the host scores the first hypotheses while
    // it runs; the scan waits for the GPU counts only if PCL's adaptive loop outlasts the host share.
    // (A loop that ends early leaves the launch unread; the next RANSAC reuses its buffers only
    // after later syncs on the same stream.)
    const int host_max = ctx ? std::max(8, 4000 / std::max(1, nidx)) : max_iter + 1;
    const int* gcnt = nullptr;
    bool gpu_launched = false;
    auto gpu_launch = [&]() -> int {
        bshot_ctx* c = ctx;
        const int nhyp = draw_until(max_iter + 1);
        if (nhyp <= 0) return BSHOT_OK;
        const size_t np = 6 * (size_t)nidx;
        if (c->rpts.ensure(np) || c->rhyp.ensure(3 * (size_t)nhyp) || c->rcnt.ensure(nhyp) || c->p_rpts.ensure(np) ||
            c->p_rhyp.ensure(3 * (size_t)nhyp) || c->p_rcnt.ensure(nhyp))
            return c->fail("ransac: alloc", BSHOT_EHIP);
        std::memcpy(c->p_rpts.p, cs.data(), sizeof(float) * 3 * nidx);
        std::memcpy(c->p_rpts.p + 3 * nidx, ct.data(), sizeof(float) * 3 * nidx);
        std::memcpy(c->p_rhyp.p, spos.data(), sizeof(int) * 3 * nhyp);
        const int sg = c->stage_begin(BSHOT_STAGE_RANSAC);
        // kernel copies from / into the pinned staging buffers (csrc/kcopy.hip): no copy engine
        if (bsh::kcopy2(c->rpts.p, c->p_rpts.p, sizeof(float) * np, c->rhyp.p, c->p_rhyp.p, sizeof(int) * 3 * nhyp,
                        c->stream) ||
            bsh::launch_ransac_score(c->rpts.p, c->rpts.p + 3 * nidx, nidx, c->rhyp.p, nhyp, thr2, c->rcnt.p,
                                     c->stream) ||
            bsh::kcopy(c->p_rcnt.p, c->rcnt.p, sizeof(int) * nhyp, c->stream))
            return c->fail("ransac: launch", BSHOT_EHIP);
        c->stage_end(sg);
        gpu_launched = true;
        return BSHOT_OK;
    };
    auto gpu_scores = [&]() -> int {
        if (!gpu_launched) return BSHOT_OK;  // empty stream
        ctx->hmark("M_rs_wait");
        if (hipStreamSynchronize(ctx->stream)) return ctx->fail("ransac: sync", BSHOT_EHIP);
        ctx->hmark("M_rs_synced");
        gcnt = ctx->p_rcnt.p;
        return BSHOT_OK;
    };
    if (ctx) {
        ctx->hmark("M_rs_begin");
        const int e = gpu_launch();
        if (e) return e;
        ctx->hmark("M_rs_launched");
    }

    // ---- phase 2: RandomSampleConsensus::computeModel acceptance scan
    const double log_prob = std::log(1.0 - 0.99);
    const double one_over_indices = 1.0 / (double)nidx;
    double k = 1.0;
    int best_cnt = -std::numeric_limits<int>::max();
    bg::Mat4f best_T = bg::Mat4f::identity();
    bool have = false;
    for (int it = 0; (double)it < k; ++it) {
        if (it >= host_max && ctx && !gcnt) {
            const int e = gpu_scores();
            if (e) return e;
        }
        if (draw_until(it + 1) <= it) break;  // the hypothesis stream ended
        int cnt;
        bg::Mat4f T;
        if (gcnt) {
            cnt = gcnt[it];
            if (cnt > best_cnt) T = model_of(it);
        } else {
            T = model_of(it);
            cnt = count_within(T, nullptr);
        }
        if (cnt > best_cnt) {
            best_cnt = cnt;
            best_T = T;
            have = true;
            const double w = (double)best_cnt * one_over_indices;
            double p_no = 1.0 - std::pow(w, 3.0);
            p_no = std::max(std::numeric_limits<double>::epsilon(), p_no);
            p_no = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no);
            k = log_prob / std::log(p_no);
        }
        if (it + 1 > max_iter) break;
    }
    if (!have) return fallback();
    std::vector<int> inl;
    count_within(best_T, &inl);
    if (inl.size() < 3) return fallback();
    std::vector<int> pos_of(ns > 0 ? ns : 1, -1);
    for (int i = 0; i < n_corr; ++i) pos_of[corr_q[i]] = i;
    for (size_t i = 0; i < inl.size(); ++i) {
        const int p = pos_of[inl[i]];
        inl_q[i] = corr_q[p];
        inl_m[i] = corr_m[p];
    }
    *n_inl = (int)inl.size();
    std::memcpy(T_out, best_T.m, sizeof(best_T.m));
    return 1;
}

}  // namespace

extern "C" int bshot_ransac(const float* src_xyz, int ns, const float* tgt_xyz, int nt, const int32_t* corr_q,
                            const int32_t* corr_m, int n_corr, int max_iter, double thresh, float* T_out,
                            int32_t* inl_q, int32_t* inl_m, int* n_inl) {
    return ransac_impl(nullptr, src_xyz, ns, tgt_xyz, nt, corr_q, corr_m, n_corr, max_iter, thresh, T_out, inl_q,
                       inl_m, n_inl);
}

extern "C" int bshot_ransac_dev(bshot_ctx* c, const float* src_xyz, int ns, const float* tgt_xyz, int nt,
                                const int32_t* corr_q, const int32_t* corr_m, int n_corr, int max_iter,
                                double thresh, float* T_out, int32_t* inl_q, int32_t* inl_m, int* n_inl) {
    if (!c) return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    const int rc = ransac_impl(c, src_xyz, ns, tgt_xyz, nt, corr_q, corr_m, n_corr, max_iter, thresh, T_out, inl_q,
                               inl_m, n_inl);
    c->resolve_events();
    return rc;
}

extern "C" int bshot_ransac_scores(bshot_ctx* c, const float* cs, const float* ct, int nidx, const int32_t* hyp,
                                   int nhyp, double thresh, int32_t* cnt) {
    if (nidx < 0 || nhyp < 0 || (nhyp > 0 && (!hyp || !cnt)) || (nidx > 0 && (!cs || !ct))) return BSHOT_EINVAL;
    for (int i = 0; i < 3 * nhyp; ++i)
        if (hyp[i] < 0 || hyp[i] >= nidx) return BSHOT_EINVAL;
    const double thr2 = thresh * thresh;
    if (!c) {
        for (int h = 0; h < nhyp; ++h) {
            double sd[9], td[9];
            for (int i = 0; i < 3; ++i)
                for (int d = 0; d < 3; ++d) {
                    sd[3 * i + d] = cs[3 * hyp[3 * h + i] + d];
                    td[3 * i + d] = ct[3 * hyp[3 * h + i] + d];
                }
            const bg::Mat4f T = bg::umeyama<double>(sd, td, 3);
            int n = 0;
            for (int i = 0; i < nidx; ++i) {
                float p[3];
                bg::xform(T, cs + 3 * i, p);
                const float dx = p[0] - ct[3 * i], dy = p[1] - ct[3 * i + 1], dz = p[2] - ct[3 * i + 2];
                const float d2 = (dx * dx + dz * dz) + (dy * dy + 0.0f);
                n += (double)d2 < thr2 ? 1 : 0;
            }
            cnt[h] = n;
        }
        return BSHOT_OK;
    }
    if (nhyp == 0) return BSHOT_OK;
    (void)hipSetDevice(c->device);
    const size_t np = 6 * (size_t)nidx;
    if (c->rpts.ensure(np) || c->rhyp.ensure(3 * (size_t)nhyp) || c->rcnt.ensure(nhyp))
        return c->fail("ransac_scores: alloc", BSHOT_EHIP);
    if (hipMemcpyAsync(c->rpts.p, cs, sizeof(float) * 3 * nidx, hipMemcpyHostToDevice, c->stream) ||
        hipMemcpyAsync(c->rpts.p + 3 * nidx, ct, sizeof(float) * 3 * nidx, hipMemcpyHostToDevice, c->stream) ||
        hipMemcpyAsync(c->rhyp.p, hyp, sizeof(int) * 3 * nhyp, hipMemcpyHostToDevice, c->stream) ||
        bsh::launch_ransac_score(c->rpts.p, c->rpts.p + 3 * nidx, nidx, c->rhyp.p, nhyp, thr2, c->rcnt.p, c->stream) ||
        hipMemcpyAsync(cnt, c->rcnt.p, sizeof(int) * nhyp, hipMemcpyDeviceToHost, c->stream) ||
        hipStreamSynchronize(c->stream))
        return c->fail("ransac_scores: launch", BSHOT_EHIP);
    return BSHOT_OK;
}
