// ctx.hip -- bshot_ctx lifecycle and the GPU half of the C ABI (include/bshot_abi.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "../host/geom.h"
#include "ctx.h"
#include "kernels.h"

#define HIPCHK(call, what)                          \
    do {                                            \
        hipError_t e_ = (call);                     \
        if (e_ != hipSuccess) return c->fail(what, e_); \
    } while (0)

int bshot_ctx::fail(const char* what, hipError_t e) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return BSHOT_EHIP;
}
int bshot_ctx::fail(const std::string& what, int code) {
    err = what;
    return code;
}
hipEvent_t bshot_ctx::get_ev() {
    if (!evpool.empty()) {
        hipEvent_t e = evpool.back();
        evpool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}
void bshot_ctx::stage_begin(int st) {
    if (!timing) return;
    StageEv s{st, get_ev(), get_ev()};
    (void)hipEventRecord(s.a, stream);
    pending.push_back(s);
}
void bshot_ctx::stage_end() {
    if (!timing || pending.empty()) return;
    (void)hipEventRecord(pending.back().b, stream);
}
void bshot_ctx::resolve_events() {
    for (auto& s : pending) {
        float ms = 0.f;
        if (hipEventSynchronize(s.b) == hipSuccess && hipEventElapsedTime(&ms, s.a, s.b) == hipSuccess) {
            stage_ms[s.stage] += ms;
            stage_n[s.stage] += 1;
        }
        evpool.push_back(s.a);
        evpool.push_back(s.b);
    }
    pending.clear();
}

namespace bsh {

int ctx_set_cloud_dev(bshot_ctx* c, const float* d_xyz, int n) {
    if (n < 0) return c->fail("bshot_set_cloud: n < 0", BSHOT_EINVAL);
    c->n = n;
    c->d_xyz = d_xyz;
    c->grids_ok = false;
    HIPCHK(c->pts4.ensure(n > 0 ? n : 1), "alloc pts4");
    if (n == 0) return BSHOT_OK;
    c->stage_begin(BSHOT_STAGE_GRID);
    HIPCHK(grid_build(c->grid_fine, d_xyz, n, c->prm.seg_radius * 0.125f, c->pts4.p, c->stream), "grid build (fine)");
    HIPCHK(grid_build(c->grid_coarse, d_xyz, n, c->prm.seg_radius * 0.5f, c->pts4.p, c->stream), "grid build (coarse)");
    c->stage_end();
    c->grids_ok = true;
    return BSHOT_OK;
}

int ctx_seg_ratio_dev(bshot_ctx* c) {
    if (c->prm.seg_max_nn < 1 || c->prm.seg_max_nn > 512) return c->fail("seg_max_nn must be in [1, 512]", BSHOT_EINVAL);
    HIPCHK(c->ratio.ensure(c->n > 0 ? c->n : 1), "alloc ratio");
    HIPCHK(c->errw.ensure(1), "alloc err");
    if (c->n == 0) return BSHOT_OK;
    HIPCHK(hipMemsetAsync(c->errw.p, 0, sizeof(int), c->stream), "memset err");
    c->stage_begin(BSHOT_STAGE_SR);
    HIPCHK(launch_seg_ratio(c->grid_fine, c->grid_coarse, c->pts4.p, c->n, c->prm.seg_radius, c->prm.seg_max_nn, c->prm.sr_type,
                            c->ratio.p, c->errw.p, c->stream),
           "seg_ratio launch");
    c->stage_end();
    return BSHOT_OK;
}

int ctx_iss_dev(bshot_ctx* c) {
    HIPCHK(c->third.ensure(c->n > 0 ? c->n : 1), "alloc third");
    HIPCHK(c->issflag.ensure(c->n > 0 ? c->n : 1), "alloc issflag");
    HIPCHK(c->errw.ensure(1), "alloc err");
    if (c->n == 0) return BSHOT_OK;
    HIPCHK(hipMemsetAsync(c->errw.p, 0, sizeof(int), c->stream), "memset err");
    c->stage_begin(BSHOT_STAGE_ISS);
    HIPCHK(grid_build(c->grid_iss, c->d_xyz, c->n, c->prm.iss_salient, c->pts4.p, c->stream), "grid build (ISS)");
    HIPCHK(launch_iss(c->grid_iss, c->pts4.p, c->n, c->prm.iss_salient, c->prm.iss_nonmax, c->prm.iss_min_nn,
                      c->prm.iss_gamma21, c->prm.iss_gamma32, c->third.p, c->issflag.p, c->errw.p, c->stream),
           "iss launch");
    c->stage_end();
    return BSHOT_OK;
}

// keypoints already in c->kps (device, k x 3)
int ctx_describe_dev(bshot_ctx* c, int k) {
    if (c->prm.normal_max_nn < 1 || c->prm.normal_max_nn > 512)
        return c->fail("normal_max_nn must be in [1, 512]", BSHOT_EINVAL);
    const int n = c->n;
    // persistent normals array: resize(n) keeps [0, min) and value-initialises new slots
    HIPCHK(c->normals.ensure(std::max(n, std::max(k, 1))), "alloc normals");
    if (n > c->normals_size)
        HIPCHK(hipMemsetAsync(c->normals.p + c->normals_size, 0, sizeof(float4) * (n - c->normals_size), c->stream),
               "zero normals");
    c->normals_size = n;
    if (k <= 0) return BSHOT_OK;
    HIPCHK(c->errw.ensure(1), "alloc err");
    HIPCHK(hipMemsetAsync(c->errw.p, 0, sizeof(int), c->stream), "memset err");
    HIPCHK(c->counts.ensure(k), "alloc counts");
    HIPCHK(c->offs.ensure(k + 1), "alloc offs");
    HIPCHK(c->rf.ensure(9 * (size_t)k), "alloc rf");
    HIPCHK(c->ok.ensure(k), "alloc ok");
    HIPCHK(c->bits.ensure(11 * (size_t)k), "alloc bits");
    HIPCHK(c->shot.ensure(352 * (size_t)k), "alloc shot");
    c->stage_begin(BSHOT_STAGE_NORMALS);
    HIPCHK(launch_normals(c->grid_fine, c->grid_coarse, c->pts4.p, c->kps.p, k, c->prm.normal_radius, c->prm.normal_max_nn,
                          c->normals.p, c->errw.p, c->stream),
           "normals launch");
    c->stage_end();
    const float R = c->prm.shot_radius;
    c->stage_begin(BSHOT_STAGE_SHOT_GATHER);
    HIPCHK(launch_shot_count(c->grid_coarse, c->kps.p, k, R, c->counts.p, c->offs.p, c->stream), "shot count");
    c->stage_end();
    long long total = 0;
    HIPCHK(hipMemcpyAsync(&total, c->offs.p + k, sizeof(long long), hipMemcpyDeviceToHost, c->stream), "D2H total");
    HIPCHK(hipStreamSynchronize(c->stream), "sync total");
    c->work[0] = total;
    HIPCHK(c->seg.ensure(total > 0 ? (size_t)total : 1), "alloc seg");
    HIPCHK(c->segtmp.ensure(total > 0 ? (size_t)total : 1), "alloc segtmp");
    c->stage_begin(BSHOT_STAGE_SHOT_GATHER);
    HIPCHK(launch_shot_gather(c->grid_coarse, c->kps.p, k, R, c->offs.p, c->seg.p, c->stream), "shot gather");
    c->stage_end();
    c->stage_begin(BSHOT_STAGE_SHOT_SORT);
    HIPCHK(launch_shot_sort(c->offs.p, k, R, c->seg.p, c->segtmp.p, c->stream), "shot sort");
    c->stage_end();
    c->stage_begin(BSHOT_STAGE_LRF);
    HIPCHK(launch_lrf(c->pts4.p, c->kps.p, k, R, c->offs.p, c->seg.p, c->rf.p, c->ok.p, c->stream), "lrf");
    c->stage_end();
    c->stage_begin(BSHOT_STAGE_HIST);
    HIPCHK(launch_shot_hist(c->pts4.p, c->normals.p, c->kps.p, k, R, c->offs.p, c->seg.p, c->rf.p, c->ok.p, c->shot.p,
                            c->bits.p, c->stream),
           "shot hist");
    c->stage_end();
    return BSHOT_OK;
}

int ctx_match_dev(bshot_ctx* c, int na, int nb) {
    HIPCHK(c->lbest.ensure(na > 0 ? na : 1), "alloc lbest");
    HIPCHK(c->rbest.ensure(nb > 0 ? nb : 1), "alloc rbest");
    HIPCHK(c->left.ensure(na > 0 ? na : 1), "alloc left");
    HIPCHK(c->right.ensure(nb > 0 ? nb : 1), "alloc right");
    HIPCHK(c->mflag.ensure(na > 0 ? na : 1), "alloc mflag");
    c->stage_begin(BSHOT_STAGE_MATCH);
    HIPCHK(launch_match(c->ma.p, na, c->mb.p, nb, c->lbest.p, c->rbest.p, c->left.p, c->right.p, c->mflag.p,
                        c->stream),
           "match launch");
    c->stage_end();
    return BSHOT_OK;
}

int ctx_gather(bshot_ctx* c, const int* h_idx, int k, DBuf<float>& dst) {
    HIPCHK(c->gidx.ensure(k > 0 ? k : 1), "alloc gidx");
    HIPCHK(dst.ensure(3 * (size_t)(k > 0 ? k : 1)), "alloc gather out");
    if (k <= 0) return BSHOT_OK;
    HIPCHK(hipMemcpyAsync(c->gidx.p, h_idx, sizeof(int) * k, hipMemcpyHostToDevice, c->stream), "H2D idx");
    HIPCHK(launch_gather(c->pts4.p, c->gidx.p, k, dst.p, c->stream), "gather");
    return BSHOT_OK;
}

int ctx_icp(bshot_ctx* c, const float* src, int ns, const float* tgt, int nt, int max_iter, float* T, int* iters) {
    bg::Mat4f fin = bg::Mat4f::identity();
    int it = 0;
    if (ns >= 3 && nt > 0) {
        HIPCHK(c->isrc.ensure(3 * (size_t)ns), "alloc icp src");
        HIPCHK(c->itgt.ensure(nt), "alloc icp tgt");
        HIPCHK(c->ibest.ensure(ns), "alloc icp best");
        HIPCHK(c->itgt3.ensure(3 * (size_t)std::max(nt, 1)), "alloc icp staging");
        HIPCHK(hipMemcpyAsync(c->itgt3.p, tgt, sizeof(float) * 3 * nt, hipMemcpyHostToDevice, c->stream), "H2D tgt");
        HIPCHK(launch_pack_points(c->itgt3.p, nt, c->itgt.p, c->stream), "pack tgt");
        std::vector<float> cur(src, src + 3 * (size_t)ns), tb(3 * (size_t)ns);
        std::vector<unsigned long long> best(ns);
        double prev_mse = 1.7976931348623157e308;
        while (true) {
            HIPCHK(hipMemcpyAsync(c->isrc.p, cur.data(), sizeof(float) * 3 * ns, hipMemcpyHostToDevice, c->stream),
                   "H2D src");
            c->stage_begin(BSHOT_STAGE_ICP);
            HIPCHK(launch_icp_nn(c->isrc.p, ns, c->itgt.p, nt, c->ibest.p, c->stream), "icp nn");
            c->stage_end();
            HIPCHK(hipMemcpyAsync(best.data(), c->ibest.p, sizeof(unsigned long long) * ns, hipMemcpyDeviceToHost,
                                  c->stream),
                   "D2H nn");
            HIPCHK(hipStreamSynchronize(c->stream), "sync icp");
            for (int i = 0; i < ns; ++i) {
                const unsigned j = (unsigned)(best[i] & 0xFFFFFFFFu);
                tb[3 * i] = tgt[3 * j]; tb[3 * i + 1] = tgt[3 * j + 1]; tb[3 * i + 2] = tgt[3 * j + 2];
            }
            bg::Mat4f Ts = bg::umeyama<float>(cur.data(), tb.data(), ns);
            for (int i = 0; i < ns; ++i) bg::xform(Ts, &cur[3 * i], &cur[3 * i]);
            fin = bg::mul(Ts, fin);
            ++it;
            if (it >= max_iter) break;
            const double cos_angle = 0.5 * (double)(((Ts.m[0] + Ts.m[5]) + Ts.m[10]) - 1.0f);
            const double tsq = (double)((Ts.m[3] * Ts.m[3] + Ts.m[7] * Ts.m[7]) + Ts.m[11] * Ts.m[11]);
            if (cos_angle >= 1.0 && tsq <= 0.0) break;
            double mse = 0;
            for (int i = 0; i < ns; ++i) mse += (double)__builtin_bit_cast(float, (unsigned)(best[i] >> 32));
            mse /= (double)ns;
            if (__builtin_fabs(mse - prev_mse) < 1e-12) break;
            prev_mse = mse;
        }
    }
    std::memcpy(T, fin.m, sizeof(float) * 16);
    *iters = it;
    return BSHOT_OK;
}

}  // namespace bsh

using namespace bsh;

extern "C" {

void bshot_default_params(bshot_params* p) {
    p->seg_radius = 3000.f; p->seg_max_nn = 300; p->sr_type = 0; p->num_keypoints = 600;
    p->iss_salient = 60.f; p->iss_nonmax = 40.f; p->iss_gamma21 = 0.975; p->iss_gamma32 = 0.975; p->iss_min_nn = 5;
    p->normal_radius = 3000.f; p->normal_max_nn = 300; p->shot_radius = 3000.f; p->map_range = 100000.f;
    p->ransac_max_iter = 2000; p->ransac_thresh = 1500.0; p->icp_max_iter = 10; p->run_icp = 1; p->run_iss = 1;
    p->run_kp_eval = 0;
}

int bshot_create(bshot_ctx** out, int device, const bshot_params* p) {
    if (!out) return BSHOT_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return BSHOT_EHIP;
    if (device < 0 || device >= ndev) return BSHOT_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return BSHOT_EHIP;
    bshot_ctx* c = new bshot_ctx();
    c->device = device;
    if (p) c->prm = *p;
    else bshot_default_params(&c->prm);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return BSHOT_EHIP;
    }
    *out = c;
    return BSHOT_OK;
}

void bshot_destroy(bshot_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    c->resolve_events();
    for (auto e : c->evpool) (void)hipEventDestroy(e);
    grid_free(c->grid_fine);
    grid_free(c->grid_coarse);
    grid_free(c->grid_iss);
    c->xyz.release(); c->pts4.release(); c->ratio.release(); c->third.release(); c->issflag.release();
    c->errw.release(); c->normals.release(); c->kps.release(); c->counts.release(); c->offs.release();
    c->seg.release(); c->segtmp.release(); c->rf.release(); c->shot.release(); c->ok.release(); c->bits.release();
    c->ma.release(); c->mb.release(); c->lbest.release(); c->rbest.release(); c->left.release(); c->right.release();
    c->mflag.release(); c->gidx.release(); c->gout.release(); c->isrc.release(); c->itgt3.release(); c->itgt.release(); c->ibest.release();
    (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* bshot_last_error(const bshot_ctx* c) { return c ? c->err.c_str() : "null context"; }

int bshot_sync(bshot_ctx* c) {
    if (hipStreamSynchronize(c->stream) != hipSuccess) return c->fail("sync", hipGetLastError());
    c->resolve_events();
    return BSHOT_OK;
}

void* bshot_stream(bshot_ctx* c) { return (void*)c->stream; }

int bshot_set_cloud(bshot_ctx* c, const float* xyz, int n) {
    if (!c || (n > 0 && !xyz)) return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    HIPCHK(c->xyz.ensure(3 * (size_t)(n > 0 ? n : 1)), "alloc xyz");
    if (n > 0) HIPCHK(hipMemcpyAsync(c->xyz.p, xyz, sizeof(float) * 3 * n, hipMemcpyHostToDevice, c->stream), "H2D xyz");
    return ctx_set_cloud_dev(c, c->xyz.p, n);
}

int bshot_set_cloud_device(bshot_ctx* c, const float* d_xyz, int n) {
    if (!c || (n > 0 && !d_xyz)) return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    return ctx_set_cloud_dev(c, d_xyz, n);
}

int bshot_seg_ratio(bshot_ctx* c, int32_t* idx, float* ratio, int* n_out) {
    if (!c || !n_out) return BSHOT_EINVAL;
    int rc = ctx_seg_ratio_dev(c);
    if (rc) return rc;
    const int n = c->n;
    c->h_ratio.resize(n > 0 ? n : 1);
    int herr = 0;
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(c->h_ratio.data(), c->ratio.p, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream), "D2H ratio");
        HIPCHK(hipMemcpyAsync(&herr, c->errw.p, sizeof(int), hipMemcpyDeviceToHost, c->stream), "D2H err");
    }
    HIPCHK(hipStreamSynchronize(c->stream), "sync ratio");
    c->resolve_events();
    if (herr) return c->fail("seg_ratio: neighbourhood with > 1024 exactly tied boundary keys", BSHOT_ECAP);
    int m = 0;
    for (int i = 0; i < n; ++i) {
        const float r = c->h_ratio[i];
        if (r != r) continue;  // origin, non-finite or NaN ratio (src/lidar_odometry.cpp:63-64,121-122)
        idx[m] = i;
        ratio[m] = r;
        ++m;
    }
    *n_out = m;
    return BSHOT_OK;
}

int bshot_iss(bshot_ctx* c, int32_t* kp_idx, int cap, int* n_out) {
    if (!c || !n_out) return BSHOT_EINVAL;
    int rc = ctx_iss_dev(c);
    if (rc) return rc;
    const int n = c->n;
    c->h_flag.resize(n > 0 ? n : 1);
    int herr = 0;
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(c->h_flag.data(), c->issflag.p, n, hipMemcpyDeviceToHost, c->stream), "D2H iss");
        HIPCHK(hipMemcpyAsync(&herr, c->errw.p, sizeof(int), hipMemcpyDeviceToHost, c->stream), "D2H err");
    }
    HIPCHK(hipStreamSynchronize(c->stream), "sync iss");
    c->resolve_events();
    if (herr & 4) return c->fail("iss: more than 512 neighbours inside the salient radius", BSHOT_ECAP);
    int m = 0;
    for (int i = 0; i < n; ++i)
        if (c->h_flag[i]) {
            if (m < cap) kp_idx[m] = i;
            ++m;
        }
    *n_out = m;
    return m <= cap ? BSHOT_OK : BSHOT_ECAP;
}

int bshot_describe(bshot_ctx* c, const float* kps, int k, float* shot, float* rf, uint32_t* bits) {
    if (!c || k < 0 || (k > 0 && (!kps || !bits))) return BSHOT_EINVAL;
    if (!c->grids_ok && c->n > 0) return c->fail("bshot_describe: no cloud set", BSHOT_ESTATE);
    HIPCHK(c->kps.ensure(3 * (size_t)(k > 0 ? k : 1)), "alloc kps");
    if (k > 0) HIPCHK(hipMemcpyAsync(c->kps.p, kps, sizeof(float) * 3 * k, hipMemcpyHostToDevice, c->stream), "H2D kps");
    int rc = ctx_describe_dev(c, k);
    if (rc) return rc;
    int herr = 0;
    if (k > 0) {
        HIPCHK(hipMemcpyAsync(bits, c->bits.p, sizeof(uint32_t) * 11 * k, hipMemcpyDeviceToHost, c->stream), "D2H bits");
        if (shot) HIPCHK(hipMemcpyAsync(shot, c->shot.p, sizeof(float) * 352 * k, hipMemcpyDeviceToHost, c->stream), "D2H shot");
        if (rf) HIPCHK(hipMemcpyAsync(rf, c->rf.p, sizeof(float) * 9 * k, hipMemcpyDeviceToHost, c->stream), "D2H rf");
        HIPCHK(hipMemcpyAsync(&herr, c->errw.p, sizeof(int), hipMemcpyDeviceToHost, c->stream), "D2H err");
    }
    HIPCHK(hipStreamSynchronize(c->stream), "sync describe");
    c->resolve_events();
    if (herr & 2) return c->fail("normals: neighbourhood with > 1024 exactly tied boundary keys", BSHOT_ECAP);
    return BSHOT_OK;
}

int bshot_get_normals(bshot_ctx* c, float* out, int n) {
    if (!c || n < 0) return BSHOT_EINVAL;
    if (n > c->normals_size) return c->fail("bshot_get_normals: n > normals size", BSHOT_EINVAL);
    if (n > 0) HIPCHK(hipMemcpyAsync(out, c->normals.p, sizeof(float4) * n, hipMemcpyDeviceToHost, c->stream), "D2H normals");
    HIPCHK(hipStreamSynchronize(c->stream), "sync normals");
    return BSHOT_OK;
}

int bshot_match(bshot_ctx* c, const uint32_t* a, int na, const uint32_t* b, int nb, int32_t* left_nn,
                int32_t* right_nn, int32_t* corr_q, int32_t* corr_m, int* n_corr) {
    if (!c || !n_corr || na < 0 || nb < 0) return BSHOT_EINVAL;
    *n_corr = 0;
    if (na == 0 || nb == 0) return BSHOT_OK;
    HIPCHK(c->ma.ensure(11 * (size_t)na), "alloc ma");
    HIPCHK(c->mb.ensure(11 * (size_t)nb), "alloc mb");
    HIPCHK(hipMemcpyAsync(c->ma.p, a, sizeof(uint32_t) * 11 * na, hipMemcpyHostToDevice, c->stream), "H2D a");
    HIPCHK(hipMemcpyAsync(c->mb.p, b, sizeof(uint32_t) * 11 * nb, hipMemcpyHostToDevice, c->stream), "H2D b");
    int rc = ctx_match_dev(c, na, nb);
    if (rc) return rc;
    std::vector<int> flag(na);
    HIPCHK(hipMemcpyAsync(left_nn, c->left.p, sizeof(int) * na, hipMemcpyDeviceToHost, c->stream), "D2H left");
    HIPCHK(hipMemcpyAsync(right_nn, c->right.p, sizeof(int) * nb, hipMemcpyDeviceToHost, c->stream), "D2H right");
    HIPCHK(hipMemcpyAsync(flag.data(), c->mflag.p, sizeof(int) * na, hipMemcpyDeviceToHost, c->stream), "D2H flag");
    HIPCHK(hipStreamSynchronize(c->stream), "sync match");
    c->resolve_events();
    int m = 0;
    for (int i = 0; i < na; ++i)
        if (flag[i]) { corr_q[m] = i; corr_m[m] = left_nn[i]; ++m; }
    *n_corr = m;
    return BSHOT_OK;
}

int bshot_icp(bshot_ctx* c, const float* src, int ns, const float* tgt, int nt, int max_iter, float* T_out, int* iters) {
    if (!c || !T_out || !iters || ns < 0 || nt < 0) return BSHOT_EINVAL;
    int rc = ctx_icp(c, src, ns, tgt, nt, max_iter, T_out, iters);
    c->resolve_events();
    return rc;
}

int bshot_stage_times(bshot_ctx* c, double* ms, int64_t* launches, int n) {
    if (!c) return BSHOT_EINVAL;
    c->resolve_events();
    for (int i = 0; i < n && i < BSHOT_NSTAGES; ++i) {
        if (ms) ms[i] = c->stage_ms[i];
        if (launches) launches[i] = c->stage_n[i];
    }
    return BSHOT_NSTAGES;
}

void bshot_stage_reset(bshot_ctx* c) {
    if (!c) return;
    c->resolve_events();
    for (int i = 0; i < BSHOT_NSTAGES; ++i) { c->stage_ms[i] = 0; c->stage_n[i] = 0; }
}

void bshot_set_timing(bshot_ctx* c, int enabled) {
    if (c) c->timing = enabled != 0;
}

int bshot_radius_pairs(bshot_ctx* c, float R, int64_t* total) {
    if (!c || !total) return BSHOT_EINVAL;
    *total = 0;
    if (c->n == 0) return BSHOT_OK;
    if (!c->grids_ok) return c->fail("bshot_radius_pairs: no cloud", BSHOT_ESTATE);
    DBuf<int> cnt;
    DBuf<long long> offs;
    HIPCHK(cnt.ensure(c->n), "alloc counts");
    HIPCHK(offs.ensure(c->n + 1), "alloc offs");
    const bsh::DevGrid& g = R <= c->prm.iss_salient * 1.5f && c->grid_iss.n == c->n ? c->grid_iss : c->grid_coarse;
    HIPCHK(launch_shot_count(g, c->d_xyz, c->n, R, cnt.p, offs.p, c->stream), "radius count");
    long long t = 0;
    HIPCHK(hipMemcpyAsync(&t, offs.p + c->n, sizeof(long long), hipMemcpyDeviceToHost, c->stream), "D2H");
    HIPCHK(hipStreamSynchronize(c->stream), "sync");
    cnt.release();
    offs.release();
    *total = t;
    return BSHOT_OK;
}

int bshot_debug_knn_stats(bshot_ctx* c, int64_t* out, int n) {
    if (!c || !out) return BSHOT_EINVAL;
    if (!c->grids_ok) return c->fail("bshot_debug_knn_stats: no cloud", BSHOT_ESTATE);
    DBuf<unsigned long long> k;
    HIPCHK(k.ensure(16), "alloc kst");
    HIPCHK(c->ratio.ensure(c->n), "alloc ratio");
    HIPCHK(c->errw.ensure(1), "alloc err");
    HIPCHK(hipMemsetAsync(k.p, 0, 16 * sizeof(unsigned long long), c->stream), "memset");
    HIPCHK(launch_seg_ratio(c->grid_fine, c->grid_coarse, c->pts4.p, c->n, c->prm.seg_radius, c->prm.seg_max_nn,
                            c->prm.sr_type, c->ratio.p, c->errw.p, c->stream, k.p),
           "seg_ratio (stats)");
    unsigned long long h[16];
    HIPCHK(hipMemcpyAsync(h, k.p, sizeof(h), hipMemcpyDeviceToHost, c->stream), "D2H");
    HIPCHK(hipStreamSynchronize(c->stream), "sync");
    k.release();
    for (int i = 0; i < n && i < 16; ++i) out[i] = (int64_t)h[i];
    return 16;
}

int bshot_work_counters(bshot_ctx* c, int64_t* out, int n) {
    if (!c) return BSHOT_EINVAL;
    for (int i = 0; i < n && i < 8; ++i) out[i] = c->work[i];
    return 8;
}

}  // extern "C"
