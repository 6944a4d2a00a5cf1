// ctx.hip -- bshot_ctx lifecycle and the GPU half of the C ABI (include/bshot_abi.h).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <thread>
#include <tuple>
#include <mutex>
#include <string>

#include "../host/geom.h"
#include "ctx.h"
#include "gmap.h"
#include "kernels.h"
#include "preprocess.h"
#include "velodyne.h"

// BSHOT_TRACE=1: entry/exit trace of the C ABI calls on stderr (diagnostics only)
static bool trace_on() {
    static const bool on = std::getenv("BSHOT_TRACE") != nullptr;
    return on;
}
struct TraceScope {
    const char* name;
    explicit TraceScope(const char* n) : name(n) {
        if (trace_on()) std::fprintf(stderr, "> %s\n", name);
    }
    ~TraceScope() {
        if (trace_on()) std::fprintf(stderr, "< %s\n", name);
    }
};

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
void bshot_ctx::hmark(const char* name) {
    if (!htrace_on) return;
    const long long t = std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
    std::lock_guard<std::mutex> lk(htmu);
    htrace.emplace_back(name, t);
}

int bshot_ctx::stage_begin(int st, hipStream_t s) {
    if (!timing || !((timing_mask >> st) & 1u)) return -1;
    std::lock_guard<std::mutex> lk(evmu);
    StageEv e{st, get_ev(), get_ev(), ++stage_seq, false};
    (void)hipEventRecord(e.a, s ? s : stream);
    pending.push_back(e);
    return e.id;
}
void bshot_ctx::stage_end(int token, hipStream_t s) {
    if (!timing || token < 0) return;
    std::lock_guard<std::mutex> lk(evmu);
    for (auto it = pending.rbegin(); it != pending.rend(); ++it)
        if (it->id == token) {
            (void)hipEventRecord(it->b, s ? s : stream);
            it->ended = true;
            return;
        }
}

void CloudState::release() {
    bsh::grid_free(grid_l16);
    bsh::grid_free(grid_l4);
    bsh::grid_free(grid_fine);
    bsh::grid_free(grid_coarse);
    bsh::grid_free(grid_iss);
    xyz.release(); pts4.release(); ratio.release(); third.release(); issflag.release(); issovf.release(); issnml.release(); issnmc.release();
    errw.release(); h_ratio.release(); h_flag.release(); h_err.release();
    for (hipEvent_t* e : {&ev_loaded, &ev_sr, &ev_iss})
        if (*e) { (void)hipEventDestroy(*e); *e = nullptr; }
}
// harvest finished stage-event pairs; wait=true blocks on all of them (stage_times queries).
// Without wait, pairs still in flight (e.g. the side stream's lookahead) stay pending, so
// instrumentation never serialises the two streams.
void bshot_ctx::resolve_events(bool wait) {
    std::lock_guard<std::mutex> lk(evmu);
    std::vector<StageEv> keep;
    for (auto& s : pending) {
        if (!s.ended || (!wait && hipEventQuery(s.b) != hipSuccess)) {
            keep.push_back(s);
            continue;
        }
        float ms = 0.f;
        if (hipEventSynchronize(s.b) == hipSuccess && hipEventElapsedTime(&ms, s.a, s.b) == hipSuccess) {
            stage_ms[s.stage] += ms;
            stage_n[s.stage] += 1;
        }
        evpool.push_back(s.a);
        evpool.push_back(s.b);
    }
    pending.swap(keep);
}

namespace bsh {

// The three low-priority streams (side: lookahead describe, pre: queued grids + SR, iss) run
// beside the high-priority main stream, whose short kernels (match, RANSAC, ICP) are the odometry
// chain's critical path. (Reserving CUs for the main stream with CU-masked side streams measured
// slower, 288 vs 380 sweeps/s, and its pruned code is in experiments/r03_pruned_variants.patch.)
int ctx_make_side_stream(bshot_ctx* c) {
    hipStream_t* sts[3] = {&c->side, &c->pre, &c->iss};
    for (hipStream_t* p : sts) {
        if (*p) {
            (void)hipStreamSynchronize(*p);
            (void)hipStreamDestroy(*p);
        }
        *p = nullptr;
    }
    int lo_prio = 0, hi_prio = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio);
    for (hipStream_t* p : sts) {
        // opt_side_prio: the describe (side) stream's priority, 0 lowest (as pre / iss) .. 2 the main stream's
        int pr = lo_prio;
        if (p == &c->side && c->opt_side_prio > 0)
            pr = c->opt_side_prio >= 2 ? hi_prio : lo_prio + (hi_prio - lo_prio) / 2;
        if (hipStreamCreateWithPriority(p, hipStreamNonBlocking, pr) != hipSuccess) return BSHOT_EHIP;
    }
    return BSHOT_OK;
}

static hipError_t ensure_events(CloudState& s) {
    for (hipEvent_t* e : {&s.ev_loaded, &s.ev_sr, &s.ev_iss})
        if (!*e) {
            hipError_t r = hipEventCreateWithFlags(e, hipEventDisableTiming);
            if (r != hipSuccess) return r;
        }
    return hipSuccess;
}

// float4 copy + radius-ladder grids of one cloud, on stream st
static int cloud_load(bshot_ctx* c, CloudState& s, const float* d_xyz, int n, hipStream_t st) {
    if (n < 0) return c->fail("set_cloud: n < 0", BSHOT_EINVAL);
    s.n = n;
    s.d_xyz = d_xyz;
    s.grids_ok = false;
    s.iss_lvl = false;
    s.prefetched = false;
    s.sr_state = 0;
    s.iss_state = 0;
    s.iss_pending = false;
    s.zeroed = 0;
    HIPCHK(ensure_events(s), "events");
    HIPCHK(s.pts4.ensure(n > 0 ? n : 1), "alloc pts4");
    HIPCHK(s.errw.ensure(2), "alloc err");
    HIPCHK(s.issovf.ensure(2 * (size_t)n + 2), "alloc iss overflow");  // count + (point, position) pairs
    if (n > 0) {
        const int sg1 = c->stage_begin(BSHOT_STAGE_GRID, st);
        if (c->opt_ladder4) {
            bsh::DevGrid* const lad[4] = {&s.grid_l16, &s.grid_fine, &s.grid_l4, &s.grid_coarse};
            // ISS's grid is the ladder's fifth, finest level (cells r/32) when those cells are at least
            // half the salient radius (no sort of its own)
            const float c0 = c->prm.seg_radius * 0.0625f;
#ifndef ISS_LEVEL5
#define ISS_LEVEL5 1  // 0: ISS on the SR ladder's level 0 (cells r/16) as in round 4 (A/B)
#endif
            s.iss_lvl = ISS_LEVEL5 && c->opt_iss_grid && 0.5f * c0 >= 0.5f * c->prm.iss_salient;  // cells r/32 >= salient / 2
            // its first kernel also zeroes the SR / ISS error words and the ISS overflow count
            HIPCHK(grid_build_ladder(lad, d_xyz, n, c0, s.pts4.p, st, 0xFu, 0, s.iss_lvl ? &s.grid_iss : nullptr,
                                     s.errw.p, s.issovf.p),
                   "grid build (ladder)");
            s.zeroed = 3;
        } else {
            HIPCHK(grid_build(s.grid_fine, d_xyz, n, c->prm.seg_radius * 0.125f, s.pts4.p, st), "grid build (r/8)");
            HIPCHK(grid_build(s.grid_coarse, d_xyz, n, c->prm.seg_radius * 0.5f, s.pts4.p, st), "grid build (r/2)");
        }
        c->stage_end(sg1, st);
    }
    s.fix_ladder(c->opt_ladder4 != 0);
    HIPCHK(hipEventRecord(s.ev_loaded, st), "record loaded");
    s.grids_ok = true;
    return BSHOT_OK;
}

// SR of cloud s on stream st; ratios and error word land in pinned host memory at s.ev_sr
static int cloud_sr(bshot_ctx* c, CloudState& s, hipStream_t st) {
    if (c->prm.seg_max_nn < 1 || c->prm.seg_max_nn > knn_max_nn())
        return c->fail("seg_max_nn must be in [1, " + std::to_string(knn_max_nn()) + "]", BSHOT_EINVAL);
    const int n = s.n;
    HIPCHK(s.ratio.ensure(n > 0 ? n : 1), "alloc ratio");
    HIPCHK(s.h_ratio.ensure(n > 0 ? n : 1), "alloc pinned ratio");
    HIPCHK(s.h_err.ensure(2), "alloc pinned err");
    if (!(s.zeroed & 1)) HIPCHK(kfill(s.errw.p, 0, sizeof(int), st), "memset err");
    s.zeroed &= ~1;
    if (n > 0) {
        const int sg2 = c->stage_begin(BSHOT_STAGE_SR, st);
        HIPCHK(launch_seg_ratio(s.ladder, c->ladder_mode(s), s.pts4.p, n, c->prm.seg_radius, c->prm.seg_max_nn, c->prm.sr_type,
                                c->opt_sr_start, s.ratio.p, s.errw.p, st, nullptr, c->opt_sr_blocks, c->opt_sr_xcd_chunk,
                                c->opt_sr_run, (float)c->opt_sr_bratio / 100.f),
               "seg_ratio launch");
        c->stage_end(sg2, st);
    }
    HIPCHK(kcopy2(s.h_ratio.p, s.ratio.p, sizeof(float) * (size_t)(n > 0 ? n : 0), s.h_err.p, s.errw.p, sizeof(int), st),
           "D2H ratio + err");
    HIPCHK(hipEventRecord(s.ev_sr, st), "record sr");
    s.sr_state = 1;
    return BSHOT_OK;
}

// ISS of cloud s on stream st; flags and error word land in pinned host memory at s.ev_iss
static int cloud_iss(bshot_ctx* c, CloudState& s, hipStream_t st) {
    const int n = s.n;
    HIPCHK(s.third.ensure(n > 0 ? n : 1), "alloc third");
    HIPCHK(s.issflag.ensure(n > 0 ? n : 1), "alloc issflag");
    HIPCHK(s.issovf.ensure(2 * (size_t)n + 2), "alloc iss overflow");  // count + (point, position) pairs
    HIPCHK(s.issnml.ensure((size_t)32 * (n > 0 ? n : 1)), "alloc iss nms lists");
    HIPCHK(s.issnmc.ensure(n > 0 ? n : 1), "alloc iss nms counts");
    HIPCHK(s.h_flag.ensure(n > 0 ? n : 1), "alloc pinned flags");
    HIPCHK(s.h_err.ensure(2), "alloc pinned err");
    const bool zeroed = (s.zeroed & 2) != 0;  // errw[1] and the overflow count, by the grid build
    s.zeroed &= ~2;
    if (!zeroed) HIPCHK(kfill(s.errw.p + 1, 0, sizeof(int), st), "memset err");
    if (n > 0) {
        const int sg3 = c->stage_begin(BSHOT_STAGE_ISS, st);
        // ISS on the SR ladder's points, no sort of its own: the ladder's fifth level (cells r/32 =
        // 93.75 mm at the reference's settings, <= 3 per axis around a 60 mm ball) when the ladder
        // built it, else its finest SR level when that cell holds the ball's cube in 2 x 2 x 2 cells
        const bool lvl5 = s.fine_ladder && s.iss_lvl && s.grid_iss.n == n;
        const bool reuse = lvl5 || (c->opt_iss_grid && c->opt_ladder4 && s.fine_ladder && s.grid_l16.n == n &&
                                    s.grid_l16.cell >= 2.f * c->prm.iss_salient);
        if (!reuse)
            HIPCHK(grid_build(s.grid_iss, s.d_xyz, n, c->prm.iss_salient * (float)c->opt_iss_cell, s.pts4.p, st, false),
                   "grid build (ISS)");
        c->hmark("Q_iss_grid");
        HIPCHK(launch_iss(reuse && !lvl5 ? s.grid_l16 : s.grid_iss, s.pts4.p, n, c->prm.iss_salient, c->prm.iss_nonmax, c->prm.iss_min_nn,
                          c->prm.iss_gamma21, c->prm.iss_gamma32, s.third.p, s.issflag.p, s.issovf.p, s.issnml.p,
                          s.issnmc.p, s.errw.p + 1, st, c->opt_iss_ovf_blocks, c->opt_iss_nms_blocks, zeroed,
                          c->opt_iss_xcd_chunk),
               "iss launch");
        c->stage_end(sg3, st);
        c->hmark("Q_iss_k");
    }
    HIPCHK(kcopy2(s.h_flag.p, s.issflag.p, (size_t)(n > 0 ? n : 0), s.h_err.p + 1, s.errw.p + 1, sizeof(int), st),
           "D2H iss + err");
    HIPCHK(hipEventRecord(s.ev_iss, st), "record iss");
    s.iss_state = 1;
    return BSHOT_OK;
}

static bool holds(const CloudState& s, const float* d_xyz, int n) {
    return s.prefetched && s.d_xyz == d_xyz && s.n == n && n > 0;
}

// slots move by value: their ladder pointers must be re-aimed at their own grids afterwards
static void swap_slots(bshot_ctx* c, CloudState& a, CloudState& b) {
    std::swap(a, b);
    a.fix_ladder(c->opt_ladder4 != 0);
    b.fix_ladder(c->opt_ladder4 != 0);
}

int ctx_set_cloud_dev(bshot_ctx* c, const float* d_xyz, int n) {
    if (!holds(c->pf, d_xyz, n) && holds(c->pf2, d_xyz, n)) {
        // queued two ahead and never promoted: adopt it through the prefetch slot
        swap_slots(c, c->pf, c->pf2);
        c->pf2.prefetched = false;
    }
    if (holds(c->pf, d_xyz, n)) {
        swap_slots(c, c->cs, c->pf);
        c->cs.prefetched = false;
        c->pf.prefetched = false;
        HIPCHK(hipStreamWaitEvent(c->stream, c->cs.ev_loaded, 0), "wait prefetch");
        return BSHOT_OK;
    }
    // the side stream may still read this cloud's buffers (ISS of the previous cloud)
    if (c->cs.iss_state == 1) HIPCHK(hipStreamWaitEvent(c->stream, c->cs.ev_iss, 0), "wait iss");
    return cloud_load(c, c->cs, d_xyz, n, c->stream);
}

int ctx_prefetch_dev(bshot_ctx* c, const float* d_xyz, int n) {
    if (n <= 0) return BSHOT_OK;
    if (holds(c->pf2, d_xyz, n)) {
        // queued earlier (grids, SR and ISS on the pre/iss streams): promote; the lookahead
        // describe on the side stream starts after its grids
        if (int rc = ctx_queue_iss(c)) return rc;
        swap_slots(c, c->pf, c->pf2);
        c->pf2.prefetched = false;
        HIPCHK(hipStreamWaitEvent(c->side, c->pf.ev_loaded, 0), "wait queued cloud");
        return BSHOT_OK;
    }
    // the prefetch slot holds an older cloud; let work already queued on the main stream finish first
    hipEvent_t e;
    {
        std::lock_guard<std::mutex> lk(c->evmu);
        e = c->get_ev();
    }
    HIPCHK(hipEventRecord(e, c->stream), "record");
    HIPCHK(hipStreamWaitEvent(c->side, e, 0), "wait main");
    {
        std::lock_guard<std::mutex> lk(c->evmu);
        c->evpool.push_back(e);
    }
    if (c->pf.iss_state == 1) HIPCHK(hipStreamWaitEvent(c->side, c->pf.ev_iss, 0), "wait old iss");
    int rc = cloud_load(c, c->pf, d_xyz, n, c->side);
    if (rc) return rc;
    rc = cloud_sr(c, c->pf, c->side);
    if (rc) return rc;
    if (c->prm.run_iss) {
        // ISS is only needed at the end of the sweep: its own stream, overlapping SR and describe
        HIPCHK(hipStreamWaitEvent(c->iss, c->pf.ev_loaded, 0), "wait cloud");
        rc = cloud_iss(c, c->pf, c->iss);
        if (rc) return rc;
    }
    c->pf.prefetched = true;
    return BSHOT_OK;
}

// the sweep after next: grids + SR on the pre stream, ISS on the iss stream, into the queue slot,
// running beside the side stream's describe of the next sweep
int ctx_queue_dev(bshot_ctx* c, const float* d_xyz, int n) {
    const int go = ctx_queue_begin(c, d_xyz, n);
    if (go <= 0) return go;
    return ctx_queue_rest(c, d_xyz, n);
}

int ctx_queue_iss(bshot_ctx* c) {
    if (!c->pf2.iss_pending) return BSHOT_OK;
    c->pf2.iss_pending = false;
    HIPCHK(hipStreamWaitEvent(c->iss, c->pf2.ev_loaded, 0), "wait cloud");
    return cloud_iss(c, c->pf2, c->iss);
}

// main-thread half of ctx_queue_dev: 1 when the cloud must be queued (the pre stream then waits
// for the work already on the main stream), 0 when it is already held, < 0 on error
int ctx_queue_begin(bshot_ctx* c, const float* d_xyz, int n) {
    if (n <= 0 || holds(c->pf, d_xyz, n) || holds(c->pf2, d_xyz, n)) return 0;
    // the queue slot's buffers may still be read by work queued on the main stream or by ISS
    hipEvent_t e;
    {
        std::lock_guard<std::mutex> lk(c->evmu);
        e = c->get_ev();
    }
    HIPCHK(hipEventRecord(e, c->stream), "record");
    HIPCHK(hipStreamWaitEvent(c->pre, e, 0), "wait main");
    {
        std::lock_guard<std::mutex> lk(c->evmu);
        c->evpool.push_back(e);
    }
    return 1;
}

// the rest of ctx_queue_dev (grids, SR, ISS of the queue slot on the pre / iss streams): touches
// only c->pf2 and those streams, so it may run on another host thread while the main thread works
int ctx_queue_rest(bshot_ctx* c, const float* d_xyz, int n) {
    (void)hipSetDevice(c->device);
    if (c->pf2.iss_state == 1) HIPCHK(hipStreamWaitEvent(c->pre, c->pf2.ev_iss, 0), "wait old iss");
    c->hmark("Q_load");
    int rc = cloud_load(c, c->pf2, d_xyz, n, c->pre);
    if (rc) return rc;
    c->hmark("Q_sr");
    rc = cloud_sr(c, c->pf2, c->pre);
    if (rc) return rc;
    c->hmark("Q_iss");
    if (c->prm.run_iss && c->opt_iss_defer) {
        c->pf2.iss_pending = true;
    } else if (c->prm.run_iss) {
        HIPCHK(hipStreamWaitEvent(c->iss, c->pf2.ev_loaded, 0), "wait cloud");
        rc = cloud_iss(c, c->pf2, c->iss);
        if (rc) return rc;
    }
    c->hmark("Q_done");
    c->pf2.prefetched = true;
    return BSHOT_OK;
}

int ctx_sr_launch(bshot_ctx* c) {
    if (!c->cs.grids_ok) return c->fail("seg_ratio: no cloud set", BSHOT_ESTATE);
    if (c->cs.sr_state == 1) return BSHOT_OK;
    return cloud_sr(c, c->cs, c->stream);
}

int ctx_iss_launch(bshot_ctx* c) {
    if (!c->cs.grids_ok) return c->fail("iss: no cloud set", BSHOT_ESTATE);
    if (c->cs.iss_state == 1) return BSHOT_OK;
    HIPCHK(hipStreamWaitEvent(c->iss, c->cs.ev_loaded, 0), "wait cloud");
    return cloud_iss(c, c->cs, c->iss);
}

int ctx_normals_snapshot(bshot_ctx* c, hipStream_t st, int k, bool defer) {
    const int m = std::min(std::max(k, 0), c->normals_size);
    c->normals_snap_size = c->normals_size;
    c->normals_snap_n = m;
    c->normals_snap_defer = 0;
    if (m > 0) {
        HIPCHK(c->normals_snap.ensure(m), "alloc normals snapshot");
        if (defer)
            c->normals_snap_defer = m;
        else
            HIPCHK(kcopy(c->normals_snap.p, c->normals.p, sizeof(float4) * m, st), "snapshot normals");
    }
    return BSHOT_OK;
}

int ctx_normals_restore(bshot_ctx* c) {
    if (c->normals_snap_size < 0) return BSHOT_OK;
    if (c->normals_snap_n > 0)
        HIPCHK(kcopy(c->normals.p, c->normals_snap.p, sizeof(float4) * c->normals_snap_n, c->stream),
               "restore normals");
    c->normals_size = c->normals_snap_size;
    c->normals_snap_size = -1;
    return BSHOT_OK;
}

void ctx_normals_discard(bshot_ctx* c) { c->normals_snap_size = -1; }

int ctx_normals_read(bshot_ctx* c, int m, float* out) {
    if (m < 0 || m > c->normals_size) return c->fail("normals read past the logical size", BSHOT_EINVAL);
    if (m == 0) return BSHOT_OK;
    HIPCHK(c->p_nrm.ensure(4 * (size_t)m), "alloc pinned normals");
    HIPCHK(kcopy(c->p_nrm.p, c->normals.p, sizeof(float4) * m, c->stream), "D2H normals");
    HIPCHK(hipStreamSynchronize(c->stream), "sync normals");
    std::memcpy(out, c->p_nrm.p, sizeof(float4) * m);
    return BSHOT_OK;
}

int ctx_normals_write(bshot_ctx* c, int size, int m, const float* slots) {
    if (size < 0 || m < 0 || m > size) return c->fail("normals state: bad sizes", BSHOT_EINVAL);
    // a lookahead describe on the side stream reads and writes the array: it must have finished
    // before the array is replaced (the caller drops its result, LidarOdometry::resetNormalsState)
    HIPCHK(hipStreamSynchronize(c->side), "sync side stream");
    HIPCHK(c->normals.ensure(std::max(size, 1)), "alloc normals");
    if (m > 0) {
        HIPCHK(c->p_nrm.ensure(4 * (size_t)m), "alloc pinned normals");
        std::memcpy(c->p_nrm.p, slots, sizeof(float4) * m);
        HIPCHK(kcopy(c->normals.p, c->p_nrm.p, sizeof(float4) * m, c->stream), "H2D normals");
    }
    if (size > m) HIPCHK(kfill(c->normals.p + m, 0, sizeof(float4) * (size - m), c->stream), "zero normals");
    HIPCHK(hipStreamSynchronize(c->stream), "sync normals");
    c->normals_size = size;
    c->normals_snap_size = -1;
    return BSHOT_OK;
}

// keypoints already in c->kps (device, k x 3)
// the SHOT rank kernel for k keypoints with about `total` neighbours: the workgroup-per-keypoint
// kernel streams large neighbourhoods (config 5: ~28k per keypoint, 2.0 -> ? ms), the wave-per-chunk
// kernel has more parallelism for small ones (config 2: ~7.8k, 0.15 vs 0.39 ms in the pipeline)
static int rank_wg_for(const bshot_ctx* c, int k, long long total) {
    if (c->opt_rank_wg != 2) return c->opt_rank_wg;
    return k > 0 && total / k > 16384 ? 1 : 0;
}

int ctx_describe_on(bshot_ctx* c, CloudState& S, hipStream_t st, int k) {
    // the SHOT-segment normals take up to 512 neighbours, the kNN engine's (k_normals) up to knn_max_nn()
    const int nmax = c->opt_normals_seg && c->prm.normal_radius == c->prm.shot_radius ? 512 : knn_max_nn();
    if (c->prm.normal_max_nn < 1 || c->prm.normal_max_nn > nmax)
        return c->fail("normal_max_nn must be in [1, " + std::to_string(nmax) + "]", BSHOT_EINVAL);
    const int n = S.n;
    // persistent normals array: resize(n) keeps [0, min) and value-initialises new slots
    HIPCHK(c->normals.ensure(std::max(n, std::max(k, 1))), "alloc normals");
    // A4: with normal_radius == shot_radius the normals' neighbours are the head of each keypoint's
    // sorted SHOT segment (k_normals_seg after the rank below); otherwise a search of their own
    const bool nseg = c->opt_normals_seg && c->prm.normal_radius == c->prm.shot_radius;
    // the device-planned describe with the normals from the segments: its count kernel is the first
    // to touch the error word and the normals, so it carries their fills
    const bool dev_plan = !c->plan_on_host && k > 0 && k <= 8192 && c->seg_hint > 0;
    const bool fold = nseg && dev_plan;
    // a deferred normals snapshot (ctx_normals_snapshot): slots [0, snap) before this describe
    const int snap = c->normals_snap_defer;
    c->normals_snap_defer = 0;
    if (snap > 0 && !fold)
        HIPCHK(kcopy(c->normals_snap.p, c->normals.p, sizeof(float4) * snap, st), "snapshot normals");
    float4* z4 = nullptr;
    int nz = 0;
    if (n > c->normals_size) {
        if (fold) {
            z4 = c->normals.p + c->normals_size;
            nz = n - c->normals_size;
        } else {
            HIPCHK(kfill(c->normals.p + c->normals_size, 0, sizeof(float4) * (n - c->normals_size), st),
                   "zero normals");
        }
    }
    c->normals_size = n;
    if (k <= 0) return BSHOT_OK;
    // errw: [0] error bits (2 normals overflow, 8 sort piece overflow, 16 device plan over
    // capacity), [2..3] the neighbourhood total as planned on the device
    HIPCHK(c->errw.ensure(4), "alloc err");
    if (!fold) HIPCHK(kfill(c->errw.p, 0, 4 * sizeof(int), st), "memset err");
    HIPCHK(c->counts.ensure(k), "alloc counts");
    HIPCHK(c->offs.ensure(k + 1), "alloc offs");
    HIPCHK(c->rf.ensure(9 * (size_t)k), "alloc rf");
    HIPCHK(c->ok.ensure(k), "alloc ok");
    HIPCHK(c->bits.ensure(11 * (size_t)k), "alloc bits");
    HIPCHK(c->shot.ensure(352 * (size_t)k), "alloc shot");
    if (!nseg) {
        const int sg4 = c->stage_begin(BSHOT_STAGE_NORMALS, st);
        HIPCHK(launch_normals(S.ladder, c->ladder_mode(S), S.pts4.p, c->kps.p, k, c->prm.normal_radius,
                              c->prm.normal_max_nn, c->normals.p, c->errw.p, st),
               "normals launch");
        c->stage_end(sg4, st);
    }
    const float R = c->prm.shot_radius;
    const int sg5 = c->stage_begin(BSHOT_STAGE_SHOT_GATHER, st);
    HIPCHK(c->sbh.ensure(1024 * (size_t)k), "alloc bucket hist");
    HIPCHK(c->sbst.ensure(1024 * (size_t)k), "alloc bucket starts");
    if (dev_plan) {
        // the whole describe queued without a host round trip: the plan (segment offsets, chunk
        // bases, LPT order) is computed on the device against capacities sized from the largest
        // neighbourhood total seen so far (the margin below); an overflow (errw bit 16) makes the caller
        // re-run this describe with the host-side plan
        // 2 x: a sequence's neighbourhood totals drift by tens of percent, and an overflow costs a
        // second describe re-planned on the host (+50% still overflowed once in a 200-sweep bench
        // region, profiles/r06zh_grow200.txt); 4-byte entries, so the margin is tens of MB of HBM
        const long long seg_cap = 2 * c->seg_hint + 1048576;
        const int chunk_cap = (int)(seg_cap / 64) + k + 1;
        HIPCHK(c->seg.ensure((size_t)seg_cap), "alloc seg");
        HIPCHK(c->segtmp.ensure((size_t)seg_cap), "alloc segtmp");
        HIPCHK(c->cb.ensure((size_t)k + 1), "alloc cb");
        HIPCHK(c->perm.ensure(k), "alloc perm");
        HIPCHK(c->owner.ensure((size_t)chunk_cap), "alloc owner");
        HIPCHK(c->cinfo.ensure((size_t)chunk_cap), "alloc chunk records");
        HIPCHK(c->csum.ensure(8 * (size_t)chunk_cap), "alloc csum");
        HIPCHK(c->eig.ensure(8 * (size_t)k), "alloc eig");
        HIPCHK(c->okf.ensure(k), "alloc okf");
        HIPCHK(launch_shot_count_plan(S.grid_coarse, c->kps.p, k, R, c->counts.p, c->sbh.p, seg_cap, chunk_cap,
                                      c->offs.p, c->cb.p, c->perm.p, c->errw.p, st, fold, z4, nz,
                                      snap > 0 ? c->normals_snap.p : nullptr, c->normals.p, snap),
               "shot count + plan");
        c->stage_end(sg5, st);
        const int sg6 = c->stage_begin(BSHOT_STAGE_SHOT_GATHER, st);
        HIPCHK(launch_shot_gather_b(S.grid_coarse, c->kps.p, k, R, c->offs.p, c->sbh.p, c->sbst.p, c->seg.p, st,
                                    c->errw.p),
               "shot gather");
        c->stage_end(sg6, st);
        Describe2Args A;
        A.k = k; A.n_plan = 0; A.n_chunks = chunk_cap; A.R = R;
        A.cb = c->cb.p; A.owner = c->owner.p; A.perm = c->perm.p; A.offs = c->offs.p;
        A.pts4 = S.pts4.p; A.normals = c->normals.p;
        A.kps = c->kps.p; A.seg = c->seg.p; A.sorted = c->segtmp.p; A.csum = c->csum.p; A.eig = c->eig.p;
        A.okf = c->okf.p; A.rf = c->rf.p; A.ok = c->ok.p;
        A.nseg_max_nn = nseg ? c->prm.normal_max_nn : 0; A.normals_out = c->normals.p;
        A.shot = c->shot.p; A.bits = c->bits.p; A.err = c->errw.p;
        A.bstart = c->sbst.p;
        A.max_blocks = c->opt_chunk_blocks > 0 ? c->opt_chunk_blocks : 8192;  // chunk kernels grid-stride to cb[k]
        A.rank_wg = rank_wg_for(c, k, c->seg_hint);
        A.slices = c->opt_desc_slices;
        A.hf_pack = c->opt_hist_pack && c->hf_pack_ok;
        A.cinfo = seg_cap < 0x7FFFFFFFll ? c->cinfo.p : nullptr;
        A.rank_max = c->opt_rank_max;
        const int sg10 = c->stage_begin(BSHOT_STAGE_SHOT_SORT, st);
        HIPCHK(launch_describe2(A, 0, st), "describe2 sort");
        c->stage_end(sg10, st);
        const int sg11 = c->stage_begin(BSHOT_STAGE_LRF, st);
        HIPCHK(launch_describe2(A, 1, st), "describe2 lrf");
        c->stage_end(sg11, st);
        const int sg12 = c->stage_begin(BSHOT_STAGE_HIST, st);
        HIPCHK(launch_describe2(A, 2, st), "describe2 hist");
        c->stage_end(sg12, st);
        return BSHOT_OK;
    }
    c->plan_on_host = false;
    HIPCHK(launch_shot_count(S.grid_coarse, c->kps.p, k, R, c->counts.p, c->offs.p, st, c->sbh.p), "shot count");
    c->stage_end(sg5, st);
    HIPCHK(c->p_offs.ensure((size_t)k + 1), "alloc pinned offs");
    HIPCHK(kcopy(c->p_offs.p, c->offs.p, sizeof(long long) * ((size_t)k + 1),
                          st),
           "D2H offs");
    HIPCHK(hipStreamSynchronize(st), "sync offs");
    const long long total = c->p_offs.p[k];
    c->work[0] = total;
    // the first total seen sets the device plan's capacities with 50% headroom on top of the
    // plan's own +50%: a sequence's totals drift upwards over its first sweeps, and each overflow
    // costs a re-planned describe plus a free + malloc of the neighbour-key buffers (hundreds of MB)
    if (total > c->seg_hint) c->seg_hint = c->seg_hint == 0 ? total + total / 2 : total;
    HIPCHK(c->seg.ensure(total > 0 ? (size_t)total : 1), "alloc seg");
    HIPCHK(c->segtmp.ensure(total > 0 ? (size_t)total : 1), "alloc segtmp");
    const int sg6 = c->stage_begin(BSHOT_STAGE_SHOT_GATHER, st);
    HIPCHK(launch_shot_gather_b(S.grid_coarse, c->kps.p, k, R, c->offs.p, c->sbh.p, c->sbst.p, c->seg.p, st),
           "shot gather");
    c->stage_end(sg6, st);
    // host plan (after a device-plan overflow): 64-rank chunks and the LPT launch order
    const int n_plan = 0;
    long long nch = 0;
    for (int q = 0; q < k; ++q) nch += (c->p_offs.p[q + 1] - c->p_offs.p[q] + 63) / 64;
    if (nch > 0x7FFFFFFF) return c->fail("describe: too many neighbourhood chunks", BSHOT_ECAP);
    HIPCHK(c->p_plan.ensure(4 * (size_t)n_plan + 2 * (size_t)k + 1), "alloc pinned plan");
    int* hcb = c->p_plan.p;
    int* hperm = hcb + k + 1;
    for (int q = 0; q < k; ++q) hperm[q] = q;
    std::stable_sort(hperm, hperm + k, [&](int x, int y) {
        return c->p_offs.p[x + 1] - c->p_offs.p[x] > c->p_offs.p[y + 1] - c->p_offs.p[y];
    });
    int cbr = 0;
    for (int q = 0; q < k; ++q) {
        hcb[q] = cbr;
        cbr += (int)((c->p_offs.p[q + 1] - c->p_offs.p[q] + 63) / 64);
    }
    hcb[k] = cbr;
    HIPCHK(c->cb.ensure((size_t)k + 1), "alloc cb");
    HIPCHK(c->owner.ensure(cbr > 0 ? (size_t)cbr : 1), "alloc owner");
    HIPCHK(c->cinfo.ensure(cbr > 0 ? (size_t)cbr : 1), "alloc chunk records");
    HIPCHK(c->csum.ensure(8 * (size_t)(cbr > 0 ? cbr : 1)), "alloc csum");
    HIPCHK(c->eig.ensure(8 * (size_t)k), "alloc eig");
    HIPCHK(c->okf.ensure(k), "alloc okf");
    HIPCHK(c->perm.ensure(k), "alloc perm");
    HIPCHK(kcopy(c->cb.p, hcb, sizeof(int) * ((size_t)k + 1), st), "H2D cb");
    HIPCHK(kcopy(c->perm.p, hperm, sizeof(int) * k, st), "H2D perm");
    Describe2Args A;
    A.k = k; A.n_plan = n_plan; A.n_chunks = cbr; A.R = R;
    A.cb = c->cb.p; A.owner = c->owner.p; A.perm = c->perm.p; A.offs = c->offs.p; A.pts4 = S.pts4.p; A.normals = c->normals.p;
    A.kps = c->kps.p; A.seg = c->seg.p; A.sorted = c->segtmp.p; A.csum = c->csum.p; A.eig = c->eig.p;
    A.okf = c->okf.p; A.rf = c->rf.p; A.ok = c->ok.p;
    A.nseg_max_nn = nseg ? c->prm.normal_max_nn : 0; A.normals_out = c->normals.p;
    A.shot = c->shot.p; A.bits = c->bits.p; A.err = c->errw.p;
    A.bstart = c->sbst.p;
    A.max_blocks = c->opt_chunk_blocks;
    A.rank_wg = rank_wg_for(c, k, total);
    A.slices = c->opt_desc_slices;
    A.hf_pack = c->opt_hist_pack && c->hf_pack_ok;
    A.rank_max = c->opt_rank_max;
    A.cinfo = total < 0x7FFFFFFFll ? c->cinfo.p : nullptr;
    const int sg10 = c->stage_begin(BSHOT_STAGE_SHOT_SORT, st);
    HIPCHK(launch_describe2(A, 0, st), "describe2 sort");
    c->stage_end(sg10, st);
    const int sg11 = c->stage_begin(BSHOT_STAGE_LRF, st);
    HIPCHK(launch_describe2(A, 1, st), "describe2 lrf");
    c->stage_end(sg11, st);
    const int sg12 = c->stage_begin(BSHOT_STAGE_HIST, st);
    HIPCHK(launch_describe2(A, 2, st), "describe2 hist");
    c->stage_end(sg12, st);
    return BSHOT_OK;
}

bool ctx_describe_replan(bshot_ctx* c, const int* err) {
    if (!(err[0] & 16)) return false;
    c->work[1]++;  // re-planned describes (bshot_work_counters)
    note_regrow("describe replan", 0);
    long long total = 0;
    std::memcpy(&total, err + 2, sizeof(total));
    if (total > c->seg_hint) c->seg_hint = total;
    c->plan_on_host = true;
    return true;
}

int ctx_describe_dev(bshot_ctx* c, int k) { return ctx_describe_on(c, c->cs, c->stream, k); }

int ctx_match_dev(bshot_ctx* c, int na, int nb) {
    HIPCHK(c->lbest.ensure((size_t)na + nb + 1), "alloc best");
    HIPCHK(c->left.ensure(2 * (size_t)na + nb + 1), "alloc match out");
    const int sg13 = c->stage_begin(BSHOT_STAGE_MATCH);
    HIPCHK(launch_match(c->ma.p, na, c->ma.p + 11 * (size_t)na, nb, c->lbest.p, c->left.p, c->stream), "match launch");
    c->stage_end(sg13);
    return BSHOT_OK;
}

// gathers read their indices from pinned staging inside the kernel (no upload launch); the host
// copy, when asked for, is written by the same kernel
static int gather_io(bshot_ctx* c, CloudState& S, hipStream_t st, const int* h_idx, int k, DBuf<float>& dst,
                     float* hout) {
    HIPCHK(dst.ensure(3 * (size_t)(k > 0 ? k : 1)), "alloc gather out");
    if (k <= 0) return BSHOT_OK;
    HIPCHK(c->p_gidx.ensure(k), "alloc pinned idx");
    std::memcpy(c->p_gidx.p, h_idx, sizeof(int) * k);
    HIPCHK(launch_gather_io(S.pts4.p, c->p_gidx.p, k, dst.p, hout, st), "gather");
    return BSHOT_OK;
}

int ctx_gather_on(bshot_ctx* c, CloudState& S, hipStream_t st, const int* h_idx, int k, DBuf<float>& dst) {
    return gather_io(c, S, st, h_idx, k, dst, nullptr);
}

int ctx_gather(bshot_ctx* c, const int* h_idx, int k, DBuf<float>& dst) {
    return ctx_gather_on(c, c->cs, c->stream, h_idx, k, dst);
}

int ctx_gather_host_on(bshot_ctx* c, CloudState& S, hipStream_t st, const int* h_idx, int k, DBuf<float>& dst,
                       float* out) {
    if (k > 0) HIPCHK(c->p_g3.ensure(3 * (size_t)k), "alloc pinned gather");
    int rc = gather_io(c, S, st, h_idx, k, dst, k > 0 ? c->p_g3.p : nullptr);
    if (rc || k <= 0) return rc;
    HIPCHK(hipStreamSynchronize(st), "sync gather");
    std::memcpy(out, c->p_g3.p, sizeof(float) * 3 * k);
    return BSHOT_OK;
}

// keypoint gather for the lookahead describe, asynchronous: H2D indices, gather into c->kps and
// D2H of the coordinates into c->p_kps3 are queued on st with buffers of their own (the ISS gather
// runs concurrently); the caller syncs st before reading c->p_kps3
int ctx_gather_kps_async(bshot_ctx* c, CloudState& S, hipStream_t st, const int* h_idx, int k) {
    HIPCHK(c->kps.ensure(3 * (size_t)(k > 0 ? k : 1)), "alloc kps");
    if (k <= 0) return BSHOT_OK;
    HIPCHK(c->p_kidx.ensure(k), "alloc pinned kidx");
    HIPCHK(c->p_kps3.ensure(3 * (size_t)k), "alloc pinned kps");
    std::memcpy(c->p_kidx.p, h_idx, sizeof(int) * k);
    HIPCHK(launch_gather_io(S.pts4.p, c->p_kidx.p, k, c->kps.p, c->p_kps3.p, st), "gather kps");
    return BSHOT_OK;
}

int ctx_gather_host(bshot_ctx* c, const int* h_idx, int k, DBuf<float>& dst, float* out) {
    return ctx_gather_host_on(c, c->cs, c->stream, h_idx, k, dst, out);
}

int ctx_sync_main(bshot_ctx* c) {
    HIPCHK(hipStreamSynchronize(c->stream), "sync");
    return BSHOT_OK;
}

// the ICP targets' nested grids (cells 1000, 2000, 4000, 8000 mm, all hashed) from one
// nested-key sort of d_tgt; float4 targets in index order -> itgt. A sort-free build by counting
// (four launches instead of ~13) measured 2-4 % slower end to end (profiles/r05g_ab_*.txt)
// A finite target beyond the grids' key range (|cell index| >= 2^20 at the 500 mm level: about
// +-524 km) would be left out of every level; the build flags it in icp_err (value 8), copied to
// pinned memory behind the build, and ctx_icp fails the call with BSHOT_ECAP instead of matching
// against a partial target set (non-finite targets are left out, as PCL's kd-tree does).
static hipError_t icp_grids(bshot_ctx* c, const float* d_tgt, int nt, int min_cap) {
    DevGrid* lad[4] = {&c->icp_lad[0], &c->icp_lad[1], &c->icp_lad[2], &c->icp_lad[3]};
    hipError_t e = c->icp_err.ensure(2);
    if (e != hipSuccess) return e;
    c->p_icp_err.coherent = true;
    if ((e = c->p_icp_err.ensure(1)) != hipSuccess) return e;
    if ((e = grid_build_ladder(lad, d_tgt, nt, 1000.f, c->itgt.p, c->stream, 0xFu, min_cap, nullptr, c->icp_err.p,
                               nullptr)) != hipSuccess)
        return e;
    return kcopy(c->p_icp_err.p, c->icp_err.p, sizeof(int), c->stream);
}

// the ICP targets' grids queued ahead (right after the map query, while the host runs RANSAC): the
// next ctx_icp on the same device targets skips its own build
int ctx_icp_prepare(bshot_ctx* c, const float* d_tgt, int nt) {
    c->icp_prep_tgt = nullptr;
    if (!d_tgt || nt <= 0) return BSHOT_OK;
    HIPCHK(c->itgt.ensure(nt), "alloc icp tgt");
    HIPCHK(icp_grids(c, d_tgt, nt, std::max(65536, 2 * nt)), "icp grids");
    c->icp_prep_tgt = d_tgt;
    c->icp_prep_nt = nt;
    return BSHOT_OK;
}

static long long ns_now() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int ctx_icp(bshot_ctx* c, const float* src, int ns, const float* tgt, int nt, int max_iter, float* T, int* iters,
            const float* d_tgt) {
    const bool prepared = d_tgt && c->icp_prep_tgt == d_tgt && c->icp_prep_nt == nt;
    c->icp_prep_tgt = nullptr;
    bg::Mat4f fin = bg::Mat4f::identity();
    int it = 0;
    if (ns >= 3 && nt > 0 && !c->opt_diag_skip_icp) {
        // the source (host, already moved by T_est) in pinned memory, read there by the kernels; the
        // targets are in HBM already (gmap) or go through pinned staging
        HIPCHK(c->p_src.ensure(3 * (size_t)ns), "alloc pinned src");
        HIPCHK(c->itgt.ensure(nt), "alloc icp tgt");
        std::memcpy(c->p_src.p, src, sizeof(float) * 3 * ns);
        if (!d_tgt) {
            HIPCHK(c->itgt3.ensure(3 * (size_t)nt), "alloc icp staging");
            HIPCHK(c->p_tgt.ensure(3 * (size_t)nt), "alloc pinned tgt");
            std::memcpy(c->p_tgt.p, tgt, sizeof(float) * 3 * nt);
            HIPCHK(kcopy(c->itgt3.p, c->p_tgt.p, sizeof(float) * 3 * nt, c->stream), "H2D icp targets");
            d_tgt = c->itgt3.p;
        }
        // the targets are fixed for the whole ICP call: their grids are built once (or were queued
        // ahead by ctx_icp_prepare)
        if (!prepared) HIPCHK(icp_grids(c, d_tgt, nt, std::max(65536, 2 * nt)), "icp grids");
        HIPCHK(c->ilst.ensure((size_t)ICP_LIST_CAP * ns), "alloc icp lists");
        HIPCHK(c->ilsd.ensure((size_t)ICP_LIST_CAP * ns), "alloc icp list distances");
        HIPCHK(c->ilcnt.ensure(ns), "alloc icp list counts");
        const DevGrid* g4[4] = {&c->icp_lad[0], &c->icp_lad[1], &c->icp_lad[2], &c->icp_lad[3]};
        HIPCHK(c->ilcen.ensure(ns), "alloc icp list centres");
        const float* d_src0 = c->p_src.p;
        bool dev_done = false;
        if (c->opt_icp_device) {
            // PCL's loop on the device (csrc/icp.hip): k_icp_lists finds iteration 0's exact 1-NN and
            // every source's candidate list, then one persistent k_icp_run iterates (per iteration:
            // every source's step and NN, then the float Umeyama and the convergence test on the last
            // workgroup to arrive); the stopping step writes the composed transform and the iteration
            // count to coherent pinned memory, seq last. The host waits once.
            HIPCHK(c->ipos.ensure(ns), "alloc icp positions");
            HIPCHK(c->irec.ensure(7 * (size_t)((ns + 3) & ~3)), "alloc icp records");  // 16-B aligned rows
            HIPCHK(c->ictl.ensure(1), "alloc icp state");
            HIPCHK(c->isync.ensure(2), "alloc icp sync");
            c->p_iout.coherent = true;
            HIPCHK(c->p_iout.ensure(1), "alloc icp result");
            IcpOut* out = c->p_iout.p;
            const int seq = ++c->icp_seq;
            const int sg14 = c->stage_begin(BSHOT_STAGE_ICP);
            HIPCHK(launch_icp(d_src0, ns, c->ilst.p, c->ilsd.p, c->ilcnt.p, ICP_LIST_CAP, g4, c->itgt.p, nt, max_iter,
                              c->ipos.p, c->ilcen.p, c->irec.p, c->ictl.p, c->isync.p, out, seq, c->stream),
                   "icp launch");
            c->stage_end(sg14);
            // spin briefly on seq, then block on the stream: a slow GPU (contention, a profiler) only
            // makes the call wait longer, it never fails it
            const long long t_a = ns_now();
            bool seen = false;
            for (unsigned spins = 0;; ++spins) {
                if (__atomic_load_n(&out->seq, __ATOMIC_ACQUIRE) == seq) { seen = true; break; }
                if ((spins & 255) == 0 && ns_now() - t_a > 5000000ll) break;
                __builtin_ia32_pause();
            }
            if (!seen) {
                HIPCHK(hipStreamSynchronize(c->stream), "sync icp");
                seen = __atomic_load_n(&out->seq, __ATOMIC_ACQUIRE) == seq;
            }
            c->work[2] += ns_now() - t_a;  // host wait for the device loop
            if (seen) {
                std::memcpy(fin.m, out->T, sizeof(fin.m));
                it = out->iters;
                c->work[5] += it;
                dev_done = true;
            } else {
                // the grid-wide loop timed out (its workgroups were not all resident at once, ADVICE
                // r04): the call runs the host loop below from the start instead of failing
                ++c->work[3];
            }
        }
        if (!dev_done) {
            // PCL's loop on the host (float Umeyama, convergence), the exact 1-NN of every iteration on
            // the device: one launch for iteration 0 (keys + every source's candidate list) and one
            // persistent launch for the rest, handed over through coherent pinned memory: the host
            // releases iteration j with its step transform, the kernel stores the keys
            // (double-buffered by iteration parity) and flags them done. One stream sync per call.
            std::vector<float> cur(src, src + 3 * (size_t)ns), tb(3 * (size_t)ns);
            c->p_isync.coherent = true;
            c->p_ibest.coherent = true;
            HIPCHK(c->p_isync.ensure(1), "alloc icp sync");
            HIPCHK(c->p_ibest.ensure(2 * (size_t)ns), "alloc icp keys");
            const int nb0 = icp_lists_blocks(ns), nb1 = icp_iter_blocks(ns);
            c->p_idone.coherent = true;
            HIPCHK(c->p_idone.ensure((size_t)nb0 + nb1), "alloc icp flags");
            HIPCHK(c->p_src2.ensure(3 * (size_t)ns), "alloc pinned icp positions");
            int* done0 = c->p_idone.p;
            int* done1 = c->p_idone.p + nb0;
            std::memset(c->p_idone.p, 0, sizeof(int) * ((size_t)nb0 + nb1));
            // host copy of the targets (the Umeyama step's pairs), before the persistent kernel is queued
            const float* tg = tgt;
            std::vector<float> h_tgt;
            if (!tg) {
                h_tgt.resize(3 * (size_t)nt);
                HIPCHK(c->p_tgt.ensure(3 * (size_t)nt), "alloc pinned tgt");
                HIPCHK(kcopy(c->p_tgt.p, d_tgt, sizeof(float) * 3 * nt, c->stream), "D2H icp targets");
                HIPCHK(hipStreamSynchronize(c->stream), "sync icp targets");
                std::memcpy(h_tgt.data(), c->p_tgt.p, sizeof(float) * 3 * nt);
                tg = h_tgt.data();
            }
            IcpSync* sy = c->p_isync.p;
            std::memset(sy, 0, sizeof(IcpSync));
            std::atomic_thread_fence(std::memory_order_seq_cst);
            const int sg14 = c->stage_begin(BSHOT_STAGE_ICP);
            HIPCHK(launch_icp_lists_host(d_src0, ns, g4, c->itgt.p, nt, ICP_LIST_CAP, c->ilst.p, c->ilsd.p, c->ilcnt.p,
                                         c->ilcen.p, c->p_ibest.p, done0, c->stream),
                   "icp lists");
            if (!c->iqstat.p) {
                HIPCHK(c->iqstat.ensure(2), "alloc icp stats");
                HIPCHK(kfill(c->iqstat.p, 0, 2 * sizeof(int), c->stream), "zero icp stats");
            }
            if (c->opt_icp_relay && !c->idsy) {
                HIPCHK(hipMalloc(&c->idsy, sizeof(IcpDevSync)), "alloc icp relay");
                HIPCHK(kfill(c->idsy, 0, sizeof(IcpDevSync), c->stream), "zero icp relay");
            }
            IcpDevSync* dsy = c->opt_icp_relay ? c->idsy : nullptr;
            HIPCHK(launch_icp_iterations(d_src0, ns, 1, c->ilst.p, c->ilsd.p, c->ilcnt.p, c->ilcen.p, ICP_LIST_CAP, g4,
                                         c->itgt.p, nt, max_iter, sy, done1, c->p_ibest.p, c->stream, c->iqstat.p, dsy,
                                         ++c->icp_relay_seq),
                   "icp iterations");
            c->stage_end(sg14);
            auto release = [&](int go) { __atomic_store_n(&sy->go, go, __ATOMIC_RELEASE); };
            int j_lists = 0;  // the iteration whose keys the lists kernel delivers (0, or a restart's)
            // iteration j's keys are complete when every workgroup's flag says so. false: the device
            // went idle without them (its kernel outwaited a slow host and exited): the
            // caller restarts the iterations from the current positions. A busy GPU is waited for.
            auto wait_keys = [&](int j) -> bool {
                const int nb = j == j_lists ? nb0 : nb1;
                int* flags = j == j_lists ? done0 : done1;
                const int want = j == j_lists ? 1 : j;
                const long long t0 = ns_now();
                unsigned spins = 0;
                for (int w = 0; w < nb; ++w) {
                    while (__atomic_load_n(&flags[w], __ATOMIC_ACQUIRE) < want) {
                        if ((++spins & 1023) == 0 && ns_now() - t0 > 2000000ll &&
                            hipStreamQuery(c->stream) == hipSuccess && __atomic_load_n(&flags[w], __ATOMIC_ACQUIRE) < want)
                            return false;
                        __builtin_ia32_pause();
                    }
                }
                return true;
            };
            // restart at iteration j from the host's current positions: the lists kernel gives
            // iteration j's keys (exact 1-NN at cur) and lists around cur; the persistent kernel then
            // runs iterations j + 1 .. (the NN are exact from any list state, so the keys are unchanged)
            auto restart = [&](int j) -> int {
                (void)hipStreamSynchronize(c->stream);
                std::memcpy(c->p_src2.p, cur.data(), sizeof(float) * 3 * ns);
                std::memset(c->p_idone.p, 0, sizeof(int) * ((size_t)nb0 + nb1));
                std::atomic_thread_fence(std::memory_order_seq_cst);
                j_lists = j;
                ++c->work[3];  // ICP restarts
                HIPCHK(launch_icp_lists_host(c->p_src2.p, ns, g4, c->itgt.p, nt, ICP_LIST_CAP, c->ilst.p, c->ilsd.p,
                                             c->ilcnt.p, c->ilcen.p, c->p_ibest.p + (size_t)ns * (j & 1), done0,
                                             c->stream),
                       "icp lists (restart)");
                HIPCHK(launch_icp_iterations(c->p_src2.p, ns, j + 1, c->ilst.p, c->ilsd.p, c->ilcnt.p, c->ilcen.p,
                                             ICP_LIST_CAP, g4, c->itgt.p, nt, max_iter, sy, done1, c->p_ibest.p,
                                             c->stream, nullptr, dsy, ++c->icp_relay_seq),
                       "icp iterations (restart)");
                return BSHOT_OK;
            };
            double prev_mse = 1.7976931348623157e308;
            bg::Mat4f Ts = bg::Mat4f::identity();
            long long tw = ns_now();
            while (true) {
                const long long t_a = ns_now();
                if (!wait_keys(it)) {
                    if (int rc = restart(it)) return rc;
                    continue;
                }
                const long long t_b = ns_now();
                c->work[2] += t_b - t_a;              // host wait for the keys
                if (it == j_lists) c->work[8] += t_b - t_a;  // of which: the lists kernel's (iteration 0 or a restart)
                if (it > 0) c->work[4] += t_a - tw;  // host step between two waits
                const unsigned long long* best = c->p_ibest.p + (size_t)ns * (it & 1);
                for (int i = 0; i < ns; ++i) {
                    const unsigned j = (unsigned)(best[i] & 0xFFFFFFFFu);
                    tb[3 * i] = tg[3 * j]; tb[3 * i + 1] = tg[3 * j + 1]; tb[3 * i + 2] = tg[3 * j + 2];
                }
                Ts = bg::umeyama<float>(cur.data(), tb.data(), ns);
                ++it;
                if (it == 3 && c->opt_icp_host_delay_ms > 0)
                    std::this_thread::sleep_for(std::chrono::milliseconds(c->opt_icp_host_delay_ms));
                // the next iteration is released before this one's bookkeeping and convergence test
                // (PCL decides after the step); if the test stops the loop, its keys are never read
                if (it < max_iter) {
                    std::memcpy(sy->T, Ts.m, sizeof(Ts.m));
                    release(it);
                }
                for (int i = 0; i < ns; ++i) bg::xform(Ts, &cur[3 * i], &cur[3 * i]);  // the device applies Ts too
                fin = bg::mul(Ts, fin);
                if (it >= max_iter) break;
                const double cos_angle = 0.5 * (double)(((Ts.m[0] + Ts.m[5]) + Ts.m[10]) - 1.0f);
                const double tsq = (double)((Ts.m[3] * Ts.m[3] + Ts.m[7] * Ts.m[7]) + Ts.m[11] * Ts.m[11]);
                if (cos_angle >= 1.0 && tsq <= 0.0) break;
                double mse = 0;
                for (int i = 0; i < ns; ++i) mse += (double)__builtin_bit_cast(float, (unsigned)(best[i] >> 32));
                mse /= (double)ns;
                if (__builtin_fabs(mse - prev_mse) < 1e-12) break;
                prev_mse = mse;
                tw = t_b;
            }
            c->work[5] += it;
            release(-1);  // the persistent kernel's waves exit
            HIPCHK(hipStreamSynchronize(c->stream), "sync icp");
        }
        // the grids' range flag: its copy ran before the ICP kernels whose results were read above
        if (__atomic_load_n(c->p_icp_err.p, __ATOMIC_ACQUIRE) & 8)
            return c->fail("ICP target beyond the target grids' coordinate range (about +-524 km from the origin)",
                           BSHOT_ECAP);
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
    TraceScope trace_scope_("bshot_create");
    if (!out) return BSHOT_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return BSHOT_EHIP;
    if (device < 0 || device >= ndev) return BSHOT_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return BSHOT_EHIP;
    bshot_ctx* c = new bshot_ctx();
    c->device = device;
    c->htrace_on = std::getenv("BSHOT_HOST_TRACE") != nullptr;
    if (p) c->prm = *p;
    else bshot_default_params(&c->prm);
    // main stream at the highest priority: its short kernels (match, ICP) run during the host
    // phases while the side stream's lookahead SR fills the rest of the GPU
    int lo_prio = 0, hi_prio = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio);
    if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi_prio) != hipSuccess ||
        bsh::ctx_make_side_stream(c) != BSHOT_OK) {
        delete c;
        return BSHOT_EHIP;
    }
    // the packed SHOT apply relies on same-address ds_add_f32 lanes applying in ascending lane
    // order: checked once per device and process (a few ms); a device that fails runs the
    // one-rank-per-instruction apply (same results, slower)
    {
        static std::mutex m;
        static int checked[64];
        static int result[64];
        std::lock_guard<std::mutex> lk(m);
        if (device < 64 && !checked[device]) {
            result[device] = bsh::lds_lane_order_check(nullptr);
            checked[device] = 1;
        }
        c->hf_pack_ok = device < 64 && result[device] == 0;
    }
    *out = c;
    return BSHOT_OK;
}

int bshot_debug_lds_lane_order(bshot_ctx* c, int* mismatches, int* sensitive, int* active) {
    TraceScope trace_scope_("bshot_debug_lds_lane_order");
    if (!c || !mismatches) return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    int sens = 0;
    const int r = bsh::lds_lane_order_check(&sens);
    if (r < 0) return c->fail("lds lane-order check: HIP error", BSHOT_EHIP);
    *mismatches = r;
    if (sensitive) *sensitive = sens;
    if (active) *active = c->opt_hist_pack && c->hf_pack_ok;
    return BSHOT_OK;
}

void bshot_destroy(bshot_ctx* c) {
    if (!c) return;
    const bool trace = std::getenv("BSHOT_TRACE") != nullptr;
    if (trace) std::fprintf(stderr, "destroy enter\n");
    c->quiesce_replicas(1);  // the exchange forgets this context (its unindexed offers are dropped)
    (void)hipSetDevice(c->device);
    if (trace) std::fprintf(stderr, "destroy step 0\n");
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamSynchronize(c->pre);
    (void)hipStreamSynchronize(c->iss);
    if (trace) std::fprintf(stderr, "destroy step 1\n");
    c->resolve_events(true);
    if (trace) std::fprintf(stderr, "destroy step 2\n");
    for (auto e : c->evpool) (void)hipEventDestroy(e);
    (void)hipStreamSynchronize(c->side);
    if (trace) std::fprintf(stderr, "destroy step 3\n");
    // a context without marks (a second one in the same process) leaves the file alone
    if (c->htrace_on && !c->htrace.empty()) {
        if (FILE* f = std::fopen(std::getenv("BSHOT_HOST_TRACE"), "w")) {
            for (auto& e : c->htrace) std::fprintf(f, "%s,%lld\n", e.first, e.second);
            std::fclose(f);
        }
    }
    c->cs.release();
    if (trace) std::fprintf(stderr, "destroy step 4\n");
    c->pf.release();
    c->pf2.release();
    bsh::gmap_free(c);
    c->gtgt.release();
    for (auto& g : c->icp_lad) bsh::grid_free(g);
    c->errw.release(); c->normals.release(); c->kps.release(); c->counts.release(); c->offs.release();
    c->seg.release(); c->segtmp.release(); c->rf.release(); c->shot.release(); c->ok.release(); c->bits.release();
    c->ma.release(); c->lbest.release(); c->left.release();
    c->p_a.release(); c->p_bits.release(); c->p_left.release(); c->p_gidx.release(); c->p_err.release();
    c->p_g3.release(); c->p_src.release(); c->p_tgt.release(); c->p_best.release(); c->p_i64.release(); c->p_xyz.release();
    c->p_nrm.release(); c->normals_snap.release();
    if (c->ev_xyz) (void)hipEventDestroy(c->ev_xyz);
    c->rpts.release(); c->rhyp.release(); c->rcnt.release(); c->p_rpts.release(); c->p_rhyp.release(); c->p_rcnt.release();
    c->sbh.release(); c->sbst.release(); c->p_kidx.release(); c->p_kps3.release();
    bsh::pre_free(c->prep);
    c->prep = nullptr;
    bsh::velo_free(c->velo);
    c->velo = nullptr;
    c->gout.release(); c->ilst.release(); c->ilsd.release(); c->ilcnt.release(); c->p_iout.release(); c->p_isync.release(); c->p_ibest.release(); c->p_idone.release(); c->p_src2.release(); c->ipos.release(); c->ilcen.release(); c->irec.release(); c->ictl.release(); c->isync.release(); c->itgt3.release(); c->itgt.release(); c->ibest.release(); c->iqstat.release();
    if (c->idsy) (void)hipFree(c->idsy);
    c->idsy = nullptr;
    if (trace) std::fprintf(stderr, "destroy step 5\n");
    (void)hipStreamDestroy(c->stream);
    if (trace) std::fprintf(stderr, "destroy step 6\n");
    (void)hipStreamDestroy(c->side);
    (void)hipStreamDestroy(c->iss);
    (void)hipStreamDestroy(c->pre);
    flush_deferred_frees();  // buffers parked by regrowths (regrow.h)
    delete c;
}

const char* bshot_last_error(const bshot_ctx* c) { return c ? c->err.c_str() : "null context"; }

int bshot_sync(bshot_ctx* c) {
    TraceScope trace_scope_("bshot_sync");
    if (hipStreamSynchronize(c->stream) != hipSuccess || hipStreamSynchronize(c->side) != hipSuccess ||
        hipStreamSynchronize(c->iss) != hipSuccess || hipStreamSynchronize(c->pre) != hipSuccess)
        return c->fail("sync", hipGetLastError());
    c->resolve_events();
    return BSHOT_OK;
}

void* bshot_stream(bshot_ctx* c) { return (void*)c->stream; }

int bshot_set_cloud(bshot_ctx* c, const float* xyz, int n) {
    TraceScope trace_scope_("bshot_set_cloud");
    if (!c || (n > 0 && !xyz)) return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    // the current cloud's buffers may still be read by the side stream (its ISS)
    if (c->cs.iss_state == 1) HIPCHK(hipStreamWaitEvent(c->stream, c->cs.ev_iss, 0), "wait iss");
    HIPCHK(c->cs.xyz.ensure(3 * (size_t)(n > 0 ? n : 1)), "alloc xyz");
    if (n > 0) {
        // staged through pinned memory and moved by a kernel (no copy engine); the staging buffer is
        // refilled only after the previous cloud's copy has run
        if (c->ev_xyz) HIPCHK(hipEventSynchronize(c->ev_xyz), "wait staged cloud");
        else HIPCHK(hipEventCreateWithFlags(&c->ev_xyz, hipEventDisableTiming), "event");
        HIPCHK(c->p_xyz.ensure(3 * (size_t)n), "alloc pinned xyz");
        std::memcpy(c->p_xyz.p, xyz, sizeof(float) * 3 * n);
        HIPCHK(kcopy(c->cs.xyz.p, c->p_xyz.p, sizeof(float) * 3 * n, c->stream), "H2D xyz");
        HIPCHK(hipEventRecord(c->ev_xyz, c->stream), "record staged cloud");
    }
    return ctx_set_cloud_dev(c, c->cs.xyz.p, n);
}

int bshot_set_cloud_device(bshot_ctx* c, const float* d_xyz, int n) {
    TraceScope trace_scope_("bshot_set_cloud_device");
    if (!c || (n > 0 && !d_xyz)) return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    return ctx_set_cloud_dev(c, d_xyz, n);
}

int bshot_prefetch_cloud_device(bshot_ctx* c, const float* d_xyz, int n) {
    TraceScope trace_scope_("bshot_prefetch_cloud_device");
    if (!c || n < 0 || (n > 0 && !d_xyz)) return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    return ctx_prefetch_dev(c, d_xyz, n);
}

int bshot_queue_cloud_device(bshot_ctx* c, const float* d_xyz, int n) {
    TraceScope trace_scope_("bshot_queue_cloud_device");
    if (!c || n < 0 || (n > 0 && !d_xyz)) return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    return ctx_queue_dev(c, d_xyz, n);
}

int bshot_seg_ratio(bshot_ctx* c, int32_t* idx, float* ratio, int* n_out) {
    TraceScope trace_scope_("bshot_seg_ratio");
    if (!c || !n_out) return BSHOT_EINVAL;
    int rc = ctx_sr_launch(c);
    if (rc) return rc;
    CloudState& s = c->cs;
    HIPCHK(hipEventSynchronize(s.ev_sr), "sync ratio");
    c->resolve_events();
    if (s.h_err.p[0]) return c->fail(sr_error_message(s.h_err.p[0]), BSHOT_ECAP);
    const int n = s.n;
    const float* h = s.h_ratio.p;
    int m = 0;
    for (int i = 0; i < n; ++i) {
        const float r = h[i];
        if (r != r) continue;  // origin, non-finite or NaN ratio (src/lidar_odometry.cpp:63-64,121-122)
        idx[m] = i;
        ratio[m] = r;
        ++m;
    }
    *n_out = m;
    return BSHOT_OK;
}

int bshot_iss(bshot_ctx* c, int32_t* kp_idx, int cap, int* n_out) {
    TraceScope trace_scope_("bshot_iss");
    if (!c || !n_out) return BSHOT_EINVAL;
    int rc = ctx_iss_launch(c);
    if (rc) return rc;
    CloudState& s = c->cs;
    HIPCHK(hipEventSynchronize(s.ev_iss), "sync iss");
    c->resolve_events();
    if (s.h_err.p[1] & 4) return c->fail("iss: more than 512 neighbours inside the salient radius", BSHOT_ECAP);
    const int n = s.n;
    int m = 0;
    for (int i = 0; i < n; ++i)
        if (s.h_flag.p[i]) {
            if (m < cap) kp_idx[m] = i;
            ++m;
        }
    *n_out = m;
    return m <= cap ? BSHOT_OK : BSHOT_ECAP;
}

int bshot_describe(bshot_ctx* c, const float* kps, int k, float* shot, float* rf, uint32_t* bits) {
    TraceScope trace_scope_("bshot_describe");
    if (!c || k < 0 || (k > 0 && (!kps || !bits))) return BSHOT_EINVAL;
    if (!c->cs.grids_ok && c->cs.n > 0) return c->fail("bshot_describe: no cloud set", BSHOT_ESTATE);
    HIPCHK(c->kps.ensure(3 * (size_t)(k > 0 ? k : 1)), "alloc kps");
    if (k > 0) HIPCHK(hipMemcpyAsync(c->kps.p, kps, sizeof(float) * 3 * k, hipMemcpyHostToDevice, c->stream), "H2D kps");
    int rc = ctx_describe_dev(c, k);
    if (rc) return rc;
    int herr[4] = {0, 0, 0, 0};
    for (int attempt = 0; attempt < 3; ++attempt) {
        if (k > 0) {
            HIPCHK(hipMemcpyAsync(bits, c->bits.p, sizeof(uint32_t) * 11 * k, hipMemcpyDeviceToHost, c->stream), "D2H bits");
            if (shot) HIPCHK(hipMemcpyAsync(shot, c->shot.p, sizeof(float) * 352 * k, hipMemcpyDeviceToHost, c->stream), "D2H shot");
            if (rf) HIPCHK(hipMemcpyAsync(rf, c->rf.p, sizeof(float) * 9 * k, hipMemcpyDeviceToHost, c->stream), "D2H rf");
            HIPCHK(hipMemcpyAsync(herr, c->errw.p, 4 * sizeof(int), hipMemcpyDeviceToHost, c->stream), "D2H err");
        }
        HIPCHK(hipStreamSynchronize(c->stream), "sync describe");
        c->resolve_events();
        if (k > 0 && ctx_describe_replan(c, herr)) {
            // the device-side plan ran out of capacity: again, planned on the host
            if ((rc = ctx_describe_dev(c, k))) return rc;
            continue;
        }
        break;
    }
    if (herr[0] & 2) return c->fail("normals: neighbourhood with too many exactly tied boundary keys (kNN list overflow)", BSHOT_ECAP);
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
    TraceScope trace_scope_("bshot_match");
    if (!c || !n_corr || na < 0 || nb < 0) return BSHOT_EINVAL;
    *n_corr = 0;
    if (na == 0 || nb == 0) return BSHOT_OK;
    HIPCHK(c->ma.ensure(11 * ((size_t)na + nb)), "alloc descriptors");
    HIPCHK(c->p_a.ensure(11 * ((size_t)na + nb)), "alloc pinned descriptors");
    HIPCHK(c->p_left.ensure(2 * (size_t)na + nb), "alloc pinned match out");
    std::memcpy(c->p_a.p, a, sizeof(uint32_t) * 11 * na);
    std::memcpy(c->p_a.p + 11 * (size_t)na, b, sizeof(uint32_t) * 11 * nb);
    HIPCHK(kcopy(c->ma.p, c->p_a.p, sizeof(uint32_t) * 11 * ((size_t)na + nb),
                          c->stream),
           "H2D descriptors");
    int rc = ctx_match_dev(c, na, nb);
    if (rc) return rc;
    HIPCHK(kcopy(c->p_left.p, c->left.p, sizeof(int) * (2 * (size_t)na + nb),
                          c->stream),
           "D2H match");
    HIPCHK(hipStreamSynchronize(c->stream), "sync match");
    c->resolve_events();
    std::memcpy(left_nn, c->p_left.p, sizeof(int) * na);
    std::memcpy(right_nn, c->p_left.p + na, sizeof(int) * nb);
    const int* flag = c->p_left.p + na + nb;
    int m = 0;
    for (int i = 0; i < na; ++i)
        if (flag[i]) { corr_q[m] = i; corr_m[m] = left_nn[i]; ++m; }
    *n_corr = m;
    return BSHOT_OK;
}

int bshot_icp(bshot_ctx* c, const float* src, int ns, const float* tgt, int nt, int max_iter, float* T_out, int* iters) {
    TraceScope trace_scope_("bshot_icp");
    if (!c || !T_out || !iters || ns < 0 || nt < 0) return BSHOT_EINVAL;
    int rc = ctx_icp(c, src, ns, tgt, nt, max_iter, T_out, iters);
    c->resolve_events();
    return rc;
}

int bshot_stage_times(bshot_ctx* c, double* ms, int64_t* launches, int n) {
    TraceScope trace_scope_("bshot_stage_times");
    if (!c) return BSHOT_EINVAL;
    c->resolve_events(true);
    for (int i = 0; i < n && i < BSHOT_NSTAGES; ++i) {
        if (ms) ms[i] = c->stage_ms[i];
        if (launches) launches[i] = c->stage_n[i];
    }
    return BSHOT_NSTAGES;
}

void bshot_stage_reset(bshot_ctx* c) {
    TraceScope trace_scope_("bshot_stage_reset");
    if (!c) return;
    c->resolve_events(true);
    for (int i = 0; i < BSHOT_NSTAGES; ++i) { c->stage_ms[i] = 0; c->stage_n[i] = 0; }
}

void bshot_set_timing(bshot_ctx* c, int enabled) {
    if (c) c->timing = enabled != 0;
}

int bshot_radius_pairs(bshot_ctx* c, float R, int64_t* total) {
    if (!c || !total) return BSHOT_EINVAL;
    *total = 0;
    if (c->cs.n == 0) return BSHOT_OK;
    if (!c->cs.grids_ok) return c->fail("bshot_radius_pairs: no cloud", BSHOT_ESTATE);
    DBuf<int> cnt;
    DBuf<long long> offs;
    HIPCHK(cnt.ensure(c->cs.n), "alloc counts");
    HIPCHK(offs.ensure(c->cs.n + 1), "alloc offs");
    const bsh::DevGrid& g = R <= c->prm.iss_salient * 1.5f && c->cs.grid_iss.n == c->cs.n ? c->cs.grid_iss : c->cs.grid_coarse;
    HIPCHK(launch_shot_count(g, c->cs.d_xyz, c->cs.n, R, cnt.p, offs.p, c->stream), "radius count");
    long long t = 0;
    HIPCHK(hipMemcpyAsync(&t, offs.p + c->cs.n, sizeof(long long), hipMemcpyDeviceToHost, c->stream), "D2H");
    HIPCHK(hipStreamSynchronize(c->stream), "sync");
    cnt.release();
    offs.release();
    *total = t;
    return BSHOT_OK;
}

int bshot_debug_knn_stats(bshot_ctx* c, int64_t* out, int n) {
    TraceScope trace_scope_("bshot_debug_knn_stats");
    if (!c || !out) return BSHOT_EINVAL;
    if (!c->cs.grids_ok) return c->fail("bshot_debug_knn_stats: no cloud", BSHOT_ESTATE);
    DBuf<unsigned long long> k;
    HIPCHK(k.ensure(32), "alloc kst");
    HIPCHK(c->cs.ratio.ensure(c->cs.n), "alloc ratio");
    HIPCHK(hipMemsetAsync(k.p, 0, 32 * sizeof(unsigned long long), c->stream), "memset");
    HIPCHK(launch_seg_ratio(c->cs.ladder, c->ladder_mode(c->cs), c->cs.pts4.p, c->cs.n, c->prm.seg_radius, c->prm.seg_max_nn, c->prm.sr_type,
                            c->opt_sr_start, c->cs.ratio.p, c->cs.errw.p, c->stream, k.p, c->opt_sr_blocks, c->opt_sr_xcd_chunk,
                                c->opt_sr_run, (float)c->opt_sr_bratio / 100.f),
           "seg_ratio (stats)");
    unsigned long long h[32];
    HIPCHK(hipMemcpyAsync(h, k.p, sizeof(h), hipMemcpyDeviceToHost, c->stream), "D2H");
    HIPCHK(hipStreamSynchronize(c->stream), "sync");
    k.release();
    for (int i = 0; i < n && i < 32; ++i) out[i] = (int64_t)h[i];
    return 32;
}

int bshot_set_option(bshot_ctx* c, const char* name, int value) {
    TraceScope trace_scope_("bshot_set_option");
    if (!c || !name) return BSHOT_EINVAL;
    const std::string k(name);
    if (k == "ladder_grids") c->opt_ladder4 = value == 4 ? 1 : 0;
    else if (k == "iss_cell") c->opt_iss_cell = value >= 2 ? 2 : 1;
    else if (k == "sr_start") c->opt_sr_start = value < 0 ? 0 : value;
    else if (k == "normals_seg") c->opt_normals_seg = value ? 1 : 0;
    else if (k == "host_map_log") c->opt_host_map_log = value ? 1 : 0;
    else if (k == "map_sync") c->opt_map_sync = value ? 1 : 0;
    else if (k == "ladder_front") c->opt_ladder_front = value ? 1 : 0;
    else if (k == "sr_blocks") c->opt_sr_blocks = value < 0 ? 0 : value;
    else if (k == "sr_xcd_chunk") c->opt_sr_xcd_chunk = value < 0 ? 0 : value;
    else if (k == "sr_run") c->opt_sr_run = value < 1 ? 1 : value;
    else if (k == "sr_bratio") c->opt_sr_bratio = value < 101 ? 101 : value;
    else if (k == "icp_device") c->opt_icp_device = value ? 1 : 0;
    else if (k == "icp_host_delay_ms") c->opt_icp_host_delay_ms = value < 0 ? 0 : value;
    else if (k == "diag_skip_icp") c->opt_diag_skip_icp = value ? 1 : 0;  // diagnostic: the period without ICP
    else if (k == "rank_max") c->opt_rank_max = value;
    else if (k == "hist_pack") c->opt_hist_pack = value ? 1 : 0;
    else if (k == "rank_wg") c->opt_rank_wg = value < 0 ? 0 : (value > 2 ? 2 : value);
    else if (k == "desc_slices") c->opt_desc_slices = value < 1 ? 1 : (value > 64 ? 64 : value);
    else if (k == "iss_defer") c->opt_iss_defer = value ? 1 : 0;
    else if (k == "gpu_map") c->opt_gpu_map = value < 0 ? 0 : (value > 2 ? 2 : value);
    else if (k == "xseq_targets") c->opt_xseq_targets = value ? 1 : 0;
    else if (k == "xchg_index") c->opt_xchg_index = value ? 1 : 0;
    else if (k == "topk_thread") c->opt_topk_thread = value ? 1 : 0;
    else if (k == "iss_grid") c->opt_iss_grid = value ? 1 : 0;
    else if (k == "iss_ovf_blocks") c->opt_iss_ovf_blocks = value < 0 ? 0 : value;
    else if (k == "iss_xcd_chunk") c->opt_iss_xcd_chunk = value < 0 ? 0 : value;
    else if (k == "gmap_slots0") c->opt_gmap_slots0 = value < 2 ? 2 : value;
    else if (k == "icp_relay") c->opt_icp_relay = value ? 1 : 0;
    else if (k == "pre_fast") c->opt_pre_fast = value ? 1 : 0;
    else if (k == "iss_nms_blocks") c->opt_iss_nms_blocks = value < 0 ? 0 : value;
    else if (k == "ransac_dev") c->opt_ransac_dev = value ? 1 : 0;
    else if (k == "chunk_blocks") c->opt_chunk_blocks = value < 0 ? 0 : value;
    else if (k == "timing_mask") c->timing_mask = (unsigned)value;
    else if (k == "dev_plan_hint") c->seg_hint = value < 0 ? 0 : value;  // tests: force / avoid a re-plan
    else if (k == "side_prio") {
        c->opt_side_prio = value < 0 ? 0 : (value > 2 ? 2 : value);
        return bsh::ctx_make_side_stream(c);
    }
    else return c->fail("bshot_set_option: unknown option " + k, BSHOT_EINVAL);
    return BSHOT_OK;
}

int bshot_work_counters(bshot_ctx* c, int64_t* out, int n) {
    if (!c) return BSHOT_EINVAL;
    c->work[6] = g_regrow_n.load();
    c->work[7] = g_regrow_bytes.load();
    if (n > 9 && c->iqstat.p) {
        int q[2] = {0, 0};
        if (hipStreamSynchronize(c->stream) == hipSuccess &&
            hipMemcpy(q, c->iqstat.p, sizeof(q), hipMemcpyDeviceToHost) == hipSuccess) {
            c->work[9] = q[0];
            c->work[10] = q[1];
        }
    }
    for (int i = 0; i < n && i < 12; ++i) out[i] = c->work[i];
    return 12;
}

}  // extern "C"
