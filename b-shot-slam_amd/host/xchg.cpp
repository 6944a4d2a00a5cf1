// xchg.cpp -- the map exchange of BASELINE config 4 in C++ over RCCL: after each
// sweep every rank all-gathers its map offer (the sweep's keypoints on the 10 mm grid, ratios and
// B-SHOT words, packed in HBM by gmap_pack_delta) and inserts the other ranks' batches into its
// GPU replicas of their maps (gmap_insert_records). Device buffers end to end, on the context's main
// stream; no host synchronisation inside the step. RCCL is loaded at run time (dlopen), so the
// library has no link-time dependency on it and shares the copy PyTorch has already loaded.
#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../csrc/ctx.h"
#include "../csrc/gmap.h"
#include "../csrc/kernels.h"
#include "../../include/bshot/lidar_odometry.h"
#include "../../include/bshot_abi.h"

namespace {

// the RCCL entry points used (rccl/rccl.h signatures; opaque types kept opaque)
struct UniqueId {  // ncclUniqueId: passed by value to ncclCommInitRank
    char internal[128];
};
typedef int (*fn_get_id)(UniqueId*);
typedef int (*fn_init_rank)(void**, int, UniqueId, int);
typedef int (*fn_all_gather)(const void*, void*, size_t, int, void*, hipStream_t);
typedef int (*fn_destroy)(void*);
typedef const char* (*fn_err)(int);
constexpr int kNcclFloat32 = 7;  // ncclFloat32 in rccl.h's ncclDataType_t

struct Rccl {
    void* h = nullptr;
    fn_get_id get_id = nullptr;
    fn_init_rank init_rank = nullptr;
    fn_all_gather all_gather = nullptr;
    fn_destroy destroy = nullptr;
    fn_err err = nullptr;
    bool load() {
        if (h) return true;
        for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
            if (h) break;
        }
        if (!h) return false;
        get_id = (fn_get_id)dlsym(h, "ncclGetUniqueId");
        init_rank = (fn_init_rank)dlsym(h, "ncclCommInitRank");
        all_gather = (fn_all_gather)dlsym(h, "ncclAllGather");
        destroy = (fn_destroy)dlsym(h, "ncclCommDestroy");
        err = (fn_err)dlsym(h, "ncclGetErrorString");
        return get_id && init_rank && all_gather && destroy;
    }
};

Rccl& rccl() {
    static Rccl r;
    return r;
}

}  // namespace

struct bshot_xchg {
    void* comm = nullptr;
    int nranks = 0, rank = 0, device = 0, kmax = 0;
    float* send = nullptr;  // GM_REC_HDR + GM_REC_W * kmax floats
    float* recv = nullptr;  // nranks x that: the buffer the current exchange gathers into (rbuf[par])
    // Replica policy (context option xchg_index):
    // 1 (default, eager): every exchange is indexed into the replicas right away, on the iss stream
    //   behind the all-gather (one batched insert for all of them, gmap_insert_records_multi); the
    //   main stream does not wait for it. The gathers alternate between two receive buffers, so the
    //   next all-gather only waits for the inserts of the exchange before last.
    // 0 (lazy): the offers are logged in HBM (below) and indexed only when something reads a replica.
    float* rbuf[2] = {nullptr, nullptr};
    hipEvent_t ev_rbuf[2] = {nullptr, nullptr};  // the eager inserts reading rbuf[i] are done (iss stream)
    bool rbuf_busy[2] = {false, false};
    int par = 0;
    hipEvent_t ev_gathered = nullptr;  // main stream: the all-gather into recv has landed
    // Received offers (lazy policy), append-only in HBM: one gathered recv image per exchange, copied
    // off recv on the main stream right after the all-gather. The replicas index them only when
    // something reads a replica (bshot_odom_gpu_replica_*, the Python transport's insert, or
    // xseq_targets, which inserts every exchange at once): the per-sweep cost without a reader is the
    // all-gather and one HBM copy. A full log is indexed (replayed in exchange order) before it takes more.
    float* log = nullptr;
    size_t log_cap = 0;                             // floats
    std::vector<std::pair<int, int>> log_entries;   // per logged exchange: include_self, sim_peers
    hipEvent_t ev_inserted = nullptr;  // the replica inserts reading the log (or recv) are done (their stream)
    bool inserts_queued = false;
    bshot_ctx* jc = nullptr;  // the context whose replicas the log feeds
    // Threading: a context is driven by one host thread at a time (bshot_abi.h), and so are the
    // exchange feeding its replicas and the replica readers (bshot_odom_gpu_replica_*, which index the
    // log through quiesce): a reader on another thread while an exchange runs is not supported -- the
    // next exchange's inserts may grow (reallocate) a replica's pools under the reader's query kernel
    // (ADVICE r05). mu only orders the log against bshot_xchg_destroy and the context's detach.
    std::mutex mu;
};

namespace {

size_t per_rank(const bshot_xchg* x) { return bsh::GM_REC_HDR + (size_t)bsh::GM_REC_W * x->kmax; }

// insert one gathered image (nranks x per floats) into the replicas on stream xs: replica r gets
// rank r's batch, the simulated peers' replicas this rank's. Batched launches, up to 8 replicas each
// (every replica's batches stay in exchange order: a replica appears once per image).
int insert_image(bshot_ctx* c, bshot_xchg* x, const float* img, int include_self, int sim_peers, hipStream_t xs) {
    const size_t per = per_rank(x);
    std::vector<int> reps;
    std::vector<const float*> recs;
    for (int r = 0; r < x->nranks; ++r) {
        if (r == x->rank && !include_self) continue;
        reps.push_back(r);
        recs.push_back(img + per * r);
    }
    for (int p = 0; p < sim_peers; ++p) {
        reps.push_back(x->nranks + p);
        recs.push_back(img + per * x->rank);
    }
    constexpr int kBatch = 8;
    for (size_t a = 0; a < reps.size(); a += kBatch) {
        const int n = (int)std::min<size_t>(kBatch, reps.size() - a);
        if (int rc = bsh::gmap_insert_records_multi(c, n, reps.data() + a, recs.data() + a, x->kmax, xs)) return rc;
    }
    return BSHOT_OK;
}

// index every logged exchange (owner order kept: exchange order per replica), queued on the iss
// stream behind the main stream's copies into the log; the log is empty afterwards
int replay_log(bshot_ctx* c, bshot_xchg* x) {
    if (x->log_entries.empty()) return BSHOT_OK;
    hipStream_t xs = c->iss;
    if (int rc = bsh::gmap_settle_replicas_noquiesce(c)) return rc;
    if (hipEventRecord(x->ev_inserted, c->stream) != hipSuccess || hipStreamWaitEvent(xs, x->ev_inserted, 0) != hipSuccess)
        return c->fail("exchange: stream wait", BSHOT_EHIP);
    const size_t img = per_rank(x) * x->nranks;
    for (size_t e = 0; e < x->log_entries.size(); ++e)
        if (int rc = insert_image(c, x, x->log + img * e, x->log_entries[e].first, x->log_entries[e].second, xs)) {
            x->log_entries.clear();
            return rc;
        }
    x->log_entries.clear();
    if (hipEventRecord(x->ev_inserted, xs) != hipSuccess) return c->fail("exchange: event", BSHOT_EHIP);
    x->inserts_queued = true;
    return BSHOT_OK;
}

// before any access to the replicas: index the log; detach: the context is being destroyed, the
// exchange must not reach it any more (the log is dropped)
int quiesce(void* arg, int detach) {
    auto* x = static_cast<bshot_xchg*>(arg);
    std::lock_guard<std::mutex> lk(x->mu);
    if (detach) {
        x->log_entries.clear();
        x->jc = nullptr;
        return BSHOT_OK;
    }
    return x->jc ? replay_log(x->jc, x) : BSHOT_OK;
}

}  // namespace

extern "C" {

int bshot_xchg_unique_id(void* id128) {
    if (!id128) return BSHOT_EINVAL;
    if (!rccl().load()) return BSHOT_EHIP;
    UniqueId id;
    if (rccl().get_id(&id) != 0) return BSHOT_EHIP;
    std::memcpy(id128, id.internal, 128);
    return BSHOT_OK;
}

int bshot_xchg_create(bshot_xchg** out, const void* id128, int nranks, int rank, int device, int kmax) {
    if (!out || !id128 || nranks < 1 || rank < 0 || rank >= nranks || kmax < 1) return BSHOT_EINVAL;
    *out = nullptr;
    if (!rccl().load()) return BSHOT_EHIP;
    if (hipSetDevice(device) != hipSuccess) return BSHOT_EHIP;
    auto* x = new bshot_xchg();
    x->nranks = nranks;
    x->rank = rank;
    x->device = device;
    x->kmax = kmax;
    const size_t per = bsh::GM_REC_HDR + (size_t)bsh::GM_REC_W * kmax;
    if (hipMalloc(&x->send, sizeof(float) * per) != hipSuccess ||
        hipMalloc(&x->rbuf[0], sizeof(float) * per * nranks) != hipSuccess ||
        hipMalloc(&x->rbuf[1], sizeof(float) * per * nranks) != hipSuccess ||
        hipEventCreateWithFlags(&x->ev_inserted, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->ev_gathered, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->ev_rbuf[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->ev_rbuf[1], hipEventDisableTiming) != hipSuccess) {
        bshot_xchg_destroy(x);
        return BSHOT_EHIP;
    }
    x->recv = x->rbuf[0];
    UniqueId id;
    std::memcpy(id.internal, id128, 128);
    if (rccl().init_rank(&x->comm, nranks, id, rank) != 0) {
        x->comm = nullptr;
        bshot_xchg_destroy(x);
        return BSHOT_EHIP;
    }
    *out = x;
    return BSHOT_OK;
}

void bshot_xchg_destroy(bshot_xchg* x) {
    if (!x) return;
    // the context (still alive: its teardown would have detached it) must not call back into x; the
    // log's offers are indexed first, so its replicas stay complete
    {
        std::lock_guard<std::mutex> lk(x->mu);
        if (x->jc && x->jc->replica_quiesce_arg == x) {
            (void)replay_log(x->jc, x);
            x->jc->replica_quiesce = nullptr;
        }
    }
    if (x->comm) rccl().destroy(x->comm);
    for (hipEvent_t* e : {&x->ev_inserted, &x->ev_rbuf[0], &x->ev_rbuf[1], &x->ev_gathered})
        if (*e) {
            (void)hipEventSynchronize(*e);
            (void)hipEventDestroy(*e);
        }
    if (x->send) (void)hipFree(x->send);
    for (float* b : x->rbuf)
        if (b) (void)hipFree(b);
    if (x->log) (void)hipFree(x->log);
    delete x;
}

}  // extern "C"

// declared in bshot_abi.h; defined here beside the exchange (uses the odometry's context).
// sim_peers > 0 (measurement, bshot_odom_exchange_sim): the gathered batch of this rank is also
// inserted into replicas nranks .. nranks + sim_peers - 1, as if that many more ranks had offered it
int bshot_odom_exchange_ctx(bshot_ctx* c, bshot_xchg* x, int include_self, int sim_peers) {
    if (!c || !x) return BSHOT_EINVAL;
    if (!c->gmap) return BSHOT_ESTATE;
    std::lock_guard<std::mutex> lk(x->mu);
    if (x->jc && x->jc != c) return c->fail("exchange: already feeding another odometry's replicas", BSHOT_EINVAL);
    const size_t per = per_rank(x), img = per * x->nranks;
    c->hmark("M_x_begin");
    int rc = bsh::gmap_pack_delta(c, x->kmax, x->send);
    if (rc) return rc;
    const bool eager = c->opt_xchg_index != 0 && !c->opt_xseq_targets;
    if (eager) {
        x->par ^= 1;
        x->recv = x->rbuf[x->par];
    }
    // the eager inserts that read this buffer (the exchange before last) are done before it is refilled
    if (x->rbuf_busy[x->par]) {
        if (hipStreamWaitEvent(c->stream, x->ev_rbuf[x->par], 0) != hipSuccess)
            return c->fail("exchange: stream wait", BSHOT_EHIP);
        x->rbuf_busy[x->par] = false;
    }
    const int e = rccl().all_gather(x->send, x->recv, per, kNcclFloat32, x->comm, c->stream);
    if (e != 0) return c->fail(std::string("ncclAllGather: ") + (rccl().err ? rccl().err(e) : "error"), BSHOT_EHIP);
    x->jc = c;
    c->replica_quiesce = quiesce;
    c->replica_quiesce_arg = x;
    if (eager) {
        // index this exchange now, on the iss stream behind the all-gather (after anything logged
        // under the lazy policy); nothing on the main stream waits for it
        if ((rc = replay_log(c, x))) return rc;
        if (hipEventRecord(x->ev_gathered, c->stream) != hipSuccess || hipStreamWaitEvent(c->iss, x->ev_gathered, 0) != hipSuccess)
            return c->fail("exchange: stream wait", BSHOT_EHIP);
        if ((rc = insert_image(c, x, x->recv, include_self, sim_peers, c->iss))) return rc;
        if (hipEventRecord(x->ev_rbuf[x->par], c->iss) != hipSuccess) return c->fail("exchange: event", BSHOT_EHIP);
        x->rbuf_busy[x->par] = true;
    } else if (c->opt_xseq_targets) {
        // the matching reads the replicas: index this exchange now (after anything logged), on the iss
        // stream, and let the main stream wait for it
        if ((rc = replay_log(c, x))) return rc;
        if ((rc = bsh::gmap_settle_replicas_noquiesce(c))) return rc;
        if (hipEventRecord(x->ev_inserted, c->stream) != hipSuccess || hipStreamWaitEvent(c->iss, x->ev_inserted, 0) != hipSuccess)
            return c->fail("exchange: stream wait", BSHOT_EHIP);
        if ((rc = insert_image(c, x, x->recv, include_self, sim_peers, c->iss))) return rc;
        if (hipEventRecord(x->ev_inserted, c->iss) != hipSuccess || hipStreamWaitEvent(c->stream, x->ev_inserted, 0) != hipSuccess)
            return c->fail("exchange: stream wait", BSHOT_EHIP);
        x->inserts_queued = true;
    } else {
        // append the gathered image to the log (a full log is indexed first; its inserts read it, so
        // the copy waits for them)
        if ((x->log_entries.size() + 1) * img > x->log_cap) {
            if ((rc = replay_log(c, x))) return rc;
            if (img > x->log_cap) {
                size_t want = (size_t)256 << 20;  // floats: 1 GiB (BSHOT_XCHG_LOG_KB: tests of the full-log path)
                if (const char* v = std::getenv("BSHOT_XCHG_LOG_KB")) want = (size_t)std::max(1L, std::atol(v)) << 8;
                if (want < 4 * img) want = 4 * img;
                if (x->inserts_queued) (void)hipEventSynchronize(x->ev_inserted);
                if (x->log) (void)hipFree(x->log);
                x->log = nullptr;
                x->log_cap = 0;
                if (hipMalloc(&x->log, sizeof(float) * want) != hipSuccess) return c->fail("exchange: log alloc", BSHOT_EHIP);
                x->log_cap = want;
            }
        }
        if (x->log_entries.empty() && x->inserts_queued && hipStreamWaitEvent(c->stream, x->ev_inserted, 0) != hipSuccess)
            return c->fail("exchange: stream wait", BSHOT_EHIP);
        if (bsh::kcopy(x->log + img * x->log_entries.size(), x->recv, sizeof(float) * img, c->stream) != hipSuccess)
            return c->fail("exchange: log copy", BSHOT_EHIP);
        x->log_entries.emplace_back(include_self, sim_peers);
    }
    c->hmark("M_x_queued");
    return BSHOT_OK;
}
