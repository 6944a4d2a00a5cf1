// xchg.cpp -- the map exchange of BASELINE config 4 in C++ over RCCL: after each
// sweep every rank all-gathers its map offer (the sweep's keypoints on the 10 mm grid, ratios and
// B-SHOT words, packed in HBM by gmap_pack_delta) and inserts the other ranks' batches into its
// GPU replicas of their maps (gmap_insert_records). Device buffers end to end, on the context's main
// stream; no host synchronisation inside the step. RCCL is loaded at run time (dlopen), so the
// library has no link-time dependency on it and shares the copy PyTorch has already loaded.
#include <dlfcn.h>

#include <condition_variable>
#include <mutex>
#include <thread>

#include <cstring>
#include <string>

#include "../csrc/ctx.h"
#include "../csrc/gmap.h"
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
    float* recv = nullptr;  // nranks x that
    hipEvent_t ev_gathered = nullptr;  // the all-gather has landed in recv (main stream)
    hipEvent_t ev_inserted = nullptr;  // the replica inserts reading recv are done (their stream)
    bool inserts_queued = false;
    std::string err;
    // the replica inserts of an exchange are queued by this thread (settle the previous ones, reserve,
    // ~10 launches per replica), so the odometry's main thread hands them over and goes on
    std::thread worker;
    std::mutex mu;
    std::condition_variable cv;
    bool job = false, busy = false, stop = false;
    bshot_ctx* jc = nullptr;
    int j_self = 0, j_sim = 0;
    int werr = 0;
    std::string werr_msg;
};

namespace {

// settle the previous inserts, then queue this exchange's on the iss stream behind the all-gather
int queue_inserts(bshot_ctx* c, bshot_xchg* x, int include_self, int sim_peers) {
    const size_t per = bsh::GM_REC_HDR + (size_t)bsh::GM_REC_W * x->kmax;
    int rc = bsh::gmap_settle_replicas_noquiesce(c);
    if (rc) return rc;
    hipStream_t xs = c->iss;
    if (hipStreamWaitEvent(xs, x->ev_gathered, 0) != hipSuccess) return c->fail("exchange: stream wait", BSHOT_EHIP);
    for (int r = 0; r < x->nranks; ++r) {
        if (r == x->rank && !include_self) continue;
        rc = bsh::gmap_insert_records(c, r, x->recv + per * r, x->kmax, false, xs);
        if (rc) return rc;
    }
    for (int p = 0; p < sim_peers; ++p) {
        rc = bsh::gmap_insert_records(c, x->nranks + p, x->recv + per * x->rank, x->kmax, false, xs);
        if (rc) return rc;
    }
    if (hipEventRecord(x->ev_inserted, xs) != hipSuccess) return c->fail("exchange: event", BSHOT_EHIP);
    x->inserts_queued = true;
    return BSHOT_OK;
}

void worker_loop(bshot_xchg* x) {
    std::unique_lock<std::mutex> lk(x->mu);
    while (true) {
        x->cv.wait(lk, [x] { return x->job || x->stop; });
        if (!x->job) break;  // stop
        x->job = false;
        x->busy = true;
        bshot_ctx* c = x->jc;
        const int self = x->j_self, sim = x->j_sim;
        lk.unlock();
        (void)hipSetDevice(x->device);
        const int rc = queue_inserts(c, x, self, sim);
        lk.lock();
        if (rc && !x->werr) {
            x->werr = rc;
            x->werr_msg = bshot_last_error(c);
        }
        x->busy = false;
        x->cv.notify_all();
    }
}

// the worker has queued every insert handed to it (called before any host access to the replicas);
// detach: the context is being destroyed, the exchange must not reach it any more
void quiesce(void* arg, int detach) {
    auto* x = static_cast<bshot_xchg*>(arg);
    std::unique_lock<std::mutex> lk(x->mu);
    x->cv.wait(lk, [x] { return !x->job && !x->busy; });
    if (detach) x->jc = nullptr;
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
        hipMalloc(&x->recv, sizeof(float) * per * nranks) != hipSuccess ||
        hipEventCreateWithFlags(&x->ev_gathered, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->ev_inserted, hipEventDisableTiming) != hipSuccess) {
        bshot_xchg_destroy(x);
        return BSHOT_EHIP;
    }
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
    if (x->worker.joinable()) {
        {
            std::lock_guard<std::mutex> lk(x->mu);
            x->stop = true;
        }
        x->cv.notify_all();
        x->worker.join();
    }
    // the context (still alive: its teardown would have detached it) must not call back into x
    if (x->jc && x->jc->replica_quiesce_arg == x) x->jc->replica_quiesce = nullptr;
    if (x->comm) rccl().destroy(x->comm);
    if (x->ev_inserted) {
        (void)hipEventSynchronize(x->ev_inserted);
        (void)hipEventDestroy(x->ev_inserted);
    }
    if (x->ev_gathered) (void)hipEventDestroy(x->ev_gathered);
    if (x->send) (void)hipFree(x->send);
    if (x->recv) (void)hipFree(x->recv);
    delete x;
}

}  // extern "C"

// declared in bshot_abi.h; defined here beside the exchange (uses the odometry's context).
// sim_peers > 0 (measurement, bshot_odom_exchange_sim): the gathered batch of this rank is also
// inserted into replicas nranks .. nranks + sim_peers - 1, as if that many more ranks had offered it
int bshot_odom_exchange_ctx(bshot_ctx* c, bshot_xchg* x, int include_self, int sim_peers) {
    if (!c || !x) return BSHOT_EINVAL;
    if (!c->gmap) return BSHOT_ESTATE;
    const size_t per = bsh::GM_REC_HDR + (size_t)bsh::GM_REC_W * x->kmax;
    c->hmark("M_x_begin");
    // the previous exchange's inserts are queued (the worker is idle) and reported no error
    quiesce(x, 0);
    if (x->werr) {
        const int e = x->werr;
        x->werr = 0;
        return c->fail(x->werr_msg, e);
    }
    c->hmark("M_x_settled");
    int rc = bsh::gmap_pack_delta(c, x->kmax, x->send);
    if (rc) return rc;
    // recv is read by the previous exchange's inserts until they are done
    if (x->inserts_queued && hipStreamWaitEvent(c->stream, x->ev_inserted, 0) != hipSuccess)
        return c->fail("exchange: stream wait", BSHOT_EHIP);
    const int e = rccl().all_gather(x->send, x->recv, per, kNcclFloat32, x->comm, c->stream);
    if (e != 0) return c->fail(std::string("ncclAllGather: ") + (rccl().err ? rccl().err(e) : "error"), BSHOT_EHIP);
    // The replica inserts run on the low-priority iss stream, off the main stream: the next sweep's
    // map query and matching (the odometry's critical chain) do not queue behind them, and the
    // worker thread queues them (the main thread hands over and goes on). Only the cross-sequence
    // targets (xseq_targets) read the replicas: then they are queued here and the main stream waits.
    if (hipEventRecord(x->ev_gathered, c->stream) != hipSuccess) return c->fail("exchange: event", BSHOT_EHIP);
    if (c->opt_xseq_targets) {
        if ((rc = queue_inserts(c, x, include_self, sim_peers))) return rc;
        if (hipStreamWaitEvent(c->stream, x->ev_inserted, 0) != hipSuccess) return c->fail("exchange: stream wait", BSHOT_EHIP);
    } else {
        std::lock_guard<std::mutex> lk(x->mu);
        if (!x->worker.joinable()) x->worker = std::thread(worker_loop, x);
        x->jc = c;
        c->replica_quiesce = quiesce;
        c->replica_quiesce_arg = x;
        x->j_self = include_self;
        x->j_sim = sim_peers;
        x->job = true;
        x->cv.notify_all();
    }
    c->hmark("M_x_queued");
    return BSHOT_OK;
}
