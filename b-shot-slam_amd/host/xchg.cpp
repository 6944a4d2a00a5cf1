// xchg.cpp -- the map exchange of BASELINE config 4 in C++ over RCCL: after each
// sweep every rank all-gathers its map offer (the sweep's keypoints on the 10 mm grid, ratios and
// B-SHOT words, packed in HBM by gmap_pack_delta) and inserts the other ranks' batches into its
// GPU replicas of their maps (gmap_insert_records). Device buffers end to end, on the context's main
// stream; no host synchronisation inside the step. RCCL is loaded at run time (dlopen), so the
// library has no link-time dependency on it and shares the copy PyTorch has already loaded.
#include <dlfcn.h>

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
    std::string err;
};

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
        hipMalloc(&x->recv, sizeof(float) * per * nranks) != hipSuccess) {
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
    if (x->comm) rccl().destroy(x->comm);
    if (x->send) (void)hipFree(x->send);
    if (x->recv) (void)hipFree(x->recv);
    delete x;
}

}  // extern "C"

// declared in bshot_abi.h; defined here beside the exchange (uses the odometry's context)
int bshot_odom_exchange_ctx(bshot_ctx* c, bshot_xchg* x, int include_self) {
    if (!c || !x) return BSHOT_EINVAL;
    if (!c->gmap) return BSHOT_ESTATE;
    const size_t per = bsh::GM_REC_HDR + (size_t)bsh::GM_REC_W * x->kmax;
    // the previous exchange's inserts (queued without a sync) must have succeeded
    int rc = bsh::gmap_settle_replicas(c);
    if (rc) return rc;
    rc = bsh::gmap_pack_delta(c, x->kmax, x->send);
    if (rc) return rc;
    const int e = rccl().all_gather(x->send, x->recv, per, kNcclFloat32, x->comm, c->stream);
    if (e != 0) return c->fail(std::string("ncclAllGather: ") + (rccl().err ? rccl().err(e) : "error"), BSHOT_EHIP);
    for (int r = 0; r < x->nranks; ++r) {
        if (r == x->rank && !include_self) continue;
        rc = bsh::gmap_insert_records(c, r, x->recv + per * r, x->kmax, false);
        if (rc) return rc;
    }
    return BSHOT_OK;
}
