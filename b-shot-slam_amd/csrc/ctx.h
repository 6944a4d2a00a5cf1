// ctx.h -- bshot_ctx: one GPU, one HIP stream, grow-only device pools (sized for 288 GB HBM:
// nothing is freed between frames). Internal C++ view of the C ABI context (include/bshot_abi.h).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/bshot_abi.h"
#include "grid.h"

template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t c = n + n / 4 + 64;
        hipError_t e = hipMalloc(&p, sizeof(T) * c);
        if (e == hipSuccess) cap = c;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct StageEv {
    int stage;
    hipEvent_t a, b;
};

struct bshot_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bshot_params prm;
    std::string err;
    bool timing = false;

    // cloud
    int n = 0;
    DBuf<float> xyz;          // owned copy (host input path)
    const float* d_xyz = nullptr;
    DBuf<float4> pts4;
    bsh::DevGrid grid_fine, grid_coarse, grid_iss;  // cells seg_radius/8, seg_radius/2, iss_salient
    bool grids_ok = false;

    // per-point outputs
    DBuf<float> ratio;
    DBuf<double> third;
    DBuf<unsigned char> issflag;
    DBuf<int> errw;

    // persistent normals (include/bshot_bits.h:59): logical size + grow-only storage
    DBuf<float4> normals;
    int normals_size = 0;

    // describe
    DBuf<float> kps;
    DBuf<int> counts;
    DBuf<long long> offs;
    DBuf<unsigned long long> seg, segtmp;
    DBuf<float> rf, shot;
    DBuf<int> ok;
    DBuf<unsigned int> bits;

    // match
    DBuf<unsigned int> ma, mb;
    DBuf<unsigned long long> lbest, rbest;
    DBuf<int> left, right, mflag;

    // icp
    DBuf<float> isrc, itgt3;
    DBuf<float4> itgt;
    DBuf<unsigned long long> ibest;

    // generic gather
    DBuf<int> gidx;
    DBuf<float> gout;

    // host staging
    std::vector<float> h_ratio;
    std::vector<unsigned char> h_flag;

    // instrumentation
    std::vector<StageEv> pending;
    std::vector<hipEvent_t> evpool;
    double stage_ms[BSHOT_NSTAGES] = {0};
    int64_t stage_n[BSHOT_NSTAGES] = {0};
    int64_t work[8] = {0};

    int fail(const char* what, hipError_t e);
    int fail(const std::string& what, int code);
    void stage_begin(int st);
    void stage_end();
    void resolve_events();
    hipEvent_t get_ev();
};

namespace bsh {
// internal entry points shared by the C ABI and the odometry driver
int ctx_set_cloud_dev(bshot_ctx* c, const float* d_xyz, int n);
int ctx_seg_ratio_dev(bshot_ctx* c);                    // writes c->ratio (device), no sync
int ctx_iss_dev(bshot_ctx* c);                          // writes c->issflag (device), no sync
int ctx_describe_dev(bshot_ctx* c, int k);              // keypoints in c->kps; bits in c->bits
int ctx_match_dev(bshot_ctx* c, int na, int nb);        // descriptors in c->ma / c->mb
// H2D indices, gather xyz of pts4[idx] into dst (device, k x 3); async
int ctx_gather(bshot_ctx* c, const int* h_idx, int k, DBuf<float>& dst);
int ctx_icp(bshot_ctx* c, const float* src, int ns, const float* tgt, int nt, int max_iter, float* T, int* iters);
}  // namespace bsh
