// gmap.h -- the GPU keypoint map (csrc/gmap.hip): host handle and entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "ctx.h"

namespace bsk {
struct Xf16g {
    float m[16];
};
}  // namespace bsk

namespace bsh {

// device counters (GMap::ctr); GM_QTOT is a host-side slot of the pinned copy (query total)
enum { GM_NBLOCKS = 0, GM_NSEG = 1, GM_ITOP = 2, GM_CTOP = 3, GM_MEMBERS = 4, GM_ERR = 5, GM_QTOT = 6, GM_NCTR = 8 };
// LDS image of one block in the insert kernel: members and buckets (the bucket count for 4096
// members is 5087, umap_order.h's chain)
constexpr int GM_LDS_N = 4096;
constexpr int GM_LDS_BK = 5120;
// exchange record batch: header words, then 15 words per keypoint (x, y, z, ratio, 11 descriptor words)
constexpr int GM_REC_HDR = 16;
constexpr int GM_REC_W = 15;

struct QueryBox {
    int x0, y0, z0, ny, nz, npos;
};

struct GBlock {
    unsigned long long id;
    int n, bkt, next_resize, cap;  // members, restated libstdc++ bucket count / next_resize, capacity
    int mslot, ord, pos, code;     // pool offsets of the member arrays (ipool; code: cpool)
    int bk, bk_cap;                // ipool offset / size of the bucket array
    int pad[2];
};

struct GMap {
    bool ready = false;
    bool q_active = false;  // the last query_count launched (its total is in p_ctr[GM_QTOT])
    int slots = 0;
    int last_k = 0;  // keypoints the last gmap_insert offered (slots [slots - last_k, slots))
    DBuf<float4> kpos;
    DBuf<unsigned int> kdesc;
    DBuf<unsigned long long> tkey;
    DBuf<int> tval;
    unsigned int tsize = 0;
    DBuf<GBlock> blk;
    size_t blk_cap = 0;
    DBuf<int> ctr;
    PinBuf<int> p_ctr;
    // an insert without a sync (the exchange) leaves the counters' copy in flight: ev_ctr marks it,
    // and gmap_settle waits for it and checks the error word before the counters are read again
    hipEvent_t ev_ctr = nullptr;
    bool ctr_pending = false;
    DBuf<int> ipool;
    size_t ipool_cap = 0;
    DBuf<unsigned long long> cpool;
    size_t cpool_cap = 0;
    // per-sweep scratch
    DBuf<float> kin, refin, hrec;
    PinBuf<float> p_kin, p_refin, p_tgt, p_hrec;
    DBuf<unsigned long long> keys;
    DBuf<unsigned int> vals;
    DBuf<int> seg, qcnt;
    DBuf<unsigned char> tmp;
    ~GMap() {
        kpos.release(); kdesc.release(); tkey.release(); tval.release(); blk.release(); ctr.release(); p_ctr.release();
        ipool.release(); cpool.release(); kin.release(); refin.release(); p_kin.release(); p_refin.release(); p_tgt.release(); hrec.release(); p_hrec.release();
        keys.release(); vals.release(); seg.release(); qcnt.release(); tmp.release();
        if (ev_ctr) (void)hipEventDestroy(ev_ctr);
    }
};

// updateMap (src/lidar_odometry.cpp:344-376): the sweep's k keypoints (host, sensor frame), ratios
// (host) and descriptors (device, 11 words each) with pose T (row-major); *map_size = entries after
int gmap_insert(bshot_ctx* c, const float* kps_host, const float* ratio_host, const unsigned int* d_bits, int k,
                const float T[16], int* map_size);
// featureMatching's targets (src/lidar_odometry.cpp:195-207): map entries around pos (block loop
// order, each block in libstdc++ order, or insertion order when canonical), then the ref keypoints
// transformed by ref_pose -> c->gtgt (float3) and c->ma rows [na, na + nb)
int gmap_query(bshot_ctx* c, const float pos[3], float range, const float* ref_kps, const unsigned int* ref_bits,
               int kref, const float ref_pose[16], int na, int canonical, int* nb_out, bool ref_uploaded = false);
// featureMatching on the device targets: source words a (host) -> c->ma rows [0, na), gmap_query,
// the Hamming match (ctx_match_dev) and one sync; targets' positions -> tgt (host, nb x 3)
int gmap_match(bshot_ctx* c, const unsigned int* a, int na, const float pos[3], float range, const float* ref_kps,
               const unsigned int* ref_bits, int kref, const float ref_pose[16], int canonical, int* nb_out,
               std::vector<float>& tgt, int32_t* left_nn, std::vector<int32_t>& right_nn, int32_t* corr_q,
               int32_t* corr_m, int* n_corr);
// this sweep's map offer (the last gmap_insert's slots) as an exchange record batch at d_rec
// (GM_REC_HDR + GM_REC_W * kmax floats), on c->stream
int gmap_pack_delta(bshot_ctx* c, int kmax, float* d_rec);
// a record batch (device, count in the header) inserted into replica map `replica` on stream st
// (nullptr: the context's main stream)
int gmap_insert_records(bshot_ctx* c, int replica, const float* d_rec, int kmax, bool sync, hipStream_t st = nullptr);
// n record batches into n distinct replicas at once (the exchange's per-sweep insert): five launches
// for all of them (kmax <= 4096, n <= 8; else the per-replica path), unsynchronised, on stream st
int gmap_insert_records_multi(bshot_ctx* c, int n, const int* replicas, const float* const* d_recs, int kmax,
                              hipStream_t st);
// host records (bshot_odom_map_delta's 15-float layout) -> replica map (synchronous)
int gmap_insert_host_records(bshot_ctx* c, int replica, const float* rec, int n);
int gmap_replica_size(bshot_ctx* c, int replica);
// every replica's last unsynchronised insert has landed without error (else BSHOT_ECAP); the
// _noquiesce form is the exchange's insert thread's own (it does not wait for itself)
int gmap_settle_replicas(bshot_ctx* c);
int gmap_settle_replicas_noquiesce(bshot_ctx* c);
// replica's entries around pos (block loop order; libstdc++ or canonical order) -> host; count or -needed
int gmap_replica_query(bshot_ctx* c, int replica, const float pos[3], float range, int canonical, float* xyz,
                       unsigned int* bits, int cap);
// the last gmap_match's target descriptors (rows [na, na + nb) of c->ma) -> host
int gmap_target_descriptors(bshot_ctx* c, int na, int nb, unsigned int* out);
void gmap_free(bshot_ctx* c);

}  // namespace bsh
