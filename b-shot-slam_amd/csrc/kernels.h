// kernels.h -- host-side launchers of the gfx950 kernels (all asynchronous on stream s).
#pragma once
#include <hip/hip_runtime.h>

#include "grid.h"

namespace bsh {

// copies / fills as kernels on stream s (csrc/kcopy.hip): device memory and the pinned staging
// buffers only (never pageable host memory). The sweep loop issues no copy-engine transfer.
// max_blocks: grid cap (a bulk copy that reads host memory holds its CUs for the transfer's
// duration; a small grid leaves the rest to the concurrent kernels)
hipError_t kcopy(void* dst, const void* src, size_t bytes, hipStream_t s, int max_blocks = 0);
// n copies in one launch where possible (up to 4 per launch; an empty or self copy is skipped)
hipError_t kcopy_n(int n, void* const* dst, const void* const* src, const size_t* bytes, hipStream_t s);
hipError_t kcopy2(void* d0, const void* s0, size_t b0, void* d1, const void* s1, size_t b1, hipStream_t s);
hipError_t kfill(void* dst, unsigned char value, size_t bytes, hipStream_t s);

// g4: the radius-ladder grids (cells r/16, r/8, r/4, r/2 for ladder modes 1, 2; r/8, r/8, r/2, r/2
// for mode 0), see ladder() in knn.hip
// largest max_nn the kNN engine's finishing arrays hold (csrc/knn.hip FL_STRIDE)
int knn_max_nn();
hipError_t launch_seg_ratio(const DevGrid* const* g4, int ladder_mode, const float4* pts4, int n, float radius,
                            int max_nn, int sr_type, int hint, float* ratio, int* err, hipStream_t s,
                            unsigned long long* kst = nullptr, int max_blocks = 8192, int xcd_chunk = 0, int run = 1,
                            float bratio = 2.83f);
hipError_t launch_normals(const DevGrid* const* g4, int ladder_mode, const float4* pts4, const float* kps, int k,
                          float radius, int max_nn, float4* normals, int* err, hipStream_t s);
hipError_t launch_iss(const DevGrid& g, const float4* pts4, int n, float salient, float nonmax, int min_nn, double g21,
                      double g32, double* third, unsigned char* flag, int* ovf, unsigned int* nml, int* nmc,
                      int* err, hipStream_t s, int ovf_blocks = 0, int nms_blocks = 0, bool ovf_zeroed = false,
                      int xcd_chunk = 0);
// bh (nullable, [k][1024] u32): per-keypoint d2-bucket histogram for the bucketed gather
hipError_t launch_shot_count(const DevGrid& g, const float* kps, int k, float R, int* counts, long long* offs,
                             hipStream_t s, unsigned int* bh = nullptr);
// bucket-grouped gather (bstart: per-keypoint bucket starts) and the in-bucket rank that sorts it
hipError_t launch_shot_gather_b(const DevGrid& g, const float* kps, int k, float R, const long long* offs,
                                const unsigned int* bh, unsigned int* bstart, unsigned int* seg, hipStream_t s,
                                const int* err = nullptr);
// count + device-side plan (offs, chunk bases cb, LPT perm) against preallocated capacities;
// err |= 16 (and empty ranges) when they do not suffice. k <= 8192. The count kernel also zeroes
// err[0..3] (zero_err) and z4[0, nz), and copies cs4[0, cm) to cd4 (the fills and the normals
// snapshot the caller would otherwise launch)
hipError_t launch_shot_count_plan(const DevGrid& g, const float* kps, int k, float R, int* counts, unsigned int* bh,
                                  long long seg_cap, int chunk_cap, long long* offs, int* cb, int* perm, int* err,
                                  hipStream_t s, bool zero_err = false, float4* z4 = nullptr, int nz = 0,
                                  float4* cd4 = nullptr, const float4* cs4 = nullptr, int cm = 0);
// seg: the gather's bucket-grouped neighbour indices; out: every segment in (d2, idx) order (4 B
// each; the rank kernels and the consumers recompute d2 from the points with the gather's
// expression, bit-identical)
// a workgroup per keypoint in perm's order (spans of whole buckets staged in LDS)
hipError_t launch_shot_rank_wg(int k, float R, const float4* pts4, const float* kps, const int* perm,
                               const long long* offs, const unsigned int* bstart, const unsigned int* seg,
                               unsigned int* out, hipStream_t s, int rank_max = -1);
// a wave per 64-rank chunk
hipError_t launch_shot_rank(int k, int n_chunks, float R, const float4* pts4, const float* kps, const long long* offs,
                            const int* cb, const int* owner, const unsigned int* bstart, const unsigned int* seg,
                            unsigned int* out, hipStream_t s, const int4* cinfo = nullptr, int max_blocks = 0);
hipError_t launch_match(const unsigned int* a, int na, const unsigned int* b, int nb, unsigned long long* best,
                        int* out, hipStream_t s);
hipError_t launch_pack_points(const float* xyz, int n, float4* out, hipStream_t s);
hipError_t launch_gather(const float4* pts4, const int* idx, int k, float* out, hipStream_t s);
// gather with the indices in pinned host memory (read by the kernel) and an optional pinned copy of
// the coordinates (hout)
hipError_t launch_gather_io(const float4* pts4, const int* h_idx, int k, float* out, float* hout, hipStream_t s);
// A11 ICP nearest neighbours on the targets' nested grids g4 (cells 1000, 2000, 4000, 8000 mm, all
// hashed) and float4 targets tgt4 (index order). Iteration 0: the exact 1-NN keys of src0 into
// best_out, and per source a candidate list (cap float4 entries: target xyz + index bits, and their
// distances from the list's centre, in ascending order; entry e of source i at [e * ns + i]), its
// count (-1: none) and radius. Iteration >= 1: the sources moved by T16 (src_in -> src_out) and
// their exact 1-NN keys; keys (d2 bits << 32 | index) land in best_out (pinned host memory).
// 256: fewer sources leave their lists for the LDS grid search, which runs slowly beside the
// SHOT histogram's LDS atomics (128 -> 256: +4.4 % sweeps/s, 512: +3.2 %; profiles/r05w_*)
#ifndef ICP_LIST_CAP
#define ICP_LIST_CAP 256
#endif
// the result of one ICP call (coherent pinned host memory): the composed transform, the iteration
// count, then seq (written last, after the others have reached host memory)
struct IcpOut {
    float T[16];
    int iters;
    int seq;
    int pad[14];
};
// the host's ICP loop (the default): host <-> device hand-over in coherent pinned memory -- the host
// releases iteration j (step transform T, then go = j; go = -1 stops the kernel); every workgroup
// writes its own completion flag once its keys are stored
struct IcpSync {
    int go;
    int pad0[31];
    float T[16];
};
// the release relayed in device memory (option icp_relay): workgroup 0 polls IcpSync in pinned host
// memory and republishes each release here; the other workgroups poll this word (device scope)
// instead of host memory. word = call sequence << 32 | (go + 1), low half 0xFFFFFFFF = stop.
struct IcpDevSync {
    unsigned long long word;
    int pad0[30];
    float T[16];
};
int icp_lists_blocks(int ns);
int icp_iter_blocks(int ns);
// iteration 0 (a wave per source): keys of src0 into best_out (pinned), the candidate lists (lcen:
// centre + radius); workgroup w sets done[w] = 1
hipError_t launch_icp_lists_host(const float* src0, int ns, const DevGrid* const* g4, const float4* tgt4, int nt, int cap,
                                 float4* lst, float* lsd, int* lcnt, float4* lcen, unsigned long long* best_out,
                                 int* done, hipStream_t s);
// iterations j0 .. max_iter - 1 (one persistent launch, a lane per source starting at src0): each
// waits for the host's release of the iteration (or go = -1), moves its source by T, stores the exact
// 1-NN key in best[(j & 1) * ns + i] (pinned) and sets done[w] = j
hipError_t launch_icp_iterations(const float* src0, int ns, int j0, const float4* lst, const float* lsd, const int* lcnt,
                                 const float4* lcen, int cap, const DevGrid* const* g4, const float4* tgt4, int nt,
                                 int max_iter, const IcpSync* sy, int* done, unsigned long long* best, hipStream_t s,
                                 int* qstat = nullptr, IcpDevSync* dsy = nullptr, unsigned int seq = 0);
// the loop state of one ICP call (device memory): the last step, the composed transform, PCL's
// previous MSE, the iteration count and the stop flag every queued kernel checks first
struct IcpCtl {
    float T[16];
    float fin[16];
    double prev_mse;
    int it;
    int stop;
};
// PCL's ICP loop on the device (option icp_device, csrc/icp.hip): k_icp_lists (iteration 0: exact 1-NN, candidate lists,
// records), then one persistent k_icp_run (per iteration: step + NN of every source on its
// workgroup, the Umeyama step + convergence test on the last workgroup to arrive), queued on s; the
// stopping step writes the composed transform and the count to *out, seq last. Scratch (HBM): lst /
// lsd (cap x ns), lcnt (ns), pos / lcen (ns float4), rec (7 x ns floats), ctl, sync (2 u32).
hipError_t launch_icp(const float* src0, int ns, float4* lst, float* lsd, int* lcnt, int cap, const DevGrid* const* g4,
                      const float4* tgt4, int nt, int max_iter, float4* pos, float4* lcen, float* rec, IcpCtl* ctl,
                      unsigned int* sync, IcpOut* out, int seq, hipStream_t s);
// load-balanced SHOT (describe2.hip): in-bucket rank, LRF over 64-rank chunks, records + ordered apply
struct Describe2Args {
    int k = 0, n_plan = 0, n_chunks = 0;
    float R = 0.f;
    const int* cb = nullptr;               // k + 1 chunk offsets
    int* owner = nullptr;                  // keypoint of every chunk
    int4* cinfo = nullptr;                 // per chunk {keypoint, chunk index, length, offset} (offsets < 2^31), or null
    const int* perm = nullptr;             // keypoints by descending neighbourhood size
    const long long* offs = nullptr;       // k + 1 segment offsets
    const float4* pts4 = nullptr;
    const float4* normals = nullptr;
    const float* kps = nullptr;
    const unsigned int* seg = nullptr;        // bucket-grouped neighbour indices (gather)
    unsigned int* sorted = nullptr;           // neighbour indices in (d2, idx) order (output of k_shot_rank)
    double* csum = nullptr;                   // 8 per chunk
    double* eig = nullptr;                    // 8 per keypoint
    int* okf = nullptr;                       // eigen ok per keypoint
    int nseg_max_nn = 0;                      // > 0: k_lrf_eig also writes the keypoint normals from the sorted
    float4* normals_out = nullptr;            //   segments' heads (normal_max_nn; normal_radius == shot_radius)
    float* rf = nullptr;
    int* ok = nullptr;
    float* shot = nullptr;
    unsigned int* bits = nullptr;
    int* err = nullptr;
    const unsigned int* bstart = nullptr;  // per-keypoint bucket starts of the bucket-grouped segment
    int max_blocks = 0;  // grid cap of the chunk kernels (0: one block per 4 chunks)
    int rank_wg = 0;     // 1: k_shot_rank_wg (workgroup per keypoint, large neighbourhoods); 0: k_shot_rank
    int rank_max = -1;   // k_shot_rank_wg: spans whose buckets all hold <= this many keys rank in place (-1: default)
    int hf_pack = 1;     // 1: the SHOT apply packs several ranks per ds_add_f32 (needs lds_lane_order_check() == 0)
    int slices = 1;      // the workgroup-per-keypoint kernels (histogram, rank_wg) in this many launches over perm
};
hipError_t launch_describe2(const Describe2Args& a, int part, hipStream_t s);
// mismatches of same-address ds_add_f32 lanes against ascending lane order on the current device
// (0 expected; *sensitive = bins where the order mattered), -1 on a HIP error
int lds_lane_order_check(int* sensitive);

// A10 RANSAC: score (inlier count) of every hypothesis (csrc/ransac.hip)
hipError_t launch_ransac_score(const float* cs, const float* ct, int nidx, const int* hyp, int nhyp, double thr2,
                               int* cnt, hipStream_t s);

}  // namespace bsh
