// ctx.h -- bshot_ctx: one GPU, one HIP stream, grow-only device pools (sized for 288 GB HBM:
// nothing is freed between frames). Internal C++ view of the C ABI context (include/bshot_abi.h).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bshot_abi.h"
#include "grid.h"
#include "regrow.h"
#include "kernels.h"

template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        defer_free(p, DEFER_DEVICE);
        p = nullptr;
        cap = 0;
        // doubling with a 64 Ki-element floor: a sequence's sizes (targets M, neighbourhood totals)
        // grow for many sweeps, and every regrowth is a free + malloc that stalls the device
        size_t c = n * 2 > (size_t)65536 ? n * 2 : (size_t)65536;
        hipError_t e = hipMalloc(&p, sizeof(T) * c);
        if (e == hipSuccess) cap = c;
        note_regrow("device", sizeof(T) * c);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// pinned host staging (async D2H), grow-only; coherent: fine-grained memory, for hand-over with a
// running kernel (system-scope atomics, csrc/icp.hip)
template <typename T>
struct PinBuf {
    T* p = nullptr;
    size_t cap = 0;
    bool coherent = false;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        defer_free(p, DEFER_PINNED);
        p = nullptr;
        cap = 0;
        // doubling with a 64 Ki-element floor: a sequence's sizes (targets M, neighbourhood totals)
        // grow for many sweeps, and every regrowth is a free + malloc that stalls the device
        size_t c = n * 2 > (size_t)65536 ? n * 2 : (size_t)65536;
        hipError_t e = hipHostMalloc((void**)&p, sizeof(T) * c, coherent ? hipHostMallocCoherent : hipHostMallocDefault);
        if (e == hipSuccess) cap = c;
        note_regrow("pinned", sizeof(T) * c);
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct StageEv {
    int stage;
    hipEvent_t a, b;
    int id;
    bool ended;
};

// Everything that belongs to one input cloud: float4 copy, radius-ladder and ISS grids, SR ratios,
// ISS results, and their pinned host copies. The context holds the current cloud and a prefetch
// slot; adopting a prefetched cloud swaps the two (pointer swaps, no copies).
struct CloudState {
    const float* d_xyz = nullptr;
    int n = 0;
    DBuf<float> xyz;  // owned copy (host input path)
    DBuf<float4> pts4;
    // radius-ladder grids (cells seg_radius/16, /8, /4, /2) and the ISS grid (cell iss_salient)
    bsh::DevGrid grid_l16, grid_fine, grid_l4, grid_coarse, grid_iss;
    const bsh::DevGrid* ladder[4] = {nullptr, nullptr, nullptr, nullptr};
    bool grids_ok = false;
    bool prefetched = false;  // loaded (and SR/ISS launched) ahead of use on the side stream
    bool iss_pending = false; // queued with option iss_defer: its ISS launches at ctx_queue_iss
    int sr_state = 0;         // 0 not launched, 1 launched (results land in h_ratio at ev_sr)
    int iss_state = 0;        // 0 not launched, 1 launched (results land in h_flag at ev_iss)
    int zeroed = 0;           // bit 0: errw[0] zeroed by the grid build, bit 1: errw[1] and issovf[0]
    DBuf<float> ratio;
    DBuf<double> third;
    DBuf<unsigned char> issflag;
    DBuf<int> issovf;  // ISS overflow list: [0] = count, [1..] = point indices
    DBuf<unsigned int> issnml;  // ISS non-max neighbour lists, [32][n]
    DBuf<int> issnmc;           // their lengths (-1: overflow point)
    DBuf<int> errw;    // [0] SR error bits, [1] ISS error bits
    PinBuf<float> h_ratio;
    PinBuf<unsigned char> h_flag;
    PinBuf<int> h_err;  // [0] SR, [1] ISS
    hipEvent_t ev_loaded = nullptr, ev_sr = nullptr, ev_iss = nullptr;
    bool fine_ladder = false;  // 4 grids + 7-step sqrt(2) radius ladder (opt_ladder4)
    bool iss_lvl = false;      // grid_iss is the ladder's fifth level (cells r/32, the ladder's points)
    void fix_ladder(bool four) {
        fine_ladder = four;
        ladder[0] = four ? &grid_l16 : &grid_fine;
        ladder[1] = &grid_fine;
        ladder[2] = four ? &grid_l4 : &grid_coarse;
        ladder[3] = &grid_coarse;
    }
    void release();
};

// the SR error word of a cloud (CloudState::errw[0]): 1 = a kNN list overflow (k_seg_ratio), 8 = a
// finite point beyond the ladder key range (k_ladder_cells4)
inline const char* sr_error_message(int bits) {
    if (bits & 8) return "seg_ratio: a point lies beyond the grid's coordinate range (|x|, |y|, |z| >= 2^20 finest cells of seg_radius / 32)";
    return "seg_ratio: neighbourhood with too many exactly tied boundary keys (kNN list overflow)";
}

namespace bsh {
struct GMap;       // csrc/gmap.hip
struct PreState;   // csrc/preprocess.hip
struct VeloState;  // csrc/velodyne.hip
}

struct bshot_ctx {
    int device = 0;
    hipStream_t stream = nullptr;  // main: describe, match, ICP, and everything synchronous
    hipStream_t side = nullptr;    // side: prefetched clouds (grids, SR) and the lookahead describe
    hipStream_t iss = nullptr;     // ISS (needed only at the end of a sweep), low priority
    hipStream_t pre = nullptr;     // grids + SR of the sweep after next (queue slot pf2), low priority
    bshot_params prm;
    std::string err;
    bool timing = false;
    unsigned timing_mask = ~0u;  // stages timed while timing is on (bit = BSHOT_STAGE_*)

    CloudState cs;  // current cloud
    CloudState pf;  // prefetch slot (next sweep: the lookahead worker describes it)
    CloudState pf2; // queue slot (the sweep after next: grids + SR + ISS only)

    // tuning knobs (bshot_set_option): results never depend on them
    int opt_ladder4 = 1;  // 1: 4 nested grids + 7-step sqrt(2) radius ladder (default); 0: 2 grids, 4 steps
    int opt_ladder_front = 1;   // two radius steps r/16, r/(8 sqrt 2) in front of the fine ladder
    int opt_sr_xcd_chunk = 1024;  // SR queries per XCD-local chunk of cell order (0: round-robin queries)
    int opt_sr_blocks = 0;      // SR grid cap (0: one run of queries per wave -- short waves let the main stream in)
    int opt_gmap_slots0 = 1 << 20;  // GPU map: keypoint slots reserved up front (grown by doubling past them)
    int opt_iss_xcd_chunk = 1024;  // ISS lane kernel: points per XCD-local chunk of cell order (0: blocks in order)
    int opt_sr_run = 4;         // SR cell-order queries per wave pass, each after the first bounded by its predecessor
    int opt_sr_bratio = 200;    // SR bounded pass: grid cell >= radius * 100 / this (percent)
    int opt_side_prio = 0;      // describe (side) stream priority: 0 low (as SR/ISS ahead), 1 middle, 2 the main stream's
    int opt_map_sync = 1;       // GPU map insert: wait for it and report the map size per sweep (0: stream-ordered, size -1)
    int opt_host_map_log = 1;   // LidarOdometry keeps the GPU map's insert log for the host Map view (bshot_odom: 0)
    int opt_normals_seg = 1;    // normals from the SHOT neighbour lists when normal_radius == shot_radius
    int opt_diag_skip_icp = 0;  // diagnostic only: ICP returns the identity without running (never in a bench line)
    int opt_hist_pack = 1;      // SHOT apply: 1 several ranks per ds_add_f32 when the device passed the lane-order check
    int hf_pack_ok = 0;         // that check's result for this context's device (bshot_create)
    int opt_rank_max = -1;      // k_shot_rank_wg's in-place threshold (-1: RK_RANKMAX; 0: every span sorted)
    int opt_rank_wg = 2;        // SHOT rank kernel: 0 wave per 64-rank chunk, 1 workgroup per keypoint, 2 by neighbourhood size
    int opt_desc_slices = 1;    // the histogram / rank_wg kernels in this many launches (LPT slices)
    int opt_iss_defer = 0;      // 1: the queued sweep's ISS launches after the current sweep's ICP
    int opt_sr_start = 80;      // SR ladder start predicted from own-cell densities (percent scale; 0: step 0)
    int opt_iss_grid = 1;       // ISS on the SR ladder's points: its fifth level, cells r/32 (0: own grid)
    int opt_iss_cell = 2;       // ISS grid cell = opt_iss_cell x salient radius (2: <= 8 cells per query)

    DBuf<int> errw;  // describe-stage error bits (normals)

    // persistent normals (include/bshot_bits.h:59): logical size + grow-only storage
    DBuf<float4> normals;
    int normals_size = 0;
    // the state a lookahead describe started from (ctx_normals_snapshot), put back if its result
    // is dropped instead of adopted (ctx_normals_restore): slots [0, snap_n) and the logical size
    DBuf<float4> normals_snap;
    int normals_snap_size = -1;  // -1: no snapshot held
    int normals_snap_n = 0;
    int normals_snap_defer = 0;  // snapshot slots the next describe copies (ctx_normals_snapshot defer)

    // describe
    DBuf<float> kps;
    DBuf<int> counts;
    DBuf<long long> offs;
    DBuf<unsigned int> seg;        // neighbour indices, bucket-grouped by d2 (gather)
    DBuf<unsigned int> segtmp;     // neighbour indices in (d2, idx) order (rank)
    DBuf<float> rf, shot;
    DBuf<int> ok;
    DBuf<unsigned int> bits;
    // load-balanced SHOT (describe2.hip)
    DBuf<int4> plan;
    DBuf<int> cb, owner, okf, perm;
    DBuf<int4> cinfo;  // per-chunk records for the chunk kernels (k_chunk_owner)
    DBuf<double> csum, eig;
    PinBuf<long long> p_offs;
    PinBuf<int> p_plan;  // plan (4 ints per item) then cb (k + 1)
    bsh::PreState* prep = nullptr;  // GPU preprocessor state (csrc/preprocess.hip), created on first use
    bsh::VeloState* velo = nullptr;  // GPU packet decode state (csrc/velodyne.hip), created on first use
    DBuf<unsigned int> sbh, sbst;  // bucketed gather: per-keypoint d2 histogram and bucket starts
    // lookahead keypoint gather (ctx_gather_kps_async): own index and staging buffers
    PinBuf<int> p_kidx;
    PinBuf<float> p_kps3;
    int opt_chunk_blocks = 0;  // grid cap of the 64-rank chunk kernels (0: one block per 4 chunks)
    bool plan_on_host = false;  // next describe: plan on the host (after a device-plan overflow)
    long long seg_hint = 0;     // largest neighbourhood total seen (device-plan capacities)
    int ladder_mode(const CloudState& s) const { return s.fine_ladder ? (opt_ladder_front ? 2 : 1) : 0; }

    // GPU keypoint map (csrc/gmap.hip): mode 0 host Map, 1 GPU map in the reference's libstdc++
    // block order (default), 2 GPU map in insertion order (canonical; not the reference's order)
    int opt_gpu_map = 1;
    bsh::GMap* gmap = nullptr;
    std::vector<bsh::GMap*> gmap_replicas;  // other sequences' maps (multi-GPU exchange, bshot_odom_exchange)
    // the exchange (host/xchg.cpp) queues its replica inserts on the iss stream, or logs the offers
    // for later (option xchg_index 0): every host access to the replicas first lets it index what it
    // has logged (detach = 1 at the context's teardown: the exchange forgets it)
    int (*replica_quiesce)(void* arg, int detach) = nullptr;
    void* replica_quiesce_arg = nullptr;
    // before any access to the replicas: the exchange indexes the offers it has logged (its error code)
    int quiesce_replicas(int detach = 0) {
        const int rc = replica_quiesce ? replica_quiesce(replica_quiesce_arg, detach) : 0;
        if (detach) replica_quiesce = nullptr;
        return rc;
    }
    int opt_xseq_targets = 0;  // 1: the replicas' entries join the matching targets (extension; 0 = reference)
    int opt_xchg_index = 1;    // replica policy: 1 index every exchange at once (iss stream), 0 log and index on read
    DBuf<float> gtgt;  // matching targets assembled on the device (float3)

    // match: ma = a rows then b rows; lbest = left keys then right keys; left = left | right | flag
    DBuf<unsigned int> ma;
    DBuf<unsigned long long> lbest;
    DBuf<int> left;

    // host timeline (diagnostics): BSHOT_HOST_TRACE=<file> records named steady-clock stamps of
    // both host threads, written as CSV when the context is destroyed
    bool htrace_on = false;
    std::mutex htmu;
    std::vector<std::pair<const char*, long long>> htrace;
    void hmark(const char* name);

    // icp
    PinBuf<bsh::IcpSync> p_isync;        // ICP host loop: host <-> kernel hand-over (coherent)
    PinBuf<unsigned long long> p_ibest;  // ICP host loop: NN keys, two iterations' worth (coherent)
    PinBuf<int> p_idone;                 // ICP host loop: per-workgroup completion flags (coherent)
    PinBuf<float> p_src2;                // ICP host loop: the current positions after a restart
    int opt_icp_device = 0;        // 1: PCL's ICP loop entirely on the device (k_icp_run); 0: the host's float Umeyama
    int opt_icp_host_delay_ms = 0;  // tests: the host loop sleeps this long before releasing iteration 3
    PinBuf<bsh::IcpOut> p_iout;  // ICP result: composed transform, iteration count, seq (coherent)
    int icp_seq = 0;             // seq of the last ICP call
    bsh::IcpDevSync* idsy = nullptr;  // ICP host loop: the release relayed in device memory (option icp_relay)
    unsigned int icp_relay_seq = 0;  // per persistent-kernel launch (a stale word never matches)
    int opt_icp_relay = 1;       // 1: workgroup 0 alone polls the host's release and relays it
    DBuf<float4> ipos, ilcen;    // ICP loop: current source positions, list centres (xyz) + radii (w)
    DBuf<float> irec;            // ICP loop: the iteration's Umeyama records (7 x ns floats)
    DBuf<bsh::IcpCtl> ictl;      // ICP loop state
    DBuf<unsigned int> isync;    // ICP loop: arrival counter, released iteration
    DBuf<float4> ilst;  // ICP candidate lists (ICP_LIST_CAP per source)
    DBuf<float> ilsd;   // their entries' distances from the list centre (ascending)
    DBuf<int> ilcnt;    // their counts (-1: none)
    int opt_ransac_dev = 1;  // 1: RANSAC hypotheses scored on the GPU (bshot_ransac_dev); 0: on the host
    int opt_topk_thread = 1;   // LidarOdometry: top-K of a queued sweep on its own host thread once its SR lands
    int opt_pre_fast = 1;  // preprocessor: one 32-bit sort for azimuth-ordered lasers with tabled verticals
    int opt_iss_ovf_blocks = 512;  // grid of the ISS overflow kernel (grid-strides over the device-side count)
    int opt_iss_nms_blocks = 1024;  // grid of the ISS overflow non-max kernel (grid-strides likewise)
    bsh::DevGrid icp_lad[4];  // ICP target grids: nested cells 1000 .. 8000 mm, one sort per ICP call
    DBuf<int> icp_err;     // the ICP target grids' error word (8: a finite target beyond the key range)
    PinBuf<int> p_icp_err;  // its copy, read after the ICP call (coherent)
    DBuf<float> itgt3;
    const float* icp_prep_tgt = nullptr;  // device targets whose ICP grids ctx_icp_prepare has queued
    int icp_prep_nt = 0;
    DBuf<float4> itgt;
    DBuf<unsigned long long> ibest;  // ICP iteration 0's NN keys

    // RANSAC scoring (bshot_ransac_dev): correspondence points, hypotheses, scores
    DBuf<float> rpts;
    DBuf<int> rhyp, rcnt;
    PinBuf<float> p_rpts;
    PinBuf<int> p_rhyp, p_rcnt;

    // generic gather
    DBuf<float> gout;

    // pinned staging of per-frame host<->device transfers (pageable copies stall behind other
    // streams' work)
    PinBuf<uint32_t> p_a, p_bits;
    PinBuf<int> p_left, p_gidx, p_err;
    PinBuf<float> p_g3, p_src, p_tgt, p_xyz;
    PinBuf<float> p_nrm;  // persistent-normals slots read / written by the frame-sharded mode
    hipEvent_t ev_xyz = nullptr;  // the staged host cloud (p_xyz) has been copied
    PinBuf<unsigned long long> p_best;
    PinBuf<long long> p_i64;

    // instrumentation
    std::mutex evmu;  // guards pending / evpool / stage_seq (the lookahead task records from its thread)
    int stage_seq = 0;
    std::vector<StageEv> pending;
    std::vector<hipEvent_t> evpool;
    double stage_ms[BSHOT_NSTAGES] = {0};
    int64_t stage_n[BSHOT_NSTAGES] = {0};
    int64_t work[12] = {0};
    DBuf<int> iqstat;  // ICP host loop: cumulative grid searches after iteration 0, and the most one wave took in an iteration

    int fail(const char* what, hipError_t e);
    int fail(const std::string& what, int code);
    // stage timing: begin returns a token for the matching end (thread-safe; -1 when timing is off)
    int stage_begin(int st, hipStream_t s = nullptr);
    void stage_end(int token, hipStream_t s = nullptr);
    void resolve_events(bool wait = false);
    hipEvent_t get_ev();
};

namespace bsh {
// internal entry points shared by the C ABI and the odometry driver
// A2 from a sweep's SR ratio array (NaN = skipped): the std::sort tail of the valid (index, ratio)
// pairs (host/topk.cpp)
int topk_from_ratios(const float* ratio, int n, int k, int32_t* kp_idx, float* kp_ratio, int* k_out, int* nv_out);
int ctx_make_side_stream(bshot_ctx* c);
int ctx_set_cloud_dev(bshot_ctx* c, const float* d_xyz, int n);  // adopts a matching prefetch
int ctx_prefetch_dev(bshot_ctx* c, const float* d_xyz, int n);   // grids + SR + ISS on the side stream
int ctx_sr_launch(bshot_ctx* c);   // SR of the current cloud (main stream) unless already launched
int ctx_iss_launch(bshot_ctx* c);  // ISS of the current cloud (side stream) unless already launched
int ctx_describe_dev(bshot_ctx* c, int k);              // keypoints in c->kps; bits in c->bits
int ctx_match_dev(bshot_ctx* c, int na, int nb);        // descriptors in c->ma / c->mb
// H2D indices, gather xyz of pts4[idx] into dst (device, k x 3); async
int ctx_gather(bshot_ctx* c, const int* h_idx, int k, DBuf<float>& dst);
int ctx_sync_main(bshot_ctx* c);
// explicit-cloud / explicit-stream variants (the lookahead task runs them on the side stream)
int ctx_queue_dev(bshot_ctx* c, const float* d_xyz, int n);
int ctx_queue_begin(bshot_ctx* c, const float* d_xyz, int n);
int ctx_queue_rest(bshot_ctx* c, const float* d_xyz, int n);
// the queued sweep's ISS when option iss_defer held it back (main thread, after ICP); no-op otherwise
int ctx_queue_iss(bshot_ctx* c);
int ctx_describe_on(bshot_ctx* c, CloudState& S, hipStream_t st, int k);
// persistent-normals state around a lookahead describe of k keypoints on stream st: a describe
// writes slots [0, k) and zero-fills past the logical size, so slots [0, min(k, size)) and the size
// are all it can change. snapshot: queued on st before the describe; restore: after the describe
// finished (the worker synchronised st), when its result is dropped; discard: when it is adopted.
// defer: the copy is left to the next ctx_describe_on on st (its count kernel carries it, or it
// queues the copy first), which must follow before anything else touches the normals.
int ctx_normals_snapshot(bshot_ctx* c, hipStream_t st, int k, bool defer = false);
int ctx_normals_restore(bshot_ctx* c);
void ctx_normals_discard(bshot_ctx* c);
// frame-sharded mode: slots [0, m) of the persistent normals array to the host (m <= its logical
// size; synchronous on the main stream), and a whole state put in place: logical size `size`, slots
// [0, m) from the host, [m, size) zero (synchronous)
int ctx_normals_read(bshot_ctx* c, int m, float* out);
int ctx_normals_write(bshot_ctx* c, int size, int m, const float* slots);
// after a describe's error word reached the host (err[0..3] as copied from c->errw): true when the
// describe must be run again -- errw bit 16, a device plan over capacity (the re-run plans on the
// host; the capacity hint grows to the total the device counted)
bool ctx_describe_replan(bshot_ctx* c, const int* err);
int ctx_gather_on(bshot_ctx* c, CloudState& S, hipStream_t st, const int* h_idx, int k, DBuf<float>& dst);
int ctx_gather_host_on(bshot_ctx* c, CloudState& S, hipStream_t st, const int* h_idx, int k, DBuf<float>& dst,
                       float* out);
// device gather of cloud points -> host (pinned staging), synchronous
int ctx_gather_host(bshot_ctx* c, const int* h_idx, int k, DBuf<float>& dst, float* out);
int ctx_gather_kps_async(bshot_ctx* c, CloudState& S, hipStream_t st, const int* h_idx, int k);
// d_tgt (nullable): the same targets already on the device (gmap), copied D2D instead of uploaded
int ctx_icp(bshot_ctx* c, const float* src, int ns, const float* tgt, int nt, int max_iter, float* T, int* iters,
            const float* d_tgt = nullptr);
// queue the grids of the ICP targets d_tgt (nt, device) now; the next ctx_icp with them skips the build
int ctx_icp_prepare(bshot_ctx* c, const float* d_tgt, int nt);
}  // namespace bsh
