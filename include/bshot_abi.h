/* bshot_abi.h -- C ABI of the MI355X-native B-SHOT hot path (libbshot_amd.so).
 *
 * The reference (TingKaiChen/B-SHOT-SLAM) has no plugin/FFI layer: its boundary is the C++ class
 * API (include/lidar_odometry.h:13-73, include/frame.h:10-51, include/keypoint.h:8-32,
 * include/mymap.h:9-51, include/bshot_bits.h:6-281). This C ABI sits UNDER the C++ API in
 * include/bshot/ (which keeps those class names) and is what ctypes/cgo/JNI would bind
 * (INTEGRATION.md). Conventions: 0 = OK, negative = error (message via bshot_last_error); no C++
 * exception crosses the ABI; host buffers are caller-owned and only read/written during the call;
 * device memory is context-owned; one context per host thread and GPU; no global mutable state.
 * Points are float32 millimetres, AoS xyz. 4x4 matrices are row-major float[16].
 * Descriptors (B-SHOT) are 11 x uint32 per keypoint: bit j of the reference's std::bitset<352> is
 * bit (j % 32) of word j / 32 (include/bshot_bits.h:25, :264-275).
 */
#ifndef BSHOT_ABI_H
#define BSHOT_ABI_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define BSHOT_WORDS 11
#define BSHOT_OK 0
#define BSHOT_EINVAL (-1)
#define BSHOT_EHIP (-2)
#define BSHOT_ECAP (-3)
#define BSHOT_ESTATE (-4)
#define BSHOT_ESTALE (-5) /* frame-sharded record described over other normals than the sequence's */

typedef struct bshot_ctx bshot_ctx;

/* Defaults = the reference's hard-coded constants (cited per field). */
typedef struct {
    float seg_radius;     /* 3000  src/lidar_odometry.cpp:68 (SR radius, mm) */
    int seg_max_nn;       /* 300   src/lidar_odometry.cpp:70 (at most 484: the kNN engine's LDS rows) */
    int sr_type;          /* 0 CV, 1 CVS, 2 CVSN: include/lidar_odometry.h:47 setSRType */
    int num_keypoints;    /* 600   src/lidar_odometry.cpp:138 (BASELINE config 2: 2048) */
    float iss_salient;    /* 60    src/lidar_odometry.cpp:452 */
    float iss_nonmax;     /* 40    src/lidar_odometry.cpp:453 */
    double iss_gamma21;   /* 0.975 src/lidar_odometry.cpp:454 */
    double iss_gamma32;   /* 0.975 src/lidar_odometry.cpp:455 */
    int iss_min_nn;       /* 5     src/lidar_odometry.cpp:456 */
    float normal_radius;  /* 3000  src/lidar_odometry.cpp:174 */
    int normal_max_nn;    /* 300   include/bshot_bits.h:66 (at most 512 when normal_radius == shot_radius,
                             else 484) */
    float shot_radius;    /* 3000  src/lidar_odometry.cpp:175 */
    float map_range;      /* 100000 src/lidar_odometry.cpp:198 */
    int ransac_max_iter;  /* 2000  src/lidar_odometry.cpp:254 */
    double ransac_thresh; /* 1500  src/lidar_odometry.cpp:256 */
    int icp_max_iter;     /* 10    (PCL IterativeClosestPoint default, :293-297) */
    int run_icp;          /* 1     test/odometry_test.cpp:41, include/lidar_odometry.h:50 */
    int run_iss;          /* 1     ISS runs every frame (src/lidar_odometry.cpp:164-170) */
    int run_kp_eval;      /* 0     kpEvaluation per frame: kp_test yes (test/kp_test.cpp:166), odometry_test no */
} bshot_params;

void bshot_default_params(bshot_params* p);

/* ---- context ------------------------------------------------------------------------------ */
int bshot_create(bshot_ctx** out, int device, const bshot_params* p);
void bshot_destroy(bshot_ctx* c);
const char* bshot_last_error(const bshot_ctx* c);
int bshot_sync(bshot_ctx* c);
/* hipStream_t the context launches on (as void*), for callers that time or chain work. */
void* bshot_stream(bshot_ctx* c);

/* ---- A0: cloud (replaces LidarOdometry::setSrcFrame, src/lidar_odometry.cpp:29-41). Points are
 *      indexed on grids whose finest cell is seg_radius / 32: a finite point farther than 2^20 such
 *      cells from the origin on any axis (+-98 km at the default 3000 mm) fails the sweep's SR with
 *      BSHOT_ECAP instead of being dropped. ------------------------------------------------------ */
int bshot_set_cloud(bshot_ctx* c, const float* xyz, int n);         /* host pointer (H2D copy) */
int bshot_set_cloud_device(bshot_ctx* c, const float* d_xyz, int n); /* device-resident input */

/* ---- lookahead (throughput mode): build the grids of a FUTURE device-resident cloud and run its SR
 *      and ISS on the context's side stream now; the next bshot_set_cloud_device with the same
 *      pointer and size adopts the results instead of recomputing them. d_xyz must stay valid. */
int bshot_prefetch_cloud_device(bshot_ctx* c, const float* d_xyz, int n);
/* queue a cloud two sweeps ahead: grids + SR on a low-priority stream and ISS now, beside the
 * describe of the prefetched cloud; a later bshot_prefetch_cloud_device (or set_cloud_device) with
 * the same pointer promotes it. */
int bshot_queue_cloud_device(bshot_ctx* c, const float* d_xyz, int n);

/* ---- A1: segmentation ratio for every point, index order, origin / NaN skipped
 *      (replaces the loop at src/lidar_odometry.cpp:53-126). idx/ratio caller-sized >= n. --- */
int bshot_seg_ratio(bshot_ctx* c, int32_t* idx, float* ratio, int* n_out);

/* ---- A2: keypoint selection = libstdc++ std::sort(ratio) tail (src/lidar_odometry.cpp:131-153).
 *      Partial introsort: returns exactly the elements/order std::sort leaves in the last k slots. */
int bshot_select_topk(const int32_t* idx, const float* ratio, int n, int k, int32_t* kp_idx, float* kp_ratio,
                      int* k_out);

/* ---- A3: ISS keypoints of the current cloud (src/lidar_odometry.cpp:447-461), index order -- */
int bshot_iss(bshot_ctx* c, int32_t* kp_idx, int cap, int* n_out);

/* ---- A4-A7: normals (persistent mis-indexed array, include/bshot_bits.h:43-94) + SHOT LRF +
 *      352-bin histogram (bshot_bits.h:113-135) + B-SHOT binarisation (bshot_bits.h:144-278).
 *      shot (K x 352) and rf (K x 9) are optional (nullable) outputs. */
int bshot_describe(bshot_ctx* c, const float* kps, int k, float* shot, float* rf, uint32_t* bits);
/* normals array readback (N x 4: nx, ny, nz, curvature) for tests */
int bshot_get_normals(bshot_ctx* c, float* out, int n);

/* ---- A9: brute-force Hamming matching, first-index argmin both ways + mutual check
 *      (src/lidar_odometry.cpp:210-242, minVect include/bshot_bits.h:6-20). -------------- */
int bshot_match(bshot_ctx* c, const uint32_t* a, int na, const uint32_t* b, int nb, int32_t* left_nn,
                int32_t* right_nn, int32_t* corr_q, int32_t* corr_m, int* n_corr);

/* ---- A10: RANSAC rejection (src/lidar_odometry.cpp:251-261; PCL SampleConsensus semantics).
 *      Returns 1 when a model was found, 0 on PCL's identity/all-correspondences fallback. -- */
int bshot_ransac(const float* src, int ns, const float* tgt, int nt, const int32_t* corr_q, const int32_t* corr_m,
                 int n_corr, int max_iter, double thresh, float* T_out, int32_t* inl_q, int32_t* inl_m, int* n_inl);
/*      Same result, hypotheses scored on the GPU in one launch on the context's main stream
 *      (csrc/ransac.hip). ----------------------------------------------- */
int bshot_ransac_dev(bshot_ctx* c, const float* src, int ns, const float* tgt, int nt, const int32_t* corr_q,
                     const int32_t* corr_m, int n_corr, int max_iter, double thresh, float* T_out, int32_t* inl_q,
                     int32_t* inl_m, int* n_inl);

/*      Kernel-level check of the scorer: inlier counts of nhyp hypotheses (3 correspondence
 *      positions each, into the nidx correspondence pairs cs[i] -> ct[i], xyz floats) under
 *      thresh; c == NULL scores on the host (the scorer bshot_ransac uses), else on the GPU. ---- */
int bshot_ransac_scores(bshot_ctx* c, const float* cs, const float* ct, int nidx, const int32_t* hyp, int nhyp,
                        double thresh, int32_t* cnt);

/* ---- A11: point-to-point ICP (PCL IterativeClosestPoint defaults, src/lidar_odometry.cpp:291-297).
 *      src is already transformed by the initial guess; T_out = ICP final transformation.
 *      A finite target beyond the target grids' key range (2^20 cells of 500 mm: about +-524 km from
 *      the origin on any axis) fails the call with BSHOT_ECAP; non-finite targets are left out, as
 *      PCL's kd-tree does. ---- */
int bshot_icp(bshot_ctx* c, const float* src, int ns, const float* tgt, int nt, int max_iter, float* T_out,
              int* iters);

/* ---- Point-cloud preprocessor (myslam::Preprocessor, include/preprocess.h:7-57,
 *      src/preprocess.cpp:38-227): Velodyne laser returns -> range image (azimuth x vertical) ->
 *      ground removal -> occluded-edge removal -> point cloud in the reference's map order
 *      (azimuth, then vertical ascending). ------------------------------------------------------ */
typedef struct {           /* velodyne::Laser (include/VelodyneCapture.h:43-50), same 32-B layout */
    double azimuth;        /* degrees */
    double vertical;       /* degrees */
    uint16_t distance;     /* 2 mm units (src/preprocess.cpp:45) */
    uint8_t intensity;
    uint8_t id;
    int64_t time;
} bshot_laser;
typedef struct {
    double vert_init;      /* setVerticalInitial, radians; default -0.6 (src/preprocess.cpp:7) */
    double lowpt_th;       /* setLowPtThreshold, mm; default -2000 (include/preprocess.h:43) */
    int have_sel_list;     /* haveSelectList; default 0 */
    int save_sel;          /* saveSelectPoints; default 1 */
} bshot_pre_params;
typedef struct {           /* one getRangeImage entry with its getRemoveMap / getSelMap values */
    double azimuth, vertical, distance; /* radians, radians, mm */
    int32_t rm;            /* 0 kept, 1 ground / lost / vert_init, 2 self-car, 3 occluded; -1 no entry */
    int32_t sel;           /* 1 / 0; -1 no entry */
} bshot_pre_cell;
void bshot_pre_default_params(bshot_pre_params* p);
/* vert_deg: setVerticalAngles (degrees, any order); sel: setSelectedPoints (any order, used when
 * have_sel_list). xyz: caller's host buffer of cap points; *n_out = points written. */
int bshot_preprocess(bshot_ctx* c, const bshot_laser* lasers, int n, const double* vert_deg, int nv,
                     const bshot_pre_params* prm, const int32_t* sel, int nsel, float* xyz, int cap, int* n_out);
/* device-resident lasers and output (d_xyz: cap points); the call syncs the context's stream for
 * the count, so d_xyz can go straight to bshot_set_cloud_device / bshot_odom_process_device */
int bshot_preprocess_device(bshot_ctx* c, const bshot_laser* d_lasers, int n, const double* vert_deg, int nv,
                            const bshot_pre_params* prm, const int32_t* sel, int nsel, float* d_xyz, int cap,
                            int* n_out);
/* getRangeImage / getRemoveMap / getSelMap of the last run, merged over rimg's keys in map order
 * (including the zero entries removeOccluded's operator[] reads insert) */
int bshot_preprocess_cells(bshot_ctx* c, bshot_pre_cell* cells, int cap, int* n_out);

/* ---- Velodyne capture (include/VelodyneCapture.h:413-525): PCAP file ->
 *      1206-B data packets (host) -> laser records grouped into rotations (GPU). -------------- */
/* Reads a classic pcap file (usec or nsec timestamps, either byte order) the way capturePCAP
 * consumes it: keeps the records whose wire length - 42 == 1206 (:432-434), copies their UDP
 * payloads (bytes 42..1247) into payloads (cap packets x 1206 B; NULL: count only) and each
 * packet's time as the reference builds it, tv_sec followed by tv_usec left-aligned zero-filled to
 * 6 digits (:437-439). Host only, no GPU. Returns 0, *n_packets = packets found. */
int bshot_pcap_load(const char* path, uint8_t* payloads, int64_t* unixtime, int cap, int* n_packets);
/* Decodes npk packets (max_lasers 32: HDL-32E, 16: VLP-16 with the interpolated second half of each
 * firing) with the reference's rotation split and specifiedframe skip. out: the pushed rotations'
 * records back to back (cap records); rotation i = out[rot_start[i] .. + rot_count[i]). A packet
 * whose sensor type is not 0x21/0x22 is an error (the reference asserts, :453). */
int bshot_velodyne_decode(bshot_ctx* c, const uint8_t* payloads, const int64_t* unixtime, int npk, int max_lasers,
                          int specified_frame, bshot_laser* out, int cap, int32_t* rot_start, int32_t* rot_count,
                          int rot_cap, int* n_rot, int* n_out);
/* device-resident packets / times; d_out holds npk x 384 records in the reference's loop order and
 * rot_start / rot_count (host) index it */
int bshot_velodyne_decode_device(bshot_ctx* c, const uint8_t* d_payloads, const int64_t* d_unixtime, int npk,
                                 int max_lasers, int specified_frame, bshot_laser* d_out, int32_t* rot_start,
                                 int32_t* rot_count, int rot_cap, int* n_rot);

/* ---- Headless odometry (test/odometry_test.cpp:159-194 frame loop over LidarOdometry) ----- */
typedef struct bshot_odom bshot_odom;
typedef struct {
    int n_points, n_valid_ratios, n_keypoints, n_iss, n_target, n_mutual, n_inliers, icp_iters, gated;
    float h_diff, t_diff;
    float T_ransac[16];
    float pose[16];
    int map_size;
    float repeat_sr, repeat_iss;
    /* host wall ms per phase (TicToc, include/tic_toc.h): extract(SR+topK), iss, describe,
       match (map query + Hamming), ransac, icp, map update, kp_eval */
    float host_ms[8];
    /* setEvaluateCorr(true) (bshot_odom option "eval_corr" 1): the reference's correspondence
       statistics (src/lidar_odometry.cpp:303-330) over the RANSAC inliers, each cloud1 keypoint
       under T_best (setEvaluateICP, option "eval_icp" 1, the default) or the RANSAC transform:
       count, float mean, SD and the sorted median at size/2 of pcl::geometry::distance; NaN with no
       inliers. corr_n = -1 (and the rest 0) when not evaluated. */
    int corr_n;
    float corr_avg, corr_sd, corr_med;
} bshot_frame_stats;

int bshot_odom_create(bshot_odom** out, int device, const bshot_params* p);
void bshot_odom_destroy(bshot_odom* o);
const char* bshot_odom_last_error(const bshot_odom* o);
/* one sweep through extract + describe + match + RANSAC + gate + ICP + map update */
int bshot_odom_process(bshot_odom* o, const float* xyz, int n, bshot_frame_stats* st);
int bshot_odom_process_device(bshot_odom* o, const float* d_xyz, int n, bshot_frame_stats* st);
/* lookahead: the device cloud the NEXT bshot_odom_process_device call will receive. Its grids, SR
 * and ISS (side stream) and its top-K + describe (worker thread) run during the current frame's
 * matching / RANSAC / ICP / map update. Results are identical; the pointer must stay valid. */
int bshot_odom_set_next_device(bshot_odom* o, const float* d_next, int n_next);
/* the cloud after that (two calls ahead): its grids, SR and ISS are queued as well, so they run
 * beside the next sweep's describe. Optional; same validity rule. */
int bshot_odom_set_next2_device(bshot_odom* o, const float* d_next2, int n_next2);
/* a sweep's upload (n points, pinned host memory -> device), queued by a kernel on the stream the
 * sweep's grids/SR/ISS run on when it is set as next2: ordered before them without a host wait.
 * Call it before bshot_odom_set_next2_device with the same d_dst. */
int bshot_odom_upload(bshot_odom* o, float* d_dst, const float* h_src, int n);
/* odometry knobs: forwarded to bshot_set_option on the odometry's context */
int bshot_odom_set_option(bshot_odom* o, const char* name, int value);
/* per-sweep metrics as JSON lines (the reference only prints them): every stage's
 * counts, gated + gate_reasons (heading / translation / inliers, src/lidar_odometry.cpp:283-290),
 * h/t diff, map size, the main thread's wall ms per phase and the 3x4 pose. path NULL or "" stops.
 * The environment variable BSHOT_METRICS=<path> turns it on (append) for every odometry created. */
int bshot_odom_set_metrics_file(bshot_odom* o, const char* path);
/* Multi-GPU map exchange (BASELINE config 4; extension, no reference counterpart):
 * one process per GPU; rank 0 makes the 128-byte RCCL id (bshot_xchg_unique_id), every rank receives
 * it (any side channel, e.g. torch.distributed) and calls bshot_xchg_create. bshot_odom_exchange,
 * after each process call, all-gathers every rank's map offer of that sweep (<= kmax keypoints:
 * 10 mm grid position, ratio, 11 descriptor words) over RCCL from device buffers and inserts the
 * other ranks' batches into GPU replicas of their maps (replica r = rank r's map; include_self also
 * inserts this rank's own batch into replica `rank`), on the context's main stream, no host sync.
 * Requires the GPU map (option gpu_map >= 1). RCCL is loaded at run time. */
typedef struct bshot_xchg bshot_xchg;
int bshot_xchg_unique_id(void* id128);
int bshot_xchg_create(bshot_xchg** out, const void* id128, int nranks, int rank, int device, int kmax);
void bshot_xchg_destroy(bshot_xchg* x);
int bshot_odom_exchange(bshot_odom* o, bshot_xchg* x, int include_self);
/* measurement of the exchange's insert cost on fewer GPUs than ranks: bshot_odom_exchange, then
 * this rank's gathered batch is also inserted into `peers` further replicas (ids nranks ..
 * nranks + peers - 1), the per-sweep insert work of a job with nranks + peers ranks */
int bshot_odom_exchange_sim(bshot_odom* o, bshot_xchg* x, int peers);
/* GPU replica of rank r's map: entry count (syncs), and its entries around pos within range (the
 * reference's block loop; libstdc++ order) -> xyz (n x 3), bits (n x 11); count or -needed.
 * Call them from the thread that drives the odometry and its exchange (between two sweeps), never
 * concurrently with bshot_odom_exchange: an exchange may grow a replica while it is read. */
int bshot_odom_gpu_replica_size(bshot_odom* o, int replica);
/* host records (bshot_odom_map_delta's layout) into GPU replica r, for transports other than RCCL */
int bshot_odom_gpu_replica_insert(bshot_odom* o, int replica, const float* rec, int n);
int bshot_odom_gpu_replica_query(bshot_odom* o, int replica, const float pos[3], float range, float* xyz,
                                 uint32_t* bits, int cap);
/* frame-sharded single sequence (extension; BASELINE config 3 over several GPUs):
 * a sweep's extraction half (A0-A7 + ISS: extractKeypoints + computeDescriptors,
 * src/lidar_odometry.cpp:51-184) on one context, packed as a record of floats -- [0] magic, [1]
 * n_points, [2] n_valid, [3] k, [4] n_iss, [5] K, [6] m = min(n_points, K) (int bits), [7] 0, then
 * k x 3 keypoints, k ratios, k x 11 descriptor words (bit patterns), n_iss x 3 ISS points and m x 4
 * floats of the persistent normals array as the sweep's SHOT read it -- and the chain half (A8-A13,
 * :186-376) of the sequence on another, in sweep order. The set_next[2]_device lookahead applies to
 * the extracting context. extract returns the record length in floats, or -length when cap is too
 * small.
 * The reference's persistent normals array (include/bshot_bits.h:58-87) carries state from one
 * describe to the next through a sweep with fewer than K keypoints: its SHOT reads slots [k, K) as
 * the sweeps before it left them. The chain owner keeps the sequence's own array state and checks
 * each record's stale slots [k, m) against it bit for bit; a record that read other values (its
 * extracting context last described a different sweep) is refused with BSHOT_ESTALE and changes
 * nothing -- the caller then runs that sweep on the owner with bshot_odom_process[_device], which
 * starts from the sequence's state, so the chain stays identical to the sequential run. Across
 * sweeps with K keypoints each no record is ever refused. */
int bshot_odom_extract_device(bshot_odom* o, const float* d_xyz, int n, float* rec, int cap);
int bshot_odom_process_record(bshot_odom* o, const float* rec, int len, bshot_frame_stats* st);
/* wait for the lookahead work started by the last process call (the prefetched sweep's describe on
 * its worker thread, the queued sweep's launches and top-K) to be issued and finished; the results
 * stay ready for the next process call. Extension (no reference counterpart). */
int bshot_odom_drain(bshot_odom* o);
int bshot_odom_get_keypoints(bshot_odom* o, float* xyz, int cap);
int bshot_odom_get_ratios(bshot_odom* o, float* r, int cap);
int bshot_odom_get_bits(bshot_odom* o, uint32_t* bits, int cap);
int bshot_odom_get_target(bshot_odom* o, float* xyz, uint32_t* bits, int cap);
int bshot_odom_get_inliers(bshot_odom* o, int32_t* q, int32_t* m, int cap);
int bshot_odom_get_iss(bshot_odom* o, float* xyz, int cap);
bshot_ctx* bshot_odom_ctx(bshot_odom* o);

/* Map replication (throughput mode, BASELINE config 4): export the last frame's map delta
 * (K x (xyz, ratio, 11 words) = 60 B records) and import another sequence's delta into a replica. */
int bshot_odom_map_delta(bshot_odom* o, float* rec, int cap);
int bshot_odom_replica_insert(bshot_odom* o, int replica, const float* rec, int n);
int bshot_odom_replica_size(bshot_odom* o, int replica);

/* ---- Keypoint map (host; include/mymap.h:9-51, src/mymap.cpp, src/keypoint.cpp): the same
 *      unordered_map blocks, hasher, 10 mm keypoint grid and 800 mm suppression. No GPU needed. */
typedef struct bshot_map bshot_map;
bshot_map* bshot_map_create(void);
void bshot_map_destroy(bshot_map* m);
/* Keypoint::createKeypoint(pos, ratio, bits) + Map::addKeypoint */
int bshot_map_add(bshot_map* m, const float* xyz, float ratio, const uint32_t* bits11);
/* Map::getKeypoints(pos, range): returns count (or -needed when cap is too small) */
int bshot_map_query(bshot_map* m, const float* pos, float range, float* xyz, uint32_t* bits, int cap);
int bshot_map_size(bshot_map* m);
uint64_t bshot_map_block_id(const float* pos);
/* getKeypoints strategy, same output: 0 (default) visits the map's blocks when cheaper than the
 * reference's 21^3 block lookups, 1 always runs the reference's lookup loop */
int bshot_map_set_query_mode(bshot_map* m, int mode);

/* ---- options. Tuning knobs (results never depend on them): "ladder_grids" 4 (default) / 2 grids for
 *      the exact-kNN radius ladder; "ladder_front" 1 (default): two more small radii in front;
 *      "sr_start" 80 (default): percent scale of the ladder-start prediction (0: step 0); "sr_blocks" SR grid cap;
 *      "sr_xcd_chunk" 1024 (default): SR queries per XCD-local chunk of cell order (0: queries dealt round-robin);
 *      "iss_grid" 1 (default): ISS on the SR ladder's finest grid when its cell >= 2 salient radii;
 *      "iss_cell" 2 (default) / 1: ISS grid cell in salient radii (grid options take effect at the
 *      next set_cloud); "iss_ovf_blocks", "iss_nms_blocks", "chunk_blocks" grid caps; "normals_seg"
 *      1 (default): keypoint normals from the first normal_max_nn entries of the SHOT neighbour
 *      lists when normal_radius == shot_radius (the same (d2, idx)-sorted radius search);
 *      "ransac_dev" 1 (default): RANSAC hypotheses scored on the GPU; "topk_thread" 1 (default);
 *      "pre_fast" 1 (default): the preprocessor's one-sort path when it applies; "side_prio";
 *      "timing_mask" stage-event mask; "rank_wg" 2 (default: by neighbourhood size) / 1 / 0: SHOT
 *      neighbour ranking with a workgroup per keypoint or a wave per 64-rank chunk; "desc_slices" 1
 *      (default): the per-keypoint histogram / rank kernels in that many launches over the LPT order;
 *      "iss_defer" 0 (default) / 1: the queued sweep's ISS launches with its grids, or after the
 *      current sweep's ICP; "hist_pack" 1
 *      (default): the SHOT apply packs 12 ranks per LDS float atomic when the device passed the
 *      lane-order check (bshot_debug_lds_lane_order); "icp_device" 0 (default) / 1: ICP iterations
 *      handed to the host's Umeyama, or the whole loop on the device. Behaviour: "gpu_map" 1 (default, libstdc++ order) / 2
 *      (canonical order) / 0 (host Map); "xseq_targets" 0 (default): other sequences' replicas join
 *      the matching targets; "xchg_index" 1 (default): the exchange indexes every gathered offer into
 *      the replicas at once (iss stream), 0: logs them in HBM and indexes on read; "host_map_log" 1 (default; 0 under bshot_odom): keep the GPU map's
 *      insert log so the host Map view (LidarOdometry::getKeypoints, getBlockKeypoints) can be
 *      rebuilt -- without it host memory stays flat over a run and that view is unavailable;
 *      "map_sync" 1 (default): the GPU map insert is waited for and bshot_frame_stats.map_size
 *      reported every sweep; 0: the insert stays stream-ordered before the next sweep's map query
 *      (which settles its counters and reports capacity errors), map_size is -1. */
int bshot_set_option(bshot_ctx* c, const char* name, int value);

/* ---- instrumentation: per-stage device time (ms) accumulated with hipEvents on the context's
 *      stream since the last reset. Stage ids below. */
enum {
    BSHOT_STAGE_GRID = 0,
    BSHOT_STAGE_SR = 1,
    BSHOT_STAGE_ISS = 2,
    BSHOT_STAGE_NORMALS = 3,
    BSHOT_STAGE_SHOT_GATHER = 4,
    BSHOT_STAGE_SHOT_SORT = 5,
    BSHOT_STAGE_LRF = 6,
    BSHOT_STAGE_HIST = 7,
    BSHOT_STAGE_MATCH = 8,
    BSHOT_STAGE_ICP = 9,
    BSHOT_STAGE_RANSAC = 10,
    BSHOT_STAGE_PRE = 11,
    BSHOT_NSTAGES = 12
};
int bshot_stage_times(bshot_ctx* c, double* ms, int64_t* launches, int n);
void bshot_stage_reset(bshot_ctx* c);
void bshot_set_timing(bshot_ctx* c, int enabled);
/* work counters: [0] neighbourhood total of the last describe (SHOT pairs), [1] describes re-run with a
 * host plan after the device plan ran out of capacity (cumulative); ICP, cumulative: [2] ns the host
 * waited for nearest neighbours (or, option icp_device, for the device loop's result), [3] restarts
 * of the iterations after their kernel outwaited a stalled host, [4] ns of host work between two
 * waits, [5] iterations; [6] / [7] pool regrowths (count / bytes); ICP host loop: [8] ns of [2] spent
 * waiting for the lists kernel (iteration 0 or a restart), [9] grid searches after iteration 0 (sources
 * that left their candidate lists), [10] the most one wave took in one iteration. Returns the count (12). */
int bshot_work_counters(bshot_ctx* c, int64_t* out, int n);
/* instrumentation (outside timed regions): sum over all points of the current cloud of
 * |B(p, R)| (strict d2 < R^2, self included) -> the P_sr / P_iss work figures of SURVEY.md §8(d). */
int bshot_radius_pairs(bshot_ctx* c, float R, int64_t* total);
/* diagnostic: re-run the SR kernel with work counters: [0] queries, [5] 64-candidate chunks
 * streamed, [6] ladder steps skipped unstreamed (cube holds < max_nn candidates), [7] refinement
 * passes, [8] sum of bitonic sizes, [9] sum of selected neighbours, [10] sum of in-radius
 * candidates at the final step, [11] queries on the streaming selection path, [12..15] cycles in
 * ladder / fast selection / streaming selection / ratio math, [16 + s] queries whose ladder
 * stopped at step s. */
int bshot_debug_knn_stats(bshot_ctx* c, int64_t* out, int n);
/* the device check behind the packed SHOT apply (k_hist_fused): same-address ds_add_f32 lanes must
 * apply in ascending lane order. mismatches = bins that differ from the ascending replay (0
 * expected), sensitive = bins where the order mattered, active = the packed apply is in use
 * (option "hist_pack" and a clean check at bshot_create). Extension (no reference counterpart). */
int bshot_debug_lds_lane_order(bshot_ctx* c, int* mismatches, int* sensitive, int* active);

#ifdef __cplusplus
}
#endif
#endif
