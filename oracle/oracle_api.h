/* oracle_api.h -- TEST INFRASTRUCTURE ONLY. C ABI of the CPU restatement (the oracle).
 * Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * PARITY UNPINNED vs PCL (see oracle_core.h). Matrices are row-major 4x4 float. */
#ifndef BSHOT_ORACLE_API_H
#define BSHOT_ORACLE_API_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    float seg_radius;       /* 3000  src/lidar_odometry.cpp:68 */
    int seg_max_nn;         /* 300   :70 */
    int sr_type;            /* 0 CV, 1 CVS, 2 CVSN  include/lidar_odometry.h:47 */
    int num_keypoints;      /* 600   src/lidar_odometry.cpp:138 */
    float iss_salient;      /* 60    :452 */
    float iss_nonmax;       /* 40    :453 */
    double iss_gamma21;     /* 0.975 :454 */
    double iss_gamma32;     /* 0.975 :455 */
    int iss_min_nn;         /* 5     :456 */
    float normal_radius;    /* 3000  :174 */
    int normal_max_nn;      /* 300   include/bshot_bits.h:66 */
    float shot_radius;      /* 3000  src/lidar_odometry.cpp:175 */
    float map_range;        /* 100000 :198 */
    int ransac_max_iter;    /* 2000  :254 */
    double ransac_thresh;   /* 1500  :256 */
    int icp_max_iter;       /* 10 (PCL default) */
    int run_icp;            /* 1     test/odometry_test.cpp:41 */
    int run_iss;            /* 1 (ISS runs every frame, :164-170) */
    int map_canonical;      /* 0: map blocks in libstdc++ unordered_map order (the reference); 1: in
                               first-insert order (the GPU map's canonical mode, not the reference's) */
    int eval_icp;           /* 1     setEvaluateICP (test/odometry_test.cpp:108): the corr statistics use
                               T_best_ (1) or the RANSAC transform (0), src/lidar_odometry.cpp:306-309 */
} oracle_params;

typedef struct {
    int n_points, n_valid_ratios, n_keypoints, n_iss, n_target, n_mutual, n_inliers, icp_iters, gated;
    float h_diff, t_diff;
    float T_ransac[16];
    float pose[16];
    int map_size;
    float repeat_sr, repeat_iss; /* kpEvaluation rates (src/lidar_odometry.cpp:392-445) */
    /* evaluate_corr_ statistics (src/lidar_odometry.cpp:303-330), always computed here: count of
       RANSAC inliers, float mean, SD and sorted median (at size/2) of their distances after the
       transform; NaN when there are none */
    int corr_n;
    float corr_avg, corr_sd, corr_med;
} oracle_frame_stats;

int oracle_seg_ratio(const float* xyz, int n, float radius, int max_nn, int sr_type, int32_t* idx_out,
                     float* ratio_out, int* n_out);
int oracle_select_keypoints(const int32_t* idx, const float* ratio, int n, int k, int32_t* kp_idx, float* kp_ratio,
                            int* k_out);
int oracle_iss(const float* xyz, int n, float salient, float nonmax, double g21, double g32, int min_nn,
               int32_t* out_idx, int cap, int* n_out, double* third_eig);
int oracle_normals(const float* xyz, int n, const float* kps, int k, float radius, int max_nn, float* normals);
int oracle_shot(const float* xyz, int n, const float* normals, const float* kps, int k, float radius, float* shot,
                float* rf_out);
int oracle_binarize(const float* shot, int k, uint32_t* bits);
int oracle_match(const uint32_t* a, int na, const uint32_t* b, int nb, int32_t* left, int32_t* right,
                 int32_t* corr_q, int32_t* corr_m, int* ncorr);
int oracle_ransac(const float* src_xyz, int ns, const float* tgt_xyz, int nt, const int32_t* corr_q,
                  const int32_t* corr_m, int ncorr, int max_iter, double thresh, float* T_out, int32_t* inl_q,
                  int32_t* inl_m, int* n_inl);
int oracle_icp(const float* src_xyz, int ns, const float* tgt_xyz, int nt, int max_iter, float* T_final,
               int* iters);

/* point-cloud preprocessor (src/preprocess.cpp), oracle_pre.cpp */
typedef struct {          /* velodyne::Laser, include/VelodyneCapture.h:43-50 (32 B) */
    double azimuth;       /* degrees */
    double vertical;      /* degrees */
    uint16_t distance;    /* 2 mm units */
    uint8_t intensity;
    uint8_t id;
    int64_t time;
} oracle_laser;
typedef struct {
    double vert_init;     /* radians, setVerticalInitial (test/odometry_test.cpp:32: -0.6) */
    double lowpt_th;      /* mm, setLowPtThreshold (test/odometry_test.cpp:33: -1950) */
    int have_sel_list;    /* haveSelectList */
    int save_sel;         /* saveSelectPoints */
} oracle_pre_params;
typedef struct {          /* one rimg entry after run(): rm / sel = -1 where rmmap / selmap lack the key */
    double azimuth, vertical, distance;
    int32_t rm, sel;
} oracle_pre_cell;
int oracle_preprocess(const oracle_laser* lasers, int n, const double* vert_deg, int nv, const oracle_pre_params* prm,
                      const int32_t* sel, int nsel, float* xyz, int cap, int* n_out, oracle_pre_cell* cells,
                      int cell_cap, int* n_cells);

/* Velodyne data-packet decode (include/VelodyneCapture.h:413-525), oracle_velo.cpp: packets of
 * 1206 B, max_lasers 32 (HDL-32E) or 16 (VLP-16); out = the pushed rotations' records in order,
 * rot_count = records per pushed rotation. */
int oracle_velodyne_decode(const uint8_t* payloads, const int64_t* unixtime, int npk, int max_lasers,
                           int specified_frame, oracle_laser* out, int cap, int32_t* rot_count, int rot_cap,
                           int* n_out, int* n_rot);

/* test hooks: exact radius search (FLANN semantics), Jacobi eigen, umeyama */
int oracle_radius_search(const float* xyz, int n, const float* q, float radius, int max_nn, int32_t* idx,
                         float* d2, int cap);
void oracle_eig3(const double* a9, double* w3, double* v9);
void oracle_umeyama(const double* src, const double* dst, int n, int use_float, double* T16);

/* OpenMP threads for the stages the reference runs with OpenMP (normals, SHOT) */
void oracle_set_threads(int n);
int oracle_get_threads(void);
/* threads for the per-point SR and ISS loops (default 1, as the reference); results do not depend on it */
void oracle_set_point_threads(int n);

void oracle_default_params(oracle_params* p);
void* oracle_odom_create(const oracle_params* p);
void oracle_odom_destroy(void* h);
int oracle_odom_process(void* h, const float* xyz, int n, oracle_frame_stats* st);
/* per-frame artefacts of the last processed frame; return count (or -needed if cap too small) */
int oracle_odom_get_keypoints(void* h, float* xyz, int cap);
int oracle_odom_get_ratios(void* h, float* r, int cap);
int oracle_odom_get_bits(void* h, uint32_t* bits, int cap);
int oracle_odom_get_target(void* h, float* xyz, uint32_t* bits, int cap);
int oracle_odom_get_inliers(void* h, int32_t* q, int32_t* m, int cap);
int oracle_odom_get_iss(void* h, float* xyz, int cap);

#ifdef __cplusplus
}
#endif
#endif
