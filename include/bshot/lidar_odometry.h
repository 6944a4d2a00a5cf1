// lidar_odometry.h -- myslam::LidarOdometry, the drop-in surface of the reference
// (include/lidar_odometry.h:13-73) used by odometry_test / kp_test. Same method names, call order
// and per-frame state; the hot stages run on the GPU through the C ABI context (bshot_abi.h).
// Differences: PCL types leave the API (PointCloudXYZ instead of
// pcl::PointCloud<pcl::PointXYZ>); the bshot member becomes private; two constructors take the
// parameter block / device; lastStats() reports per-frame counters.
#pragma once
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../bshot_abi.h"
#include "bshot_bits.h"
#include "frame.h"
#include "mymap.h"
#include "types.h"

namespace myslam {

class LidarOdometry {
  public:
    LidarOdometry();
    explicit LidarOdometry(const bshot_params& p, int device = 0);
    ~LidarOdometry();
    LidarOdometry(const LidarOdometry&) = delete;
    LidarOdometry& operator=(const LidarOdometry&) = delete;

    enum STATUS { INITIAL, RUN };

    void setRefFrame(Frame::Ptr ref);
    void setSrcFrame(Frame::Ptr src);
    // device-resident cloud (n x 3 floats already in HBM); the Frame keeps a host copy lazily
    void setSrcFrameDevice(Frame::Ptr src, const float* d_xyz, int n);
    // extension (throughput mode): start the NEXT device-resident sweep now -- grids, SR and ISS on
    // the side stream, then top-K, keypoint gather and describe on a host worker thread -- while
    // this sweep's matching, RANSAC, ICP and map update run. Call after computeDescriptors(); the
    // next setSrcFrameDevice() with the same pointer adopts the results (identical to computing
    // them in order).
    void prefetchFrameDevice(const float* d_xyz, int n);
    // the sweep after the prefetched one: grids, SR and ISS queued now (no worker), promoted by
    // the next prefetchFrameDevice() with the same pointer
    void queueFrameDevice(const float* d_xyz, int n);
    // wait until the lookahead work in flight (worker, queue and top-K threads) has been issued and
    // finished on the host; the prefetched results stay ready for adoption
    void drainLookahead();
    // replace the persistent normals array (include/bshot_bits.h:58-87) by a sequence's state
    // (logical size, slots [0, m)); a pending lookahead describe is joined and dropped first.
    // Extension: the frame-sharded chain owner's own extraction (bshot_odom_process_record)
    void resetNormalsState(int size, int m, const float* slots);
    void extractKeypoints();
    void computeDescriptors();
    void featureMatching();
    void poseEstimation();
    void evaluateEstimation();
    void updateMap();
    void updateCorrespondence();
    void kpEvaluation();
    PointCloudXYZ issKpDetection(const PointCloudXYZ& kps);
    void passSrc2Ref();
    bool isInitial() { return status_ == INITIAL; }
    Frame::Ptr getRefFrame() { return ref_; }
    Frame::Ptr getSrcFrame() { return src_; }
    Frame::PCPtr getKeypoints();
    Frame::PCPtr getSrcKeypoints();
    Frame::PCPtr getRefKeypoints();
    Frame::PCPtr getISSKeypoints();
    typedef std::vector<Vector3f> PC;
    std::vector<PC> getBlockKeypoints();
    Matrix4f getTransformationDiff() { return src_->getPose() * ref_->getPose().inverse(); }
    std::vector<std::pair<Vector3f, Vector3f>> getCorrespondences() { return corrs; }
    PointCloudXYZ eigen2pcl(Frame::PCPtr pcptr);
    std::vector<bshot_descriptor> eigen2dc(Frame::DCPPtr pcptr);
    void setSRType(std::string sr_type);
    void setEvaluateCorr(bool eval_corr) { evaluate_corr_ = eval_corr; }
    void setEvaluateICP(bool eval_icp) { evaluate_icp_ = eval_icp; }
    void setRunICP(bool run_icp) { run_icp_ = run_icp; }

    // extension (frame-sharded single sequence): the extraction half of a sweep
    // (A0-A7 + ISS: extractKeypoints + computeDescriptors) as data, so one context can extract a
    // sweep and another -- another GPU's -- run the chain on it
    struct Extracted {
        int n_points = 0, n_valid = 0;
        PointCloudXYZ kps, iss;
        std::vector<float> ratios;
        std::vector<uint32_t> words;  // 11 per keypoint (bits_to_words)
        // the persistent normals array (include/bshot_bits.h:58-87) as this sweep's SHOT read it:
        // slots [0, min(n_points, K)) x (nx, ny, nz, curvature). Slots [0, k) are the sweep's own;
        // [k, min(n_points, K)) are stale ones left by earlier describes of the extracting context,
        // which the chain owner checks against the sequence's own (bshot_odom_process_record).
        // Filled by extractedWithNormals(); empty from extracted().
        std::vector<float> normals;
    };
    // the current sweep's extraction half (after computeDescriptors)
    Extracted extracted() const;
    // the same plus the persistent normals slots [0, min(n_points, K)) (one device read, synchronous)
    Extracted extractedWithNormals();
    // adopt another context's extraction of this sweep: the next extractKeypoints/computeDescriptors
    // take it as computed here (matching, RANSAC, ICP and the map update then run as usual)
    void setSrcFrameExtracted(Frame::Ptr src, std::shared_ptr<const Extracted> ex);

    // extensions (not in the reference)
    const bshot_frame_stats& lastStats() const { return stats_; }
    const bshot_params& params() const { return prm_; }
    bshot_ctx* context() { return ctx_; }
    const std::vector<float>& segRatios() const { return seg_ratios_; }
    const PointCloudXYZ& targetKeypoints() const { return cloud2_kps_; }
    // with the GPU map the target descriptors stay in HBM until asked for
    const std::vector<bshot_descriptor>& targetDescriptors();
    const std::vector<std::pair<int, int>>& inlierCorrespondences() const { return corr_; }
    Map& globalMap() {
        syncHostMap();
        return globalMap_;
    }
    const std::string& lastError() const { return err_; }

  private:
    void check(int rc, const char* where);
    struct Lookahead;
    struct TopkAhead;
    void runAhead(Lookahead& la);
    void joinAhead();
    void dropTopkAhead();
    void dropReady();
    std::shared_ptr<TopkAhead> topk_ahead_;  // sweep after next: top-K on its own thread once its SR lands
    std::shared_ptr<Lookahead> ahead_;  // next sweep, in flight on the worker thread
    std::shared_ptr<Lookahead> ready_;  // adopted for the current sweep

    bshot_params prm_;
    bshot_ctx* ctx_ = nullptr;
    Frame::Ptr ref_, src_;
    PointCloudXYZ src_pc_, ref_pc_;  // src_pcl_ / ref_pcl_ (src/lidar_odometry.cpp:29-41)
    const float* src_dev_ = nullptr;  // device cloud of the current sweep (null for host or external frames)
    const void* src_ext_ = nullptr;   // identity of an external frame's record (setSrcFrameExtracted); never read
    int src_n_ = 0;
    // identity the adopted lookahead / record must match for the current sweep
    const void* srcId() const { return src_ext_ ? src_ext_ : static_cast<const void*>(src_dev_); }
    STATUS status_;
    std::vector<float> seg_ratios_;
    Map globalMap_;
    PointCloudXYZ cloud1_kps_, cloud2_kps_;
    std::vector<bshot_descriptor> cloud1_bshot_, cloud2_bshot_;
    std::vector<std::pair<int, int>> corr_;  // RANSAC inliers (index_query, index_match)
    std::vector<std::pair<Vector3f, Vector3f>> corrs;
    Matrix4f T_best_, T_ransac_;
    bool shouldUpdateMap;
    std::string sr_type_;
    bool evaluate_icp_, evaluate_corr_, run_icp_;
    PointCloudXYZ isskps_src, isskps_ref;
    bshot_frame_stats stats_;
    std::string err_;
    // GPU map (context option gpu_map, csrc/gmap.hip): the map lives in HBM; the host Map above is
    // rebuilt on demand (getKeypoints, getBlockKeypoints, globalMap) by replaying what updateMap
    // offered it, in order
    struct MapLogEntry {
        Frame::PCPtr kps;
        Frame::DCPPtr desc;
        std::vector<float> ratios;
        Matrix4f T;
    };
    std::vector<MapLogEntry> map_log_;  // kept only with context option host_map_log (default 1)
    size_t map_log_done_ = 0;
    size_t map_log_skipped_ = 0;  // sweeps inserted while host_map_log was 0: the host view is incomplete
    bool targets_on_device_ = false;  // cloud2_bshot_ not filled: the rows are in the context
    int last_na_ = 0;
    void syncHostMap();
    bool gpuMap() const;
    void ransacStep(int na, int nb, const std::vector<int32_t>& cq, const std::vector<int32_t>& cm, int nc);
};

}  // namespace myslam
