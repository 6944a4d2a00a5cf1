// preprocess.h -- myslam::Preprocessor, same members and methods as the reference
// (include/preprocess.h:7-57), running on the GPU (csrc/preprocess.hip) through the C ABI.
// run() = readFrame + removeGround + removeOccluded + writePointCloud, each phase a set of kernels on
// the preprocessor's context; the getters rebuild the reference's std::maps from the device table.
// Differences: run() on an empty laser list returns with an empty cloud (the reference spins in
// `while(!readFrame())`); the preprocessor owns a bshot_ctx on `device` (default 0).
#pragma once
#include <map>
#include <memory>
#include <vector>

#include "../bshot_abi.h"
#include "types.h"
#include "velodyne.h"

namespace myslam {

class Preprocessor {
  public:
    typedef std::shared_ptr<Preprocessor> Ptr;
    typedef std::map<double, double> RangeImgCol;
    typedef std::map<double, RangeImgCol> RangeImg;
    typedef std::map<double, int> RemoveCol;
    typedef std::map<double, RemoveCol> RemoveMap;
    typedef std::map<double, bool> SelCol;
    typedef std::map<double, SelCol> SelMap;

    Preprocessor();
    Preprocessor(std::vector<velodyne::Laser>& lasers, std::vector<double>& vertAngle,
                 std::shared_ptr<std::vector<Vector3f>> pc);
    explicit Preprocessor(int device);
    ~Preprocessor();
    Preprocessor(const Preprocessor&) = delete;
    Preprocessor& operator=(const Preprocessor&) = delete;

    void setLasers(std::vector<velodyne::Laser>& lasers);
    void setSelectedPoints(std::vector<int>& selptlist);
    void saveSelectPoints(bool savesel) { prm_.save_sel = savesel ? 1 : 0; }
    void haveSelectList(bool havesellist) { prm_.have_sel_list = havesellist ? 1 : 0; }
    void setVerticalAngles(std::vector<double>& vertAngle);
    void setVerticalInitial(double vertinit) { prm_.vert_init = vertinit; }
    void setLowPtThreshold(double lowptth) { prm_.lowpt_th = lowptth; }
    void setPointCloud(std::shared_ptr<std::vector<Vector3f>> pc) { pc_ = pc; }
    bool readFrame();        // Read in a frame
    void removeGround();     // Remove ground points
    void removeOccluded();   // Remove occluded points
    void writePointCloud();  // append the kept points to the point cloud
    void run();
    RangeImg getRangeImage();
    RemoveMap getRemoveMap();
    SelMap getSelMap();

    // extension: device-resident lasers -> device-resident points (d_xyz: cap points), for
    // LidarOdometry::setSrcFrameDevice; returns the point count
    int runDevice(const velodyne::Laser* d_lasers, int n, float* d_xyz, int cap);
    bshot_ctx* context() { return ctx_; }

  private:
    std::vector<bshot_pre_cell> cells();

    bshot_ctx* ctx_ = nullptr;
    bshot_pre_params prm_;
    std::vector<double> vertAngle_;
    std::vector<int> selpts_;
    std::vector<velodyne::Laser> lasers_;
    std::shared_ptr<std::vector<Vector3f>> pc_;
    bool have_frame_ = false;
};

}  // namespace myslam
