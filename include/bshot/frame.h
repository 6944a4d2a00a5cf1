// frame.h -- myslam::Frame, same members and methods as the reference (include/frame.h:10-51).
#pragma once
#include <bitset>
#include <memory>
#include <vector>

#include "types.h"

namespace myslam {

class Frame {
  public:
    typedef std::shared_ptr<Frame> Ptr;
    typedef std::shared_ptr<std::vector<Vector3f>> PCPtr;
    typedef std::shared_ptr<std::vector<std::bitset<352>>> DCPPtr;
    unsigned long id_;
    long long timestamp_;
    Matrix4f T_c_w_;
    PCPtr pointcloud_;
    PCPtr keypoints_;
    DCPPtr descriptors_;
    bool is_key_frame_;

  public:
    Frame();
    Frame(long id, double time_stamp = 0, Matrix4f T_c_w = Matrix4f::Identity(), PCPtr pc = nullptr,
          PCPtr kps = nullptr, DCPPtr dcpts = nullptr, bool isKeyframe = false);
    ~Frame();

    static Frame::Ptr createFrame();

    void setTimestamp(const long long timestamp);
    void setPose(const Matrix4f& T_c_w);
    void setPointCloud(PCPtr pc);
    void setKeypoints(PCPtr kps);
    void setDescriptors(DCPPtr dcpts);
    unsigned long getID() { return id_; }
    long long getTimestamp() { return timestamp_; }
    Matrix4f getPose() { return T_c_w_; }
    PCPtr getPointCloud() { return pointcloud_; }
    PCPtr getKeypoints() { return keypoints_; }
    DCPPtr getDescriptors() { return descriptors_; }
    bool isKeyframe() { return is_key_frame_; }
};

}  // namespace myslam
