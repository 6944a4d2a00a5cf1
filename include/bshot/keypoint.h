// keypoint.h -- myslam::Keypoint, same API as the reference (include/keypoint.h:8-32).
#pragma once
#include <memory>

#include "bshot_bits.h"
#include "types.h"

namespace myslam {

class Keypoint {
  public:
    typedef std::shared_ptr<Keypoint> Ptr;
    Keypoint();
    Keypoint(unsigned long id, Vector3f& position, float& seg_ratio, bshot_descriptor& descriptor);

    inline Vector3f getPosition() const { return pos_; }
    inline bshot_descriptor getDescriptor() const { return descriptor_; }
    inline unsigned long getId() const { return id_; }
    inline float getSegRatio() const { return seg_ratio_; }

    // quantises the position to a 10 mm grid (src/keypoint.cpp:23-32)
    static Keypoint::Ptr createKeypoint(Vector3f& pos, float seg_ratio, bshot_descriptor descriptor);

  private:
    unsigned long id_;
    static unsigned long factory_id_;
    Vector3f pos_;
    float seg_ratio_ = 0.f;
    bshot_descriptor descriptor_;
};

}  // namespace myslam
