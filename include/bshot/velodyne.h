// velodyne.h -- velodyne::Laser and the PCAP capture classes of the reference
// (include/VelodyneCapture.h:43-60, :62-525, :528-612), same names and retrieval API.
// The capture decodes on the GPU (csrc/velodyne.hip): open() reads the whole file, decodes every
// packet in one pass and queues the rotations the reference's capture thread would have queued;
// operator>> / retrieve pop them. No UDP socket mode (Boost absent) and no capture thread: the queue
// is complete when open() returns, so isRun() is "rotations left".
#pragma once
#include <algorithm>
#include <deque>
#include <string>
#include <vector>

#include "../bshot_abi.h"

namespace velodyne {

struct Laser {
    double azimuth;           // degrees
    double vertical;          // degrees
    unsigned short distance;  // 2 mm units
    unsigned char intensity;
    unsigned char id;
    long long time;

    bool operator<(const Laser& laser) const {
        if (azimuth == laser.azimuth) return id < laser.id;
        return azimuth < laser.azimuth;
    }
};
static_assert(sizeof(Laser) == sizeof(bshot_laser), "velodyne::Laser must match bshot_laser (32 B)");

class VelodyneCapture {
  public:
    VelodyneCapture();
    virtual ~VelodyneCapture();
    bool open(const std::string& filename);
    bool isOpen();
    bool isRun();
    void close();
    void retrieve(std::vector<Laser>& lasers, const bool sort = false);
    void operator>>(std::vector<Laser>& lasers) { retrieve(lasers, false); }
    void setDevice(int device) { device_ = device; }  // GPU used by open() (default 0)

  protected:
    int MAX_NUM_LASERS = 32;
    std::vector<double> lut;
    int specifiedframe = 0;

  private:
    std::deque<std::vector<Laser>> queue_;
    std::string filename_;
    bool opened_ = false;
    int device_ = 0;
};

class VLP16Capture : public VelodyneCapture {
  public:
    VLP16Capture() { initialize(); }
    explicit VLP16Capture(const std::string& filename) {
        initialize();
        open(filename);
    }

  private:
    void initialize() {
        MAX_NUM_LASERS = 16;
        lut = {-15.0, 1.0, -13.0, 3.0, -11.0, 5.0, -9.0, 7.0, -7.0, 9.0, -5.0, 11.0, -3.0, 13.0, -1.0, 15.0};
    }
};

class HDL32ECapture : public VelodyneCapture {
  public:
    HDL32ECapture() { initialize(); }
    HDL32ECapture(const std::string& filename, int spframe) {
        initialize();
        specifiedframe = spframe;
        open(filename);
    }
    std::vector<double> getVerticalAngle() { return lut; }

  private:
    void initialize() {
        MAX_NUM_LASERS = 32;
        lut = {-30.67, -9.3299999, -29.33, -8.0, -28, -6.6700001, -26.67, -5.3299999, -25.33, -4.0, -24.0,
               -2.6700001, -22.67, -1.33, -21.33, 0.0, -20.0, 1.33, -18.67, 2.6700001, -17.33, 4.0, -16,
               5.3299999, -14.67, 6.6700001, -13.33, 8.0, -12.0, 9.3299999, -10.67, 10.67};
    }
};

}  // namespace velodyne
