// velodyne.h -- velodyne::Laser, the laser-return record of the reference's capture
// (include/VelodyneCapture.h:43-60), with the same members, layout and ordering operator.
#pragma once
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

}  // namespace velodyne
