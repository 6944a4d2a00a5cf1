// oracle_velo.cpp -- TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's Velodyne packet
// decode: VelodyneCapture::capturePCAP's per-packet loop
// (include/VelodyneCapture.h:413-525) over already-framed 1206-byte data packets, with the
// HDL32ECapture / VLP16Capture vertical tables (:534, :572) and packet layout (:86-110). The queue
// of rotations it fills (:383-389 / :500-506) is returned flattened: records in push order plus
// the record count of every pushed rotation. Loaded only by tests/ as the checker. The reference
// ships no capture file: parity unpinned vs the reference binary, pinned by the restatement only.
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle_api.h"

namespace {

#pragma pack(push, 1)
struct LaserReturn {
    uint16_t distance;
    uint8_t intensity;
};
#pragma pack(pop)
struct FiringData {
    uint16_t blockIdentifier;
    uint16_t rotationalPosition;
    LaserReturn laserReturns[32];
};
struct DataPacket {
    FiringData firingData[12];
    uint32_t gpsTimestamp;
    uint8_t mode;
    uint8_t sensorType;
};
// only LaserReturn is packed in the reference (:89-95): sizeof(DataPacket) is 1208 there too, the
// cast views 1206 payload bytes (sensorType at offset 1205)
static_assert(offsetof(DataPacket, sensorType) == 1205, "Velodyne data packet");

const double kLut32[32] = {-30.67, -9.3299999, -29.33, -8.0, -28, -6.6700001, -26.67, -5.3299999,
                           -25.33, -4.0, -24.0, -2.6700001, -22.67, -1.33, -21.33, 0.0,
                           -20.0, 1.33, -18.67, 2.6700001, -17.33, 4.0, -16, 5.3299999,
                           -14.67, 6.6700001, -13.33, 8.0, -12.0, 9.3299999, -10.67, 10.67};
const double kLut16[16] = {-15.0, 1.0, -13.0, 3.0, -11.0, 5.0, -9.0, 7.0, -7.0, 9.0, -5.0, 11.0, -3.0, 13.0, -1.0, 15.0};

}  // namespace

extern "C" int oracle_velodyne_decode(const uint8_t* payloads, const int64_t* unixtime, int npk, int max_lasers,
                                      int specified_frame, oracle_laser* out, int cap, int32_t* rot_count,
                                      int rot_cap, int* n_out, int* n_rot) {
    const int LASER_PER_FIRING = 32, FIRING_PER_PKT = 12;
    const int MAX_NUM_LASERS = max_lasers;
    const double* lut = max_lasers == 16 ? kLut16 : kLut32;
    int specifiedframe = specified_frame;
    double last_azimuth = 0.0;
    std::vector<oracle_laser> lasers;
    std::vector<std::vector<oracle_laser>> queue;
    for (int p = 0; p < npk; ++p) {
        DataPacket pk;
        std::memset(&pk, 0, sizeof(pk));
        std::memcpy(&pk, payloads + (size_t)p * 1206, 1206);
        const DataPacket* packet = &pk;
        if (!(packet->sensorType == 0x21 || packet->sensorType == 0x22)) return -1;  // assert (:453)
        const long long unixtime_p = unixtime[p];
        double interpolated = 0.0;
        if (packet->firingData[1].rotationalPosition < packet->firingData[0].rotationalPosition) {
            interpolated =
                ((packet->firingData[1].rotationalPosition + 36000) - packet->firingData[0].rotationalPosition) / 2.0;
        } else {
            interpolated = (packet->firingData[1].rotationalPosition - packet->firingData[0].rotationalPosition) / 2.0;
        }
        for (int firing_index = 0; firing_index < FIRING_PER_PKT; firing_index++) {
            const FiringData firing_data = packet->firingData[firing_index];
            for (int laser_index = 0; laser_index < LASER_PER_FIRING; laser_index++) {
                double azimuth = static_cast<double>(firing_data.rotationalPosition);
                if (laser_index >= MAX_NUM_LASERS) azimuth += interpolated;
                if (azimuth >= 36000) azimuth -= 36000;
                if (last_azimuth > azimuth) specifiedframe--;
                if (specifiedframe > 0) {
                    last_azimuth = azimuth;
                    continue;
                }
                if (last_azimuth > azimuth) {
                    queue.push_back(lasers);
                    lasers.clear();
                }
                oracle_laser laser;
                std::memset(&laser, 0, sizeof(laser));
                laser.azimuth = azimuth / 100.0;
                laser.vertical = lut[laser_index % MAX_NUM_LASERS];
                laser.distance = firing_data.laserReturns[laser_index % MAX_NUM_LASERS].distance;
                laser.intensity = firing_data.laserReturns[laser_index % MAX_NUM_LASERS].intensity;
                laser.id = static_cast<unsigned char>(laser_index % MAX_NUM_LASERS);
                laser.time = unixtime_p;
                lasers.push_back(laser);
                last_azimuth = azimuth;
            }
        }
    }
    int k = 0;
    for (size_t r = 0; r < queue.size(); ++r) {
        if ((int)r < rot_cap) rot_count[r] = (int)queue[r].size();
        for (const oracle_laser& l : queue[r]) {
            if (k < cap) out[k] = l;
            ++k;
        }
    }
    *n_out = k;
    *n_rot = (int)queue.size();
    return (k > cap || (int)queue.size() > rot_cap) ? -2 : 0;
}
