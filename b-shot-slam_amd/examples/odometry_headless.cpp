// odometry_headless.cpp -- test/odometry_test.cpp's frame loop (:111-194) without the PCAP
// capture and cv::viz window, compiled against the drop-in C++ API (include/bshot/) and linked
// with libbshot_amd.so. Input: deterministic synthetic sweeps, or (pre=1) synthetic laser returns
// through myslam::Preprocessor as odometry_test feeds them (:111-117, :143-163).
// Output: one line per frame, "frame <id> <n_points> <n_inliers> <pose row-major, 16 x %a>".
//
//   bin/odometry_headless [frames=5] [keypoints=600] [sensor=0] [sr_type=CV] [pre=0] [pcap=<file>]
//                         [trajectory=<file>]
// The trajectory file is odometry_test's "Save trajectories" output (:348-361): the translation of
// every frame's pose, "x y z" per line (default stream formatting), then an empty line.
// With a pcap file (HDL-32E packets) the loop is odometry_test's whole chain: HDL32ECapture ->
// Preprocessor -> LidarOdometry (:60-61, :111-194).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "../../include/bshot/lidar_odometry.h"
#include "../../include/bshot/preprocess.h"
#include "../../include/bshot/velodyne.h"

extern "C" int synth_sweep(int sensor, uint32_t scene_seed, int frame, int no_ground, float max_range, float* xyz,
                           int cap, float* pose_out);
extern "C" int synth_lasers(int sensor, uint32_t scene_seed, int frame, float max_range, float sensor_height,
                            void* out, int cap);

int main(int argc, char** argv) {
    const int frames = argc > 1 ? std::atoi(argv[1]) : 5;
    const int k = argc > 2 ? std::atoi(argv[2]) : 600;
    const int sensor = argc > 3 ? std::atoi(argv[3]) : 0;
    const std::string sr = argc > 4 ? argv[4] : "CV";
    const std::string pcap = argc > 6 ? argv[6] : "";
    const bool pre = (argc > 5 && std::atoi(argv[5]) != 0) || !pcap.empty();
    const std::string traj_file = argc > 7 ? argv[7] : "";
    std::vector<myslam::Vector3f> trajectory;
    bshot_params p;
    bshot_default_params(&p);
    p.num_keypoints = k;
    try {
        myslam::LidarOdometry lo(p, 0);
        lo.setSRType(sr);
        std::vector<float> buf(3 * 400000);
        // odometry_test.cpp:111-117: vertical table, vert_init -0.6, lowpt_th -1950
        std::unique_ptr<myslam::Preprocessor> prep;
        std::vector<double> vertAngle;
        std::unique_ptr<velodyne::HDL32ECapture> capture;
        if (!pcap.empty()) {
            capture.reset(new velodyne::HDL32ECapture(pcap, 0));
            vertAngle = capture->getVerticalAngle();
            std::sort(vertAngle.begin(), vertAngle.end());
        } else if (pre) {
            std::vector<velodyne::Laser> probe(400000);
            const int nl = synth_lasers(sensor, 42, 0, 120000.f, 2450.f, probe.data(), (int)probe.size());
            if (nl < 0) return 2;
            for (int i = 0; i < nl && (int)vertAngle.size() < 256; ++i) {
                if (i > 0 && probe[i].azimuth != probe[0].azimuth) break;
                vertAngle.push_back(probe[i].vertical);
            }
            std::sort(vertAngle.begin(), vertAngle.end());
        }
        if (pre) {
            prep.reset(new myslam::Preprocessor());
            prep->setVerticalAngles(vertAngle);
            prep->setVerticalInitial(-0.6);
            prep->setLowPtThreshold(-1950);
        }
        for (int f = 0; f < frames; ++f) {
            auto pc = std::make_shared<std::vector<myslam::Vector3f>>();
            int n = 0;
            if (pre) {
                std::vector<velodyne::Laser> lasers;
                if (capture) {
                    if (!capture->isRun()) break;
                    *capture >> lasers;
                    if (lasers.empty()) { --f; continue; }
                } else {
                    lasers.resize(400000);
                    const int nl = synth_lasers(sensor, 42, f, 120000.f, 2450.f, lasers.data(), (int)lasers.size());
                    if (nl < 0) return 2;
                    lasers.resize(nl);
                }
                prep->setPointCloud(pc);
                prep->setLasers(lasers);
                prep->haveSelectList(false);
                prep->saveSelectPoints(true);
                prep->run();
                n = (int)pc->size();
            } else {
                n = synth_sweep(sensor, 42, f, 0, 120000.f, buf.data(), 400000, nullptr);
                if (n < 0) return 2;
                pc->reserve(n);
                for (int i = 0; i < n; ++i) pc->emplace_back(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]);
            }
            myslam::Frame::Ptr fptr = myslam::Frame::createFrame();
            fptr->setPointCloud(pc);
            if (!lo.isInitial()) lo.passSrc2Ref();
            lo.setSrcFrame(fptr);
            lo.extractKeypoints();
            lo.computeDescriptors();
            lo.featureMatching();
            lo.evaluateEstimation();
            lo.poseEstimation();
            lo.updateMap();
            lo.updateCorrespondence();
            const myslam::Matrix4f P = fptr->getPose();
            trajectory.push_back(P.topRightCorner());  // odometry_test.cpp:195-198
            std::printf("frame %d %d %d", f, n, (int)lo.inlierCorrespondences().size());
            for (int j = 0; j < 16; ++j) std::printf(" %a", P.m[j]);
            std::printf("\n");
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "odometry_headless: %s\n", e.what());
        return 1;
    }
    if (!traj_file.empty()) {
        std::ofstream ofs(traj_file);
        for (const myslam::Vector3f& p : trajectory) ofs << p[0] << " " << p[1] << " " << p[2] << std::endl;
        ofs << std::endl;
    }
    return 0;
}
