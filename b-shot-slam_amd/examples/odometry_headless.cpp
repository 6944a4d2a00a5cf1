// odometry_headless.cpp -- test/odometry_test.cpp's frame loop (:122-194) without the PCAP
// capture, preprocessor and cv::viz window, compiled against the drop-in C++ API
// (include/bshot/) and linked with libbshot_amd.so. Input: deterministic synthetic sweeps.
// Output: one line per frame, "frame <id> <n_points> <n_inliers> <pose row-major, 16 x %a>".
//
//   bin/odometry_headless [frames=5] [keypoints=600] [sensor=0] [sr_type=CV]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "../../include/bshot/lidar_odometry.h"

extern "C" int synth_sweep(int sensor, uint32_t scene_seed, int frame, int no_ground, float max_range, float* xyz,
                           int cap, float* pose_out);

int main(int argc, char** argv) {
    const int frames = argc > 1 ? std::atoi(argv[1]) : 5;
    const int k = argc > 2 ? std::atoi(argv[2]) : 600;
    const int sensor = argc > 3 ? std::atoi(argv[3]) : 0;
    const std::string sr = argc > 4 ? argv[4] : "CV";
    bshot_params p;
    bshot_default_params(&p);
    p.num_keypoints = k;
    try {
        myslam::LidarOdometry lo(p, 0);
        lo.setSRType(sr);
        std::vector<float> buf(3 * 400000);
        for (int f = 0; f < frames; ++f) {
            const int n = synth_sweep(sensor, 42, f, 0, 120000.f, buf.data(), 400000, nullptr);
            if (n < 0) return 2;
            auto pc = std::make_shared<std::vector<myslam::Vector3f>>();
            pc->reserve(n);
            for (int i = 0; i < n; ++i) pc->emplace_back(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]);
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
            std::printf("frame %d %d %d", f, n, (int)lo.inlierCorrespondences().size());
            for (int j = 0; j < 16; ++j) std::printf(" %a", P.m[j]);
            std::printf("\n");
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "odometry_headless: %s\n", e.what());
        return 1;
    }
    return 0;
}
