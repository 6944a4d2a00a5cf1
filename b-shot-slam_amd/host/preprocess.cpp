// preprocess.cpp -- myslam::Preprocessor (include/bshot/preprocess.h) over the GPU preprocessor
// phases (csrc/preprocess.hip). Mirrors src/preprocess.cpp:4-227 call by call.
#include "../../include/bshot/preprocess.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "../csrc/preprocess.h"

namespace myslam {

static void pcheck(bshot_ctx* c, int rc, const char* what) {
    if (rc != BSHOT_OK)
        throw std::runtime_error(std::string("Preprocessor::") + what + ": " + (c ? bshot_last_error(c) : "no context"));
}

Preprocessor::Preprocessor() : Preprocessor(0) {}

Preprocessor::Preprocessor(int device) {
    bshot_pre_default_params(&prm_);
    if (bshot_create(&ctx_, device, nullptr) != BSHOT_OK) throw std::runtime_error("Preprocessor: bshot_create failed");
}

Preprocessor::Preprocessor(std::vector<velodyne::Laser>& lasers, std::vector<double>& vertAngle,
                           std::shared_ptr<std::vector<Vector3f>> pc)
    : Preprocessor(0) {
    lasers_ = lasers;
    pc_ = pc;
    setVerticalAngles(vertAngle);
}

Preprocessor::~Preprocessor() { bshot_destroy(ctx_); }

void Preprocessor::setLasers(std::vector<velodyne::Laser>& lasers) { lasers_ = lasers; }

void Preprocessor::setSelectedPoints(std::vector<int>& selptlist) {
    selpts_ = selptlist;
    std::sort(selpts_.begin(), selpts_.end());
}

void Preprocessor::setVerticalAngles(std::vector<double>& vertAngle) {
    vertAngle_ = vertAngle;  // degrees
    std::sort(vertAngle_.begin(), vertAngle_.end());
}

bool Preprocessor::readFrame() {
    have_frame_ = false;
    if (lasers_.empty()) return false;
    const bshot_laser* d = nullptr;
    const int n = (int)lasers_.size();
    pcheck(ctx_, bsh::pre_stage_lasers(ctx_, reinterpret_cast<const bshot_laser*>(lasers_.data()), n, &d),
           "readFrame");
    pcheck(ctx_, bsh::pre_read(ctx_, d, n, vertAngle_.data(), (int)vertAngle_.size(), &prm_, selpts_.data(),
                               (int)selpts_.size()),
           "readFrame");
    have_frame_ = true;
    return true;
}

void Preprocessor::removeGround() {
    if (have_frame_) pcheck(ctx_, bsh::pre_ground(ctx_), "removeGround");
}

void Preprocessor::removeOccluded() {
    if (have_frame_) pcheck(ctx_, bsh::pre_occluded(ctx_), "removeOccluded");
}

void Preprocessor::writePointCloud() {
    if (!have_frame_ || !pc_) return;
    const int n = (int)lasers_.size();
    float* d = bsh::pre_out_buffer(ctx_, n);
    if (!d) throw std::runtime_error("Preprocessor::writePointCloud: alloc");
    int np = 0;
    pcheck(ctx_, bsh::pre_write(ctx_, d, n, &np), "writePointCloud");
    const size_t base = pc_->size();
    pc_->resize(base + (size_t)np);
    static_assert(sizeof(Vector3f) == 12, "Vector3f is three packed floats");
    if (np > 0 && hipMemcpy(pc_->data() + base, d, sizeof(float) * 3 * (size_t)np, hipMemcpyDeviceToHost) != hipSuccess)
        throw std::runtime_error("Preprocessor::writePointCloud: D2H");
}

void Preprocessor::run() {
    if (pc_) pc_->clear();
    if (!readFrame()) return;
    removeGround();
    removeOccluded();
    writePointCloud();
}

int Preprocessor::runDevice(const velodyne::Laser* d_lasers, int n, float* d_xyz, int cap) {
    int np = 0;
    pcheck(ctx_, bshot_preprocess_device(ctx_, reinterpret_cast<const bshot_laser*>(d_lasers), n, vertAngle_.data(),
                                         (int)vertAngle_.size(), &prm_, selpts_.data(), (int)selpts_.size(), d_xyz,
                                         cap, &np),
           "runDevice");
    return np;
}

std::vector<bshot_pre_cell> Preprocessor::cells() {
    std::vector<bshot_pre_cell> v;
    pcheck(ctx_, bsh::pre_cells(ctx_, v), "getRangeImage");
    return v;
}

Preprocessor::RangeImg Preprocessor::getRangeImage() {
    RangeImg r;
    for (const bshot_pre_cell& e : cells()) r[e.azimuth][e.vertical] = e.distance;
    return r;
}

Preprocessor::RemoveMap Preprocessor::getRemoveMap() {
    RemoveMap r;
    for (const bshot_pre_cell& e : cells())
        if (e.rm >= 0) r[e.azimuth][e.vertical] = e.rm;
    return r;
}

Preprocessor::SelMap Preprocessor::getSelMap() {
    SelMap r;
    for (const bshot_pre_cell& e : cells())
        if (e.sel >= 0) r[e.azimuth][e.vertical] = e.sel != 0;
    return r;
}

}  // namespace myslam
