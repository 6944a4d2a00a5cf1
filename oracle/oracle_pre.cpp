// oracle_pre.cpp -- TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's point-cloud
// preprocessor: range image from Velodyne laser returns, ground removal,
// occluded-edge removal, point-cloud write-out. Loaded only by tests/ as the checker.
//
// Restates /root/reference/src/preprocess.cpp:38-227 with include/preprocess.h:39-55, keeping its
// data structures (std::map<double, std::map<double, ...>>, so the iteration order, the
// operator[] insertions of removeOccluded and every last-write-wins overwrite are the reference's
// by construction). Arithmetic is the reference's expression by expression: double range-image
// geometry, float Eigen::Vector3f points (norm = sqrt((x*x + y*y) + z*z), no FMA: the project-wide
// -ffp-contract=off convention), float std::asin (using namespace std: asin(float) is
// asinf), glibc sin/cos/tan. The reference ships no fixture for this stage: parity unpinned vs the
// reference binary, pinned by the restatement only.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

#include "oracle_api.h"

namespace {

const double kPi = 3.1415926535897932384626433832795;  // CV_PI

struct F3 {
    float x, y, z;
    float norm() const { return std::sqrt((x * x + y * y) + z * z); }
};

struct Pre {
    // include/preprocess.h:39-55
    std::vector<double> vertAngle_;
    double vert_init_ = -0.6;
    double grad_th = 45;
    double lowpt_th = -2000;
    double height_th = 500;
    double dist_th = 3000;
    double angdiff_th = 1.0 * kPi / 180.0;
    std::map<double, std::map<double, double>> rimg;
    std::map<double, std::map<double, int>> rmmap;
    std::map<double, std::map<double, bool>> selmap;
    std::vector<int> selpts_;
    bool save_sel_ = true;
    bool have_sel_list_ = false;
    std::vector<F3> pc;

    // src/preprocess.cpp:38-70
    void readFrame(const oracle_laser* lasers, int n) {
        int i = 0;
        size_t selidx = 0;
        for (int l = 0; l < n; ++l) {
            const oracle_laser& laser = lasers[l];
            const double distance = static_cast<double>(laser.distance) * 2;
            const double azimuth = laser.azimuth * kPi / 180.0;
            const double vertical = laser.vertical * kPi / 180.0;
            rimg[azimuth][vertical] = distance;
            rimg[azimuth][vert_init_] = 2450 / std::sin(vert_init_);
            rmmap[azimuth][vertical] = 0;
            rmmap[azimuth][vert_init_] = 1;
            if (!have_sel_list_) {
                selmap[azimuth][vertical] = true;
            } else if (selidx < selpts_.size() && selpts_[selidx] == i) {
                selmap[azimuth][vertical] = true;
                selidx++;
            } else {
                selmap[azimuth][vertical] = false;
            }
            i++;
        }
    }

    // src/preprocess.cpp:72-164
    void removeGround() {
        for (auto& col : rimg) {
            bool isInitVert = true, lost_pt = false, set_th_pt = false, prev_is_ground = true;
            double vert_prev = vert_init_;
            const double x_0 = (-2450 / std::tan(vert_prev)) * std::sin(col.first);
            const double y_0 = (-2450 / std::tan(vert_prev)) * std::cos(col.first);
            const double z_0 = -2450;
            F3 p_prev{(float)x_0, (float)y_0, (float)z_0};
            F3 p_th = p_prev;
            for (auto& vert : col.second) {
                if (isInitVert) {
                    isInitVert = false;
                    continue;
                }
                const double x = vert.second * std::cos(vert.first) * std::sin(col.first);
                const double y = vert.second * std::cos(vert.first) * std::cos(col.first);
                const double z = vert.second * std::sin(vert.first);
                const F3 p_curr{(float)x, (float)y, (float)z};
                const F3 d{p_curr.x - p_prev.x, p_curr.y - p_prev.y, p_curr.z - p_prev.z};
                // asin(float) * 180 is float arithmetic; the division by CV_PI promotes to double
                const double grad = (double)(std::asin((p_curr.z - p_prev.z) / d.norm()) * 180.0f) / kPi;
                if (prev_is_ground && (grad > grad_th || vert.second == 0 || vert.second < p_prev.norm())) {
                    set_th_pt = true;
                    p_th = p_prev;
                }
                if (prev_is_ground) {
                    if (grad < grad_th && !lost_pt) {
                        rmmap[col.first][vert.first] = 1;
                        prev_is_ground = true;
                    } else {
                        rmmap[col.first][vert.first] = 0;
                        prev_is_ground = false;
                    }
                } else if (!prev_is_ground && p_curr.z < lowpt_th && grad < grad_th) {
                    rmmap[col.first][vert.first] = 1;
                    prev_is_ground = true;
                    set_th_pt = false;
                }
                if (vert.second == 0) {
                    rmmap[col.first][vert.first] = 1;
                    lost_pt = true;
                    prev_is_ground = false;
                } else {
                    lost_pt = false;
                }
                if (vert.second < p_prev.norm() && vert.second != 0) {
                    rmmap[col.first][vert.first] = 0;
                    prev_is_ground = false;
                }
                if (set_th_pt && (p_curr.z - p_th.z) < height_th && p_curr.z < p_prev.z) {
                    set_th_pt = false;
                    rmmap[col.first][vert.first] = 1;
                    prev_is_ground = true;
                }
                if (x <= 820 && x >= -820 && y <= 1300 && y >= -1800 && z <= 100 && z >= -2000)
                    rmmap[col.first][vert.first] = 2;
                p_prev = p_curr;
                vert_prev = vert.first;
            }
        }
    }

    // src/preprocess.cpp:166-195 (operator[] inserts zero entries exactly as the reference does)
    void removeOccluded() {
        for (auto& vert : vertAngle_) {
            const double v = vert * kPi / 180.0;
            double prev_hor = 0;
            bool isFirst = true;
            for (auto& col : rimg) {
                if (isFirst) {
                    prev_hor = col.first;
                    isFirst = false;
                } else if (rimg[col.first][v] == 0) {
                    continue;
                } else {
                    const double d_dist = rimg[col.first][v] - rimg[prev_hor][v];
                    const double d_hor = col.first - prev_hor;
                    if (std::fabs(d_dist) > dist_th && std::fabs(d_hor) < angdiff_th) {
                        if (d_dist > 0) {
                            if (rmmap[col.first][v] == 0) rmmap[col.first][v] = 3;
                        } else {
                            if (rmmap[prev_hor][v] == 0) rmmap[prev_hor][v] = 3;
                        }
                    }
                    prev_hor = col.first;
                }
            }
        }
    }

    // src/preprocess.cpp:197-215
    void writePointCloud() {
        for (auto& col : rimg) {
            for (auto& vert : col.second) {
                if (vert.second == 0 || vert.first == vert_init_) continue;
                const double x = vert.second * std::cos(vert.first) * std::sin(col.first);
                const double y = vert.second * std::cos(vert.first) * std::cos(col.first);
                const double z = vert.second * std::sin(vert.first);
                if (rmmap[col.first][vert.first] == 0 && selmap[col.first][vert.first] == save_sel_)
                    pc.push_back(F3{(float)x, (float)y, (float)z});
            }
        }
    }
};

}  // namespace

extern "C" int oracle_preprocess(const oracle_laser* lasers, int n, const double* vert_deg, int nv,
                                 const oracle_pre_params* prm, const int32_t* sel, int nsel, float* xyz, int cap,
                                 int* n_out, oracle_pre_cell* cells, int cell_cap, int* n_cells) {
    Pre P;
    P.vertAngle_.assign(vert_deg, vert_deg + nv);
    std::sort(P.vertAngle_.begin(), P.vertAngle_.end());  // setVerticalAngles sorts (src/preprocess.cpp:30-33)
    P.vert_init_ = prm->vert_init;
    P.lowpt_th = prm->lowpt_th;
    P.have_sel_list_ = prm->have_sel_list != 0;
    P.save_sel_ = prm->save_sel != 0;
    if (sel && nsel > 0) {
        P.selpts_.assign(sel, sel + nsel);
        std::sort(P.selpts_.begin(), P.selpts_.end());  // setSelectedPoints sorts (:25-28)
    }
    // run() (src/preprocess.cpp:217-226)
    P.readFrame(lasers, n);
    P.removeGround();
    P.removeOccluded();
    // the maps as getRangeImage/getRemoveMap/getSelMap return them after run(): rimg keys, with
    // rm = -1 / sel = -1 where rmmap / selmap have no entry (taken before writePointCloud, whose
    // operator[] reads insert nothing new: every key it visits exists in all three maps or is skipped)
    int nc = 0;
    for (auto& col : P.rimg)
        for (auto& vert : col.second) {
            if (cells && nc < cell_cap) {
                oracle_pre_cell& c = cells[nc];
                c.azimuth = col.first;
                c.vertical = vert.first;
                c.distance = vert.second;
                auto ri = P.rmmap.find(col.first);
                int rm = -1;
                if (ri != P.rmmap.end()) {
                    auto rj = ri->second.find(vert.first);
                    if (rj != ri->second.end()) rm = rj->second;
                }
                auto si = P.selmap.find(col.first);
                int sl = -1;
                if (si != P.selmap.end()) {
                    auto sj = si->second.find(vert.first);
                    if (sj != si->second.end()) sl = sj->second ? 1 : 0;
                }
                c.rm = rm;
                c.sel = sl;
            }
            nc++;
        }
    if (n_cells) *n_cells = nc;
    P.writePointCloud();
    const int np = (int)P.pc.size();
    if (n_out) *n_out = np;
    if (np > cap) return -np;
    for (int i = 0; i < np; ++i) {
        xyz[3 * i] = P.pc[i].x;
        xyz[3 * i + 1] = P.pc[i].y;
        xyz[3 * i + 2] = P.pc[i].z;
    }
    return nc > cell_cap && cells ? -nc : 0;
}
