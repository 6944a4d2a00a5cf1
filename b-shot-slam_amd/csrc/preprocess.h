// preprocess.h -- GPU preprocessor entry (csrc/preprocess.hip; reference myslam::Preprocessor,
// include/preprocess.h:7-57, src/preprocess.cpp). Its device state (bsh::PreState) is owned by
// bshot_ctx (c->pre), created on first use, grow-only like every other context pool.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/bshot_abi.h"

// the reference's thresholds (include/preprocess.h:42-47) and -2450/tan(vert_init_) (:80-81)
struct PreConsts {
    double grad_th, lowpt_th, height_th, dist_th, angdiff_th, init_r;
};

namespace bsh {

struct PreState;
// the reference's run() phases on the context's main stream (lasers on the device): readFrame
// (range-image cells), removeGround, removeOccluded, writePointCloud (kept points -> d_xyz, float3
// AoS in map order, *n_out their count; syncs the stream)
int pre_read(bshot_ctx* c, const bshot_laser* d_lasers, int n, const double* vert_deg, int nv,
             const bshot_pre_params* prm, const int32_t* sel, int nsel);
int pre_ground(bshot_ctx* c);
int pre_occluded(bshot_ctx* c);
int pre_write(bshot_ctx* c, float* d_xyz, int cap, int* n_out);
int pre_run(bshot_ctx* c, const bshot_laser* d_lasers, int n, const double* vert_deg, int nv,
            const bshot_pre_params* prm, const int32_t* sel, int nsel, float* d_xyz, int cap, int* n_out);
// host lasers -> the context's device staging buffer (async on the main stream)
int pre_stage_lasers(bshot_ctx* c, const bshot_laser* lasers, int n, const bshot_laser** d_out);
// context-owned output buffer for n points (grow-only)
float* pre_out_buffer(bshot_ctx* c, int n);
// the maps of the last run as the reference's getters return them, merged (bshot_preprocess_cells)
int pre_cells(bshot_ctx* c, std::vector<bshot_pre_cell>& out);
void pre_free(PreState* p);

}  // namespace bsh
