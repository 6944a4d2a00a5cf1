// velodyne.h -- GPU Velodyne packet decode (csrc/velodyne.hip; reference
// include/VelodyneCapture.h:413-525). Device state owned by bshot_ctx (c->velo).
#pragma once
#include <vector>

#include "../../include/bshot_abi.h"

namespace bsh {

struct VeloState;
// npk device-resident 1206-B packets -> d_rec (npk * 384 records of 32 B, record order = the
// reference's loop order); rot_start / rot_count: the rotations the reference's capture would push
int velo_decode(bshot_ctx* c, const unsigned char* d_pk, const long long* d_ut, int npk, int max_lasers,
                int specified_frame, unsigned long long* d_rec, std::vector<int>& rot_start, std::vector<int>& rot_count);
void velo_free(VeloState* v);

}  // namespace bsh
