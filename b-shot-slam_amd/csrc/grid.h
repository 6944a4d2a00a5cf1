// grid.h -- host-side handle of one hashed voxel grid (device buffers, grow-only).
#pragma once
#include <hip/hip_runtime.h>

#include "dev_common.h"

namespace bsh {

struct DevGrid {
    int cap = 0, n = 0;
    unsigned int H = 0;
    float cell = 0.f;
    unsigned long long *keys = nullptr, *keys2 = nullptr;
    unsigned int *vals = nullptr, *vals2 = nullptr;
    float4* spts = nullptr;
    CellEntry* table = nullptr;
    int* ncells = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    bool alias = false;  // spts borrowed from another grid (nested ladder build)

    GridView view() const {
        GridView v;
        v.spts = spts;
        v.table = table;
        v.mask = H - 1;
        v.cell = cell;
        v.inv_cell = 1.0f / cell;
        return v;
    }
};

// Builds the grid of d_xyz (N x 3 floats, device) with edge `cell`; writes float4 copies of the
// points in index order to d_pts4 (N entries).
// write_pts4 = false: d_pts4 already holds the cloud (another grid built it) and is only read.
// min_cap: capacity floor when the buffers (re)grow -- for clouds whose size keeps growing (the ICP
// targets), so that regrowth, a device-wide stall (hipFree), is rare
hipError_t grid_build(DevGrid& g, const float* d_xyz, int n, float cell, float4* d_pts4, hipStream_t s,
                      bool write_pts4 = true, int min_cap = 0);
// defer: park the buffers until context teardown (regrowth inside the sweep loop; regrow.h)
void grid_free(DevGrid& g, bool defer = false);
// four nested grids (cells c0, 2c0, 4c0, 8c0) from one sort; g[1..3].spts alias g[0].spts.
// level_mask: the levels whose hash tables are built (the sorted points are always written);
// min_cap as grid_build's; finer (nullable): a fifth grid of cells c0 / 2 on the same points (ISS's);
// zero0 / zero1 (nullable, n >= 1): two ints each that the build's first kernel zeroes
hipError_t grid_build_ladder(DevGrid* const* g, const float* d_xyz, int n, float c0, float4* d_pts4, hipStream_t s,
                             unsigned level_mask = 0xFu, int min_cap = 0, DevGrid* finer = nullptr,
                             int* zero0 = nullptr, int* zero1 = nullptr);


}  // namespace bsh
