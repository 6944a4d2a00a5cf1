// grid.hip -- hashed voxel grid build on gfx950 (the "hashed-voxel radius-neighbour search" of
// BASELINE.json north_star). Replaces pcl::KdTreeFLANN::setInputCloud
// (src/lidar_odometry.cpp:53-54, include/bshot_bits.h:52-53) with a counting structure that every
// radius query kernel streams with coalesced float4 loads.
//
// Build: keys -> rocprim radix sort of (cell key, idx) -> cell-start detection (binary search for
// the run end) + hash insert -> scatter float4 points into cell order. All O(N), no host sync.
#include <algorithm>

#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include "dev_common.h"
#include "grid.h"
#include "kernels.h"
#include "regrow.h"

// the ladder's 63-bit key sort: rocprim's default picks block sort + merge passes below 1M items
// (~1 + 7 launches at 130k keys); GRID_SORT_ONESWEEP (diagnostic builds) forces its onesweep radix
// passes instead
#ifndef GRID_SORT_ONESWEEP
#define GRID_SORT_ONESWEEP 0
#endif
#ifndef GRID_SORT_BLOCK_ITEMS
#define GRID_SORT_BLOCK_ITEMS 0  // 0: rocprim's default block sort (1024 keys); else 256 x this / 256 keys per block
#endif
#if GRID_SORT_ONESWEEP
using LadderSortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                    rocprim::default_config, 0>;
#elif GRID_SORT_BLOCK_ITEMS > 0
using LadderSortConfig = rocprim::radix_sort_config<rocprim::default_config,
                                                    rocprim::merge_sort_config<256, 256, GRID_SORT_BLOCK_ITEMS / 256>,
                                                    rocprim::default_config>;
#else
using LadderSortConfig = rocprim::default_config;
#endif

namespace bsk {

__global__ void k_grid_keys(const float* __restrict__ xyz, int n, float cell, unsigned long long* __restrict__ keys,
                            unsigned int* __restrict__ vals, float4* __restrict__ pts4) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    if (pts4) pts4[i] = make_float4(x, y, z, __uint_as_float((unsigned)i));
    unsigned long long k = BS_EMPTY_KEY;
    if (__builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z)) {
        const int ix = cell_of(x, cell), iy = cell_of(y, cell), iz = cell_of(z, cell);
        if (ix > -(1 << 20) && ix < (1 << 20) && iy > -(1 << 20) && iy < (1 << 20) && iz > -(1 << 20) && iz < (1 << 20))
            k = cell_key(ix, iy, iz);
    }
    keys[i] = k;
    vals[i] = (unsigned)i;
}

__global__ void k_grid_clear(CellEntry* __restrict__ table, unsigned int H) {
    const unsigned int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < H) {
        table[i].key = BS_EMPTY_KEY;
        table[i].start = 0;
        table[i].count = 0;
    }
}

__global__ void k_grid_cells(const unsigned long long* __restrict__ keys, const unsigned int* __restrict__ vals,
                             const float4* __restrict__ pts4, int n, CellEntry* __restrict__ table, unsigned int mask,
                             float4* __restrict__ spts, int* __restrict__ ncells) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    spts[j] = pts4[vals[j]];
    const unsigned long long k = keys[j];
    if (k == BS_EMPTY_KEY) return;
    if (j > 0 && keys[j - 1] == k) return;
    // run end: first position > j whose key differs (keys sorted ascending)
    int lo = j + 1, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] == k) lo = mid + 1;
        else hi = mid;
    }
    unsigned int h = hash_key(k) & mask;
    while (true) {
        const unsigned long long prev = atomicCAS(&table[h].key, BS_EMPTY_KEY, k);
        if (prev == BS_EMPTY_KEY) break;
        h = (h + 1) & mask;
    }
    table[h].start = (unsigned)j;
    table[h].count = (unsigned)(lo - j);
    atomicAdd(ncells, 1);
}

// ---- nested ladder grids (cells c/2, c, 2c, 4c, 8c) from ONE sort ------------------------
// floor(x / (2^L c)) == floor(x / c) >> L exactly (division by a power of two commutes with the
// double rounding), so a cell of any level is a prefix of the hierarchical key
//   (17-bit biased level-3 x, y, z) | level-2 | level-1 | level-0 | level-(-1) child bits
// (63 bits) and points sorted by that key are contiguous per cell at every level. The range rule
// |ix| < 2^20 at the finest level (cells c/2: cell_key's range; +-98 km per axis at c = 187.5 mm,
// +-524 km at the ICP's c = 1000 mm) keeps the level-3 coordinate in 17 bits; every grid of the
// ladder indexes the same points. The finest level (c/2) is ISS's grid when the caller asks for it.
__device__ __forceinline__ bool ladder_cells(float x, float y, float z, float c0, int& ix, int& iy, int& iz) {
    if (!(__builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z))) return false;
    const float ch = c0 * 0.5f;
    ix = cell_of(x, ch);
    iy = cell_of(y, ch);
    iz = cell_of(z, ch);
    const int lim = 1 << 20;
    return ix > -lim && ix < lim && iy > -lim && iy < lim && iz > -lim && iz < lim;
}

// zero (nullable): two int pairs the cloud's next kernels expect zeroed (SR / ISS error words, ISS
// overflow count), so the build carries those fills
struct ZeroWords {
    int* p[2];
};
__global__ void k_ladder_keys(const float* __restrict__ xyz, int n, float c0, unsigned long long* __restrict__ keys,
                              unsigned int* __restrict__ vals, float4* __restrict__ pts4, ZeroWords zero) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 4 && zero.p[threadIdx.x >> 1]) zero.p[threadIdx.x >> 1][threadIdx.x & 1] = 0;
    if (i >= n) return;
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    pts4[i] = make_float4(x, y, z, __uint_as_float((unsigned)i));
    unsigned long long k = BS_EMPTY_KEY;
    int ix, iy, iz;  // cells c0 / 2
    if (ladder_cells(x, y, z, c0, ix, iy, iz)) {
        const unsigned long long x3 = (unsigned)((ix >> 4) + (1 << 16)), y3 = (unsigned)((iy >> 4) + (1 << 16)),
                                 z3 = (unsigned)((iz >> 4) + (1 << 16));
        k = (x3 << 46) | (y3 << 29) | (z3 << 12);
#pragma unroll
        for (int m = 3; m >= 1; --m) {  // the child bits of levels 2, 1, 0, -1 (cells c0/2 >> m)
            const unsigned cbits = (unsigned)((((ix >> m) & 1) << 2) | (((iy >> m) & 1) << 1) | ((iz >> m) & 1));
            k |= (unsigned long long)cbits << (3 * m);
        }
        k |= (unsigned long long)(((ix & 1) << 2) | ((iy & 1) << 1) | (iz & 1));
    }
    keys[i] = k;
    vals[i] = (unsigned)i;
}

// the levels' hash tables of one ladder build, cleared and filled in one launch
// each: entries 0..3 = levels 0..3 (cells c0 .. 8 c0), entry 4 = the finest level (c0 / 2)
#define GRID_LEVELS 5
struct Tables4 {
    CellEntry* t[GRID_LEVELS];
    unsigned int mask[GRID_LEVELS];
    unsigned int H[GRID_LEVELS];
};
// a level's cell in the ladder's finest cells (c0 / 2) and its prefix shift in the key
__device__ __forceinline__ int level_shift(int L) { return L == 4 ? 0 : L + 1; }

__global__ void k_grid_clear4(Tables4 T, unsigned level_mask) {
    const unsigned int i = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int L = 0; L < GRID_LEVELS; ++L)
        if (((level_mask >> L) & 1u) && i < T.H[L]) {
            T.t[L][i].key = BS_EMPTY_KEY;
            T.t[L][i].start = 0;
            T.t[L][i].count = 0;
        }
}

// the cells of every level in level_mask at once, and the points in key order
// range_err (nullable): bit 8 set when a finite point lies beyond the key range (|cell| >= 2^20 at the
// finest level: +-98 km per axis at c0 = 187.5 mm). Such a point is in no cell, so no search finds
// it; the SR error word carries the bit and the sweep fails loudly instead of dropping the point
// (ADVICE r05). Non-finite points have no cell by design (the reference's searches skip them too).
__global__ void k_ladder_cells4(const unsigned long long* __restrict__ keys, const unsigned int* __restrict__ vals,
                                const float4* __restrict__ pts4, int n, float c0, Tables4 T, unsigned level_mask,
                                float4* __restrict__ spts, int* __restrict__ range_err) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const float4 p = pts4[vals[j]];
    spts[j] = p;
    const unsigned long long k = keys[j];
    if (k == BS_EMPTY_KEY) {
        if (range_err && __builtin_isfinite(p.x) && __builtin_isfinite(p.y) && __builtin_isfinite(p.z))
            atomicOr(range_err, 8);
        return;
    }
    const unsigned long long km1 = j > 0 ? keys[j - 1] : BS_EMPTY_KEY;
    int ix, iy, iz;
    ladder_cells(p.x, p.y, p.z, c0, ix, iy, iz);
#pragma unroll
    for (int L = 0; L < GRID_LEVELS; ++L) {
        if (!((level_mask >> L) & 1u)) continue;
        const int m = level_shift(L);
        const unsigned long long pk = k >> (3 * m);
        if (j > 0 && (km1 >> (3 * m)) == pk) continue;  // not the first of its run at this level
        int lo = j + 1, hi = n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((keys[mid] >> (3 * m)) == pk) lo = mid + 1;
            else hi = mid;
        }
        const unsigned long long ck = cell_key(ix >> m, iy >> m, iz >> m);
        unsigned int h = hash_key(ck) & T.mask[L];
        while (true) {
            const unsigned long long prev = atomicCAS(&T.t[L][h].key, BS_EMPTY_KEY, ck);
            if (prev == BS_EMPTY_KEY) break;
            h = (h + 1) & T.mask[L];
        }
        T.t[L][h].start = (unsigned)j;
        T.t[L][h].count = (unsigned)(lo - j);
    }
}

}  // namespace bsk

// host side --------------------------------------------------------------------------------
namespace bsh {

static unsigned int pow2_at_least(unsigned int x) {
    unsigned int p = 1024;
    while (p < x) p <<= 1;
#ifdef GRID_H_FIXED
    // diagnostic builds only (table-size sensitivity; safe only for clouds with < 2^GRID_H_FIXED cells)
    if (p > (1u << GRID_H_FIXED)) p = 1u << GRID_H_FIXED;
#endif
    return p;
}

// g[0..3]: grids of cell c0, 2 c0, 4 c0, 8 c0 built from one 63-bit radix sort; g[0] owns the
// sort buffers and the cell-sorted points, g[1..3] own only their hash tables and alias g[0].spts
hipError_t grid_build_ladder(DevGrid* const* gp, const float* d_xyz, int n, float c0, float4* d_pts4, hipStream_t s,
                             unsigned level_mask, int min_cap, DevGrid* finer, int* zero0, int* zero1) {
    hipError_t e;
    DevGrid& g0 = *gp[0];
    bool fresh = n > g0.cap || !g0.keys || g0.alias;
    for (int L = 1; L < 4; ++L) fresh = fresh || !gp[L]->alias || gp[L]->spts != g0.spts || !gp[L]->table;
    if (finer && !fresh && (!finer->alias || finer->spts != g0.spts || !finer->table || finer->cap != g0.cap)) {
        // the finest level joins an existing ladder: its own table, the ladder's points
        grid_free(*finer, true);
        finer->cap = g0.cap;
        finer->H = pow2_at_least(2u * (unsigned)g0.cap);
        if ((e = hipMalloc(&finer->table, sizeof(CellEntry) * finer->H))) return e;
        finer->spts = g0.spts;
        finer->alias = true;
    }
    if (fresh) {
        for (int L = 0; L < 4; ++L) grid_free(*gp[L], true);
        if (finer) grid_free(*finer, true);
        g0.cap = std::max(n + n / 4 + 1024, min_cap);
        note_regrow("ladder grids", (size_t)g0.cap * 48);
        if ((e = hipMalloc(&g0.keys, sizeof(unsigned long long) * g0.cap))) return e;
        if ((e = hipMalloc(&g0.keys2, sizeof(unsigned long long) * g0.cap))) return e;
        if ((e = hipMalloc(&g0.vals, sizeof(unsigned int) * g0.cap))) return e;
        if ((e = hipMalloc(&g0.vals2, sizeof(unsigned int) * g0.cap))) return e;
        if ((e = hipMalloc(&g0.spts, sizeof(float4) * g0.cap))) return e;
        size_t tb = 0;
        if ((e = rocprim::radix_sort_pairs<LadderSortConfig>(nullptr, tb, g0.keys, g0.keys2, g0.vals, g0.vals2, (unsigned)g0.cap, 0, 63,
                                           s)))
            return e;
        g0.tmp_bytes = tb;
        if ((e = hipMalloc(&g0.tmp, tb))) return e;
        for (int L = 0; L < 4; ++L) {
            DevGrid& gl = *gp[L];
            gl.cap = g0.cap;
            gl.H = pow2_at_least(2u * (unsigned)g0.cap);
            if ((e = hipMalloc(&gl.table, sizeof(CellEntry) * gl.H))) return e;
            if (L > 0) {
                gl.spts = g0.spts;
                gl.alias = true;
            }
        }
        if (finer) {
            finer->cap = g0.cap;
            finer->H = pow2_at_least(2u * (unsigned)g0.cap);
            if ((e = hipMalloc(&finer->table, sizeof(CellEntry) * finer->H))) return e;
            finer->spts = g0.spts;
            finer->alias = true;
        }
    }
    const int B = 256;
    bsk::k_ladder_keys<<<(n + B - 1) / B, B, 0, s>>>(d_xyz, n, c0, g0.keys, g0.vals, d_pts4, bsk::ZeroWords{{zero0, zero1}});
    size_t tb = g0.tmp_bytes;
    if ((e = rocprim::radix_sort_pairs<LadderSortConfig>(g0.tmp, tb, g0.keys, g0.keys2, g0.vals, g0.vals2, (unsigned)n, 0, 63, s)))
        return e;
    // the levels' tables: one clear and one fill launch for all of them (the sorted points are
    // always scattered: the other levels alias them)
    bsk::Tables4 T;
    unsigned int hmax = 0;
    level_mask &= 0xFu;
    for (int L = 0; L < 5; ++L) {
        DevGrid* gl = L < 4 ? gp[L] : finer;
        if (!gl) {
            T.t[L] = nullptr;
            T.mask[L] = 0;
            T.H[L] = 0;
            continue;
        }
        gl->n = n;
        gl->cell = L < 4 ? c0 * (float)(1 << L) : c0 * 0.5f;
        T.t[L] = gl->table;
        T.mask[L] = gl->H - 1;
        T.H[L] = gl->H;
        if (L == 4) level_mask |= 1u << 4;
        if ((level_mask >> L) & 1u) hmax = std::max(hmax, gl->H);
    }
    if (hmax) bsk::k_grid_clear4<<<(hmax + B - 1) / B, B, 0, s>>>(T, level_mask);
    bsk::k_ladder_cells4<<<(n + B - 1) / B, B, 0, s>>>(g0.keys2, g0.vals2, d_pts4, n, c0, T, level_mask, g0.spts,
                                                        zero0);
    return hipGetLastError();
}

hipError_t grid_build(DevGrid& g, const float* d_xyz, int n, float cell, float4* d_pts4, hipStream_t s,
                      bool write_pts4, int min_cap) {
    hipError_t e;
    if (n > g.cap || g.alias || !g.keys) {
        grid_free(g, true);
        g.cap = std::max(n + n / 4 + 1024, min_cap);
        note_regrow("grid", (size_t)g.cap * 48);
        if ((e = hipMalloc(&g.keys, sizeof(unsigned long long) * g.cap))) return e;
        if ((e = hipMalloc(&g.keys2, sizeof(unsigned long long) * g.cap))) return e;
        if ((e = hipMalloc(&g.vals, sizeof(unsigned int) * g.cap))) return e;
        if ((e = hipMalloc(&g.vals2, sizeof(unsigned int) * g.cap))) return e;
        if ((e = hipMalloc(&g.spts, sizeof(float4) * g.cap))) return e;
        g.H = pow2_at_least(2u * (unsigned)g.cap);
        if ((e = hipMalloc(&g.table, sizeof(CellEntry) * g.H))) return e;
        if ((e = hipMalloc(&g.ncells, sizeof(int)))) return e;
        size_t tb = 0;
        if ((e = rocprim::radix_sort_pairs(nullptr, tb, g.keys, g.keys2, g.vals, g.vals2, (unsigned)g.cap, 0, 64, s))) return e;
        g.tmp_bytes = tb;
        if ((e = hipMalloc(&g.tmp, tb))) return e;
    }
    g.n = n;
    g.cell = cell;
    const int B = 256;
    bsk::k_grid_keys<<<(n + B - 1) / B, B, 0, s>>>(d_xyz, n, cell, g.keys, g.vals, write_pts4 ? d_pts4 : nullptr);
    size_t tb = g.tmp_bytes;
    if ((e = rocprim::radix_sort_pairs(g.tmp, tb, g.keys, g.keys2, g.vals, g.vals2, (unsigned)n, 0, 64, s))) return e;
    bsk::k_grid_clear<<<(g.H + B - 1) / B, B, 0, s>>>(g.table, g.H);
    if ((e = kfill(g.ncells, 0, sizeof(int), s))) return e;
    bsk::k_grid_cells<<<(n + B - 1) / B, B, 0, s>>>(g.keys2, g.vals2, d_pts4, n, g.table, g.H - 1, g.spts, g.ncells);
    return hipGetLastError();
}

void grid_free(DevGrid& g, bool defer) {
    if (g.alias) g.spts = nullptr;  // owned by the ladder's level-0 grid
    for (void* p : {(void*)g.keys, (void*)g.keys2, (void*)g.vals, (void*)g.vals2, (void*)g.spts, (void*)g.table,
                    (void*)g.ncells, (void*)g.tmp}) {
        if (!p) continue;
        if (defer) defer_free(p, DEFER_DEVICE);  // a regrowth inside the sweep loop
        else (void)hipFree(p);
    }
    g = DevGrid();
}


}  // namespace bsh

void flush_deferred_frees() {
    std::vector<std::pair<void*, int>> v;
    {
        std::lock_guard<std::mutex> lk(g_defer_mu);
        v.swap(g_deferred);
    }
    for (auto& e : v) {
        if (e.second == DEFER_PINNED) (void)hipHostFree(e.first);
        else (void)hipFree(e.first);
    }
}
