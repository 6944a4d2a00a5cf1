// dev_common.h -- device-side building blocks for the gfx950 kernels of libbshot_amd.
//
// HBM layout of one hashed voxel grid (DESIGN.md "Data layout"):
//   pts4[N]     float4 (x, y, z, bits(idx)) in original index order
//   spts[N]     float4 (x, y, z, bits(idx)) sorted by (cell key, idx): every cell is one
//               contiguous, 16-B aligned run, so a wave streams a cell with coalesced dwordx4 loads
//   table[H]    open-addressed hash (H = pow2 >= 2 * #points): {u64 key, u32 start, u32 count}
// Cell key = 21-bit biased (ix, iy, iz) packed into a u64; empty slot = ~0.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BS_WAVE 64
#define BS_EMPTY_KEY 0xFFFFFFFFFFFFFFFFull

struct __attribute__((aligned(16))) CellEntry {
    unsigned long long key;
    unsigned int start;
    unsigned int count;
};

struct GridView {
    const float4* spts;       // cell-sorted points
    const CellEntry* table;   // hash table
    unsigned int mask;        // H - 1
    float cell;               // cell edge (mm)
    float inv_cell;           // 1 / cell (only used for speed-insensitive cell ranges, see cell_of)
};

// the exact-kNN radius ladder: step s searches radius r * frac[s] on grid g[gi[s]]; the last
// step is r itself (frac 1). Any radius is exact once it holds >= max_nn points.
struct LadderGrids {
    GridView g[4];
    float frac[9];
    int gi[9];
    int nsteps;
};

__device__ __forceinline__ unsigned long long cell_key(int ix, int iy, int iz) {
    return ((unsigned long long)(unsigned)(ix + (1 << 20)) << 42) | ((unsigned long long)(unsigned)(iy + (1 << 20)) << 21) |
           (unsigned long long)(unsigned)(iz + (1 << 20));
}

__device__ __forceinline__ unsigned int hash_key(unsigned long long k) {
    k ^= k >> 29;
    k *= 0xBF58476D1CE4E5B9ull;
    k ^= k >> 32;
    return (unsigned int)k;
}

// cell coordinate of a coordinate value: floor(x / cell) computed in double (matches the grid build)
__device__ __forceinline__ int cell_of(float x, float cell) { return (int)floor((double)x / (double)cell); }

__device__ __forceinline__ bool grid_lookup(const GridView& g, unsigned long long key, unsigned int& start,
                                            unsigned int& count) {
    unsigned int h = hash_key(key) & g.mask;
    for (unsigned int probe = 0; probe <= g.mask; ++probe) {
        // the whole 16-B entry in one load: key, start and count in one L2 round trip
        const uint4 e = *reinterpret_cast<const uint4*>(&g.table[h]);
        const unsigned long long k = ((unsigned long long)e.y << 32) | e.x;
        if (k == key) {
            start = e.z;
            count = e.w;
            return true;
        }
        if (k == BS_EMPTY_KEY) return false;
        h = (h + 1) & g.mask;
    }
    return false;
}

// grid_lookup split in two, so several lookups' first probes can be in flight together: the first
// probe's entry (issued by the caller), then its resolution (further probes only on a collision)
__device__ __forceinline__ uint4 grid_probe0(const GridView& g, unsigned long long key) {
    return *reinterpret_cast<const uint4*>(&g.table[hash_key(key) & g.mask]);
}
__device__ __forceinline__ bool grid_resolve(const GridView& g, unsigned long long key, uint4 e, unsigned int& start,
                                             unsigned int& count) {
    const unsigned long long k = ((unsigned long long)e.y << 32) | e.x;
    if (k == key) {
        start = e.z;
        count = e.w;
        return true;
    }
    if (k == BS_EMPTY_KEY) return false;
    unsigned int h = ((hash_key(key) & g.mask) + 1) & g.mask;
    for (unsigned int probe = 1; probe <= g.mask; ++probe) {
        const uint4 f = *reinterpret_cast<const uint4*>(&g.table[h]);
        const unsigned long long kf = ((unsigned long long)f.y << 32) | f.x;
        if (kf == key) {
            start = f.z;
            count = f.w;
            return true;
        }
        if (kf == BS_EMPTY_KEY) return false;
        h = (h + 1) & g.mask;
    }
    return false;
}

// FLANN L2_Simple squared distance in float: ((dx*dx + dy*dy) + dz*dz), dx = q - p (no FMA:
// the library is built with -ffp-contract=off).
__device__ __forceinline__ float d2_flann(float qx, float qy, float qz, float px, float py, float pz) {
    const float dx = qx - px, dy = qy - py, dz = qz - pz;
    return (dx * dx + dy * dy) + dz * dz;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// ---- wave-wide scans on DPP (no LDS round trip): Hillis-Steele inside each 16-lane row
// (row_shr 1, 2, 4, 8), then row_bcast:15 into rows 1/3 and row_bcast:31 into rows 2/3.
// Lanes whose DPP source lies outside the row read the identity. Call from converged code.
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_i(int identity, int v) {
    return __builtin_amdgcn_update_dpp(identity, v, CTRL, ROWS, 0xf, false);
}

__device__ __forceinline__ int wave_incl_add_i(int v) {
    v += dpp_i<0x111, 0xf>(0, v);
    v += dpp_i<0x112, 0xf>(0, v);
    v += dpp_i<0x114, 0xf>(0, v);
    v += dpp_i<0x118, 0xf>(0, v);
    v += dpp_i<0x142, 0xa>(0, v);
    v += dpp_i<0x143, 0xc>(0, v);
    return v;
}

__device__ __forceinline__ int wave_incl_max_i(int v) {
    const int I = -2147483647 - 1;
    v = max(v, dpp_i<0x111, 0xf>(I, v));
    v = max(v, dpp_i<0x112, 0xf>(I, v));
    v = max(v, dpp_i<0x114, 0xf>(I, v));
    v = max(v, dpp_i<0x118, 0xf>(I, v));
    v = max(v, dpp_i<0x142, 0xa>(I, v));
    v = max(v, dpp_i<0x143, 0xc>(I, v));
    return v;
}

__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// wave-wide exclusive prefix sum of an int (64 lanes); total = sum over the wave (uniform)
__device__ __forceinline__ int wave_excl_scan(int v, int& total) {
    const int x = wave_incl_add_i(v);
    total = readlane_i(x, 63);
    return x - v;
}

__device__ __forceinline__ int wave_sum_i(int v) { return readlane_i(wave_incl_add_i(v), 63); }

// the value of lane (lane ^ OFF), without the LDS crossbar (ds_bpermute): gfx950's
// v_permlane32/16_swap for the cross-row offsets, DPP row rotate / shifts / quad permutes inside a row
template <int OFF>
__device__ __forceinline__ unsigned int xor_lane_u32(unsigned int v) {
    const int lane = lane_id();
    if constexpr (OFF == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // {lanes 32..63 <- 0..31, 0..31 <- 32..63}
        return (lane & 32) ? r[0] : r[1];
    } else if constexpr (OFF == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // odd rows <- even rows and back
        return (lane & 16) ? r[0] : r[1];
    } else if constexpr (OFF == 8) {
        return (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (OFF == 4) {
        const unsigned int up = (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0xF, false);  // row_shl:4
        const unsigned int dn = (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
        return (lane & 4) ? dn : up;
    } else if constexpr (OFF == 2) {
        return (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else {
        static_assert(OFF == 1, "xor offsets 32, 16, 8, 4, 2, 1");
        return (unsigned int)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    }
}

template <int OFF>
__device__ __forceinline__ unsigned long long xor_lane_u64(unsigned long long v) {
    const unsigned int lo = xor_lane_u32<OFF>((unsigned int)v), hi = xor_lane_u32<OFF>((unsigned int)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

template <int OFF>
__device__ __forceinline__ double xor_lane_d(double v) {
    return __longlong_as_double((long long)xor_lane_u64<OFF>((unsigned long long)__double_as_longlong(v)));
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
    unsigned long long o;
    o = xor_lane_u64<32>(v); v = o < v ? o : v;
    o = xor_lane_u64<16>(v); v = o < v ? o : v;
    o = xor_lane_u64<8>(v); v = o < v ? o : v;
    o = xor_lane_u64<4>(v); v = o < v ? o : v;
    o = xor_lane_u64<2>(v); v = o < v ? o : v;
    o = xor_lane_u64<1>(v); v = o < v ? o : v;
    return v;
}

// pairwise butterfly sum with a FIXED tree (lane 0's association: partner = lane ^ off,
// off = 32, 16, ..., 1). Documented convention for the LRF covariance.
__device__ __forceinline__ double wave_tree_sum_d(double v) {
    v = v + xor_lane_d<32>(v);
    v = v + xor_lane_d<16>(v);
    v = v + xor_lane_d<8>(v);
    v = v + xor_lane_d<4>(v);
    v = v + xor_lane_d<2>(v);
    v = v + xor_lane_d<1>(v);
    return v;
}

// diagnostic cycle stamp (debug counters only; never on the product path)
__device__ __forceinline__ unsigned long long cycle_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__device__ __forceinline__ unsigned int f2u(float f) { return __float_as_uint(f); }
