// dev_cand.h -- wave-cooperative candidate streaming over a hashed grid + LDS bitonic sort.
//
// for_candidates(g, mark, q, rs, rs2, f): every point of every grid cell that can hold a point
// with d2 < rs^2 is visited once; f(valid, d2, idx) is called by ALL 64 lanes per chunk (valid =
// d2 < rs2). Cells of the query's cube are taken 64 per round (lane = cell; cells whose box lies
// farther than rs + 1 mm are pruned), a wave prefix sum flattens their runs, and each chunk of 64
// consecutive candidates is mapped to its cell by a max-scan over "run starts here" marks (one
// LDS write + read + 6 shuffles; no per-candidate search). Lanes then read consecutive float4s of
// the cell-sorted point array: coalesced dwordx4 loads.
#pragma once
#include <hip/hip_runtime.h>

#include "dev_common.h"

namespace bsk {

template <class F>
__device__ __forceinline__ void for_candidates(const GridView& g, int* mark, float qx, float qy, float qz, float rs,
                                               float rs2, F&& f) {
    const int lane = lane_id();
    const double c = (double)g.cell;
    const int x0 = (int)floor(((double)qx - rs) / c), x1 = (int)floor(((double)qx + rs) / c);
    const int y0 = (int)floor(((double)qy - rs) / c), y1 = (int)floor(((double)qy + rs) / c);
    const int z0 = (int)floor(((double)qz - rs) / c), z1 = (int)floor(((double)qz + rs) / c);
    const int nx = x1 - x0 + 1, ny = y1 - y0 + 1, nz = z1 - z0 + 1;
    const int ncell = nx * ny * nz;
    const double lim = (double)rs + 1.0;
    for (int base = 0; base < ncell; base += 64) {
        const int cidx = base + lane;
        unsigned int st = 0, cnt = 0;
        if (cidx < ncell) {
            const int iz = cidx % nz, t = cidx / nz, iy = t % ny, ix = t / ny;
            const int cx = x0 + ix, cy = y0 + iy, cz = z0 + iz;
            const double bx0 = cx * c, by0 = cy * c, bz0 = cz * c;
            double dx = 0, dy = 0, dz = 0;
            if (qx < bx0) dx = bx0 - qx; else if (qx > bx0 + c) dx = qx - (bx0 + c);
            if (qy < by0) dy = by0 - qy; else if (qy > by0 + c) dy = qy - (by0 + c);
            if (qz < bz0) dz = bz0 - qz; else if (qz > bz0 + c) dz = qz - (bz0 + c);
            if (dx * dx + dy * dy + dz * dz <= lim * lim) {
                if (!grid_lookup(g, cell_key(cx, cy, cz), st, cnt)) cnt = 0;
            }
        }
        int total;
        const int off = wave_excl_scan((int)cnt, total);
        if (total == 0) continue;
        const unsigned long long nonempty = __ballot(cnt > 0);
        int carry = (int)__ffsll((long long)nonempty) - 1;
        for (int t0 = 0; t0 < total; t0 += 64) {
            mark[lane] = -1;
            __builtin_amdgcn_wave_barrier();
            if (cnt > 0 && off >= t0 && off < t0 + 64) mark[off - t0] = lane;
            __builtin_amdgcn_wave_barrier();
            int m = mark[lane];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_up(m, d, 64);
                if (lane >= d) m = y > m ? y : m;
            }
            m = m > carry ? m : carry;
            carry = __shfl(m, 63, 64);
            const unsigned int cst = (unsigned int)__shfl((int)st, m, 64);
            const int coff = __shfl(off, m, 64);
            const int t = t0 + lane;
            bool valid = t < total;
            float d2 = 0.f;
            unsigned int idx = 0;
            if (valid) {
                const float4 p = g.spts[cst + (unsigned)(t - coff)];
                d2 = d2_flann(qx, qy, qz, p.x, p.y, p.z);
                idx = __float_as_uint(p.w);
                valid = d2 < rs2;
            }
            f(valid, d2, idx);
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// bitonic sort of a[0, P) ascending, P power of two, one wave
__device__ __forceinline__ void wave_bitonic(unsigned long long* a, int P) {
    const int lane = lane_id();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = lane; i < P; i += 64) {
                const int p = i ^ j;
                if (p > i) {
                    const unsigned long long x = a[i], y = a[p];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) { a[i] = y; a[p] = x; }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

}  // namespace bsk
