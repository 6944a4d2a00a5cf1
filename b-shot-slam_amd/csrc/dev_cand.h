// dev_cand.h -- wave-cooperative candidate streaming over a hashed grid + LDS bitonic sort.
//
// for_candidates(g, cs, q, rs, rs2, f): every point of every grid cell that can hold a point
// with d2 < rs^2 is visited once; f(valid, d2, idx) is called by ALL 64 lanes per chunk of 64
// candidates (valid = d2 < rs2), chunks in cell-run order. Cells of the query's cube are taken 64
// per round (lane = cell; cells whose box lies farther than rs + 1 mm are pruned), a DPP prefix
// sum flattens their runs. Candidates then go in groups of 4 chunks: every cell whose run starts
// inside the group writes a tagged mark at its start position (tags carry a per-wave epoch, so the
// marks never need clearing), each lane reads its 4 marks and a DPP max-scan gives the owning
// cell, one bpermute fetches that cell's base, and the 4 coalesced dwordx4 loads of the
// cell-sorted points are in flight together before the 4 callbacks run.
#pragma once
#include <hip/hip_runtime.h>

#include "dev_common.h"

namespace bsk {

#define CAND_GROUP 4

struct CandLds {
    int mark[64 * CAND_GROUP];
    int epoch;
    int pad_[3];
};

// once per wave before the first for_candidates on this CandLds
__device__ __forceinline__ void cand_init(CandLds* cs) {
    const int lane = lane_id();
#pragma unroll
    for (int j = 0; j < CAND_GROUP; ++j) cs->mark[lane + 64 * j] = -1;
    if (lane == 0) cs->epoch = 0;
    __builtin_amdgcn_wave_barrier();
}

template <int GROUP = CAND_GROUP, class F>
__device__ __forceinline__ void for_candidates(const GridView& g, CandLds* cs, float qx, float qy, float qz, float rs,
                                               float rs2, F&& f) {
    const int lane = lane_id();
    const double c = (double)g.cell;
    const int x0 = (int)floor(((double)qx - rs) / c), x1 = (int)floor(((double)qx + rs) / c);
    const int y0 = (int)floor(((double)qy - rs) / c), y1 = (int)floor(((double)qy + rs) / c);
    const int z0 = (int)floor(((double)qz - rs) / c), z1 = (int)floor(((double)qz + rs) / c);
    const int nx = x1 - x0 + 1, ny = y1 - y0 + 1, nz = z1 - z0 + 1;
    const int ncell = nx * ny * nz;
    const double lim = (double)rs + 1.0;
    int epoch = cs->epoch;
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
        const int cbase = (int)st - off;  // spts index of flattened candidate t is cbase(cell) + t
        const unsigned long long nonempty = __ballot(cnt > 0);
        int carry = (int)__ffsll((long long)nonempty) - 1;
        for (int t0 = 0; t0 < total; t0 += 64 * GROUP) {
            ++epoch;
            const int tag = epoch << 6;
            if (cnt > 0 && off >= t0 && off < t0 + 64 * GROUP) cs->mark[off - t0] = tag | lane;
            __builtin_amdgcn_wave_barrier();
            int owner[GROUP];
#pragma unroll
            for (int j = 0; j < GROUP; ++j) {
                const int v = cs->mark[64 * j + lane];
                owner[j] = (v & ~63) == tag ? (v & 63) : -1;
            }
#pragma unroll
            for (int j = 0; j < GROUP; ++j) {
                int m = wave_incl_max_i(owner[j]);
                m = m > carry ? m : carry;
                carry = readlane_i(m, 63);
                owner[j] = m;
            }
            float4 p[GROUP];
#pragma unroll
            for (int j = 0; j < GROUP; ++j) {
                const int cb = __builtin_amdgcn_ds_bpermute(owner[j] << 2, cbase);
                const int t = t0 + 64 * j + lane;
                p[j] = t < total ? g.spts[cb + t] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int j = 0; j < GROUP; ++j) {
                if (t0 + 64 * j < total) {
                    const int t = t0 + 64 * j + lane;
                    const float d2 = d2_flann(qx, qy, qz, p[j].x, p[j].y, p[j].z);
                    f(t < total && d2 < rs2, d2, __float_as_uint(p[j].w));
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (lane == 0) cs->epoch = epoch;
    __builtin_amdgcn_wave_barrier();
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
