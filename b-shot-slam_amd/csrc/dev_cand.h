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

#ifndef CAND_GROUP
#define CAND_GROUP 4
#endif

// marks are 16-bit: (epoch << 6) | lane with a 10-bit epoch in 1 .. 1023; 0 is never a tag, so the
// marks are cleared to 0 when the epoch wraps (every 1023 candidate groups)
#define CAND_EPOCHS 1024
struct CandLds {
    unsigned short mark[64 * CAND_GROUP];
    int epoch;
    int pad_[3];
};

__device__ __forceinline__ void cand_clear_marks(CandLds* cs) {
    const int lane = lane_id();
#pragma unroll
    for (int j = 0; j < CAND_GROUP; ++j) cs->mark[lane + 64 * j] = 0;
    __builtin_amdgcn_wave_barrier();
}

// once per wave before the first for_candidates on this CandLds
__device__ __forceinline__ void cand_init(CandLds* cs) {
    cand_clear_marks(cs);
    if (lane_id() == 0) cs->epoch = 0;
    __builtin_amdgcn_wave_barrier();
}

// streams the candidates of one 64-cell round (lane = cell: spts run [st, st + cnt), off = its
// exclusive prefix among the round's runs, total = their sum). nparts > 1: only the groups
// g = part, part + nparts, ... (the waves of a workgroup share one query's candidates); each
// group's first owner then comes from the runs directly instead of the previous group.
template <int GROUP, class F>
__device__ __forceinline__ void cand_stream_round(const GridView& g, CandLds* cs, int& epoch, float qx, float qy,
                                                  float qz, float rs2, unsigned int st, unsigned int cnt, int off,
                                                  int total, F& f, int part = 0, int nparts = 1) {
    static_assert(GROUP >= 1 && GROUP <= CAND_GROUP, "CandLds::mark holds CAND_GROUP chunks of marks");
    const int lane = lane_id();
    const int cbase = (int)st - off;  // spts index of flattened candidate t is cbase(cell) + t
    const unsigned long long nonempty = __ballot(cnt > 0);
    int carry = (int)__ffsll((long long)nonempty) - 1;
    for (int t0 = part * 64 * GROUP; t0 < total; t0 += 64 * GROUP * nparts) {
        if (nparts > 1) {
            // the non-empty run holding position t0: the last one starting at or before it
            const unsigned long long started = __ballot(cnt > 0 && off <= t0);
            carry = 63 - __clzll((long long)started);
        }
        if (++epoch == CAND_EPOCHS) {
            cand_clear_marks(cs);  // wave-uniform, once per 1023 groups
            epoch = 1;
        }
        const int tag = epoch << 6;
        if (cnt > 0 && off >= t0 && off < t0 + 64 * GROUP) cs->mark[off - t0] = (unsigned short)(tag | lane);
        __builtin_amdgcn_wave_barrier();
        int owner[GROUP];
#pragma unroll
        for (int j = 0; j < GROUP; ++j) {
            const int v = (int)cs->mark[64 * j + lane];
            owner[j] = (v & ~63) == tag ? (v & 63) : -1;
        }
#pragma unroll
        for (int j = 0; j < GROUP; ++j) {
            int m = wave_incl_max_i(owner[j]);
            m = m > carry ? m : carry;
            carry = readlane_i(m, 63);
            owner[j] = m;
        }
        // the owners' run bases first, then all GROUP loads unconditionally (a lane past the total
        // reads spts[0] and is masked by the validity flag): a load under a branch made the
        // compiler wait for each one before issuing the next, serialising GROUP L2 round trips
        int cb[GROUP];
#pragma unroll
        for (int j = 0; j < GROUP; ++j) cb[j] = __builtin_amdgcn_ds_bpermute(owner[j] << 2, cbase);
        float4 p[GROUP];
#pragma unroll
        for (int j = 0; j < GROUP; ++j) {
            const int t = t0 + 64 * j + lane;
            p[j] = g.spts[t < total ? cb[j] + t : 0];
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

// lane's cell of round `base` of the query cube: its spts run (cnt = 0 when pruned or empty). The
// cube and the pruning only decide which cells are visited, never which points count (every
// candidate is tested d2 < rs^2), so they run in float with a slack that covers float rounding:
// lim = rs + slack (cand_slack; a conservative cube: never a cell with an in-ball point left out).
// rnz, rny: 1 / nz, 1 / ny (the cell index splits by float reciprocals: exact for these small
// integers with the +0.5 bias, and no integer division sequence per lane)
// lane's cell of round `base` of the query cube: its key, and whether it can hold an in-ball point
// (in the cube and its box within lim of the query)
__device__ __forceinline__ bool cand_cell(const GridView& g, int x0, int y0, int z0, int ny, int nz, float rny,
                                          float rnz, int ncell, int cidx, float qx, float qy, float qz, float lim,
                                          unsigned long long& key) {
    key = BS_EMPTY_KEY;
    if (cidx >= ncell) return false;
    const int t = (int)(((float)cidx + 0.5f) * rnz), iz = cidx - t * nz;
    const int ix = (int)(((float)t + 0.5f) * rny), iy = t - ix * ny;
    const int cx = x0 + ix, cy = y0 + iy, cz = z0 + iz;
    const float c = g.cell;
    const float bx0 = (float)cx * c, by0 = (float)cy * c, bz0 = (float)cz * c;
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (qx < bx0) dx = bx0 - qx; else if (qx > bx0 + c) dx = qx - (bx0 + c);
    if (qy < by0) dy = by0 - qy; else if (qy > by0 + c) dy = qy - (by0 + c);
    if (qz < bz0) dz = bz0 - qz; else if (qz > bz0 + c) dz = qz - (bz0 + c);
    if (!(dx * dx + dy * dy + dz * dz <= lim * lim)) return false;
    key = cell_key(cx, cy, cz);
    return true;
}

// lane's cell of round `base` of the query cube: its spts run (cnt = 0 when pruned or empty). The
// cube and the pruning only decide which cells are visited, never which points count (every
// candidate is tested d2 < rs^2), so they run in float with a slack that covers float rounding:
// lim = rs + slack (cand_slack; a conservative cube: never a cell with an in-ball point left out).
// rnz, rny: 1 / nz, 1 / ny (the cell index splits by float reciprocals: exact for these small
// integers with the +0.5 bias, and no integer division sequence per lane)
__device__ __forceinline__ void cand_lookup(const GridView& g, int x0, int y0, int z0, int ny, int nz, float rny,
                                            float rnz, int ncell, int cidx, float qx, float qy, float qz, float lim,
                                            unsigned int& st, unsigned int& cnt) {
    st = 0;
    cnt = 0;
    unsigned long long key;
    if (cand_cell(g, x0, y0, z0, ny, nz, rny, rnz, ncell, cidx, qx, qy, qz, lim, key))
        if (!grid_lookup(g, key, st, cnt)) cnt = 0;
}

// the float slack of a query's cube (see cand_lookup): 2^-20 of the query's magnitude (16 ulps of
// its largest coordinate, far above the rounding of the cube bounds and box distances) + 0.05 mm. A
// 1 mm slack streamed 4.5 % more candidates (cells whose face lies within 1 mm outside the ball).
__device__ __forceinline__ float cand_slack(float qx, float qy, float qz) {
    return 0.05f + fmaxf(fabsf(qx), fmaxf(fabsf(qy), fabsf(qz))) * 9.5367431640625e-07f;  // 2^-20
}

// Returns false (and streams nothing) when the cube holds fewer than min_total candidates -- the
// ball then holds fewer too. Cubes of <= 128 cells do all their lookups before streaming.
// part / nparts: this wave streams only its share of the candidate groups (see cand_stream_round);
// every wave of the share does the cell lookups itself.
template <int GROUP = CAND_GROUP, class F>
__device__ __forceinline__ bool for_candidates(const GridView& g, CandLds* cs, float qx, float qy, float qz, float rs,
                                               float rs2, F&& f, int min_total = 0, int part = 0, int nparts = 1) {
    const int lane = lane_id();
    const float ic = g.inv_cell, lim = rs + cand_slack(qx, qy, qz);
    const int x0 = (int)floorf((qx - lim) * ic), x1 = (int)floorf((qx + lim) * ic);
    const int y0 = (int)floorf((qy - lim) * ic), y1 = (int)floorf((qy + lim) * ic);
    const int z0 = (int)floorf((qz - lim) * ic), z1 = (int)floorf((qz + lim) * ic);
    const int nx = x1 - x0 + 1, ny = y1 - y0 + 1, nz = z1 - z0 + 1;
    const int ncell = nx * ny * nz;
    const float rny = 1.f / (float)ny, rnz = 1.f / (float)nz;
    int epoch = cs->epoch;
    bool streamed = true;
    if (ncell <= 128) {
        // both rounds' first probes in flight together, then their resolution
        unsigned int st0 = 0, cnt0 = 0, st1 = 0, cnt1 = 0;
        unsigned long long k0, k1;
        const bool w0 = cand_cell(g, x0, y0, z0, ny, nz, rny, rnz, ncell, lane, qx, qy, qz, lim, k0);
        const bool w1 = cand_cell(g, x0, y0, z0, ny, nz, rny, rnz, ncell, 64 + lane, qx, qy, qz, lim, k1);
        const uint4 e0 = grid_probe0(g, w0 ? k0 : 0ull);
        const uint4 e1 = grid_probe0(g, w1 ? k1 : 0ull);
        if (w0 && !grid_resolve(g, k0, e0, st0, cnt0)) cnt0 = 0;
        if (w1 && !grid_resolve(g, k1, e1, st1, cnt1)) cnt1 = 0;
        int tot0, tot1 = 0;
        const int off0 = wave_excl_scan((int)cnt0, tot0);
        const int off1 = ncell > 64 ? wave_excl_scan((int)cnt1, tot1) : 0;
        if (tot0 + tot1 < min_total) {
            streamed = false;
        } else {
#pragma unroll 1
            for (int r = 0; r < 2; ++r) {
                const int tot = r ? tot1 : tot0;
                if (tot > 0)
                    cand_stream_round<GROUP>(g, cs, epoch, qx, qy, qz, rs2, r ? st1 : st0, r ? cnt1 : cnt0,
                                             r ? off1 : off0, tot, f, part, nparts);
            }
        }
    } else {
        for (int base = 0; base < ncell; base += 64) {
            unsigned int st, cnt;
            cand_lookup(g, x0, y0, z0, ny, nz, rny, rnz, ncell, base + lane, qx, qy, qz, lim, st, cnt);
            int total;
            const int off = wave_excl_scan((int)cnt, total);
            if (total == 0) continue;
            cand_stream_round<GROUP>(g, cs, epoch, qx, qy, qz, rs2, st, cnt, off, total, f, part, nparts);
        }
    }
    if (lane == 0) cs->epoch = epoch;
    __builtin_amdgcn_wave_barrier();
    return streamed;
}

// bitonic sort of a[0, P) ascending, P power of two, one wave
__device__ __forceinline__ void wave_bitonic(unsigned long long* a, int P) {
    const int lane = lane_id();
    // kept rolled: where a caller bounds P (icp_build_list) the unrolled stages cost its kernel ~40
    // VGPRs and a scratch spill
#pragma unroll 1
    for (int k = 2; k <= P; k <<= 1) {
#pragma unroll 1
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
