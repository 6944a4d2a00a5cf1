// describe.hip -- A5 neighbourhoods on gfx950 for K keypoints (PCL SHOTEstimationOMP /
// SHOTLocalReferenceFrameEstimation radius search, include/bshot_bits.h:113-135): the sorted
// (d2, idx) neighbour list of every keypoint that csrc/describe2.hip's LRF / histogram kernels read.
//
//   k_shot_count    workgroup/keypoint: |B(kp, R)| over the hashed grid + a 1024-bucket d2 histogram
//   k_desc_plan     one workgroup: segment offsets, 64-rank chunk bases, LPT order, on the device
//   k_excl_scan     one workgroup: segment offsets (host-planned describe after a plan overflow)
//   k_shot_gather_b workgroup/keypoint: neighbour indices scattered bucket-grouped (4 B each; the
//                   rank kernels rebuild the (d2 bits << 32 | idx) keys from the points)
//   k_shot_rank_wg  workgroup per keypoint: exact rank inside each bucket, span by span in LDS ->
//                   FLANN's sorted order (k_shot_rank: the wave-per-64-rank-chunk variant)
#include <hip/hip_runtime.h>

#include "bshot_math.h"
#include "dev_cand.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

#define SG_BUCKETS 1024

// the gather's key of neighbour idx of the keypoint (kx, ky, kz): d2 by for_candidates' expression
// and operands (pts4 holds the grid's coordinates), so the bits equal the ones the gather bucketed
__device__ __forceinline__ unsigned long long sg_key(const float4* __restrict__ pts4, float kx, float ky, float kz,
                                                     unsigned int idx) {
    const float4 p = pts4[idx];
    return ((unsigned long long)__float_as_uint(d2_flann(kx, ky, kz, p.x, p.y, p.z)) << 32) | idx;
}

// d2 bucket of the bucketed gather (k_shot_count/k_shot_gather_b/k_shot_rank): monotone in d2
__device__ __forceinline__ int sg_bucket(float d2, float sc) {
    int b = (int)(d2 * sc);
    return b < 0 ? 0 : (b > SG_BUCKETS - 1 ? SG_BUCKETS - 1 : b);
}

// bh (nullable): per-keypoint histogram of the in-radius d2 over SG_BUCKETS buckets, [k][SG_BUCKETS].
// A workgroup per keypoint: its 4 waves stream every 4th candidate group of the keypoint's cube
// (for_candidates' part / nparts), so a large neighbourhood takes a quarter of the dependent
// round trips (the wave-per-keypoint kernel's tail was its largest keypoint: 0.33 ms under load).
#define SG_WAVES 4
// zw (nullable): the describe's 4-int error word, zeroed here; z4 / nz: float4s zeroed across the
// grid (the new slots of the persistent normals array); cs4 -> cd4, cm float4s (the normals
// snapshot, disjoint from z4) -- the fills and the copy this launch carries
__global__ void __launch_bounds__(64 * SG_WAVES) k_shot_count(GridView g, const float* __restrict__ kps, int k, float R,
                                                             int* __restrict__ counts, unsigned int* __restrict__ bh,
                                                             int* __restrict__ zw, float4* __restrict__ z4, int nz,
                                                             float4* __restrict__ cd4, const float4* __restrict__ cs4,
                                                             int cm) {
    __shared__ CandLds lds[SG_WAVES];
    if (zw && blockIdx.x == 0 && threadIdx.x < 4) zw[threadIdx.x] = 0;
    for (int i = blockIdx.x * 64 * SG_WAVES + threadIdx.x; i < nz; i += gridDim.x * 64 * SG_WAVES)
        z4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = blockIdx.x * 64 * SG_WAVES + threadIdx.x; i < cm; i += gridDim.x * 64 * SG_WAVES) cd4[i] = cs4[i];
    __shared__ unsigned int hist[SG_BUCKETS];
    __shared__ int tot;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    cand_init(&lds[wave]);
    const float R2 = (float)((double)R * (double)R);
    const float sc = (float)SG_BUCKETS / R2;
    for (int q = blockIdx.x; q < k; q += gridDim.x) {
        const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
        if (bh)
            for (int j = threadIdx.x; j < SG_BUCKETS; j += 64 * SG_WAVES) hist[j] = 0u;
        if (threadIdx.x == 0) tot = 0;
        __syncthreads();
        int c = 0;
        if (__builtin_isfinite(kx) && __builtin_isfinite(ky) && __builtin_isfinite(kz))
            for_candidates(g, &lds[wave], kx, ky, kz, R, R2, [&](bool v, float d2, unsigned int) {
                c += __popcll(__ballot(v));
                if (bh && v) atomicAdd(&hist[sg_bucket(d2, sc)], 1u);
            }, 0, wave, SG_WAVES);
        if (lane == 0) atomicAdd(&tot, c);
        __syncthreads();
        if (bh)
            for (int j = threadIdx.x; j < SG_BUCKETS; j += 64 * SG_WAVES) bh[(size_t)q * SG_BUCKETS + j] = hist[j];
        if (threadIdx.x == 0) counts[q] = tot;
        __syncthreads();
    }
}

// Device-side describe plan (no host round trip): offs = exclusive scan of counts (segment
// starts, offs[k] = total), cb = exclusive scan of ceil(counts / 64) (chunk bases), perm = keypoints
// by descending neighbourhood size (the apply's LPT launch order; results do not depend on it). When the total or the chunk count exceed the preallocated capacities, err |= 16
// and every segment / chunk range is emptied so no later kernel writes out of bounds; the host
// then re-plans on its side. One workgroup, k <= DP_MAXK.
#define DP_MAXK 8192
__global__ void __launch_bounds__(1024) k_desc_plan(const int* __restrict__ counts, int k, long long seg_cap,
                                                    int chunk_cap, long long* __restrict__ offs, int* __restrict__ cb,
                                                    int* __restrict__ perm, int* __restrict__ err) {
    __shared__ long long ps[1024];
    __shared__ int pc[1024];
    __shared__ int bad;
    const int t = threadIdx.x;
    const int per = (k + 1023) / 1024;
    const int b = t * per, e = min(k, b + per);
    long long s = 0;
    int sc = 0;
    for (int i = b; i < e; ++i) { s += counts[i]; sc += (counts[i] + 63) / 64; }
    ps[t] = s;
    pc[t] = sc;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const long long v = t >= off ? ps[t - off] : 0;
        const int w = t >= off ? pc[t - off] : 0;
        __syncthreads();
        ps[t] += v;
        pc[t] += w;
        __syncthreads();
    }
    if (t == 0) bad = (ps[1023] > seg_cap || pc[1023] > chunk_cap) ? 1 : 0;
    __syncthreads();
    long long run = ps[t] - s;
    int runc = pc[t] - sc;
    for (int i = b; i < e; ++i) {
        offs[i] = bad ? 0 : run;
        cb[i] = bad ? 0 : runc;
        run += counts[i];
        runc += (counts[i] + 63) / 64;
    }
    if (t == 1023) {
        offs[k] = bad ? 0 : ps[1023];
        cb[k] = bad ? 0 : pc[1023];
        *reinterpret_cast<long long*>(err + 2) = ps[1023];  // err is 16-byte aligned (errw)
        if (bad) atomicOr(err, 16);
    }
    // perm: keypoints by descending neighbourhood size in 16-point buckets (a counting sort; the
    // order inside a bucket is arbitrary -- it only orders the apply launch, never the results)
    __syncthreads();
    pc[t] = 0;
    __syncthreads();
    for (int i = t; i < k; i += 1024) atomicAdd(&pc[1023 - min(1023, counts[i] >> 4)], 1);
    __syncthreads();
    const int own = pc[t];
    for (int off = 1; off < 1024; off <<= 1) {
        const int w = t >= off ? pc[t - off] : 0;
        __syncthreads();
        pc[t] += w;
        __syncthreads();
    }
    pc[t] -= own;  // exclusive bucket starts
    __syncthreads();
    for (int i = t; i < k; i += 1024) perm[atomicAdd(&pc[1023 - min(1023, counts[i] >> 4)], 1)] = i;
}

// exclusive scan of counts[0, k) by one workgroup of 1024 threads; offs[k] = total
__global__ void __launch_bounds__(1024) k_excl_scan(const int* __restrict__ counts, int k,
                                                    long long* __restrict__ offs) {
    __shared__ long long part[1024];
    const int t = threadIdx.x;
    const int per = (k + 1023) / 1024;
    const int b = t * per, e = min(k, b + per);
    long long s = 0;
    for (int i = b; i < e; ++i) s += counts[i];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const long long v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    long long run = part[t] - s;
    for (int i = b; i < e; ++i) {
        offs[i] = run;
        run += counts[i];
    }
    if (t == 1023) offs[k] = part[1023];
}

// Bucketed gather: the keys land grouped by d2 bucket (buckets ascending, any order inside a
// bucket): the workgroup scans its keypoint's bucket histogram (bh, from k_shot_count) into LDS
// cursors, writes the bucket starts (bstart, relative to the segment) for k_shot_rank, and its 4
// waves scatter the index of every in-radius neighbour of their share of the candidate groups to its
// bucket's next slot (a workgroup per keypoint, as k_shot_count). 4-byte entries: the scatter's
// partial-line writes cost 2.1 x the 8-byte keys' bytes (profiles/r05n_gather_pmc.txt), and the
// rank kernels recompute d2 from the L2-resident points instead.
// SG_STAGE > 0 (diagnostic builds): a segment of at most SG_STAGE entries is scattered into LDS
// and written out whole afterwards, coalesced; a larger one is scattered directly (the entries'
// positions are the same either way). It cuts the partial-line writes VERDICT r05 #4 measured
// (config 2: 185.6 -> 126.5 MB per launch at 8192 entries, 82.4 at 16384; config 5: 1380 -> 1233 /
// 913) and the standalone gather 0.163 -> 0.137 ms, but the 33-65 KB of LDS every workgroup then
// holds slowed config 5 by 3-4 % and left config 2 even in the pipeline (profiles/r06t_*), so the
// product scatters directly.
#ifndef SG_STAGE
#define SG_STAGE 0
#endif
__global__ void __launch_bounds__(64 * SG_WAVES) k_shot_gather_b(GridView g, const float* __restrict__ kps, int k, float R,
                                                                const long long* __restrict__ offs,
                                                                const unsigned int* __restrict__ bh,
                                                                unsigned int* __restrict__ bstart,
                                                                unsigned int* __restrict__ seg,
                                                                const int* __restrict__ err) {
    __shared__ CandLds lds[SG_WAVES];
    __shared__ unsigned int cu[SG_BUCKETS];
    __shared__ int wsum[SG_WAVES];
#if SG_STAGE > 0
    __shared__ unsigned int stg[SG_STAGE];
#endif
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    cand_init(&lds[wave]);
    const float R2 = (float)((double)R * (double)R);
    const float sc = (float)SG_BUCKETS / R2;
    constexpr int PER = SG_BUCKETS / (64 * SG_WAVES);  // buckets per thread
    if (err && (*err & 16)) return;  // device plan overflowed its capacity: the host re-plans
    for (int q = blockIdx.x; q < k; q += gridDim.x) {
        const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
        if (!(__builtin_isfinite(kx) && __builtin_isfinite(ky) && __builtin_isfinite(kz))) continue;
        // exclusive scan of the histogram: thread t owns buckets [PER t, PER t + PER)
        unsigned int hv[PER];
        int s = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            hv[j] = bh[(size_t)q * SG_BUCKETS + PER * threadIdx.x + j];
            s += (int)hv[j];
        }
        int wt;
        int run = wave_excl_scan(s, wt);
        if (lane == 0) wsum[wave] = wt;
        __syncthreads();
        for (int w = 0; w < wave; ++w) run += wsum[w];
        unsigned int ur = (unsigned int)run;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            cu[PER * threadIdx.x + j] = ur;
            bstart[(size_t)q * SG_BUCKETS + PER * threadIdx.x + j] = ur;
            ur += hv[j];
        }
        __syncthreads();
        const long long o = offs[q];
        unsigned int* out = seg + o;
#if SG_STAGE > 0
        const int n = (int)(offs[q + 1] - o);
        if (n <= SG_STAGE) {
            for_candidates(g, &lds[wave], kx, ky, kz, R, R2, [&](bool v, float d2, unsigned int idx) {
                if (v) stg[atomicAdd(&cu[sg_bucket(d2, sc)], 1u)] = idx;
            }, 0, wave, SG_WAVES);
            __syncthreads();
            for (int i = threadIdx.x; i < n; i += 64 * SG_WAVES) out[i] = stg[i];
        } else
#endif
            for_candidates(g, &lds[wave], kx, ky, kz, R, R2, [&](bool v, float d2, unsigned int idx) {
                if (v) out[atomicAdd(&cu[sg_bucket(d2, sc)], 1u)] = idx;
            }, 0, wave, SG_WAVES);
        __syncthreads();  // cu, wsum and stg are rewritten for the next keypoint
    }
}

// wave per 64-rank chunk of a bucket-grouped segment: every key's exact (d2, idx) rank inside its
// bucket -> the sorted segment, stored as the neighbour indices alone (keys are unique, buckets hold a
// few keys each; sg_key rebuilds them from the gathered indices). The buckets the chunk's keys belong
// to span [lo, hi) of the segment (the chunk plus the parts of its two end buckets outside it). The
// wave first stages the keys of a window of SR_WPRE ranks either side of the chunk (its indices and
// their points in flight together, before the bucket starts are known): a span inside it is ranked
// from there; a larger one is restaged (<= SR_STAGE keys) or ranked from HBM.
#define SR_STAGE 256
#define SR_WPRE 32
// SRK_WAVES waves per workgroup (4). 1-wave workgroups (2 KB of LDS, fitting beside SR's
// workgroups as the ICP kernels' do) measured slower: their many small workgroups slowed the main
// stream's matching 0.25 -> 0.31 ms per sweep (profiles/r06zl_ab*.txt)
#ifndef SRK_WAVES
#define SRK_WAVES 4
#endif
__global__ void __launch_bounds__(64 * SRK_WAVES) k_shot_rank(int k, float R, const float4* __restrict__ pts4,
                                                   const float* __restrict__ kps, const long long* __restrict__ offs,
                                                   const int* __restrict__ cb, const int* __restrict__ owner,
                                                   const unsigned int* __restrict__ bstart,
                                                   const unsigned int* __restrict__ seg,
                                                   unsigned int* __restrict__ out, const int4* __restrict__ cinfo) {
    __shared__ unsigned long long stage[SRK_WAVES][SR_STAGE];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    // grid-stride over chunks: a capped grid (Describe2Args::max_blocks) instead of a block per 4 chunks
    for (int c = blockIdx.x * SRK_WAVES + wave; c < cb[k]; c += gridDim.x * SRK_WAVES) [&]() {
        int q, n, c0;
        long long o;
        if (cinfo) {
            // one load: keypoint, chunk index, segment length and offset (k_chunk_owner)
            const int4 ci = cinfo[c];
            q = ci.x;
            c0 = ci.y * 64;
            n = ci.z;
            o = (long long)(unsigned int)ci.w;
        } else {
            q = owner[c];
            o = offs[q];
            n = (int)(offs[q + 1] - o);
            c0 = (c - cb[q]) * 64;
        }
        const int i = c0 + lane;
        const int last = min(n, c0 + 64) - 1;  // last valid rank of the chunk (wave-uniform)
        const float R2 = (float)((double)R * (double)R);
        const float sc = (float)SG_BUCKETS / R2;
        const unsigned int* bs = bstart + (size_t)q * SG_BUCKETS;
        const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
        const unsigned int* sg = seg + o;
        unsigned long long* st = stage[wave];
        // the window [w0, w0 + 128): both loads of every lane issued before their points
        const int w0 = c0 - SR_WPRE;
        const int pa = w0 + lane, pb = w0 + 64 + lane;
        const unsigned int ia = sg[pa < 0 ? 0 : (pa < n ? pa : n - 1)], ib = sg[pb < n ? pb : n - 1];
        const unsigned long long ka = sg_key(pts4, kx, ky, kz, ia), kb = sg_key(pts4, kx, ky, kz, ib);
        st[lane] = pa >= 0 && pa < n ? ka : ~0ull;
        st[64 + lane] = pb < n ? kb : ~0ull;
        __builtin_amdgcn_wave_barrier();
        const unsigned long long key = st[SR_WPRE + lane];  // rank i = c0 + lane (~0 past n)
        const int b = sg_bucket(__uint_as_float((unsigned int)(key >> 32)), sc);
        const int b_lo = readlane_i(b, 0), b_hi = readlane_i(b, last - c0);
        const unsigned int lo = bs[b_lo], hi = b_hi + 1 < SG_BUCKETS ? bs[b_hi + 1] : (unsigned int)n;
        unsigned int s0 = 0, e0 = 0;
        if (i < n) {
            s0 = bs[b];
            e0 = b + 1 < SG_BUCKETS ? bs[b + 1] : (unsigned int)n;
        }
        unsigned int rank = 0;
        if ((int)lo >= w0 && (int)hi <= w0 + 128) {
            if (i < n)
                for (unsigned int j = s0; j < e0; ++j) rank += st[j - w0] < key ? 1u : 0u;
        } else if (hi - lo <= SR_STAGE) {
            __builtin_amdgcn_wave_barrier();  // every lane holds its key: restage the span
            for (unsigned int j = lane; j < hi - lo; j += 64) st[j] = sg_key(pts4, kx, ky, kz, sg[lo + j]);
            __builtin_amdgcn_wave_barrier();
            if (i < n)
                for (unsigned int j = s0; j < e0; ++j) rank += st[j - lo] < key ? 1u : 0u;
        } else if (i < n) {
            for (unsigned int j = s0; j < e0; ++j) rank += sg_key(pts4, kx, ky, kz, sg[j]) < key ? 1u : 0u;
        }
        if (i < n) out[o + s0 + rank] = (unsigned int)(key & 0xFFFFFFFFu);
        __builtin_amdgcn_wave_barrier();  // the next chunk restages
    }();
}

// Workgroup per keypoint (LPT order): the keypoint's bucket-grouped segment is ordered span by span,
// a span being whole buckets holding <= RK_SPAN keys: staged in LDS with coalesced loads, then every
// key ranked inside its bucket (small buckets), or the span sorted there (bitonic; its cost does not
// grow with the bucket sizes), indices written to their sorted slots.
// Two dependent global round trips per span instead of ~5 per 64-rank chunk (owner, offsets, keys,
// bucket starts, bucket keys): the kernel streams a large neighbourhood (config 5: ~28k keys per
// keypoint) instead of waiting on it. A bucket alone larger than RK_SPAN is ranked from HBM.
#define RK_T 256
#define RK_SPAN 2048
#define RK_PER (RK_SPAN / RK_T)
// the keys of span positions [0, n) (n <= P <= RK_SPAN) into st[0, P), ~0 past n: each thread's
// index loads, then its point loads, all in flight before the first key is formed
__device__ __forceinline__ void rk_stage(unsigned long long* st, const unsigned int* __restrict__ sg, unsigned int n,
                                         int P, const float4* __restrict__ pts4, float kx, float ky, float kz) {
    const int t = threadIdx.x;
    unsigned int id[RK_PER];
#pragma unroll
    for (int j = 0; j < RK_PER; ++j) {
        const unsigned int i = t + j * RK_T;
        id[j] = sg[i < n ? i : (n ? n - 1 : 0)];  // (a span of empty buckets: n = 0, lo < the segment's end)
    }
    float4 p[RK_PER];
#pragma unroll
    for (int j = 0; j < RK_PER; ++j) p[j] = pts4[id[j]];
#pragma unroll
    for (int j = 0; j < RK_PER; ++j) {
        const int i = t + j * RK_T;
        if (i < P)
            st[i] = i < (int)n ? ((unsigned long long)__float_as_uint(d2_flann(kx, ky, kz, p[j].x, p[j].y, p[j].z)) << 32) |
                                     id[j]
                               : ~0ull;
    }
}
#ifndef RK_RANKMAX
#define RK_RANKMAX 64  // spans whose buckets all hold <= this many keys rank in place; larger ones sort
#endif
__global__ void __launch_bounds__(RK_T) k_shot_rank_wg(int k, float R, const float4* __restrict__ pts4,
                                                      const float* __restrict__ kps, const int* __restrict__ perm,
                                                      const long long* __restrict__ offs,
                                                      const unsigned int* __restrict__ bstart,
                                                      const unsigned int* __restrict__ seg,
                                                      unsigned int* __restrict__ out, unsigned int rank_max) {
    __shared__ unsigned long long st[RK_SPAN];
    __shared__ unsigned int sbs[SG_BUCKETS + 1];
    __shared__ int s_e;
    __shared__ unsigned int s_maxb;
    const int t = threadIdx.x;
    const int q = perm[blockIdx.x];
    const long long o = offs[q];
    const int n = (int)(offs[q + 1] - o);
    if (n <= 0) return;
    const float R2 = (float)((double)R * (double)R);
    const float sc = (float)SG_BUCKETS / R2;
    const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
    const unsigned int* sg = seg + o;
    unsigned int* op = out + o;
    // the bucket starts, and end(1024) = n
    for (int b = t; b < SG_BUCKETS; b += RK_T) sbs[b] = bstart[(size_t)q * SG_BUCKETS + b];
    if (t == 0) sbs[SG_BUCKETS] = (unsigned int)n;
    __syncthreads();
    int b0 = 0;
    while (true) {
        const unsigned int lo = sbs[b0];
        if (lo >= (unsigned int)n) break;
        // the span: buckets [b0, e) with e the largest bucket end within RK_SPAN keys of lo
        if (t == 0) {
            s_e = b0;
            s_maxb = 0;
        }
        __syncthreads();
        int best = b0;
        for (int e = b0 + 1 + t; e <= SG_BUCKETS; e += RK_T)
            if (sbs[e] - lo <= RK_SPAN) best = e;  // monotone in e: the per-thread max is a prefix bound
        if (best > b0) atomicMax(&s_e, best);
        __syncthreads();
        int e = s_e;
        // the span's largest bucket decides how it is ordered
        unsigned int mb = 0;
        for (int b = b0 + t; b < e; b += RK_T) mb = max(mb, sbs[b + 1] - sbs[b]);
        if (mb) atomicMax(&s_maxb, mb);
        __syncthreads();
        const bool rank_path = s_maxb <= rank_max;
        if (e == b0) {
            // bucket b0 alone exceeds the span: rank it from HBM
            const unsigned int s0 = lo, e0 = sbs[b0 + 1];
            for (unsigned int i = s0 + t; i < e0; i += RK_T) {
                const unsigned long long key = sg_key(pts4, kx, ky, kz, sg[i]);
                unsigned int rank = 0;
                for (unsigned int j = s0; j < e0; ++j) rank += sg_key(pts4, kx, ky, kz, sg[j]) < key ? 1u : 0u;
                op[s0 + rank] = (unsigned int)(key & 0xFFFFFFFFu);
            }
            e = b0 + 1;
        } else if (rank_path) {
            // small buckets: every key ranked against its bucket in LDS
            const unsigned int hi = sbs[e], m = hi - lo;
            rk_stage(st, sg + lo, m, (int)m, pts4, kx, ky, kz);
            __syncthreads();
            for (unsigned int i = t; i < m; i += RK_T) {
                const unsigned long long key = st[i];
                const int b = sg_bucket(__uint_as_float((unsigned int)(key >> 32)), sc);
                const unsigned int s0 = sbs[b] - lo, e0 = sbs[b + 1] - lo;
                unsigned int rank = 0;
                for (unsigned int j = s0; j < e0; ++j) rank += st[j] < key ? 1u : 0u;
                op[lo + s0 + rank] = (unsigned int)(key & 0xFFFFFFFFu);
            }
        } else {
            // the span holds whole buckets in bucket order, and the bucket is monotone in d2, so the
            // span sorted by (d2 bits, idx) is its slice of the keypoint's order: an LDS bitonic sort
            // (cost independent of the bucket sizes, unlike ranking each key against its bucket), then
            // coalesced index writes
            const unsigned int hi = sbs[e], m = hi - lo;
            int P = 64;
            while (P < (int)m) P <<= 1;
            rk_stage(st, sg + lo, m, P, pts4, kx, ky, kz);
            __syncthreads();
            for (int size = 2; size <= P; size <<= 1) {
                for (int stride = size >> 1; stride > 0; stride >>= 1) {
                    for (int i = t; i < P / 2; i += RK_T) {
                        const int a = 2 * i - (i & (stride - 1)), b = a + stride;
                        const bool up = (a & size) == 0;
                        const unsigned long long x = st[a], y = st[b];
                        if ((x > y) == up) {
                            st[a] = y;
                            st[b] = x;
                        }
                    }
                    __syncthreads();
                }
            }
            for (unsigned int i = t; i < m; i += RK_T) op[lo + i] = (unsigned int)(st[i] & 0xFFFFFFFFu);
        }
        __syncthreads();  // st and s_e are rewritten for the next span
        b0 = e;
        if (b0 >= SG_BUCKETS) break;
    }
}

}  // namespace bsk

namespace bsh {

hipError_t launch_shot_count(const DevGrid& g, const float* kps, int k, float R, int* counts, long long* offs,
                             hipStream_t s, unsigned int* bh) {
    if (k <= 0) return hipSuccess;
    bsk::k_shot_count<<<k, 64 * SG_WAVES, 0, s>>>(g.view(), kps, k, R, counts, bh, nullptr, nullptr, 0, nullptr,
                                                  nullptr, 0);
    bsk::k_excl_scan<<<1, 1024, 0, s>>>(counts, k, offs);
    return hipGetLastError();
}

hipError_t launch_shot_count_plan(const DevGrid& g, const float* kps, int k, float R, int* counts, unsigned int* bh,
                                  long long seg_cap, int chunk_cap, long long* offs, int* cb, int* perm, int* err,
                                  hipStream_t s, bool zero_err, float4* z4, int nz, float4* cd4, const float4* cs4,
                                  int cm) {
    if (k <= 0) return hipSuccess;
    if (k > DP_MAXK) return hipErrorInvalidValue;
#ifdef DIAG_COUNT_TWICE
    // diagnostic builds only: the count kernel twice (it overwrites its outputs) -- its marginal cost
    bsk::k_shot_count<<<k, 64 * SG_WAVES, 0, s>>>(g.view(), kps, k, R, counts, bh, nullptr, nullptr, 0, nullptr,
                                                  nullptr, 0);
#endif
    bsk::k_shot_count<<<k, 64 * SG_WAVES, 0, s>>>(g.view(), kps, k, R, counts, bh, zero_err ? err : nullptr, z4, nz,
                                                  cd4, cs4, cm);
    bsk::k_desc_plan<<<1, 1024, 0, s>>>(counts, k, seg_cap, chunk_cap, offs, cb, perm, err);
    return hipGetLastError();
}

hipError_t launch_shot_gather_b(const DevGrid& g, const float* kps, int k, float R, const long long* offs,
                                const unsigned int* bh, unsigned int* bstart, unsigned int* seg, hipStream_t s,
                                const int* err) {
    if (k <= 0) return hipSuccess;
    bsk::k_shot_gather_b<<<k, 64 * SG_WAVES, 0, s>>>(g.view(), kps, k, R, offs, bh, bstart, seg, err);
    return hipGetLastError();
}

hipError_t launch_shot_rank_wg(int k, float R, const float4* pts4, const float* kps, const int* perm,
                               const long long* offs, const unsigned int* bstart, const unsigned int* seg,
                               unsigned int* out, hipStream_t s, int rank_max) {
    if (k <= 0) return hipSuccess;
    bsk::k_shot_rank_wg<<<k, RK_T, 0, s>>>(k, R, pts4, kps, perm, offs, bstart, seg, out,
                                             rank_max < 0 ? (unsigned int)RK_RANKMAX : (unsigned int)rank_max);
    return hipGetLastError();
}

hipError_t launch_shot_rank(int k, int n_chunks, float R, const float4* pts4, const float* kps, const long long* offs,
                            const int* cb, const int* owner, const unsigned int* bstart, const unsigned int* seg,
                            unsigned int* out, hipStream_t s, const int4* cinfo, int max_blocks) {
    if (k <= 0 || n_chunks <= 0) return hipSuccess;
    int blocks = (n_chunks + SRK_WAVES - 1) / SRK_WAVES;
    // max_blocks caps the grid in 4-wave units (the chunk kernels' convention): the same waves in flight
    const int cap = max_blocks > 0 ? max_blocks * 4 / SRK_WAVES : 0;
    if (cap > 0 && blocks > cap) blocks = cap;
    bsk::k_shot_rank<<<blocks, 64 * SRK_WAVES, 0, s>>>(k, R, pts4, kps, offs, cb, owner, bstart, seg, out, cinfo);
    return hipGetLastError();
}

}  // namespace bsh
