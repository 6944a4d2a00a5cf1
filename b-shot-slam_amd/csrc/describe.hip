// describe.hip -- A5-A7 on gfx950: SHOT local reference frame, 352-bin SHOT histogram and B-SHOT
// binarisation for K keypoints (replaces include/bshot_bits.h:113-278, i.e. PCL
// SHOTEstimationOMP + SHOTLocalReferenceFrameEstimation + compute_bshot_from_SHOT).
//
// Pipeline (all on the context stream):
//   k_shot_count   wave/keypoint: |B(kp, R)| over the hashed grid
//   k_excl_scan    single workgroup: per-keypoint segment offsets (+ total)
//   k_shot_gather  wave/keypoint: u64 keys (d2bits<<32 | idx) of all neighbours -> segment
//   k_shot_sort    workgroup/keypoint: 1024-bucket counting sort on d2 + exact rank inside each
//                  bucket -> segment sorted by (d2, idx) (FLANN sorted radius-search order)
//   k_lrf          workgroup/keypoint: weighted covariance (double; per-64 chunk butterfly tree,
//                  chunks summed in rank order -- DESIGN.md convention), Jacobi eigensolve,
//                  PCL sign disambiguation (count rule + median-5 rule)
//   k_shot_hist    wave/keypoint: per-neighbour quadrilinear contributions computed in parallel
//                  (double math, fdlibm acos/atan2), applied to the LDS histogram in rank order
//                  (ds_add_f32 from one wave executes in issue order: identical float sums to the
//                  sequential PCL loop), L2 normalisation, B-SHOT bits.
#include <hip/hip_runtime.h>

#include "bshot_math.h"
#include "dev_cand.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

#define SB_BUCKETS 1024
#define SG_BUCKETS 1024

// d2 bucket of the bucketed gather (k_shot_count/k_shot_gather_b/k_shot_rank): monotone in d2
__device__ __forceinline__ int sg_bucket(float d2, float sc) {
    int b = (int)(d2 * sc);
    return b < 0 ? 0 : (b > SG_BUCKETS - 1 ? SG_BUCKETS - 1 : b);
}

// bh (nullable): per-keypoint histogram of the in-radius d2 over SG_BUCKETS buckets, [k][SG_BUCKETS]
__global__ void __launch_bounds__(256) k_shot_count(GridView g, const float* __restrict__ kps, int k, float R,
                                                    int* __restrict__ counts, unsigned int* __restrict__ bh) {
    __shared__ CandLds lds[4];
    __shared__ unsigned int hist[4][SG_BUCKETS];
    const int wave = threadIdx.x >> 6, lane = lane_id();
    cand_init(&lds[wave]);
    const float R2 = (float)((double)R * (double)R);
    const float sc = (float)SG_BUCKETS / R2;
    unsigned int* h = hist[wave];
    for (int q = blockIdx.x * 4 + wave; q < k; q += gridDim.x * 4) {
        const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
        if (bh) {
            for (int j = lane; j < SG_BUCKETS; j += 64) h[j] = 0u;
            __builtin_amdgcn_wave_barrier();
        }
        int c = 0;
        if (__builtin_isfinite(kx) && __builtin_isfinite(ky) && __builtin_isfinite(kz))
            for_candidates(g, &lds[wave], kx, ky, kz, R, R2, [&](bool v, float d2, unsigned int) {
                c += __popcll(__ballot(v));
                if (bh && v) atomicAdd(&h[sg_bucket(d2, sc)], 1u);
            });
        if (bh) {
            __builtin_amdgcn_wave_barrier();
            for (int j = lane; j < SG_BUCKETS; j += 64) bh[(size_t)q * SG_BUCKETS + j] = h[j];
        }
        if (lane == 0) counts[q] = c;
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

__global__ void __launch_bounds__(256) k_shot_gather(GridView g, const float* __restrict__ kps, int k, float R,
                                                     const long long* __restrict__ offs,
                                                     unsigned long long* __restrict__ seg) {
    __shared__ CandLds lds[4];
    const int wave = threadIdx.x >> 6;
    cand_init(&lds[wave]);
    const float R2 = (float)((double)R * (double)R);
    for (int q = blockIdx.x * 4 + wave; q < k; q += gridDim.x * 4) {
        const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
        if (!(__builtin_isfinite(kx) && __builtin_isfinite(ky) && __builtin_isfinite(kz))) continue;
        unsigned long long* out = seg + offs[q];
        int cnt = 0;
        for_candidates(g, &lds[wave], kx, ky, kz, R, R2, [&](bool v, float d2, unsigned int idx) {
            const unsigned long long m = __ballot(v);
            if (v) {
                const int slot = cnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                out[slot] = ((unsigned long long)__float_as_uint(d2) << 32) | idx;
            }
            cnt += __popcll(m);
        });
    }
}

// Bucketed gather: the keys land grouped by d2 bucket (buckets ascending, any order inside a
// bucket): each wave scans its keypoint's bucket histogram (bh, from k_shot_count) into LDS
// cursors, writes the bucket starts (bstart, relative to the segment) for k_shot_rank, and
// scatters every in-radius key to its bucket's next slot.
__global__ void __launch_bounds__(256) k_shot_gather_b(GridView g, const float* __restrict__ kps, int k, float R,
                                                       const long long* __restrict__ offs,
                                                       const unsigned int* __restrict__ bh,
                                                       unsigned int* __restrict__ bstart,
                                                       unsigned long long* __restrict__ seg,
                                                       const int* __restrict__ err) {
    __shared__ CandLds lds[4];
    __shared__ unsigned int cur[4][SG_BUCKETS];
    const int wave = threadIdx.x >> 6, lane = lane_id();
    cand_init(&lds[wave]);
    const float R2 = (float)((double)R * (double)R);
    const float sc = (float)SG_BUCKETS / R2;
    unsigned int* cu = cur[wave];
    constexpr int PER = SG_BUCKETS / 64;
    if (err && (*err & 16)) return;  // device plan overflowed its capacity: the host re-plans
    for (int q = blockIdx.x * 4 + wave; q < k; q += gridDim.x * 4) {
        const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
        if (!(__builtin_isfinite(kx) && __builtin_isfinite(ky) && __builtin_isfinite(kz))) continue;
        // exclusive scan of the histogram: lane owns buckets [PER lane, PER lane + PER)
        unsigned int hv[PER];
        int s = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            hv[j] = bh[(size_t)q * SG_BUCKETS + PER * lane + j];
            s += (int)hv[j];
        }
        int tot;
        unsigned int run = (unsigned int)wave_excl_scan(s, tot);
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            cu[PER * lane + j] = run;
            bstart[(size_t)q * SG_BUCKETS + PER * lane + j] = run;
            run += hv[j];
        }
        __builtin_amdgcn_wave_barrier();
        unsigned long long* out = seg + offs[q];
        for_candidates(g, &lds[wave], kx, ky, kz, R, R2, [&](bool v, float d2, unsigned int idx) {
            if (v) out[atomicAdd(&cu[sg_bucket(d2, sc)], 1u)] = ((unsigned long long)__float_as_uint(d2) << 32) | idx;
        });
        __builtin_amdgcn_wave_barrier();
    }
}

// wave per 64-rank chunk of a bucket-grouped segment: every key's exact (d2, idx) rank inside its
// bucket -> the sorted segment (keys are unique, buckets hold a few keys each). The buckets the
// chunk's keys belong to span [lo, hi) of the segment (the chunk plus the parts of its two end
// buckets outside it); when that fits SR_STAGE keys it is staged in LDS and ranked from there.
#define SR_STAGE 256
__global__ void __launch_bounds__(256) k_shot_rank(int k, float R, const long long* __restrict__ offs,
                                                   const int* __restrict__ cb, const int* __restrict__ owner,
                                                   const unsigned int* __restrict__ bstart,
                                                   const unsigned long long* __restrict__ seg,
                                                   unsigned long long* __restrict__ out) {
    __shared__ unsigned long long stage[4][SR_STAGE];
    const int wave = threadIdx.x >> 6, lane = lane_id();
    // grid-stride over chunks: a capped grid (Describe2Args::max_blocks) instead of a block per 4 chunks
    for (int c = blockIdx.x * 4 + wave; c < cb[k]; c += gridDim.x * 4) [&]() {
        const int q = owner[c];
        const long long o = offs[q];
        const int n = (int)(offs[q + 1] - o);
        const int c0 = (c - cb[q]) * 64;
        const int i = c0 + lane;
        const int last = min(n, c0 + 64) - 1;  // last valid rank of the chunk (wave-uniform)
        const float R2 = (float)((double)R * (double)R);
        const float sc = (float)SG_BUCKETS / R2;
        const unsigned int* bs = bstart + (size_t)q * SG_BUCKETS;
        const unsigned long long* sg = seg + o;
        const unsigned long long key = i < n ? sg[i] : ~0ull;
        const int b = sg_bucket(__uint_as_float((unsigned int)(key >> 32)), sc);
        const int b_lo = readlane_i(b, 0), b_hi = readlane_i(b, last - c0);
        const unsigned int lo = bs[b_lo], hi = b_hi + 1 < SG_BUCKETS ? bs[b_hi + 1] : (unsigned int)n;
        unsigned int s0 = 0, e0 = 0;
        if (i < n) {
            s0 = bs[b];
            e0 = b + 1 < SG_BUCKETS ? bs[b + 1] : (unsigned int)n;
        }
        unsigned int rank = 0;
        if (hi - lo <= SR_STAGE) {
            unsigned long long* st = stage[wave];
            for (unsigned int j = lane; j < hi - lo; j += 64) st[j] = sg[lo + j];
            __builtin_amdgcn_wave_barrier();
            if (i < n)
                for (unsigned int j = s0; j < e0; ++j) rank += st[j - lo] < key ? 1u : 0u;
        } else if (i < n) {
            for (unsigned int j = s0; j < e0; ++j) rank += sg[j] < key ? 1u : 0u;
        }
        if (i < n) out[o + s0 + rank] = key;
        __builtin_amdgcn_wave_barrier();  // the next chunk restages
    }();
}

// counting sort of one keypoint's segment by d2 bucket, then exact rank inside the bucket
__global__ void __launch_bounds__(256) k_shot_sort(const long long* __restrict__ offs, int k, float R,
                                                   unsigned long long* __restrict__ seg,
                                                   unsigned long long* __restrict__ tmp) {
    __shared__ unsigned int hist[SB_BUCKETS];
    __shared__ unsigned int boff[SB_BUCKETS];
    __shared__ unsigned int cur[SB_BUCKETS];
    __shared__ unsigned int wsum[4];
    const float R2 = (float)((double)R * (double)R);
    const float sc = (float)SB_BUCKETS / R2;
    const int t = threadIdx.x;
    for (int q = blockIdx.x; q < k; q += gridDim.x) {
        const long long o = offs[q];
        const int n = (int)(offs[q + 1] - o);
        if (n <= 1) continue;
        unsigned long long* a = seg + o;
        unsigned long long* b = tmp + o;
        for (int i = t; i < SB_BUCKETS; i += 256) hist[i] = 0;
        __syncthreads();
        for (int i = t; i < n; i += 256) {
            const float d2 = __uint_as_float((unsigned)(a[i] >> 32));
            int bk = (int)(d2 * sc);
            bk = bk < 0 ? 0 : (bk > SB_BUCKETS - 1 ? SB_BUCKETS - 1 : bk);
            atomicAdd(&hist[bk], 1u);
        }
        __syncthreads();
        // exclusive scan of 1024 buckets: 4 per thread
        unsigned int s4 = hist[4 * t] + hist[4 * t + 1] + hist[4 * t + 2] + hist[4 * t + 3];
        int tot;
        const int ex = wave_excl_scan((int)s4, tot);
        if (lane_id() == 63) wsum[t >> 6] = (unsigned)tot;
        __syncthreads();
        unsigned int base = 0;
        for (int w = 0; w < (t >> 6); ++w) base += wsum[w];
        unsigned int run = base + (unsigned)ex;
        for (int j = 0; j < 4; ++j) {
            boff[4 * t + j] = run;
            cur[4 * t + j] = run;
            run += hist[4 * t + j];
        }
        __syncthreads();
        for (int i = t; i < n; i += 256) {
            const unsigned long long key = a[i];
            const float d2 = __uint_as_float((unsigned)(key >> 32));
            int bk = (int)(d2 * sc);
            bk = bk < 0 ? 0 : (bk > SB_BUCKETS - 1 ? SB_BUCKETS - 1 : bk);
            const unsigned int pos = atomicAdd(&cur[bk], 1u);
            b[pos] = key;
        }
        __syncthreads();
        for (int i = t; i < n; i += 256) {
            const unsigned long long key = b[i];
            const float d2 = __uint_as_float((unsigned)(key >> 32));
            int bk = (int)(d2 * sc);
            bk = bk < 0 ? 0 : (bk > SB_BUCKETS - 1 ? SB_BUCKETS - 1 : bk);
            const unsigned int s0 = boff[bk], c = hist[bk];
            unsigned int rank = 0;
            for (unsigned int j = 0; j < c; ++j) rank += b[s0 + j] < key ? 1u : 0u;
            a[s0 + rank] = key;
        }
        __syncthreads();
    }
}

// LRF: one workgroup (4 waves) per keypoint. Output rf row-major (x axis, y axis, z axis) and
// ok flag (0 -> NaN LRF).
__global__ void __launch_bounds__(256) k_lrf(const float4* __restrict__ pts4, const float* __restrict__ kps, int k,
                                             float R, const long long* __restrict__ offs,
                                             const unsigned long long* __restrict__ seg, float* __restrict__ rf_out,
                                             int* __restrict__ ok_out) {
    __shared__ double csum[4][8];
    __shared__ double tot[8];
    __shared__ int vcnt[4];
    __shared__ double evs[9];
    __shared__ int okflag;
    const int t = threadIdx.x, wave = t >> 6, lane = lane_id();
    const double Rd = (double)R;
    for (int q = blockIdx.x; q < k; q += gridDim.x) {
        const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
        const long long o = offs[q];
        const int n = (int)(offs[q + 1] - o);
        const unsigned long long* a = seg + o;
        if (t < 8) tot[t] = 0.0;
        int valid_total = 0;
        __syncthreads();
        const int nch = (n + 63) >> 6;
        for (int c0 = 0; c0 < nch; c0 += 4) {
            const int c = c0 + wave;
            double v[7] = {0, 0, 0, 0, 0, 0, 0};
            int isv = 0;
            if (c < nch) {
                const int i = c * 64 + lane;
                if (i < n) {
                    const unsigned long long key = a[i];
                    const float4 p = pts4[(unsigned)(key & 0xFFFFFFFFu)];
                    if (!(p.x == kx && p.y == ky && p.z == kz)) {
                        const double vx = (double)(p.x - kx), vy = (double)(p.y - ky), vz = (double)(p.z - kz);
                        const double w = Rd - sqrt((double)__uint_as_float((unsigned)(key >> 32)));
                        v[0] = w * (vx * vx); v[1] = w * (vx * vy); v[2] = w * (vx * vz);
                        v[3] = w * (vy * vy); v[4] = w * (vy * vz); v[5] = w * (vz * vz);
                        v[6] = w;
                        isv = 1;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 7; ++j) v[j] = wave_tree_sum_d(v[j]);
            const int nv = __popcll(__ballot(isv != 0));
            if (lane == 0) {
#pragma unroll
                for (int j = 0; j < 7; ++j) csum[wave][j] = v[j];
                vcnt[wave] = nv;
            }
            __syncthreads();
            if (t < 7) {
                double acc = tot[t];
                for (int w = 0; w < 4 && c0 + w < nch; ++w) acc = acc + csum[w][t];
                tot[t] = acc;
            }
            for (int w = 0; w < 4 && c0 + w < nch; ++w) valid_total += vcnt[w];
            __syncthreads();
        }
        if (t == 0) {
            okflag = 0;
            if (valid_total >= 5) {
                const double sum = tot[6];
                double cov[9];
                cov[0] = tot[0] / sum; cov[1] = tot[1] / sum; cov[2] = tot[2] / sum;
                cov[4] = tot[3] / sum; cov[5] = tot[4] / sum; cov[8] = tot[5] / sum;
                cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
                double w[3], ev[9];
                bm::jacobi3(cov, w, ev);
                if (bm::isfin(w[0]) && bm::isfin(w[1]) && bm::isfin(w[2])) {
                    okflag = 1;
                    for (int j = 0; j < 9; ++j) evs[j] = ev[j];
                }
            }
        }
        __syncthreads();
        if (okflag) {
            const double v1x = evs[2], v1y = evs[5], v1z = evs[8];  // largest -> x axis
            const double v3x = evs[0], v3y = evs[3], v3z = evs[6];  // smallest -> z axis
            int pt = 0, pn = 0;
            for (int i = t; i < n; i += 256) {
                const unsigned long long key = a[i];
                const float4 p = pts4[(unsigned)(key & 0xFFFFFFFFu)];
                if (!(p.x == kx && p.y == ky && p.z == kz)) {
                    const double vx = (double)(p.x - kx), vy = (double)(p.y - ky), vz = (double)(p.z - kz);
                    if (((vx * v1x + vy * v1y) + vz * v1z) >= 0) pt++;
                    if (((vx * v3x + vy * v3y) + vz * v3z) >= 0) pn++;
                }
            }
            pt = wave_sum_i(pt);
            pn = wave_sum_i(pn);
            if (lane == 0) { csum[wave][0] = pt; csum[wave][1] = pn; }
            __syncthreads();
            if (t == 0) {
                int PT = 0, PN = 0;
                for (int w = 0; w < 4; ++w) { PT += (int)csum[w][0]; PN += (int)csum[w][1]; }
                double x[3] = {v1x, v1y, v1z}, z[3] = {v3x, v3y, v3z};
                PT = 2 * PT - valid_total;
                PN = 2 * PN - valid_total;
                if (PT == 0 || PN == 0) {
                    // median-5 rule over valid neighbours by rank (rare path, serial scan)
                    const int med = valid_total / 2;
                    int r = 0, addT = 0, addN = 0;
                    for (int i = 0; i < n && r <= med + 2; ++i) {
                        const unsigned long long key = a[i];
                        const float4 p = pts4[(unsigned)(key & 0xFFFFFFFFu)];
                        if (p.x == kx && p.y == ky && p.z == kz) continue;
                        if (r >= med - 2) {
                            const double vx = (double)(p.x - kx), vy = (double)(p.y - ky), vz = (double)(p.z - kz);
                            if (((vx * v1x + vy * v1y) + vz * v1z) > 0) addT++;
                            if (((vx * v3x + vy * v3y) + vz * v3z) > 0) addN++;
                        }
                        ++r;
                    }
                    if (PT == 0) { if (addT < 3) { x[0] = -x[0]; x[1] = -x[1]; x[2] = -x[2]; } }
                    if (PN == 0) { if (addN < 3) { z[0] = -z[0]; z[1] = -z[1]; z[2] = -z[2]; } }
                }
                if (PT < 0) { x[0] = -x[0]; x[1] = -x[1]; x[2] = -x[2]; }
                if (PN < 0) { z[0] = -z[0]; z[1] = -z[1]; z[2] = -z[2]; }
                const float x0 = (float)x[0], x1 = (float)x[1], x2 = (float)x[2];
                const float z0 = (float)z[0], z1 = (float)z[1], z2 = (float)z[2];
                float* r9 = rf_out + 9 * (size_t)q;
                r9[0] = x0; r9[1] = x1; r9[2] = x2;
                r9[3] = z1 * x2 - z2 * x1; r9[4] = z2 * x0 - z0 * x2; r9[5] = z0 * x1 - z1 * x0;
                r9[6] = z0; r9[7] = z1; r9[8] = z2;
                ok_out[q] = 1;
            }
        } else if (t == 0) {
            float* r9 = rf_out + 9 * (size_t)q;
            for (int j = 0; j < 9; ++j) r9[j] = __builtin_nanf("");
            ok_out[q] = 0;
        }
        __syncthreads();
    }
}

__device__ __forceinline__ float dot4f(float a0, float a1, float a2, float b0, float b1, float b2) {
    return (a0 * b0 + a2 * b2) + (a1 * b1 + 0.0f);
}

#define PST_RAD_45 0.78539816339744830961566084581988
#define PST_RAD_90 1.5707963267948966192313216916398
#define PST_RAD_135 2.3561944901923449288469825374596
#define PST_RAD_PI_7_8 2.7488935718910690836548129603691

// one wave per keypoint: ordered histogram accumulation, normalisation, binarisation
__global__ void __launch_bounds__(64) k_shot_hist(const float4* __restrict__ pts4, const float4* __restrict__ normals,
                                                  const float* __restrict__ kps, int k, float R,
                                                  const long long* __restrict__ offs,
                                                  const unsigned long long* __restrict__ seg,
                                                  const float* __restrict__ rf_in, const int* __restrict__ ok_in,
                                                  float* __restrict__ shot_out, unsigned int* __restrict__ bits_out) {
    __shared__ float hist[384];
    __shared__ int rbin[64 * 5];
    __shared__ float rval[64 * 5];
    const int lane = lane_id();
    const double Rd = (double)R;
    const double r12 = Rd / 2, r34 = (Rd * 3) / 4, r14 = Rd / 4;
    const int nr_bins = 10;
    for (int q = blockIdx.x; q < k; q += gridDim.x) {
        const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
        const long long o = offs[q];
        const int n = (int)(offs[q + 1] - o);
        const unsigned long long* a = seg + o;
        const bool fin = __builtin_isfinite(kx) && __builtin_isfinite(ky) && __builtin_isfinite(kz);
        const bool good = fin && ok_in[q] && n >= 5;
        for (int j = lane; j < 384; j += 64) hist[j] = 0.0f;
        __builtin_amdgcn_wave_barrier();
        float rf[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) rf[j] = rf_in[9 * (size_t)q + j];
        if (good) {
            for (int c0 = 0; c0 < n; c0 += 64) {
                const int i = c0 + lane;
                int bins[5] = {-1, -1, -1, -1, -1};
                float vals[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
                if (i < n) {
                    const unsigned long long key = a[i];
                    const unsigned int idx = (unsigned int)(key & 0xFFFFFFFFu);
                    const float4 nv = normals[idx];
                    if (__builtin_isfinite(nv.x) && __builtin_isfinite(nv.y) && __builtin_isfinite(nv.z)) {
                        double cosd = (double)dot4f(nv.x, nv.y, nv.z, rf[6], rf[7], rf[8]);
                        if (cosd > 1.0) cosd = 1.0;
                        if (cosd < -1.0) cosd = -1.0;
                        double bd = ((1.0 + cosd) * nr_bins) / 2;
                        const float4 p = pts4[idx];
                        const float dx = p.x - kx, dy = p.y - ky, dz = p.z - kz;
                        const double distance = sqrt((double)__uint_as_float((unsigned)(key >> 32)));
                        if (!(fabs(distance - 0.0) < 1e-15)) {
                            double xr = (double)dot4f(dx, dy, dz, rf[0], rf[1], rf[2]);
                            double yr = (double)dot4f(dx, dy, dz, rf[3], rf[4], rf[5]);
                            double zr = (double)dot4f(dx, dy, dz, rf[6], rf[7], rf[8]);
                            if (fabs(yr) < 1E-30) yr = 0;
                            if (fabs(xr) < 1E-30) xr = 0;
                            if (fabs(zr) < 1E-30) zr = 0;
                            const unsigned bit4 = ((yr > 0) || ((yr == 0.0) && (xr < 0))) ? 1u : 0u;
                            const unsigned bit3 = ((xr > 0) || ((xr == 0.0) && (yr > 0))) ? (bit4 ? 0u : 1u) : bit4;
                            int desc = (int)((bit4 << 3) + (bit3 << 2));
                            desc = desc << 1;
                            if ((xr * yr > 0) || (xr == 0.0)) desc += (fabs(xr) >= fabs(yr)) ? 0 : 4;
                            else desc += (fabs(xr) > fabs(yr)) ? 4 : 0;
                            desc += zr > 0 ? 1 : 0;
                            desc += (distance > r12) ? 2 : 0;
                            const int step = (int)floor(bd + 0.5);
                            const int vol = desc * (nr_bins + 1);
                            bd -= step;
                            double w = (1 - fabs(bd));
                            if (bd > 0) { bins[0] = vol + ((step + 1) % nr_bins); vals[0] = (float)bd; }
                            else { bins[0] = vol + ((step - 1 + nr_bins) % nr_bins); vals[0] = -(float)bd; }
                            if (distance > r12) {
                                const double rd = (distance - r34) / r12;
                                if (distance > r34) w += 1 - rd;
                                else { w += 1 + rd; bins[1] = (desc - 2) * (nr_bins + 1) + step; vals[1] = (float)(-rd); }
                            } else {
                                const double rd = (distance - r14) / r12;
                                if (distance < r14) w += 1 + rd;
                                else { w += 1 - rd; bins[1] = (desc + 2) * (nr_bins + 1) + step; vals[1] = (float)rd; }
                            }
                            double ic = zr / distance;
                            if (ic < -1.0) ic = -1.0;
                            if (ic > 1.0) ic = 1.0;
                            const double incl = bm::acos_(ic);
                            if (incl > PST_RAD_90 || (fabs(incl - PST_RAD_90) < 1e-30 && zr <= 0)) {
                                const double id = (incl - PST_RAD_135) / PST_RAD_90;
                                if (incl > PST_RAD_135) w += 1 - id;
                                else { w += 1 + id; bins[2] = (desc + 1) * (nr_bins + 1) + step; vals[2] = -(float)id; }
                            } else {
                                const double id = (incl - PST_RAD_45) / PST_RAD_90;
                                if (incl < PST_RAD_45) w += 1 + id;
                                else { w += 1 - id; bins[2] = (desc - 1) * (nr_bins + 1) + step; vals[2] = (float)id; }
                            }
                            if (yr != 0.0 || xr != 0.0) {
                                const double az = bm::atan2_(yr, xr);
                                const int sel = desc >> 2;
                                double ad = (az - (-PST_RAD_PI_7_8 + PST_RAD_45 * sel)) / PST_RAD_45;
                                ad = fmax(-0.5, fmin(ad, 0.5));
                                if (ad > 0) {
                                    w += 1 - ad;
                                    bins[3] = ((desc + 4) % 32) * (nr_bins + 1) + step; vals[3] = (float)ad;
                                } else {
                                    w += 1 + ad;
                                    bins[3] = ((desc - 4 + 32) % 32) * (nr_bins + 1) + step; vals[3] = -(float)ad;
                                }
                            }
                            bins[4] = vol + step;
                            vals[4] = (float)w;
                        }
                    }
                }
                // ordered application: neighbour r's (<= 5, pairwise distinct) bins in one ds_add
                // instruction, neighbours in rank order (LDS executes one wave's ops in issue
                // order). Lanes 0..4 each own one record slot; 16 records are loaded into VGPRs
                // per batch (one LDS wait), then issued as 16 back-to-back ds_add_f32. Unused
                // records add +0.0f to padding slot 360.
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    rbin[lane * 5 + j] = bins[j] < 0 ? 360 : bins[j];
                    rval[lane * 5 + j] = bins[j] < 0 ? 0.f : vals[j];
                }
                __builtin_amdgcn_wave_barrier();
                if (lane < 5) {
#pragma unroll
                    for (int g = 0; g < 64; g += 16) {
                        int bb[16];
                        float vv[16];
#pragma unroll
                        for (int u = 0; u < 16; ++u) {
                            bb[u] = rbin[(g + u) * 5 + lane];
                            vv[u] = rval[(g + u) * 5 + lane];
                        }
#pragma unroll
                        for (int u = 0; u < 16; ++u) atomicAdd(&hist[bb[u]], vv[u]);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        __builtin_amdgcn_wave_barrier();
        // normalizeHistogram: double accumulation of float squares in bin order
        float sv[6];
        if (good) {
            double acc = 0.0;
            if (lane == 0)
                for (int j = 0; j < 352; j += 8) {
                    float h[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) h[u] = hist[j + u];
#pragma unroll
                    for (int u = 0; u < 8; ++u) acc = acc + (double)(h[u] * h[u]);
                }
            acc = __shfl(acc, 0, 64);
            const float fa = (float)sqrt(acc);
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int b = lane + 64 * j;
                sv[j] = b < 352 ? hist[b] / fa : 0.f;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 6; ++j) sv[j] = __builtin_nanf("");
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const int b = lane + 64 * j;
            if (b < 352) {
                hist[b] = sv[j];
                if (shot_out) shot_out[352 * (size_t)q + b] = sv[j];
            }
        }
        __builtin_amdgcn_wave_barrier();
        // B-SHOT: 88 groups of 4 (include/bshot_bits.h:144-278)
        unsigned int code[2] = {0u, 0u};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int gidx = lane + 64 * h;
            if (gidx < 88) {
                const float v0 = hist[4 * gidx], v1 = hist[4 * gidx + 1], v2 = hist[4 * gidx + 2], v3 = hist[4 * gidx + 3];
                const float sum = ((v0 + v1) + v2) + v3;
                const double th = 0.9 * (double)sum;
                unsigned b;
                if (v0 == 0 && v1 == 0 && v2 == 0 && v3 == 0) b = 0;
                else if ((double)v0 > th) b = 1;
                else if ((double)v1 > th) b = 2;
                else if ((double)v2 > th) b = 4;
                else if ((double)v3 > th) b = 8;
                else if ((double)(v0 + v1) > th) b = 3;
                else if ((double)(v1 + v2) > th) b = 6;
                else if ((double)(v2 + v3) > th) b = 12;
                else if ((double)(v0 + v3) > th) b = 9;
                else if ((double)(v1 + v3) > th) b = 10;
                else if ((double)(v0 + v2) > th) b = 5;
                else if ((double)((v0 + v1) + v2) > th) b = 7;
                else if ((double)((v1 + v2) + v3) > th) b = 14;
                else if ((double)((v0 + v2) + v3) > th) b = 13;
                else if ((double)((v0 + v1) + v3) > th) b = 11;
                else b = 15;
                code[h] = b;
            }
        }
        // word w holds groups 8w..8w+7 (4 bits each)
        __shared__ unsigned int gcode[88];
        if (lane < 88) gcode[lane] = code[0];
        if (lane + 64 < 88) gcode[lane + 64] = code[1];
        __builtin_amdgcn_wave_barrier();
        if (lane < 11) {
            unsigned int w = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) w |= gcode[8 * lane + j] << (4 * j);
            bits_out[11 * (size_t)q + lane] = w;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace bsk

namespace bsh {

hipError_t launch_shot_count(const DevGrid& g, const float* kps, int k, float R, int* counts, long long* offs,
                             hipStream_t s, unsigned int* bh) {
    if (k <= 0) return hipSuccess;
    bsk::k_shot_count<<<(k + 3) / 4, 256, 0, s>>>(g.view(), kps, k, R, counts, bh);
    bsk::k_excl_scan<<<1, 1024, 0, s>>>(counts, k, offs);
    return hipGetLastError();
}

hipError_t launch_shot_gather(const DevGrid& g, const float* kps, int k, float R, const long long* offs,
                              unsigned long long* seg, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    bsk::k_shot_gather<<<(k + 3) / 4, 256, 0, s>>>(g.view(), kps, k, R, offs, seg);
    return hipGetLastError();
}

hipError_t launch_shot_count_plan(const DevGrid& g, const float* kps, int k, float R, int* counts, unsigned int* bh,
                                  long long seg_cap, int chunk_cap, long long* offs, int* cb, int* perm, int* err,
                                  hipStream_t s) {
    if (k <= 0) return hipSuccess;
    if (k > DP_MAXK) return hipErrorInvalidValue;
    bsk::k_shot_count<<<(k + 3) / 4, 256, 0, s>>>(g.view(), kps, k, R, counts, bh);
    bsk::k_desc_plan<<<1, 1024, 0, s>>>(counts, k, seg_cap, chunk_cap, offs, cb, perm, err);
    return hipGetLastError();
}

hipError_t launch_shot_gather_b(const DevGrid& g, const float* kps, int k, float R, const long long* offs,
                                const unsigned int* bh, unsigned int* bstart, unsigned long long* seg, hipStream_t s,
                                const int* err) {
    if (k <= 0) return hipSuccess;
    bsk::k_shot_gather_b<<<(k + 3) / 4, 256, 0, s>>>(g.view(), kps, k, R, offs, bh, bstart, seg, err);
    return hipGetLastError();
}

hipError_t launch_shot_rank(int k, int n_chunks, float R, const long long* offs, const int* cb, const int* owner,
                            const unsigned int* bstart, const unsigned long long* seg, unsigned long long* out,
                            hipStream_t s, int max_blocks) {
    if (k <= 0 || n_chunks <= 0) return hipSuccess;
    int blocks = (n_chunks + 3) / 4;
    if (max_blocks > 0 && blocks > max_blocks) blocks = max_blocks;
    bsk::k_shot_rank<<<blocks, 256, 0, s>>>(k, R, offs, cb, owner, bstart, seg, out);
    return hipGetLastError();
}

hipError_t launch_shot_sort(const long long* offs, int k, float R, unsigned long long* seg, unsigned long long* tmp,
                            hipStream_t s) {
    if (k <= 0) return hipSuccess;
    bsk::k_shot_sort<<<k, 256, 0, s>>>(offs, k, R, seg, tmp);
    return hipGetLastError();
}

hipError_t launch_lrf(const float4* pts4, const float* kps, int k, float R, const long long* offs,
                      const unsigned long long* seg, float* rf, int* ok, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    bsk::k_lrf<<<k, 256, 0, s>>>(pts4, kps, k, R, offs, seg, rf, ok);
    return hipGetLastError();
}

hipError_t launch_shot_hist(const float4* pts4, const float4* normals, const float* kps, int k, float R,
                            const long long* offs, const unsigned long long* seg, const float* rf, const int* ok,
                            float* shot, unsigned int* bits, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    bsk::k_shot_hist<<<k, 64, 0, s>>>(pts4, normals, kps, k, R, offs, seg, rf, ok, shot, bits);
    return hipGetLastError();
}

}  // namespace bsh
