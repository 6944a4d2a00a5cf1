// knn.hip -- exact radius-capped k-NN on the hashed grids + the two kernels built on it:
//   * k_seg_ratio : A1, segmentation ratio of every point (src/lidar_odometry.cpp:53-126)
//   * k_normals   : A4, keypoint normals (include/bshot_bits.h:43-94, pcl::computePointNormal)
//
// Selection semantics (FLANN KNNRadiusResultSet, sorted): the max_nn smallest (d2, idx) with
// d2 < r2, in ascending (d2, idx) order. One wavefront per query:
//   1. radius ladder rs = r * 2^(-k/2) for k = 8 .. 0 (9 steps, r/16 .. r; ladder mode 2, the
//      default), each step streamed from the nested hashed grid whose cell is rs/2 or rs/sqrt(2)
//      (r/16 for the two front steps); the first step is predicted from the query's own-cell counts
//      (ladder_start). Stop at the first rs with >= max_nn points inside (then every one of the
//      max_nn nearest lies strictly inside rs) -- exact whatever the start;
//   2. that step also stored its first KNN_CAP in-radius keys (d2 bits << 32 | idx) in LDS: a
//      KNN_NB-bucket d2 histogram of them bounds the prefix, and a counting sort + in-bucket rank
//      orders it in place (the rare crowded cases re-stream with <= 3 refinement levels);
//   3. ordered float reductions in rank order exactly as PCL (computeCentroid, covariance).
#include <hip/hip_runtime.h>

#include "bshot_math.h"
#include "dev_cand.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

#ifndef KNN_NB
#define KNN_NB 128
#endif
// k_seg_ratio's candidate streaming is bound by dependent L2 round trips, so waves per CU set its
// speed (3 -> 4 waves per SIMD: 1.05 -> 0.86 ms, profiles/ab_sr_stream.txt; 5 -> 6: 0.621 -> 0.601
// ms standalone, profiles/r05_ab_sr_w6.txt). Per wave: the key list (KNN_CAP keys), hist, offsets
// (u16) and the 16-bit candidate marks = 6.3 KB, so 24 waves fit the CU's 160 KB LDS, matched by
// <= 80 VGPRs (waves_per_eu 6). The list holds every in-radius key of the deciding ladder step when
// they fit (a 640-key list sends 8 % of the queries down the streaming path, 704 keys 6 %); the
// counting sort of the selected prefix (<= KNN_PRE keys) runs in place through registers.
#ifndef KNN_CAP
#define KNN_CAP 640
#endif
#define KNN_PRE 512  // largest prefix the counting sort handles (8 keys per lane)
#ifndef KNN_WAVES
#define KNN_WAVES 2
#endif
#ifndef SR_DIAG_NOFIN
#define SR_DIAG_NOFIN 0  // diagnostic: 1 = skip the ratio computation (timing of the selection alone)
#endif
#ifndef SR_WPE
#define SR_WPE 6  // VGPRs <= 80: 6 waves per SIMD
#endif
#if SR_WPE > 0
#define SR_ATTR __attribute__((amdgpu_waves_per_eu(SR_WPE)))
#else
#define SR_ATTR
#endif

// list, hist and boff are contiguous: after the selection they double as the rank-order float
// arrays of the finishing math (3 x FL_STRIDE coordinates, so max_nn <= FL_STRIDE, host-checked; the
// CVS terms overwrite the x array)
struct KnnLds {
    unsigned long long list[KNN_CAP];  // in-radius keys of the last ladder step; then the sorted result
    unsigned int hist[KNN_NB];
    unsigned short boff[KNN_NB + 4];   // counting-sort bucket starts (<= KNN_PRE)
    CandLds cand;
};
// the finishing math's 3 coordinate arrays sit FL_STRIDE floats apart: 480 + 4, so lanes reading
// x[r], y[r], z[r] together hit 3 different LDS banks (a multiple of 32 put all three in one bank)
#ifndef FL_STRIDE
#define FL_STRIDE 484
#endif
static_assert(sizeof(unsigned long long) * KNN_CAP + 4 * KNN_NB + 2 * (KNN_NB + 4) >= 3 * FL_STRIDE * 4,
              "list + hist + boff must hold 3 x FL_STRIDE floats");
static_assert(KNN_CAP >= KNN_PRE, "the prefix must fit the list (and the bitonic sort's 512 keys)");
static_assert(KNN_CAP % 64 == 0 && KNN_NB % 64 == 0, "lane-strided loops");

__device__ __forceinline__ int bucket_of(float d2, float lo, float sc) {
    const float v = (d2 - lo) * sc;
    int b = (int)v;
    if (!(v >= 0.f)) b = 0;
    if (b > KNN_NB - 1) b = KNN_NB - 1;
    return b;
}

__device__ __forceinline__ unsigned long long knn_key(float d2, unsigned int idx) {
    return ((unsigned long long)__float_as_uint(d2) << 32) | idx;
}

// wave: bucket B where the cumulative count reaches `need` (1-based); *below = count before B
__device__ __forceinline__ int hist_cross(KnnLds* L, int need, int* below) {
    const int lane = lane_id();
    int s = 0;
#pragma unroll
    for (int j = 0; j < KNN_NB / 64; ++j) s += (int)L->hist[lane * (KNN_NB / 64) + j];
    int tot;
    const int ex = wave_excl_scan(s, tot);
    const bool mine = ex < need && ex + s >= need;
    const unsigned long long m = __ballot(mine);
    const int owner = m ? (int)__ffsll((long long)m) - 1 : 63;
    int B = 0, bl = 0;
    if (lane == owner) {
        int acc = ex;
        B = lane * (KNN_NB / 64) + (KNN_NB / 64) - 1;
        for (int j = 0; j < KNN_NB / 64; ++j) {
            const int h = (int)L->hist[lane * (KNN_NB / 64) + j];
            if (acc + h >= need) { B = lane * (KNN_NB / 64) + j; break; }
            acc += h;
        }
        bl = acc;
    }
    B = readlane_i(B, owner);
    *below = readlane_i(bl, owner);
    return B;
}

__device__ __forceinline__ void hist_clear(KnnLds* L) {
    const int lane = lane_id();
#pragma unroll
    for (int j = 0; j < KNN_NB / 64; ++j) L->hist[lane + 64 * j] = 0;
    __builtin_amdgcn_wave_barrier();
}

// counting-sort offsets of buckets [0, Bmax]: boff[b] = start, hist[b] = cursor; returns the
// number of keys in those buckets
__device__ __forceinline__ int prefix_offsets(KnnLds* L, int Bmax) {
    const int lane = lane_id();
    int s = 0;
#pragma unroll
    for (int j = 0; j < KNN_NB / 64; ++j) {
        const int b = lane * (KNN_NB / 64) + j;
        s += b <= Bmax ? (int)L->hist[b] : 0;
    }
    int tot;
    int run = wave_excl_scan(s, tot);
    if (tot <= KNN_PRE) {
#pragma unroll
        for (int j = 0; j < KNN_NB / 64; ++j) {
            const int b = lane * (KNN_NB / 64) + j;
            const int h = b <= Bmax ? (int)L->hist[b] : 0;
            L->boff[b] = (unsigned short)run;
            L->hist[b] = (unsigned)run;
            run += h;
        }
        if (lane == 63) L->boff[KNN_NB] = (unsigned short)tot;
    }
    __builtin_amdgcn_wave_barrier();
    return tot;
}

// keys scattered bucket-grouped in list[0, tot) -> exact (d2, idx) order in list[0, tot), in place
// (every lane ranks its keys against the bucket first, then all write)
__device__ __forceinline__ void rank_in_place(KnnLds* L, int tot, float sc0) {
    const int lane = lane_id();
    unsigned long long kk[KNN_PRE / 64];
    unsigned int dst[KNN_PRE / 64];
#pragma unroll
    for (int j = 0; j < KNN_PRE / 64; ++j) {
        const int i = lane + 64 * j;
        kk[j] = 0;
        dst[j] = 0;
        if (i < tot) {
            const unsigned long long key = L->list[i];
            const int b = bucket_of(__uint_as_float((unsigned)(key >> 32)), 0.f, sc0);
            const unsigned s0 = L->boff[b], e0 = L->boff[b + 1];
            unsigned rank = 0;
            for (unsigned q = s0; q < e0; ++q) rank += L->list[q] < key ? 1u : 0u;
            kk[j] = key;
            dst[j] = s0 + rank;
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < KNN_PRE / 64; ++j)
        if (lane + 64 * j < tot) L->list[dst[j]] = kk[j];
    __builtin_amdgcn_wave_barrier();
}

// level-0 d2 histogram of the delivering ladder step: the keys of list[0, nl) (its first KNN_CAP
// in-radius keys) added to the histogram of the keys past the list, which the step counted as it
// streamed (zero when it did not overflow). Built after the step instead of per streamed chunk, so
// steps that fall short cost no LDS atomics.
__device__ __forceinline__ void hist_of_list(KnnLds* L, int nl, float sc0) {
    const int lane = lane_id();
    for (int i = lane; i < nl; i += 64)
        atomicAdd(&L->hist[bucket_of(__uint_as_float((unsigned)(L->list[i] >> 32)), 0.f, sc0)], 1u);
    __builtin_amdgcn_wave_barrier();
}

// cube radius that holds every point of level-0 buckets [0, b] (bucket_of(d2, 0, KNN_NB / rs2) <= b
// implies d2 < (b + 1) / KNN_NB * rs2 up to float rounding, covered by the 1e-4 margin): the
// streaming path's later passes only keep such points, so their cube shrinks to this radius
__device__ __forceinline__ float bucket_radius(float rs, int b) {
    if (b >= KNN_NB - 1) return rs;
    return fminf(rs, rs * sqrtf((float)(b + 1) / (float)KNN_NB) * 1.0001f + 0.01f);
}

template <bool DIAG>
__device__ __forceinline__ bool knn_finish(const GridView& g, KnnLds* L, float qx, float qy, float qz, float rs, float rs2,
                                           int max_nn, int total, int* need_out, unsigned long long* kst,
                                           unsigned long long chunks, unsigned long long ts1,
                                           const unsigned long long** sorted);

// Exact selection: leaves the `*need` nearest (d2, idx) sorted in (*sorted)[0, *need).
// Returns false when > KNN_CAP keys tie at the boundary after 3 refinement levels (reported).
// DIAG: the instantiation behind bshot_debug_knn_stats() accumulates work counters into kst; the
// product instantiation has no counters, cycle stamps or chunk tallies at all (they cost registers
// and, at one query per wave, spill stores in every wave's prologue).
//
// Fast path: the ladder step that first holds >= max_nn points also stored every in-radius key
// in LDS (ballot compaction), so when they fit (<= KNN_CAP) the selection is a histogram of that
// list plus a counting sort over LDS only -- no second pass over the candidates.
// start_step: first ladder step tried (any step is exact; a later start only costs work);
// rb > 0 (round 6): a radius known to hold >= max_nn points (an earlier query's
// exact max_nn-th distance plus the distance between the two queries, k_seg_ratio's runs): one pass
// at rb on the grid whose cell is >= rb / bratio replaces the ladder; if it holds fewer (float
// slack, or a bound that does not hold), the ladder continues from the first step beyond rb. Exact
// either way: the selection only needs a ball of radius <= r with >= max_nn points inside.
// *kth_d2: d2 of the max_nn-th neighbour (the next query's bound), -1 when fewer than max_nn lie within r.
template <bool DIAG>
__device__ __forceinline__ bool knn_select(const LadderGrids& lg, KnnLds* L, float qx, float qy, float qz, float r, int max_nn,
                           int start_step, float rb, float bratio, int* need_out, float* kth_d2,
                           unsigned long long* kst, const unsigned long long** sorted) {
    unsigned long long chunks = 0, chunks_before = 0;
    const int lane = lane_id();
    unsigned long long ts0 = 0ull;
    if constexpr (DIAG) ts0 = cycle_stamp();
    const float r2 = (float)((double)r * (double)r);
    float rs = r, rs2 = r2;
    int total = 0;
    const int last = lg.nsteps - 1;
    int step = start_step;
    if (step > last) step = last;
    int gl = lg.gi[step];
    int blev = 3;  // the bounded pass's grid: the finest whose cell is >= rb / bratio
    if (rb > 0.f && rb < r) {
        step = -1;
        for (int l = 2; l >= 0; --l)
            if (rb <= bratio * lg.g[l].cell) blev = l;
    }
    for (; step <= last; ++step) {
        if (step < 0) {
            rs = rb;
            rs2 = (float)((double)rb * (double)rb);
            gl = blev;
        } else {
            rs = step == last ? r : r * lg.frac[step];
            rs2 = step == last ? r2 : (float)((double)rs * (double)rs);
            gl = lg.gi[step];
        }
        const float sc = (float)KNN_NB / rs2;
        int cnt = 0;
        // keys past the LDS list are counted into the level-0 histogram as they stream (the list's
        // own keys join it afterwards, knn_finish): a step that overflows needs no extra pass for it
        hist_clear(L);
        // a step whose cube holds fewer than max_nn candidates cannot deliver: skipped unstreamed
        const bool went = for_candidates(lg.g[gl], &L->cand, qx, qy, qz, rs, rs2, [&](bool v, float d2, unsigned int idx) {
            if constexpr (DIAG) ++chunks;
            const unsigned long long m = __ballot(v);
            if (v) {
                const int slot = cnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                if (slot < KNN_CAP) L->list[slot] = knn_key(d2, idx);
                else atomicAdd(&L->hist[bucket_of(d2, 0.f, sc)], 1u);
            }
            cnt += __popcll(m);
        }, step == last ? 0 : max_nn);
        __builtin_amdgcn_wave_barrier();
        total = cnt;
        if constexpr (DIAG) {
            if (!went && lane == 0) atomicAdd(&kst[6], 1ull);
            if (step < 0 && lane == 0) atomicAdd(&kst[total >= max_nn ? 27 : 28], 1ull);
        }
        if (total >= max_nn) break;
        if constexpr (DIAG) {
            if (went && step < last && lane == 0) {
                atomicAdd(&kst[25], 1ull);
                atomicAdd(&kst[26], chunks - chunks_before);
            }
            chunks_before = chunks;
        }
        if (step < 0) {
            // the bound did not deliver: the ladder from its first step beyond rb
            int s0 = 0;
            while (s0 < last && r * lg.frac[s0] <= rb) ++s0;
            step = s0 - 1;
        }
    }
    unsigned long long ts1 = 0ull;
    if constexpr (DIAG) {
        ts1 = cycle_stamp();
        if (lane == 0) {
            atomicAdd(&kst[12], ts1 - ts0);
            atomicAdd(&kst[0], 1ull);
            if (step >= 0) atomicAdd(&kst[16 + (step > last ? last : step)], 1ull);
            atomicAdd(&kst[9], (unsigned long long)(total < max_nn ? total : max_nn));
            atomicAdd(&kst[10], (unsigned long long)total);
        }
    }
    const bool ok = knn_finish<DIAG>(lg.g[gl], L, qx, qy, qz, rs, rs2, max_nn, total, need_out, kst, chunks, ts1, sorted);
    *kth_d2 = -1.f;
    if (ok && total >= max_nn) *kth_d2 = __uint_as_float((unsigned)((*sorted)[max_nn - 1] >> 32));
    return ok;
}

// The selection once a ladder step (radius rs, rs2 = its square, streamed on grid g) has delivered
// (>= max_nn keys in radius, or the last step): L->list holds that step's first KNN_CAP in-radius
// keys, in any candidate order (the result does not depend on it).
template <bool DIAG>
__device__ __forceinline__ bool knn_finish(const GridView& g, KnnLds* L, float qx, float qy, float qz, float rs, float rs2,
                                           int max_nn, int total, int* need_out, unsigned long long* kst,
                                           unsigned long long chunks, unsigned long long ts1,
                                           const unsigned long long** sorted) {
    const int lane = lane_id();
    const int need = total < max_nn ? total : max_nn;
    *need_out = need;
    if (need == 0) return true;
    const float sc0 = (float)KNN_NB / rs2;
    // L->hist: the level-0 histogram of the whole ball (the streamed overflow + the list's keys)
    hist_of_list(L, total < KNN_CAP ? total : KNN_CAP, sc0);

    // ---- fast path: every in-radius key is in L->list
    if (total <= KNN_CAP) {
        int Bmax = KNN_NB - 1;
        if (total > need) {
            int below;
            Bmax = hist_cross(L, need, &below);
        }
        const int tot = prefix_offsets(L, Bmax);
        if (tot <= KNN_PRE) {
            // scatter the prefix bucket-grouped into the front of the list, through registers
            unsigned long long kk[KNN_CAP / 64];
#pragma unroll
            for (int j = 0; j < KNN_CAP / 64; ++j) {
                const int i = lane + 64 * j;
                kk[j] = i < total ? L->list[i] : ~0ull;
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = 0; j < KNN_CAP / 64; ++j) {
                if (lane + 64 * j < total) {
                    const int b = bucket_of(__uint_as_float((unsigned)(kk[j] >> 32)), 0.f, sc0);
                    if (b <= Bmax) L->list[atomicAdd(&L->hist[b], 1u)] = kk[j];
                }
            }
            __builtin_amdgcn_wave_barrier();
            rank_in_place(L, tot, sc0);
            *sorted = L->list;
            if constexpr (DIAG) {
                const unsigned long long ts2 = cycle_stamp();
                if (lane == 0) { atomicAdd(&kst[5], chunks); atomicAdd(&kst[13], ts2 - ts1); }
            }
            return true;
        }
        // a boundary bucket too crowded for the in-place counting sort: refine by streaming (rare)
    }
    if constexpr (DIAG) {
        if (lane == 0) atomicAdd(&kst[11], 1ull);
    }

    // ---- streaming path: > KNN_CAP keys in radius, or a crowded boundary bucket (total > need
    // here: the prefix of a ball with total <= need <= KNN_PRE always fits the counting sort).
    // Rare, so its passes stream 2 chunks at a time: fewer live registers, no spills.
    int B[3] = {KNN_NB, KNN_NB, KNN_NB};
    float lo[3] = {0.f, 0.f, 0.f}, sc[3] = {sc0, 0.f, 0.f};
    int levels = 0;
    {
        int below_acc = 0;
        float w = rs2;
#pragma unroll
        for (int lev = 0; lev < 3; ++lev) {
            if (lev > 0) {
                hist_clear(L);
                if constexpr (DIAG) {
                    if (lev > 0 && lane == 0) atomicAdd(&kst[7], 1ull);
                }
                for_candidates<2>(g, &L->cand, qx, qy, qz, bucket_radius(rs, B[0]), rs2, [&](bool v, float d2, unsigned int) {
                    if constexpr (DIAG) ++chunks;
                    if (!v) return;
                    int b = bucket_of(d2, lo[0], sc[0]);
                    if (b != B[0]) return;
                    b = bucket_of(d2, lo[1], sc[1]);
                    if (lev == 1) { atomicAdd(&L->hist[b], 1u); return; }
                    if (b != B[1]) return;
                    atomicAdd(&L->hist[bucket_of(d2, lo[2], sc[2])], 1u);
                });
                __builtin_amdgcn_wave_barrier();
            }
            int below;
            const int Bl = hist_cross(L, need - below_acc, &below);
            B[lev] = Bl;
            levels = lev + 1;
            below_acc += below;
            if (below_acc + (int)L->hist[Bl] <= KNN_PRE) break;
            if (lev == 2) {
                if (below_acc + (int)L->hist[Bl] <= KNN_CAP) break;
                return false;
            }
            const float wb = w / (float)KNN_NB;
            lo[lev + 1] = lo[lev] + (float)Bl * wb;
            sc[lev + 1] = (float)KNN_NB / wb;
            w = wb;
        }
    }
    const int lv = levels;
    if (lv <= 1) {
        // level-0 histogram is current: counting sort of the prefix, streamed
        const int Bmax = lv >= 1 ? B[0] : KNN_NB - 1;
        const int tot = prefix_offsets(L, Bmax);
        if (tot <= KNN_PRE) {
            for_candidates<2>(g, &L->cand, qx, qy, qz, bucket_radius(rs, Bmax), rs2, [&](bool v, float d2, unsigned int idx) {
                if constexpr (DIAG) ++chunks;
                if (v) {
                    const int b = bucket_of(d2, 0.f, sc0);
                    if (b <= Bmax) L->list[atomicAdd(&L->hist[b], 1u)] = knn_key(d2, idx);
                }
            });
            __builtin_amdgcn_wave_barrier();
            rank_in_place(L, tot, sc0);
            *sorted = L->list;
            if constexpr (DIAG) {
                const unsigned long long ts2 = cycle_stamp();
                if (lane == 0) { atomicAdd(&kst[5], chunks); atomicAdd(&kst[14], ts2 - ts1); }
            }
            return true;
        }
    }
    // general path: collect the (refined) prefix and bitonic-sort it
    int cnt = 0;
    for_candidates<2>(g, &L->cand, qx, qy, qz, lv > 0 ? bucket_radius(rs, B[0]) : rs, rs2, [&](bool v, float d2, unsigned int idx) {
        if constexpr (DIAG) ++chunks;
        bool take = v;
        if (take && lv > 0) {
            const int b0 = bucket_of(d2, lo[0], sc[0]);
            if (b0 > B[0]) take = false;
            else if (b0 == B[0] && lv > 1) {
                const int b1 = bucket_of(d2, lo[1], sc[1]);
                if (b1 > B[1]) take = false;
                else if (b1 == B[1] && lv > 2) {
                    if (bucket_of(d2, lo[2], sc[2]) > B[2]) take = false;
                }
            }
        }
        const unsigned long long m = __ballot(take);
        if (take) {
            const int slot = cnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            if (slot < KNN_CAP) L->list[slot] = knn_key(d2, idx);
        }
        cnt += __popcll(m);
    });
    if (cnt > KNN_CAP) return false;
    int P = 64;
    while (P < cnt) P <<= 1;
    if constexpr (DIAG) {
        const unsigned long long ts2 = cycle_stamp();
        if (lane == 0) {
            atomicAdd(&kst[5], chunks);
            atomicAdd(&kst[8], (unsigned long long)P);
            atomicAdd(&kst[14], ts2 - ts1);
        }
    }
    if (P <= KNN_PRE) {
        unsigned long long* buf = L->list;
        for (int i = cnt + lane; i < P; i += 64) buf[i] = ~0ull;
        __builtin_amdgcn_wave_barrier();
        wave_bitonic(buf, P);
    } else {
        // more keys than the bitonic buffer: every key's rank among all (keys are distinct), in place
        unsigned long long kk[KNN_CAP / 64];
        unsigned int dst[KNN_CAP / 64];
#pragma unroll
        for (int j = 0; j < KNN_CAP / 64; ++j) {
            const int i = lane + 64 * j;
            kk[j] = i < cnt ? L->list[i] : ~0ull;
            dst[j] = 0;
        }
        for (int q = 0; q < cnt; ++q) {
            const unsigned long long o = L->list[q];
#pragma unroll
            for (int j = 0; j < KNN_CAP / 64; ++j) dst[j] += o < kk[j] ? 1u : 0u;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < KNN_CAP / 64; ++j)
            if (lane + 64 * j < cnt) L->list[dst[j]] = kk[j];
        __builtin_amdgcn_wave_barrier();
    }
    *sorted = L->list;
    return true;
}

// First ladder step worth streaming, from the point counts of the query's own cell in each ladder
// grid (lanes 0..3 look them up in one round trip): step s is predicted to hold
// own(g[gi[s]]) * pi * (rs / cell)^2 * 100 / pct points (a surface through the cell). Speed only --
// any start step is exact, a late one just streams a larger ball.
__device__ __forceinline__ int ladder_start(const LadderGrids& lg, float qx, float qy, float qz, float r, int max_nn,
                                            int pct) {
    const int lane = lane_id();
    unsigned int st = 0, cnt = 0;
    if (lane < 4) {
        // the own cell in float (a boundary query may read a neighbour cell's count: speed only)
        const GridView& g = lg.g[lane];
        const float ic = g.inv_cell;
        if (!grid_lookup(g, cell_key((int)floorf(qx * ic), (int)floorf(qy * ic), (int)floorf(qz * ic)), st, cnt))
            cnt = 0;
    }
    const float c0 = (float)readlane_i((int)cnt, 0), c1 = (float)readlane_i((int)cnt, 1);
    const float c2 = (float)readlane_i((int)cnt, 2), c3 = (float)readlane_i((int)cnt, 3);
    const float k = 3.14159265f * 100.f / (float)pct;
    for (int s = 0; s < lg.nsteps - 1; ++s) {
        const int L = lg.gi[s];
        const float own = L == 0 ? c0 : L == 1 ? c1 : L == 2 ? c2 : c3;
        const float rc = r * lg.frac[s] / lg.g[L].cell;
        if (own * k * rc * rc >= (float)max_nn) return s;
    }
    return lg.nsteps - 1;
}

// sequential float sum of a[0, n) in index order (a 16-B aligned LDS row). Software-pipelined over
// two register groups: each group's 8 elements are loaded while the other group's 8 dependent adds
// run, so the LDS latency hides behind the chain (the plain loop waited for its own loads every 8
// elements: the ratio phase was a quarter of the kernel's wave time, profiles/r06c_sr_bench.txt). The
// empty asm with a memory clobber keeps the compiler from sinking a prefetch back to its use.
__device__ __forceinline__ float seq_sum(const float* a, int n) {
    float acc = 0.f;
    const int n8 = n & ~7;
    const float4* a4 = reinterpret_cast<const float4*>(a);
    if (n8 > 0) {
        float4 a0 = a4[0], a1 = a4[1];
        for (int r = 0; r < n8; r += 16) {
            const int nb = (r + 8 < n8 ? r + 8 : r) >> 2;
            const float4 b0 = a4[nb], b1 = a4[nb + 1];
            asm volatile("" ::: "memory");
            acc = acc + a0.x; acc = acc + a0.y; acc = acc + a0.z; acc = acc + a0.w;
            acc = acc + a1.x; acc = acc + a1.y; acc = acc + a1.z; acc = acc + a1.w;
            if (r + 8 >= n8) break;
            const int na = (r + 16 < n8 ? r + 16 : r + 8) >> 2;
            a0 = a4[na];
            a1 = a4[na + 1];
            asm volatile("" ::: "memory");
            acc = acc + b0.x; acc = acc + b0.y; acc = acc + b0.z; acc = acc + b0.w;
            acc = acc + b1.x; acc = acc + b1.y; acc = acc + b1.z; acc = acc + b1.w;
        }
    }
    for (int r = n8; r < n; ++r) acc = acc + a[r];
    return acc;
}

__device__ __forceinline__ float seq_dot(const float* a, const float* b, int n) {
    float acc = 0.f;
    int r = 0;
    for (; r + 4 <= n; r += 4) {
        const float p0 = a[r] * b[r], p1 = a[r + 1] * b[r + 1], p2 = a[r + 2] * b[r + 2], p3 = a[r + 3] * b[r + 3];
        acc = acc + p0; acc = acc + p1; acc = acc + p2; acc = acc + p3;
    }
    for (; r < n; ++r) acc = acc + a[r] * b[r];
    return acc;
}

// gather neighbour coordinates (rank order) into the LDS list region as 3 float arrays of 512
// (FL_STRIDE apart)
__device__ __forceinline__ void gather_xyz(const unsigned long long* sorted, const float4* __restrict__ pts4, int need,
                                           float* fl) {
    const int lane = lane_id();
    unsigned int myidx[512 / 64];
#pragma unroll
    for (int j = 0; j < 512 / 64; ++j) {
        const int r = lane + 64 * j;
        myidx[j] = r < need ? (unsigned int)(sorted[r] & 0xFFFFFFFFu) : 0u;
    }
    __builtin_amdgcn_wave_barrier();
    // all loads issued before any store (unconditional: ranks past `need` read point 0), so the
    // gathers' L2 round trips overlap instead of running one after another under a branch
    float4 p[512 / 64];
#pragma unroll
    for (int j = 0; j < 512 / 64; ++j) p[j] = pts4[myidx[j]];
#pragma unroll
    for (int j = 0; j < 512 / 64; ++j) {
        const int r = lane + 64 * j;
        if (r < need) { fl[r] = p[j].x; fl[FL_STRIDE + r] = p[j].y; fl[2 * FL_STRIDE + r] = p[j].z; }
    }
    __builtin_amdgcn_wave_barrier();
}

// segmentation ratio of a query from its `need` (> 0) sorted neighbours (src/lidar_odometry.cpp:86-123)
__device__ float sr_of_neighbours(const unsigned long long* sorted, const float4* __restrict__ pts4, int need, float* fl,
                                  float4 sp, int sr_type) {
    const int lane = lane_id();
    float out;
    gather_xyz(sorted, pts4, need, fl);
    // pcl::computeCentroid: sequential float sums in rank order (lanes 0,1,2)
    float acc = 0.f;
    if (lane < 3) acc = seq_sum(fl + FL_STRIDE * lane, need);
    const float fn = (float)need;
    const float cx = __shfl(acc, 0, 64) / fn, cy = __shfl(acc, 1, 64) / fn, cz = __shfl(acc, 2, 64) / fn;
    const float tx = sp.x - cx, ty = sp.y - cy, tz = sp.z - cz;
    if (sr_type == 0) {
        int pos = 0, neg = 0;
        for (int r0 = 0; r0 < need; r0 += 64) {
            const int r = r0 + lane;
            bool p = false, m = false;
            if (r < need) {
                const float vx = fl[r] - sp.x, vy = fl[FL_STRIDE + r] - sp.y, vz = fl[2 * FL_STRIDE + r] - sp.z;
                const float dot = tx * vx + (ty * vy + tz * vz);
                p = dot > 0.f;
                m = dot < 0.f;
            }
            pos += __popcll(__ballot(p));
            neg += __popcll(__ballot(m));
        }
        const float fp = (float)pos, fm = (float)neg;
        out = 1.0f - fminf(fp, fm) / fmaxf(fp, fm);
    } else {
        // CVS / CVSN: per-neighbour terms in parallel, sequential float sum in rank order
        const float ctn = sqrtf(tx * tx + (ty * ty + tz * tz));
        // a skipped neighbour stores +0: sum + (+0) == sum, as sum starts at +0 and so
        // is never -0 (the only value +0 changes). Each term overwrites its own x coordinate
        // (read first, by the same lane).
        float* term = fl;
        for (int r0 = 0; r0 < need; r0 += 64) {
            const int r = r0 + lane;
            if (r < need) {
                const float vx = fl[r] - sp.x, vy = fl[FL_STRIDE + r] - sp.y, vz = fl[2 * FL_STRIDE + r] - sp.z;
                const float vn = sqrtf(vx * vx + (vy * vy + vz * vz));
                const float dot = tx * vx + (ty * vy + tz * vz);
                const bool use = !(ctn == 0.f || vn == 0.f);
                term[r] = !use ? 0.f : (sr_type == 1 ? dot : dot / (ctn * vn));
            }
        }
        __builtin_amdgcn_wave_barrier();
        float sum = 0.f;
        if (lane == 0)
            for (int r = 0; r < need; ++r) sum = sum + term[r];
        sum = __shfl(sum, 0, 64);
        out = fabsf(sum) / (float)need;
    }
    return out;
}

// ------------------------------------------------------------------------------------------
// A1: segmentation ratio of every point. max_nn <= 512 (host-checked).
// Queries go in the ladder grids' cell order (g[0].spts, a permutation of the cloud whose .w holds
// each point's index), in XCD-local chunks (zc > 0, below) or dealt round-robin over the grid's
// waves (consecutive workgroups sit on different XCDs; one contiguous stretch of cell order per XCD
// would hand one XCD the dense near-sensor region). One query per wave pass: short waves let the other streams' kernels in
// (runs of several cell-order queries per wave, each starting its ladder at its predecessor's
// step, streamed 11-18 % fewer candidates but were slower in the pipeline,
// profiles/r03_ab_sr_order_runs.txt).
// DIAG (bshot_debug_knn_stats only): kst work counters and cycle stamps; the product launch is the
// DIAG = false instantiation, which has none.
template <bool DIAG>
__global__ void __launch_bounds__(64 * KNN_WAVES) SR_ATTR k_seg_ratio(LadderGrids lg, const float4* __restrict__ pts4, int n,
                                                              float radius, int max_nn, int sr_type, int hint,
                                                              float* __restrict__ ratio, int* __restrict__ err,
                                                              unsigned long long* __restrict__ kst, int zc, int run,
                                                              float bratio) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // the wave index in an SGPR: the wave's LDS base is then rematerialised, not held in a VGPR
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    KnnLds* L = reinterpret_cast<KnnLds*>(smem) + wave;
    cand_init(&L->cand);
    const int nw = gridDim.x * KNN_WAVES;
    const int nu = (n + run - 1) / run;  // runs of `run` consecutive cell-order queries, one per wave pass
    const float4* __restrict__ order = lg.g[0].spts;
    float* fl = reinterpret_cast<float*>(L->list);
    int u0 = blockIdx.x * KNN_WAVES + wave;
    if (zc > 0) {
        // XCD-local chunks of cell order: workgroups b, b + 8, ... share an XCD (the dispatcher deals
        // workgroups round-robin over the 8 XCDs), so the workgroups of label g = b % 8 take chunks
        // g, g + 8, g + 16, ... of zc workgroups each: the 8 XCDs work on 8 adjacent chunks at a time
        // (similar density, so the in-order dealing stays balanced) and each XCD's L2 holds its own
        // chunk's neighbourhood instead of all eight holding the same one
        const int g = blockIdx.x & 7, i = blockIdx.x >> 3;
        const int m = i / zc, o = i - m * zc;
        u0 = ((m * 8 + g) * zc + o) * KNN_WAVES + wave;
    }
    for (int u = u0; u < nu; u += nw) {
        // the run's queries chain their radii: the exact max_nn-th distance of the previous query
        // (pr, at pp) bounds this one's by pr + |q - pp| (triangle inequality), so after the first
        // query of a run each streams one ball barely larger than its own max_nn-NN ball instead of
        // the sqrt(2) radius ladder (consecutive cell-order queries lie a few cm apart)
        float pr = -1.f;
        float4 pp = make_float4(0.f, 0.f, 0.f, 0.f);
        const int jend = (u + 1) * run < n ? (u + 1) * run : n;
        for (int j = u * run; j < jend; ++j) {
            const float4 sp = order[j];
            const int q = (int)__float_as_uint(sp.w);
            float out = __builtin_nanf("");
            const bool origin = sp.x == 0.f && sp.y == 0.f && sp.z == 0.f;
            const bool fin = __builtin_isfinite(sp.x) && __builtin_isfinite(sp.y) && __builtin_isfinite(sp.z);
            if (!origin && fin) {
                int need = 0;
                float kd2 = -1.f;
                const unsigned long long* sorted = nullptr;
                float rb = 0.f;
                if (pr >= 0.f) {
                    // relative 1e-5 and 0.01 mm of slack over the float rounding of both distances;
                    // exactness does not depend on it (a ball holding fewer than max_nn falls back)
                    const double dx = (double)sp.x - pp.x, dy = (double)sp.y - pp.y, dz = (double)sp.z - pp.z;
                    rb = (float)((sqrt((double)pr) + sqrt(dx * dx + dy * dy + dz * dz)) * (1.0 + 1e-5) + 0.01);
                }
                const int start = rb == 0.f && hint > 0 ? ladder_start(lg, sp.x, sp.y, sp.z, radius, max_nn, hint) : 0;
                const bool ok = knn_select<DIAG>(lg, L, sp.x, sp.y, sp.z, radius, max_nn, start, rb, bratio, &need, &kd2,
                                                 kst, &sorted);
                pr = kd2;
                pp = sp;
                unsigned long long tm0 = 0ull;
                if constexpr (DIAG) tm0 = cycle_stamp();
                if (!ok) {
                    if (lane == 0) atomicOr(err, 1);
                } else if (need > 0) {
#if SR_DIAG_NOFIN
                    out = (float)need;  // diagnostic builds only: the selection without the ratio
#else
                    out = sr_of_neighbours(sorted, pts4, need, fl, sp, sr_type);
#endif
                }
                if constexpr (DIAG) {
                    const unsigned long long tm1 = cycle_stamp();
                    if (lane == 0) atomicAdd(&kst[15], tm1 - tm0);
                }
            }
            if (lane == 0) ratio[q] = out;
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// ------------------------------------------------------------------------------------------
// A4: normals of K keypoints written to slots [0, K) of the persistent N-sized array
__global__ void __launch_bounds__(64 * KNN_WAVES) k_normals(LadderGrids lg, const float4* __restrict__ pts4,
                                                            const float* __restrict__ kps, int k, float radius,
                                                            int max_nn, float4* __restrict__ normals,
                                                            int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    KnnLds* L = reinterpret_cast<KnnLds*>(smem) + wave;
    cand_init(&L->cand);
    float* fl = reinterpret_cast<float*>(L->list);
    const float qn = __builtin_nanf("");
    for (int q = blockIdx.x * KNN_WAVES + wave; q < k; q += gridDim.x * KNN_WAVES) {
        const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
        float nx = qn, ny = qn, nz = qn, curv = qn;
        if (__builtin_isfinite(kx) && __builtin_isfinite(ky) && __builtin_isfinite(kz)) {
            int need = 0;
            float kd2;
            const unsigned long long* sorted = nullptr;
            if (!knn_select<false>(lg, L, kx, ky, kz, radius, max_nn, 0, 0.f, 0.f, &need, &kd2, nullptr, &sorted)) {
                if (lane == 0) atomicOr(err, 2);
            } else if (need > 0) {
                if (need >= 3) {
                    gather_xyz(sorted, pts4, need, fl);
                    // pcl::computeMeanAndCovarianceMatrix: 9 float accumulators in rank order
                    float acc = 0.f;
                    if (lane < 9) {
                        const int a = lane < 6 ? (lane < 3 ? 0 : (lane < 5 ? 1 : 2)) : lane - 6;
                        const int bsel = lane < 6 ? (lane < 3 ? lane : (lane < 5 ? lane - 2 : 2)) : -1;
                        acc = bsel >= 0 ? seq_dot(fl + FL_STRIDE * a, fl + FL_STRIDE * bsel, need) : seq_sum(fl + FL_STRIDE * a, need);
                    }
                    float ac[9];
#pragma unroll
                    for (int a = 0; a < 9; ++a) ac[a] = __shfl(acc, a, 64);
                    const float fn = (float)need;
#pragma unroll
                    for (int a = 0; a < 9; ++a) ac[a] = ac[a] / fn;
                    float cov[9];
                    cov[0] = ac[0] - ac[6] * ac[6];
                    cov[1] = ac[1] - ac[6] * ac[7];
                    cov[2] = ac[2] - ac[6] * ac[8];
                    cov[4] = ac[3] - ac[7] * ac[7];
                    cov[5] = ac[4] - ac[7] * ac[8];
                    cov[8] = ac[5] - ac[8] * ac[8];
                    cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
                    float ev, vec[3];
                    bm::eigen33_min(cov, &ev, vec);
                    nx = vec[0]; ny = vec[1]; nz = vec[2];
                    const float eig_sum = (cov[0] + cov[4]) + cov[8];
                    curv = (eig_sum != 0.f) ? fabsf(ev / eig_sum) : 0.f;
                }
                const float vx = 0.f - kx, vy = 0.f - ky, vz = 0.f - kz;
                const float cth = (vx * nx + vy * ny) + vz * nz;
                if (cth < 0.f) { nx *= -1.f; ny *= -1.f; nz *= -1.f; }
            }
        }
        if (lane == 0) normals[q] = make_float4(nx, ny, nz, curv);
        __builtin_amdgcn_wave_barrier();
    }
}

#ifndef KNN_LDS_PAD
#define KNN_LDS_PAD 0  // diagnostic: extra LDS per workgroup (occupancy sensitivity)
#endif
size_t knn_lds_bytes() { return sizeof(KnnLds) * KNN_WAVES + KNN_LDS_PAD; }

}  // namespace bsk

namespace bsh {

int knn_max_nn() { return FL_STRIDE; }

// g4[0..3]: grids of cell r/16, r/8, r/4, r/2 when fine_ladder, else {r/8, r/8, r/2, r/2}
// mode 0: grids r/8, r/8, r/2, r/2, radii r 2^-k (4 steps); 1: nested grids r/16 .. r/2, radii
// r 2^(-k/2) from r/8 (7 steps); 2: as 1 with two more steps r/16, r/(8 sqrt 2) in front (9 steps),
// so dense neighbourhoods stop at a ball whose keys fit the LDS list
static LadderGrids ladder(const DevGrid* const* g4, int mode) {
    LadderGrids lg;
    for (int i = 0; i < 4; ++i) lg.g[i] = g4[i]->view();
    if (mode >= 1) {
        // each step on the grid whose cell is rs/2 or rs/sqrt(2) (r/16 for the two front steps)
        const float f[9] = {0.0625f, 0.08838835f, 0.125f, 0.17677669f, 0.25f, 0.35355339f, 0.5f, 0.70710678f, 1.0f};
        // (each step on the next finer grid instead: 0.54 -> 0.88 ms, 4.8 failed chunks per query,
        // profiles/r05_ab_sr_w6.txt)
        const int gi[9] = {0, 0, 0, 1, 1, 2, 2, 3, 3};
        const int o = mode == 2 ? 0 : 2;
        lg.nsteps = 9 - o;
        for (int i = 0; i < lg.nsteps; ++i) { lg.frac[i] = f[o + i]; lg.gi[i] = gi[o + i]; }
    } else {
        const float f[4] = {0.125f, 0.25f, 0.5f, 1.0f};
        lg.nsteps = 4;
        for (int i = 0; i < 4; ++i) { lg.frac[i] = f[i]; lg.gi[i] = i; }
    }
    return lg;
}

hipError_t launch_seg_ratio(const DevGrid* const* g4, int ladder_mode, const float4* pts4, int n, float radius,
                            int max_nn, int sr_type, int hint, float* ratio, int* err, hipStream_t s,
                            unsigned long long* kst, int max_blocks, int xcd_chunk, int run, float bratio) {
    const size_t lds = bsk::knn_lds_bytes();
    if (run < 1) run = 1;
    const int nu = (n + run - 1) / run;  // wave passes: runs of `run` consecutive cell-order queries
    int blocks = (nu + KNN_WAVES - 1) / KNN_WAVES;
    // fewer, longer-lived waves cost less dispatch; more, short-lived ones let high-priority
    // kernels of other streams in sooner
    if (max_blocks > 0 && blocks > max_blocks) blocks = max_blocks;
    int zc = 0;  // workgroups per XCD-local chunk (one query per wave only)
    if (xcd_chunk > 0 && (max_blocks <= 0 || blocks < max_blocks)) {
        zc = (xcd_chunk + KNN_WAVES * run - 1) / (KNN_WAVES * run);
        const int rounds = (blocks + 8 * zc - 1) / (8 * zc);
        blocks = rounds * 8 * zc;  // whole rounds of 8 chunks; the workgroups past n exit at once
    }
#ifdef DIAG_SR_TWICE
    // diagnostic builds only: SR twice (idempotent) -- its marginal cost
    bsk::k_seg_ratio<false><<<blocks, 64 * KNN_WAVES, lds, s>>>(ladder(g4, ladder_mode), pts4, n, radius, max_nn, sr_type,
                                                                hint, ratio, err, nullptr, zc, run, bratio);
#endif
    if (kst)
        bsk::k_seg_ratio<true><<<blocks, 64 * KNN_WAVES, lds, s>>>(ladder(g4, ladder_mode), pts4, n, radius, max_nn, sr_type,
                                                                   hint, ratio, err, kst, zc, run, bratio);
    else
        bsk::k_seg_ratio<false><<<blocks, 64 * KNN_WAVES, lds, s>>>(ladder(g4, ladder_mode), pts4, n, radius, max_nn, sr_type,
                                                                    hint, ratio, err, nullptr, zc, run, bratio);
    return hipGetLastError();
}

hipError_t launch_normals(const DevGrid* const* g4, int ladder_mode, const float4* pts4, const float* kps, int k,
                          float radius, int max_nn, float4* normals, int* err, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    const size_t lds = bsk::knn_lds_bytes();
    int blocks = (k + KNN_WAVES - 1) / KNN_WAVES;
    bsk::k_normals<<<blocks, 64 * KNN_WAVES, lds, s>>>(ladder(g4, ladder_mode), pts4, kps, k, radius, max_nn, normals, err);
    return hipGetLastError();
}

}  // namespace bsh
