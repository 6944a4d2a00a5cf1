// icp.hip -- A11 point-to-point ICP on gfx950 (PCL IterativeClosestPoint defaults,
// src/lidar_odometry.cpp:291-297: CorrespondenceEstimation::determineCorrespondences, 1-NN, no
// distance cap; TransformationEstimationSVD; DefaultConvergenceCriteria). The whole loop runs on the
// device: the exact 1-NN of every iteration, the float Umeyama step in Eigen's operation order and
// PCL's convergence test; the host launches two kernels and waits once. Exact: the packed key (float
// bits of d2 << 32 | target index) min picks the smallest squared distance, smallest index on ties
// (DESIGN.md convention for FLANN's traversal-dependent tie), independent of the reduction order.
//
// Iteration 0 (k_icp_lists, a wave per source): the exact 1-NN at the source's starting position
// q0, and a candidate list: every target within R of q0, R = d0 + {3000, 1500, 750, 350} mm (the
// largest whose count fits the list capacity; d0 = the NN distance), sorted by distance from q0.
// Iterations (k_icp_step + k_icp_nn per iteration, queued back to back): each iteration's Umeyama
// + convergence test on one workgroup, then the sources move rigidly by the step; a source's NN
// among its list is the global NN whenever dm + |q - q0| < R (with float slack): a target outside
// the list lies at least R from q0, so at least R - |q - q0| from q, farther than the list's best.
// Sources failing the test (moved too far, no list, non-finite) take the exact grid search of
// iteration 0 (a wave each) and get a new list.
// The targets' nested grids (cells 1000, 2000, 4000, 8000 mm) are built once per ICP call, queued
// ahead of RANSAC (ctx_icp_prepare).
#include <hip/hip_runtime.h>

#include "bshot_math.h"
#include "dev_cand.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

struct Xf16 {
    float m[16];
};

struct IcpGrids {
    GridView g[4];  // cells 1000, 2000, 4000, 8000 mm (a ball of radius rs is searched on the grid of cell rs)
};

// exact 1-NN of q, the whole wave: balls of radius 1000, 2000, 4000, 8000 mm (the cube of each on
// the grid whose cell is its radius: <= 27 cells, one lookup round). Every target with d2 < rs^2 is
// visited (for_candidates), so the smallest key inside the first non-empty ball is the global one,
// ties included: a target outside the ball has d2 >= rs^2 > the key's d2. No target within 8000 mm
// (or a non-finite q): every target is scanned, as the reference's kd-tree would find it.
__device__ __forceinline__ unsigned long long icp_wave_nn(const IcpGrids& G, CandLds* cs, float qx, float qy, float qz,
                                                          const float4* __restrict__ tgt4, int nt) {
    const int lane = lane_id();
    unsigned long long m = ~0ull;
    const bool fin = __builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz);
    if (fin) {
#pragma unroll
        for (int L = 0; L < 4; ++L) {
            const float rs = G.g[L].cell;
            const float rs2 = (float)((double)rs * (double)rs);
            for_candidates(G.g[L], cs, qx, qy, qz, rs, rs2, [&](bool v, float d2, unsigned int idx) {
                if (v) {
                    const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | idx;
                    m = key < m ? key : m;
                }
            });
            m = wave_min_u64(m);
            if (m != ~0ull) return m;
        }
    }
    for (int j = lane; j < nt; j += 64) {
        const float4 p = tgt4[j];
        const float d2 = d2_flann(qx, qy, qz, p.x, p.y, p.z);
        const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)j;
        m = key < m ? key : m;
    }
    return wave_min_u64(m);
}

// grid level whose cell is >= rs / 2 (a cube of <= 5^3 cells); the coarsest beyond 16 m
__device__ __forceinline__ int icp_level_for(const IcpGrids& G, float rs) {
    int L = 0;
    while (L < 3 && 2.f * G.g[L].cell < rs) ++L;
    return L;
}

template <class F>
__device__ __forceinline__ void icp_stream_level(const IcpGrids& G, int L, CandLds* cs, float qx, float qy, float qz,
                                                 float rs, float rs2, F&& f) {
    // constant grid indices (the views are kernel arguments; a dynamic index would copy them to scratch)
    if (L == 0) for_candidates(G.g[0], cs, qx, qy, qz, rs, rs2, f);
    else if (L == 1) for_candidates(G.g[1], cs, qx, qy, qz, rs, rs2, f);
    else if (L == 2) for_candidates(G.g[2], cs, qx, qy, qz, rs, rs2, f);
    else for_candidates(G.g[3], cs, qx, qy, qz, rs, rs2, f);
}

// The list's LDS sort row. The bitonic sort pads a list of n <= cap keys to the next power of two
// P >= n (>= 64). Round 5's 384-entry experiment sized the row to cap (384) while P reached 512: the
// pad's ~0 keys landed in the next wave's row, whose list then held key ~0 and loaded
// tgt4[0xFFFFFFFF] (a GPU memory fault, session r05zb). The row is now the padded length itself,
// ICP_LIST_ROW = the power of two >= max(cap, 64), so for any capacity the pad of a list that fits
// (n <= cap) ends inside its own row; the launchers refuse any cap but ICP_LIST_CAP.
__host__ __device__ constexpr int icp_pow2_at_least(int x) { return x <= 64 ? 64 : 2 * icp_pow2_at_least((x + 1) / 2); }
#define ICP_LIST_ROW (icp_pow2_at_least(ICP_LIST_CAP))
static_assert(ICP_LIST_ROW >= ICP_LIST_CAP && (ICP_LIST_ROW & (ICP_LIST_ROW - 1)) == 0, "sort row");

// Candidate list of source q (the whole wave) around its exact NN key m: every target within R of
// q, R = d0 + {3000, 1500, 750, 350} mm (the largest whose count fits cap; d0 = the NN distance),
// entries in ascending distance from q (sk: ICP_LIST_ROW keys of LDS scratch for the sort, cap <=
// ICP_LIST_ROW): entry e at dst[e * stride] (xyz, index bits) and its distance from q at
// dsd[e * stride]; *count = -1 (no list) when even the smallest overflows or q is not finite.
__device__ __forceinline__ void icp_build_list(const IcpGrids& G, CandLds* cs, float qx, float qy, float qz,
                                               unsigned long long m, const float4* __restrict__ tgt4, float4* dst,
                                               float* dsd, int stride, int cap, unsigned long long* sk, int* count_out,
                                               float* R_out) {
    int count = -1;
    float R = 0.f;
    const bool fin = __builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz);
    const float d0 = sqrtf(__uint_as_float((unsigned)(m >> 32)));
    if (fin && d0 < 1.0e6f) {
        // candidate radii (largest first) and their counts, one pass over the largest ball
        float Rk[4], R2k[4];
        const float add[4] = {3000.f, 1500.f, 750.f, 350.f};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            Rk[k] = d0 + add[k];
            R2k[k] = (float)((double)Rk[k] * (double)Rk[k]);
        }
        int ck[4] = {0, 0, 0, 0};
        icp_stream_level(G, icp_level_for(G, Rk[0]), cs, qx, qy, qz, Rk[0], R2k[0], [&](bool v, float d2, unsigned int) {
#pragma unroll
            for (int k = 0; k < 4; ++k) ck[k] += __popcll(__ballot(v && d2 < R2k[k]));
        });
        int kk = -1;
#pragma unroll
        for (int k = 3; k >= 0; --k)
            if (ck[k] <= cap) kk = k;
        if (kk >= 0) {
            float rs = Rk[0], rs2 = R2k[0];
#pragma unroll
            for (int k = 1; k < 4; ++k)
                if (kk == k) { rs = Rk[k]; rs2 = R2k[k]; }
            int n = 0;
            icp_stream_level(G, icp_level_for(G, rs), cs, qx, qy, qz, rs, rs2, [&](bool v, float d2, unsigned int idx) {
                const unsigned long long bm = __ballot(v);
                if (v) {
                    const int slot = n + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
                    if (slot < cap) sk[slot] = ((unsigned long long)__float_as_uint(d2) << 32) | idx;
                }
                n += __popcll(bm);
            });
            if (n <= cap) {
                // ascending distance from q: a later scan stops at the first entry too far to matter;
                // the pad stays inside this wave's row: P is the power of two >= n (>= 64), n <= cap, and
                // the row holds ICP_LIST_ROW = the power of two >= max(cap, 64) keys, so P <= the row.
                // (A compile-time clamp of P or n here let the compiler bound and unroll the pad and
                // write loops: 66 -> 105 VGPRs and a scratch spill in k_icp_lists.)
                int P = 64;
                while (P < n) P <<= 1;
                for (int e = n + lane_id(); e < P; e += 64) sk[e] = ~0ull;
                __builtin_amdgcn_wave_barrier();
                wave_bitonic(sk, P);
                for (int e = lane_id(); e < n; e += 64) {
                    const unsigned long long key = sk[e];
                    const unsigned idx = (unsigned)(key & 0xFFFFFFFFu);
                    const float4 p = tgt4[idx];
                    dst[(size_t)e * stride] = make_float4(p.x, p.y, p.z, __uint_as_float(idx));
                    dsd[(size_t)e * stride] = sqrtf(__uint_as_float((unsigned)(key >> 32)));
                }
                __builtin_amdgcn_wave_barrier();
                count = n;
                R = rs;
            }
        }
    }
    *count_out = count;
    *R_out = R;
}

// Hand-over stores to pinned host memory (the host's loop) are system-scope relaxed stores (written
// through to the host, never held in L2), ordered by waiting for their completion (vmcnt 0, which on
// gfx9 counts stores) before the flag is written. No release fence: at system scope a fence writes
// back the XCD's whole L2, tens of us with the lookahead's kernels' dirty lines in it.
__device__ __forceinline__ void icp_put_key(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void icp_put_flag(int* p, int v) {
    __builtin_amdgcn_s_waitcnt(0);  // this wave's key stores have completed
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// waves (sources) per k_icp_lists workgroup: 1. The lists kernel runs on the main stream beside the
// lookahead's SR, which fills a CU's LDS to 5.8 KB of 160 (24 waves x 6.4 KB): a 4-wave workgroup
// (10.3 KB) waited for SR workgroups to exit, a 1-wave one (2.6 KB) starts at once -- ICP's
// iteration-0 wait 0.21 -> 0.06 ms per sweep, 683 / 666 -> 707 / 722 sweeps/s (r06l)
#ifndef ICP_WAVES
#define ICP_WAVES 1
#endif
// per-source Umeyama record of an iteration, SoA rows in rec (row stride icp_rs(ns): 16-B aligned
// rows): source xyz (the source's current position), its NN target xyz, the NN's d2
__host__ __device__ __forceinline__ int icp_rs(int ns) { return (ns + 3) & ~3; }
__device__ __forceinline__ void icp_put_rec(float* rec, int ns, int i, float qx, float qy, float qz, float4 t,
                                            unsigned long long m) {
    ns = icp_rs(ns);
    rec[i] = qx;
    rec[(size_t)ns + i] = qy;
    rec[2 * (size_t)ns + i] = qz;
    rec[3 * (size_t)ns + i] = t.x;
    rec[4 * (size_t)ns + i] = t.y;
    rec[5 * (size_t)ns + i] = t.z;
    rec[6 * (size_t)ns + i] = __uint_as_float((unsigned)(m >> 32));
}

__device__ __forceinline__ void icp_ctl_init(bsh::IcpCtl* ctl) {
    for (int u = 0; u < 16; ++u) {
        ctl->fin[u] = (u % 5 == 0) ? 1.f : 0.f;
        ctl->T[u] = ctl->fin[u];
    }
    ctl->prev_mse = 1.7976931348623157e308;
    ctl->it = 0;
    ctl->stop = 0;
}

// iteration 0: the exact 1-NN of every source at its starting position, its candidate list, its
// Umeyama record and its loop state (position, list centre + radius)
// rec != null (the device loop): also the records, positions, loop state; best != null (the host's
// loop): the keys in pinned memory (system-scope stores) and per-workgroup done flags
__global__ void __launch_bounds__(64 * ICP_WAVES) k_icp_lists(const float* __restrict__ src0, int ns, IcpGrids G,
                                                              const float4* __restrict__ tgt4, int nt, int cap,
                                                              float4* __restrict__ lst, float* __restrict__ lsd,
                                                              int* __restrict__ lcnt, float4* __restrict__ lcen,
                                                              float4* __restrict__ pos, float* __restrict__ rec,
                                                              bsh::IcpCtl* ctl, unsigned int* __restrict__ sync,
                                                              unsigned long long* __restrict__ best, int* done) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    __shared__ CandLds cl[ICP_WAVES];
    __shared__ unsigned long long skl[ICP_WAVES][ICP_LIST_ROW];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    CandLds* cs = &cl[wave];
    cand_init(cs);
    if (rec && blockIdx.x == 0 && threadIdx.x == 0) {
        icp_ctl_init(ctl);
        sync[0] = 0u;
        sync[1] = 0u;
    }
    for (int i = blockIdx.x * ICP_WAVES + wave; i < ns; i += gridDim.x * ICP_WAVES) {
        const float qx = src0[3 * i], qy = src0[3 * i + 1], qz = src0[3 * i + 2];
        const unsigned long long m = icp_wave_nn(G, cs, qx, qy, qz, tgt4, nt);
        int count;
        float R;
        icp_build_list(G, cs, qx, qy, qz, m, tgt4, lst + i, lsd + i, ns, cap, skl[wave], &count, &R);  // entry e at [e * ns + i]
        if (lane == 0) {
            lcnt[i] = count;
            lcen[i] = make_float4(qx, qy, qz, R);
            if (rec) {
                pos[i] = make_float4(qx, qy, qz, 0.f);
                icp_put_rec(rec, ns, i, qx, qy, qz, tgt4[(unsigned)(m & 0xFFFFFFFFu)], m);
            }
            if (best) icp_put_key(&best[i], m);
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (done) {
        __builtin_amdgcn_s_waitcnt(0);  // every wave's key stores have completed
        __syncthreads();
        if (threadIdx.x == 0) icp_put_flag(&done[blockIdx.x], 1);
    }
}

// The host's loop (the default): iterations >= 1 in one persistent launch, a
// workgroup (one wave) per 64 sources, a lane per source holding its position. For iteration j the
// wave waits until the host has released it (IcpSync.go >= j after the host's float Umeyama step of
// iteration j - 1; -1 = stop), moves its source by the step (pcl::transformPointCloud's float
// expression, as the host's bg::xform), takes the NN among the source's list when the bound proves
// it global and queues the others for the grid search (which also rebuilds the source's list
// around its current position), stores the keys in pinned host memory and sets its flag done[w] =
// j. Its LDS (~4 KB) fits beside a CU the SR kernel fills (7 KB left of 160): the device loop's
// larger workgroups waited for CUs to drain under the lookahead's load. Every wave exits on go = -1,
// after max_iter - 1 iterations, or when a wait exceeds ICP_WAIT_TICKS; the host then restarts the
// iterations from the current positions (ctx_icp).
#define ICPH_THREADS 64
// waves per iteration workgroup: wave 0 owns the workgroup's 64 sources (lane per source) and alone
// polls the host's release (system-scope loads); a source that leaves its list takes a wave-wide
// grid search and list rebuild, and on the sweeps where ICP moves far (a gated frame starts from the
// previous pose) hundreds leave -- the 18 sweeps of 199 with >= 60 such searches waited 0.89 ms for
// iterations 1.. against 0.07 ms (corr 0.93, profiles/r06e_icp_tail.txt). The workgroup's waves take
// the queued searches in turn; the helper waits at the workgroup barrier (no polling, no issue
// slots). 2 waves (7.5 KB of LDS): ICP 0.35-0.36 ms per sweep, 736 / 739 sweeps/s; 1 wave (4.9 KB)
// 0.36, 707 / 722; 4 waves (12.7 KB, more than SR leaves a CU) 0.49, 716 / 725 (r06l). More polling
// waves instead (fewer sources per wave) made every hand-over slower: 32 -> 128 / 256 polling waves
// took the whole ICP phase 0.68 -> 2.2 / 3.0 ms (r06f).
#ifndef ICPH_WAVES
#define ICPH_WAVES 2
#endif
#define ICP_WAIT_TICKS 100000000ll  // 1 s at the 100 MHz wall clock: a launch that cannot finish exits
#ifndef ICPH_WPE
#define ICPH_WPE 0
#endif
// list entries a lane loads per round trip of its scan (the wave waits for its longest scan; beside
// the SHOT histogram the lists' lines come from the MALL, not the L2): 4 -> 16 cut the iterations'
// wait 0.23 -> 0.19 ms per sweep (134 VGPRs; profiles/r05z_*)
#ifndef ICPH_BATCH
#define ICPH_BATCH 16
#endif
#if ICPH_WPE > 0
#define ICPH_ATTR __attribute__((amdgpu_waves_per_eu(ICPH_WPE)))
#else
#define ICPH_ATTR
#endif
__global__ void __launch_bounds__(ICPH_THREADS * ICPH_WAVES) ICPH_ATTR k_icp_iterations(const float* __restrict__ src0, int ns, int j0,
                                                                 const float4* lst, const float* lsd,
                                                                 const int* __restrict__ lcnt,
                                                                 const float4* __restrict__ lcen, int cap, IcpGrids G,
                                                                 const float4* __restrict__ tgt4, int nt, int max_iter,
                                                                 const bsh::IcpSync* sy, int* done,
                                                                 unsigned long long* best, int* qstat,
                                                                 bsh::IcpDevSync* dsy, unsigned int seq) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    __shared__ CandLds cl[ICPH_WAVES];
    __shared__ float4 q_queue[ICPH_THREADS];
    __shared__ float4 q_new[ICPH_THREADS];  // rebuilt lists: new centre (xyz) and radius (w)
    __shared__ int n_new[ICPH_THREADS];     // their counts; -2 = unchanged
    __shared__ int nq;
    __shared__ int go_sh;                    // the release wave 0 saw (-1: stop)
    __shared__ float T_sh[16];               // its step transform
    __shared__ unsigned long long skl[ICPH_WAVES][ICP_LIST_ROW];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    cand_init(&cl[wave]);
    if (wave == 0) n_new[lane] = -2;
    const int i = blockIdx.x * ICPH_THREADS + lane;
    const bool have = wave == 0 && i < ns;
    float qx = 0.f, qy = 0.f, qz = 0.f, x0 = 0.f, y0 = 0.f, z0 = 0.f, R = 0.f;
    int n = -1;
    if (have) {
        qx = src0[3 * i]; qy = src0[3 * i + 1]; qz = src0[3 * i + 2];
        const float4 c0 = lcen[i];
        x0 = c0.x; y0 = c0.y; z0 = c0.z; R = c0.w;
        n = lcnt[i];
    }
    float4* lst_w = const_cast<float4*>(lst);
    float* lsd_w = const_cast<float*>(lsd);
    const float4* L = lst + (have ? i : 0);  // entry e at L[e * ns]: the wave's lanes read one 1 KB row
    const float* Ld = lsd + (have ? i : 0);
    for (int j = j0; j < max_iter; ++j) {
        if (wave == 0) {
            // the host's release of iteration j: read from pinned host memory by workgroup 0 (every
            // workgroup without the relay), which republishes it in device memory for the others --
            // 32 waves polling host memory made every hand-over slower (r06f: 64 pollers doubled the
            // ICP phase). Relaxed device-scope stores and loads, ordered by waiting for the stores'
            // completion before the word: no L2 write-back fence.
            const bool host_poll = !dsy || blockIdx.x == 0;
            int g = 0;
            if (lane == 0) {
                const long long t0 = wall_clock64();
                while (true) {
                    if (host_poll) {
                        g = __hip_atomic_load(&sy->go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        if (g < 0 || g >= j) break;
                    } else {
                        const unsigned long long w = __hip_atomic_load(&dsy->word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((unsigned int)(w >> 32) == seq) {
                            const unsigned int lo = (unsigned int)w;
                            if (lo == 0xFFFFFFFFu) { g = -1; break; }
                            if ((int)lo - 1 >= j) { g = (int)lo - 1; break; }
                        }
                    }
                    if (wall_clock64() - t0 > ICP_WAIT_TICKS) { g = -1; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
                go_sh = g;
                nq = 0;
            }
            g = __shfl(g, 0, 64);
            float t = 0.f;
            if (g >= 0 && lane < 16) {
                t = host_poll ? __hip_atomic_load(&sy->T[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                              : __hip_atomic_load(&dsy->T[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                T_sh[lane] = t;
            }
            if (dsy && blockIdx.x == 0) {
                // republish: the step first, then the word once the step's stores have completed
                if (g >= 0 && lane < 16) __hip_atomic_store(&dsy->T[lane], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_s_waitcnt(0);
                if (lane == 0)
                    __hip_atomic_store(&dsy->word,
                                       ((unsigned long long)seq << 32) | (g < 0 ? 0xFFFFFFFFull : (unsigned long long)(g + 1)),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        if (go_sh < 0) break;  // every wave of the workgroup
        if (have) {
            float T[12];
#pragma unroll
            for (int u = 0; u < 12; ++u) T[u] = T_sh[u];
            const float x = qx, y = qy, z = qz;
            qx = ((T[0] * x + T[1] * y) + T[2] * z) + T[3];
            qy = ((T[4] * x + T[5] * y) + T[6] * z) + T[7];
            qz = ((T[8] * x + T[9] * y) + T[10] * z) + T[11];
            bool ok = false;
            unsigned long long m = ~0ull;
            if (n >= 0 && __builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz)) {
                // entries in ascending distance from the list's centre q0: an entry e with
                // |e - q0| - |q - q0| beyond the best distance so far (with float slack) lies farther
                // from q than the best, and so do all later ones -- the scan stops there
                const double ex = (double)qx - (double)x0, ey = (double)qy - (double)y0, ez = (double)qz - (double)z0;
                const double delta = sqrt(ex * ex + ey * ey + ez * ez);
                double stop = 1e300;
                for (int k = 0; k < n; k += ICPH_BATCH) {
                    float4 p[ICPH_BATCH];
                    float dd[ICPH_BATCH];
#pragma unroll
                    for (int u = 0; u < ICPH_BATCH; ++u) {
                        const int e = k + u < n ? k + u : n - 1;
                        p[u] = L[(size_t)e * ns];
                        dd[u] = Ld[(size_t)e * ns];
                    }
                    if ((double)dd[0] - delta > stop) break;
#pragma unroll
                    for (int u = 0; u < ICPH_BATCH; ++u) {
                        if (k + u < n) {
                            const float d2 = d2_flann(qx, qy, qz, p[u].x, p[u].y, p[u].z);
                            const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | __float_as_uint(p[u].w);
                            m = key < m ? key : m;
                        }
                    }
                    stop = sqrt((double)__uint_as_float((unsigned)(m >> 32))) * (1.0 + 1e-5) + 1.0;
                }
                if (m != ~0ull) {
                    // |q - q0| + (the list best's distance) < R with slack for float rounding: relative
                    // 1e-5 on the distances, 1 mm absolute gap between the best and any outside target
                    const double dm = sqrt((double)__uint_as_float((unsigned)(m >> 32)));
                    ok = dm * (1.0 + 1e-5) + delta + 1.0 < (double)R * (1.0 - 1e-5);
                }
            }
            if (ok) icp_put_key(&best[(size_t)(j & 1) * ns + i], m);
            else q_queue[atomicAdd(&nq, 1)] = make_float4(qx, qy, qz, __int_as_float(i));
        }
        __syncthreads();
        const int nqueued = nq;
        if (qstat && threadIdx.x == 0 && nqueued) {  // instrumentation (bshot_work_counters 9, 10): grid searches
            atomicAdd(&qstat[0], nqueued);
            atomicMax(&qstat[1], nqueued);
        }
        for (int t = wave; t < nqueued; t += ICPH_WAVES) {
            // the exact grid search, then a new list around the current position (its owner lane
            // takes over the new centre, count and radius below), so a source that outgrew its list
            // pays the search once
            const float4 q = q_queue[t];
            const int qi = __float_as_int(q.w);
            const unsigned long long m = icp_wave_nn(G, &cl[wave], q.x, q.y, q.z, tgt4, nt);
            if (lane == 0) icp_put_key(&best[(size_t)(j & 1) * ns + qi], m);
            int cnt2;
            float R2;
            icp_build_list(G, &cl[wave], q.x, q.y, q.z, m, tgt4, lst_w + qi, lsd_w + qi, ns, cap, skl[wave], &cnt2, &R2);
            if (lane == 0) { q_new[qi - (int)blockIdx.x * ICPH_THREADS] = make_float4(q.x, q.y, q.z, R2); n_new[qi - (int)blockIdx.x * ICPH_THREADS] = cnt2; }
        }
        // every wave's key stores have completed before the flag (wave 0 sets it after the barrier);
        // the rebuilt lists (same CU) are read by their owner lanes from the next iteration on
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
        if (have && n_new[lane] != -2) {
            const float4 c = q_new[lane];
            x0 = c.x; y0 = c.y; z0 = c.z; R = c.w;
            n = n_new[lane];
            n_new[lane] = -2;
        }
        if (wave == 0) icp_put_flag(&done[blockIdx.x], j);
    }
}

// PCL's loop after iteration 0's neighbours: ONE persistent launch (k_icp_run) of a workgroup per
// 256 sources. Per iteration every workgroup moves its sources by the last step and finds their NN
// (the list scan below, else the grid search), writes the Umeyama records and arrives at a counter;
// the LAST to arrive computes the step -- the float Umeyama in Eigen's order (the means as 6
// sequential float sums in source order, the cross-covariance as 9 sequential sums of
// (d_r - dm_r)(s_c - sm_c), each sum on its own lane of wave 0 over the records staged in LDS and
// centred in place; PCL's MSE, a sequential double sum of the d2, on wave 1) and
// DefaultConvergenceCriteria (max_iter, transformation epsilon 0, MSE epsilon 1e-12) -- and releases
// the next iteration. No host round trip and no kernel boundary per iteration (under the lookahead's
// load each queued launch waited tens of us to dispatch). Cross-workgroup data (records, the loop
// state, the counters) moves with agent-scope relaxed loads and stores, ordered by waiting for the
// stores' completion before the arrival: no L2 write-back fence (the workgroups sit on different
// XCDs). A stop writes the result to pinned memory, seq last.
//   NN of a moved source: its NN among its candidate list is the global NN when dm + |q - q0| < R
//   (with float slack); otherwise the exact grid search by one of the workgroup's waves, which also
//   rebuilds the source's list.
// Sequential chains over LDS rows (the host's summation order): batches of 32 elements are read
// 8 x ds_read_b128 ahead of the dependent adds, so the LDS latency overlaps the previous batch's
// chain instead of stalling every 4 elements. Rows are 16-B aligned; k0 = the first index.
__device__ __forceinline__ float chain_sum_f(const float* a, int k0, int n, float acc) {
    int k = k0;
    for (; k < n && (k & 3); ++k) acc = acc + a[k];
    while (k + 32 <= n) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(a + k + 4 * u);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            acc = acc + v[u].x; acc = acc + v[u].y; acc = acc + v[u].z; acc = acc + v[u].w;
        }
        k += 32;
    }
    for (; k + 4 <= n; k += 4) {
        const float4 v = *reinterpret_cast<const float4*>(a + k);
        acc = acc + v.x; acc = acc + v.y; acc = acc + v.z; acc = acc + v.w;
    }
    for (; k < n; ++k) acc = acc + a[k];
    return acc;
}

__device__ __forceinline__ float chain_dot_f(const float* e, const float* f, int k0, int n, float acc) {
    int k = k0;
    for (; k < n && (k & 3); ++k) acc = acc + e[k] * f[k];
    while (k + 16 <= n) {
        float4 u[4], v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            u[j] = *reinterpret_cast<const float4*>(e + k + 4 * j);
            v[j] = *reinterpret_cast<const float4*>(f + k + 4 * j);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float p0 = u[j].x * v[j].x, p1 = u[j].y * v[j].y, p2 = u[j].z * v[j].z, p3 = u[j].w * v[j].w;
            acc = acc + p0; acc = acc + p1; acc = acc + p2; acc = acc + p3;
        }
        k += 16;
    }
    for (; k + 4 <= n; k += 4) {
        const float4 u = *reinterpret_cast<const float4*>(e + k);
        const float4 v = *reinterpret_cast<const float4*>(f + k);
        const float p0 = u.x * v.x, p1 = u.y * v.y, p2 = u.z * v.z, p3 = u.w * v.w;
        acc = acc + p0; acc = acc + p1; acc = acc + p2; acc = acc + p3;
    }
    for (; k < n; ++k) acc = acc + e[k] * f[k];
    return acc;
}

__device__ __forceinline__ double chain_sum_d(const float* a, int k0, int n, double acc) {
    int k = k0;
    for (; k < n && (k & 3); ++k) acc += (double)a[k];
    while (k + 32 <= n) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(a + k + 4 * u);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            acc += (double)v[u].x; acc += (double)v[u].y; acc += (double)v[u].z; acc += (double)v[u].w;
        }
        k += 32;
    }
    for (; k + 4 <= n; k += 4) {
        const float4 v = *reinterpret_cast<const float4*>(a + k);
        acc += (double)v.x; acc += (double)v.y; acc += (double)v.z; acc += (double)v.w;
    }
    for (; k < n; ++k) acc += (double)a[k];
    return acc;
}

// 4 waves per workgroup (256 sources), up to 2048 records staged in LDS at once. A one-wave form
// with 256-record chunks (~10 KB of LDS, 128 VGPRs, so that its workgroups fit beside SR's) was
// slower in the pipeline: 1.34 vs 1.11 ms per ICP call (profiles/r05d_icp_ab.txt) -- the step's
// sequential chains then share one wave (PCL's MSE chain after the covariance instead of beside it)
#ifndef ICPR_WAVES
#define ICPR_WAVES 4
#endif
#define ICPR_THREADS (64 * ICPR_WAVES)
#ifndef ICPR_CH
#define ICPR_CH 2048  // records staged in LDS at once by the stepping workgroup (7 floats each)
#endif
// PCL's MSE chain: wave 1's lane 0 beside wave 0's covariance lanes, or lane 9 of a lone wave
#define ICPR_MSE_LANE(wave, lane) (ICPR_WAVES > 1 ? ((wave) == 1 && (lane) == 0) : ((lane) == 9))

__device__ __forceinline__ void st_dev(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float ld_dev(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_dev_i(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int ld_dev_i(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_dev_d(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ double ld_dev_d(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ void icp_put_rec_dev(float* rec, int ns, int i, float qx, float qy, float qz, float4 t,
                                                unsigned long long m) {
    ns = icp_rs(ns);
    st_dev(rec + i, qx);
    st_dev(rec + (size_t)ns + i, qy);
    st_dev(rec + 2 * (size_t)ns + i, qz);
    st_dev(rec + 3 * (size_t)ns + i, t.x);
    st_dev(rec + 4 * (size_t)ns + i, t.y);
    st_dev(rec + 5 * (size_t)ns + i, t.z);
    st_dev(rec + 6 * (size_t)ns + i, __uint_as_float((unsigned)(m >> 32)));
}

// the step of one iteration by the whole (last-arriving) workgroup: Umeyama of the records, the
// composed transform and PCL's convergence test into ctl; a stop writes out.
// The records are staged in LDS chunk by chunk: every thread issues its share of the chunk's
// coherent (agent-scope) loads at once into registers, and the next chunk's are in flight while the
// current chunk's chains run (a load-then-store loop waited for each load: ~56 serialised L2 round
// trips per step).
__device__ __forceinline__ void icp_step(int ns, const float* rec, int max_iter, bsh::IcpCtl* ctl, bsh::IcpOut* out,
                                         int seq, float* srec, float* smean, float* sacc, double* smse) {
    const int tid = threadIdx.x, lane = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool big = ns > ICPR_CH;
    const int chs = big ? ICPR_CH : ((ns + 3) & ~3);  // LDS row stride (16-B aligned rows)
    const int rs = icp_rs(ns);
    const float one_over_n = 1.f / (float)ns;
    static_assert(ICPR_CH % (4 * ICPR_THREADS) == 0, "a chunk row is whole float4s, one per thread");
    constexpr int PF = ICPR_CH / (4 * ICPR_THREADS);  // float4s per thread per row
    float4 nx[7][PF];
    auto fetch = [&](int c0) {  // rows [c0, c0 + chs) -> registers (a row tail past rs is never read)
#pragma unroll
        for (int c = 0; c < 7; ++c)
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int k = 4 * (tid + u * ICPR_THREADS);
                const float* r = rec + (size_t)c * rs + (c0 + k < rs ? c0 + k : 0);
                nx[c][u] = make_float4(ld_dev(r), ld_dev(r + 1), ld_dev(r + 2), ld_dev(r + 3));
            }
    };
    auto put = [&]() {
#pragma unroll
        for (int c = 0; c < 7; ++c)
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int k = 4 * (tid + u * ICPR_THREADS);
                if (k < chs) *reinterpret_cast<float4*>(srec + c * chs + k) = nx[c][u];
            }
    };
    // ---- means: lanes 0..5 of wave 0, source order (the first element starts the sum)
    float acc = 0.f;
    fetch(0);
    for (int c0 = 0; c0 < ns; c0 += chs) {
        const int cn = ns - c0 < chs ? ns - c0 : chs;
        __syncthreads();  // the previous chunk's chains are done with srec
        put();
        __syncthreads();
        if (c0 + chs < ns) fetch(c0 + chs);  // in flight during this chunk's chains
        if (wave == 0 && lane < 6) {
            const float* a = srec + lane * chs;
            if (c0 == 0) acc = chain_sum_f(a, 1, cn, a[0]);
            else acc = chain_sum_f(a, 0, cn, acc);
        }
    }
    if (wave == 0 && lane < 6) smean[lane] = acc * one_over_n;
    if (big) fetch(0);
    __syncthreads();
    // ---- cross-covariance (wave 0, lane r * 3 + c) and PCL's MSE
    const float sm0 = smean[0], sm1 = smean[1], sm2 = smean[2], dm0 = smean[3], dm1 = smean[4], dm2 = smean[5];
    float cov = 0.f;
    double mse = 0.0;
    for (int c0 = 0; c0 < ns; c0 += chs) {
        const int cn = ns - c0 < chs ? ns - c0 : chs;
        if (big) {
            __syncthreads();
            put();
            __syncthreads();
            if (c0 + chs < ns) fetch(c0 + chs);
        }
        // centre in place: s - sm, d - dm (the host's s0..s2, d0..d2)
        for (int t = tid; t < 6 * cn; t += ICPR_THREADS) {
            const int c = t / cn, k = t - c * cn;
            const float m = c == 0 ? sm0 : c == 1 ? sm1 : c == 2 ? sm2 : c == 3 ? dm0 : c == 4 ? dm1 : dm2;
            srec[c * chs + k] = srec[c * chs + k] - m;
        }
        __syncthreads();
        if (wave == 0 && lane < 9) {
            const float* e = srec + (3 + lane / 3) * chs;  // d_r - dm_r
            const float* f = srec + (lane % 3) * chs;      // s_c - sm_c
            if (c0 == 0) cov = chain_dot_f(e, f, 1, cn, e[0] * f[0]);
            else cov = chain_dot_f(e, f, 0, cn, cov);
        } else if (ICPR_MSE_LANE(wave, lane)) {
            mse = chain_sum_d(srec + 6 * chs, 0, cn, mse);
        }
    }
    if (wave == 0 && lane < 9) sacc[lane] = cov;
    if (ICPR_MSE_LANE(wave, lane)) *smse = mse;
    __syncthreads();
    // ---- the step, PCL's convergence test (the host loop's order: the step is composed first, then
    // max_iter, the transformation epsilon, the MSE epsilon)
    if (tid == 0) {
        float sigma[9], sm[3] = {sm0, sm1, sm2}, dm[3] = {dm0, dm1, dm2}, o[16], fin[16], nf[16];
#pragma unroll
        for (int u = 0; u < 9; ++u) sigma[u] = sacc[u] * one_over_n;
        bm::umeyama_finish<float>(sigma, sm, dm, o);
#pragma unroll
        for (int u = 0; u < 16; ++u) fin[u] = ld_dev(&ctl->fin[u]);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                nf[r * 4 + c] = ((o[r * 4] * fin[c] + o[r * 4 + 1] * fin[4 + c]) + o[r * 4 + 2] * fin[8 + c]) +
                                o[r * 4 + 3] * fin[12 + c];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            st_dev(&ctl->fin[u], nf[u]);
            st_dev(&ctl->T[u], o[u]);
        }
        const int it = ld_dev_i(&ctl->it) + 1;
        st_dev_i(&ctl->it, it);
        int stop = it >= max_iter;
        if (!stop) {
            const double cos_angle = 0.5 * (double)(((o[0] + o[5]) + o[10]) - 1.0f);
            const double tsq = (double)((o[3] * o[3] + o[7] * o[7]) + o[11] * o[11]);
            if (cos_angle >= 1.0 && tsq <= 0.0) stop = 1;
        }
        if (!stop) {
            const double m = *smse / (double)ns;
            if (__builtin_fabs(m - ld_dev_d(&ctl->prev_mse)) < 1e-12) stop = 1;
            st_dev_d(&ctl->prev_mse, m);
        }
        st_dev_i(&ctl->stop, stop);
        if (stop) {
#pragma unroll
            for (int u = 0; u < 16; ++u) __hip_atomic_store(&out->T[u], nf[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&out->iters, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_s_waitcnt(0);  // T and the count have reached host memory before seq
            __hip_atomic_store(&out->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// sync[0]: arrivals (nb per iteration), sync[1]: the last released iteration (zeroed by k_icp_lists)
#ifndef ICPR_WPE
#define ICPR_WPE 0  // no cap (a cap of 128 VGPRs spills)
#endif
#if ICPR_WPE > 0
#define ICPR_ATTR __attribute__((amdgpu_waves_per_eu(ICPR_WPE)))
#else
#define ICPR_ATTR
#endif
__global__ void __launch_bounds__(ICPR_THREADS) ICPR_ATTR k_icp_run(int ns, float4* lst, float* lsd, int* lcnt,
                                                          float4* __restrict__ lcen, float4* __restrict__ pos, int cap,
                                                          IcpGrids G, const float4* __restrict__ tgt4, int nt, float* rec,
                                                          int max_iter, bsh::IcpCtl* ctl, unsigned int* sync,
                                                          bsh::IcpOut* out, int seq) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    extern __shared__ __attribute__((aligned(16))) float srec[];  // the stepping workgroup's records
    __shared__ CandLds cl[ICPR_WAVES];
    __shared__ unsigned long long skl[ICPR_WAVES][ICP_LIST_ROW];
    __shared__ float4 qq[ICPR_THREADS];
    __shared__ int nq, s_last, s_stop;
    __shared__ float sT[12];
    __shared__ float smean[6];
    __shared__ float sacc[9];
    __shared__ double smse;
    const int tid = threadIdx.x, lane = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const unsigned int nb = gridDim.x;
    cand_init(&cl[wave]);
    const int i = blockIdx.x * ICPR_THREADS + tid;
    for (int j = 0;; ++j) {
        if (j > 0) {
            // wait for step j - 1 (released by whichever workgroup arrived last)
            if (tid == 0) {
                const long long t0 = wall_clock64();
                int stop = 0;
                while ((int)__hip_atomic_load(&sync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < j) {
                    if (wall_clock64() - t0 > ICP_WAIT_TICKS) { stop = 1; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                s_stop = stop || ld_dev_i(&ctl->stop);
            }
            if (tid < 12) sT[tid] = ld_dev(&ctl->T[tid]);
            __syncthreads();
            if (s_stop) break;
            if (tid == 0) nq = 0;
            __syncthreads();
            if (i < ns) {
                // pcl::transformPointCloud's float expression (the host's bg::xform)
                const float4 p = pos[i];
                const float qx = ((sT[0] * p.x + sT[1] * p.y) + sT[2] * p.z) + sT[3];
                const float qy = ((sT[4] * p.x + sT[5] * p.y) + sT[6] * p.z) + sT[7];
                const float qz = ((sT[8] * p.x + sT[9] * p.y) + sT[10] * p.z) + sT[11];
                pos[i] = make_float4(qx, qy, qz, 0.f);
                const float4 c0 = lcen[i];
                const int n = lcnt[i];
                bool ok = false;
                unsigned long long m = ~0ull;
                float4 best = make_float4(0.f, 0.f, 0.f, 0.f);
                if (n >= 0 && __builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz)) {
                    // entries ascend in distance from the list's centre q0: an entry e with
                    // |e - q0| - |q - q0| beyond the best distance so far (with float slack) lies
                    // farther from q than the best, and so do all later ones -- the scan stops there
                    const float4* L = lst + i;  // entry e at L[e * ns]
                    const float* Ld = lsd + i;
                    const double ex = (double)qx - (double)c0.x, ey = (double)qy - (double)c0.y, ez = (double)qz - (double)c0.z;
                    const double delta = sqrt(ex * ex + ey * ey + ez * ez);
                    double stopd = 1e300;
                    for (int k = 0; k < n; k += 4) {
                        float4 pp[4];
                        float dd[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int e = k + u < n ? k + u : n - 1;
                            pp[u] = L[(size_t)e * ns];
                            dd[u] = Ld[(size_t)e * ns];
                        }
                        if ((double)dd[0] - delta > stopd) break;
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (k + u < n) {
                                const float d2 = d2_flann(qx, qy, qz, pp[u].x, pp[u].y, pp[u].z);
                                const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | __float_as_uint(pp[u].w);
                                if (key < m) { m = key; best = pp[u]; }
                            }
                        }
                        stopd = sqrt((double)__uint_as_float((unsigned)(m >> 32))) * (1.0 + 1e-5) + 1.0;
                    }
                    if (m != ~0ull) {
                        // |q - q0| + (the list best's distance) < R with slack for float rounding:
                        // relative 1e-5 on the distances, 1 mm absolute gap to any outside target
                        const double dm = sqrt((double)__uint_as_float((unsigned)(m >> 32)));
                        ok = dm * (1.0 + 1e-5) + delta + 1.0 < (double)c0.w * (1.0 - 1e-5);
                    }
                }
                if (ok) icp_put_rec_dev(rec, ns, i, qx, qy, qz, best, m);
                else qq[atomicAdd(&nq, 1)] = make_float4(qx, qy, qz, __int_as_float(i));
            }
            __syncthreads();
            const int nqueued = nq;
            for (int t = wave; t < nqueued; t += ICPR_WAVES) {
                // the exact grid search, then a new list around the current position, so a source
                // that outgrew its list pays the search once
                const float4 q = qq[t];
                const int qi = __float_as_int(q.w);
                const unsigned long long m = icp_wave_nn(G, &cl[wave], q.x, q.y, q.z, tgt4, nt);
                int cnt2;
                float R2;
                icp_build_list(G, &cl[wave], q.x, q.y, q.z, m, tgt4, lst + qi, lsd + qi, ns, cap, skl[wave], &cnt2, &R2);
                if (lane == 0) {
                    icp_put_rec_dev(rec, ns, qi, q.x, q.y, q.z, tgt4[(unsigned)(m & 0xFFFFFFFFu)], m);
                    lcnt[qi] = cnt2;
                    lcen[qi] = make_float4(q.x, q.y, q.z, R2);
                }
            }
        }
        // arrive: this workgroup's records have reached the coherence point first
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (tid == 0) {
            const unsigned int a = __hip_atomic_fetch_add(&sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = a == nb * (unsigned)(j + 1) - 1u;
        }
        __syncthreads();
        if (s_last) {
            icp_step(ns, rec, max_iter, ctl, out, seq, srec, smean, sacc, &smse);
            __builtin_amdgcn_s_waitcnt(0);  // the loop state has reached the coherence point
            __syncthreads();
            if (tid == 0) __hip_atomic_store(&sync[1], (unsigned int)(j + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ void k_pack_tgt(const float* __restrict__ xyz, int n, float4* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 0.f);
}

__global__ void k_gather(const float4* __restrict__ pts4, const int* __restrict__ idx, int k, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) {
        const float4 p = pts4[idx[i]];
        out[3 * i] = p.x; out[3 * i + 1] = p.y; out[3 * i + 2] = p.z;
    }
}

// the same with the indices read straight from the caller's pinned staging and the coordinates also
// written to pinned staging (hout, nullable): one launch instead of copy + gather + copy
__global__ void k_gather_io(const float4* __restrict__ pts4, const int* __restrict__ h_idx, int k,
                            float* __restrict__ out, float* __restrict__ hout) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) {
        const float4 p = pts4[h_idx[i]];
        out[3 * i] = p.x; out[3 * i + 1] = p.y; out[3 * i + 2] = p.z;
        if (hout) { hout[3 * i] = p.x; hout[3 * i + 1] = p.y; hout[3 * i + 2] = p.z; }
    }
}

}  // namespace bsk

namespace bsh {

hipError_t launch_pack_points(const float* xyz, int n, float4* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    bsk::k_pack_tgt<<<(n + 255) / 256, 256, 0, s>>>(xyz, n, out);
    return hipGetLastError();
}

hipError_t launch_gather(const float4* pts4, const int* idx, int k, float* out, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    bsk::k_gather<<<(k + 255) / 256, 256, 0, s>>>(pts4, idx, k, out);
    return hipGetLastError();
}

hipError_t launch_gather_io(const float4* pts4, const int* h_idx, int k, float* out, float* hout, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    bsk::k_gather_io<<<(k + 255) / 256, 256, 0, s>>>(pts4, h_idx, k, out, hout);
    return hipGetLastError();
}

static bsk::IcpGrids icp_views(const DevGrid* const* g4) {
    bsk::IcpGrids G;
    for (int L = 0; L < 4; ++L) G.g[L] = g4[L]->view();
    return G;
}

hipError_t launch_icp(const float* src0, int ns, float4* lst, float* lsd, int* lcnt, int cap, const DevGrid* const* g4,
                      const float4* tgt4, int nt, int max_iter, float4* pos, float4* lcen, float* rec, IcpCtl* ctl,
                      unsigned int* sync, IcpOut* out, int seq, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    if (cap != ICP_LIST_CAP) return hipErrorInvalidValue;
    const bsk::IcpGrids G = icp_views(g4);
    bsk::k_icp_lists<<<(ns + ICP_WAVES - 1) / ICP_WAVES, 64 * ICP_WAVES, 0, s>>>(src0, ns, G, tgt4, nt, cap, lst, lsd, lcnt,
                                                                               lcen, pos, rec, ctl, sync, nullptr,
                                                                               nullptr);
    const int chs = ns > ICPR_CH ? ICPR_CH : ((ns + 3) & ~3);
    const size_t lds = sizeof(float) * 7 * (size_t)chs;
    const int nb = (ns + ICPR_THREADS - 1) / ICPR_THREADS;
    // every workgroup of the persistent launch must fit on the chip at once (they wait for each other)
    if (nb > 256) return hipErrorInvalidValue;
    bsk::k_icp_run<<<nb, ICPR_THREADS, lds, s>>>(ns, lst, lsd, lcnt, lcen, pos, cap, G, tgt4, nt, rec,
                                                 max_iter > 1 ? max_iter : 1, ctl, sync, out, seq);
    return hipGetLastError();
}

int icp_lists_blocks(int ns) { return (ns + ICP_WAVES - 1) / ICP_WAVES; }
int icp_iter_blocks(int ns) { return (ns + ICPH_THREADS - 1) / ICPH_THREADS; }

hipError_t launch_icp_lists_host(const float* src0, int ns, const DevGrid* const* g4, const float4* tgt4, int nt, int cap,
                                 float4* lst, float* lsd, int* lcnt, float4* lcen, unsigned long long* best_out,
                                 int* done, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    if (cap != ICP_LIST_CAP) return hipErrorInvalidValue;
    bsk::k_icp_lists<<<icp_lists_blocks(ns), 64 * ICP_WAVES, 0, s>>>(src0, ns, icp_views(g4), tgt4, nt, cap, lst, lsd, lcnt,
                                                                     lcen, nullptr, nullptr, nullptr, nullptr, best_out,
                                                                     done);
    return hipGetLastError();
}

hipError_t launch_icp_iterations(const float* src0, int ns, int j0, const float4* lst, const float* lsd, const int* lcnt,
                                 const float4* lcen, int cap, const DevGrid* const* g4, const float4* tgt4, int nt,
                                 int max_iter, const IcpSync* sy, int* done, unsigned long long* best, hipStream_t s,
                                 int* qstat, IcpDevSync* dsy, unsigned int seq) {
    if (ns <= 0 || nt <= 0 || max_iter <= j0) return hipSuccess;
    if (cap != ICP_LIST_CAP) return hipErrorInvalidValue;
    bsk::k_icp_iterations<<<icp_iter_blocks(ns), ICPH_THREADS * ICPH_WAVES, 0, s>>>(src0, ns, j0, lst, lsd, lcnt, lcen, cap, icp_views(g4),
                                                                      tgt4, nt, max_iter, sy, done, best, qstat, dsy, seq);
    return hipGetLastError();
}

}  // namespace bsh
