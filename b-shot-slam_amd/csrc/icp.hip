// icp.hip -- A11 point-to-point ICP on gfx950 (PCL IterativeClosestPoint defaults,
// src/lidar_odometry.cpp:291-297: CorrespondenceEstimation::determineCorrespondences, 1-NN, no
// distance cap; TransformationEstimationSVD; DefaultConvergenceCriteria). The host runs PCL's loop
// (float Umeyama, convergence test); the GPU finds every iteration's exact 1-NN. Exact: the packed
// key (float bits of d2 << 32 | target index) min picks the smallest squared distance, smallest
// index on ties (DESIGN.md convention for FLANN's traversal-dependent tie), independent of the
// reduction order.
//
// Iteration 0 (k_icp_lists, a wave per source): the exact 1-NN at the source's starting position
// q0, and a candidate list: every target within R of q0, R = d0 + {3000, 1500, 750, 350} mm (the
// largest whose count fits the list capacity; d0 = the NN distance), sorted by distance from q0.
// Iterations >= 1 (k_icp_iterations, one persistent launch, a lane per source): the source moves
// rigidly by the step transform; its NN among the list is the global NN whenever
// dm + |q - q0| < R (with float slack): a target outside the list lies at least R from q0, so at
// least R - |q - q0| from q, farther than the list's best. Sources failing the test (moved too far,
// no list, non-finite) take the exact grid search of iteration 0 (a wave each) and get a new list.
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

// Hand-over stores to pinned host memory are system-scope relaxed stores (written through to the
// host, never held in L2), ordered by waiting for their completion (vmcnt 0, which on gfx9 counts
// stores) before the flag is written. No release fence: at system scope a fence writes back the
// XCD's whole L2, tens of us with the lookahead's kernels' dirty lines in it.
__device__ __forceinline__ void icp_put_key(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void icp_put_flag(int* p, int v) {
    __builtin_amdgcn_s_waitcnt(0);  // this wave's key stores have completed
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Candidate list of source q (the whole wave) around its exact NN key m: every target within R of
// q, R = d0 + {3000, 1500, 750, 350} mm (the largest whose count fits cap; d0 = the NN distance),
// entries in ascending distance from q (sk: cap keys of LDS scratch for the sort): entry e at
// dst[e * stride] (xyz, index bits) and its distance from q at dsd[e * stride]; *count = -1 (no
// list) when even the smallest overflows or q is not finite. cap: a power of two.
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
                // ascending distance from q: a later scan stops at the first entry too far to matter
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

#define ICP_WAVES 4
__global__ void __launch_bounds__(64 * ICP_WAVES) k_icp_lists(const float* __restrict__ src0, int ns, IcpGrids G,
                                                              const float4* __restrict__ tgt4, int nt, int cap,
                                                              float4* __restrict__ lst, float* __restrict__ lsd,
                                                              int* __restrict__ lcnt, float* __restrict__ lrad,
                                                              unsigned long long* __restrict__ best_out,
                                                              int* __restrict__ done) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    __shared__ CandLds cl[ICP_WAVES];
    __shared__ unsigned long long skl[ICP_WAVES][ICP_LIST_CAP];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    CandLds* cs = &cl[wave];
    cand_init(cs);
    for (int i = blockIdx.x * ICP_WAVES + wave; i < ns; i += gridDim.x * ICP_WAVES) {
        const float qx = src0[3 * i], qy = src0[3 * i + 1], qz = src0[3 * i + 2];
        const unsigned long long m = icp_wave_nn(G, cs, qx, qy, qz, tgt4, nt);
        if (lane == 0) icp_put_key(&best_out[i], m);
        int count;
        float R;
        icp_build_list(G, cs, qx, qy, qz, m, tgt4, lst + i, lsd + i, ns, cap, skl[wave], &count, &R);  // entry e at [e * ns + i]
        if (lane == 0) {
            lcnt[i] = count;
            lrad[i] = R;
        }
        __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_s_waitcnt(0);  // every wave's key stores have completed
    __syncthreads();
    if (threadIdx.x == 0) icp_put_flag(&done[blockIdx.x], 1);
}

// Iterations >= 1, one persistent launch: a workgroup (one wave) per 64 sources, a lane per source
// holding its position. For iteration j the wave waits until the host has released it (IcpSync.go
// >= j after the host's Umeyama step of iteration j - 1; -1 = stop), moves its source by the step
// (pcl::transformPointCloud's float expression, as the host's bg::xform), takes the NN among the
// source's list when the bound proves it global and queues the others for the grid search (which
// also rebuilds the source's list around its current position), stores
// the keys in pinned host memory and sets its flag done[w] = j. No launch, no stream sync per
// iteration: the host and the waves hand over through coherent host memory (the per-iteration
// launch + wait cost ~40 us under the lookahead's load, 10 times per sweep). Every wave exits on
// go = -1, after max_iter - 1 iterations, or when a wait exceeds ICP_WAIT_TICKS (wall clock).
#define ICPN_THREADS 64
#define ICP_WAIT_TICKS 100000000ll  // 1 s at the 100 MHz wall clock
__global__ void __launch_bounds__(ICPN_THREADS) k_icp_iterations(const float* __restrict__ src0, int ns,
                                                                 const float4* lst, const float* lsd,
                                                                 const int* __restrict__ lcnt,
                                                                 const float* __restrict__ lrad, int cap, IcpGrids G,
                                                                 const float4* __restrict__ tgt4, int nt, int max_iter,
                                                                 const bsh::IcpSync* sy, int* done,
                                                                 unsigned long long* best) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    __shared__ CandLds cl;
    __shared__ float4 q_queue[ICPN_THREADS];
    __shared__ float4 q_new[ICPN_THREADS];  // rebuilt lists: new centre (xyz) and radius (w)
    __shared__ int n_new[ICPN_THREADS];     // their counts; -2 = unchanged
    __shared__ int nq;
    __shared__ unsigned long long skl[ICP_LIST_CAP];
    const int lane = lane_id();
    cand_init(&cl);
    n_new[lane] = -2;
    const int i = blockIdx.x * ICPN_THREADS + lane;
    const bool have = i < ns;
    float x0 = 0.f, y0 = 0.f, z0 = 0.f;
    if (have) { x0 = src0[3 * i]; y0 = src0[3 * i + 1]; z0 = src0[3 * i + 2]; }
    float qx = x0, qy = y0, qz = z0;
    int n = have ? lcnt[i] : -1;
    float R = have ? lrad[i] : 0.f;
    float4* lst_w = const_cast<float4*>(lst);
    float* lsd_w = const_cast<float*>(lsd);
    const float4* L = lst + (have ? i : 0);  // entry e at L[e * ns]: the wave's lanes read one 1 KB row
    const float* Ld = lsd + (have ? i : 0);
    for (int j = 1; j < max_iter; ++j) {
        int g = 0;
        if (lane == 0) {
            const long long t0 = wall_clock64();
            while (true) {
                g = __hip_atomic_load(&sy->go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (g < 0 || g >= j) break;
                if (wall_clock64() - t0 > ICP_WAIT_TICKS) { g = -1; break; }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        g = __shfl(g, 0, 64);
        if (g < 0) break;
        float Tl = lane < 16 ? __hip_atomic_load(&sy->T[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0.f;
        float T[12];
#pragma unroll
        for (int u = 0; u < 12; ++u) T[u] = __shfl(Tl, u, 64);
        if (lane == 0) nq = 0;
        __builtin_amdgcn_wave_barrier();
        if (have) {
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
                for (int k = 0; k < n; k += 4) {
                    float4 p[4];
                    float dd[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int e = k + u < n ? k + u : n - 1;
                        p[u] = L[(size_t)e * ns];
                        dd[u] = Ld[(size_t)e * ns];
                    }
                    if ((double)dd[0] - delta > stop) break;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
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
        __builtin_amdgcn_wave_barrier();
        const int nqueued = nq;
        for (int t = 0; t < nqueued; ++t) {
            // the exact grid search, then a new list around the current position (its owner lane
            // takes over the new centre, count and radius below), so a source that outgrew its list
            // pays the search once
            const float4 q = q_queue[t];
            const int qi = __float_as_int(q.w);
            const unsigned long long m = icp_wave_nn(G, &cl, q.x, q.y, q.z, tgt4, nt);
            if (lane == 0) icp_put_key(&best[(size_t)(j & 1) * ns + qi], m);
            int cnt2;
            float R2;
            icp_build_list(G, &cl, q.x, q.y, q.z, m, tgt4, lst_w + qi, lsd_w + qi, ns, cap, skl, &cnt2, &R2);
            if (lane == 0) { q_new[qi - (int)blockIdx.x * ICPN_THREADS] = make_float4(q.x, q.y, q.z, R2); n_new[qi - (int)blockIdx.x * ICPN_THREADS] = cnt2; }
        }
        // the rebuilt lists (stored by this wave) are read by their owner lanes from the next iteration on
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
        if (have && n_new[lane] != -2) {
            const float4 c = q_new[lane];
            x0 = c.x; y0 = c.y; z0 = c.z; R = c.w;
            n = n_new[lane];
            n_new[lane] = -2;
        }
        __builtin_amdgcn_wave_barrier();
        icp_put_flag(&done[blockIdx.x], j);
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

static bsk::IcpGrids icp_views(const DevGrid* const* g4) {
    bsk::IcpGrids G;
    for (int L = 0; L < 4; ++L) G.g[L] = g4[L]->view();
    return G;
}

int icp_lists_blocks(int ns) { return (ns + ICP_WAVES - 1) / ICP_WAVES; }
int icp_iter_blocks(int ns) { return (ns + ICPN_THREADS - 1) / ICPN_THREADS; }

hipError_t launch_icp_lists(const float* src0, int ns, const DevGrid* const* g4, const float4* tgt4, int nt, int cap,
                            float4* lst, float* lsd, int* lcnt, float* lrad, unsigned long long* best_out, int* done,
                            hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    if (cap != ICP_LIST_CAP) return hipErrorInvalidValue;
    bsk::k_icp_lists<<<icp_lists_blocks(ns), 64 * ICP_WAVES, 0, s>>>(src0, ns, icp_views(g4), tgt4, nt, cap, lst, lsd, lcnt,
                                                                     lrad, best_out, done);
    return hipGetLastError();
}

hipError_t launch_icp_iterations(const float* src0, int ns, const float4* lst, const float* lsd, const int* lcnt,
                                 const float* lrad, int cap, const DevGrid* const* g4, const float4* tgt4, int nt,
                                 int max_iter, const IcpSync* sy, int* done, unsigned long long* best, hipStream_t s) {
    if (ns <= 0 || nt <= 0 || max_iter <= 1) return hipSuccess;
    if (cap != ICP_LIST_CAP) return hipErrorInvalidValue;
    if (max_iter > ICP_MAX_ITER) return hipErrorInvalidValue;
    bsk::k_icp_iterations<<<icp_iter_blocks(ns), ICPN_THREADS, 0, s>>>(src0, ns, lst, lsd, lcnt, lrad, cap, icp_views(g4), tgt4,
                                                                      nt, max_iter, sy, done, best);
    return hipGetLastError();
}

}  // namespace bsh
