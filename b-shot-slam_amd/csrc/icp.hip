// icp.hip -- A11 nearest-neighbour step of point-to-point ICP on gfx950 (PCL IterativeClosestPoint
// defaults, src/lidar_odometry.cpp:291-297: CorrespondenceEstimation::determineCorrespondences,
// 1-NN, no distance cap). Exact: the packed key (float bits of d2 << 32 | target index) min picks
// the smallest squared distance, smallest index on ties (DESIGN.md convention for FLANN's
// traversal-dependent tie), independent of the reduction order.
#include <hip/hip_runtime.h>

#include "bshot_math.h"
#include "dev_cand.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

using bsh::IcpState;

#define ICP_THREADS 256
// small LDS tile (4 KB): ICP runs on the main stream beside LDS-heavy side-stream kernels
#define ICP_TILE 256

struct Xf16 {
    float m[16];
};

// One ICP iteration, LDS-tiled: a workgroup holds 256 source points (a thread each) and one
// contiguous span of the targets (blockIdx.y), streamed through LDS in tiles of 512 float4 that
// every lane reads by broadcast, so each target is fetched once per workgroup instead of once per
// source point. The span minima meet in `part`; the last workgroup of a source block (agent-scope
// counter, reset by that workgroup) reduces them and stores the packed (d2 bits << 32 | index)
// minimum straight into best_out (pinned host memory), as k_icp_wave does.
#define ICPT_TILE 512
__global__ void __launch_bounds__(256) k_icp_tile(const float* __restrict__ src_in, float* __restrict__ src_out,
                                                  Xf16 T, int apply, int ns, const float* __restrict__ tgt, int nt,
                                                  int span, unsigned long long* __restrict__ part,
                                                  unsigned int* __restrict__ cnt,
                                                  unsigned long long* __restrict__ best_out) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    __shared__ float4 tt[ICPT_TILE];
    __shared__ int last;
    const int t = threadIdx.x, i = blockIdx.x * 256 + t;
    const int S = gridDim.y, sp = blockIdx.y;
    float qx = 0.f, qy = 0.f, qz = 0.f;
    if (i < ns) {
        const float x = src_in[3 * i], y = src_in[3 * i + 1], z = src_in[3 * i + 2];
        qx = x; qy = y; qz = z;
        if (apply) {
            qx = ((T.m[0] * x + T.m[1] * y) + T.m[2] * z) + T.m[3];
            qy = ((T.m[4] * x + T.m[5] * y) + T.m[6] * z) + T.m[7];
            qz = ((T.m[8] * x + T.m[9] * y) + T.m[10] * z) + T.m[11];
        }
        if (sp == 0) {
            src_out[3 * i] = qx; src_out[3 * i + 1] = qy; src_out[3 * i + 2] = qz;
        }
    }
    unsigned long long m = ~0ull;
    const int r0 = sp * span, r1 = min(nt, r0 + span);
    for (int b = r0; b < r1; b += ICPT_TILE) {
        const int nb = min(ICPT_TILE, r1 - b);
        __syncthreads();
        for (int u = t; u < nb; u += 256) {
            const float* p3 = tgt + 3 * (size_t)(b + u);
            tt[u] = make_float4(p3[0], p3[1], p3[2], 0.f);
        }
        __syncthreads();
        if (i < ns) {
            int u = 0;
            for (; u + 4 <= nb; u += 4) {
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const float4 p = tt[u + v];
                    const float d2 = d2_flann(qx, qy, qz, p.x, p.y, p.z);
                    const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)(b + u + v);
                    m = key < m ? key : m;
                }
            }
            for (; u < nb; ++u) {
                const float4 p = tt[u];
                const float d2 = d2_flann(qx, qy, qz, p.x, p.y, p.z);
                const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)(b + u);
                m = key < m ? key : m;
            }
        }
    }
    if (S == 1) {
        if (i < ns) best_out[i] = m;
        return;
    }
    if (i < ns) __hip_atomic_store(&part[(size_t)sp * ns + i], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (t == 0)
        last = __hip_atomic_fetch_add(&cnt[blockIdx.x], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(S - 1);
    __syncthreads();
    if (!last) return;
    if (i < ns) {
        unsigned long long r = ~0ull;
        for (int s2 = 0; s2 < S; ++s2) {
            const unsigned long long v =
                __hip_atomic_load(&part[(size_t)s2 * ns + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            r = v < r ? v : r;
        }
        best_out[i] = r;
    }
    if (t == 0) __hip_atomic_store(&cnt[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One ICP iteration on hashed grids of the targets (built once per ICP call): a wave per source
// point searches balls of growing radius (g1: r1, 2 r1; g2: r2, 2 r2). Every target with d2 < rs^2
// is visited (for_candidates), so the smallest (d2 bits << 32 | index) key found inside the first
// non-empty ball is the global one, ties included: a target outside the ball has d2 >= rs^2 > the
// key's d2. A source with no target inside the largest ball (or non-finite) scans every target,
// exactly as k_icp_tile. The step transform is applied with k_icp_tile's float expressions.
#define ICPG_WAVES 4
__global__ void __launch_bounds__(64 * ICPG_WAVES) k_icp_grid(const float* __restrict__ src_in, float* __restrict__ src_out,
                                                              Xf16 T, int apply, int ns, GridView g1, GridView g2,
                                                              float r1, float r2, const float4* __restrict__ tgt4, int nt,
                                                              unsigned long long* __restrict__ best_out,
                                                              const IcpState* __restrict__ st) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    // device-resident loop (st != null): the step transform and whether to apply it come from the
    // loop state; a converged loop's remaining launches return at once
    if (st) {
        if (st->done) return;
        apply = st->it > 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) T.m[q] = st->T[q];
    }
    __shared__ CandLds cl[ICPG_WAVES];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    CandLds* cs = &cl[wave];
    cand_init(cs);
    for (int i = blockIdx.x * ICPG_WAVES + wave; i < ns; i += gridDim.x * ICPG_WAVES) {
        const float x = src_in[3 * i], y = src_in[3 * i + 1], z = src_in[3 * i + 2];
        float qx = x, qy = y, qz = z;
        if (apply) {
            qx = ((T.m[0] * x + T.m[1] * y) + T.m[2] * z) + T.m[3];
            qy = ((T.m[4] * x + T.m[5] * y) + T.m[6] * z) + T.m[7];
            qz = ((T.m[8] * x + T.m[9] * y) + T.m[10] * z) + T.m[11];
        }
        if (lane == 0) { src_out[3 * i] = qx; src_out[3 * i + 1] = qy; src_out[3 * i + 2] = qz; }
        unsigned long long m = ~0ull;
        const bool fin = __builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz);
        if (fin) {
#pragma unroll 1
            for (int step = 0; step < 4; ++step) {
                const float rs = (step & 1) ? 2.f * ((step < 2) ? r1 : r2) : ((step < 2) ? r1 : r2);
                const float rs2 = (float)((double)rs * (double)rs);
                for_candidates((step < 2) ? g1 : g2, cs, qx, qy, qz, rs, rs2, [&](bool v, float d2, unsigned int idx) {
                    if (v) {
                        const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | idx;
                        m = key < m ? key : m;
                    }
                });
                m = wave_min_u64(m);
                if (m != ~0ull) break;
            }
        }
        if (m == ~0ull) {
            for (int j = lane; j < nt; j += 64) {
                const float4 p = tgt4[j];
                const float d2 = d2_flann(qx, qy, qz, p.x, p.y, p.z);
                const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)j;
                m = key < m ? key : m;
            }
            m = wave_min_u64(m);
        }
        if (lane == 0) best_out[i] = m;
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- device-resident ICP loop: the host enqueues max_iter (NN, update) pairs and syncs once.
// The update kernel restates ctx_icp's host step exactly (bg::umeyama<float> sequential sums,
// bm::umeyama_finish, bg::mul, PCL's convergence tests); once converged, later launches return.

// one NN pass with the state's step T (applied when it > 0)
__global__ void __launch_bounds__(ICP_THREADS) k_icp_nn_dev(const float* __restrict__ src_in, float* __restrict__ src_out,
                                                            const IcpState* __restrict__ st, int ns,
                                                            const float4* __restrict__ tgt, int nt, int tile,
                                                            unsigned long long* __restrict__ best,
                                                            unsigned long long* __restrict__ best_next) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    if (st->done) return;
    __shared__ float4 tt[ICP_TILE];
    const int t = threadIdx.x;
    const int i = blockIdx.x * ICP_THREADS + t;
    const int r0 = blockIdx.y * tile, r1 = min(nt, r0 + tile);
    const bool apply = st->it > 0;
    float qx = 0.f, qy = 0.f, qz = 0.f;
    if (i < ns) {
        const float x = src_in[3 * i], y = src_in[3 * i + 1], z = src_in[3 * i + 2];
        if (apply) {
            const float* T = st->T;
            qx = ((T[0] * x + T[1] * y) + T[2] * z) + T[3];
            qy = ((T[4] * x + T[5] * y) + T[6] * z) + T[7];
            qz = ((T[8] * x + T[9] * y) + T[10] * z) + T[11];
        } else {
            qx = x; qy = y; qz = z;
        }
        if (blockIdx.y == 0) {
            src_out[3 * i] = qx; src_out[3 * i + 1] = qy; src_out[3 * i + 2] = qz;
            best_next[i] = ~0ull;
        }
    }
    unsigned long long m = ~0ull;
    for (int s0 = r0; s0 < r1; s0 += ICP_TILE) {
        const int cnt = min(ICP_TILE, r1 - s0);
        __syncthreads();
        for (int j = t; j < cnt; j += ICP_THREADS) tt[j] = tgt[s0 + j];
        __syncthreads();
        for (int j = 0; j < cnt; ++j) {
            const float4 p = tt[j];
            const float d2 = d2_flann(qx, qy, qz, p.x, p.y, p.z);
            const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)(s0 + j);
            m = key < m ? key : m;
        }
    }
    if (i < ns) atomicMin(&best[i], m);
}

#define ICPU_TILE 512
#define ICPU_THREADS 256

// sequential float chain acc = acc + a[i], i in [i0, n) (8 independent LDS loads per step)
__device__ __forceinline__ float chain_f(float acc, const float* a, int i0, int n) {
    int i = i0;
    for (; i + 8 <= n; i += 8) {
        const float a0 = a[i], a1 = a[i + 1], a2 = a[i + 2], a3 = a[i + 3];
        const float a4 = a[i + 4], a5 = a[i + 5], a6 = a[i + 6], a7 = a[i + 7];
        acc = acc + a0; acc = acc + a1; acc = acc + a2; acc = acc + a3;
        acc = acc + a4; acc = acc + a5; acc = acc + a6; acc = acc + a7;
    }
    for (; i < n; ++i) acc = acc + a[i];
    return acc;
}

// Umeyama step + convergence test, one workgroup. cur: the moved source (ns x 3, this iteration's
// NN queries), best: their NN keys. Tiles of ICPU_TILE points are staged in LDS as
// S[3][tile] (source), D[3][tile] (matched target) and, for the covariance, P[9][tile] =
// (d_r - dm_r)(s_c - sm_c); lanes of wave 0 run the 6 mean chains and then the 9 covariance chains,
// lane 0 of wave 1 the double mse chain.
__global__ void __launch_bounds__(ICPU_THREADS) k_icp_update(IcpState* __restrict__ st, const float* __restrict__ cur,
                                                             const float4* __restrict__ tgt,
                                                             const unsigned long long* __restrict__ best, int ns) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    if (st->done) return;
    __shared__ float S[3][ICPU_TILE], D[3][ICPU_TILE], P[9][ICPU_TILE], E[ICPU_TILE];
    __shared__ float means[6];
    __shared__ double mse_sh;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    auto stage = [&](int b0, int cnt) {
        for (int j = t; j < cnt; j += ICPU_THREADS) {
            const int i = b0 + j;
            S[0][j] = cur[3 * i]; S[1][j] = cur[3 * i + 1]; S[2][j] = cur[3 * i + 2];
            const unsigned long long key = best[i];
            const float4 q = tgt[(unsigned)(key & 0xFFFFFFFFu)];
            D[0][j] = q.x; D[1][j] = q.y; D[2][j] = q.z;
            E[j] = __uint_as_float((unsigned)(key >> 32));
        }
    };
    // ---- means (bg::umeyama: ss = src[d]; ss = ss + src[i*3+d]) and the mse sum
    float acc = 0.f;
    double msum = 0.0;
    for (int b0 = 0; b0 < ns; b0 += ICPU_TILE) {
        const int cnt = min(ICPU_TILE, ns - b0);
        __syncthreads();
        stage(b0, cnt);
        __syncthreads();
        if (wave == 0 && lane < 6) {
            const float* a = lane < 3 ? S[lane] : D[lane - 3];
            if (b0 == 0) acc = chain_f(a[0], a, 1, cnt);
            else acc = chain_f(acc, a, 0, cnt);
        } else if (wave == 1 && lane == 0) {
            int j = 0;
            for (; j + 8 <= cnt; j += 8) {
                const float e0 = E[j], e1 = E[j + 1], e2 = E[j + 2], e3 = E[j + 3];
                const float e4 = E[j + 4], e5 = E[j + 5], e6 = E[j + 6], e7 = E[j + 7];
                msum += (double)e0; msum += (double)e1; msum += (double)e2; msum += (double)e3;
                msum += (double)e4; msum += (double)e5; msum += (double)e6; msum += (double)e7;
            }
            for (; j < cnt; ++j) msum += (double)E[j];
        }
    }
    const float one_over_n = 1.0f / (float)ns;
    if (wave == 0 && lane < 6) means[lane] = acc * one_over_n;
    if (wave == 1 && lane == 0) mse_sh = msum;
    __syncthreads();
    const float sm0 = means[0], sm1 = means[1], sm2 = means[2], dm0 = means[3], dm1 = means[4], dm2 = means[5];
    // ---- cross-covariance: acc = (d_r - dm_r)(s_c - sm_c) at i = 0, then acc = acc + ... for i >= 1
    float sacc = 0.f;
    for (int b0 = 0; b0 < ns; b0 += ICPU_TILE) {
        const int cnt = min(ICPU_TILE, ns - b0);
        __syncthreads();
        stage(b0, cnt);
        __syncthreads();
        for (int j = t; j < cnt; j += ICPU_THREADS) {
            const float s0 = S[0][j] - sm0, s1 = S[1][j] - sm1, s2 = S[2][j] - sm2;
            const float d0 = D[0][j] - dm0, d1 = D[1][j] - dm1, d2 = D[2][j] - dm2;
            P[0][j] = d0 * s0; P[1][j] = d0 * s1; P[2][j] = d0 * s2;
            P[3][j] = d1 * s0; P[4][j] = d1 * s1; P[5][j] = d1 * s2;
            P[6][j] = d2 * s0; P[7][j] = d2 * s1; P[8][j] = d2 * s2;
        }
        __syncthreads();
        if (wave == 0 && lane < 9) {
            if (b0 == 0) sacc = chain_f(P[lane][0], P[lane], 1, cnt);
            else sacc = chain_f(sacc, P[lane], 0, cnt);
        }
    }
    __shared__ float sigma[9];
    if (wave == 0 && lane < 9) sigma[lane] = sacc * one_over_n;
    __syncthreads();
    if (t == 0) {
        const float sm[3] = {sm0, sm1, sm2}, dm[3] = {dm0, dm1, dm2};
        float sg[9], Ts[16];
        for (int q = 0; q < 9; ++q) sg[q] = sigma[q];
        bm::umeyama_finish<float>(sg, sm, dm, Ts);
        // fin = Ts * fin (bg::mul order)
        float F[16];
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c)
                F[r * 4 + c] = ((Ts[r * 4] * st->fin[c] + Ts[r * 4 + 1] * st->fin[4 + c]) +
                                Ts[r * 4 + 2] * st->fin[8 + c]) + Ts[r * 4 + 3] * st->fin[12 + c];
        for (int q = 0; q < 16; ++q) { st->fin[q] = F[q]; st->T[q] = Ts[q]; }
        const int it = st->it + 1;
        st->it = it;
        int done = 0;
        if (it >= st->max_iter) {
            done = 1;
        } else {
            // PCL DefaultConvergenceCriteria with the reference's epsilons (ctx_icp)
            const double cos_angle = 0.5 * (double)(((Ts[0] + Ts[5]) + Ts[10]) - 1.0f);
            const double tsq = (double)((Ts[3] * Ts[3] + Ts[7] * Ts[7]) + Ts[11] * Ts[11]);
            if (cos_angle >= 1.0 && tsq <= 0.0) {
                done = 1;
            } else {
                const double mse = mse_sh / (double)ns;
                if (fabs(mse - st->prev_mse) < 1e-12) done = 1;
                st->prev_mse = mse;
            }
        }
        st->done = done;
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

__global__ void k_fill_u64b(unsigned long long* p, int n, unsigned long long v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
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

hipError_t launch_icp_grid(const float* src_in, float* src_out, const float* T16, int apply, int ns, const DevGrid& g1,
                           const DevGrid& g2, const float4* tgt4, int nt, unsigned long long* best_out, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    bsk::Xf16 T;
    for (int i = 0; i < 16; ++i) T.m[i] = T16 ? T16[i] : ((i % 5) == 0 ? 1.f : 0.f);
    const int blocks = (ns + ICPG_WAVES - 1) / ICPG_WAVES;
    bsk::k_icp_grid<<<blocks, 64 * ICPG_WAVES, 0, s>>>(src_in, src_out, T, apply, ns, g1.view(), g2.view(), g1.cell,
                                                        g2.cell, tgt4, nt, best_out, nullptr);
    return hipGetLastError();
}

hipError_t launch_icp_grid_dev(const float* src_in, float* src_out, IcpState* st, int ns, const DevGrid& g1,
                               const DevGrid& g2, const float4* tgt4, int nt, unsigned long long* best, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    bsk::Xf16 T;
    for (int i = 0; i < 16; ++i) T.m[i] = (i % 5) == 0 ? 1.f : 0.f;
    const int blocks = (ns + ICPG_WAVES - 1) / ICPG_WAVES;
    bsk::k_icp_grid<<<blocks, 64 * ICPG_WAVES, 0, s>>>(src_in, src_out, T, 0, ns, g1.view(), g2.view(), g1.cell, g2.cell,
                                                        tgt4, nt, best, st);
    bsk::k_icp_update<<<1, ICPU_THREADS, 0, s>>>(st, src_out, tgt4, best, ns);
    return hipGetLastError();
}

// spans: about 1024 workgroups in all, each span >= 256 targets; part holds S x ns keys, cnt one
// counter per 256-source block (zero on entry, left zero)
hipError_t launch_icp_tile(const float* src_in, float* src_out, const float* T16, int apply, int ns, const float* tgt,
                           int nt, unsigned long long* part, int part_cap, unsigned int* cnt,
                           unsigned long long* best_out, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    bsk::Xf16 T;
    for (int i = 0; i < 16; ++i) T.m[i] = T16 ? T16[i] : ((i % 5) == 0 ? 1.f : 0.f);
    const int qb = (ns + 255) / 256;
    int S = icp_tile_splits(ns, nt);
    if ((long long)S * ns > part_cap) return hipErrorInvalidValue;
    const int span = (nt + S - 1) / S;
    S = (nt + span - 1) / span;
    bsk::k_icp_tile<<<dim3(qb, S), 256, 0, s>>>(src_in, src_out, T, apply, ns, tgt, nt, span, part, cnt, best_out);
    return hipGetLastError();
}

int icp_tile_splits(int ns, int nt) {
    const int qb = (ns + 255) / 256;
    int S = (1024 + qb - 1) / qb;
    const int smax = (nt + 255) / 256;
    if (S > smax) S = smax;
    return S < 1 ? 1 : S;
}

hipError_t launch_icp_dev(const float* src_in, float* src_out, IcpState* st, int ns, const float4* tgt, int nt,
                          unsigned long long* best, unsigned long long* best_next, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    const int qb = (ns + ICP_THREADS - 1) / ICP_THREADS;
    int splits = (1024 + qb - 1) / qb;
    int tile = (nt + splits - 1) / splits;
    if (tile < 256) tile = 256;
    splits = (nt + tile - 1) / tile;
    bsk::k_icp_nn_dev<<<dim3(qb, splits), ICP_THREADS, 0, s>>>(src_in, src_out, st, ns, tgt, nt, tile, best,
                                                                best_next);
    bsk::k_icp_update<<<1, ICPU_THREADS, 0, s>>>(st, src_out, tgt, best, ns);
    return hipGetLastError();
}

}  // namespace bsh
