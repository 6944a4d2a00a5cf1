// icp.hip -- A11 point-to-point ICP on gfx950 (PCL IterativeClosestPoint defaults,
// src/lidar_odometry.cpp:291-297: CorrespondenceEstimation::determineCorrespondences, 1-NN, no
// distance cap; TransformationEstimationSVD; DefaultConvergenceCriteria). k_icp_loop runs the whole
// loop in one launch; k_icp_grid is one NN pass (the host loop, for source sets beyond the loop
// kernel's LDS). Exact: the packed key (float bits of d2 << 32 | target index) min picks
// the smallest squared distance, smallest index on ties (DESIGN.md convention for FLANN's
// traversal-dependent tie), independent of the reduction order.
#include <hip/hip_runtime.h>

#include "bshot_math.h"
#include "dev_cand.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

using bsh::IcpResult;

struct Xf16 {
    float m[16];
};

// One ICP iteration on hashed grids of the targets (built once per ICP call): a wave per source
// point searches balls of growing radius (g1: r1, 2 r1; g2: r2, 2 r2). Every target with d2 < rs^2
// is visited (for_candidates), so the smallest (d2 bits << 32 | index) key found inside the first
// non-empty ball is the global one, ties included: a target outside the ball has d2 >= rs^2 > the
// key's d2. A source with no target inside the largest ball (or non-finite) scans every target,
// the reference way. The step transform is applied with pcl::transformPointCloud's float expressions.
#define ICPG_WAVES 4
__global__ void __launch_bounds__(64 * ICPG_WAVES) k_icp_grid(const float* __restrict__ src_in, float* __restrict__ src_out,
                                                              Xf16 T, int apply, int ns, GridView g1, GridView g2,
                                                              float r1, float r2, const float4* __restrict__ tgt4, int nt,
                                                              unsigned long long* __restrict__ best_out) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
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

// ---- A11 as one launch: the whole ICP loop (<= max_iter iterations) in one workgroup.
// PCL IterativeClosestPoint with the reference's defaults (src/lidar_odometry.cpp:291-297): per
// iteration the exact 1-NN of every moved source point, Eigen::umeyama in float on the pairs
// (bm::umeyama_seq's sequential sums: the means, then the cross-covariance), final = step * final,
// and PCL's DefaultConvergenceCriteria (iteration cap, identity step, |delta mse| < 1e-12). The
// result equals the host loop's (ctx_icp with the k_icp_grid launches) bit for bit: the same NN
// keys, the same float / double expressions in the same order.
//
// The earlier design ran one NN launch per iteration and the Umeyama step on the host: 10
// dependent launch -> wait -> host round trips, each launch queued behind the lookahead's side-
// stream kernels (0.82 ms of the main thread's 2.2 ms sweep). Here the host
// launches once and waits once; the kernel needs one CU.
//
// NN: lane per source point. Ball radius rs = 1000, 2000, 4000, 8000 mm, each searched on the
// targets' grid whose cell is rs (<= 27 cells of the cube [q - rs, q + rs], cells farther than
// rs + 1 mm pruned in double, as cand_lookup): the smallest (d2 bits << 32 | index) key with
// d2 < rs^2 inside the first non-empty ball is the global minimum (any target outside the ball
// has d2 >= rs^2 > the key's d2), ties to the smallest index. Sources with no target inside
// 8000 mm (or non-finite ones) are queued and scanned against every target, a wave per source.
// LDS: source positions S[3][ns], matched targets D[3][ns], NN d2 E[ns], the brute-force queue.
#define ICPL_THREADS 1024
#define ICPL_WAVES (ICPL_THREADS / 64)

struct IcpGrids {
    GridView g[4];  // cells 1000, 2000, 4000, 8000 mm
};

__device__ __forceinline__ unsigned long long icp_lane_nn(const IcpGrids& G, float qx, float qy, float qz) {
#pragma unroll 1
    for (int L = 0; L < 4; ++L) {
        const GridView& g = G.g[L];
        const float rs = g.cell;
        const float rs2 = (float)((double)rs * (double)rs);
        const double c = (double)g.cell;
        const int x0 = (int)floor(((double)qx - rs) / c), x1 = (int)floor(((double)qx + rs) / c);
        const int y0 = (int)floor(((double)qy - rs) / c), y1 = (int)floor(((double)qy + rs) / c);
        const int z0 = (int)floor(((double)qz - rs) / c), z1 = (int)floor(((double)qz + rs) / c);
        const double lim = (double)rs + 1.0;
        unsigned long long m = ~0ull;
#pragma unroll 1
        for (int cx = x0; cx <= x1; ++cx) {
            const double bx0 = cx * c;
            const double dx = qx < bx0 ? bx0 - qx : (qx > bx0 + c ? qx - (bx0 + c) : 0.0);
#pragma unroll 1
            for (int cy = y0; cy <= y1; ++cy) {
                const double by0 = cy * c;
                const double dy = qy < by0 ? by0 - qy : (qy > by0 + c ? qy - (by0 + c) : 0.0);
#pragma unroll 1
                for (int cz = z0; cz <= z1; ++cz) {
                    const double bz0 = cz * c;
                    const double dz = qz < bz0 ? bz0 - qz : (qz > bz0 + c ? qz - (bz0 + c) : 0.0);
                    if (dx * dx + dy * dy + dz * dz > lim * lim) continue;
                    unsigned int st, cnt;
                    if (!grid_lookup(g, cell_key(cx, cy, cz), st, cnt)) continue;
                    for (unsigned int j = st; j < st + cnt; ++j) {
                        const float4 p = g.spts[j];
                        const float d2 = d2_flann(qx, qy, qz, p.x, p.y, p.z);
                        if (d2 < rs2) {
                            const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | __float_as_uint(p.w);
                            m = key < m ? key : m;
                        }
                    }
                }
            }
        }
        if (m != ~0ull) return m;
    }
    return ~0ull;
}

__global__ void __launch_bounds__(ICPL_THREADS) k_icp_loop(const float* __restrict__ src0, int ns, IcpGrids G,
                                                           const float4* __restrict__ tgt4, int nt, int max_iter,
                                                           IcpResult* __restrict__ out) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    extern __shared__ __attribute__((aligned(16))) float icl[];
    float* Sx = icl;
    float* Sy = Sx + ns;
    float* Sz = Sy + ns;
    float* Dx = Sz + ns;
    float* Dy = Dx + ns;
    float* Dz = Dy + ns;
    float* E = Dz + ns;
    int* bq = reinterpret_cast<int*>(E + ns);
    __shared__ float Ts[16], fin[16], means[6], sigma[9];
    __shared__ double mse_sh;
    __shared__ int nbq, done_sh;
    const int t = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = lane_id();
    for (int i = t; i < ns; i += ICPL_THREADS) {
        Sx[i] = src0[3 * i];
        Sy[i] = src0[3 * i + 1];
        Sz[i] = src0[3 * i + 2];
    }
    if (t < 16) fin[t] = (t % 5) == 0 ? 1.f : 0.f;
    double prev_mse = 1.7976931348623157e308;  // thread 0's
    int it = 0;
    const float one_over_n = 1.0f / (float)ns;
    while (true) {
        if (t == 0) nbq = 0;
        __syncthreads();
        // ---- 1-NN of every source (this iteration's positions)
        for (int i = t; i < ns; i += ICPL_THREADS) {
            const float qx = Sx[i], qy = Sy[i], qz = Sz[i];
            unsigned long long m = ~0ull;
            if (__builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz)) m = icp_lane_nn(G, qx, qy, qz);
            if (m == ~0ull) {
                bq[atomicAdd(&nbq, 1)] = i;
            } else {
                const float4 p = tgt4[(unsigned)(m & 0xFFFFFFFFu)];
                Dx[i] = p.x; Dy[i] = p.y; Dz[i] = p.z;
                E[i] = __uint_as_float((unsigned)(m >> 32));
            }
        }
        __syncthreads();
        // sources with no target within 8000 mm: every target, a wave per source
        for (int j = wave; j < nbq; j += ICPL_WAVES) {
            const int i = bq[j];
            const float qx = Sx[i], qy = Sy[i], qz = Sz[i];
            unsigned long long m = ~0ull;
            for (int u = lane; u < nt; u += 64) {
                const float4 p = tgt4[u];
                const float d2 = d2_flann(qx, qy, qz, p.x, p.y, p.z);
                const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)u;
                m = key < m ? key : m;
            }
            m = wave_min_u64(m);
            if (lane == 0) {
                const float4 p = tgt4[(unsigned)(m & 0xFFFFFFFFu)];
                Dx[i] = p.x; Dy[i] = p.y; Dz[i] = p.z;
                E[i] = __uint_as_float((unsigned)(m >> 32));
            }
        }
        __syncthreads();
        // ---- umeyama means (sequential from element 0) and the double mse sum of the NN d2
        if (wave == 0 && lane < 6) {
            const float* a = lane == 0 ? Sx : lane == 1 ? Sy : lane == 2 ? Sz : lane == 3 ? Dx : lane == 4 ? Dy : Dz;
            float acc = a[0];
            int i = 1;
            for (; i + 8 <= ns; i += 8) {
                const float a0 = a[i], a1 = a[i + 1], a2 = a[i + 2], a3 = a[i + 3];
                const float a4 = a[i + 4], a5 = a[i + 5], a6 = a[i + 6], a7 = a[i + 7];
                acc = acc + a0; acc = acc + a1; acc = acc + a2; acc = acc + a3;
                acc = acc + a4; acc = acc + a5; acc = acc + a6; acc = acc + a7;
            }
            for (; i < ns; ++i) acc = acc + a[i];
            means[lane] = acc * one_over_n;
        } else if (wave == 1 && lane == 0) {
            double ms = 0.0;
            int i = 0;
            for (; i + 8 <= ns; i += 8) {
                const float e0 = E[i], e1 = E[i + 1], e2 = E[i + 2], e3 = E[i + 3];
                const float e4 = E[i + 4], e5 = E[i + 5], e6 = E[i + 6], e7 = E[i + 7];
                ms += (double)e0; ms += (double)e1; ms += (double)e2; ms += (double)e3;
                ms += (double)e4; ms += (double)e5; ms += (double)e6; ms += (double)e7;
            }
            for (; i < ns; ++i) ms += (double)E[i];
            mse_sh = ms;
        }
        __syncthreads();
        // ---- cross-covariance acc[r][c] = sum (d_r - dm_r)(s_c - sm_c), sequential from element 0
        if (wave == 0 && lane < 9) {
            const int r = lane / 3, cc = lane % 3;
            const float* dv = r == 0 ? Dx : r == 1 ? Dy : Dz;
            const float* sv = cc == 0 ? Sx : cc == 1 ? Sy : Sz;
            const float dm = means[3 + r], smv = means[cc];
            float acc = (dv[0] - dm) * (sv[0] - smv);
            int i = 1;
            for (; i + 8 <= ns; i += 8) {
                float p[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) p[u] = (dv[i + u] - dm) * (sv[i + u] - smv);
#pragma unroll
                for (int u = 0; u < 8; ++u) acc = acc + p[u];
            }
            for (; i < ns; ++i) acc = acc + (dv[i] - dm) * (sv[i] - smv);
            sigma[lane] = acc * one_over_n;
        }
        __syncthreads();
        // ---- the step, the accumulated transform and PCL's convergence test (thread 0)
        if (t == 0) {
            const float sm3[3] = {means[0], means[1], means[2]}, dm3[3] = {means[3], means[4], means[5]};
            float sg[9], T[16];
#pragma unroll
            for (int q = 0; q < 9; ++q) sg[q] = sigma[q];
            bm::umeyama_finish<float>(sg, sm3, dm3, T);
            float F[16];
            for (int r = 0; r < 4; ++r)
                for (int cc = 0; cc < 4; ++cc)
                    F[r * 4 + cc] = ((T[r * 4] * fin[cc] + T[r * 4 + 1] * fin[4 + cc]) + T[r * 4 + 2] * fin[8 + cc]) +
                                    T[r * 4 + 3] * fin[12 + cc];
            for (int q = 0; q < 16; ++q) { fin[q] = F[q]; Ts[q] = T[q]; }
            ++it;
            int done = 0;
            if (it >= max_iter) {
                done = 1;
            } else {
                const double cos_angle = 0.5 * (double)(((T[0] + T[5]) + T[10]) - 1.0f);
                const double tsq = (double)((T[3] * T[3] + T[7] * T[7]) + T[11] * T[11]);
                if (cos_angle >= 1.0 && tsq <= 0.0) {
                    done = 1;
                } else {
                    const double mse = mse_sh / (double)ns;
                    if (fabs(mse - prev_mse) < 1e-12) done = 1;
                    prev_mse = mse;
                }
            }
            done_sh = done;
        }
        __syncthreads();
        if (done_sh) break;
        // ---- move the sources by the step (pcl::transformPointCloud's float expression)
        for (int i = t; i < ns; i += ICPL_THREADS) {
            const float x = Sx[i], y = Sy[i], z = Sz[i];
            Sx[i] = ((Ts[0] * x + Ts[1] * y) + Ts[2] * z) + Ts[3];
            Sy[i] = ((Ts[4] * x + Ts[5] * y) + Ts[6] * z) + Ts[7];
            Sz[i] = ((Ts[8] * x + Ts[9] * y) + Ts[10] * z) + Ts[11];
        }
    }
    if (t < 16) out->fin[t] = fin[t];
    if (t == 0) out->iters = it;
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
                                                        g2.cell, tgt4, nt, best_out);
    return hipGetLastError();
}

size_t icp_loop_lds(int ns) { return (size_t)ns * 8 * sizeof(float); }

hipError_t launch_icp_loop(const float* src0, int ns, const DevGrid* const* g4, const float4* tgt4, int nt, int max_iter,
                           IcpResult* out, hipStream_t s) {
    if (ns < 3 || nt <= 0 || max_iter < 1 || ns > ICP_LOOP_MAXN) return hipErrorInvalidValue;
    bsk::IcpGrids G;
    for (int L = 0; L < 4; ++L) G.g[L] = g4[L]->view();
    static const hipError_t attr = hipFuncSetAttribute((const void*)bsk::k_icp_loop,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)icp_loop_lds(ICP_LOOP_MAXN));
    if (attr != hipSuccess) return attr;
    bsk::k_icp_loop<<<1, ICPL_THREADS, icp_loop_lds(ns), s>>>(src0, ns, G, tgt4, nt, max_iter, out);
    return hipGetLastError();
}

}  // namespace bsh
