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
// The loop (k_icp_loop, one workgroup): each iteration's Umeyama + convergence test, then the sources
// move rigidly by the step; a source's NN among its list is the global NN whenever
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
                                                              unsigned long long* __restrict__ best_out) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    __shared__ CandLds cl[ICP_WAVES];
    __shared__ unsigned long long skl[ICP_WAVES][ICP_LIST_CAP];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    CandLds* cs = &cl[wave];
    cand_init(cs);
    for (int i = blockIdx.x * ICP_WAVES + wave; i < ns; i += gridDim.x * ICP_WAVES) {
        const float qx = src0[3 * i], qy = src0[3 * i + 1], qz = src0[3 * i + 2];
        const unsigned long long m = icp_wave_nn(G, cs, qx, qy, qz, tgt4, nt);
        if (lane == 0) best_out[i] = m;
        int count;
        float R;
        icp_build_list(G, cs, qx, qy, qz, m, tgt4, lst + i, lsd + i, ns, cap, skl[wave], &count, &R);  // entry e at [e * ns + i]
        if (lane == 0) {
            lcnt[i] = count;
            lrad[i] = R;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// The whole of PCL's loop after iteration 0's neighbours, on the device (one launch, one workgroup of
// ICPL_THREADS): per iteration the float Umeyama of (current sources, their NN targets), PCL's
// convergence test, then every source moved by the step and its exact 1-NN found for the next
// iteration. One workgroup keeps every hand-over inside one CU (LDS + __syncthreads): no host round
// trip, no grid barrier, no cross-XCD coherence traffic, and nothing waits for another workgroup to
// be scheduled.
//
// Umeyama (bm::umeyama_seq<float>, Eigen::umeyama's order): the means are 6 sequential float sums in
// source order, the cross-covariance 9 sequential sums of (d_r - dm_r)(s_c - sm_c), each sum on its
// own lane of wave 0 (the sums' own orders are the host's, so the bits are); the per-source terms
// are staged in LDS as 7 arrays (s xyz, d xyz, d2), centred in place by the whole workgroup between
// the two passes. PCL's MSE (a sequential double sum of the keys' d2) runs on wave 1 meanwhile.
// Sources beyond ICPL_CH are staged chunk by chunk from HBM (rec_g) instead.
//
// Neighbours: a thread per source scans the source's candidate list (k_icp_lists) while the bound
// proves the list's best global (dm + |q - q0| < R with float slack); the others are queued and the
// exact grid search runs on ICPL_SW waves (a wave per queued source), which also rebuilds the
// source's list around its current position.
#define ICPL_THREADS 512
#define ICPL_SW 8      // waves that run the queued grid searches
#define ICPL_CH 2048   // sources whose Umeyama terms are staged in LDS at once (7 floats each)

__global__ void __launch_bounds__(ICPL_THREADS) k_icp_loop(const float* __restrict__ src0, int ns, float4* lst, float* lsd,
                                                           int* lcnt, float* lrad, int cap, IcpGrids G,
                                                           const float4* __restrict__ tgt4, int nt, int max_iter,
                                                           const unsigned long long* __restrict__ best0,
                                                           float4* __restrict__ pos, float4* __restrict__ lcen,
                                                           int* __restrict__ queue, float* __restrict__ rec_g,
                                                           bsh::IcpOut* out, int seq) {
    extern __shared__ __attribute__((aligned(16))) float rec[];  // 7 x chs floats
    __shared__ CandLds cl[ICPL_SW];
    __shared__ unsigned long long skl[ICPL_SW][ICP_LIST_CAP];
    __shared__ float sT[16];
    __shared__ float smean[6];
    __shared__ float sacc[9];
    __shared__ double smse;
    __shared__ int sstop, nq;
    const int tid = threadIdx.x, lane = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool big = ns > ICPL_CH;
    const int chs = big ? ICPL_CH : ((ns + 3) & ~3);  // LDS row stride (16-B aligned rows)
    if (wave < ICPL_SW) cand_init(&cl[wave]);
    // record c of source i: LDS row c (small) or HBM row c (big: staged per chunk)
    auto put = [&](int c, int i, float v) {
        if (big) rec_g[(size_t)c * ns + i] = v;
        else rec[c * chs + i] = v;
    };
    // iteration 0: the sources as given, the keys of k_icp_lists
    for (int i = tid; i < ns; i += ICPL_THREADS) {
        const float x = src0[3 * i], y = src0[3 * i + 1], z = src0[3 * i + 2];
        pos[i] = make_float4(x, y, z, 0.f);
        lcen[i] = make_float4(x, y, z, lrad[i]);
        const unsigned long long m = best0[i];
        const float4 t = tgt4[(unsigned)(m & 0xFFFFFFFFu)];
        put(0, i, x); put(1, i, y); put(2, i, z);
        put(3, i, t.x); put(4, i, t.y); put(5, i, t.z);
        put(6, i, __uint_as_float((unsigned)(m >> 32)));
    }
    // thread 0's loop state: the composed transform (LDS), the previous MSE
    __shared__ float fin[16];
    if (tid < 16) fin[tid] = (tid % 5 == 0) ? 1.f : 0.f;
    double prev_mse = 1.7976931348623157e308;
    const float one_over_n = 1.f / (float)ns;
    int it = 0;
    __syncthreads();
    while (true) {
        // ---- means: lanes 0..5 of wave 0, source order (the first element starts the sum)
        float acc = 0.f;
        for (int c0 = 0; c0 < ns; c0 += chs) {
            const int cn = ns - c0 < chs ? ns - c0 : chs;
            if (big) {
                __syncthreads();
                for (int t = tid; t < 7 * cn; t += ICPL_THREADS) {
                    const int c = t / cn, k = t - c * cn;
                    rec[c * chs + k] = rec_g[(size_t)c * ns + c0 + k];
                }
                __syncthreads();
            }
            if (wave == 0 && lane < 6) {
                const float* a = rec + lane * chs;
                int k = 0;
                if (c0 == 0) { acc = a[0]; k = 1; }
                for (; k < cn && (k & 3); ++k) acc = acc + a[k];
                for (; k + 4 <= cn; k += 4) {
                    const float4 v = *reinterpret_cast<const float4*>(a + k);
                    acc = acc + v.x; acc = acc + v.y; acc = acc + v.z; acc = acc + v.w;
                }
                for (; k < cn; ++k) acc = acc + a[k];
            }
        }
        if (wave == 0 && lane < 6) smean[lane] = acc * one_over_n;
        __syncthreads();
        // ---- cross-covariance (wave 0, lane r * 3 + c) and PCL's MSE (wave 1, lane 0)
        const float sm0 = smean[0], sm1 = smean[1], sm2 = smean[2], dm0 = smean[3], dm1 = smean[4], dm2 = smean[5];
        float cov = 0.f;
        double mse = 0.0;
        for (int c0 = 0; c0 < ns; c0 += chs) {
            const int cn = ns - c0 < chs ? ns - c0 : chs;
            if (big) {
                __syncthreads();
                for (int t = tid; t < 7 * cn; t += ICPL_THREADS) {
                    const int c = t / cn, k = t - c * cn;
                    rec[c * chs + k] = rec_g[(size_t)c * ns + c0 + k];
                }
                __syncthreads();
            }
            // centre in place: s - sm, d - dm (the host's s0..s2, d0..d2)
            for (int t = tid; t < 6 * cn; t += ICPL_THREADS) {
                const int c = t / cn, k = t - c * cn;
                const float m = c == 0 ? sm0 : c == 1 ? sm1 : c == 2 ? sm2 : c == 3 ? dm0 : c == 4 ? dm1 : dm2;
                rec[c * chs + k] = rec[c * chs + k] - m;
            }
            __syncthreads();
            if (wave == 0 && lane < 9) {
                const float* e = rec + (3 + lane / 3) * chs;  // d_r - dm_r
                const float* f = rec + (lane % 3) * chs;      // s_c - sm_c
                int k = 0;
                if (c0 == 0) { cov = e[0] * f[0]; k = 1; }
                for (; k < cn && (k & 3); ++k) cov = cov + e[k] * f[k];
                for (; k + 4 <= cn; k += 4) {
                    const float4 u = *reinterpret_cast<const float4*>(e + k);
                    const float4 v = *reinterpret_cast<const float4*>(f + k);
                    const float p0 = u.x * v.x, p1 = u.y * v.y, p2 = u.z * v.z, p3 = u.w * v.w;
                    cov = cov + p0; cov = cov + p1; cov = cov + p2; cov = cov + p3;
                }
                for (; k < cn; ++k) cov = cov + e[k] * f[k];
            } else if (wave == 1 && lane == 0) {
                const float* d2 = rec + 6 * chs;
                int k = 0;
                for (; k < cn && (k & 3); ++k) mse += (double)d2[k];
                for (; k + 4 <= cn; k += 4) {
                    const float4 v = *reinterpret_cast<const float4*>(d2 + k);
                    mse += (double)v.x; mse += (double)v.y; mse += (double)v.z; mse += (double)v.w;
                }
                for (; k < cn; ++k) mse += (double)d2[k];
            }
        }
        if (wave == 0 && lane < 9) sacc[lane] = cov;
        if (wave == 1 && lane == 0) smse = mse;
        __syncthreads();
        // ---- the step, PCL's convergence test (the host loop's order: the step is applied and
        // composed first, then max_iter, the transformation epsilon and the MSE epsilon)
        if (tid == 0) {
            float sigma[9], sm[3] = {sm0, sm1, sm2}, dm[3] = {dm0, dm1, dm2}, o[16];
#pragma unroll
            for (int u = 0; u < 9; ++u) sigma[u] = sacc[u] * one_over_n;
            bm::umeyama_finish<float>(sigma, sm, dm, o);
            float f2[16];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    f2[r * 4 + c] = ((o[r * 4] * fin[c] + o[r * 4 + 1] * fin[4 + c]) + o[r * 4 + 2] * fin[8 + c]) +
                                    o[r * 4 + 3] * fin[12 + c];
#pragma unroll
            for (int u = 0; u < 16; ++u) { fin[u] = f2[u]; sT[u] = o[u]; }
            ++it;
            int stop = it >= max_iter;
            if (!stop) {
                const double cos_angle = 0.5 * (double)(((o[0] + o[5]) + o[10]) - 1.0f);
                const double tsq = (double)((o[3] * o[3] + o[7] * o[7]) + o[11] * o[11]);
                if (cos_angle >= 1.0 && tsq <= 0.0) stop = 1;
            }
            if (!stop) {
                const double m = smse / (double)ns;
                if (__builtin_fabs(m - prev_mse) < 1e-12) stop = 1;
                prev_mse = m;
            }
            sstop = stop;
            nq = 0;
        }
        __syncthreads();
        if (sstop) break;  // (it, fin and prev_mse live in thread 0)
        float T[12];
#pragma unroll
        for (int u = 0; u < 12; ++u) T[u] = sT[u];
        // ---- every source moved by the step (pcl::transformPointCloud's float expression, as the
        // host's bg::xform), its NN from its list when the bound proves it global, else queued
        for (int i = tid; i < ns; i += ICPL_THREADS) {
            const float4 p = pos[i];
            const float qx = ((T[0] * p.x + T[1] * p.y) + T[2] * p.z) + T[3];
            const float qy = ((T[4] * p.x + T[5] * p.y) + T[6] * p.z) + T[7];
            const float qz = ((T[8] * p.x + T[9] * p.y) + T[10] * p.z) + T[11];
            pos[i] = make_float4(qx, qy, qz, 0.f);
            const float4 c0 = lcen[i];
            const int n = lcnt[i];
            const float R = c0.w;
            bool ok = false;
            unsigned long long m = ~0ull;
            float4 best = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n >= 0 && __builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz)) {
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
                    const double dm = sqrt((double)__uint_as_float((unsigned)(m >> 32)));
                    ok = dm * (1.0 + 1e-5) + delta + 1.0 < (double)R * (1.0 - 1e-5);
                }
            }
            put(0, i, qx); put(1, i, qy); put(2, i, qz);
            if (ok) {
                put(3, i, best.x); put(4, i, best.y); put(5, i, best.z);
                put(6, i, __uint_as_float((unsigned)(m >> 32)));
            } else {
                queue[atomicAdd(&nq, 1)] = i;
            }
        }
        __syncthreads();
        // ---- the queued sources: exact grid search + a new list around the current position
        const int nqueued = nq;
        if (wave < ICPL_SW) {
            for (int t = wave; t < nqueued; t += ICPL_SW) {
                const int qi = queue[t];
                const float4 q = pos[qi];
                const unsigned long long m = icp_wave_nn(G, &cl[wave], q.x, q.y, q.z, tgt4, nt);
                int cnt2;
                float R2;
                icp_build_list(G, &cl[wave], q.x, q.y, q.z, m, tgt4, lst + qi, lsd + qi, ns, cap, skl[wave], &cnt2, &R2);
                if (lane == 0) {
                    const float4 tp = tgt4[(unsigned)(m & 0xFFFFFFFFu)];
                    put(3, qi, tp.x); put(4, qi, tp.y); put(5, qi, tp.z);
                    put(6, qi, __uint_as_float((unsigned)(m >> 32)));
                    lcnt[qi] = cnt2;
                    lcen[qi] = make_float4(q.x, q.y, q.z, R2);
                }
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
#pragma unroll
        for (int u = 0; u < 16; ++u) __hip_atomic_store(&out->T[u], fin[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&out->iters, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_waitcnt(0);  // T and the count have reached host memory before the flag
        __hip_atomic_store(&out->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

hipError_t launch_icp_lists(const float* src0, int ns, const DevGrid* const* g4, const float4* tgt4, int nt, int cap,
                            float4* lst, float* lsd, int* lcnt, float* lrad, unsigned long long* best_out, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    if (cap != ICP_LIST_CAP) return hipErrorInvalidValue;
    bsk::k_icp_lists<<<icp_lists_blocks(ns), 64 * ICP_WAVES, 0, s>>>(src0, ns, icp_views(g4), tgt4, nt, cap, lst, lsd, lcnt,
                                                                     lrad, best_out);
    return hipGetLastError();
}

size_t icp_loop_rec_floats(int ns) { return ns > ICPL_CH ? (size_t)7 * ns : 0; }

hipError_t launch_icp_loop(const float* src0, int ns, float4* lst, float* lsd, int* lcnt, float* lrad, int cap,
                           const DevGrid* const* g4, const float4* tgt4, int nt, int max_iter,
                           const unsigned long long* best0, float4* pos, float4* lcen, int* queue, float* rec_g,
                           IcpOut* out, int seq, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    if (cap != ICP_LIST_CAP) return hipErrorInvalidValue;
    const int chs = ns > ICPL_CH ? ICPL_CH : ((ns + 3) & ~3);
    const size_t lds = sizeof(float) * 7 * (size_t)chs;
    bsk::k_icp_loop<<<1, ICPL_THREADS, lds, s>>>(src0, ns, lst, lsd, lcnt, lrad, cap, icp_views(g4), tgt4, nt, max_iter, best0,
                                                 pos, lcen, queue, rec_g, out, seq);
    return hipGetLastError();
}

}  // namespace bsh
