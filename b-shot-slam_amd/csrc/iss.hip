// iss.hip -- A3 on gfx950: ISS keypoints (src/lidar_odometry.cpp:447-461 parameters; PCL
// ISSKeypoint3D::detectKeypoints semantics).
//   k_iss_scatter  wave/point: all neighbours within the salient radius (hashed grid, cell =
//                  salient radius), sorted by (d2, idx); double scatter matrix summed in rank
//                  order (6 lanes), Jacobi eigenvalues, gamma21/gamma32 test -> third[i] (0 = none)
//   k_iss_nms      lane/point: count >= min_nn within the non-max radius and no neighbour with a
//                  strictly larger third eigenvalue -> flag[i]
#include <hip/hip_runtime.h>

#include "bshot_math.h"
#include "dev_cand.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

#define ISS_CAP 512
#define ISS_WAVES 2

struct IssLds {
    unsigned long long list[ISS_CAP];
    double dd[3][ISS_CAP / 2];
    CandLds cand;
};

__device__ __forceinline__ double iss_third(const double* sm, double g21, double g32) {
    double cm[9] = {sm[0], sm[1], sm[2], sm[1], sm[3], sm[4], sm[2], sm[4], sm[5]};
    double w[3], v[9];
    bm::jacobi3(cm, w, v);
    const double e1c = w[2], e2c = w[1], e3c = w[0];
    if (bm::isfin(e1c) && bm::isfin(e2c) && bm::isfin(e3c) && !(e3c < 0))
        if ((e2c / e1c) < g21 && (e3c / e2c) < g32) return e3c;
    return 0.0;
}

// wave/point fallback for the points whose neighbourhood overflowed the lane kernel's list:
// ovf[0] = count, ovf[1..] = point indices
__global__ void __launch_bounds__(64 * ISS_WAVES) k_iss_scatter(GridView g, const float4* __restrict__ pts4,
                                                                const int* __restrict__ ovf, float salient, int min_nn,
                                                                double g21, double g32, double* __restrict__ third,
                                                                int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6, lane = lane_id();
    IssLds* L = reinterpret_cast<IssLds*>(smem) + wave;
    cand_init(&L->cand);
    const float r2 = (float)((double)salient * (double)salient);
    const int n_ovf = ovf[0];
    for (int oi = blockIdx.x * ISS_WAVES + wave; oi < n_ovf; oi += gridDim.x * ISS_WAVES) {
        const int q = ovf[1 + oi];
        const float4 c = pts4[q];
        double out = 0.0;
        if (__builtin_isfinite(c.x) && __builtin_isfinite(c.y) && __builtin_isfinite(c.z)) {
            int cnt = 0;
            for_candidates<1>(g, &L->cand, c.x, c.y, c.z, salient, r2, [&](bool v, float d2, unsigned int idx) {
                const unsigned long long m = __ballot(v);
                if (v) {
                    const int slot = cnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                    if (slot < ISS_CAP) L->list[slot] = ((unsigned long long)__float_as_uint(d2) << 32) | idx;
                }
                cnt += __popcll(m);
            });
            if (cnt > ISS_CAP) {
                if (lane == 0) atomicOr(err, 4);
            } else if (cnt >= min_nn) {
                int P = 64;
                while (P < cnt) P <<= 1;
                for (int i = cnt + lane; i < P; i += 64) L->list[i] = ~0ull;
                __builtin_amdgcn_wave_barrier();
                wave_bitonic(L->list, P);
                // neighbour offsets in double (neigh - central), rank order
                const double cx = c.x, cy = c.y, cz = c.z;
                const int half = ISS_CAP / 2;
                double cov[6] = {0, 0, 0, 0, 0, 0};
                for (int base = 0; base < cnt; base += half) {
                    const int m = min(half, cnt - base);
                    for (int r = lane; r < m; r += 64) {
                        const float4 p = pts4[(unsigned)(L->list[base + r] & 0xFFFFFFFFu)];
                        L->dd[0][r] = (double)p.x - cx;
                        L->dd[1][r] = (double)p.y - cy;
                        L->dd[2][r] = (double)p.z - cz;
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (lane < 6) {
                        const int a = lane < 3 ? 0 : (lane < 5 ? 1 : 2);
                        const int bb = lane < 3 ? lane : (lane < 5 ? lane - 2 : 2);
                        double acc = cov[0];
                        for (int r = 0; r < m; ++r) acc = acc + L->dd[a][r] * L->dd[bb][r];
                        cov[0] = acc;
                    }
                    __builtin_amdgcn_wave_barrier();
                }
                const double sm[6] = {__shfl(cov[0], 0, 64), __shfl(cov[0], 1, 64), __shfl(cov[0], 2, 64),
                                      __shfl(cov[0], 3, 64), __shfl(cov[0], 4, 64), __shfl(cov[0], 5, 64)};
                if (lane == 0) out = iss_third(sm, g21, g32);
            }
        }
        if (lane == 0) third[q] = out;
        __builtin_amdgcn_wave_barrier();
    }
}

// lane/point: every lane owns one point. Neighbours within the salient radius are insertion-sorted
// by (d2, idx) into a private LDS list of ISS_LCAP keys while the 27 cells are scanned; the double
// scatter matrix is summed sequentially in rank order and the Jacobi eigensolve runs per lane.
// Points with more than ISS_LCAP neighbours go to the overflow list (wave kernel above).
#define ISS_LCAP 32
#define ISS_LBLOCK 64

__global__ void __launch_bounds__(ISS_LBLOCK) k_iss_lane(GridView g, const float4* __restrict__ pts4, int n,
                                                        float salient, int min_nn, double g21, double g32,
                                                        double* __restrict__ third, int* __restrict__ ovf) {
    __shared__ unsigned long long keys[ISS_LCAP][ISS_LBLOCK];  // [slot][thread]: conflict-free columns
    const int t = threadIdx.x;
    const int q = blockIdx.x * ISS_LBLOCK + t;
    if (q >= n) return;
    const float4 c = pts4[q];
    double out = 0.0;
    if (__builtin_isfinite(c.x) && __builtin_isfinite(c.y) && __builtin_isfinite(c.z)) {
        const float r2 = (float)((double)salient * (double)salient);
        const double cs = (double)g.cell;
        const int x0 = (int)floor(((double)c.x - salient) / cs), x1 = (int)floor(((double)c.x + salient) / cs);
        const int y0 = (int)floor(((double)c.y - salient) / cs), y1 = (int)floor(((double)c.y + salient) / cs);
        const int z0 = (int)floor(((double)c.z - salient) / cs), z1 = (int)floor(((double)c.z + salient) / cs);
        int cnt = 0;
        for (int ix = x0; ix <= x1; ++ix)
            for (int iy = y0; iy <= y1; ++iy)
                for (int iz = z0; iz <= z1; ++iz) {
                    unsigned int st, ct;
                    if (!grid_lookup(g, cell_key(ix, iy, iz), st, ct)) continue;
                    for (unsigned int j = 0; j < ct; ++j) {
                        const float4 p = g.spts[st + j];
                        const float d2 = d2_flann(c.x, c.y, c.z, p.x, p.y, p.z);
                        if (!(d2 < r2)) continue;
                        if (cnt < ISS_LCAP) {
                            const unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) |
                                                           __float_as_uint(p.w);
                            int pos = cnt;
                            while (pos > 0 && keys[pos - 1][t] > key) {
                                keys[pos][t] = keys[pos - 1][t];
                                --pos;
                            }
                            keys[pos][t] = key;
                        }
                        ++cnt;
                    }
                }
        if (cnt > ISS_LCAP) {
            ovf[1 + atomicAdd(&ovf[0], 1)] = q;
            return;  // third[q] written by the overflow pass
        }
        if (cnt >= min_nn) {
            // pcl ISS scatter matrix: double, (neighbour - centre) outer products in rank order
            const double cx = c.x, cy = c.y, cz = c.z;
            double sm[6] = {0, 0, 0, 0, 0, 0};
            for (int r = 0; r < cnt; ++r) {
                const float4 p = pts4[(unsigned)(keys[r][t] & 0xFFFFFFFFu)];
                const double dx = (double)p.x - cx, dy = (double)p.y - cy, dz = (double)p.z - cz;
                sm[0] = sm[0] + dx * dx; sm[1] = sm[1] + dx * dy; sm[2] = sm[2] + dx * dz;
                sm[3] = sm[3] + dy * dy; sm[4] = sm[4] + dy * dz; sm[5] = sm[5] + dz * dz;
            }
            out = iss_third(sm, g21, g32);
        }
    }
    third[q] = out;
}

__global__ void __launch_bounds__(256) k_iss_nms(GridView g, const float4* __restrict__ pts4, int n, float nonmax,
                                                 int min_nn, const double* __restrict__ third,
                                                 unsigned char* __restrict__ flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned char f = 0;
    const double ti = third[i];
    const float4 c = pts4[i];
    if (ti > 0.0 && __builtin_isfinite(c.x) && __builtin_isfinite(c.y) && __builtin_isfinite(c.z)) {
        const float r2 = (float)((double)nonmax * (double)nonmax);
        const double cs = (double)g.cell;
        const int x0 = (int)floor(((double)c.x - nonmax) / cs), x1 = (int)floor(((double)c.x + nonmax) / cs);
        const int y0 = (int)floor(((double)c.y - nonmax) / cs), y1 = (int)floor(((double)c.y + nonmax) / cs);
        const int z0 = (int)floor(((double)c.z - nonmax) / cs), z1 = (int)floor(((double)c.z + nonmax) / cs);
        int cnt = 0;
        bool is_max = true;
        for (int ix = x0; ix <= x1; ++ix)
            for (int iy = y0; iy <= y1; ++iy)
                for (int iz = z0; iz <= z1; ++iz) {
                    unsigned int st, ct;
                    if (!grid_lookup(g, cell_key(ix, iy, iz), st, ct)) continue;
                    for (unsigned int j = 0; j < ct; ++j) {
                        const float4 p = g.spts[st + j];
                        if (d2_flann(c.x, c.y, c.z, p.x, p.y, p.z) < r2) {
                            ++cnt;
                            if (ti < third[__float_as_uint(p.w)]) is_max = false;
                        }
                    }
                }
        f = (cnt >= min_nn && is_max) ? 1 : 0;
    }
    flag[i] = f;
}

}  // namespace bsk

namespace bsh {

hipError_t launch_iss(const DevGrid& g, const float4* pts4, int n, float salient, float nonmax, int min_nn, double g21,
                      double g32, double* third, unsigned char* flag, int* ovf, int* err, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(ovf, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    bsk::k_iss_lane<<<(n + ISS_LBLOCK - 1) / ISS_LBLOCK, ISS_LBLOCK, 0, s>>>(g.view(), pts4, n, salient, min_nn, g21,
                                                                             g32, third, ovf);
    const size_t lds = sizeof(bsk::IssLds) * ISS_WAVES;
    // the overflow count is device-side: launch a full grid, idle waves exit at once
    bsk::k_iss_scatter<<<4096, 64 * ISS_WAVES, lds, s>>>(g.view(), pts4, ovf, salient, min_nn, g21, g32, third, err);
    bsk::k_iss_nms<<<(n + 255) / 256, 256, 0, s>>>(g.view(), pts4, n, nonmax, min_nn, third, flag);
    return hipGetLastError();
}

}  // namespace bsh
