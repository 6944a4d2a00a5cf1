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

__global__ void __launch_bounds__(64 * ISS_WAVES) k_iss_scatter(GridView g, const float4* __restrict__ pts4, int n,
                                                                float salient, int min_nn, double g21, double g32,
                                                                double* __restrict__ third, int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = threadIdx.x >> 6, lane = lane_id();
    IssLds* L = reinterpret_cast<IssLds*>(smem) + wave;
    cand_init(&L->cand);
    const float r2 = (float)((double)salient * (double)salient);
    const int G = gridDim.x, b = blockIdx.x;
    const int xg = b & 7, gi = b >> 3, ng = (G + 7 - xg) >> 3;
    const int per = (n + 7) >> 3;
    const int q_begin = xg * per, q_end = min(n, q_begin + per);
    for (int q = q_begin + gi * ISS_WAVES + wave; q < q_end; q += ng * ISS_WAVES) {
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
                double cm[9];
                const double s00 = __shfl(cov[0], 0, 64), s01 = __shfl(cov[0], 1, 64), s02 = __shfl(cov[0], 2, 64);
                const double s11 = __shfl(cov[0], 3, 64), s12 = __shfl(cov[0], 4, 64), s22 = __shfl(cov[0], 5, 64);
                cm[0] = s00; cm[1] = s01; cm[2] = s02; cm[3] = s01; cm[4] = s11; cm[5] = s12; cm[6] = s02; cm[7] = s12; cm[8] = s22;
                if (lane == 0) {
                    double w[3], v[9];
                    bm::jacobi3(cm, w, v);
                    const double e1c = w[2], e2c = w[1], e3c = w[0];
                    if (bm::isfin(e1c) && bm::isfin(e2c) && bm::isfin(e3c) && !(e3c < 0))
                        if ((e2c / e1c) < g21 && (e3c / e2c) < g32) out = e3c;
                }
            }
        }
        if (lane == 0) third[q] = out;
        __builtin_amdgcn_wave_barrier();
    }
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
                      double g32, double* third, unsigned char* flag, int* err, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const size_t lds = sizeof(bsk::IssLds) * ISS_WAVES;
    int blocks = (n + ISS_WAVES - 1) / ISS_WAVES;
    if (blocks > 8 * 256 * 4) blocks = 8 * 256 * 4;
    blocks = (blocks + 7) & ~7;
    bsk::k_iss_scatter<<<blocks, 64 * ISS_WAVES, lds, s>>>(g.view(), pts4, n, salient, min_nn, g21, g32, third, err);
    bsk::k_iss_nms<<<(n + 255) / 256, 256, 0, s>>>(g.view(), pts4, n, nonmax, min_nn, third, flag);
    return hipGetLastError();
}

}  // namespace bsh
