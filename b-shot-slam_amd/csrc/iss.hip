// iss.hip -- A3 on gfx950: ISS keypoints (src/lidar_odometry.cpp:447-461 parameters; PCL
// ISSKeypoint3D::detectKeypoints semantics).
//   k_iss_scatter  wave/point: all neighbours within the salient radius (hashed grid, cell =
//                  salient radius), sorted by (d2, idx); double scatter matrix summed in rank
//                  order (6 lanes), Jacobi eigenvalues, gamma21/gamma32 test -> third[i] (0 = none)
//   k_iss_nms      lane/point: count >= min_nn within the non-max radius and no neighbour with a
//                  strictly larger third eigenvalue -> flag[i]
#include <hip/hip_runtime.h>

#include <cstring>

#include "bshot_math.h"
#include "dev_cand.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

#define ISS_CAP 512
#define ISS_WAVES 2
#ifndef ISS_OVF_GROUP
#define ISS_OVF_GROUP 4  // candidate chunks in flight in the overflow kernel
#endif

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

#ifndef ISS_CELL_ORDER
#define ISS_CELL_ORDER 1
#endif
// A point's list position: its place in the grid's cell order (ISS_CELL_ORDER, spts .w = index) or
// its index. The overflow list and the non-max lists nml[slot][position] are kept by position, so
// the lane kernel's lanes (consecutive positions) write whole lines.
__device__ __forceinline__ int iss_point_of(const GridView& g, int jp) {
#if ISS_CELL_ORDER
    return (int)__float_as_uint(g.spts[jp].w);
#else
    return jp;
#endif
}

// wave/point fallback for the points whose neighbourhood overflowed the lane kernel's list:
// ovf[0] = count, then from ovf + 2 one (point index, list position) pair per overflow point
// nml != null (nonmax <= salient): a point whose non-max neighbours (a prefix of its sorted list) number
// at most 32 also gets its NMS list, as the lane kernel's points do (nmc >= 0: k_iss_nms_list
// decides it; -1 leaves it to the wave NMS)
__global__ void __launch_bounds__(64 * ISS_WAVES) k_iss_scatter(GridView g, const float4* __restrict__ pts4,
                                                                const int* __restrict__ ovf, float salient, int min_nn,
                                                                double g21, double g32, double* __restrict__ third,
                                                                int* __restrict__ err, unsigned int r2nm_bits,
                                                                unsigned int* __restrict__ nml, int* __restrict__ nmc,
                                                                int n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    IssLds* L = reinterpret_cast<IssLds*>(smem) + wave;
    cand_init(&L->cand);
    const float r2 = (float)((double)salient * (double)salient);
    const int n_ovf = ovf[0];
    // the eigen test of up to 64 points at once: lane k keeps the k-th pending point's scatter
    // matrix, and the Jacobi solves run on all lanes together (one lane per point)
    double psm[6] = {0, 0, 0, 0, 0, 0};
    int pq = -1, npend = 0;
    auto flush = [&]() {
        if (pq >= 0) third[pq] = iss_third(psm, g21, g32);
        pq = -1;
        npend = 0;
    };
    for (int oi = blockIdx.x * ISS_WAVES + wave; oi < n_ovf; oi += gridDim.x * ISS_WAVES) {
        const int2 e = reinterpret_cast<const int2*>(ovf + 2)[oi];  // the point and its list position
        const int q = e.x, jp = e.y;
        const float4 c = pts4[q];
        double out = 0.0;
        bool pend = false;
        if (__builtin_isfinite(c.x) && __builtin_isfinite(c.y) && __builtin_isfinite(c.z)) {
            int cnt = 0;
            for_candidates<ISS_OVF_GROUP>(g, &L->cand, c.x, c.y, c.z, salient, r2, [&](bool v, float d2, unsigned int idx) {
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
                if (nml) {
                    // the non-max prefix of the sorted list: its length, then its indices when they fit
                    int cnm = 0;
                    for (int r = lane; r < cnt; r += 64)
                        cnm += __popcll(__ballot((unsigned int)(L->list[r] >> 32) < r2nm_bits));
                    if (cnm <= 32) {
                        if (lane < cnm) nml[(size_t)lane * n + jp] = (unsigned int)L->list[lane];
                        if (lane == 0) nmc[jp] = cnm;
                    }
                }
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
                if (lane == npend) {
#pragma unroll
                    for (int u = 0; u < 6; ++u) psm[u] = sm[u];
                    pq = q;
                }
                pend = true;
            }
        }
        if (pend) {
            if (++npend == 64) flush();
        } else if (lane == 0) {
            third[q] = out;
        }
        __builtin_amdgcn_wave_barrier();
    }
    flush();
}

// lane/point: every lane owns one point. Neighbours within the salient radius are appended to a
// private LDS column (no ordering work while the cells stream by); a lane stops scanning as soon
// as it holds more than ISS_LCAP neighbours and hands the point to the overflow list (wave kernel
// above). The kept keys are then sorted by (d2, idx) in registers with a bitonic network sized to
// the wave's longest list, and the double scatter matrix is summed in that rank order.
#ifndef ISS_LCAP
#define ISS_LCAP 32
#endif
#define ISS_LBLOCK 64
#ifndef ISS_SCAN
#define ISS_SCAN 4  // points of a cell loaded at once by a lane (8: 108 VGPRs, the same sweeps/s, r05i)
#endif
#ifndef ISS_PRUNE
#define ISS_PRUNE 1  // 0: every cell of the 3 x 3 x 3 cube probed and scanned (A/B)
#endif
#ifndef ISS_MERGE32
#define ISS_MERGE32 1  // 0: the 32-key register network (A/B)
#endif

template <int N>
__device__ __forceinline__ void sort_net(unsigned long long* k) {
#pragma unroll
    for (int size = 2; size <= N; size <<= 1)
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool up = (i & size) == 0;
                    const unsigned long long a = k[i], b = k[j];
                    const bool sw = up ? (a > b) : (a < b);
                    k[i] = sw ? b : a;
                    k[j] = sw ? a : b;
                }
            }
}

// sorts the lane's kept keys, sums the scatter matrix in rank order and writes the neighbours
// inside the non-max radius (a prefix of the sorted list, nonmax <= salient) to nml[slot * n + q];
// returns their count
template <int N>
__device__ __forceinline__ int iss_sum_sorted(const unsigned long long (*keys)[ISS_LBLOCK], int t, int cnt,
                                              const float4* __restrict__ pts4, double cx, double cy, double cz,
                                              double* sm, unsigned int r2nm_bits, unsigned int* __restrict__ nml,
                                              int n, int jp) {
    unsigned long long k[N];
#pragma unroll
    for (int i = 0; i < N; ++i) k[i] = i < cnt ? keys[i][t] : ~0ull;
    sort_net<N>(k);
    int cnm = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (i < cnt && (unsigned int)(k[i] >> 32) < r2nm_bits) {  // d2 >= 0: bit order = float order
            nml[(size_t)i * n + jp] = (unsigned int)k[i];
            cnm = i + 1;
        }
#pragma unroll
    for (int r0 = 0; r0 < N; r0 += 8) {
        if (r0 >= cnt) break;
        float4 pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pp[u] = pts4[r0 + u < cnt ? (unsigned)(k[r0 + u] & 0xFFFFFFFFu) : 0u];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (r0 + u >= cnt) break;
            const double dx = (double)pp[u].x - cx, dy = (double)pp[u].y - cy, dz = (double)pp[u].z - cz;
            sm[0] = sm[0] + dx * dx; sm[1] = sm[1] + dx * dy; sm[2] = sm[2] + dx * dz;
            sm[3] = sm[3] + dy * dy; sm[4] = sm[4] + dy * dz; sm[5] = sm[5] + dz * dz;
        }
    }
    return cnm;
}

// the same for lists of 17..32 keys without 32 keys in registers (the 32-key network alone took 64
// VGPRs and held the kernel at 139, 1.8 waves/CU): each half of 16 is sorted in registers and put
// back in its LDS slots, then the two runs are merged in rank order as the sum consumes them, 8
// ranks at a time (the keys are unique: the index breaks d2 ties)
__device__ __forceinline__ int iss_sum_merge32(unsigned long long (*keys)[ISS_LBLOCK], int t, int cnt,
                                               const float4* __restrict__ pts4, double cx, double cy, double cz,
                                               double* sm, unsigned int r2nm_bits, unsigned int* __restrict__ nml,
                                               int n, int jp) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        unsigned long long k[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) k[i] = 16 * h + i < cnt ? keys[16 * h + i][t] : ~0ull;
        sort_net<16>(k);
#pragma unroll
        for (int i = 0; i < 16; ++i) keys[16 * h + i][t] = k[i];
    }
    int ia = 0, ib = 16;
    unsigned long long ha = keys[0][t], hb = keys[16][t];  // run heads (~0 past a run's valid keys)
    int cnm = 0;
#pragma unroll
    for (int r0 = 0; r0 < 32; r0 += 8) {
        if (r0 >= cnt) break;
        unsigned long long kk[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool ta = ha < hb;
            kk[u] = ta ? ha : hb;
            ia += ta ? 1 : 0;
            ib += ta ? 0 : 1;
            // both heads reloaded unconditionally (a load under the branch would serialise the steps)
            const unsigned long long na = keys[ia < 16 ? ia : 15][t], nb = keys[ib < 32 ? ib : 31][t];
            ha = ia < 16 ? na : ~0ull;
            hb = ib < 32 ? nb : ~0ull;
        }
        float4 pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = r0 + u;
            pp[u] = pts4[i < cnt ? (unsigned)(kk[u] & 0xFFFFFFFFu) : 0u];  // unconditional: loads in flight together
            if (i < cnt) {
                if ((unsigned int)(kk[u] >> 32) < r2nm_bits) {  // d2 >= 0: bit order = float order
                    nml[(size_t)i * n + jp] = (unsigned int)kk[u];
                    cnm = i + 1;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (r0 + u >= cnt) break;
            const double dx = (double)pp[u].x - cx, dy = (double)pp[u].y - cy, dz = (double)pp[u].z - cz;
            sm[0] = sm[0] + dx * dx; sm[1] = sm[1] + dx * dy; sm[2] = sm[2] + dx * dz;
            sm[3] = sm[3] + dy * dy; sm[4] = sm[4] + dy * dz; sm[5] = sm[5] + dz * dz;
        }
    }
    return cnm;
}

__global__ void __launch_bounds__(ISS_LBLOCK) k_iss_lane(GridView g, const float4* __restrict__ pts4, int n,
                                                        float salient, float nonmax, int min_nn, double g21,
                                                        double g32, double* __restrict__ third, int* __restrict__ ovf,
                                                        unsigned int* __restrict__ nml, int* __restrict__ nmc, int zc) {
    static_assert(ISS_LCAP == 16 || ISS_LCAP == 32, "the sort networks cover 8, 16 and 32 keys");
    __shared__ unsigned long long keys[ISS_LCAP][ISS_LBLOCK];  // [slot][thread]: conflict-free columns
    const int t = threadIdx.x;
    int blk = blockIdx.x;
    if (zc > 0) {
        // XCD-local chunks (as k_seg_ratio): the workgroups of label g = b % 8 (one XCD) take chunks
        // g, g + 8, ... of zc workgroups each, so each XCD's L2 holds its own stretch of cell order:
        // its points, their cells' hash-table lines and the neighbours they read
        const int gx = blockIdx.x & 7, i = blockIdx.x >> 3;
        const int m = i / zc, o = i - m * zc;
        blk = (m * 8 + gx) * zc + o;
    }
#if ISS_CELL_ORDER
    // points in the grid's cell order (spts .w = index): a wave's lanes scan the same or adjacent
    // cells, so their loops and loads stay together
    const int j = blk * ISS_LBLOCK + t;
    const bool live = j < n;
    const float4 sp = live ? g.spts[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int q = live ? (int)__float_as_uint(sp.w) : n;
    const float4 c = sp;
#else
    const int q = blk * ISS_LBLOCK + t;
    const bool live = q < n;
    const float4 c = live ? pts4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int j = q;
#endif
    const bool fin = live && __builtin_isfinite(c.x) && __builtin_isfinite(c.y) && __builtin_isfinite(c.z);
    int cnt = 0;
    if (fin) {
        const float r2 = (float)((double)salient * (double)salient);
        // the cube in float with for_candidates' slack (cells visited, never points counted)
        const float ic = g.inv_cell, lim = salient + cand_slack(c.x, c.y, c.z);
        const int x0 = (int)floorf((c.x - lim) * ic), x1 = (int)floorf((c.x + lim) * ic);
        const int y0 = (int)floorf((c.y - lim) * ic), y1 = (int)floorf((c.y + lim) * ic);
        const int z0 = (int)floorf((c.z - lim) * ic), z1 = (int)floorf((c.z + lim) * ic);
        auto take = [&](const float4& p) {
            if (d2_flann(c.x, c.y, c.z, p.x, p.y, p.z) < r2) {
                if (cnt < ISS_LCAP)
                    keys[cnt][t] = ((unsigned long long)__float_as_uint(d2_flann(c.x, c.y, c.z, p.x, p.y, p.z))
                                    << 32) | __float_as_uint(p.w);
                ++cnt;
            }
        };
        // returns false once the lane overflowed (no need to look further)
        // a cell's points ISS_SCAN at a time, every load issued together (the tail too: the index is
        // clamped and the extra points skipped), one L2 round trip per group
        auto scan_cell = [&](unsigned int st, unsigned int ct) -> bool {
            for (unsigned int j = 0; j < ct; j += ISS_SCAN) {
                float4 p[ISS_SCAN];
#pragma unroll
                for (int u = 0; u < ISS_SCAN; ++u) p[u] = g.spts[st + (j + u < ct ? j + u : ct - 1)];
#pragma unroll
                for (int u = 0; u < ISS_SCAN; ++u)
                    if (j + u < ct) take(p[u]);
                if (cnt > ISS_LCAP) return false;
            }
            return true;
        };
        const int nx = x1 - x0 + 1, ny = y1 - y0 + 1, nz = z1 - z0 + 1;
        if (nx <= 3 && ny <= 3 && nz <= 3) {
            // cell >= radius: at most 3 x 3 x 3 cells, visited 8 at a time with the first probes of
            // the 8 issued together (one batch when the cell is >= 2 x radius)
            const int ncell = nx * ny * nz;
            bool go = true;
            for (int b0 = 0; go && b0 < ncell; b0 += 8) {
                unsigned long long ck[8];
                CellEntry e[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int v = b0 + u, iz = z0 + v % nz, r = v / nz, iy = y0 + r % ny, ix = x0 + r / ny;
                    ck[u] = v < ncell ? cell_key(ix, iy, iz) : BS_EMPTY_KEY;
#if ISS_PRUNE
                    // a cube cell whose box lies farther than lim from the point holds no in-ball
                    // point (for_candidates' rule, cand_cell): neither probed nor scanned
                    const float cl = g.cell, bx0 = (float)ix * cl, by0 = (float)iy * cl, bz0 = (float)iz * cl;
                    float dx = 0.f, dy = 0.f, dz = 0.f;
                    if (c.x < bx0) dx = bx0 - c.x; else if (c.x > bx0 + cl) dx = c.x - (bx0 + cl);
                    if (c.y < by0) dy = by0 - c.y; else if (c.y > by0 + cl) dy = c.y - (by0 + cl);
                    if (c.z < bz0) dz = bz0 - c.z; else if (c.z > bz0 + cl) dz = c.z - (bz0 + cl);
                    if (!(dx * dx + dy * dy + dz * dz <= lim * lim)) ck[u] = BS_EMPTY_KEY;
#endif
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (ck[u] != BS_EMPTY_KEY) e[u] = g.table[hash_key(ck[u]) & g.mask];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    if (ck[u] == BS_EMPTY_KEY) continue;
                    unsigned int st = 0, ct = 0;
                    if (e[u].key == ck[u]) { st = e[u].start; ct = e[u].count; }
                    else if (e[u].key != BS_EMPTY_KEY && !grid_lookup(g, ck[u], st, ct)) ct = 0;
                    if (ct && !scan_cell(st, ct)) { go = false; break; }
                }
            }
        } else {
            bool go = true;
            for (int ix = x0; go && ix <= x1; ++ix)
                for (int iy = y0; go && iy <= y1; ++iy)
                    for (int iz = z0; go && iz <= z1; ++iz) {
                        unsigned int st, ct;
                        if (grid_lookup(g, cell_key(ix, iy, iz), st, ct)) go = scan_cell(st, ct);
                    }
        }
    }
    const bool over = cnt > ISS_LCAP;
    if (over) reinterpret_cast<int2*>(ovf + 2)[atomicAdd(&ovf[0], 1)] = make_int2(q, j);  // third[q]: the overflow pass
    const bool work = fin && !over && cnt >= min_nn;
    double out = 0.0;
    // wave-uniform network size: the longest kept list of the wave
    int wmax = work ? cnt : 0;
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, __shfl_xor(wmax, o, 64));
    if (work) {
        double sm[6] = {0, 0, 0, 0, 0, 0};
        const double cx = c.x, cy = c.y, cz = c.z;
        const unsigned int r2nm = __float_as_uint((float)((double)nonmax * (double)nonmax));
        int cnm;
        if (wmax <= 8) cnm = iss_sum_sorted<8>(keys, t, cnt, pts4, cx, cy, cz, sm, r2nm, nml, n, j);
        else if (wmax <= 16) cnm = iss_sum_sorted<16>(keys, t, cnt, pts4, cx, cy, cz, sm, r2nm, nml, n, j);
#if ISS_LCAP > 16
#if ISS_MERGE32
        else cnm = iss_sum_merge32(keys, t, cnt, pts4, cx, cy, cz, sm, r2nm, nml, n, j);
#else
        else cnm = iss_sum_sorted<32>(keys, t, cnt, pts4, cx, cy, cz, sm, r2nm, nml, n, j);
#endif
#endif
        out = iss_third(sm, g21, g32);
        nmc[j] = cnm;
    }
    if (live && over) nmc[j] = -1;
    if (live && !over) third[q] = out;
}

// non-maximum suppression from the lane kernel's lists (nonmax <= salient): flag[i] = the point has
// at least min_nn neighbours inside the non-max radius and none with a strictly larger third
// eigenvalue. Overflow points (nmc = -1) are left to k_iss_nms_ovf.
__global__ void __launch_bounds__(256) k_iss_nms_list(GridView g, int n, int min_nn, const double* __restrict__ third,
                                                      const unsigned int* __restrict__ nml,
                                                      const int* __restrict__ nmc, unsigned char* __restrict__ flag) {
    const int jp = blockIdx.x * blockDim.x + threadIdx.x;  // list position
    if (jp >= n) return;
    const int i = iss_point_of(g, jp);
    const int m = nmc[jp];  // non-max lists and their counts are kept by list position
    const double ti = third[i];
    if (!(ti > 0.0)) {
        flag[i] = 0;
        return;
    }
    if (m < 0) return;
    bool bigger = false;
    for (int s0 = 0; s0 < m; s0 += 8) {
        unsigned int j[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) j[u] = s0 + u < m ? nml[(size_t)(s0 + u) * n + jp] : (unsigned int)i;
        double tj[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) tj[u] = third[j[u]];
#pragma unroll
        for (int u = 0; u < 8; ++u) bigger = bigger || (ti < tj[u]);
    }
    flag[i] = (m >= min_nn && !bigger) ? 1 : 0;
}

// wave/point non-maximum suppression for the overflow list (and for every point when nonmax > salient,
// all = true): the wave sweeps the cells around the point with 64 lanes
__global__ void __launch_bounds__(256) k_iss_nms_wave(GridView g, const float4* __restrict__ pts4, int n,
                                                      const int* __restrict__ ovf, int all, float nonmax, int min_nn,
                                                      const double* __restrict__ third,
                                                      unsigned char* __restrict__ flag, const int* __restrict__ nmc) {
    const int lane = lane_id();
    const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    const int cnt_pts = all ? n : ovf[0];
    const float r2 = (float)((double)nonmax * (double)nonmax);
    for (int oi = wv; oi < cnt_pts; oi += nw) {
        const int2 e = all ? make_int2(oi, oi) : reinterpret_cast<const int2*>(ovf + 2)[oi];
        const int q = e.x;
        if (!all && nmc[e.y] >= 0) continue;  // decided from its list (k_iss_nms_list)
        const double tq = third[q];
        const float4 c = pts4[q];
        unsigned char f = 0;
        if (tq > 0.0 && __builtin_isfinite(c.x) && __builtin_isfinite(c.y) && __builtin_isfinite(c.z)) {
            const float ic = g.inv_cell, lim = nonmax + cand_slack(c.x, c.y, c.z);
            const int x0 = (int)floorf((c.x - lim) * ic), x1 = (int)floorf((c.x + lim) * ic);
            const int y0 = (int)floorf((c.y - lim) * ic), y1 = (int)floorf((c.y + lim) * ic);
            const int z0 = (int)floorf((c.z - lim) * ic), z1 = (int)floorf((c.z + lim) * ic);
            int cnt = 0;
            bool bigger = false;
            for (int ix = x0; ix <= x1 && !bigger; ++ix)
                for (int iy = y0; iy <= y1 && !bigger; ++iy)
                    for (int iz = z0; iz <= z1 && !bigger; ++iz) {
                        unsigned int st, ct;
                        if (!grid_lookup(g, cell_key(ix, iy, iz), st, ct)) continue;
                        for (unsigned int j0 = 0; j0 < ct; j0 += 64) {
                            bool in = false, big = false;
                            if (j0 + lane < ct) {
                                const float4 p = g.spts[st + j0 + lane];
                                in = d2_flann(c.x, c.y, c.z, p.x, p.y, p.z) < r2;
                                big = in && tq < third[__float_as_uint(p.w)];
                            }
                            cnt += __popcll(__ballot(in));
                            if (__ballot(big)) bigger = true;
                        }
                    }
            f = (cnt >= min_nn && !bigger) ? 1 : 0;
        }
        if (lane == 0) flag[q] = f;
    }
}

}  // namespace bsk

namespace bsh {

hipError_t launch_iss(const DevGrid& g, const float4* pts4, int n, float salient, float nonmax, int min_nn, double g21,
                      double g32, double* third, unsigned char* flag, int* ovf, unsigned int* nml, int* nmc, int* err,
                      hipStream_t s, int ovf_blocks, int nms_blocks, bool ovf_zeroed, int xcd_chunk) {
    if (n <= 0) return hipSuccess;
#ifdef DIAG_ISS_TWICE
    // diagnostic builds only: the lane kernel an extra time (its outputs are rewritten below)
    {
        hipError_t e0 = kfill(ovf, 0, sizeof(int), s);
        if (e0 != hipSuccess) return e0;
        bsk::k_iss_lane<<<(n + ISS_LBLOCK - 1) / ISS_LBLOCK, ISS_LBLOCK, 0, s>>>(g.view(), pts4, n, salient, nonmax, min_nn,
                                                                                 g21, g32, third, ovf, nml, nmc, 0);
    }
#endif
    hipError_t e = ovf_zeroed ? hipSuccess : kfill(ovf, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    int lblocks = (n + ISS_LBLOCK - 1) / ISS_LBLOCK, zc = 0;
    if (xcd_chunk > 0) {
        // whole rounds of 8 XCD-local chunks; the workgroups past n exit at once
        zc = (xcd_chunk + ISS_LBLOCK - 1) / ISS_LBLOCK;
        lblocks = (lblocks + 8 * zc - 1) / (8 * zc) * (8 * zc);
    }
    bsk::k_iss_lane<<<lblocks, ISS_LBLOCK, 0, s>>>(g.view(), pts4, n, salient, nonmax, min_nn, g21, g32, third, ovf, nml,
                                                   nmc, zc);
    const size_t lds = sizeof(bsk::IssLds) * ISS_WAVES;
    // the overflow count is device-side: a fixed grid strides over it, idle waves exit at once
#ifndef ISS_OVF_NML
#define ISS_OVF_NML 1  // 0: every overflow point through the wave NMS (A/B)
#endif
    const bool lists = ISS_OVF_NML && nonmax <= salient;
    const float r2nm = (float)((double)nonmax * (double)nonmax);
    unsigned int r2nm_bits;
    std::memcpy(&r2nm_bits, &r2nm, sizeof r2nm_bits);
    bsk::k_iss_scatter<<<ovf_blocks > 0 ? ovf_blocks : 4096, 64 * ISS_WAVES, lds, s>>>(
        g.view(), pts4, ovf, salient, min_nn, g21, g32, third, err, r2nm_bits, lists ? nml : nullptr, nmc, n);
    if (nonmax <= salient) {
        // the non-max neighbours are a prefix of the lane kernel's sorted salient neighbours
        bsk::k_iss_nms_list<<<(n + 255) / 256, 256, 0, s>>>(g.view(), n, min_nn, third, nml, nmc, flag);
        bsk::k_iss_nms_wave<<<nms_blocks > 0 ? nms_blocks : 1024, 256, 0, s>>>(g.view(), pts4, n, ovf, 0, nonmax, min_nn,
                                                                               third, flag, nmc);
    } else {
        bsk::k_iss_nms_wave<<<4096, 256, 0, s>>>(g.view(), pts4, n, ovf, 1, nonmax, min_nn, third, flag, nmc);
    }
    return hipGetLastError();
}

}  // namespace bsh
