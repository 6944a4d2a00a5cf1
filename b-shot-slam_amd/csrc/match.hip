// match.hip -- A9 on gfx950: brute-force B-SHOT Hamming matching (src/lidar_odometry.cpp:210-242).
// Integer-exact. minVect's FIRST-index argmin (include/bshot_bits.h:6-20) is a min over a packed key
// (dist << shift | index): the smallest index wins every distance tie, whatever the reduction order,
// so tiles may be reduced with atomicMin across workgroups.
//   k_ham_pair (both directions, one pass over the K x M distances): a workgroup owns a tile of
//   query rows (A, two per thread, 22 words in VGPRs) and streams a tile of reference rows (B)
//   through LDS (48-B padded rows, broadcast reads). Each distance feeds the row minimum (the
//   thread's running key (d << 23 | j)) and the column minimum (key (d << 23 | i): the thread's two
//   rows, then a DPP min over the wave, collected one column per lane (lane jj keeps column jj's) and merged
//   across the waves with ds_min_u32); one global atomicMin per row and per column per workgroup.
//   The 23-bit indices cover any realistic K and M (<= 8,388,607); beyond, k_ham_min below.
//   k_ham_min (fallback): each thread owns one query descriptor, packed 64-bit keys, one launch per
//   direction pair (left: A vs B, right: B vs A) -- twice the popcount work.
//   k_mutual: corr flag i <=> right[left[i]] == i.
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "kernels.h"

namespace bsk {

#define HM_THREADS 256
// a small LDS tile (6 KB): the launch runs on the main stream beside the side stream's LDS-heavy
// kernels, and a workgroup only starts on a CU with that much LDS free
#define HM_TILE 128

// both directions in one launch: blockIdx.z == 0 -> A vs B (left), 1 -> B vs A (right)
struct HamDir {
    const unsigned int* q;
    const unsigned int* r;
    unsigned long long* best;
    int nq, nr, tile, qb, splits;
};

__global__ void __launch_bounds__(HM_THREADS) k_ham_min(HamDir d0, HamDir d1) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    const HamDir& D = blockIdx.z == 0 ? d0 : d1;
    if ((int)blockIdx.x >= D.qb || (int)blockIdx.y >= D.splits) return;
    const unsigned int* __restrict__ q = D.q;
    const unsigned int* __restrict__ r = D.r;
    unsigned long long* __restrict__ best = D.best;
    const int nq = D.nq, nr = D.nr, tile = D.tile;
    __shared__ uint4 rt[HM_TILE * 3];
    const int t = threadIdx.x;
    const int qi = blockIdx.x * HM_THREADS + t;
    const int r0 = blockIdx.y * tile;
    const int r1 = min(nr, r0 + tile);
    unsigned int a[11];
#pragma unroll
    for (int w = 0; w < 11; ++w) a[w] = qi < nq ? q[11 * (size_t)qi + w] : 0u;
    unsigned long long m = ~0ull;
    for (int s0 = r0; s0 < r1; s0 += HM_TILE) {
        const int cnt = min(HM_TILE, r1 - s0);
        __syncthreads();
        for (int i = t; i < cnt * 12; i += HM_THREADS) {
            const int row = i / 12, w = i % 12;
            reinterpret_cast<unsigned int*>(rt)[i] = w < 11 ? r[11 * (size_t)(s0 + row) + w] : 0u;
        }
        __syncthreads();
        for (int j = 0; j < cnt; ++j) {
            const uint4 b0 = rt[3 * j], b1 = rt[3 * j + 1], b2 = rt[3 * j + 2];
            unsigned int d = __builtin_popcount(a[0] ^ b0.x);
            d += __builtin_popcount(a[1] ^ b0.y);
            d += __builtin_popcount(a[2] ^ b0.z);
            d += __builtin_popcount(a[3] ^ b0.w);
            d += __builtin_popcount(a[4] ^ b1.x);
            d += __builtin_popcount(a[5] ^ b1.y);
            d += __builtin_popcount(a[6] ^ b1.z);
            d += __builtin_popcount(a[7] ^ b1.w);
            d += __builtin_popcount(a[8] ^ b2.x);
            d += __builtin_popcount(a[9] ^ b2.y);
            d += __builtin_popcount(a[10] ^ b2.z);
            const unsigned long long key = ((unsigned long long)d << 32) | (unsigned)(s0 + j);
            m = key < m ? key : m;
        }
    }
    if (qi < nq) atomicMin(&best[qi], m);
}

#define HP_THREADS 256
#define HP_ROWS 2                          // query rows per thread
#define HP_TROWS (HP_THREADS * HP_ROWS)    // query rows per workgroup
#ifndef HP_TILE
#define HP_TILE 128  // reference rows per LDS tile
#endif
#define HP_SHIFT 23

// wave-wide min of a u32 (DPP: row shifts, then the row broadcasts; the result is in lane 63)
__device__ __forceinline__ unsigned int wave_min_u32_to63(unsigned int v) {
    const int I = -1;
    v = min(v, (unsigned int)dpp_i<0x111, 0xf>(I, (int)v));
    v = min(v, (unsigned int)dpp_i<0x112, 0xf>(I, (int)v));
    v = min(v, (unsigned int)dpp_i<0x114, 0xf>(I, (int)v));
    v = min(v, (unsigned int)dpp_i<0x118, 0xf>(I, (int)v));
    v = min(v, (unsigned int)dpp_i<0x142, 0xa>(I, (int)v));
    v = min(v, (unsigned int)dpp_i<0x143, 0xc>(I, (int)v));
    return v;
}

__device__ __forceinline__ unsigned int ham11(const unsigned int* a, uint4 b0, uint4 b1, uint4 b2) {
    unsigned int d = __builtin_popcount(a[0] ^ b0.x);
    d += __builtin_popcount(a[1] ^ b0.y);
    d += __builtin_popcount(a[2] ^ b0.z);
    d += __builtin_popcount(a[3] ^ b0.w);
    d += __builtin_popcount(a[4] ^ b1.x);
    d += __builtin_popcount(a[5] ^ b1.y);
    d += __builtin_popcount(a[6] ^ b1.z);
    d += __builtin_popcount(a[7] ^ b1.w);
    d += __builtin_popcount(a[8] ^ b2.x);
    d += __builtin_popcount(a[9] ^ b2.y);
    d += __builtin_popcount(a[10] ^ b2.z);
    return d;
}

// grid: (row tiles, column splits); split y covers references [y * span, (y + 1) * span)
__global__ void __launch_bounds__(HP_THREADS) k_ham_pair(const unsigned int* __restrict__ a, int na,
                                                          const unsigned int* __restrict__ b, int nb, int span,
                                                          unsigned int* __restrict__ rowbest,
                                                          unsigned int* __restrict__ colbest) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    __shared__ uint4 rt[HP_TILE * 3];
    __shared__ unsigned int scol[HP_TILE];
    const int t = threadIdx.x, lane = lane_id();
    const int i0 = blockIdx.x * HP_TROWS + t, i1 = i0 + HP_THREADS;  // this thread's two rows
    const int r0 = blockIdx.y * span, r1 = min(nb, r0 + span);
    unsigned int qa[11], qb[11];
#pragma unroll
    for (int w = 0; w < 11; ++w) {
        qa[w] = i0 < na ? a[11 * (size_t)i0 + w] : 0u;
        qb[w] = i1 < na ? a[11 * (size_t)i1 + w] : 0u;
    }
    // rows past na never win a column: their keys are forced to the maximum
    const unsigned int ka = i0 < na ? (unsigned int)i0 : 0xFFFFFFFFu, kb = i1 < na ? (unsigned int)i1 : 0xFFFFFFFFu;
    unsigned int ma = 0xFFFFFFFFu, mb = 0xFFFFFFFFu;
    for (int s0 = r0; s0 < r1; s0 += HP_TILE) {
        const int cnt = min(HP_TILE, r1 - s0);
        __syncthreads();
        for (int i = t; i < cnt * 12; i += HP_THREADS) {
            const int row = i / 12, w = i % 12;
            reinterpret_cast<unsigned int*>(rt)[i] = w < 11 ? b[11 * (size_t)(s0 + row) + w] : 0u;
        }
        for (int i = t; i < HP_TILE; i += HP_THREADS) scol[i] = 0xFFFFFFFFu;
        __syncthreads();
        for (int c0 = 0; c0 < cnt; c0 += 64) {
            unsigned int colv = 0xFFFFFFFFu;  // lane l: this wave's minimum of column c0 + l
            const int ce = min(64, cnt - c0);
            for (int jj = 0; jj < ce; ++jj) {
                const int j = c0 + jj;
                const uint4 b0 = rt[3 * j], b1 = rt[3 * j + 1], b2 = rt[3 * j + 2];
                const unsigned int da = ham11(qa, b0, b1, b2), db = ham11(qb, b0, b1, b2);
                const unsigned int jr = (unsigned int)(s0 + j);
                ma = min(ma, (da << HP_SHIFT) | jr);
                mb = min(mb, (db << HP_SHIFT) | jr);
                const unsigned int ca = ka == 0xFFFFFFFFu ? ka : (da << HP_SHIFT) | ka;
                const unsigned int cb = kb == 0xFFFFFFFFu ? kb : (db << HP_SHIFT) | kb;
                const unsigned int wm = wave_min_u32_to63(min(ca, cb));
                const unsigned int wj = (unsigned int)__builtin_amdgcn_readlane((int)wm, 63);
                colv = lane == jj ? wj : colv;
            }
            if (lane < ce) atomicMin(&scol[c0 + lane], colv);
        }
        __syncthreads();
        for (int i = t; i < cnt; i += HP_THREADS)
            if (scol[i] != 0xFFFFFFFFu) atomicMin(&colbest[s0 + i], scol[i]);
    }
    if (i0 < na) atomicMin(&rowbest[i0], ma);
    if (i1 < na) atomicMin(&rowbest[i1], mb);
}

__global__ void k_mutual32(const unsigned int* __restrict__ lbest, int na, const unsigned int* __restrict__ rbest,
                           int* __restrict__ left, int* __restrict__ right, int nb, int* __restrict__ flag) {
    __builtin_amdgcn_s_setprio(3);
    const unsigned int M = (1u << HP_SHIFT) - 1;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nb) right[i] = (int)(rbest[i] & M);
    if (i < na) {
        const int l = (int)(lbest[i] & M);
        left[i] = l;
        flag[i] = ((int)(rbest[l] & M) == i) ? 1 : 0;
    }
}

__global__ void k_mutual(const unsigned long long* __restrict__ lbest, int na, const unsigned long long* __restrict__ rbest,
                         int* __restrict__ left, int* __restrict__ right, int nb, int* __restrict__ flag) {
    __builtin_amdgcn_s_setprio(3);  // latency-critical main-stream kernel: issue ahead of side-stream waves
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nb) right[i] = (int)(rbest[i] & 0xFFFFFFFFu);
    if (i < na) {
        const int l = (int)(lbest[i] & 0xFFFFFFFFu);
        left[i] = l;
        flag[i] = ((int)(rbest[l] & 0xFFFFFFFFu) == i) ? 1 : 0;
    }
}

}  // namespace bsk

namespace bsh {

static bsk::HamDir ham_dir(const unsigned int* q, int nq, const unsigned int* r, int nr, unsigned long long* best) {
    // split the reference set so the launch has >= ~1024 workgroups when nq is small
    bsk::HamDir d;
    d.q = q; d.r = r; d.best = best; d.nq = nq; d.nr = nr;
    d.qb = (nq + HM_THREADS - 1) / HM_THREADS;
    int splits = (1024 + d.qb - 1) / d.qb;
    int tile = (nr + splits - 1) / splits;
    if (tile < HM_TILE) tile = HM_TILE;
    d.tile = tile;
    d.splits = (nr + tile - 1) / tile;
    return d;
}

// a: na x 11 words, b: nb x 11 words; best: na + nb packed keys (left then right), reset here;
// out: left[na] | right[nb] | flag[na]
hipError_t launch_match(const unsigned int* a, int na, const unsigned int* b, int nb, unsigned long long* best,
                        int* out, hipStream_t s) {
    if (na <= 0 || nb <= 0) return hipSuccess;
    hipError_t e;
    const int m = na > nb ? na : nb;
    if (na < (1 << HP_SHIFT) && nb < (1 << HP_SHIFT)) {
        // one pass, 32-bit keys: best holds na + nb u32 (left then right)
        unsigned int* kb = reinterpret_cast<unsigned int*>(best);
        if ((e = kfill(kb, 0xFF, sizeof(unsigned int) * ((size_t)na + nb), s)) != hipSuccess) return e;
        const int rt = (na + HP_TROWS - 1) / HP_TROWS;
        // ~1024 workgroups, >= one LDS tile of references each
        int splits = (1024 + rt - 1) / rt;
        int span = (nb + splits - 1) / splits;
        if (span < HP_TILE) span = HP_TILE;
        splits = (nb + span - 1) / span;
        bsk::k_ham_pair<<<dim3(rt, splits), HP_THREADS, 0, s>>>(a, na, b, nb, span, kb, kb + na);
        bsk::k_mutual32<<<(m + 255) / 256, 256, 0, s>>>(kb, na, kb + na, out, out + na, nb, out + na + nb);
        return hipGetLastError();
    }
    if ((e = kfill(best, 0xFF, sizeof(unsigned long long) * ((size_t)na + nb), s)) != hipSuccess) return e;
    const bsk::HamDir d0 = ham_dir(a, na, b, nb, best), d1 = ham_dir(b, nb, a, na, best + na);
    dim3 grid(d0.qb > d1.qb ? d0.qb : d1.qb, d0.splits > d1.splits ? d0.splits : d1.splits, 2);
    bsk::k_ham_min<<<grid, HM_THREADS, 0, s>>>(d0, d1);
    bsk::k_mutual<<<(m + 255) / 256, 256, 0, s>>>(best, na, best + na, out, out + na, nb, out + na + nb);
    return hipGetLastError();
}

}  // namespace bsh
