// match.hip -- A9 on gfx950: brute-force B-SHOT Hamming matching (src/lidar_odometry.cpp:210-242).
// Integer-exact. minVect's FIRST-index argmin (include/bshot_bits.h:6-20) is a min over the packed
// key (dist << 32 | index): the smallest index wins every distance tie, whatever the reduction
// order, so tiles may be reduced with 64-bit atomicMin across workgroups.
//   k_ham_min: each thread owns one query descriptor (11 words in VGPRs); the workgroup streams a
//   tile of reference descriptors through LDS (48-B padded rows, broadcast reads:
//   3 x ds_read_b128 per reference), XOR + popcount, running packed min; one atomicMin per
//   (query, tile). Run once per direction (left: A vs B, right: B vs A).
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
    hipError_t e = kfill(best, 0xFF, sizeof(unsigned long long) * ((size_t)na + nb), s);
    if (e != hipSuccess) return e;
    const bsk::HamDir d0 = ham_dir(a, na, b, nb, best), d1 = ham_dir(b, nb, a, na, best + na);
    dim3 grid(d0.qb > d1.qb ? d0.qb : d1.qb, d0.splits > d1.splits ? d0.splits : d1.splits, 2);
    bsk::k_ham_min<<<grid, HM_THREADS, 0, s>>>(d0, d1);
    const int m = na > nb ? na : nb;
    bsk::k_mutual<<<(m + 255) / 256, 256, 0, s>>>(best, na, best + na, out, out + na, nb, out + na + nb);
    return hipGetLastError();
}

}  // namespace bsh
