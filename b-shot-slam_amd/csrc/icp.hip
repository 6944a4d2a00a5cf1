// icp.hip -- A11 nearest-neighbour step of point-to-point ICP on gfx950 (PCL IterativeClosestPoint
// defaults, src/lidar_odometry.cpp:291-297: CorrespondenceEstimation::determineCorrespondences,
// 1-NN, no distance cap). Exact: the packed key (float bits of d2 << 32 | target index) min picks
// the smallest squared distance, smallest index on ties (DESIGN.md convention for FLANN's
// traversal-dependent tie), independent of the reduction order.
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "kernels.h"

namespace bsk {

#define ICP_THREADS 256
// small LDS tile (4 KB): ICP runs on the main stream beside LDS-heavy side-stream kernels
#define ICP_TILE 256

__global__ void __launch_bounds__(ICP_THREADS) k_icp_nn(const float* __restrict__ src, int ns,
                                                        const float4* __restrict__ tgt, int nt, int tile,
                                                        unsigned long long* __restrict__ best) {
    __shared__ float4 tt[ICP_TILE];
    const int t = threadIdx.x;
    const int i = blockIdx.x * ICP_THREADS + t;
    const int r0 = blockIdx.y * tile, r1 = min(nt, r0 + tile);
    float qx = 0.f, qy = 0.f, qz = 0.f;
    if (i < ns) { qx = src[3 * i]; qy = src[3 * i + 1]; qz = src[3 * i + 2]; }
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

struct Xf16 {
    float m[16];
};

// One ICP iteration in one launch: every source point is first moved by the previous iteration's
// step T (when apply; same float expression as the host's bg::xform), the moved cloud is written
// to src_out by the blockIdx.y == 0 blocks, the 1-NN keys go to best via atomicMin, and the
// next iteration's best array is reset -- no separate H2D, fill or transform launches.
__global__ void __launch_bounds__(ICP_THREADS) k_icp_iter(const float* __restrict__ src_in, float* __restrict__ src_out,
                                                          Xf16 T, int apply, int ns, const float4* __restrict__ tgt,
                                                          int nt, int tile, unsigned long long* __restrict__ best,
                                                          unsigned long long* __restrict__ best_next) {
    __shared__ float4 tt[ICP_TILE];
    const int t = threadIdx.x;
    const int i = blockIdx.x * ICP_THREADS + t;
    const int r0 = blockIdx.y * tile, r1 = min(nt, r0 + tile);
    float qx = 0.f, qy = 0.f, qz = 0.f;
    if (i < ns) {
        const float x = src_in[3 * i], y = src_in[3 * i + 1], z = src_in[3 * i + 2];
        if (apply) {
            qx = ((T.m[0] * x + T.m[1] * y) + T.m[2] * z) + T.m[3];
            qy = ((T.m[4] * x + T.m[5] * y) + T.m[6] * z) + T.m[7];
            qz = ((T.m[8] * x + T.m[9] * y) + T.m[10] * z) + T.m[11];
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

hipError_t launch_icp_nn(const float* src, int ns, const float4* tgt, int nt, unsigned long long* best, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    bsk::k_fill_u64b<<<(ns + 255) / 256, 256, 0, s>>>(best, ns, ~0ull);
    const int qb = (ns + ICP_THREADS - 1) / ICP_THREADS;
    int splits = (1024 + qb - 1) / qb;
    int tile = (nt + splits - 1) / splits;
    if (tile < 256) tile = 256;
    splits = (nt + tile - 1) / tile;
    dim3 grid(qb, splits);
    bsk::k_icp_nn<<<grid, ICP_THREADS, 0, s>>>(src, ns, tgt, nt, tile, best);
    return hipGetLastError();
}

hipError_t launch_icp_iter(const float* src_in, float* src_out, const float* T16, int apply, int ns, const float4* tgt,
                           int nt, unsigned long long* best, unsigned long long* best_next, hipStream_t s) {
    if (ns <= 0 || nt <= 0) return hipSuccess;
    const int qb = (ns + ICP_THREADS - 1) / ICP_THREADS;
    int splits = (1024 + qb - 1) / qb;
    int tile = (nt + splits - 1) / splits;
    if (tile < 256) tile = 256;
    splits = (nt + tile - 1) / tile;
    bsk::Xf16 T;
    for (int i = 0; i < 16; ++i) T.m[i] = T16 ? T16[i] : ((i % 5) == 0 ? 1.f : 0.f);
    bsk::k_icp_iter<<<dim3(qb, splits), ICP_THREADS, 0, s>>>(src_in, src_out, T, apply, ns, tgt, nt, tile, best,
                                                              best_next);
    return hipGetLastError();
}

}  // namespace bsh
