// ransac.hip -- A10 on gfx950: scores of every RANSAC hypothesis in one launch (SURVEY.md §8f
// rank 2). The reference's RandomSampleConsensus (src/lidar_odometry.cpp:251-261, PCL
// CorrespondenceRejectorSampleConsensus) draws its 3-point samples from a stream that does not
// depend on model scores, so the host draws them all first (host/ransac.cpp, mt19937(12345) >> 1,
// partial Fisher-Yates, isSampleGood), this kernel scores them all at once, and the host replays
// PCL's best-model / adaptive-k scan over the scores. Same arithmetic as the host scorer: double
// umeyama over the 3 sample pairs (bm::umeyama_seq) rounded to float, pcl::transformPointCloud's
// float expression, Vector4f squaredNorm's SSE order, (double)d2 < thresh^2.
#include <hip/hip_runtime.h>

#include "bshot_math.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

#define RS_WAVES 4

// Workgroup per 64 hypotheses, lane per hypothesis. Wave 0 computes the 64 models (one double
// umeyama per lane, not one per wave replicated over its 64 lanes: the FP64 work is 1/64 of a
// wave-per-hypothesis kernel, which matters because this kernel runs on the main stream while the
// lookahead's FP64-heavy SHOT producers hold the SIMDs), stores them component-major in LDS, then
// each of the 4 waves scores the 64 models over its quarter of the correspondences: the
// correspondence index is wave-uniform, so the point loads are uniform (scalar) loads and every
// lane tests its own model. Partial counts are integers, summed in any order.
// cs/ct: correspondence source/target points (3 floats each, correspondence order); hyp: 3
// correspondence positions per hypothesis
#define RS_HYP 64
// <= 72 VGPRs (the double umeyama's registers spill): a workgroup then fits beside the SR launch's
// 6 waves of 80 VGPRs per SIMD as soon as one of them retires, instead of waiting for two
// (profiles/r05_ab_sr_w6.txt: the RANSAC phase 0.49 -> 0.19 ms under the 6-wave SR)
#ifndef RS_WPE
#define RS_WPE 7
#endif
#if RS_WPE > 0
#define RS_ATTR __attribute__((amdgpu_waves_per_eu(RS_WPE)))
#else
#define RS_ATTR
#endif
__global__ void __launch_bounds__(64 * RS_WAVES) RS_ATTR k_ransac_score(const float* __restrict__ cs,
                                                                const float* __restrict__ ct, int nidx,
                                                                const int* __restrict__ hyp, int nhyp, double thr2,
                                                                int* __restrict__ cnt) {
    __builtin_amdgcn_s_setprio(3);  // main-stream kernel on the odometry chain's critical path
    __shared__ float Ts[12][RS_HYP];
    __shared__ int part[RS_WAVES][RS_HYP];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id();
    const int h = blockIdx.x * RS_HYP + lane;
    if (w == 0) {
        float T[12];
        if (h < nhyp) {
            double sd[9], td[9];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int p = hyp[3 * h + i];
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    sd[3 * i + d] = (double)cs[3 * p + d];
                    td[3 * i + d] = (double)ct[3 * p + d];
                }
            }
            double md[16];
            bm::umeyama_seq<double>(sd, td, 3, md);
#pragma unroll
            for (int k = 0; k < 12; ++k) T[k] = (float)md[k];
        } else {
#pragma unroll
            for (int k = 0; k < 12; ++k) T[k] = 0.0f;
        }
#pragma unroll
        for (int k = 0; k < 12; ++k) Ts[k][lane] = T[k];
    }
    __syncthreads();
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = Ts[k][lane];
    const int per = (nidx + RS_WAVES - 1) / RS_WAVES;
    const int i0 = w * per;
    const int i1 = min(nidx, i0 + per);
    int c = 0;
#pragma unroll 4
    for (int i = i0; i < i1; ++i) {
        const float x = cs[3 * i], y = cs[3 * i + 1], z = cs[3 * i + 2];
        const float px = ((T[0] * x + T[1] * y) + T[2] * z) + T[3];
        const float py = ((T[4] * x + T[5] * y) + T[6] * z) + T[7];
        const float pz = ((T[8] * x + T[9] * y) + T[10] * z) + T[11];
        const float dx = px - ct[3 * i], dy = py - ct[3 * i + 1], dz = pz - ct[3 * i + 2];
        const float d2 = (dx * dx + dz * dz) + (dy * dy + 0.0f);
        c += (double)d2 < thr2 ? 1 : 0;
    }
    part[w][lane] = c;
    __syncthreads();
    if (w == 0 && h < nhyp) {
        int s = 0;
#pragma unroll
        for (int v = 0; v < RS_WAVES; ++v) s += part[v][lane];
        cnt[h] = s;
    }
}

}  // namespace bsk

namespace bsh {

hipError_t launch_ransac_score(const float* cs, const float* ct, int nidx, const int* hyp, int nhyp, double thr2,
                               int* cnt, hipStream_t s) {
    if (nhyp <= 0) return hipSuccess;
    bsk::k_ransac_score<<<(nhyp + RS_HYP - 1) / RS_HYP, 64 * RS_WAVES, 0, s>>>(cs, ct, nidx, hyp, nhyp, thr2, cnt);
    return hipGetLastError();
}

}  // namespace bsh
