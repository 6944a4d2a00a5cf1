// describe2.hip -- A5/A6/A7 on gfx950, load-balanced: the SHOT stages split every keypoint's
// neighbourhood (up to ~22k points for keypoints near the sensor, ~3x the mean) into 64-rank chunks
// so no single keypoint bounds a launch (PCL SHOTEstimationOMP / SHOTLocalReferenceFrameEstimation,
// include/bshot_bits.h:113-135; compute_bshot_from_SHOT :144-278).
//
//   (sorting: k_shot_rank, csrc/describe.hip -- exact rank inside the count pass's d2 buckets)
//   k_lrf_chunks  wave per 64-rank chunk: 7 weighted-covariance terms by the xor-butterfly tree
//   k_lrf_eig     two waves per keypoint: chunk sums in chunk order (a lane per term) + Jacobi
//                 eigenvectors; with normal_radius == shot_radius the other wave writes the keypoint
//                 normal (segment_normal)
//   k_hist_fused  workgroup per keypoint: the x/z sign counts and PCL's count + median-5 rule
//                 (float LRF rows) first,
//                 then 7 waves compute the <= 5 (bin, value)
//                 interpolation records of every neighbour into a double-buffered LDS batch while
//                 one wave applies them in rank order to the LDS histogram (in-order ds_add_f32),
//                 then L2 normalisation and B-SHOT bits
// Chunk c of keypoint q covers ranks [64 (c - cb[q]), ...) where cb is the exclusive scan of
// ceil(n_q / 64) (k_desc_plan, or the host plan after an overflow).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bshot_math.h"
#include "dev_common.h"
#include "kernels.h"

namespace bsk {

// owner[c] = keypoint of chunk c (block per keypoint); with cinfo, also the chunk's record
// {keypoint, chunk index in the keypoint, segment length, segment offset} in one 16-B load, so the
// chunk kernels skip the owner -> offsets/chunk-base round trip (segments below 2^31 keys)
__global__ void __launch_bounds__(256) k_chunk_owner(int k, const int* __restrict__ cb, int* __restrict__ owner,
                                                     const long long* __restrict__ offs, int4* __restrict__ cinfo) {
    const int q = blockIdx.x;
    if (q >= k) return;
    const int c0 = cb[q], c1 = cb[q + 1];
    const long long o = cinfo ? offs[q] : 0;
    const int n = cinfo ? (int)(offs[q + 1] - o) : 0;
    for (int c = c0 + threadIdx.x; c < c1; c += 256) {
        owner[c] = q;
        if (cinfo) cinfo[c] = make_int4(q, c - c0, n, (int)o);
    }
}

// The 7 butterfly sums of wave_tree_sum_d (partners lane ^ 32, ^ 16, ..., ^ 1 in that order), all at
// once with 10 cross-lane exchanges instead of 42: at the xor-32 level the lanes with bit 5 clear
// keep terms 0..3 and receive their partners' 0..3 while the others keep 4..6 (+ a zero pad), at xor
// 16 each keeps two, at xor 8 one, then a plain butterfly over xor 4, 2, 1. Every term still adds
// the same pairs at every level (x + y == y + x), so each sum has wave_tree_sum_d's bits. Returns
// term (lane >> 3): lanes 8 j .. 8 j + 7 hold term j's sum.
__device__ __forceinline__ double wave_tree_sum7(const double* v) {
    const int lane = lane_id();
    const bool b5 = (lane & 32) != 0, b4 = (lane & 16) != 0, b3 = (lane & 8) != 0;
    double a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const double lo = v[j], hi = j + 4 < 7 ? v[j + 4] : 0.0;
        a[j] = (b5 ? hi : lo) + xor_lane_d<32>(b5 ? lo : hi);
    }
    double b[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = (b4 ? a[j + 2] : a[j]) + xor_lane_d<16>(b4 ? a[j] : a[j + 2]);
    double c = (b3 ? b[1] : b[0]) + xor_lane_d<8>(b3 ? b[0] : b[1]);
    c = c + xor_lane_d<4>(c);
    c = c + xor_lane_d<2>(c);
    c = c + xor_lane_d<1>(c);
    return c;
}

// csum[8 c + 0..5]: weighted covariance terms, [6]: weight sum, [7]: valid count of chunk c =
// ranks [64 t, 64 t + 64) of keypoint q (wave; lanes 0..7 store)
__device__ __forceinline__ void lrf_chunk_terms(const float4* __restrict__ pts4, float kx, float ky, float kz, float R,
                                                const unsigned int* __restrict__ sg, int n, int t,
                                                double* __restrict__ out8) {
    const int lane = lane_id();
    const int i = t * 64 + lane;
    double v[7] = {0, 0, 0, 0, 0, 0, 0};
    int isv = 0;
    if (i < n) {
        const float4 p = pts4[sg[i]];
        if (!(p.x == kx && p.y == ky && p.z == kz)) {
            const double vx = (double)(p.x - kx), vy = (double)(p.y - ky), vz = (double)(p.z - kz);
            // the gather's d2 (same expression and operands: the same bits as the ranked key's)
            const double w = (double)R - sqrt((double)d2_flann(kx, ky, kz, p.x, p.y, p.z));
            v[0] = w * (vx * vx); v[1] = w * (vx * vy); v[2] = w * (vx * vz);
            v[3] = w * (vy * vy); v[4] = w * (vy * vz); v[5] = w * (vz * vz);
            v[6] = w;
            isv = 1;
        }
    }
    const double sum = wave_tree_sum7(v);  // term (lane >> 3)
    const int nv = __popcll(__ballot(isv != 0));
    if ((lane & 7) == 0) out8[lane >> 3] = (lane >> 3) < 7 ? sum : (double)nv;
}

__global__ void __launch_bounds__(256) k_lrf_chunks(const float4* __restrict__ pts4, const float* __restrict__ kps,
                                                    int k, float R, const long long* __restrict__ offs,
                                                    const int* __restrict__ cb, const int* __restrict__ owner,
                                                    const unsigned int* __restrict__ seg,
                                                    double* __restrict__ csum, const int4* __restrict__ cinfo) {
    // grid-stride over chunks: a capped grid (Describe2Args::max_blocks) instead of a block per 4 chunks
    for (int c = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); c < cb[k]; c += gridDim.x * 4) {
        if (cinfo) {
            const int4 ci = cinfo[c];
            lrf_chunk_terms(pts4, kps[3 * ci.x], kps[3 * ci.x + 1], kps[3 * ci.x + 2], R, seg + (unsigned int)ci.w, ci.z,
                            ci.y, csum + 8 * (size_t)c);
        } else {
            const int q = owner[c];
            const long long o = offs[q];
            lrf_chunk_terms(pts4, kps[3 * q], kps[3 * q + 1], kps[3 * q + 2], R, seg + o, (int)(offs[q + 1] - o),
                            c - cb[q], csum + 8 * (size_t)c);
        }
    }
}

// A4 from the SHOT neighbour lists (include/bshot_bits.h:63-80): with normal_radius == shot_radius
// the normals' FLANN radius search (the normal_max_nn smallest (d2, idx) with d2 < r^2, in that
// order) is the first min(n, normal_max_nn) entries of the keypoint's sorted SHOT segment, so no
// search of its own is needed. One wave: the neighbours' coordinates in LDS (f: 3 x NF_STRIDE floats), the
// 9 accumulators of pcl::computeMeanAndCovarianceMatrix as sequential float sums in rank order
// (lanes 0..5: xx xy xz yy yz zz products, lanes 6..8: x y z -- k_normals' order), then eigen33 and
// the flip towards the origin. Returns (nx, ny, nz, curvature), NaN as k_normals.
// the 3 coordinate arrays sit NF_STRIDE floats apart (512 + 4: the 9 summing lanes read x[r], y[r],
// z[r] together from 3 different LDS banks; a 512 stride put them in one bank)
#define NF_STRIDE 516
__device__ __forceinline__ float4 segment_normal(const float4* __restrict__ pts4, float kx, float ky, float kz,
                                                 const unsigned int* __restrict__ sg, long long cnt, int max_nn,
                                                 float* f) {
    const int lane = lane_id();
    const float qn = __builtin_nanf("");
    float nx = qn, ny = qn, nz = qn, curv = qn;
    if (__builtin_isfinite(kx) && __builtin_isfinite(ky) && __builtin_isfinite(kz)) {
        const int need = (int)(cnt < max_nn ? cnt : max_nn);
        if (need > 0) {
            float acc = 0.f;
            if (need >= 3) {
                for (int r = lane; r < need; r += 64) {
                    const float4 p = pts4[sg[r]];
                    f[r] = p.x; f[NF_STRIDE + r] = p.y; f[2 * NF_STRIDE + r] = p.z;
                }
                __builtin_amdgcn_wave_barrier();
                if (lane < 9) {
                    const bool prod = lane < 6;
                    const int a = prod ? (lane < 3 ? 0 : (lane < 5 ? 1 : 2)) : lane - 6;
                    const int b = lane < 3 ? lane : (lane < 5 ? lane - 2 : 2);
                    const float* pa = f + NF_STRIDE * a;
                    const float* pb = f + NF_STRIDE * (prod ? b : a);
                    int r = 0;
                    for (; r + 4 <= need; r += 4) {
                        float v[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) v[u] = prod ? pa[r + u] * pb[r + u] : pa[r + u];
#pragma unroll
                        for (int u = 0; u < 4; ++u) acc = acc + v[u];
                    }
                    for (; r < need; ++r) acc = acc + (prod ? pa[r] * pb[r] : pa[r]);
                }
            }
            if (need >= 3) {
                float ac[9];
                const float fn = (float)need;
#pragma unroll
                for (int a = 0; a < 9; ++a) ac[a] = __shfl(acc, a, 64) / fn;
                float cov[9];
                cov[0] = ac[0] - ac[6] * ac[6];
                cov[1] = ac[1] - ac[6] * ac[7];
                cov[2] = ac[2] - ac[6] * ac[8];
                cov[4] = ac[3] - ac[7] * ac[7];
                cov[5] = ac[4] - ac[7] * ac[8];
                cov[8] = ac[5] - ac[8] * ac[8];
                cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
                float ev, vec[3];
                bm::eigen33_min(cov, &ev, vec);
                nx = vec[0]; ny = vec[1]; nz = vec[2];
                const float eig_sum = (cov[0] + cov[4]) + cov[8];
                curv = (eig_sum != 0.f) ? fabsf(ev / eig_sum) : 0.f;
            }
            const float vx = 0.f - kx, vy = 0.f - ky, vz = 0.f - kz;
            const float cth = (vx * nx + vy * ny) + vz * nz;
            if (cth < 0.f) { nx *= -1.f; ny *= -1.f; nz *= -1.f; }
        }
    }
    return make_float4(nx, ny, nz, curv);
}

// Jacobi eigenvectors of keypoint q's weighted covariance (tot: the 7 chunk-ordered sums, valid: the
// valid-neighbour count): e[0..2] = x axis (largest), [3..5] = z axis (smallest), [6] = valid count;
// returns the ok flag
__device__ __forceinline__ int lrf_eig_of_sums(const double* tot, long long valid, double* e) {
    int ok = 0;
    if (valid >= 5) {
        const double sum = tot[6];
        double cov[9];
        cov[0] = tot[0] / sum; cov[1] = tot[1] / sum; cov[2] = tot[2] / sum;
        cov[4] = tot[3] / sum; cov[5] = tot[4] / sum; cov[8] = tot[5] / sum;
        cov[3] = cov[1]; cov[6] = cov[2]; cov[7] = cov[5];
        double w[3], ev[9];
        bm::jacobi3(cov, w, ev);
        if (bm::isfin(w[0]) && bm::isfin(w[1]) && bm::isfin(w[2])) {
            ok = 1;
            e[0] = ev[2]; e[1] = ev[5]; e[2] = ev[8];
            e[3] = ev[0]; e[4] = ev[3]; e[5] = ev[6];
        }
    }
    e[6] = (double)valid;
    return ok;
}

// eig[8 q + 0..6] (lrf_eig_of_sums), okf[q]. A wave per keypoint: lane j < 7 sums column j of the
// keypoint's chunk partials in chunk order (sequential double adds; the 8 lanes of a chunk read its
// 64 B together), lane 7 the valid counts (integers); lane 0 then runs the Jacobi solver.
// nmax > 0: the same wave first writes the keypoint's normal from the head of its sorted segment
// (segment_normal; normal_radius == shot_radius), which the histogram kernel reads.
#ifndef LE_WAVES
#define LE_WAVES 4  // 2 x the keypoints per workgroup (even: the LRF sums; odd: the normal)
#endif
__global__ void __launch_bounds__(64 * LE_WAVES) k_lrf_eig(int k, const int* __restrict__ cb,
                                                           const double* __restrict__ csum, double* __restrict__ eig,
                                                           int* __restrict__ okf, const float4* __restrict__ pts4,
                                                           const float* __restrict__ kps,
                                                           const long long* __restrict__ offs,
                                                           const unsigned int* __restrict__ seg, int nmax,
                                                           float4* __restrict__ normals) {
    __shared__ float fl[LE_WAVES / 2][3 * NF_STRIDE];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    // two waves per keypoint: the odd one computes the normal (nmax > 0), the even one the LRF eigen
    // system -- two independent sequential chains side by side instead of one after the other
    const int q = blockIdx.x * (LE_WAVES / 2) + (wave >> 1);
    if (q >= k) return;  // no workgroup barrier below
    if (wave & 1) {
        if (nmax > 0) {
            const long long o = offs[q];
            const float4 nv = segment_normal(pts4, kps[3 * q], kps[3 * q + 1], kps[3 * q + 2], seg + o, offs[q + 1] - o,
                                             nmax, fl[wave >> 1]);
            if (lane == 0) normals[q] = nv;
        }
        return;
    }
    const int c0 = cb[q], c1 = cb[q + 1];
    double acc = 0.0;
    long long valid = 0;
    if (lane < 8) {
        const double* col = csum + lane;
        int c = c0;
        for (; c + 8 <= c1; c += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = col[8 * (size_t)(c + u)];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (lane < 7) acc = acc + v[u];
                else valid += (long long)v[u];
            }
        }
        for (; c < c1; ++c) {
            const double v = col[8 * (size_t)c];
            if (lane < 7) acc = acc + v;
            else valid += (long long)v;
        }
    }
    double tot[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) tot[j] = __shfl(acc, j, 64);
    valid = __shfl(valid, 7, 64);
    if (lane == 0) {
        double e[7] = {0, 0, 0, 0, 0, 0, 0};
        const int ok = lrf_eig_of_sums(tot, valid, e);
        double* eo = eig + 8 * (size_t)q;
        if (ok)
            for (int j = 0; j < 6; ++j) eo[j] = e[j];
        eo[6] = e[6];
        okf[q] = ok;
    }
}

// PCL's sign disambiguation of keypoint q's eigenvectors e (count rule from the summed sign
// counts st / sn, median-5 rule over valid neighbours by rank) -> float LRF rows r9
__device__ __forceinline__ void lrf_fin_one(const float4* __restrict__ pts4, float kx, float ky, float kz,
                                            const unsigned int* __restrict__ sg, int n, const double* e, int st,
                                            int sn, float* r9) {
    const int valid_total = (int)e[6];
    double x[3] = {e[0], e[1], e[2]}, z[3] = {e[3], e[4], e[5]};
    int PT = 2 * st - valid_total;
    int PN = 2 * sn - valid_total;
    if (PT == 0 || PN == 0) {
        // median-5 rule over valid neighbours by rank. Excluded neighbours (exact duplicates of the
        // keypoint) have d2 == 0, so they sit in the leading d2 == 0 run: scan that run, then the
        // valid rank r lives at index r + (excluded count).
        const int med = valid_total / 2;
        int addT = 0, addN = 0;
        int z0n = 0, excl = 0;
        while (z0n < n) {
            const float4 p = pts4[sg[z0n]];
            if (__float_as_uint(d2_flann(kx, ky, kz, p.x, p.y, p.z)) != 0u) break;  // d2 > 0 (never -0)
            if (p.x == kx && p.y == ky && p.z == kz) ++excl;
            ++z0n;
        }
        for (int r = med - 2; r <= med + 2; ++r) {
            if (r < 0) continue;
            int i;
            if (r < z0n - excl) {
                // rank inside the zero run: walk it (at most a few keys)
                int rr = 0;
                i = -1;
                for (int u = 0; u < z0n; ++u) {
                    const float4 p = pts4[sg[u]];
                    if (p.x == kx && p.y == ky && p.z == kz) continue;
                    if (rr == r) { i = u; break; }
                    ++rr;
                }
            } else {
                i = r + excl;
            }
            if (i < 0 || i >= n) continue;
            const float4 p = pts4[sg[i]];
            const double vx = (double)(p.x - kx), vy = (double)(p.y - ky), vz = (double)(p.z - kz);
            if (((vx * x[0] + vy * x[1]) + vz * x[2]) > 0) addT++;
            if (((vx * z[0] + vy * z[1]) + vz * z[2]) > 0) addN++;
        }
        if (PT == 0 && addT < 3) { x[0] = -x[0]; x[1] = -x[1]; x[2] = -x[2]; }
        if (PN == 0 && addN < 3) { z[0] = -z[0]; z[1] = -z[1]; z[2] = -z[2]; }
    }
    if (PT < 0) { x[0] = -x[0]; x[1] = -x[1]; x[2] = -x[2]; }
    if (PN < 0) { z[0] = -z[0]; z[1] = -z[1]; z[2] = -z[2]; }
    const float x0 = (float)x[0], x1 = (float)x[1], x2 = (float)x[2];
    const float z0 = (float)z[0], z1 = (float)z[1], z2 = (float)z[2];
    r9[0] = x0; r9[1] = x1; r9[2] = x2;
    r9[3] = z1 * x2 - z2 * x1; r9[4] = z2 * x0 - z0 * x2; r9[5] = z0 * x1 - z1 * x0;
    r9[6] = z0; r9[7] = z1; r9[8] = z2;
}

__device__ __forceinline__ float dot4f_2(float a0, float a1, float a2, float b0, float b1, float b2) {
    return (a0 * b0 + a2 * b2) + (a1 * b1 + 0.0f);
}

#define PST2_RAD_45 0.78539816339744830961566084581988
#define PST2_RAD_90 1.5707963267948966192313216916398
#define PST2_RAD_135 2.3561944901923449288469825374596
#define PST2_RAD_PI_7_8 2.7488935718910690836548129603691

// the <= 5 (bin, value) interpolation records of neighbour idx, in PCL's add order (cos
// neighbour, radius, inclination, azimuth, main bin); unused slots: bin -1
// (from the neighbour's normal nv and point p, both already loaded)
__device__ __forceinline__ void shot_records_of(float4 nv, float4 p, float kx, float ky, float kz, float R,
                                                const float* rf, int* bins, float* vals) {
        const double Rd = (double)R;
        const double r12 = Rd / 2, r34 = (Rd * 3) / 4, r14 = Rd / 4;
        const int nr_bins = 10;
    #pragma unroll
        for (int j = 0; j < 5; ++j) { bins[j] = -1; vals[j] = 0.f; }
        if (__builtin_isfinite(nv.x) && __builtin_isfinite(nv.y) && __builtin_isfinite(nv.z)) {
            double cosd = (double)dot4f_2(nv.x, nv.y, nv.z, rf[6], rf[7], rf[8]);
            if (cosd > 1.0) cosd = 1.0;
            if (cosd < -1.0) cosd = -1.0;
            double bd = ((1.0 + cosd) * nr_bins) / 2;
            const float dx = p.x - kx, dy = p.y - ky, dz = p.z - kz;
            // the gather's d2 (same expression and operands as the ranked key's)
            const double distance = sqrt((double)d2_flann(kx, ky, kz, p.x, p.y, p.z));
            if (!(fabs(distance - 0.0) < 1e-15)) {
                double xr = (double)dot4f_2(dx, dy, dz, rf[0], rf[1], rf[2]);
                double yr = (double)dot4f_2(dx, dy, dz, rf[3], rf[4], rf[5]);
                double zr = (double)dot4f_2(dx, dy, dz, rf[6], rf[7], rf[8]);
                if (fabs(yr) < 1E-30) yr = 0;
                if (fabs(xr) < 1E-30) xr = 0;
                if (fabs(zr) < 1E-30) zr = 0;
                const unsigned bit4 = ((yr > 0) || ((yr == 0.0) && (xr < 0))) ? 1u : 0u;
                const unsigned bit3 = ((xr > 0) || ((xr == 0.0) && (yr > 0))) ? (bit4 ? 0u : 1u) : bit4;
                int desc = (int)((bit4 << 3) + (bit3 << 2));
                desc = desc << 1;
                if ((xr * yr > 0) || (xr == 0.0)) desc += (fabs(xr) >= fabs(yr)) ? 0 : 4;
                else desc += (fabs(xr) > fabs(yr)) ? 4 : 0;
                desc += zr > 0 ? 1 : 0;
                desc += (distance > r12) ? 2 : 0;
                const int step = (int)floor(bd + 0.5);
                const int vol = desc * (nr_bins + 1);
                bd -= step;
                double w = (1 - fabs(bd));
                if (bd > 0) { bins[0] = vol + ((step + 1) % nr_bins); vals[0] = (float)bd; }
                else { bins[0] = vol + ((step - 1 + nr_bins) % nr_bins); vals[0] = -(float)bd; }
                // the radial, inclination and azimuth interpolations in select form: each lane
                // evaluates exactly its branch's expressions, with one division per interpolation
                // for the whole wavefront (the lanes of a chunk take every branch)
                {
                    const bool outer = distance > r12;
                    const double rd = (distance - (outer ? r34 : r14)) / r12;
                    const bool self = outer ? distance > r34 : distance < r14;  // votes only for itself
                    const bool plus = outer ? !self : self;                      // w += 1 + rd
                    w += plus ? 1 + rd : 1 - rd;
                    if (!self) {
                        bins[1] = (desc + (outer ? -2 : 2)) * (nr_bins + 1) + step;
                        vals[1] = outer ? (float)(-rd) : (float)rd;
                    }
                }
                double ic = zr / distance;
                if (ic < -1.0) ic = -1.0;
                if (ic > 1.0) ic = 1.0;
                const double incl = bm::acos_sel(ic);
                {
                    const bool lower = incl > PST2_RAD_90 || (fabs(incl - PST2_RAD_90) < 1e-30 && zr <= 0);
                    const double id = (incl - (lower ? PST2_RAD_135 : PST2_RAD_45)) / PST2_RAD_90;
                    const bool self = lower ? incl > PST2_RAD_135 : incl < PST2_RAD_45;
                    const bool plus = lower ? !self : self;  // w += 1 + id
                    w += plus ? 1 + id : 1 - id;
                    if (!self) {
                        bins[2] = (desc + (lower ? 1 : -1)) * (nr_bins + 1) + step;
                        vals[2] = lower ? -(float)id : (float)id;
                    }
                }
                if (yr != 0.0 || xr != 0.0) {
                    const double az = bm::atan2_sel(yr, xr);
                    const int sel = desc >> 2;
                    double ad = (az - (-PST2_RAD_PI_7_8 + PST2_RAD_45 * sel)) / PST2_RAD_45;
                    ad = fmax(-0.5, fmin(ad, 0.5));
                    const bool pos = ad > 0;
                    w += pos ? 1 - ad : 1 + ad;
                    bins[3] = ((desc + (pos ? 4 : 28)) % 32) * (nr_bins + 1) + step;
                    vals[3] = pos ? (float)ad : -(float)ad;
                }
                bins[4] = vol + step;
                vals[4] = (float)w;
            }
        }
}

__device__ __forceinline__ void shot_records(const float4* __restrict__ pts4, const float4* __restrict__ normals,
                                             float kx, float ky, float kz, float R, const float* rf,
                                             unsigned int idx, int* bins, float* vals) {
    shot_records_of(normals[idx], pts4[idx], kx, ky, kz, R, rf, bins, vals);
}

// normalizeHistogram + B-SHOT of one keypoint's histogram h (wave-uniform q, good)
__device__ __forceinline__ void hist_finish(float* h, unsigned int* gcode, int q, bool good, int lane,
                                            float* __restrict__ shot_out, unsigned int* __restrict__ bits_out) {
    // normalizeHistogram: double accumulation of float squares in bin order
    float sv[6];
    if (good) {
        double acc = 0.0;
        if (lane == 0)
            for (int j = 0; j < 352; j += 8) {
                float hv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) hv[u] = h[j + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc = acc + (double)(hv[u] * hv[u]);
            }
        acc = __shfl(acc, 0, 64);
        const float fa = (float)sqrt(acc);
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const int b = lane + 64 * j;
            sv[j] = b < 352 ? h[b] / fa : 0.f;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 6; ++j) sv[j] = __builtin_nanf("");
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const int b = lane + 64 * j;
        if (b < 352) {
            h[b] = sv[j];
            if (shot_out) shot_out[352 * (size_t)q + b] = sv[j];
        }
    }
    __builtin_amdgcn_wave_barrier();
    // B-SHOT: 88 groups of 4 (include/bshot_bits.h:144-278)
    unsigned int code[2] = {0u, 0u};
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        const int gidx = lane + 64 * hh;
        if (gidx < 88) {
            const float v0 = h[4 * gidx], v1 = h[4 * gidx + 1], v2 = h[4 * gidx + 2], v3 = h[4 * gidx + 3];
            const float sum = ((v0 + v1) + v2) + v3;
            const double th = 0.9 * (double)sum;
            unsigned b;
            if (v0 == 0 && v1 == 0 && v2 == 0 && v3 == 0) b = 0;
            else if ((double)v0 > th) b = 1;
            else if ((double)v1 > th) b = 2;
            else if ((double)v2 > th) b = 4;
            else if ((double)v3 > th) b = 8;
            else if ((double)(v0 + v1) > th) b = 3;
            else if ((double)(v1 + v2) > th) b = 6;
            else if ((double)(v2 + v3) > th) b = 12;
            else if ((double)(v0 + v3) > th) b = 9;
            else if ((double)(v1 + v3) > th) b = 10;
            else if ((double)(v0 + v2) > th) b = 5;
            else if ((double)((v0 + v1) + v2) > th) b = 7;
            else if ((double)((v1 + v2) + v3) > th) b = 14;
            else if ((double)((v0 + v2) + v3) > th) b = 13;
            else if ((double)((v0 + v1) + v3) > th) b = 11;
            else b = 15;
            code[hh] = b;
        }
    }
    if (lane < 88) gcode[lane] = code[0];
    if (lane + 64 < 88) gcode[lane + 64] = code[1];
    __builtin_amdgcn_wave_barrier();
    if (lane < 11) {
        unsigned int w = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) w |= gcode[8 * lane + j] << (4 * j);
        bits_out[11 * (size_t)q + lane] = w;
    }
    __builtin_amdgcn_wave_barrier();
}

// Records and ordered apply fused: a workgroup per keypoint (LPT order); waves 1..HF_B compute the
// interpolation records of HF_B chunks into an LDS batch (shot_records) while wave 0 applies the
// previous batch in rank order (one in-order ds_add_f32 per rank on lanes 0..4: every bin sees its
// adds in PCL's order), double-buffered, so the records never leave LDS. The CU's LDS float-atomic
// unit (~3 cycles per lane-op) bounds the applying wave; keypoints launch in descending
// neighbourhood size so the largest start first.
#ifndef HF_NW
#define HF_NW 8
#endif
#ifndef HF_WPE
#define HF_WPE 0
#endif
#ifndef HF_PREF
#define HF_PREF 1  // producers load a chunk's normals and points one chunk ahead
#endif
#ifndef HF_PACK
#define HF_PACK 12  // ranks per ds_add_f32 in the packed apply (5 lanes each)
#endif
#ifndef HF_DIAG
#define HF_DIAG 0  // diagnostic builds only: 1 = no apply, 2 = no record computation
#endif
#ifndef HF_APQ
#define HF_APQ 4  // the applying wave reads a chunk's records in HF_APQ parts
#endif
#if HF_WPE > 0
#define HF_ATTR __attribute__((amdgpu_waves_per_eu(HF_WPE)))
#else
#define HF_ATTR
#endif
template <int HF_WAVES, int PACK>
__global__ void __launch_bounds__(64 * HF_WAVES) HF_ATTR k_hist_fused(const float4* __restrict__ pts4,
                                                              const float4* __restrict__ normals,
                                                              const float* __restrict__ kps, int k, float R,
                                                              const int* __restrict__ perm,
                                                              const long long* __restrict__ offs,
                                                              const int* __restrict__ cb,
                                                              const unsigned int* __restrict__ seg,
                                                              const double* __restrict__ eig,
                                                              const int* __restrict__ okf,
                                                              float* __restrict__ rf_out, int* __restrict__ ok_out,
                                                              float* __restrict__ shot_out,
                                                              unsigned int* __restrict__ bits_out) {
    constexpr int HF_B = HF_WAVES - 1;  // chunks per batch (one per producing wave)
    __shared__ float hist[384];
    __shared__ float rfs[9];
    __shared__ int okq;
    __shared__ int sgn[2];
    __shared__ unsigned int gcode[88];
    __shared__ __attribute__((aligned(16))) unsigned short sS[2][HF_B][320];  // [buffer][chunk][slot x 64 ranks]
    __shared__ __attribute__((aligned(16))) float sV[2][HF_B][320];
    __shared__ int suse[2][HF_B];  // [buffer][chunk]: bit j = the chunk has a slot-j record of nonzero value
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    if ((int)blockIdx.x >= k) return;
    const int q = perm[blockIdx.x];
    const long long o = offs[q];
    const int n = (int)(offs[q + 1] - o);
    const float kx = kps[3 * q], ky = kps[3 * q + 1], kz = kps[3 * q + 2];
    // the LRF's sign disambiguation first (SHOTLocalReferenceFrameEstimation: PCL's count rule, then
    // the median-5 rule on ties, lrf_fin_one): #(v . x >= 0) and #(v . z >= 0) over the valid
    // neighbours, counted by the whole workgroup (integers, any order)
    const int ok0 = okf[q];
    if (threadIdx.x < 2) sgn[threadIdx.x] = 0;
    __syncthreads();
    double ev[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) ev[j] = ok0 ? eig[8 * (size_t)q + j] : 0.0;
    if (ok0) {
        int pt = 0, pn = 0;
        // pipelined like the record producers: the next pass's point and the index after it are
        // loaded while this pass's dot products run
        constexpr int SP = 64 * HF_WAVES;
        auto sidx = [&](int i) -> unsigned int { return i < n ? seg[o + i] : 0u; };
        float4 pnext = pts4[sidx((int)threadIdx.x)];
        unsigned int inext = sidx((int)threadIdx.x + SP);
        for (int i0 = 0; i0 < n; i0 += SP) {
            const int i = i0 + (int)threadIdx.x;
            bool a = false, c = false;
            const float4 p = pnext;
            pnext = pts4[inext];
            inext = sidx(i + 2 * SP);
            if (i < n) {
                if (!(p.x == kx && p.y == ky && p.z == kz)) {
                    const double vx = (double)(p.x - kx), vy = (double)(p.y - ky), vz = (double)(p.z - kz);
                    a = ((vx * ev[0] + vy * ev[1]) + vz * ev[2]) >= 0;
                    c = ((vx * ev[3] + vy * ev[4]) + vz * ev[5]) >= 0;
                }
            }
            pt += __popcll(__ballot(a));
            pn += __popcll(__ballot(c));
        }
        if (lane == 0) {
            atomicAdd(&sgn[0], pt);
            atomicAdd(&sgn[1], pn);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float r9[9];
        if (ok0) {
            double e[7];
            for (int j = 0; j < 6; ++j) e[j] = ev[j];
            e[6] = eig[8 * (size_t)q + 6];
            lrf_fin_one(pts4, kx, ky, kz, seg + o, n, e, sgn[0], sgn[1], r9);
        } else {
            for (int j = 0; j < 9; ++j) r9[j] = __builtin_nanf("");
        }
        for (int j = 0; j < 9; ++j) {
            rfs[j] = r9[j];
            rf_out[9 * (size_t)q + j] = r9[j];
        }
        ok_out[q] = ok0;
        okq = ok0;
    }
    for (int j = threadIdx.x; j < 384; j += 64 * HF_WAVES) hist[j] = 0.0f;
    __syncthreads();
    const bool good = __builtin_isfinite(kx) && __builtin_isfinite(ky) && __builtin_isfinite(kz) && okq && n >= 5;
    const int nch = good ? cb[q + 1] - cb[q] : 0;
    float rf[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) rf[j] = good ? rfs[j] : 0.f;
#if HF_PREF
    // producer pipeline: wave w's chunks are m HF_B + w - 1, m = 0, 1, ...; a chunk's normals and
    // points are loaded while the previous chunk's records are computed, its indices one chunk
    // earlier still (the FP64 record code then waits on no gather)
    auto chunk_idx = [&](int t) -> unsigned int {
        const int i = t * 64 + lane;
        return (t < nch && i < n) ? seg[o + i] : 0u;
    };
    float4 cur_nv = make_float4(0.f, 0.f, 0.f, 0.f), cur_p = cur_nv;
    unsigned int nxt_idx = 0u;
    if (wave >= 1) {
        const unsigned int i0 = chunk_idx(wave - 1);
        nxt_idx = chunk_idx(HF_B + wave - 1);
        cur_nv = normals[i0];
        cur_p = pts4[i0];
    }
#endif
    auto produce = [&](int t, int buf, int bi) {
        const int i = t * 64 + lane;
        int bins[5] = {-1, -1, -1, -1, -1};
        float vals[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#if HF_PREF && HF_DIAG != 2
        const float4 nx_nv = normals[nxt_idx], nx_p = pts4[nxt_idx];
        nxt_idx = chunk_idx(t + 2 * HF_B);
        if (i < n) shot_records_of(cur_nv, cur_p, kx, ky, kz, R, rf, bins, vals);
        cur_nv = nx_nv;
        cur_p = nx_p;
#elif HF_DIAG == 2
        // diagnostic: no records computed (apply cost alone)
        if (i < n) {
#pragma unroll
            for (int j = 0; j < 5; ++j) { bins[j] = (64 * j + lane) % 352; vals[j] = 1.0f; }
        }
#else
        if (i < n) shot_records(pts4, normals, kx, ky, kz, R, rf, seg[o + i], bins, vals);
#endif
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            sS[buf][bi][64 * j + lane] = bins[j] < 0 ? (unsigned short)360 : (unsigned short)bins[j];
            sV[buf][bi][64 * j + lane] = bins[j] < 0 ? 0.f : vals[j];
        }
        // which slots hold a live record (nonzero value): slot 0 (the cosine interpolation) adds +-0
        // for every neighbour whose normal slot is zero, i.e. all but the few with index < K in the
        // reference's mis-indexed normals array; slot 1 (the radial one) is live only for distances
        // in [R/4, 3R/4], a contiguous rank range since ranks ascend in distance
        int use = 0;
#pragma unroll
        for (int j = 0; j < 5; ++j) use |= __ballot(bins[j] >= 0 && vals[j] != 0.f) != 0ull ? 1 << j : 0;
        if (lane == 0) suse[buf][bi] = use;
    };
    if (wave >= 1 && wave - 1 < nch) produce(wave - 1, 0, wave - 1);
    __syncthreads();
    const int nb = (nch + HF_B - 1) / HF_B;
    for (int b = 0; b < nb; ++b) {
        const int buf = b & 1;
        if (wave == 0) {
            // a slot whose records in this batch all add +-0 sits the batch out (one wave-uniform
            // exec mask per batch, no per-record branch): adding +-0 leaves a bin's bits unchanged
            // (bins start at +0 and every record value is >= +0 or -0, so no bin is ever -0), and the
            // LDS atomic unit's time is per active lane
            int use = 0;
            for (int bi = 0; bi < HF_B && b * HF_B + bi < nch; ++bi) use |= suse[buf][bi];
            if constexpr (PACK > 0) {
            // PACK ranks per ds_add_f32: lane 5 g + j applies slot j of rank r0 + g. Lanes that share a
            // bin within one instruction must be applied in ascending lane order (rank, then slot) --
            // what the LDS atomic unit does (experiments/microbench/lds_lane_order.hip; checked on the
            // device at context creation, lds_lane_order_mismatches, else PACK = 0 runs)
            {
                constexpr int G = PACK;
                const int g = lane / 5, j = lane - 5 * (lane / 5);
                if (HF_DIAG != 1 && lane < 5 * G && ((use >> j) & 1)) {
                    for (int bi = 0; bi < HF_B && b * HF_B + bi < nch; ++bi) {
                        const unsigned short* sb = &sS[buf][bi][64 * j];
                        const float* sv = &sV[buf][bi][64 * j];
                        unsigned int bn[(64 + G - 1) / G];
                        float vv[(64 + G - 1) / G];
#pragma unroll
                        for (int u = 0; u < (64 + G - 1) / G; ++u) {
                            const int r = G * u + g;
                            bn[u] = r < 64 ? (unsigned int)sb[r] : 360u;
                            vv[u] = r < 64 ? sv[r] : 0.f;
                        }
#pragma unroll
                        for (int u = 0; u < (64 + G - 1) / G; ++u)
                            if (vv[u] != 0.f) atomicAdd(&hist[bn[u]], vv[u]);
                    }
                }
            }
            } else if (HF_DIAG != 1 && lane < 5 && ((use >> lane) & 1)) {
                for (int part = 0; part < HF_APQ * HF_B && b * HF_B + part / HF_APQ < nch; ++part) {
                    // 64 / HF_APQ ranks of chunk part / HF_APQ at a time (keeps the applying path's
                    // registers low: the producers' FP64 code sets the kernel's VGPR budget)
                    const int bi = part / HF_APQ, r0 = (64 / HF_APQ) * (part % HF_APQ);
                    const uint4* b4 = reinterpret_cast<const uint4*>(&sS[buf][bi][64 * lane + r0]);
                    const float4* v4 = reinterpret_cast<const float4*>(&sV[buf][bi][64 * lane + r0]);
                    constexpr int NB = 8 / HF_APQ;  // uint4 (8 ranks) per part
                    uint4 bw[NB];
                    float4 vw[2 * NB];
#pragma unroll
                    for (int u = 0; u < NB; ++u) bw[u] = b4[u];
#pragma unroll
                    for (int u = 0; u < 2 * NB; ++u) vw[u] = v4[u];
#pragma unroll
                    for (int u = 0; u < NB; ++u) {
                        const unsigned int w[4] = {bw[u].x, bw[u].y, bw[u].z, bw[u].w};
#pragma unroll
                        for (int h = 0; h < 4; ++h) {
                            const int r = 8 * u + 2 * h;
                            const float4 va = vw[r >> 2];
                            const float v0 = (r & 3) == 0 ? va.x : va.z;
                            const float v1 = (r & 3) == 0 ? va.y : va.w;
                            atomicAdd(&hist[w[h] & 0xFFFFu], v0);
                            atomicAdd(&hist[w[h] >> 16], v1);
                        }
                    }
                }
            }
        } else {
            const int t = (b + 1) * HF_B + wave - 1;
            if (t < nch) produce(t, buf ^ 1, wave - 1);
        }
        __syncthreads();
    }
    if (wave == 0) hist_finish(hist, gcode, q, good, lane, shot_out, bits_out);
}

// The packed SHOT apply needs one ds_add_f32 to apply lanes that share an address in ascending lane
// order. 8 waves, each on its own 64 bins: LC_TRIALS trials of LC_OPS atomic adds with hashed
// addresses (1, 4, 16 or 64 distinct), exec masks and values of mixed magnitude (order-sensitive
// float sums); lane 0 of each wave replays every trial sequentially in ascending lane order and the
// wave counts the bins whose bits differ. out[0] += mismatches, out[1] += order-sensitive bins (where
// the descending order differs: the check's power).
#define LC_TRIALS 16
#define LC_OPS 16
__device__ __forceinline__ unsigned int lc_hash(unsigned int a, unsigned int b, unsigned int c) {
    unsigned int h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return h;
}
__device__ __forceinline__ float lc_val(unsigned int h) {
    const float m = (float)(h & 0xFFFFFu) / 1048576.0f - 0.5f;
    return ldexpf(m, (int)((h >> 20) % 40u) - 20);
}
__device__ __forceinline__ unsigned long long lc_mask(unsigned int t, unsigned int op) {
    const unsigned int k = op % 3u;
    if (k == 0) return ~0ull;
    if (k == 1) return 0x0FFFFFFFFFFFFFFFull;  // the packed apply's 60 lanes
    return ((unsigned long long)lc_hash(t, op, 1000u) << 32) | lc_hash(t, op, 2000u);
}
__global__ void __launch_bounds__(512) k_lds_lane_order(unsigned int seed, int* __restrict__ out) {
    __shared__ float bins[8][64];
    __shared__ float ref[8][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int mism = 0, sens = 0;
    for (int t0 = 0; t0 < LC_TRIALS; ++t0) {
        const unsigned int t = seed + (unsigned int)(blockIdx.x * 8 + wave) * LC_TRIALS + (unsigned int)t0;
        const float init = lc_val(lc_hash(t, 77u, (unsigned int)lane)) * 1000.f;
        bins[wave][lane] = init;
        ref[wave][lane] = init;
        __builtin_amdgcn_wave_barrier();
        for (unsigned int op = 0; op < LC_OPS; ++op) {
            const unsigned int span = 1u << (2u * (op & 3u));  // 1, 4, 16, 64
            const unsigned int h = lc_hash(t, op, (unsigned int)lane);
            if ((lc_mask(t, op) >> lane) & 1ull) atomicAdd(&bins[wave][h % span], lc_val(h >> 6));
        }
        __builtin_amdgcn_wave_barrier();
        float dn = init;  // descending replay of this lane's bin (the check's power)
        if (lane == 0) {
            for (unsigned int op = 0; op < LC_OPS; ++op) {
                const unsigned int span = 1u << (2u * (op & 3u));
                const unsigned long long m = lc_mask(t, op);
                for (int l = 0; l < 64; ++l) {
                    const unsigned int h = lc_hash(t, op, (unsigned int)l);
                    if ((m >> l) & 1ull) ref[wave][h % span] = ref[wave][h % span] + lc_val(h >> 6);
                }
            }
        }
        for (unsigned int op = 0; op < LC_OPS; ++op) {
            const unsigned int span = 1u << (2u * (op & 3u));
            const unsigned long long m = lc_mask(t, op);
            for (int l = 63; l >= 0; --l) {
                const unsigned int h = lc_hash(t, op, (unsigned int)l);
                if (((m >> l) & 1ull) && (int)(h % span) == lane) dn = dn + lc_val(h >> 6);
            }
        }
        __builtin_amdgcn_wave_barrier();
        mism += __float_as_uint(bins[wave][lane]) != __float_as_uint(ref[wave][lane]) ? 1 : 0;
        sens += __float_as_uint(dn) != __float_as_uint(ref[wave][lane]) ? 1 : 0;
        __builtin_amdgcn_wave_barrier();
    }
    if (mism) atomicAdd(&out[0], mism);
    if (sens) atomicAdd(&out[1], sens);
}

}  // namespace bsk

namespace bsh {

int lds_lane_order_check(int* sensitive) {
    int* d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(int)) != hipSuccess) return -1;
    int h[2] = {0, 0};
    bool ok = hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) == hipSuccess;
    if (ok) {
        bsk::k_lds_lane_order<<<64, 512>>>(12345u, d);
        ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
             hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess;
    }
    (void)hipFree(d);
    if (!ok) return -1;
    if (sensitive) *sensitive = h[1];
    return h[0];
}

// part 0: in-bucket rank (sorted segments); 1: LRF; 2: histogram records + ordered apply
hipError_t launch_describe2(const Describe2Args& A, int part, hipStream_t s) {
    if (A.k <= 0) return hipSuccess;
    hipError_t e;
    int cblocks = (A.n_chunks + 3) / 4;
    if (A.max_blocks > 0 && cblocks > A.max_blocks) cblocks = A.max_blocks;
    if (part == 0) {
        if (A.n_chunks > 0) {
            bsk::k_chunk_owner<<<A.k, 256, 0, s>>>(A.k, A.cb, A.owner, A.offs, A.cinfo);
            if (A.rank_wg) {
                // slices (option desc_slices): consecutive ranges of the LPT order, each launch shorter, so
                // the main stream's small grids find CUs between them; results do not depend on it
                const int step = (A.k + A.slices - 1) / (A.slices > 0 ? A.slices : 1);
                for (int s0 = 0; s0 < A.k; s0 += step)
                    if ((e = launch_shot_rank_wg(std::min(step, A.k - s0), A.R, A.pts4, A.kps, A.perm + s0, A.offs, A.bstart, A.seg, A.sorted, s,
                                                 A.rank_max)))
                        return e;
            } else if ((e = launch_shot_rank(A.k, A.n_chunks, A.R, A.pts4, A.kps, A.offs, A.cb, A.owner, A.bstart, A.seg, A.sorted, s, A.cinfo,
                                             A.max_blocks))) {
                return e;
            }
        }
        return hipGetLastError();
    }
    if (part == 1) {
        if (A.n_chunks > 0) {
            bsk::k_lrf_chunks<<<cblocks, 256, 0, s>>>(A.pts4, A.kps, A.k, A.R, A.offs, A.cb, A.owner, A.sorted,
                                                       A.csum, A.cinfo);
        }
        // nmax > 0: the keypoint normals from the sorted segments in the same launch
        bsk::k_lrf_eig<<<(A.k + LE_WAVES / 2 - 1) / (LE_WAVES / 2), 64 * LE_WAVES, 0, s>>>(
            A.k, A.cb, A.csum, A.eig, A.okf, A.pts4, A.kps, A.offs, A.sorted, A.nseg_max_nn, A.normals_out);
        // the sign counts and PCL's sign rule (k_lrf_sign / k_lrf_fin of round 2) run at the start of
        // the histogram kernel
        return hipGetLastError();
    }
    // HF_NW waves per workgroup: 1 applies, HF_NW - 1 produce records
#ifdef DIAG_HF_TWICE
    // diagnostic builds only: the histogram kernel twice (idempotent) -- its marginal cost
    if (A.hf_pack)
        bsk::k_hist_fused<HF_NW, HF_PACK><<<A.k, 64 * HF_NW, 0, s>>>(A.pts4, A.normals, A.kps, A.k, A.R, A.perm, A.offs, A.cb,
                                                               A.sorted, A.eig, A.okf, A.rf, A.ok, A.shot, A.bits);
#endif
    const int step = (A.k + A.slices - 1) / (A.slices > 0 ? A.slices : 1);
    for (int s0 = 0; s0 < A.k; s0 += step) {
        const int m = std::min(step, A.k - s0);
        if (A.hf_pack)
            bsk::k_hist_fused<HF_NW, HF_PACK><<<m, 64 * HF_NW, 0, s>>>(A.pts4, A.normals, A.kps, m, A.R, A.perm + s0, A.offs,
                                                                   A.cb, A.sorted, A.eig, A.okf, A.rf, A.ok, A.shot, A.bits);
        else
            bsk::k_hist_fused<HF_NW, 0><<<m, 64 * HF_NW, 0, s>>>(A.pts4, A.normals, A.kps, m, A.R, A.perm + s0, A.offs, A.cb,
                                                             A.sorted, A.eig, A.okf, A.rf, A.ok, A.shot, A.bits);
    }
    return hipGetLastError();
}

}  // namespace bsh
