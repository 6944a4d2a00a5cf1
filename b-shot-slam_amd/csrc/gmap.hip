// gmap.hip -- the keypoint map on the GPU: Map::addKeypoint with the 800 mm
// suppression (src/mymap.cpp:4-26), Keypoint::createKeypoint's 10 mm grid (src/keypoint.cpp:23-32),
// getBlockID (src/mymap.cpp:95-105), and Map::getKeypoints' 21^3 block loop (src/mymap.cpp:28-74)
// with the ref keypoints appended (src/lidar_odometry.cpp:195-207) -- the matching targets are
// assembled in HBM, where the Hamming matcher and ICP read them.
//
// Order. A block's entries come out in the iteration order of the reference's
// std::unordered_map<Vector3f, Keypoint::Ptr, MapHasher> (include/mymap.h:11-25), restated by
// umap_order.h (checked against libstdc++ itself); that order decides first-index ties in the
// Hamming match, so this mode is bit-exact with the host map. Mode 2 ("canonical") emits a block's
// entries in insertion order instead (not the reference's order; the oracle has the same mode).
//
// Layout (device, grow-only):
//   slots      kpos[s] = (x, y, z, ratio) on the 10 mm grid, kdesc[s] = 11 words; every keypoint a
//              sweep offers gets a slot (slot_base + i), rejected ones are never referenced
//   blocks     open-addressed table block id -> block index; GBlock headers
//   members    per block, in insertion order: mslot (current slot of the key: a replaced value
//              points at the newer slot), hash code; plus ord[n] (iteration order), pos (inverse)
//              and the bucket array of the restated libstdc++ table -- all in two bump pools
// Insert: one wave per block touched by the sweep, its keypoints in sweep order (the reference's
// loop order); the block's arrays are staged in LDS, the suppression scan and the list shifts are
// wave-parallel, the libstdc++ bookkeeping runs on lane 0.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.h"
#include "kernels.h"
#include "dev_common.h"
#include "gmap.h"
#include "umap_order.h"

namespace bsk {

using bsh::GBlock;
using bsh::GM_CTOP;
using bsh::GM_ERR;
using bsh::GM_ITOP;
using bsh::GM_LDS_BK;
using bsh::GM_LDS_N;
using bsh::GM_MEMBERS;
using bsh::GM_NBLOCKS;
using bsh::GM_NSEG;
using bsh::GM_REC_HDR;
using bsh::GM_REC_W;

struct GMapDev {
    float4* kpos;
    unsigned int* kdesc;
    unsigned long long* tkey;
    int* tval;
    unsigned int tmask;
    GBlock* blk;
    int blk_cap;
    int* ctr;  // GM_* counters
    int* ipool;
    long long ipool_cap;
    unsigned long long* cpool;
    long long cpool_cap;
};

__device__ __forceinline__ unsigned long long block_id_of(float gx, float gy, float gz) {
    // Map::getBlockID: low 21 bits of each coordinate of the 10 m grid position
    const int prec = 10000;
    const int bx = (int)(float)((int)roundf(gx / (float)prec) * prec);
    const int by = (int)(float)((int)roundf(gy / (float)prec) * prec);
    const int bz = (int)(float)((int)roundf(gz / (float)prec) * prec);
    const unsigned long long i = ((unsigned long long)(long long)bx << 42) & (0x1FFFFFull << 42);
    const unsigned long long j = ((unsigned long long)(long long)by << 21) & (0x1FFFFFull << 21);
    const unsigned long long k = ((unsigned long long)(long long)bz) & 0x1FFFFFull;
    return i | j | k;
}

__device__ __forceinline__ unsigned long long map_hash(float x, float y, float z) {
    // MapHasher: abs(round(p.sum())) on the float sum, Eigen's redux order x + (y + z)
    return (unsigned long long)fabsf(roundf(x + (y + z)));
}

__device__ __forceinline__ int find_block(const GMapDev& m, unsigned long long id) {
    unsigned int h = hash_key(id) & m.tmask;
    for (unsigned int probe = 0; probe <= m.tmask; ++probe) {
        const unsigned long long k = m.tkey[h];
        if (k == id) return m.tval[h];
        if (k == BS_EMPTY_KEY) return -1;
        h = (h + 1) & m.tmask;
    }
    return -1;
}

// the sweep's keypoints -> world position on the 10 mm grid (updateMap: R * p + T, then
// createKeypoint), their slots, block ids (sort keys) and hash codes
__global__ void k_gmap_prep(const float* __restrict__ kps, const float* __restrict__ ratio,
                            const unsigned int* __restrict__ bits, int k, Xf16g T, int slot_base, GMapDev m,
                            unsigned long long* __restrict__ keys, unsigned int* __restrict__ vals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    const float x = kps[3 * i], y = kps[3 * i + 1], z = kps[3 * i + 2];
    // Matrix3f * Vector3f (Eigen 3.2 coefficient order) + T
    const float wx = ((T.m[0] * x + T.m[1] * y) + T.m[2] * z) + T.m[3];
    const float wy = ((T.m[4] * x + T.m[5] * y) + T.m[6] * z) + T.m[7];
    const float wz = ((T.m[8] * x + T.m[9] * y) + T.m[10] * z) + T.m[11];
    const float gx = (float)((int)truncf(wx / 10.f) * 10);
    const float gy = (float)((int)truncf(wy / 10.f) * 10);
    const float gz = (float)((int)truncf(wz / 10.f) * 10);
    const int s = slot_base + i;
    m.kpos[s] = make_float4(gx, gy, gz, ratio[i]);
#pragma unroll
    for (int w = 0; w < 11; ++w) m.kdesc[11 * (size_t)s + w] = bits[11 * (size_t)i + w];
    keys[i] = block_id_of(gx, gy, gz);
    vals[i] = (unsigned int)i;
}

// Exchange records (BASELINE config 4): word 0 of a 16-word header = the count (int bits), then kmax
// records of 15 words: x, y, z (10 mm grid, world), ratio, 11 descriptor words.
__global__ void k_gmap_pack(GMapDev m, int slot_base, int k, int kmax, float* __restrict__ rec) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) rec[0] = __int_as_float(k);
    if (i >= k) return;
    const int s = slot_base + i;
    float* r = rec + GM_REC_HDR + GM_REC_W * (size_t)i;
    const float4 p = m.kpos[s];
    r[0] = p.x; r[1] = p.y; r[2] = p.z; r[3] = p.w;
#pragma unroll
    for (int w = 0; w < 11; ++w) r[4 + w] = __uint_as_float(m.kdesc[11 * (size_t)s + w]);
}

// a record batch -> slots (positions are already on the grid: createKeypoint is idempotent on them),
// block ids; records past the count get the empty key (sorted last, skipped by k_gmap_segments)
__device__ __forceinline__ void prep_rec_at(const float* __restrict__ rec, int i, int kmax, int slot_base, const GMapDev& m,
                                            unsigned long long* __restrict__ keys, unsigned int* __restrict__ vals) {
    if (i >= kmax) return;
    const int cnt = __float_as_int(rec[0]);
    vals[i] = (unsigned int)i;
    if (i >= cnt) {
        keys[i] = BS_EMPTY_KEY;
        return;
    }
    const float* r = rec + GM_REC_HDR + GM_REC_W * (size_t)i;
    const int s = slot_base + i;
    m.kpos[s] = make_float4(r[0], r[1], r[2], r[3]);
#pragma unroll
    for (int w = 0; w < 11; ++w) m.kdesc[11 * (size_t)s + w] = __float_as_uint(r[4 + w]);
    keys[i] = block_id_of(r[0], r[1], r[2]);
}

__global__ void k_gmap_prep_rec(const float* __restrict__ rec, int kmax, int slot_base, GMapDev m,
                                unsigned long long* __restrict__ keys, unsigned int* __restrict__ vals) {
    prep_rec_at(rec, blockIdx.x * blockDim.x + threadIdx.x, kmax, slot_base, m, keys, vals);
}

// the block of id: found, or created (um::initial(): one bucket, nothing allocated); -1 past capacity
__device__ int find_or_create_block(const GMapDev& m, unsigned long long id) {
    int b = find_block(m, id);
    if (b >= 0) return b;
    b = atomicAdd(&m.ctr[GM_NBLOCKS], 1);
    if (b >= m.blk_cap) {
        atomicOr(&m.ctr[GM_ERR], 1);
        return -1;
    }
    GBlock B;
    B.id = id;
    B.n = 0; B.bkt = 1; B.next_resize = 0; B.cap = 0;
    B.mslot = B.ord = B.pos = B.code = -1;
    B.bk = -1; B.bk_cap = 0;
    m.blk[b] = B;
    unsigned int h = hash_key(id) & m.tmask;
    while (atomicCAS(&m.tkey[h], BS_EMPTY_KEY, id) != BS_EMPTY_KEY) h = (h + 1) & m.tmask;
    m.tval[h] = b;
    return b;
}

// one thread per run of equal block ids in the sorted keys: find or create the block, record the run
__global__ void k_gmap_segments(const unsigned long long* __restrict__ keys, int k, GMapDev m, int* __restrict__ seg) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    const unsigned long long id = keys[j];
    if (id == BS_EMPTY_KEY) return;  // padding of a record batch (k_gmap_prep_rec)
    if (j > 0 && keys[j - 1] == id) return;
    int lo = j + 1, hi = k;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] == id) lo = mid + 1;
        else hi = mid;
    }
    const int b = find_or_create_block(m, id);
    if (b < 0) return;
    const int s = atomicAdd(&m.ctr[GM_NSEG], 1);
    seg[3 * s] = j;
    seg[3 * s + 1] = lo - j;
    seg[3 * s + 2] = b;
}

// Batches of <= GM_SORT_MAX keypoints (every own-map insert: K <= 4096): the sort, the runs and the
// segment count in one workgroup. Bitonic sort of (block id, index) pairs in LDS: the indices are
// the batch's sweep order and unique, so the order equals the stable radix sort's. Segments are
// numbered by an exclusive scan of the run starts (deterministic, no counter to clear). Writes the
// sorted indices to vals_out and m.ctr[GM_NSEG].
#define GM_SORT_MAX 4096
#ifndef GM_SORT_T
#define GM_SORT_T 1024  // 256 threads: 40 -> 85 us per launch under load, the same sweeps/s (r05g)
#endif
__device__ __forceinline__ void sort_segments_wg(const unsigned long long* __restrict__ keys,
                                                 const unsigned int* __restrict__ vals, int k, GMapDev m,
                                                 unsigned int* __restrict__ vals_out, int* __restrict__ seg) {
    __shared__ unsigned long long sk[GM_SORT_MAX];
    __shared__ unsigned int sv[GM_SORT_MAX];
    __shared__ int wsum[GM_SORT_T / 64];
    const int t = threadIdx.x;
    int P = 64;
    while (P < k) P <<= 1;
    for (int i = t; i < P; i += GM_SORT_T) {
        sk[i] = i < k ? keys[i] : BS_EMPTY_KEY;
        sv[i] = i < k ? vals[i] : 0xFFFFFFFFu;
    }
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = t; i < P / 2; i += GM_SORT_T) {
                const int a = 2 * i - (i & (stride - 1));  // lower index of the pair
                const int b = a + stride;
                const bool up = (a & size) == 0;
                const unsigned long long ka = sk[a], kb = sk[b];
                const unsigned int va = sv[a], vb = sv[b];
                const bool gt = ka > kb || (ka == kb && va > vb);
                if (gt == up) {
                    sk[a] = kb; sk[b] = ka;
                    sv[a] = vb; sv[b] = va;
                }
            }
            __syncthreads();
        }
    }
    for (int i = t; i < k; i += GM_SORT_T) vals_out[i] = sv[i];
    // runs: each thread owns GM_SORT_MAX / GM_SORT_T consecutive positions
    constexpr int PER = GM_SORT_MAX / GM_SORT_T;
    const int j0 = PER * t;
    int starts = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int j = j0 + u;
        starts += (j < k && sk[j] != BS_EMPTY_KEY && (j == 0 || sk[j - 1] != sk[j])) ? 1 : 0;
    }
    // exclusive scan of the per-thread counts (wave scan, then the waves' totals)
    const int lane = t & 63, wv = t >> 6;
    int incl = starts;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wv; ++w) base += wsum[w];
    int s = base + incl - starts;
    if (t == GM_SORT_T - 1) m.ctr[GM_NSEG] = base + incl;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int j = j0 + u;
        if (!(j < k && sk[j] != BS_EMPTY_KEY && (j == 0 || sk[j - 1] != sk[j]))) continue;
        const unsigned long long id = sk[j];
        int e = j + 1, hi = k;
        while (e < hi) {
            const int mid = (e + hi) >> 1;
            if (sk[mid] == id) e = mid + 1;
            else hi = mid;
        }
        // a block past capacity (error bit set) leaves an empty run: the insert skips it
        const int b = find_or_create_block(m, id);
        seg[3 * s] = j;
        seg[3 * s + 1] = b < 0 ? 0 : e - j;
        seg[3 * s + 2] = b < 0 ? 0 : b;
        ++s;
    }
}

__global__ void __launch_bounds__(GM_SORT_T) k_gmap_sort_segments(const unsigned long long* __restrict__ keys,
                                                                 const unsigned int* __restrict__ vals, int k,
                                                                 GMapDev m, unsigned int* __restrict__ vals_out,
                                                                 int* __restrict__ seg) {
    sort_segments_wg(keys, vals, k, m, vals_out, seg);
}

// Batched replica inserts (the exchange: one sweep's offers into up to GM_XB replicas): one launch
// per stage for all of them, the replica in blockIdx.y (insert, prep) or blockIdx.x (sort). The job
// table travels as a kernel argument (blockIdx-uniform: scalar loads from the argument segment).
#define GM_XB 8
struct GMapJob {
    GMapDev m;
    const float* rec;          // record batch (count in the header)
    unsigned long long* keys;  // scratch: kmax block ids
    unsigned int* vals;        // scratch: 2 kmax (batch order, then the sorted order)
    int* seg;                  // scratch: 3 kmax
    int* p_ctr;                // pinned copy of the counters (host-coherent)
    int slot_base;
};
struct GMapJobs {
    GMapJob j[GM_XB];
};

__global__ void k_gmap_prep_rec_x(GMapJobs J, int kmax) {
    const GMapJob& jb = J.j[blockIdx.y];
    prep_rec_at(jb.rec, blockIdx.x * blockDim.x + threadIdx.x, kmax, jb.slot_base, jb.m, jb.keys, jb.vals);
}

__global__ void __launch_bounds__(GM_SORT_T) k_gmap_sort_segments_x(GMapJobs J, int k) {
    const GMapJob& jb = J.j[blockIdx.x];
    sort_segments_wg(jb.keys, jb.vals, k, jb.m, jb.vals + k, jb.seg);
}

// every replica's counters -> its pinned copy (one wave per replica)
__global__ void k_gmap_ctr_x(GMapJobs J) {
    const GMapJob& jb = J.j[blockIdx.x];
    if (threadIdx.x < bsh::GM_QTOT) jb.p_ctr[threadIdx.x] = jb.m.ctr[threadIdx.x];
}

// bump allocation from a pool (lane 0); false when the pool is exhausted (error bit 2)
__device__ __forceinline__ bool pool_alloc(int* ctr_top, long long cap, long long need, int* err, long long* off) {
    const long long o = (long long)atomicAdd(ctr_top, (int)need);
    if (o + need > cap) {
        atomicOr(err, 2);
        return false;
    }
    *off = o;
    return true;
}

// one workgroup per touched block (grid-strides over the device-side segment count). A batch's
// candidates are first tested against the block's members as staged (all pairs, in parallel):
// members are never removed and their ratios only change through an exact-position replacement,
// so until the batch makes one, a candidate is rejected exactly when a staged member or a member
// the batch has added so far rejects it. The candidates then go in sweep order: the added members
// are tested, the insert position is found (lane 0, um::) and the bucket-order list is shifted by
// the whole workgroup. After a replacement the remaining candidates are tested against every member.
#define GM_INS_T 512
#define GM_SMALL_N 1024   // members: buckets stay <= 1109 (the libstdc++ prime after 541)
#define GM_SMALL_BK 1152
template <int LN, int LBK>
__device__ __forceinline__ void insert_wg(const GMapDev& m, const unsigned int* __restrict__ vals, int* __restrict__ seg,
                                          int slot_base, int wg, int nwg) {
    // the block's LDS image (142 KiB, one workgroup per CU; a sweep touches ~100 blocks): list
    // indices as ushort, hash codes as u32 (10 mm-grid keys), each member's current position + ratio,
    // and the batch's per-candidate results against the staged members
    __shared__ unsigned short s_ord[LN], s_pos[LN], s_nxt[LN], s_bk[LBK];
    __shared__ int s_slot[LN];
    __shared__ unsigned int s_code[LN];
    __shared__ float4 s_mem[LN];
    __shared__ unsigned short s_hit0[LN];  // staged member at the candidate's position (0xFFFF: none)
    __shared__ unsigned char s_rej0[LN];   // rejected by a staged member
    __shared__ int s_rej, s_hit, s_at, s_nb, s_nr;
    __shared__ GBlock s_B;
    const int tid = threadIdx.x;
    const int nseg = m.ctr[GM_NSEG];
    for (int sg = wg; sg < nseg; sg += nwg) {
        const int j0 = seg[3 * sg], cnt = seg[3 * sg + 1], b = seg[3 * sg + 2];
        if (cnt == 0) continue;  // a run whose block could not be created (GM_ERR is set)
        GBlock B = m.blk[b];
        // two instantiations split the blocks: the small LDS image (<= GM_SMALL_N members after the
        // batch) leaves the CU room for other kernels' workgroups; the full one takes the rest
        if (B.n + cnt > LN) {
            if (LN == GM_LDS_N && tid == 0) atomicOr(&m.ctr[GM_ERR], 4);  // block larger than the LDS image
            continue;
        }
        if (LN == GM_LDS_N && B.n + cnt <= GM_SMALL_N) continue;
        // stage the block
        for (int i = tid; i < B.n; i += GM_INS_T) {
            s_ord[i] = (unsigned short)m.ipool[B.ord + i];
            s_pos[i] = (unsigned short)m.ipool[B.pos + i];
            const int sl = m.ipool[B.mslot + i];
            s_slot[i] = sl;
            s_mem[i] = m.kpos[sl];
            s_code[i] = (unsigned int)m.cpool[B.code + i];
        }
        if (B.bk >= 0)
            for (int i = tid; i < B.bkt; i += GM_INS_T) s_bk[i] = (unsigned short)m.ipool[B.bk + i];
        for (int t = tid; t < cnt; t += GM_INS_T) {
            s_hit0[t] = 0xFFFF;
            s_rej0[t] = 0;
        }
        __syncthreads();
        // src/mymap.cpp:14-22: rejected when a keypoint of the block within 800 mm has a
        // segmentation ratio >= this one's; an exact key hit is the entry operator[] replaces.
        // Threads = C candidates (their loads all in flight) x R member ranges, members read from LDS.
        const int S0 = B.n;
        {
            const int C = cnt < GM_INS_T ? cnt : GM_INS_T, R = GM_INS_T / C;
            const int part = tid / C, tc = tid - part * C;
            const int span = (S0 + R - 1) / R, i0 = part * span, i1 = min(S0, i0 + span);
            if (part < R && i0 < i1)
                for (int t = tc; t < cnt; t += C) {
                    const float4 p = m.kpos[slot_base + (int)vals[j0 + t]];
                    bool r = false;
                    int h = -1;
                    for (int i = i0; i < i1; ++i) {
                        const float4 e = s_mem[i];
                        const float dx = p.x - e.x, dy = p.y - e.y, dz = p.z - e.z;
                        r = r || (sqrtf(dx * dx + (dy * dy + dz * dz)) < 800.f && p.w <= e.w);
                        if (e.x == p.x && e.y == p.y && e.z == p.z) h = i;  // members are unique
                    }
                    if (r) s_rej0[t] = 1;
                    if (h >= 0) s_hit0[t] = (unsigned short)h;
                }
        }
        __syncthreads();
        um::State S{B.n, B.bkt, B.next_resize};
        int added = 0;
        bool exact = false;  // a replacement changed a staged member's ratio: full scans from here on
        for (int t = 0; t < cnt; ++t) {
            if (!exact && s_rej0[t]) continue;  // rejected by a staged member
            const int slot = slot_base + (int)vals[j0 + t];
            const float4 p = m.kpos[slot];
            const int lo = exact ? 0 : S0;  // members to test now
            bool rej = false;
            int hit = (!exact && s_hit0[t] != 0xFFFF) ? (int)s_hit0[t] : -1;
            if (!rej && S.n > lo) {
                if (tid == 0) { s_rej = 0; s_hit = 0x7FFFFFFF; }
                __syncthreads();
                bool r = false;
                int h = 0x7FFFFFFF;
                for (int i = lo + tid; i < S.n; i += GM_INS_T) {
                    const float4 e = s_mem[i];
                    const float dx = p.x - e.x, dy = p.y - e.y, dz = p.z - e.z;
                    if (sqrtf(dx * dx + (dy * dy + dz * dz)) < 800.f && p.w <= e.w) r = true;
                    if (e.x == p.x && e.y == p.y && e.z == p.z) h = i;
                }
                if (r) s_rej = 1;
                if (h != 0x7FFFFFFF) atomicMin(&s_hit, h);
                __syncthreads();
                rej = s_rej != 0;
                if (s_hit != 0x7FFFFFFF) hit = s_hit;
                __syncthreads();  // s_rej / s_hit are rewritten by the next candidate
            }
            if (rej) continue;
            if (hit >= 0) {
                if (tid == 0) { s_slot[hit] = slot; s_mem[hit] = p; }
                exact = true;
                __syncthreads();
                continue;
            }
            const int x = S.n;
            if (tid == 0) {
                const unsigned long long code = map_hash(p.x, p.y, p.z);
                if (code > 0xFFFFFFFFull) atomicOr(&m.ctr[GM_ERR], 8);
                s_slot[x] = slot;
                s_mem[x] = p;
                s_code[x] = (unsigned int)code;
                int nb;
                if (um::need_rehash(S, &nb)) um::rehash(S, nb, s_ord, s_pos, s_code, s_bk, s_nxt);
                s_at = um::insert_position(S, x, s_ord, s_pos, s_code, s_bk);
                s_nb = S.bkt;
                s_nr = S.next_resize;
            }
            __syncthreads();
            const int at = s_at;
            S.bkt = s_nb;
            S.next_resize = s_nr;
            // shift ord[at, n) one place up, top chunk first (reads of a chunk never overlap the
            // writes of the chunks before it)
            for (int hi = S.n; hi > at; hi -= GM_INS_T) {
                const int i = hi - tid;
                unsigned short v = 0;
                if (i > at) v = s_ord[i - 1];
                __syncthreads();
                if (i > at) { s_ord[i] = v; s_pos[v] = (unsigned short)i; }
                __syncthreads();
            }
            if (tid == 0) { s_ord[at] = (unsigned short)x; s_pos[x] = (unsigned short)at; }
            __syncthreads();
            S.n += 1;
            ++added;
        }
        // write the block back (arrays regrow by doubling)
        if (tid == 0) {
            long long off = 0;
            bool ok = true;
            if (S.n > B.cap) {
                const int nc = std::max(16, std::max(S.n, 2 * B.cap));
                long long io = 0, co = 0;
                ok = pool_alloc(&m.ctr[GM_ITOP], m.ipool_cap, 3LL * nc, &m.ctr[GM_ERR], &io) &&
                     pool_alloc(&m.ctr[GM_CTOP], m.cpool_cap, nc, &m.ctr[GM_ERR], &co);
                if (ok) {
                    B.cap = nc;
                    B.ord = (int)io; B.pos = (int)(io + nc); B.mslot = (int)(io + 2 * nc);
                    B.code = (int)co;
                }
            }
            if (ok && S.bkt > B.bk_cap) {
                ok = pool_alloc(&m.ctr[GM_ITOP], m.ipool_cap, S.bkt, &m.ctr[GM_ERR], &off);
                if (ok) { B.bk = (int)off; B.bk_cap = S.bkt; }
            }
            s_rej = ok ? 1 : 0;
            if (ok) {
                B.n = S.n; B.bkt = S.bkt; B.next_resize = S.next_resize;
                m.blk[b] = B;
                s_B = B;
                if (added) atomicAdd(&m.ctr[GM_MEMBERS], added);
            }
        }
        __syncthreads();
        if (s_rej) {
            const GBlock Bw = s_B;
            for (int i = tid; i < S.n; i += GM_INS_T) {
                m.ipool[Bw.ord + i] = s_ord[i];
                m.ipool[Bw.pos + i] = s_pos[i];
                m.ipool[Bw.mslot + i] = s_slot[i];
                m.cpool[Bw.code + i] = s_code[i];
            }
            for (int i = tid; i < S.bkt; i += GM_INS_T) {
                const unsigned short v = s_bk[i];
                m.ipool[Bw.bk + i] = v == (unsigned short)um::UM_EMPTY ? um::UM_EMPTY : (v == (unsigned short)um::UM_BB ? um::UM_BB : (int)v);
            }
        }
        // the segment is done: the small-image launch owns it (it decided from B.n before its own
        // insert), so the full-image launch that follows must not take it again after B.n has grown
        if (LN != GM_LDS_N && tid == 0) seg[3 * sg + 1] = 0;
        __syncthreads();
    }
}

template <int LN, int LBK>
__global__ void __launch_bounds__(GM_INS_T) k_gmap_insert(GMapDev m, const unsigned int* __restrict__ vals,
                                                          int* __restrict__ seg, int slot_base) {
    insert_wg<LN, LBK>(m, vals, seg, slot_base, blockIdx.x, gridDim.x);
}

template <int LN, int LBK>
__global__ void __launch_bounds__(GM_INS_T) k_gmap_insert_x(GMapJobs J, int k) {
    const GMapJob& jb = J.j[blockIdx.y];
    insert_wg<LN, LBK>(jb.m, jb.vals + k, jb.seg, jb.slot_base, blockIdx.x, gridDim.x);
}

// Map::getKeypoints: one thread per position of the x/y/z loop -> its block's entry count
__global__ void k_gmap_qcount(GMapDev m, int x0, int y0, int z0, int ny, int nz, int npos, int* __restrict__ cnt,
                              int* __restrict__ bidx) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npos) return;
    const int iz = t % nz, r = t / nz, iy = r % ny, ix = r / ny;
    const int prec = 10000;
    const int x = x0 + ix * prec, y = y0 + iy * prec, z = z0 + iz * prec;
    const int b = find_block(m, block_id_of((float)x, (float)y, (float)z));
    bidx[t] = b;
    cnt[t] = b >= 0 ? m.blk[b].n : 0;
}

// exclusive scan of cnt[0, npos) in one workgroup; total -> *tot. 256 threads: a one-workgroup
// kernel of the main stream needs a CU with that many free wave slots, and under the lookahead's
// load a 1024-thread workgroup (16 waves on one CU) waited for one to drain
#ifndef GM_SCAN_T
#define GM_SCAN_T 256
#endif
// tot: the total, written straight to the pinned host counters (no copy launch)
__global__ void __launch_bounds__(GM_SCAN_T) k_gmap_scan(const int* __restrict__ cnt, int npos, int* __restrict__ off,
                                                         int* __restrict__ tot) {
    __shared__ int part[GM_SCAN_T];
    const int t = threadIdx.x;
    const int per = (npos + GM_SCAN_T - 1) / GM_SCAN_T;
    const int a = t * per, e = min(npos, a + per);
    int s = 0;
    for (int i = a; i < e; ++i) s += cnt[i];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < GM_SCAN_T; d <<= 1) {
        const int v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = t > 0 ? part[t - 1] : 0;
    for (int i = a; i < e; ++i) { off[i] = run; run += cnt[i]; }
    if (t == GM_SCAN_T - 1) *tot = part[GM_SCAN_T - 1];
}

// one wave per loop position: the block's entries in iteration order (mode 1) or insertion order
// (mode 2) -> target positions (float3) and descriptors (11 words at dst_desc)
__global__ void __launch_bounds__(256) k_gmap_qfill(GMapDev m, const int* __restrict__ cnt, const int* __restrict__ bidx,
                                                    const int* __restrict__ off, int npos, int canonical,
                                                    float* __restrict__ dst_pos, unsigned int* __restrict__ dst_desc) {
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = lane_id();
    const int nw = (gridDim.x * blockDim.x) >> 6;
    for (int t = wave; t < npos; t += nw) {
        const int n = cnt[t];
        if (n == 0) continue;
        const GBlock B = m.blk[bidx[t]];
        const int o = off[t];
        for (int r = lane; r < n; r += 64) {
            const int mi = canonical ? r : m.ipool[B.ord + r];
            const int s = m.ipool[B.mslot + mi];
            const float4 p = m.kpos[s];
            dst_pos[3 * (size_t)(o + r)] = p.x;
            dst_pos[3 * (size_t)(o + r) + 1] = p.y;
            dst_pos[3 * (size_t)(o + r) + 2] = p.z;
#pragma unroll
            for (int w = 0; w < 11; ++w) dst_desc[11 * (size_t)(o + r) + w] = m.kdesc[11 * (size_t)s + w];
        }
    }
}

// the ref keypoints after the map's: transformPointCloud with the ref pose (src/lidar_odometry.cpp:202)
__global__ void k_gmap_ref(const float* __restrict__ kps, const unsigned int* __restrict__ bits, int k, Xf16g T,
                           float* __restrict__ dst_pos, unsigned int* __restrict__ dst_desc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    const float x = kps[3 * i], y = kps[3 * i + 1], z = kps[3 * i + 2];
    dst_pos[3 * i] = ((T.m[0] * x + T.m[1] * y) + T.m[2] * z) + T.m[3];
    dst_pos[3 * i + 1] = ((T.m[4] * x + T.m[5] * y) + T.m[6] * z) + T.m[7];
    dst_pos[3 * i + 2] = ((T.m[8] * x + T.m[9] * y) + T.m[10] * z) + T.m[11];
#pragma unroll
    for (int w = 0; w < 11; ++w) dst_desc[11 * (size_t)i + w] = bits[11 * (size_t)i + w];
}

}  // namespace bsk

namespace bsh {

#define HIPCHK(call, what)                              \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return c->fail(what, e_); \
    } while (0)

static bsk::GMapDev dev_view(GMap& g) {
    bsk::GMapDev v;
    v.kpos = g.kpos.p;
    v.kdesc = g.kdesc.p;
    v.tkey = g.tkey.p;
    v.tval = g.tval.p;
    v.tmask = g.tsize - 1;
    v.blk = g.blk.p;
    v.blk_cap = (int)g.blk_cap;
    v.ctr = g.ctr.p;
    v.ipool = g.ipool.p;
    v.ipool_cap = (long long)g.ipool_cap;
    v.cpool = g.cpool.p;
    v.cpool_cap = (long long)g.cpool_cap;
    return v;
}

static bsk::Xf16g xf(const float* T16) {
    bsk::Xf16g T;
    for (int i = 0; i < 16; ++i) T.m[i] = T16[i];
    return T;
}

// device copy (keeps contents) when a buffer must grow; the map's pools and tables carry state
template <typename T>
static hipError_t grow_keep(DBuf<T>& b, size_t used, size_t need, hipStream_t s) {
    if (need <= b.cap) return hipSuccess;
    size_t c = std::max(need, 2 * b.cap);
    T* p = nullptr;
    hipError_t e = hipMalloc(&p, sizeof(T) * c);
    if (e != hipSuccess) return e;
    note_regrow("gmap", sizeof(T) * c);
    if (used) {
        e = kcopy(p, b.p, sizeof(T) * used, s);
        if (e != hipSuccess) return e;
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
    }
    defer_free(b.p, DEFER_DEVICE);  // stream-ordered copy above; freed at context teardown
    b.p = p;
    b.cap = c;
    return hipSuccess;
}

// Up-front room for the map's keypoints (option gmap_slots0, default 2^20: 16 + 44 B each, 60 MB of
// the GPU's 288 GB) and for the matcher's target descriptors: a grow_keep inside the sweep loop
// costs a hipMalloc and a sync of the main stream, and a 20-sweep bench region held five of them as
// the map doubled from 2 Ki slots (BSHOT_GROW_TRACE, profiles/r06ze_grow.txt). Past the reservation
// the map still grows by doubling (test_gpu_map_modes_vs_oracle runs it from 64 slots).
#ifndef GM_TARGETS0
#define GM_TARGETS0 (1 << 18)
#endif
static int gmap_init(bshot_ctx* c, GMap& g, hipStream_t st = nullptr) {
    if (!st) st = c->stream;
    if (g.ready) return BSHOT_OK;
    const size_t s0 = (size_t)c->opt_gmap_slots0;
    HIPCHK(grow_keep(g.kpos, 0, s0, st), "gmap slots");
    HIPCHK(grow_keep(g.kdesc, 0, 11 * s0, st), "gmap slots");
    g.tsize = 1u << 16;
    HIPCHK(g.tkey.ensure(g.tsize), "gmap table");
    HIPCHK(g.tval.ensure(g.tsize), "gmap table");
    HIPCHK(kfill(g.tkey.p, 0xFF, sizeof(unsigned long long) * g.tsize, st), "gmap table clear");
    g.blk_cap = 1 << 14;
    HIPCHK(g.blk.ensure(g.blk_cap), "gmap blocks");
    g.ipool_cap = (size_t)1 << 24;
    g.cpool_cap = (size_t)1 << 22;
    HIPCHK(g.ipool.ensure(g.ipool_cap), "gmap pool");
    HIPCHK(g.cpool.ensure(g.cpool_cap), "gmap pool");
    g.ipool_cap = g.ipool.cap;
    g.cpool_cap = g.cpool.cap;
    HIPCHK(g.ctr.ensure(GM_NCTR), "gmap counters");
    HIPCHK(kfill(g.ctr.p, 0, sizeof(int) * GM_NCTR, st), "gmap counters");
    HIPCHK(g.p_ctr.ensure(GM_NCTR), "gmap pinned counters");
    std::memset(g.p_ctr.p, 0, sizeof(int) * GM_NCTR);
    g.slots = 0;
    g.ready = true;
    return BSHOT_OK;
}

static GMap& own_map(bshot_ctx* c) {
    if (!c->gmap) c->gmap = new GMap();
    return *c->gmap;
}

static GMap& replica_map(bshot_ctx* c, int r) {
    if ((int)c->gmap_replicas.size() <= r) c->gmap_replicas.resize(r + 1, nullptr);
    if (!c->gmap_replicas[r]) c->gmap_replicas[r] = new GMap();
    return *c->gmap_replicas[r];
}

// the counters' copy of an unsynchronised insert has landed, and that insert reported no error
// (a replica's capacity failure must not pass silently)
static int gmap_settle(bshot_ctx* c, GMap& g) {
    if (!g.ctr_pending) return BSHOT_OK;
    HIPCHK(hipEventSynchronize(g.ev_ctr), "sync map counters");
    g.ctr_pending = false;
    if (g.p_ctr.p[GM_ERR]) return c->fail("gpu map: capacity exceeded (block > 4096 members, or pool)", BSHOT_ECAP);
    return BSHOT_OK;
}

// room for one more batch of k keypoints (counters as of the map's last D2H, which gmap_settle or a
// later sync on the stream has completed): slots, blocks, table load <= 1/2, pools at most half full
// (a batch can at most double what its blocks hold)
static int gmap_reserve(bshot_ctx* c, GMap& g, int k, hipStream_t st = nullptr) {
    if (!st) st = c->stream;
    if (int rc = gmap_settle(c, g)) return rc;
    const int* h = g.p_ctr.p;
    HIPCHK(grow_keep(g.kpos, (size_t)g.slots, (size_t)g.slots + k + 1, st), "gmap slots");
    HIPCHK(grow_keep(g.kdesc, 11 * (size_t)g.slots, 11 * ((size_t)g.slots + k + 1), st), "gmap slots");
    const size_t nb = (size_t)h[GM_NBLOCKS];
    HIPCHK(grow_keep(g.blk, nb, nb + k + 1, st), "gmap blocks");
    g.blk_cap = g.blk.cap;
    if (2 * (nb + k) > g.tsize) {
        // rehash the block table on the host side of a sync: rebuilt from the headers
        HIPCHK(hipStreamSynchronize(st), "sync map table");
        unsigned int ts = g.tsize;
        while (2 * (nb + k) > ts) ts <<= 1;
        std::vector<GBlock> hb(nb);
        if (nb) HIPCHK(hipMemcpy(hb.data(), g.blk.p, sizeof(GBlock) * nb, hipMemcpyDeviceToHost), "gmap headers");
        std::vector<unsigned long long> key(ts, BS_EMPTY_KEY);
        std::vector<int> val(ts, -1);
        for (size_t b = 0; b < nb; ++b) {
            unsigned long long kk = hb[b].id;
            kk ^= kk >> 29;
            kk *= 0xBF58476D1CE4E5B9ull;
            kk ^= kk >> 32;
            unsigned int x = (unsigned int)kk & (ts - 1);
            while (key[x] != BS_EMPTY_KEY) x = (x + 1) & (ts - 1);
            key[x] = hb[b].id;
            val[x] = (int)b;
        }
        HIPCHK(g.tkey.ensure(ts), "gmap table");
        HIPCHK(g.tval.ensure(ts), "gmap table");
        HIPCHK(hipMemcpy(g.tkey.p, key.data(), sizeof(unsigned long long) * ts, hipMemcpyHostToDevice), "gmap table");
        HIPCHK(hipMemcpy(g.tval.p, val.data(), sizeof(int) * ts, hipMemcpyHostToDevice), "gmap table");
        g.tsize = ts;
    }
    const size_t itop = (size_t)(unsigned)h[GM_ITOP], ctop = (size_t)(unsigned)h[GM_CTOP];
    HIPCHK(grow_keep(g.ipool, itop, 2 * itop + 64 * (size_t)k + 4096, st), "gmap pool");
    HIPCHK(grow_keep(g.cpool, ctop, 2 * ctop + 16 * (size_t)k + 1024, st), "gmap pool");
    g.ipool_cap = g.ipool.cap;
    g.cpool_cap = g.cpool.cap;
    return BSHOT_OK;
}

// sort the batch's block ids (stable: sweep order inside a block), runs -> segments, insert waves;
// the counters go to the pinned copy (synchronously when sync)
static int gmap_run_insert(bshot_ctx* c, GMap& g, int k, bool sync, hipStream_t st = nullptr) {
    if (!st) st = c->stream;
    const int B = 256;
    if (k <= GM_SORT_MAX) {
        bsk::k_gmap_sort_segments<<<1, GM_SORT_T, 0, st>>>(g.keys.p, g.vals.p, k, dev_view(g), g.vals.p + k, g.seg.p);
    } else {
        size_t tb = 0;
        HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, g.keys.p, g.keys.p + k, g.vals.p, g.vals.p + k, (unsigned)k, 0, 64,
                                         st), "gmap sort size");
        HIPCHK(g.tmp.ensure(tb + 16), "gmap sort tmp");
        HIPCHK(rocprim::radix_sort_pairs(g.tmp.p, tb, g.keys.p, g.keys.p + k, g.vals.p, g.vals.p + k, (unsigned)k, 0, 64,
                                         st), "gmap sort");
        HIPCHK(kfill(g.ctr.p + GM_NSEG, 0, sizeof(int), st), "gmap seg count");
        bsk::k_gmap_segments<<<(k + B - 1) / B, B, 0, st>>>(g.keys.p + k, k, dev_view(g), g.seg.p);
    }
    // a workgroup holds a whole CU's LDS (the block image), and a batch touches a few hundred blocks
    // at most: more workgroups than that only occupy CUs to exit. Replica inserts (another stream,
    // off the critical chain) take fewer, leaving the CUs to the lookahead.
    const int wgs = std::min(k, st == c->stream ? 256 : 64);
    bsk::k_gmap_insert<GM_SMALL_N, GM_SMALL_BK><<<wgs, GM_INS_T, 0, st>>>(dev_view(g), g.vals.p + k, g.seg.p, g.slots);
    // blocks past GM_SMALL_N members are few: a handful of full-image workgroups (each needs a whole
    // CU's LDS to start) grid-stride over the segments
    bsk::k_gmap_insert<GM_LDS_N, GM_LDS_BK><<<std::min(k, 16), GM_INS_T, 0, st>>>(dev_view(g), g.vals.p + k, g.seg.p, g.slots);
    HIPCHK(hipGetLastError(), "gmap insert launch");
    g.slots += k;
    HIPCHK(kcopy(g.p_ctr.p, g.ctr.p, sizeof(int) * GM_QTOT, st), "D2H map counters");
    if (sync) {
        HIPCHK(hipStreamSynchronize(st), "sync map");
        g.ctr_pending = false;
        if (g.p_ctr.p[GM_ERR]) return c->fail("gpu map: capacity exceeded (block > 4096 members, or pool)", BSHOT_ECAP);
    } else {
        if (!g.ev_ctr) HIPCHK(hipEventCreateWithFlags(&g.ev_ctr, hipEventDisableTiming), "map event");
        HIPCHK(hipEventRecord(g.ev_ctr, st), "record map counters");
        g.ctr_pending = true;
    }
    return BSHOT_OK;
}

static int gmap_scratch(bshot_ctx* c, GMap& g, int k) {
    HIPCHK(g.keys.ensure(2 * (size_t)k), "gmap keys");
    HIPCHK(g.vals.ensure(2 * (size_t)k), "gmap vals");
    HIPCHK(g.seg.ensure(3 * (size_t)k), "gmap segments");
    return BSHOT_OK;
}

int gmap_insert(bshot_ctx* c, const float* kps_host, const float* ratio_host, const unsigned int* d_bits, int k,
                const float T[16], int* map_size) {
    GMap& g = own_map(c);
    int rc = gmap_init(c, g);
    if (rc) return rc;
    g.last_k = k;
    if (k > 0) {
        if ((rc = gmap_reserve(c, g, k)) || (rc = gmap_scratch(c, g, k))) return rc;
        HIPCHK(g.kin.ensure(4 * (size_t)k), "gmap in");
        HIPCHK(g.p_kin.ensure(4 * (size_t)k), "gmap pinned in");
        std::memcpy(g.p_kin.p, kps_host, sizeof(float) * 3 * k);
        std::memcpy(g.p_kin.p + 3 * (size_t)k, ratio_host, sizeof(float) * k);
        HIPCHK(kcopy(g.kin.p, g.p_kin.p, sizeof(float) * 4 * k, c->stream), "H2D map in");
        bsk::k_gmap_prep<<<(k + 255) / 256, 256, 0, c->stream>>>(g.kin.p, g.kin.p + 3 * (size_t)k, d_bits, k, xf(T),
                                                                 g.slots, dev_view(g), g.keys.p, g.vals.p);
        // option map_sync 0: no host wait for the insert here -- the next map query is stream-ordered
        // behind it and settles its counters (capacity errors surface there); the size is not read back
        if ((rc = gmap_run_insert(c, g, k, c->opt_map_sync != 0))) return rc;
    } else if (c->opt_map_sync) {
        HIPCHK(kcopy(g.p_ctr.p, g.ctr.p, sizeof(int) * GM_QTOT, c->stream), "D2H map counters");
        HIPCHK(hipStreamSynchronize(c->stream), "sync map");
    }
    *map_size = c->opt_map_sync ? g.p_ctr.p[GM_MEMBERS] : -1;
    return BSHOT_OK;
}

int gmap_pack_delta(bshot_ctx* c, int kmax, float* d_rec) {
    GMap& g = own_map(c);
    int rc = gmap_init(c, g);
    if (rc) return rc;
    if (g.last_k > kmax)
        return c->fail("map exchange: the sweep offered " + std::to_string(g.last_k) + " keypoints, more than the "
                       "exchange's kmax " + std::to_string(kmax), BSHOT_EINVAL);
    const int k = g.last_k;
    bsk::k_gmap_pack<<<(std::max(k, 1) + 255) / 256, 256, 0, c->stream>>>(dev_view(g), g.slots - g.last_k, k, kmax, d_rec);
    HIPCHK(hipGetLastError(), "gmap pack launch");
    return BSHOT_OK;
}

int gmap_insert_records(bshot_ctx* c, int replica, const float* d_rec, int kmax, bool sync, hipStream_t st) {
    if (!st) st = c->stream;
    GMap& g = replica_map(c, replica);
    int rc = gmap_init(c, g, st);
    if (rc) return rc;
    if (kmax <= 0) return BSHOT_OK;
    if ((rc = gmap_reserve(c, g, kmax, st)) || (rc = gmap_scratch(c, g, kmax))) return rc;
    bsk::k_gmap_prep_rec<<<(kmax + 255) / 256, 256, 0, st>>>(d_rec, kmax, g.slots, dev_view(g), g.keys.p, g.vals.p);
    return gmap_run_insert(c, g, kmax, sync, st);
}

int gmap_insert_records_multi(bshot_ctx* c, int n, const int* replicas, const float* const* d_recs, int kmax,
                              hipStream_t st) {
    if (!st) st = c->stream;
    if (n <= 0) return BSHOT_OK;
    for (int a = 0; a < n; ++a)
        for (int b = a + 1; b < n; ++b)
            if (replicas[a] == replicas[b]) return c->fail("gmap_insert_records_multi: replica listed twice", BSHOT_EINVAL);
    if (kmax > GM_SORT_MAX || n > GM_XB) {
        // large batches: the per-replica path (radix sort), in order
        for (int a = 0; a < n; ++a)
            if (int rc = gmap_insert_records(c, replicas[a], d_recs[a], kmax, false, st)) return rc;
        return BSHOT_OK;
    }
    bsk::GMapJobs J;
    std::memset(&J, 0, sizeof(J));
    for (int a = 0; a < n; ++a) {
        GMap& g = replica_map(c, replicas[a]);
        int rc = gmap_init(c, g, st);
        if (rc) return rc;
        if (kmax <= 0) continue;
        if ((rc = gmap_reserve(c, g, kmax, st)) || (rc = gmap_scratch(c, g, kmax))) return rc;
        bsk::GMapJob& jb = J.j[a];
        jb.m = dev_view(g);
        jb.rec = d_recs[a];
        jb.keys = g.keys.p;
        jb.vals = g.vals.p;
        jb.seg = g.seg.p;
        jb.p_ctr = g.p_ctr.p;
        jb.slot_base = g.slots;
    }
    if (kmax <= 0) return BSHOT_OK;
    bsk::k_gmap_prep_rec_x<<<dim3((kmax + 255) / 256, n), 256, 0, st>>>(J, kmax);
    bsk::k_gmap_sort_segments_x<<<n, GM_SORT_T, 0, st>>>(J, kmax);
    // as gmap_run_insert's replica launches, per replica
    bsk::k_gmap_insert_x<GM_SMALL_N, GM_SMALL_BK><<<dim3(std::min(kmax, 64), n), GM_INS_T, 0, st>>>(J, kmax);
    bsk::k_gmap_insert_x<GM_LDS_N, GM_LDS_BK><<<dim3(std::min(kmax, 16), n), GM_INS_T, 0, st>>>(J, kmax);
    bsk::k_gmap_ctr_x<<<n, 64, 0, st>>>(J);
    HIPCHK(hipGetLastError(), "gmap batched insert launch");
    for (int a = 0; a < n; ++a) {
        GMap& g = *c->gmap_replicas[replicas[a]];
        g.slots += kmax;
        if (!g.ev_ctr) HIPCHK(hipEventCreateWithFlags(&g.ev_ctr, hipEventDisableTiming), "map event");
        HIPCHK(hipEventRecord(g.ev_ctr, st), "record map counters");
        g.ctr_pending = true;
    }
    return BSHOT_OK;
}

int gmap_insert_host_records(bshot_ctx* c, int replica, const float* rec, int n) {
    if (int rc = c->quiesce_replicas()) return rc;
    // host records (bshot_odom_map_delta layout: x, y, z, ratio, 11 words) -> a device batch
    GMap& g = replica_map(c, replica);
    int rc = gmap_init(c, g);
    if (rc) return rc;
    const size_t per = GM_REC_HDR + (size_t)GM_REC_W * (n > 0 ? n : 1);
    HIPCHK(g.hrec.ensure(per), "alloc replica batch");
    HIPCHK(g.p_hrec.ensure(per), "alloc pinned replica batch");
    std::memset(g.p_hrec.p, 0, sizeof(float) * GM_REC_HDR);
    std::memcpy(g.p_hrec.p, &n, sizeof(int));
    if (n > 0) std::memcpy(g.p_hrec.p + GM_REC_HDR, rec, sizeof(float) * GM_REC_W * n);
    HIPCHK(kcopy(g.hrec.p, g.p_hrec.p, sizeof(float) * per, c->stream), "H2D batch");
    return gmap_insert_records(c, replica, g.hrec.p, n, true);
}

int gmap_settle_replicas_noquiesce(bshot_ctx* c) {
    for (GMap* g : c->gmap_replicas)
        if (g)
            if (int rc = gmap_settle(c, *g)) return rc;
    return BSHOT_OK;
}

int gmap_settle_replicas(bshot_ctx* c) {
    if (int rc = c->quiesce_replicas()) return rc;
    return gmap_settle_replicas_noquiesce(c);
}

int gmap_replica_size(bshot_ctx* c, int replica) {
    if (c->quiesce_replicas()) return -1;
    if (replica < 0 || replica >= (int)c->gmap_replicas.size() || !c->gmap_replicas[replica]) return 0;
    GMap& g = *c->gmap_replicas[replica];
    // its inserts may run on another stream (the exchange's): wait for the counters' copy itself
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -1;
    if (g.ctr_pending && hipEventSynchronize(g.ev_ctr) != hipSuccess) return -1;
    g.ctr_pending = false;
    if (g.p_ctr.p[GM_ERR]) return -2;
    return g.p_ctr.p[GM_MEMBERS];
}

// the 21^3 block loop over one map: counts + scan (async; the total lands in the pinned GM_QTOT slot)
static int query_count(bshot_ctx* c, GMap& g, const QueryBox& q) {
    // (an insert whose counters are still in flight may have made the map non-empty: query it)
    if (q.npos <= 0 || (!g.ctr_pending && g.p_ctr.p[GM_NBLOCKS] <= 0)) {
        g.p_ctr.p[GM_QTOT] = 0;
        g.q_active = false;
        return BSHOT_OK;
    }
    HIPCHK(g.qcnt.ensure((size_t)3 * q.npos + 1), "gmap query");
    int* cnt = g.qcnt.p;
    bsk::k_gmap_qcount<<<(q.npos + 255) / 256, 256, 0, c->stream>>>(dev_view(g), q.x0, q.y0, q.z0, q.ny, q.nz, q.npos, cnt,
                                                                    cnt + q.npos);
    bsk::k_gmap_scan<<<1, GM_SCAN_T, 0, c->stream>>>(cnt, q.npos, cnt + 2 * q.npos, g.p_ctr.p + GM_QTOT);
    HIPCHK(hipGetLastError(), "gmap query scan");
    g.q_active = true;
    return BSHOT_OK;
}

static QueryBox query_box(const float pos[3], float range) {
    const int prec = 10000;
    // the reference's loop bounds (src/mymap.cpp:30-36), as Map::getKeypoints computes them
    QueryBox q;
    q.x0 = (int)std::round((pos[0] - range) / (float)prec) * prec;
    const int x_max = (int)std::round((pos[0] + range) / (float)prec) * prec;
    q.y0 = (int)std::round((pos[1] - range) / (float)prec) * prec;
    const int y_max = (int)std::round((pos[1] + range) / (float)prec) * prec;
    q.z0 = (int)std::round((pos[2] - range) / (float)prec) * prec;
    const int z_max = (int)std::round((pos[2] + range) / (float)prec) * prec;
    q.npos = 0;
    q.ny = q.nz = 0;
    if (x_max >= q.x0 && y_max >= q.y0 && z_max >= q.z0) {
        const int nx = (x_max - q.x0) / prec + 1;
        q.ny = (y_max - q.y0) / prec + 1;
        q.nz = (z_max - q.z0) / prec + 1;
        q.npos = nx * q.ny * q.nz;
    }
    return q;
}

// stage the reference keypoints (positions + descriptors) in g.p_refin; the caller uploads them to
// g.refin (gmap_match: in one launch with its descriptors)
static int stage_ref(GMap& g, const float* ref_kps, const unsigned int* ref_bits, int kref) {
    if (kref <= 0) return BSHOT_OK;
    if (g.refin.ensure(14 * (size_t)kref) != hipSuccess || g.p_refin.ensure(14 * (size_t)kref) != hipSuccess)
        return BSHOT_EHIP;
    std::memcpy(g.p_refin.p, ref_kps, sizeof(float) * 3 * kref);
    std::memcpy(g.p_refin.p + 3 * (size_t)kref, ref_bits, sizeof(unsigned int) * 11 * kref);
    return BSHOT_OK;
}

int gmap_query(bshot_ctx* c, const float pos[3], float range, const float* ref_kps, const unsigned int* ref_bits,
               int kref, const float ref_pose[16], int na, int canonical, int* nb_out, bool ref_uploaded) {
    GMap& g = own_map(c);
    int rc = gmap_init(c, g);
    if (rc) return rc;
    const QueryBox q = query_box(pos, range);
    // the maps whose entries become targets: this sequence's, then (option xseq_targets, an
    // extension for cross-sequence matching; off reproduces the reference) the replicas in rank order
    std::vector<GMap*> maps{&g};
    if (c->opt_xseq_targets) {
        if ((rc = gmap_settle_replicas(c))) return rc;  // a replica that failed an insert is not matched against
        for (GMap* r : c->gmap_replicas)
            if (r && r->ready) maps.push_back(r);
    }
    bool any = false;
    for (GMap* m : maps) {
        if ((rc = query_count(c, *m, q))) return rc;
        any = any || m->q_active;
    }
    if (any) {
        HIPCHK(hipStreamSynchronize(c->stream), "sync map query");
        // the stream sync covers this map's last unsynchronised insert (option map_sync 0): its
        // counters have landed; an insert that ran out of capacity fails the sweep here
        if ((rc = gmap_settle(c, g))) return rc;
    }
    c->hmark("M_q_synced");
    int mtot = 0;
    for (GMap* m : maps) mtot += m->q_active ? m->p_ctr.p[GM_QTOT] : 0;
    const int nb = mtot + kref;
    // targets: positions in c->gtgt (float3), descriptors in c->ma after the na source rows
    HIPCHK(c->gtgt.ensure(3 * (size_t)(nb > 0 ? nb : 1)), "alloc targets");
    // at least GM_TARGETS0 rows from the first sweep on (the targets grow with the map)
    const size_t ma_need = 11 * std::max((size_t)na + nb, (size_t)GM_TARGETS0);
    if (c->ma.cap < ma_need) {
        // keep the source rows already staged at the front
        HIPCHK(grow_keep(c->ma, 11 * (size_t)na, ma_need, c->stream), "alloc descriptors");
    }
    int base = 0;
    for (GMap* m : maps) {
        if (!m->q_active) continue;
        const int mm = m->p_ctr.p[GM_QTOT];
        if (mm > 0) {
            int* cnt = m->qcnt.p;
            bsk::k_gmap_qfill<<<std::min((q.npos + 3) / 4, 2048), 256, 0, c->stream>>>(
                dev_view(*m), cnt, cnt + q.npos, cnt + 2 * q.npos, q.npos, canonical, c->gtgt.p + 3 * (size_t)base,
                c->ma.p + 11 * ((size_t)na + base));
        }
        base += mm;
    }
    if (kref > 0) {
        if (!ref_uploaded) {
            if ((rc = stage_ref(g, ref_kps, ref_bits, kref))) return c->fail("gmap ref alloc", rc);
            HIPCHK(kcopy(g.refin.p, g.p_refin.p, sizeof(float) * 14 * kref, c->stream), "H2D ref");
        }
        bsk::k_gmap_ref<<<(kref + 255) / 256, 256, 0, c->stream>>>(
            g.refin.p, reinterpret_cast<const unsigned int*>(g.refin.p + 3 * (size_t)kref), kref, xf(ref_pose),
            c->gtgt.p + 3 * (size_t)mtot, c->ma.p + 11 * ((size_t)na + mtot));
    }
    HIPCHK(hipGetLastError(), "gmap query launch");
    *nb_out = nb;
    return BSHOT_OK;
}

int gmap_replica_query(bshot_ctx* c, int replica, const float pos[3], float range, int canonical, float* xyz,
                       unsigned int* bits, int cap) {
    if (int rc = c->quiesce_replicas()) return rc;
    if (replica < 0 || replica >= (int)c->gmap_replicas.size() || !c->gmap_replicas[replica]) return 0;
    GMap& g = *c->gmap_replicas[replica];
    const QueryBox q = query_box(pos, range);
    HIPCHK(hipStreamSynchronize(c->stream), "sync replica");
    if (int rc = gmap_settle(c, g)) return rc;  // inserts on the exchange's stream have landed
    int rc = query_count(c, g, q);
    if (rc) return rc;
    if (!g.q_active) return 0;
    HIPCHK(hipStreamSynchronize(c->stream), "sync replica query");
    const int m = g.p_ctr.p[GM_QTOT];
    if (m > cap) return -m;
    if (m == 0) return 0;
    DBuf<float> pos3;
    DBuf<unsigned int> desc;
    HIPCHK(pos3.ensure(3 * (size_t)m), "alloc replica query");
    HIPCHK(desc.ensure(11 * (size_t)m), "alloc replica query");
    int* cnt = g.qcnt.p;
    bsk::k_gmap_qfill<<<std::min((q.npos + 3) / 4, 2048), 256, 0, c->stream>>>(dev_view(g), cnt, cnt + q.npos,
                                                                               cnt + 2 * q.npos, q.npos, canonical,
                                                                               pos3.p, desc.p);
    HIPCHK(hipMemcpyAsync(xyz, pos3.p, sizeof(float) * 3 * m, hipMemcpyDeviceToHost, c->stream), "D2H replica");
    HIPCHK(hipMemcpyAsync(bits, desc.p, sizeof(unsigned int) * 11 * m, hipMemcpyDeviceToHost, c->stream), "D2H replica");
    HIPCHK(hipStreamSynchronize(c->stream), "sync replica");
    pos3.release();
    desc.release();
    return m;
}

int gmap_match(bshot_ctx* c, const unsigned int* a, int na, const float pos[3], float range, const float* ref_kps,
               const unsigned int* ref_bits, int kref, const float ref_pose[16], int canonical, int* nb_out,
               std::vector<float>& tgt, int32_t* left_nn, std::vector<int32_t>& right_nn, int32_t* corr_q,
               int32_t* corr_m, int* n_corr) {
    *n_corr = 0;
    HIPCHK(grow_keep(c->ma, 0, 11 * std::max((size_t)(na > 0 ? na : 1), (size_t)GM_TARGETS0), c->stream),
           "alloc descriptors");
    GMap& g0 = own_map(c);
    int rc = gmap_init(c, g0);
    if (rc) return rc;
    if ((rc = stage_ref(g0, ref_kps, ref_bits, kref))) return c->fail("gmap ref alloc", rc);
    if (na > 0) {
        HIPCHK(c->p_a.ensure(11 * (size_t)na), "alloc pinned descriptors");
        std::memcpy(c->p_a.p, a, sizeof(uint32_t) * 11 * na);
    }
    // the descriptors and the reference keypoints in one launch
    HIPCHK(kcopy2(c->ma.p, c->p_a.p, sizeof(uint32_t) * 11 * (size_t)(na > 0 ? na : 0), g0.refin.p, g0.p_refin.p,
                  sizeof(float) * 14 * (size_t)(kref > 0 ? kref : 0), c->stream),
           "H2D descriptors + ref");
    int nb = 0;
    rc = gmap_query(c, pos, range, ref_kps, ref_bits, kref, ref_pose, na, canonical, &nb, true);
    if (rc) return rc;
    *nb_out = nb;
    tgt.resize(3 * (size_t)nb);
    right_nn.assign(nb > 0 ? nb : 1, 0);
    // its own pinned staging: the context's gather buffer (p_g3) belongs to the lookahead worker's
    // ISS gather, which runs concurrently
    GMap& g = *c->gmap;
    HIPCHK(g.p_tgt.ensure(3 * (size_t)(nb > 0 ? nb : 1)), "alloc pinned targets");
    const bool run = na > 0 && nb > 0;
    if (run) {
        HIPCHK(c->p_left.ensure(2 * (size_t)na + nb), "alloc pinned match out");
        rc = ctx_match_dev(c, na, nb);
        if (rc) return rc;
    }
    // the targets' positions and the match result in one launch
    HIPCHK(kcopy2(g.p_tgt.p, c->gtgt.p, sizeof(float) * 3 * (size_t)(nb > 0 ? nb : 0), c->p_left.p, c->left.p,
                  run ? sizeof(int) * (2 * (size_t)na + nb) : 0, c->stream),
           "D2H targets + match");
    c->hmark("M_m_launched");
    HIPCHK(hipStreamSynchronize(c->stream), "sync match");
    c->hmark("M_m_synced");
    c->resolve_events();
    if (nb > 0) std::memcpy(tgt.data(), g.p_tgt.p, sizeof(float) * 3 * nb);
    if (!run) return BSHOT_OK;
    std::memcpy(left_nn, c->p_left.p, sizeof(int) * na);
    std::memcpy(right_nn.data(), c->p_left.p + na, sizeof(int) * nb);
    const int* flag = c->p_left.p + na + nb;
    int m = 0;
    for (int i = 0; i < na; ++i)
        if (flag[i]) { corr_q[m] = i; corr_m[m] = left_nn[i]; ++m; }
    *n_corr = m;
    return BSHOT_OK;
}

int gmap_target_descriptors(bshot_ctx* c, int na, int nb, unsigned int* out) {
    if (nb > 0)
        HIPCHK(hipMemcpy(out, c->ma.p + 11 * (size_t)na, sizeof(unsigned int) * 11 * nb, hipMemcpyDeviceToHost),
               "D2H target descriptors");
    return BSHOT_OK;
}

void gmap_free(bshot_ctx* c) {
    delete c->gmap;
    c->gmap = nullptr;
    for (GMap* r : c->gmap_replicas) delete r;
    c->gmap_replicas.clear();
}

}  // namespace bsh
