// kcopy.hip -- copies and fills issued as kernels on the caller's stream.
//
// Every per-sweep transfer of the odometry loop is device<->device or between device memory and
// the context's pinned staging buffers (hipHostMalloc: mapped into the GPU's address space), so a
// kernel can move it with plain vector loads and stores. Doing so keeps the sweep loop off the
// copy engines: with SDMA copies in the loop, about half of the 20-sweep runs carried one 6-18 ms
// GPU-wide stall, gone whenever no copy engine was used (profiles/r02h_stalls.txt).
// Kernel completion orders the data as a copy would: a stream wait, an event or a later kernel on
// the same stream sees it, and host memory written here is visible to the host once it has
// synchronised with the stream.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.h"

namespace bsk {

#define KC_THREADS 256
#define KC_MAX_BLOCKS 1024

// dst/src 16-B aligned: uint4 body; the tail (bytes % 16) byte by byte
__global__ void __launch_bounds__(KC_THREADS) k_copy16(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n16,
                                                       unsigned char* __restrict__ dtail,
                                                       const unsigned char* __restrict__ stail, int ntail) {
    const size_t stride = (size_t)gridDim.x * KC_THREADS;
    for (size_t i = (size_t)blockIdx.x * KC_THREADS + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < ntail) dtail[threadIdx.x] = stail[threadIdx.x];
}

__global__ void __launch_bounds__(KC_THREADS) k_copy4(unsigned int* __restrict__ dst, const unsigned int* __restrict__ src,
                                                      size_t n4, unsigned char* __restrict__ dtail,
                                                      const unsigned char* __restrict__ stail, int ntail) {
    const size_t stride = (size_t)gridDim.x * KC_THREADS;
    for (size_t i = (size_t)blockIdx.x * KC_THREADS + threadIdx.x; i < n4; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < ntail) dtail[threadIdx.x] = stail[threadIdx.x];
}

__global__ void __launch_bounds__(KC_THREADS) k_copy1(unsigned char* __restrict__ dst, const unsigned char* __restrict__ src,
                                                      size_t n) {
    const size_t stride = (size_t)gridDim.x * KC_THREADS;
    for (size_t i = (size_t)blockIdx.x * KC_THREADS + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

__global__ void __launch_bounds__(KC_THREADS) k_fill16(uint4* __restrict__ dst, uint4 v, size_t n16,
                                                       unsigned char* __restrict__ dtail, unsigned char b, int ntail) {
    const size_t stride = (size_t)gridDim.x * KC_THREADS;
    for (size_t i = (size_t)blockIdx.x * KC_THREADS + threadIdx.x; i < n16; i += stride) dst[i] = v;
    if (blockIdx.x == 0 && (int)threadIdx.x < ntail) dtail[threadIdx.x] = b;
}

__global__ void __launch_bounds__(KC_THREADS) k_fill1(unsigned char* __restrict__ dst, unsigned char b, size_t n) {
    const size_t stride = (size_t)gridDim.x * KC_THREADS;
    for (size_t i = (size_t)blockIdx.x * KC_THREADS + threadIdx.x; i < n; i += stride) dst[i] = b;
}

// up to KC_JOBS copies in one launch (blockIdx.y = the copy), each with its own alignment path
#define KC_JOBS 4
struct CopyJob {
    unsigned char* d;
    const unsigned char* s;
    size_t bytes;
    int align;  // 16, 4 or 1: the widest unit both pointers are aligned to
};
struct CopyJobs {
    CopyJob j[KC_JOBS];
};

__global__ void __launch_bounds__(KC_THREADS) k_copy_multi(CopyJobs J) {
    const CopyJob& jb = J.j[blockIdx.y];
    const size_t stride = (size_t)gridDim.x * KC_THREADS;
    const size_t t0 = (size_t)blockIdx.x * KC_THREADS + threadIdx.x;
    size_t body = 0;
    if (jb.align == 16) {
        const size_t n = jb.bytes / 16;
        for (size_t i = t0; i < n; i += stride) reinterpret_cast<uint4*>(jb.d)[i] = reinterpret_cast<const uint4*>(jb.s)[i];
        body = 16 * n;
    } else if (jb.align == 4) {
        const size_t n = jb.bytes / 4;
        for (size_t i = t0; i < n; i += stride)
            reinterpret_cast<unsigned int*>(jb.d)[i] = reinterpret_cast<const unsigned int*>(jb.s)[i];
        body = 4 * n;
    }
    for (size_t i = body + t0; i < jb.bytes; i += stride) jb.d[i] = jb.s[i];
}

}  // namespace bsk

namespace bsh {

static inline int kc_blocks(size_t units, int cap = KC_MAX_BLOCKS) {
    const size_t b = (units + KC_THREADS - 1) / KC_THREADS;
    return (int)(b < 1 ? 1 : (b > (size_t)cap ? (size_t)cap : b));
}

hipError_t kcopy(void* dst, const void* src, size_t bytes, hipStream_t s, int max_blocks) {
    if (max_blocks < 1) max_blocks = KC_MAX_BLOCKS;
    if (bytes == 0 || dst == src) return hipSuccess;
    if (!dst || !src) return hipErrorInvalidValue;
    const uintptr_t a = (uintptr_t)dst | (uintptr_t)src;
    unsigned char* d = static_cast<unsigned char*>(dst);
    const unsigned char* p = static_cast<const unsigned char*>(src);
    if ((a & 15) == 0) {
        const size_t n16 = bytes / 16;
        const int tail = (int)(bytes % 16);
        bsk::k_copy16<<<kc_blocks(n16, max_blocks), KC_THREADS, 0, s>>>(reinterpret_cast<uint4*>(d), reinterpret_cast<const uint4*>(p),
                                                            n16, d + 16 * n16, p + 16 * n16, tail);
    } else if ((a & 3) == 0) {
        const size_t n4 = bytes / 4;
        const int tail = (int)(bytes % 4);
        bsk::k_copy4<<<kc_blocks(n4, max_blocks), KC_THREADS, 0, s>>>(reinterpret_cast<unsigned int*>(d),
                                                          reinterpret_cast<const unsigned int*>(p), n4, d + 4 * n4,
                                                          p + 4 * n4, tail);
    } else {
        bsk::k_copy1<<<kc_blocks(bytes, max_blocks), KC_THREADS, 0, s>>>(d, p, bytes);
    }
    return hipGetLastError();
}

hipError_t kcopy_n(int n, void* const* dst, const void* const* src, const size_t* bytes, hipStream_t s) {
    bsk::CopyJobs J;
    int m = 0;
    size_t units = 0;
    for (int i = 0; i < n; ++i) {
        if (bytes[i] == 0 || dst[i] == src[i]) continue;
        if (!dst[i] || !src[i]) return hipErrorInvalidValue;
        if (m == KC_JOBS) {  // more copies than one launch takes: the rest in further launches
            if (hipError_t e = kcopy_n(n - i, dst + i, src + i, bytes + i, s)) return e;
            break;
        }
        const uintptr_t a = (uintptr_t)dst[i] | (uintptr_t)src[i];
        bsk::CopyJob& jb = J.j[m++];
        jb.d = static_cast<unsigned char*>(dst[i]);
        jb.s = static_cast<const unsigned char*>(src[i]);
        jb.bytes = bytes[i];
        jb.align = (a & 15) == 0 ? 16 : ((a & 3) == 0 ? 4 : 1);
        units = std::max(units, bytes[i] / (size_t)jb.align);
    }
    if (m == 0) return hipSuccess;
    if (m == 1) return kcopy(J.j[0].d, J.j[0].s, J.j[0].bytes, s);
    bsk::k_copy_multi<<<dim3(kc_blocks(units), m), KC_THREADS, 0, s>>>(J);
    return hipGetLastError();
}

hipError_t kcopy2(void* d0, const void* s0, size_t b0, void* d1, const void* s1, size_t b1, hipStream_t s) {
    void* d[2] = {d0, d1};
    const void* src[2] = {s0, s1};
    const size_t b[2] = {b0, b1};
    return kcopy_n(2, d, src, b, s);
}

hipError_t kfill(void* dst, unsigned char value, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    if (!dst) return hipErrorInvalidValue;
    unsigned char* d = static_cast<unsigned char*>(dst);
    if (((uintptr_t)dst & 15) == 0) {
        const unsigned int w = 0x01010101u * value;
        const size_t n16 = bytes / 16;
        bsk::k_fill16<<<kc_blocks(n16), KC_THREADS, 0, s>>>(reinterpret_cast<uint4*>(d), make_uint4(w, w, w, w), n16,
                                                            d + 16 * n16, value, (int)(bytes % 16));
    } else {
        bsk::k_fill1<<<kc_blocks(bytes), KC_THREADS, 0, s>>>(d, value, bytes);
    }
    return hipGetLastError();
}

}  // namespace bsh
