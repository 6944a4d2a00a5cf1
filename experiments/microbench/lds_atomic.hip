// Microbenchmark: cost of in-order LDS float atomics issued by a few lanes of one wave
// (the ordered SHOT histogram accumulation pattern). Prints cycles per ds_add instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// mode 0: ds_add_f32 (atomicAdd, no return) by lanes 0..4, bins from a table
// mode 1: plain ds_read + add + ds_write by lanes 0..4 (dependent RMW chain)
// mode 2: ds_add_f32 by all 64 lanes to distinct bins
// mode 3: ds_add_f32 by lanes 0..2 only
// mode 4: lanes 0..4, each add exec-masked off when its bin is = 0 mod 8 or odd (about 56% kept)
// mode 5: as 4, the exec mask set around each ds_add_f32 in inline asm (no branch)
// mode 6: ds_add_u32 (integer atomic) by all 64 lanes to distinct bins
// mode 7: ds_add_u32 by all 64 lanes to random bins of 192 (SR histogram pattern)
template <int MODE>
__global__ void k(const int* __restrict__ bins, int nops, unsigned long long* out, float* sink) {
    __shared__ float hist[384];
    __shared__ unsigned int ihist[384];
    __shared__ int bt[1024 * 5];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 384; i += blockDim.x) { hist[i] = 0.f; ihist[i] = 0u; }
    for (int i = threadIdx.x; i < 1024 * 5; i += blockDim.x) bt[i] = bins[i];
    __syncthreads();
    const unsigned long long t0 = stamp();
    if (MODE == 6 || MODE == 7) {
        for (int r0 = 0; r0 < nops; r0 += 16) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int b = MODE == 6 ? ((lane * 5 + u) % 352) : bt[((r0 + u) % 1024) * 5 + (lane % 5)] % 192 + (lane & 7) * 0;
                atomicAdd(&ihist[MODE == 7 ? (b + lane * 7) % 192 : b], 1u);
            }
        }
    } else if (MODE == 2 || lane < (MODE == 3 ? 3 : 5)) {
        for (int r0 = 0; r0 < nops; r0 += 16) {
            int bb[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) bb[u] = MODE == 2 ? ((lane * 5 + u) % 352) : bt[((r0 + u) % 1024) * 5 + lane];
            if (MODE == 1) {
#pragma unroll
                for (int u = 0; u < 16; ++u) hist[bb[u]] = hist[bb[u]] + 0.5f;
            } else if (MODE == 5) {
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const unsigned int keep = ((bb[u] & 1) == 0 && (bb[u] & 7) != 0) ? 1u : 0u;
                    const unsigned int addr = (unsigned int)(size_t)&hist[bb[u]];
                    asm volatile(
                        "s_mov_b64 s[40:41], exec\n\t"
                        "v_cmp_ne_u32 vcc, 0, %0\n\t"
                        "s_and_b64 exec, exec, vcc\n\t"
                        "ds_add_f32 %1, %2\n\t"
                        "s_mov_b64 exec, s[40:41]"
                        :
                        : "v"(keep), "v"(addr), "v"(0.5f)
                        : "s40", "s41", "vcc", "memory");
                }
            } else if (MODE == 4) {
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if ((bb[u] & 1) == 0 && (bb[u] & 7) != 0) atomicAdd(&hist[bb[u]], 0.5f);
            } else {
#pragma unroll
                for (int u = 0; u < 16; ++u) atomicAdd(&hist[bb[u]], 0.5f);
            }
        }
    }
    __syncthreads();
    const unsigned long long t1 = stamp();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (threadIdx.x < 352) sink[blockIdx.x * 352 + threadIdx.x] = hist[threadIdx.x] + (float)ihist[threadIdx.x];
}

int main() {
    const int nops = 4096;
    std::vector<int> hb(1024 * 5);
    unsigned s = 12345;
    for (auto& b : hb) { s = s * 1664525u + 1013904223u; b = (s >> 8) % 352; }
    int* db; unsigned long long* dout; float* sink;
    // out / sink hold one slot per block of the largest launch below (16384 blocks)
    const int max_blocks = 16384;
    hipMalloc(&db, hb.size() * 4); hipMalloc(&dout, 8 * (size_t)max_blocks); hipMalloc(&sink, (size_t)max_blocks * 352 * 4);
    hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
    auto run = [&](auto kern, const char* name, int blocks, int threads) {
        if (blocks > max_blocks) { printf("%s: %d blocks > %d slots, skipped\n", name, blocks, max_blocks); return; }
        kern<<<blocks, threads>>>(db, nops, dout, sink);
        hipDeviceSynchronize();
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipEventRecord(a);
        kern<<<blocks, threads>>>(db, nops, dout, sink);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        std::vector<unsigned long long> h(blocks);
        hipMemcpy(h.data(), dout, 8 * blocks, hipMemcpyDeviceToHost);
        double avg = 0; for (auto v : h) avg += v; avg /= blocks;
        printf("%-34s blocks %5d x %4d thr: %.3f ms, %.1f ticks/op per wave (avg block %.0f ticks)\n", name, blocks,
               threads, ms, avg / nops, avg);
    };
    run(k<0>, "ds_add lanes0-4, 1 wave/block", 1, 64);
    run(k<1>, "rmw lanes0-4, 1 wave/block", 1, 64);
    run(k<2>, "ds_add 64 lanes, 1 wave/block", 1, 64);
    run(k<6>, "ds_add_u32 64 lanes distinct, 1 wave", 1, 64);
    run(k<7>, "ds_add_u32 64 lanes random/192, 1 wave", 1, 64);
    run(k<2>, "ds_add_f32 64 lanes distinct, 8 waves, 256 blk", 256, 512);
    run(k<6>, "ds_add_u32 64 lanes distinct, 8 waves, 256 blk", 256, 512);
    run(k<7>, "ds_add_u32 64 lanes random/192, 8 waves, 256 blk", 256, 512);
    run(k<3>, "ds_add lanes0-2, 1 wave/block", 1, 64);
    run(k<4>, "ds_add lanes0-4 masked ~40%, 1 wave", 1, 64);
    run(k<5>, "ds_add lanes0-4 asm-masked, 1 wave", 1, 64);
    run(k<0>, "ds_add lanes0-4, 8 waves, 256 blk", 256, 512);
    run(k<5>, "ds_add lanes0-4 asm-masked, 8 waves, 256 blk", 256, 512);
    run(k<3>, "ds_add lanes0-2, 8 waves, 256 blk", 256, 512);
    run(k<4>, "ds_add lanes0-4 masked, 8 waves, 256 blk", 256, 512);
    run(k<0>, "ds_add lanes0-4, 1 wave, 2048 blk", 2048, 64);
    run(k<0>, "ds_add lanes0-4, 8 waves, 2048 blk", 2048, 512);
    run(k<0>, "ds_add lanes0-4, 1 wave, 16384 blk", 16384, 64);
    return 0;
}
