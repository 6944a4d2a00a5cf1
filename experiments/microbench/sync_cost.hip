// Round trip of one small kernel on gfx950: launch + hipStreamSynchronize vs launch + host spin on a
// flag the kernel's last workgroup stores to pinned host memory (system-scope release).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <emmintrin.h>

__global__ void k_work(float* out, int n, unsigned long long* ctr, unsigned long long expect, volatile int* flag, int seq) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = out[i] * 0.5f + 1.0f;
    __syncthreads();
    if (threadIdx.x == 0 && flag) {
        __threadfence_system();
        if (atomicAdd(ctr, 1ull) == expect) {
            __threadfence_system();
            *flag = seq;
            __threadfence_system();
        }
    }
}

int main() {
    (void)hipSetDevice(0);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    float* d;
    unsigned long long* ctr;
    int* flag;
    const int n = 2048 * 4, B = 256, G = (n + B - 1) / B;
    (void)hipMalloc(&d, n * 4);
    (void)hipMalloc(&ctr, 8);
    (void)hipMemset(ctr, 0, 8);
    (void)hipHostMalloc((void**)&flag, 64, hipHostMallocDefault);
    *flag = 0;
    for (int mode = 0; mode < 2; ++mode) {
        double best = 1e9, tot = 0;
        unsigned long long base = 0;
        const int reps = 2000;
        for (int r = 0; r < reps; ++r) {
            auto t0 = std::chrono::steady_clock::now();
            if (mode == 0) {
                k_work<<<G, B, 0, s>>>(d, n, ctr, 0, nullptr, 0);
                (void)hipStreamSynchronize(s);
            } else {
                const int seq = r + 1;
                k_work<<<G, B, 0, s>>>(d, n, ctr, base + G - 1, flag, seq);
                base += G;
                while (*(volatile int*)flag != seq) _mm_pause();
            }
            auto t1 = std::chrono::steady_clock::now();
            const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
            tot += us;
            if (us < best) best = us;
        }
        (void)hipStreamSynchronize(s);
        std::printf("%s: mean %.2f us, min %.2f us per launch + wait\n", mode == 0 ? "hipStreamSynchronize" : "flag spin   ",
                    tot / reps, best);
    }
    return 0;
}
