// Host cost of a kernel launch on gfx950 (ROCm 7.2): one thread launching on its own stream, then
// two and four threads launching concurrently on separate streams (the odometry's main thread,
// lookahead worker and queue share the device this way). Prints microseconds per launch.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

__global__ void k_empty(int* p, int n) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) p[0] = n;
}

static double run(int nthreads, int launches, bool with_memset) {
    std::vector<hipStream_t> st(nthreads);
    int* buf = nullptr;
    (void)hipMalloc(&buf, 4096);
    for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::vector<double> us(nthreads);
    auto body = [&](int t) {
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < launches; ++i) {
            if (with_memset && (i & 7) == 0) (void)hipMemsetAsync(buf + t, 0, 4, st[t]);
            k_empty<<<256, 256, 0, st[t]>>>(buf, i);
        }
        auto t1 = std::chrono::steady_clock::now();
        us[t] = std::chrono::duration<double, std::micro>(t1 - t0).count() / launches;
        (void)hipStreamSynchronize(st[t]);
    };
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(body, t);
    for (auto& x : th) x.join();
    for (auto& s : st) (void)hipStreamDestroy(s);
    (void)hipFree(buf);
    double m = 0;
    for (double v : us) m = v > m ? v : m;
    return m;
}

int main() {
    (void)hipSetDevice(0);
    run(1, 200, false);  // warm up
    for (int nt : {1, 2, 4})
        for (int ms : {0, 1})
            std::printf("threads %d memset %d : %.2f us per launch (slowest thread)\n", nt, ms, run(nt, 2000, ms != 0));
    return 0;
}
