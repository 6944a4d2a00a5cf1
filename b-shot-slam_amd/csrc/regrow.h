// regrow.h -- process-wide count of grow-only pool reallocations (each one a hipFree, which
// waits for the device, plus a hipMalloc): bshot_work_counters [6] count, [7] bytes.
#pragma once
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

// process-wide regrowth events of the grow-only pools (bshot_work_counters [6] count, [7] bytes);
// BSHOT_GROW_TRACE=1 prints each one (kind, bytes) to stderr
inline std::atomic<long long> g_regrow_n{0}, g_regrow_bytes{0};
inline void note_regrow(const char* kind, size_t bytes) {
    g_regrow_n++;
    g_regrow_bytes += (long long)bytes;
    static const bool tr = std::getenv("BSHOT_GROW_TRACE") != nullptr;
    if (tr) {
        const double ms = std::chrono::duration<double, std::milli>(
                              std::chrono::steady_clock::now().time_since_epoch()).count();
        std::fprintf(stderr, "[bshot grow] t=%.3f ms %s %zu bytes (event %lld)\n", ms, kind, bytes, g_regrow_n.load());
    }
}


// Buffers replaced by a regrowth are not freed in the sweep loop: hipFree waits for the whole
// device and unmaps memory from the GPU, and measured stalls of 6-7 ms of the odometry chain
// followed such frees (profiles/r02h_stalls.txt). They are parked here and freed when a context is
// destroyed (after its streams are synchronised); growth is geometric, so at most about as much
// memory as the live pools is parked.
enum DeferKind { DEFER_DEVICE = 0, DEFER_PINNED = 1 };
inline std::mutex g_defer_mu;
inline std::vector<std::pair<void*, int>> g_deferred;
inline void defer_free(void* p, int kind) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_defer_mu);
    g_deferred.emplace_back(p, kind);
}
// frees every parked buffer (bshot_destroy; hipFree synchronises the device first)
void flush_deferred_frees();
