// regrow.h -- process-wide count of grow-only pool reallocations (each one a hipFree, which
// waits for the device, plus a hipMalloc): bshot_work_counters [6] count, [7] bytes.
#pragma once
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstdlib>

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

