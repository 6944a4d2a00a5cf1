// tic_toc.h -- TicToc steady_clock millisecond timer, same semantics as the reference
// (include/tic_toc.h:7-24); used for the per-phase host timers in bshot_frame_stats.host_ms.
#pragma once
#include <chrono>

class TicToc {
  public:
    TicToc() { tic(); }
    void tic() { start = std::chrono::steady_clock::now(); }
    double toc() {
        end = std::chrono::steady_clock::now();
        std::chrono::duration<double> elapsed_seconds = end - start;
        return elapsed_seconds.count() * 1000;
    }

  private:
    std::chrono::time_point<std::chrono::steady_clock> start, end;
};
