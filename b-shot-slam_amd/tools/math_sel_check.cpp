// The select forms bm::atan_sel / atan2_sel / acos_sel (csrc/bshot_math.h; the SHOT record producers
// of csrc/describe2.hip) against the branchy fdlibm forms bm::atan_ / atan2_ / acos_ they replace, bit
// for bit, on the argument domains the records use: random doubles across every fdlibm range and their
// boundaries, signed zeros, huge / tiny ratios. Host build (same IEEE +-*/ sqrt, -ffp-contract=off).
// usage: math_sel_check <millions of random cases>; exit 1 on the first mismatch
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../csrc/bshot_math.h"

static uint64_t bits(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}

int main(int argc, char** argv) {
    const long m = argc > 1 ? std::atol(argv[1]) : 4;
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    const double edges[] = {0.0, -0.0, 0.4375, 0.6875, 1.1875, 2.4375, 0.5, 1.0, -1.0, -0.5, 1.862645149230957e-09,
                            6.938893903907228e-18, 3.6893488147419103e+19, 1e-300, 1e300};
    long bad = 0, n = 0;
    auto check = [&](double y, double x) {
        ++n;
        const double a0 = bm::atan2_(y, x), a1 = bm::atan2_sel(y, x);
        if (!(y == 0.0 && x == 0.0) && bits(a0) != bits(a1)) {
            if (++bad < 10) std::printf("atan2(%.17g, %.17g): %.17g vs %.17g\n", y, x, a0, a1);
        }
        const double c = x < -1.0 ? -1.0 : (x > 1.0 ? 1.0 : x);
        const double b0 = bm::acos_(c), b1 = bm::acos_sel(c);
        if (bits(b0) != bits(b1) && !(b0 != b0 && b1 != b1)) {
            if (++bad < 10) std::printf("acos(%.17g): %.17g vs %.17g\n", c, b0, b1);
        }
    };
    for (double e : edges)
        for (double f : edges)
            for (int s = 0; s < 4; ++s) {
                const double y = (s & 1) ? -e : e, x = (s & 2) ? -f : f;
                check(y, x);
                check(std::nextafter(y, 1e308), std::nextafter(x, -1e308));
            }
    for (long i = 0; i < m * 1000000; ++i) {
        const double scale = std::ldexp(1.0, (int)(rng() % 80) - 40);
        const double y = u(rng) * scale, x = u(rng) * (rng() & 1 ? scale : 1.0);
        check(y, x);
        check(u(rng), u(rng));  // acos domain and atan2 of O(1) ratios
    }
    std::printf("cases %ld mismatches %ld\n", n, bad);
    return bad ? 1 : 0;
}
