/* a / c by reciprocal + FMA residual + FMA correction vs IEEE division (describe2.hip div_c):
   gcc -O2 -ffp-contract=off divc_check.c -lm && ./a.out */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline double dc(double a, double c, double rc) { double q = a * rc; double r = fma(-q, c, a); return fma(r, rc, q); }
int main(void) {
    const double cs[] = {0.78539816339744830961566084581988, 1.5707963267948966192313216916398, 1500.0, 2500.0, 1000.0, 750.0, 1234.5, 3.0, 0.1, 1.0/3.0, 0.7853981633974483 * 3};
    long bad = 0, tot = 0;
    for (int ci = 0; ci < (int)(sizeof cs / sizeof cs[0]); ++ci) {
        const double c = cs[ci], rc = 1.0 / c;
        for (long i = 0; i < 200000000L / 11; ++i) {
            uint64_t u = xr();
            double a;
            if (i & 1) { a = ((double)(u >> 11) * 0x1p-53) * 8.0 - 4.0; a *= c; }      /* |a/c| < 4 */
            else { uint64_t bits = (u & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 - 40 + (u >> 52) % 80) << 52); memcpy(&a, &bits, 8); }
            double t = a / c, m = dc(a, c, rc);
            ++tot;
            if (memcmp(&t, &m, 8) != 0) { if (bad < 5) printf("mismatch c=%.17g a=%.17g %.17g %.17g\n", c, a, t, m); ++bad; }
        }
    }
    printf("tested %ld, mismatches %ld\n", tot, bad);
    return 0;
}
