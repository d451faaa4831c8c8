/* Checks that the FMA-corrected quotient used by the kernels' div_exact
 * (q = x*r, e = fma(-q, n, x), q' = fma(e, r, q) with r = RN(1/n)) equals the
 * IEEE quotient x / n for small integer divisors and random finite x over a
 * wide exponent range (Markstein's theorem: exact whenever r is the
 * correctly rounded reciprocal and no under/overflow occurs).
 * Usage: div_exact_check <max_n> <samples_per_n> <seed>; prints mismatches. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s;
static uint64_t next(void) {   /* splitmix64 */
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  const int max_n = argc > 1 ? atoi(argv[1]) : 256;
  const long per = argc > 2 ? atol(argv[2]) : 100000;
  s = argc > 3 ? strtoull(argv[3], 0, 10) : 1;
  long bad = 0, total = 0;
  for (int n = 1; n <= max_n; ++n) {
    const double nd = (double)n, r = 1.0 / nd;
    for (long i = 0; i < per; ++i) {
      /* random sign, mantissa and exponent in [-300, 300] */
      uint64_t b = next();
      uint64_t e = (uint64_t)(1023 - 300 + (next() % 601));
      b = (b & 0x800FFFFFFFFFFFFFull) | (e << 52);
      double x;
      memcpy(&x, &b, 8);
      if (i & 1) x = (double)(int64_t)(next() % 2000001) * 0.001; /* price-like decimals */
      const double q = x * r;
      const double err = fma(-q, nd, x);
      const double got = fma(err, r, q);
      const double want = x / nd;
      ++total;
      if (got != want && !(x == 0.0)) {
        if (bad < 10) printf("mismatch n=%d x=%.17g got=%.17g want=%.17g\n", n, x, got, want);
        ++bad;
      }
    }
  }
  printf("checked %ld mismatches %ld\n", total, bad);
  return bad != 0;
}
