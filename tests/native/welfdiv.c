/* The Welford chain's division (sctools_amd/csrc/finalize.h) must equal the IEEE quotient
 * RN(delta / k) that Python's `mean += delta / count` computes (stats.py:82-87).  Two forms:
 *   Markstein:     y = RN(1/k), q0 = RN(delta * y), r = fma(-q0, k, delta) (exact), q = RN(q0 + r * y);
 *   double-double: y_hi = RN(1/k), y_lo = RN(fma(-k, y_hi, 1) * y_hi), q = fma(delta, y_hi, RN(delta * y_lo))
 *                  (two dependent operations after delta instead of three).
 * Random non-zero deltas over 71 binades and both signs, k up to 2^31 (uniform, small, near
 * powers of two).  Prints the number of mismatches of each form ("markstein double_double").
 * Usage: welfdiv N [seed] */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t rnd(void) {
  s ^= s << 13;
  s ^= s >> 7;
  s ^= s << 17;
  return s;
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 1000000;
  if (argc > 2) s ^= (uint64_t)atoll(argv[2]) * 0x9E3779B97F4A7C15ull;
  long bad = 0, bad_dd = 0;
  for (long it = 0; it < n; it++) {
    uint64_t u = rnd();
    double k;
    switch (it % 4) {
      case 0: k = (double)(1 + u % 2000); break;
      case 1: k = (double)(1 + u % (1ull << 31)); break;
      case 2: k = (double)(1 + u % 1000000); break;
      default: k = (double)((1ull << (u % 31)) + (int)((u >> 40) % 3) - 1 + (((u % 31) == 0) ? 1 : 0));
    }
    if (k < 1) k = 1;
    uint64_t v = rnd();
    uint64_t e = 1023 - 60 + v % 71;
    uint64_t bits = ((v >> 8) & 1ull) << 63 | e << 52 | (rnd() & ((1ull << 52) - 1));
    double delta;
    memcpy(&delta, &bits, 8);
    double y = 1.0 / k;
    double q0 = delta * y;
    double r = fma(-q0, k, delta);
    double q = fma(r, y, q0);
    const double want = delta / k;
    if (q != want) {
      if (bad < 5) printf("mismatch delta=%a k=%.0f\n", delta, k);
      bad++;
    }
    const double y_lo = fma(-k, y, 1.0) * y;
    const double qd = fma(delta, y, delta * y_lo);
    if (memcmp(&qd, &want, 8) != 0) {
      if (bad_dd < 5) printf("double-double mismatch delta=%a k=%.0f\n", delta, k);
      bad_dd++;
    }
  }
  printf("%ld %ld\n", bad, bad_dd);
  return 0;
}
