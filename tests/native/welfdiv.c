/* The Welford chain's division in k_welford_wave (sctools_amd/csrc/finalize.h): with
 * y = RN(1/k), q0 = RN(delta * y), r = fma(-q0, k, delta) (exact) and q = RN(q0 + r * y),
 * q must equal the IEEE quotient RN(delta / k) that Python's `mean += delta / count`
 * computes (stats.py:82-87).  Random deltas over 71 binades and both signs, k up to 2^31
 * (uniform, small, near powers of two).  Prints the number of mismatches.
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
  long bad = 0;
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
    if (q != delta / k) {
      if (bad < 5) printf("mismatch delta=%a k=%.0f\n", delta, k);
      bad++;
    }
  }
  printf("%ld\n", bad);
  return 0;
}
