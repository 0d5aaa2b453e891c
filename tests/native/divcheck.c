/* divcheck.c -- exhaustive check of the division-free quotient used by the HIP kernels
 * (sctools_amd/csrc/util.h ratio_rcp): with y = RN(1/b),
 *     q0 = RN(a*y),  r = RN(a - q0*b) (exact, one FMA),  q = RN(q0 + r*y) (one FMA)
 * must equal the IEEE quotient RN(a/b) -- Python's int / int (aggregator.py:191-231, 291)
 * -- for every a in [0, 2^16) and b in [1, 2^16): all values the uint8 / uint16 record
 * columns can hold.  Prints the mismatch count; exit status 0 iff there are none. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

int main(void) {
  long long bad = 0, tot = 0;
#pragma omp parallel for reduction(+ : bad, tot) schedule(dynamic, 64)
  for (int b = 1; b < 65536; b++) {
    const double db = (double)b;
    const double y = 1.0 / db;
    for (int a = 0; a < 65536; a++) {
      const double da = (double)a;
      const double q0 = da * y;
      const double r = fma(-q0, db, da);
      const double q = fma(r, y, q0);
      const double ref = da / db;
      uint64_t x, z;
      memcpy(&x, &q, 8);
      memcpy(&z, &ref, 8);
      tot++;
      bad += x != z;
    }
  }
  printf("%lld %lld\n", tot, bad);
  return bad != 0;
}
