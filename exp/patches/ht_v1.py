import sys
p = sys.argv[1] + "/bucket.h"
s = open(p).read()
old = """  E old;
  while (true) {
    old = atomicCAS(&T[h], (E)0, (E)(key | 1));
    if (old == 0 || (old & ~(E)3) == key) break;
    h = h + 1 == (uint32_t)kHTCap ? 0u : h + 1;
  }
  ev = ht_state(T, h, old);
  return h;"""
new = """  while (true) {
    const E old = atomicCAS(&T[h], (E)0, (E)(key | 1));
    if (old == 0) {
      ev = 1;
      return h;
    }
    if ((old & ~(E)3) == key) {
      ev = 0;
      if (!(old & 2) && !(atomicOr(&T[h], (E)2) & 2)) ev = 2;
      return h;
    }
    h = h + 1 == (uint32_t)kHTCap ? 0u : h + 1;
  }"""
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
