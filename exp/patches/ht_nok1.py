# timing ablation only (wrong results): no (bucket, k1) insert in k_hash_tile
import sys
p = sys.argv[1] + "/bucket.h"
s = open(p).read()
old = """    if (em != 0) ht_insert_cap<K1E>(s_k1, (K1E)((((uint64_t)bs << b.k1) | (key >> sh_k1)) << 2), ek);"""
assert old in s
s = s.replace(old, """    ek = em;""", 1)
open(p, "w").write(s)
