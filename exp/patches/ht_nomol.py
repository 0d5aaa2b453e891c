# timing ablation only (wrong results): no molecule-table insert in k_hash_tile
import sys
p = sys.argv[1] + "/bucket.h"
s = open(p).read()
old = """    const uint32_t ms =
        ht_insert_cap<unsigned long long>(s_mol, (((uint64_t)bs << mol_bits) | (key >> sh_mol)) << 2, em);"""
assert old in s
s = s.replace(old, """    em = 1 + (int)(key & 1);
    const uint32_t ms = (uint32_t)(key >> sh_mol) & 1023u;""", 1)
open(p, "w").write(s)
