# timing ablation only (wrong results): no fragment insert in k_hash_tile
import sys
p = sys.argv[1] + "/bucket.h"
s = open(p).read()
old = """      ht_insert_cap<unsigned long long>(s_frg, fk << 2, ef);
    }
    // split groups"""
assert old in s
s = s.replace(old, """      ef = 1 + (int)(fk & 1);
    }
    // split groups""", 1)
open(p, "w").write(s)
