# the single-window hash tile (k_hash_tile)
import sys
p = sys.argv[1] + "/sct_engine.hip"
s = open(p).read()
s = s.replace("#define SCT_HASH_PIPE 1", "#define SCT_HASH_PIPE 0")
open(p, "w").write(s)
