import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
s = s.replace("#define SCT_GENE_CHUNK_HOT 65536", "#define SCT_GENE_CHUNK_HOT 16384", 1)
open(p, "w").write(s)
