import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
s = s.replace("#define SCT_GENE_CHUNK 16384", "#define SCT_GENE_CHUNK 65536", 1)
open(p, "w").write(s)
