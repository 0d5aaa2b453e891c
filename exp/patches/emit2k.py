import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
s = s.replace("#define SCT_EMIT_STAGE 4096", "#define SCT_EMIT_STAGE 2048")
open(p, "w").write(s)
