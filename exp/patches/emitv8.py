import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
s = s.replace("#define SCT_EMIT_VEC 4", "#define SCT_EMIT_VEC 8")
open(p, "w").write(s)
