import sys
p = sys.argv[1] + "/finalize.h"
s = open(p).read()
s = s.replace("#define SCT_WF_PAIRS 2", "#define SCT_WF_PAIRS 1")
open(p, "w").write(s)
