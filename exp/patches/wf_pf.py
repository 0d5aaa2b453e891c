import sys
p = sys.argv[1] + "/finalize.h"
s = open(p).read()
s = s.replace("#define SCT_WF_PF 0", "#define SCT_WF_PF 1", 1)
open(p, "w").write(s)
