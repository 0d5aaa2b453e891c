import sys
p = sys.argv[1] + "/tagsort.h"
s = open(p).read()
s = s.replace("#define SCT_TIE_V2 1", "#define SCT_TIE_V2 0", 1)
open(p, "w").write(s)
