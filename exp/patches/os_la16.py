import sys
p = sys.argv[1] + "/radix.h"
s = open(p).read()
s = s.replace("#define SCT_LOOKAHEAD 8", "#define SCT_LOOKAHEAD 16", 1)
open(p, "w").write(s)
