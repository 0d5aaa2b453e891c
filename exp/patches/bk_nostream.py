import sys
p = sys.argv[1] + "/segment.h"
s = open(p).read()
old = "  if constexpr (kStreams) stream_tile<kCell>(r, base, tile_n, my_heads, my_ex, ebase, s_rcp, s_tab, partials,"
assert old in s
s = s.replace(old, "  if constexpr (false) stream_tile<kCell>(r, base, tile_n, my_heads, my_ex, ebase, s_rcp, s_tab, partials,")
open(p, "w").write(s)
