import sys
p = sys.argv[1] + "/segment.h"
s = open(p).read()
old = """      // MetricAggregator.parse_molecule (aggregator.py:259-334)
      acc.v[0] += 1;"""
assert old in s
s = s.replace(old, """      if (bt == 0xee && xf == 0xee) acc.v[0] += 1;
      if (false)""")
open(p, "w").write(s)
