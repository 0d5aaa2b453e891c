import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
old = "    if (!v || (int32_t)gene >= n_gene_ids) continue;\n    atomicAdd((unsigned long long*)&partials[(int64_t)gene * SCT_NP + lane], (unsigned long long)(int64_t)v);"
assert old in s
s = s.replace(old, "    if (!v || (int32_t)gene >= n_gene_ids) continue;\n    if (v == 0x7fffffff) partials[(int64_t)gene * SCT_NP + lane] = v;")
old = "    if (!v || (int32_t)gene >= n_gene_ids) continue;\n    atomicAdd((unsigned long long*)&partials[(int64_t)gene * SCT_NP + P_FLOAT + lane], v);"
assert old in s
s = s.replace(old, "    if (!v || (int32_t)gene >= n_gene_ids) continue;\n    if (v == 0x7fffffffull) partials[(int64_t)gene * SCT_NP + P_FLOAT + lane] = v;")
open(p, "w").write(s)
