# decoder experiment: map the BAM with MAP_POPULATE (page tables filled by the kernel) instead of the
# 16-thread prefault
import sys
p = sys.argv[1] + "/gbam.hip"
s = open(p).read()
old = "mmap(nullptr, fsize, PROT_READ, MAP_PRIVATE, fd, 0);"
assert old in s
s = s.replace(old, "mmap(nullptr, fsize, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);", 1)
old2 = "  prefault(f, fsize);\n  std::vector<Block>& blocks = G->blocks;"
assert old2 in s
s = s.replace(old2, "  std::vector<Block>& blocks = G->blocks;", 1)
open(p, "w").write(s)
