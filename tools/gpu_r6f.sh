#!/bin/bash
# Round 6: config-5 A/B in one box session: group sort with 4096-item 32-bit radix tiles and position
# values (tree), the same with 2048-item tiles (c5t2k), and the first group sort (c5prev = 5090612).
set -o pipefail
bash tools/gpu_tl_ab.sh r6f2 --args "--config 5" tree=tree t2k=exp/c5t2k.so prev=exp/c5prev.so
