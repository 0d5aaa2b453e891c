#!/bin/bash
# Round 5: k_welford_chains against the three-wave head kernel on one 272k-record entity, alone (0),
# beside an HBM copy (1) and beside FP64 FMA chains on every SIMD (2).
set -o pipefail
for h in 0 1 2; do echo "== background $h"; timeout -k 10 120 ./tools/debug/w2_16 272000 256 $h || exit 1; done
