#!/bin/bash
# Device decoder A/B on a 20M-record config-2-shaped BAM: tree (2 KB window, 8-bit literal table) vs a 7-bit literal
# table, a 1 KB window, and both (the kernel is at 26 waves per CU by LDS, 28 by SGPRs).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4zc
mkdir -p $OUT
g++ -O2 -fopenmp -o tools/synthbam tools/synthbam.cpp -lz || exit 1
for L in "" exp/gbam_lit7.so exp/gbam_w1k.so exp/gbam_lit7w1k.so "" exp/gbam_lit7.so exp/gbam_w1k.so exp/gbam_lit7w1k.so; do
  n=$(basename ${L:-tree} .so)
  SCT_GBAM_LIB_PATH=$L timeout -k 10 400 python -u tools/e2e_bench.py --synth --records 20000000 > $OUT/e_$n.json 2> $OUT/e_$n.err || { tail -30 $OUT/e_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/e_$n.json')); print('$n', d['GatherCellMetrics_s'], round(d['device_decode_stages_s']['inflate'], 4))"
done
