#!/bin/bash
# Device decoder A/B on a 20M-record config-2-shaped BAM: tree (2 KB window, 8-bit literal table) vs a 1 KB window, and a 7-bit literal
# table and a 1 KB window, each with amdgpu_waves_per_eu(8) on k_inflate (SGPRs 106 -> 78, 21 spilled to VGPR lanes).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4zd
mkdir -p $OUT
g++ -O2 -fopenmp -o tools/synthbam tools/synthbam.cpp -lz || exit 1
for L in "" exp/gbam_w1k_w8.so exp/gbam_lit7w1k_w8.so "" exp/gbam_w1k_w8.so exp/gbam_lit7w1k_w8.so; do
  n=$(basename ${L:-tree} .so)
  SCT_GBAM_LIB_PATH=$L timeout -k 10 400 python -u tools/e2e_bench.py --synth --records 20000000 > $OUT/e_$n.json 2> $OUT/e_$n.err || { tail -30 $OUT/e_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/e_$n.json')); print('$n', d['GatherCellMetrics_s'], round(d['device_decode_stages_s']['inflate'], 4))"
done
