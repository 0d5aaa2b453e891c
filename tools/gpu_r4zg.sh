#!/bin/bash
# Device decoder A/B on the 50M-record config-2-shaped BAM: tree (16-thread prefault of the mapping) vs MAP_POPULATE
# (exp/patches/gbam_populate.py).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4zg
mkdir -p $OUT
g++ -O2 -fopenmp -o tools/synthbam tools/synthbam.cpp -lz || exit 1
for L in "" exp/gbam_populate.so "" exp/gbam_populate.so; do
  n=$(basename ${L:-tree} .so)
  SCT_GBAM_LIB_PATH=$L timeout -k 10 400 python -u tools/e2e_bench.py --synth --records 50000000 > $OUT/e_$n.json 2> $OUT/e_$n.err || { tail -30 $OUT/e_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/e_$n.json')); st=d['device_decode_stages_s']; print('$n', d['GatherCellMetrics_s'], round(st['map_scan'], 4), round(st['h2d'], 4), round(st['inflate'], 4))"
done
