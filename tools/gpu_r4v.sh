#!/bin/bash
# Device decoder A/B on a 20M-record config-2-shaped BAM: the 4 KB inflate window (tree) vs 2 KB.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4v
mkdir -p $OUT
g++ -O2 -fopenmp -o tools/synthbam tools/synthbam.cpp -lz || exit 1
for L in "" exp/gbam_w2k.so "" exp/gbam_w2k.so; do
  n=$(basename ${L:-tree} .so)
  SCT_GBAM_LIB_PATH=$L timeout -k 10 400 python -u tools/e2e_bench.py --synth --records 20000000 > $OUT/e_$n.json 2> $OUT/e_$n.err || { tail -30 $OUT/e_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/e_$n.json')); print('$n', d['GatherCellMetrics_s'], d['device_decode_stages_s'])"
done
