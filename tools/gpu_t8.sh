#!/bin/bash
# Radix tile size A/B (config 5 bench + count matrix bench): tree (8 items / thread) vs exp libraries.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/t8; mkdir -p $OUT
for L in "" exp/si4.so exp/si6.so ""; do
  if [ -n "$L" ]; then E="env SCT_LIB_PATH=$L"; n=$(basename $L .so); else E=""; n=tree; fi
  timeout -k 10 300 $E python bench.py --config 5 --no-cpu-baseline --steps 5 > $OUT/c5_$n.json 2> $OUT/c5_$n.err || { tail -20 $OUT/c5_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c5_$n.json')); k=d['kernel_ms_per_step']; print('c5 $n', round(d['ms_per_step'],3), round(d['roofline']['frac'],3), {x: k[x] for x in ['radix_downsweep','radix_upsweep','scan']})"
  timeout -k 10 300 $E python tools/count_bench.py > $OUT/cm_$n.json 2> $OUT/cm_$n.err || { tail -20 $OUT/cm_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/cm_$n.json').read().strip().splitlines()[-1]); print('cm $n', round(d['ms_per_step'],3))"
done
