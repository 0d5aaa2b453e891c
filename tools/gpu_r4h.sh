#!/bin/bash
# 1. onesweep look-ahead depth (config 5): tree (8) / 4 / 16 with SCT_RADIX_ONESWEEP=1, and off.
# 2. End to end on a config-2-shaped 50M-record BAM (tools/synthbam.cpp): GatherCellMetrics with the
#    device decoder, with devices=[0,0,0] (three parts), and with the host decoder; CSVs compared.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4h
mkdir -p $OUT
c5() {  # name lib onesweep
  SCT_LIB_PATH=$2 SCT_RADIX_ONESWEEP=$3 timeout -k 10 300 python bench.py --no-cpu-baseline --no-check --config 5 > $OUT/c5_$1.json 2> $OUT/c5_$1.err || { tail -20 $OUT/c5_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c5_$1.json')); k=d['kernel_ms_per_step']; print('$1', d['ms_per_step'], {x: k[x] for x in k if 'radix' in x or x == 'scan'})"
}
c5 off "" 0
c5 la8 "" 1
c5 la4 exp/os_la4.so 1
c5 la16 exp/os_la16.so 1
g++ -O2 -fopenmp -o tools/synthbam tools/synthbam.cpp -lz || exit 1
timeout -k 10 900 python -u tools/e2e_bench.py --synth --records 50000000 --host-decoder --devices 3 > $OUT/e2e_synth50m.json 2> $OUT/e2e_synth50m.err || { tail -30 $OUT/e2e_synth50m.err; exit 1; }
cat $OUT/e2e_synth50m.json
