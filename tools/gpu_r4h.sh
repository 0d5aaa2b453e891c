#!/bin/bash
# End to end on a config-2-shaped 50M-record BAM (tools/synthbam.cpp): GatherCellMetrics with the
# device decoder, with devices=[0,0,0] (three parts), and with the host decoder; CSVs compared.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4h
mkdir -p $OUT
g++ -O2 -fopenmp -o tools/synthbam tools/synthbam.cpp -lz || exit 1
timeout -k 10 1000 python -u tools/e2e_bench.py --synth --records 50000000 --host-decoder --devices 3 > $OUT/e2e_synth50m.json 2> $OUT/e2e_synth50m.err || { tail -30 $OUT/e2e_synth50m.err; exit 1; }
cat $OUT/e2e_synth50m.json
