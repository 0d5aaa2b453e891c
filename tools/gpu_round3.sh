#!/bin/bash
# One GPU call: tools/gpu_round.sh (all GPU tests, smoke, PMC traffic, config-2 bench, rocprofv3
# stats), the end-to-end GatherCellMetrics bench, the config-4 / config-5 benches, and the device
# decode of the e2e BAM with any experimental gbam libraries given.
# Usage: bash tools/gpu_round3.sh <tag> [exp/gbam*.so ...]
set -o pipefail
T=${1:-run}; shift
bash tools/gpu_round.sh $T || exit 1
OUT=gpurun_out/$T
timeout -k 10 600 python -u tools/e2e_bench.py --records 24000000 --host-decoder > $OUT/e2e.json 2> $OUT/e2e.err || { tail -30 $OUT/e2e.err; exit 1; }
cat $OUT/e2e.json
for L in "" "$@"; do
  if [ -n "$L" ]; then E="env SCT_GBAM_LIB_PATH=$L"; n=$(basename $L .so); else E=""; n=tree; fi
  timeout -k 10 120 $E python tools/gbam_time.py /tmp/sct_e2e_24000000.bam > $OUT/gbam_$n.json 2> $OUT/gbam_$n.err || { tail -5 $OUT/gbam_$n.err; exit 1; }
  echo "$n $(cat $OUT/gbam_$n.json)"
done
for c in 4 5; do
  timeout -k 10 400 python bench.py --config $c > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || { tail -20 $OUT/bench_c$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_c$c.json')); print('c$c', round(d['ms_per_step'],3), d['roofline']['kernel'], round(d['roofline']['frac'],3), d['kernel_ms_per_step'])"
done
