#!/bin/bash
# The config-2 / 4 / 5 bench lines with their own committed PMC traffic files (profiles/r03/final).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-benches3}; mkdir -p $OUT
for c in 2 4 5; do
  timeout -k 10 400 python bench.py --config $c --traffic-json profiles/r03/final/pmc_traffic_c$c.json > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || { tail -30 $OUT/bench_c$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_c$c.json')); r=d['roofline']; print('c$c', round(d['ms_per_step'],3), r['kernel'], round(r['frac'],3), r.get('traffic'), r.get('step_traffic_frac'), d.get('dropin_cell_welford_ms'))"
done
