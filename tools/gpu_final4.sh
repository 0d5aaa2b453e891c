#!/bin/bash
# End-of-round GPU call (round 4): all GPU tests, smoke, then per config (2, 4, 5) the PMC traffic
# passes and the bench line reading that PMC file; rocprofv3 kernel stats of the config-2 bench.
# Outputs under gpurun_out/<tag>.  (The 50M-record end-to-end bench runs in its own call.)
set -o pipefail
export TMPDIR=/tmp
T=${1:-final4}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
for c in 2 4 5; do
  bash tools/pmc_passes.sh $T/pmc_c$c --config $c || { tail -20 $OUT/pmc_c$c/*.log; exit 1; }
  timeout -k 10 400 python bench.py --config $c --traffic-json $OUT/pmc_c$c/pmc_traffic.json > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || { tail -30 $OUT/bench_c$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_c$c.json')); r=d['roofline']; print('c$c', round(d['ms_per_step'],3), r['kernel'], round(r['frac'],3), r.get('traffic'), round(r.get('step_traffic_frac') or 0, 3), d.get('dropin_cell_welford_ms'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o sct -- python bench.py --steps 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -30 $OUT/bench_prof.err; exit 1; }
echo done
