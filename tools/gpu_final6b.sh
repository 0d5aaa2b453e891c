#!/bin/bash
# End-of-round GPU call B (round 6): per config (2, 4, 5) the PMC traffic passes and the bench line
# reading that PMC file; rocprofv3 kernel stats of the config-2 bench; SQ counter passes (config 2).
set -o pipefail
export TMPDIR=/tmp
T=${1:-final6b}
OUT=gpurun_out/$T
mkdir -p $OUT
for c in 2 4 5; do
  bash tools/pmc_passes.sh $T/pmc_c$c --config $c || { tail -20 $OUT/pmc_c$c/*.log; exit 1; }
  timeout -k 10 400 python bench.py --config $c --traffic-json $OUT/pmc_c$c/pmc_traffic.json > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || { tail -30 $OUT/bench_c$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_c$c.json')); r=d['roofline']; print('c$c', round(d['ms_per_step'],3), r['kernel'], round(r['frac'],3), r.get('traffic'), round(r.get('step_traffic_frac') or 0, 3), d.get('dropin_cell_welford_ms'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o sct -- python bench.py --steps 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -30 $OUT/bench_prof.err; exit 1; }
bash tools/pmc_sq.sh $T/sq || exit 1
echo done
# the Welford start gate under three concurrent drop-in passes: kernel trace of the probe
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/concurrent -o tr -- python3 $GRAFT_REPO_ROOT/tools/concurrent_welford_probe.py > $GRAFT_REPO_ROOT/$OUT/concurrent.txt 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/concurrent.txt; exit 1; }
cd $GRAFT_REPO_ROOT && tail -4 $OUT/concurrent.txt
