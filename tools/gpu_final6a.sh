#!/bin/bash
# End-of-round GPU call A (round 6): all GPU tests, smoke, the default bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final6a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print(round(d['ms_per_step'],3), d['value'], r['kernel'], round(r['frac'],3), r.get('traffic'), round(r.get('step_traffic_frac') or 0, 3), d['cpu_baseline']['value'], d.get('dropin_cell_welford_ms'))"
timeout -k 10 400 python bench.py --config 5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -30 $OUT/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c5.json')); r=d['roofline']; print('c5', round(d['ms_per_step'],3), r['kernel'], round(r['frac'],3), r.get('traffic'), round(r.get('step_traffic_frac') or 0, 3))"
