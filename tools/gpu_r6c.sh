#!/bin/bash
# Round 6: the group tag sort (tagsort.h, 32-bit group keys) -- the whole GPU suite (tag-sort tests,
# config 5 at 100M against numpy's lexsort included), bench config 5 and config 2 with kernel tables.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.log || { tail -20 $O/bench_c5.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c5.json'));print('c5', d['ms_per_step'], d['kernel_ms_per_step'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.log || { tail -20 $O/bench_c2.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', d['ms_per_step'], d['dropin_cell_welford_ms'])"
