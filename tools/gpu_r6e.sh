#!/bin/bash
# Round 6: group tag sort with the first pass's histogram in the pack and position values.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tagsort.py tests/test_gpu_exchange.py tests/test_gpu_configs.py -k "tag or exchange or sorted or config5 or group" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.log || { tail -20 $O/bench_c5.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c5.json'));print('c5', d['ms_per_step'], d['kernel_ms_per_step'])"
