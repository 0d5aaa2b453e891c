#!/bin/bash
# Classify with wave-aggregated big-bucket reservations: tests and A/B against the per-thread atomics.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4u
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_buckets.py tests/test_gpu_parity.py "tests/test_gpu_configs.py" -k "buckets or parity or config2 or config4" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAIL|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_variants.sh r4u/var exp/cl_v1.so || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/var/base2.json 2> $OUT/var/base2.err || { tail -20 $OUT/var/base2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/var/base2.json')); print('base2', round(d['ms_per_step'],3), d['kernel_ms_per_step'])"
