#!/bin/bash
# Packed 16-bit counter flush in the key pass (tree) vs the per-counter flush (exp/pf0.so): parity
# tests, then configs 2 and 4 in A B B A order.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/t11; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "config or parity or api" > $OUT/pytest.log 2>&1; tail -2 $OUT/pytest.log
grep -q " passed" $OUT/pytest.log && ! grep -q failed $OUT/pytest.log || exit 1
for c in 4 2; do
  for L in "" exp/pf0.so exp/pf0.so ""; do
    if [ -n "$L" ]; then E="env SCT_LIB_PATH=$L"; n=pf0; else E=""; n=tree; fi
    timeout -k 10 300 $E python bench.py --config $c --no-cpu-baseline --steps 10 > $OUT/c${c}_$n.json 2> $OUT/c${c}_$n.err || { tail -20 $OUT/c${c}_$n.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/c${c}_$n.json')); k=d['kernel_ms_per_step']; print('c$c $n', round(d['ms_per_step'],3), {x: k[x] for x in list(k)[:4]})"
  done
done
