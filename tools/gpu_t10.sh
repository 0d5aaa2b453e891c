#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/t10; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gbam or api or multigpu" > $OUT/pytest.log 2>&1; tail -2 $OUT/pytest.log
grep -q " passed" $OUT/pytest.log && ! grep -q failed $OUT/pytest.log || exit 1
timeout -k 10 600 python -u tools/e2e_bench.py --records 24000000 > $OUT/e2e.json 2> $OUT/e2e.err || { tail -20 $OUT/e2e.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/e2e.json')); print('e2e', d['GatherCellMetrics_s'], round(d['GatherCellMetrics_records_per_s']/1e6,1), d['device_decode_stages_s'])"
for L in exp/gbam_prev.so "" exp/gbam_prev.so ""; do
  if [ -n "$L" ]; then E="env SCT_GBAM_LIB_PATH=$L"; n=prev; else E=""; n=tree; fi
  timeout -k 10 120 $E python tools/gbam_time.py /tmp/sct_e2e_24000000.bam > $OUT/gbam_$n.json 2> $OUT/gbam_$n.err || { tail -5 $OUT/gbam_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/gbam_$n.json')); print('$n', round(d['decode_s'],4), {k: round(v,4) for k,v in d['stages_s'].items()})"
done
