#!/bin/bash
# Round 6: the group sort's long groups of <= 256 records on one-wave blocks: tag-sort and
# config-5 tests on the tree, then the sort alone (tools/c5_sort_probe.py) tree vs HEAD, then bench c5.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6n
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tagsort.py tests/test_gpu_configs.py -k "tag or group or config5" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
  timeout -k 10 240 python3 tools/c5_sort_probe.py > $OUT/tree$rep.txt 2>&1 || { tail -20 $OUT/tree$rep.txt; exit 1; }
  SCT_LIB_PATH=$R/exp/head.so timeout -k 10 240 python3 tools/c5_sort_probe.py > $OUT/head$rep.txt 2>&1 || { tail -20 $OUT/head$rep.txt; exit 1; }
done
tail -n 1 $OUT/tree*.txt $OUT/head*.txt
timeout -k 10 300 python3 bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.log || { tail -20 $OUT/bench_c5.log; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_c5.json')); print('c5', d['ms_per_step'], d['roofline'].get('step_traffic_bytes'))"
