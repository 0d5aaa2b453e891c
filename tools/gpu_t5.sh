#!/bin/bash
# One GPU call (round 3 experiments): device-decode tests with the tree's gbam (8 KB window),
# Welford tests + A/B, config-4 bench, then the device decode timed per inflate window variant.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gbam or api or sortorder or tagsort" > gpurun_out/t5/pytest.log 2>&1; tail -3 gpurun_out/t5/pytest.log; grep -q ' passed' gpurun_out/t5/pytest.log && ! grep -q failed gpurun_out/t5/pytest.log || exit 1
timeout -k 10 300 python -u tools/e2e_bench.py --records 24000000 > gpurun_out/t5/e2e.json 2> gpurun_out/t5/e2e.err || { tail -20 gpurun_out/t5/e2e.err; exit 1; }
cat gpurun_out/t5/e2e.json
for v in gbam_head gbam4096 tree gbam16384 gbam_head tree; do
  if [ $v = tree ]; then E=""; else E="env SCT_GBAM_LIB_PATH=exp/$v.so"; fi
  timeout -k 10 120 $E python tools/gbam_time.py /tmp/sct_e2e_24000000.bam > gpurun_out/t5/gbam_$v.json 2>&1 || { tail -5 gpurun_out/t5/gbam_$v.json; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/t5/gbam_$v.json')); print('$v', round(d['decode_s'],4), {k: round(v,4) for k,v in d['stages_s'].items()})"
done
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/t5/bench_c4.json 2> gpurun_out/t5/bench_c4.err; python -c "import json; d=json.load(open('gpurun_out/t5/bench_c4.json')); print('c4', d['ms_per_step'], d['kernel_ms_per_step'])"
