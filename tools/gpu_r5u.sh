#!/bin/bash
# Round 5: gene reduce on a fixed grid (768 blocks, tree; 1536: gb1536) with the bins flushed once per
# bucket run, against round-5 HEAD (base5): gene tests, timelines at configs 2 and 4, PMC writes.
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_buckets.py tests/test_api_gpu.py > gpurun_out/r5u_tests.log 2>&1 || { tail -30 gpurun_out/r5u_tests.log; exit 1; }
tail -2 gpurun_out/r5u_tests.log
bash tools/gpu_tl_ab.sh gr2 base=exp/base5.so g768=tree g1536=exp/gb1536.so || exit 1
bash tools/gpu_tl_ab.sh gr4 --args "--config 4" base=exp/base5.so g768=tree g1536=exp/gb1536.so || exit 1
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gr_pmc -o write -- python3 $GRAFT_REPO_ROOT/tools/pmc_probe.py > $GRAFT_REPO_ROOT/gpurun_out/gr_pmc/write.log 2>&1 || exit 1
echo pmc done
