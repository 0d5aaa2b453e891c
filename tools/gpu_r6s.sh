#!/bin/bash
# Round 6: the stream lanes' run boundaries flushed by the owning thread alone (tree) against the
# wave-wide per-item flush (HEAD): parity at 100M / 125M, then configs 4 and 2 timelines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_buckets.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_tl_ab.sh r6s_c4 --args "--config 4" tree=tree head=exp/head.so tree2=tree head2=exp/head.so || exit 1
bash tools/gpu_tl_ab.sh r6s_c2 tree=tree head=exp/head.so
