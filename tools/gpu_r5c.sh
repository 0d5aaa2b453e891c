#!/bin/bash
# Round 5: a kernel-trace timeline of the config-2 step (idle gaps between kernels: host syncs and
# launch latency inside the step), plus the new tests of this round (finalize after a caught error,
# gbam empty parts).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5c
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_api_gpu.py::test_finalize_after_a_caught_error_matches_reference "tests/test_gbam.py::test_parts_with_empty_parts_match_host" tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o tr -- python3 $R/tools/pmc_probe.py --reps 3 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
cd $R
python3 tools/timeline.py $OUT/trace > $OUT/timeline.txt || exit 1
tail -45 $OUT/timeline.txt
