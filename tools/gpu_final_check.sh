#!/bin/bash
# End-of-session check: every GPU test, smoke(), the default bench line.
set -o pipefail
mkdir -p gpurun_out/final_check
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_check/pytest.log 2>&1 || { tail -30 gpurun_out/final_check/pytest.log; exit 1; }
tail -2 gpurun_out/final_check/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_check/smoke.log 2>&1 || { tail -20 gpurun_out/final_check/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/final_check/bench.json 2> gpurun_out/final_check/bench.err || { tail -20 gpurun_out/final_check/bench.err; exit 1; }
cat gpurun_out/final_check/bench.json
