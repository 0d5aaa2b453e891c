#!/bin/bash
# Round 5: the head kernel's per-wave barrier waits inside the drop-in Welford pass (configs 2, 4).
set -o pipefail
for c in 2 4; do SCT_LIB_PATH=$GRAFT_REPO_ROOT/exp/h2prof.so timeout -k 10 200 python3 tools/w2_prof_probe.py $c || exit 1; done
