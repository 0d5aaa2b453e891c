#!/bin/bash
# Round 5: with the start gate, the head kernel with (tree) / without (wf0) its 12 register-holding waves.
set -o pipefail
bash tools/gpu_tl_ab.sh wfillb2 --args "--welford" fill12=tree fill0=exp/wf0.so || exit 1
bash tools/gpu_tl_ab.sh wfillb4 --args "--welford --config 4" fill12=tree fill0=exp/wf0.so || exit 1
