#!/bin/bash
# Round 5: the Welford drop-in timeline, head kernel with / without the filler waves, configs 2 and 4.
set -o pipefail
export SCT_WF_HEAD_LDS_KB=0
bash tools/gpu_tl_ab.sh f2 --args "--welford" h2f0=exp/h2f0.so h2f12=exp/h2f12.so || exit 1
bash tools/gpu_tl_ab.sh f4 --args "--welford --config 4" h2f0=exp/h2f0.so h2f12=exp/h2f12.so || exit 1
