#!/bin/bash
# Round 5: what the gene reduce's in-loop run flushes cost (ablation: dropped), config 2 and 4.
set -o pipefail
bash tools/gpu_tl_ab.sh gnf2 base=exp/base5.so noinflush=exp/gr_noinflush.so || exit 1
bash tools/gpu_tl_ab.sh gnf4 --args "--config 4" base=exp/base5.so noinflush=exp/gr_noinflush.so || exit 1
