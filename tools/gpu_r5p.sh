#!/bin/bash
# Round 5: build_keys ablations (no stream lanes / no counters / every batch one run), config 2.
set -o pipefail
bash tools/gpu_tl_ab.sh bkab base=exp/base5.so nostream=exp/bk_nostream.so nocount=exp/bk_nocount.so noheads=exp/bk_noheads.so || exit 1
