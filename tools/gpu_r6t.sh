#!/bin/bash
# Round 6: config 4's key pass with every batch taken as one run (timing only)
set -o pipefail
bash tools/gpu_tl_ab.sh r6t --args "--config 4" tree=tree onerun=exp/r6_bk_onerun.so
