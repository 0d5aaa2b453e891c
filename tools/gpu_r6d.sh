#!/bin/bash
# Round 6: gene-view head-bucket ablations (timing only) against the tree.
set -o pipefail
bash tools/gpu_tl_ab.sh r6d tree=tree grnohead=exp/r6_gr_nohead.so emitnohead=exp/r6_emit_nohead.so
