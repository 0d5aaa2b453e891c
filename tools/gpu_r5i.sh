#!/bin/bash
# Round 5: timeline of the drop-in Welford cell pass (config 2 and 4), in-tree library.
set -o pipefail
bash tools/gpu_tl_ab.sh wf2 --args "--welford" tree=tree || exit 1
bash tools/gpu_tl_ab.sh wf4 --args "--welford --config 4" tree=tree || exit 1
