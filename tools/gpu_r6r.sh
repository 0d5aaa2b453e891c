#!/bin/bash
# Round 6: config 4's key pass -- the stream lanes' cost (nostream) and their boundary path's (fastonly)
set -o pipefail
bash tools/gpu_tl_ab.sh r6r --args "--config 4" tree=tree nostream=exp/bk_nostream.so fastonly=exp/r6_bk_fastonly.so
