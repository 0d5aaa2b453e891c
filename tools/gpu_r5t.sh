#!/bin/bash
# Round 5: gene buckets of 32 / 16 genes against 64 (base5), configs 2 and 4.
set -o pipefail
bash tools/gpu_tl_ab.sh gb2 base=exp/base5.so g32=exp/g32.so g16=exp/g16.so || exit 1
bash tools/gpu_tl_ab.sh gb4 --args "--config 4" base=exp/base5.so g32=exp/g32.so g16=exp/g16.so || exit 1
