#!/bin/bash
set -o pipefail
OUT=gpurun_out/r4k
mkdir -p $OUT
for v in base nodpp nodpp_noasm pure noload; do
  timeout -k 10 60 ./exp/wm_$v 272000 | sed "s/^/$v /" | tee -a $OUT/wm.txt || exit 1
done
