#!/bin/bash
set -o pipefail
OUT=gpurun_out/r4p
mkdir -p $OUT
for v in base dpp_noasm dpp_noasm_noload simple simple_noload2 pairs0; do
  timeout -k 10 60 ./exp/wm_$v 272000 | sed "s/^/$v /" | tee -a $OUT/wm.txt || exit 1
done
