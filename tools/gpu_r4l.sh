#!/bin/bash
set -o pipefail
OUT=gpurun_out/r4l
mkdir -p $OUT
timeout -k 10 60 ./exp/fp64_issue | tee $OUT/fp64_issue.txt
