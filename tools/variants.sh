#!/bin/bash
# Per-kernel times of build variants of the engine (SCT_LIB_PATH) on the config-2 workload.
set -o pipefail
OUT=gpurun_out/${1:-variants}
mkdir -p $OUT
shift
for lib in "$@"; do
  SCT_LIB_PATH=$PWD/$lib timeout -k 10 200 python tools/kernel_times.py --only cell_and_gene --reps 3 > $OUT/$(basename $lib .so).json 2> $OUT/$(basename $lib .so).err || { tail -20 $OUT/$(basename $lib .so).err; exit 1; }
  echo "== $lib"; cat $OUT/$(basename $lib .so).json
done
