#!/bin/bash
# Experiments only: build the working-tree engine with extra compiler flags into exp/<name>.so (tools/gpu_ab.sh).
# Usage: bash tools/build_flags.sh <name> <flags...>     e.g. bash tools/build_flags.sh noseg -DSCT_SEGACC=0
set -e
NAME=$1
shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/exp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wall "$@" \
  -o "$ROOT/exp/$NAME.so" "$ROOT/sctools_amd/csrc/sct_engine.hip" -L/opt/rocm/lib -lrccl
echo "$ROOT/exp/$NAME.so"
