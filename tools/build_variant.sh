#!/bin/bash
# Build the engine of a git revision (default HEAD) into exp/<name>.so for tools/gpu_ab.sh.
# Usage: bash tools/build_variant.sh <name> [rev]
set -e
NAME=$1
REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" sctools_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$ROOT/exp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wall \
  -o "$ROOT/exp/$NAME.so" "$TMP/sctools_amd/csrc/sct_engine.hip" -L/opt/rocm/lib -lrccl
rm -rf "$TMP"
echo "$ROOT/exp/$NAME.so"
