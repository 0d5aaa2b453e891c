#!/bin/bash
# Experiments only: build the working-tree engine with a python patch applied to a copy of csrc.
# Usage: bash tools/build_patched.sh <name> <patch.py>   (patch.py edits files under $1 = copy root)
set -e
NAME=$1
PATCH=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
mkdir -p "$TMP/sctools_amd" "$TMP/include"
cp -r "$ROOT/sctools_amd/csrc" "$TMP/sctools_amd/"
cp "$ROOT"/include/*.h "$TMP/include/"
python3 "$PATCH" "$TMP/sctools_amd/csrc"
mkdir -p "$ROOT/exp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wall \
  -o "$ROOT/exp/$NAME.so" "$TMP/sctools_amd/csrc/sct_engine.hip" -L/opt/rocm/lib -lrccl
rm -rf "$TMP"
echo "$ROOT/exp/$NAME.so"
