#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_variants.sh r4d/var exp/emitv8.so exp/emitv16.so || exit 1
