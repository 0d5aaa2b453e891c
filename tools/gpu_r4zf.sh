#!/bin/bash
# Timing ablations for the round-5 hash_tile plan (results wrong on purpose, bench --no-check): k_hash_tile without
# its molecule-table insert, without its (bucket, k1) insert, without its fragment insert.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_variants.sh r4zf/var exp/ht_nomol.so exp/ht_nok1.so exp/ht_nofrg.so || exit 1
