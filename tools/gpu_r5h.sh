#!/bin/bash
# Round 5: the three-wave Welford head kernel with an LDS-only block barrier, chunks of 16 / 32 records,
# alone on one 272k-record entity against k_welford_chains.
set -o pipefail
for c in 16; do timeout -k 10 120 ./tools/debug/w2_$c 272000 || exit 1; done
