#!/bin/bash
# Round 5: where the waves of a small workgroup land (SIMDs), and the Welford head kernels alone on one
# 272k-record entity.
set -o pipefail
timeout -k 10 60 ./tools/debug/hwid || exit 1
timeout -k 10 120 ./tools/debug/w2 272000 || exit 1
bash tools/gpu_tl_ab.sh r5g_tl tree=tree e1=exp/e1_emitpf.so
