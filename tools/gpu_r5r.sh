#!/bin/bash
# Round 5: is the key pass bound by its load instructions?  Without the byte-column loads / without
# the ref + pos loads, config 2.
set -o pipefail
bash tools/gpu_tl_ab.sh bkld base=exp/base5.so nostream=exp/bk_nostream.so nobytes=exp/bk_nobytes.so noref=exp/bk_noref.so || exit 1
