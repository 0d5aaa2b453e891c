#!/bin/bash
# Round 5: gene_reduce with the nibble flag table (nib) and also the gq_gt30 table (nibgq), config 2 and 4.
set -o pipefail
bash tools/gpu_tl_ab.sh nib2 base=exp/base5.so nib=exp/nib.so nibgq=exp/nibgq.so || exit 1
bash tools/gpu_tl_ab.sh nib4 --args "--config 4" base=exp/base5.so nib=exp/nib.so nibgq=exp/nibgq.so || exit 1
