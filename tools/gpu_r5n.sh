#!/bin/bash
# Round 5: the bench step's kernel timeline with gene_reduce ablations (sort only / no gq streams /
# no stream math at all / no global atomics), config 2.
set -o pipefail
bash tools/gpu_tl_ab.sh grab tree=tree sortonly=exp/gr_sortonly.so nostream=exp/gr_nostream.so nouy=exp/gr_nouy.so noatom=exp/gr_noatom.so || exit 1
