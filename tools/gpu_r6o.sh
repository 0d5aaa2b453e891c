#!/bin/bash
# Round 6: XCD-grouped tiles for the key pass (bk), the gene emit (ge) or both, against the tree (config 2),
# twice each
set -o pipefail
bash tools/gpu_tl_ab.sh r6o tree=tree bk=exp/r6_bk_xcd.so ge=exp/r6_ge_xcd.so bkge=exp/r6_bkge_xcd.so tree2=tree bk2=exp/r6_bk_xcd.so ge2=exp/r6_ge_xcd.so
