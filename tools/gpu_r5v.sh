#!/bin/bash
# Round 5: the staged emit with packed byte / halfword columns (epk), and with 2048-record stages at
# 4 / 5 waves per SIMD (epk2k4 / epk2k5), against round-5 HEAD (base5), configs 2 and 4.
set -o pipefail
bash tools/gpu_tl_ab.sh em2 base=exp/base5.so epk=exp/epk.so epk2k4=exp/epk2k4.so epk2k5=exp/epk2k5.so || exit 1
bash tools/gpu_tl_ab.sh em4 --args "--config 4" base=exp/base5.so epk=exp/epk.so epk2k4=exp/epk2k4.so epk2k5=exp/epk2k5.so || exit 1
