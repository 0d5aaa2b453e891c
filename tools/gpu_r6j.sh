#!/bin/bash
# Round 6: MSD group sort -- tree (segment tile bases in LDS, XCD-grouped segment tiles), lsd (no MSD)
set -o pipefail
bash tools/gpu_tl_ab.sh r6j --args "--config 5" tree=tree msd5=exp/msd5.so
