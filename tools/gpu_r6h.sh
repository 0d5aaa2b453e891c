#!/bin/bash
# Round 6: config-5 row-gather locality probe (experiment)
set -o pipefail
timeout -k 10 400 python tools/c5_locality_probe.py 2>&1 | grep -v amdgpu.ids
