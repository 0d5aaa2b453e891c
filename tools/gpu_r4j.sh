#!/bin/bash
# Welford chain microbenchmarks (the engine kernel on one 272k-record entity, variants), config 4
# bench, and a PMC pass preview of config 2 (gene_reduce writes with the hot-bucket items).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4j
mkdir -p $OUT
for v in base pairs0 nom2 noload nodiv; do
  timeout -k 10 60 ./exp/wm_$v 272000 | sed "s/^/$v /" | tee -a $OUT/wm.txt || exit 1
done
timeout -k 10 120 ./exp/wc_chain > $OUT/wc_chain.txt 2>&1 || { cat $OUT/wc_chain.txt; exit 1; }
cat $OUT/wc_chain.txt
timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || { tail -20 $OUT/c4.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c4.json')); print('c4', d['ms_per_step'], d.get('dropin_cell_welford_ms'), d['kernel_ms_per_step'])"
bash tools/pmc_passes.sh r4j/pmc_c2 --config 2 || exit 1
python -c "import json; d=json.load(open('$OUT/pmc_c2/pmc_traffic.json')); k=d['kernels']; print({x: (round(k[x]['hbm_bytes_per_launch']/1e6,1), round(k[x]['WRITE_SIZE_KiB']*1024/1e6,1)) for x in k})"
