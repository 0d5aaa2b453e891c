set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4_base
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['kernel_ms_per_step'])"
