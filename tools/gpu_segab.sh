set -o pipefail
mkdir -p gpurun_out/segab
timeout -k 10 60 ./tools/debug/fp64_chain > gpurun_out/segab/fp64.txt 2>&1 && cat gpurun_out/segab/fp64.txt && \
bash tools/gpu_ab.sh segab exp/noseg.so skip-tests && \
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/segab/c4_a.json 2> gpurun_out/segab/c4_a.err && \
SCT_LIB_PATH=exp/noseg.so timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/segab/c4_b.json 2> gpurun_out/segab/c4_b.err && \
python -c "
import json
for f in ('a','b'):
    d=json.load(open('gpurun_out/segab/c4_%s.json'%f)); k=d['kernel_ms_per_step']; print('c4', f, 'ms/step %.3f'%d['ms_per_step'], {x: k[x] for x in list(k)[:6]})"
