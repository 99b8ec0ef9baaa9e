#!/bin/bash
# round 3: GPU suite, quick headline bench, and the self-launched N=2 rehearsal (gloo on one GPU)
# whose textures digest must equal the N=1 run's on the same fixed-seed table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03_gpu_tests.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > gpurun_out/r03_bquick.json 2> gpurun_out/r03_bquick.err || { tail -20 gpurun_out/r03_bquick.err; exit 1; }
cut -c1-300 gpurun_out/r03_bquick.json
timeout -k 10 300 python bench.py --gpus 1 --total-splats 2000000 --dist-python --backend gloo --steps 1 --warmup 1 --no-verify > gpurun_out/r03_n1.json 2> gpurun_out/r03_n1.err || { tail -20 gpurun_out/r03_n1.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --total-splats 2000000 --dist-python --backend gloo --steps 1 --warmup 1 --no-verify > gpurun_out/r03_n2.json 2> gpurun_out/r03_n2.err || { tail -20 gpurun_out/r03_n2.err; exit 1; }
python - <<'P'
import json
a = json.load(open('gpurun_out/r03_n1.json')); b = json.load(open('gpurun_out/r03_n2.json'))
print('n1', a['n_gpus'], a['value'], a['textures_sha256'])
print('n2', b['n_gpus'], b['value'], b['textures_sha256'])
print('digest equal:', a['textures_sha256'] == b['textures_sha256'])
P
