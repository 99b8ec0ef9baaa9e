#!/bin/bash
# the whole GPU test suite, then one bench step with the stage table and the container
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -2 gpurun_out/gpu_all.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-paths > gpurun_out/all_bench.json 2> gpurun_out/all_bench.err || { tail -20 gpurun_out/all_bench.err; exit 1; }
python3 - <<'P'
import json
d = json.load(open('gpurun_out/all_bench.json'))
print(d['value'], d['ms_per_step'], (d.get('verification') or {}).get('ok'))
print(json.dumps(d['stages_ms']))
print(json.dumps(d.get('container')))
P
