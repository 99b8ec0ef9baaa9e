#!/bin/bash
# round 3: the whole GPU suite, then the quick headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03_gpu_tests.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > gpurun_out/r03_bquick.json 2> gpurun_out/r03_bquick.err || { tail -20 gpurun_out/r03_bquick.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r03_bquick.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified']); print(json.dumps(d['sog_stages']))"
