#!/bin/bash
# 1-D k-means: parity tests touching cluster1d / the SOG writer, one bench step with the stage
# table, then a kernel trace of the 1-D block and the codebook tail (tools/k1_trace.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_dist_gpu.py tests/test_sog65k.py tests/test_typed_columns.py -x -q --timeout 300 --timeout-method thread -k "cluster1d or sog or kmeans or typed" > gpurun_out/k1_tests.log 2>&1 || { tail -40 gpurun_out/k1_tests.log; exit 1; }
tail -2 gpurun_out/k1_tests.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > gpurun_out/k1_bench.json 2> gpurun_out/k1_bench.err || { tail -20 gpurun_out/k1_bench.err; exit 1; }
python3 - <<'P'
import json
d = json.load(open('gpurun_out/k1_bench.json'))
print(d['value'], d['ms_per_step'], d.get('verification', {}).get('ok'))
print(json.dumps(d['stages_ms']))
print(json.dumps({k: v['ms'] for k, v in d['sog_stages'].items()}))
P
bash tools/k1_trace.sh
