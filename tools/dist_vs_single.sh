#!/bin/bash
# per-rank overhead of the sharded writer: bench.py --dist (st_dev_sog_sharded over a one-rank RCCL
# communicator) against the single-device st_dev_sog, interleaved twice on one box
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --dist --backend nccl --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > gpurun_out/dvs_dist$i.json 2> gpurun_out/dvs_dist$i.err || { tail -20 gpurun_out/dvs_dist$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > gpurun_out/dvs_single$i.json 2> gpurun_out/dvs_single$i.err || { tail -20 gpurun_out/dvs_single$i.err; exit 1; }
done
python3 - <<'P'
import json
for k in ['dist1', 'single1', 'dist2', 'single2']:
    d = json.load(open(f'gpurun_out/dvs_{k}.json'))
    print(k, round(d['ms_per_step'], 2), d.get('verified'), round(d['roofline']['avg_launch_ms'], 2), d['config'].get('workload'))
P
