#!/bin/bash
# round 5: BASELINE configs 3/4/5 at full size in the GPU suite (tests/test_configs_full_gpu.py),
# the bench launch test, then the default bench line (one 10M workload at every N + extra records)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 780 python -u -m pytest tests/test_configs_full_gpu.py tests/test_bench_launch.py -m gpu -x -v \
  --timeout 700 --timeout-method thread > gpurun_out/r05_configs.log 2>&1 || { tail -60 gpurun_out/r05_configs.log; exit 1; }
tail -8 gpurun_out/r05_configs.log
timeout -k 10 360 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05_bench1.json 2> gpurun_out/r05_bench1.err \
  || { tail -40 gpurun_out/r05_bench1.err; exit 1; }
python3 -c "
import json; r=json.load(open('gpurun_out/r05_bench1.json'))
print(r['value'], r['ms_per_step'], r['config']['workload'], r['verified'])
print(json.dumps(r['extra_records'], indent=1))
print(r['end_to_end_file']['ms'] if r['end_to_end_file'] else None, r['kernels'])"
