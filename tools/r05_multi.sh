#!/bin/bash
# round 5 (late): the sharded writer's cluster1d pair on rank 0 -- the multi-rank GPU tests
# (host-staged groups, one-process-per-rank over shared memory, RCCL at world 1, config 4 / 5 at
# full size), then the bench line with its sharded world-1 record
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests/test_multi_gpu.py tests/test_multiproc_gpu.py tests/test_dist_gpu.py tests/test_configs_full_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/multi_tests.log 2>&1 || { echo tests fail; tail -40 gpurun_out/multi_tests.log; exit 1; }
tail -2 gpurun_out/multi_tests.log
timeout -k 10 400 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-paths --no-verify > gpurun_out/multi_bench.json 2> gpurun_out/multi_bench.err || { echo bench fail; tail gpurun_out/multi_bench.err; exit 1; }
python3 -c "
import json; b=json.load(open('gpurun_out/multi_bench.json'))
print('value', round(b['value'], 3), 'ms', round(b['ms_per_step'], 2))
for k, v in b.get('extra_records', {}).items(): print(k, round(v.get('value', 0), 3), round(v.get('ms_per_step', 0), 2))"
