#!/bin/bash
# 1-D parity tests, then the headline step's 1-D stages under the default build and under each
# given environment switch (e.g. ST_K1_ASSIGN_CHAIN): tools/k1_ab.sh VAR [VAR ...]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_dist_gpu.py tests/test_sog65k.py tests/test_typed_columns.py -x -q --timeout 300 --timeout-method thread -k "cluster1d or sog or kmeans or typed" > gpurun_out/k1ab_tests.log 2>&1 || { tail -40 gpurun_out/k1ab_tests.log; exit 1; }
tail -1 gpurun_out/k1ab_tests.log
run() {
  timeout -k 10 300 env $1 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > gpurun_out/k1ab_$2.json 2> gpurun_out/k1ab_$2.err || { tail -20 gpurun_out/k1ab_$2.err; exit 1; }
  python3 - gpurun_out/k1ab_$2.json $2 <<'P'
import json, sys
d = json.load(open(sys.argv[1]))
s = d['stages_ms']
print(sys.argv[2], round(d['ms_per_step'], 2), d.get('verification', {}).get('ok'), 'k1.assign', round(s['k1.assign'], 3), 'k1.update', round(s['k1.update'], 3),
      {k: round(v['ms'], 3) for k, v in d['sog_stages'].items() if k != 'sog.shkmeans'})
P
}
run ST_NONE=1 base && run ST_NONE=1 base2 || exit 1
for v in "$@"; do run $v=1 $v || exit 1; done
