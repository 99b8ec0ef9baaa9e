#!/bin/bash
# round 5 (late): the SOG / k-means GPU tests after the grouping, the deferred large-cluster
# check and the SH point set prepared beside the 1-D block; then a short bench line (verified)
# and a kernel trace of one step (tools/k1_trace.sh)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_sog65k.py -m gpu -x -q --timeout 300 --timeout-method thread -k "kmeans or sog or cluster1d" > gpurun_out/q2_tests.log 2>&1 || { echo tests fail; tail -30 gpurun_out/q2_tests.log; exit 1; }
tail -2 gpurun_out/q2_tests.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-paths --no-extra > gpurun_out/q2_bench.json 2> gpurun_out/q2_bench.err || { echo bench fail; tail gpurun_out/q2_bench.err; exit 1; }
python3 -c "import json; b=json.load(open('gpurun_out/q2_bench.json')); print('value', b['value'], 'ms', b['ms_per_step'], 'verified', b.get('verified'), 'stages', {k: round(v['ms'], 2) for k, v in (b.get('sog_stages') or {}).items()})"
bash tools/k1_trace.sh
