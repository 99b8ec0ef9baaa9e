#!/bin/bash
# round 5 (late): the N-D assign classification (st_ctx_last_kmeans_stats) -- the parity tests that
# check it, then the SH palette shape at 10M on Gaussian and heavy-tailed (t3) data, 3 iterations
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kmeans_vs_oracle" > gpurun_out/stats_tests.log 2>&1 || { tail -30 gpurun_out/stats_tests.log; exit 1; }
tail -1 gpurun_out/stats_tests.log
for dist in gauss t3; do
  timeout -k 10 300 python3 tools/kn_bench.py --n 10000000 --iters 3 --dist $dist > gpurun_out/stats_$dist.txt 2>&1 || { tail gpurun_out/stats_$dist.txt; exit 1; }
  grep "kmeans total\|assign classification" gpurun_out/stats_$dist.txt
done
