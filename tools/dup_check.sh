#!/bin/bash
# duplicated-points k-means: the duplicated-row tests, then kn_bench timings (2M x 45, K = 65,536:
# no duplicates, 30% all-zero rows; 10M x 45 with 30%)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_edges.py -k "duplicated or split_cluster" -x -q --timeout 300 --timeout-method thread > gpurun_out/dup_tests.log 2>&1 || { tail -30 gpurun_out/dup_tests.log; exit 1; }
tail -2 gpurun_out/dup_tests.log
for zf in 0 0.3; do
  timeout -k 10 300 python tools/kn_bench.py --n 2000000 --iters 2 --zero-frac $zf > gpurun_out/dup_kn_2m_$zf.log 2>&1 || { tail -20 gpurun_out/dup_kn_2m_$zf.log; exit 1; }
  cat gpurun_out/dup_kn_2m_$zf.log
done
timeout -k 10 300 python tools/kn_bench.py --n 10000000 --iters 3 --zero-frac 0.3 > gpurun_out/dup_kn_10m_0.3.log 2>&1 || { tail -20 gpurun_out/dup_kn_10m_0.3.log; exit 1; }
cat gpurun_out/dup_kn_10m_0.3.log
