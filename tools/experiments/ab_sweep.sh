#!/bin/bash
# k-means parity tests on the current library, then the N-D k-means micro-bench on the saved
# baseline library (tools/var/base.so) and the current one, alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 200 --timeout-method thread -k "kmeans or assign or sog or cluster1d or ties" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for v in base cur base cur; do
  if [ $v = base ]; then export ST_LIB=tools/var/base.so; else unset ST_LIB; fi
  echo "== $v"
  timeout -k 10 200 python3 tools/kn_bench.py --n ${KN_N:-10000000} --iters 2 2>&1 | grep -v amdgpu.ids || exit 1
done
