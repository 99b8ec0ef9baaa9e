#!/bin/bash
# a k-means test selection + kn_bench timings (a quick check of a kernel change)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_sog65k.py tests/test_config2_gpu.py tests/test_dist_gpu.py \
  tests/test_multi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_quick.log 2>&1 || { tail -40 gpurun_out/r05_quick.log; exit 1; }
tail -2 gpurun_out/r05_quick.log
for rep in 1 2; do
  timeout -k 10 170 python3 tools/kn_bench.py --n 10000000 --iters 3 --dist gauss > gpurun_out/q_$rep.log 2>&1 || { tail -20 gpurun_out/q_$rep.log; exit 1; }
  echo "$rep: $(grep -h 'kmeans total\|kn.fixrow\|kn.sweep' gpurun_out/q_$rep.log | tr '\n' ' ')"
done
