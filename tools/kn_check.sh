#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "kmeans or assign or sog or cluster1d or ties" > gpurun_out/kn_tests.log 2>&1 || { tail -40 gpurun_out/kn_tests.log; exit 1; }
tail -15 gpurun_out/kn_tests.log
timeout -k 10 300 python tools/kn_bench.py --n 10000000 --iters 3 > gpurun_out/kn_bench.log 2>&1 || { tail -20 gpurun_out/kn_bench.log; exit 1; }
cat gpurun_out/kn_bench.log
