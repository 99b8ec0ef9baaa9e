#!/bin/bash
# sharded writer: the multi-rank GPU tests (host-staged and RCCL world 1) and the dist harness
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_multi_gpu.py tests/test_dist_gpu.py tests/test_bench_launch.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -40 gpurun_out/dist_tests.log; exit 1; }
tail -2 gpurun_out/dist_tests.log
