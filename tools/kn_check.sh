#!/bin/bash
# k-means parity tests (single device + sharded) and the N-D k-means micro-bench at the bench shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_sog65k.py tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread -k "kmeans or assign or sog or ties or partials or dist or step" > gpurun_out/kn_tests.log 2>&1 || { tail -30 gpurun_out/kn_tests.log; exit 1; }
tail -2 gpurun_out/kn_tests.log
timeout -k 10 300 python3 tools/kn_bench.py --n 10000000 --iters 2 2>&1 | grep -v amdgpu.ids
