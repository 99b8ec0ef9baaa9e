#!/bin/bash
# k-means parity tests on tools/var/ring.so, then base vs ring micro-bench (experiment)
set -o pipefail
mkdir -p gpurun_out
ST_LIB=tools/var/ring.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 200 --timeout-method thread -k "kmeans or assign or sog or ties" > gpurun_out/ring_tests.log 2>&1 || { tail -30 gpurun_out/ring_tests.log; exit 1; }
tail -2 gpurun_out/ring_tests.log
KN_N=10000000 bash tools/var_run.sh base ring base ring
