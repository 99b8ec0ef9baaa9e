#!/bin/bash
# k-means parity tests on tools/var/$1.so, then base vs $1 k-means micro-bench (experiment):
#   tools/experiments/ab_var.sh VARIANT   (build both with tools/experiments/mkvar.sh first)
set -o pipefail
v=${1:-ring}
mkdir -p gpurun_out
ST_LIB=tools/var/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 200 --timeout-method thread -k "kmeans or assign or sog or ties" > gpurun_out/${v}_tests.log 2>&1 || { tail -30 gpurun_out/${v}_tests.log; exit 1; }
tail -2 gpurun_out/${v}_tests.log
KN_N=10000000 bash tools/experiments/var_run.sh base $v base $v
