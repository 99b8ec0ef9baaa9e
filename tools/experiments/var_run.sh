#!/bin/bash
# time the N-D k-means kernels of each variant library: tools/experiments/var_run.sh v0 v1 ...
set -o pipefail
for v in "$@"; do
  echo "== $v"
  ST_LIB=tools/var/$v.so timeout -k 10 300 python3 tools/kn_bench.py --n ${KN_N:-4000000} --iters 2 2>&1 | grep -v amdgpu.ids || exit 1
done
