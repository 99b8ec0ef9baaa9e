#!/bin/bash
# one pytest selection against several variant libraries: tools/experiments/var_tests.sh "-k expr" v1 v2 ...
sel=$1; shift
for v in "$@"; do
  echo "== $v"
  ST_LIB=tools/var/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -q --timeout 200 --timeout-method thread $sel 2>&1 | grep -E "passed|failed|FAILED|mismatches" | head -8
done
