#!/bin/bash
# HBM traffic of the assign sweep at the bench size: FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes (kernel trace only), per MI355X_MICROARCH.md's HBM/rocprofv3 section
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/traffic_$c -o pmc --output-format csv -- \
      python3 tools/kn_bench.py --n 10000000 --iters 1 > gpurun_out/traffic_$c.log 2>&1 || { tail -20 gpurun_out/traffic_$c.log; exit 1; }
done
echo done
