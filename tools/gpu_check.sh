#!/bin/bash
# GPU round trip: parity tests, then one bench line (no CPU baseline).
# usage: tools/gpu_check.sh [tag] [bench args...]
set -o pipefail
tag=${1:-run}; shift || true
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
