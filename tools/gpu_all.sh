#!/bin/bash
# the whole GPU suite, then a short headline bench (no CPU baseline / container legs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > gpurun_out/bquick.json 2> gpurun_out/bquick.err
rc=$?
echo rc=$rc; tail -3 gpurun_out/gpu_all.log; cut -c1-220 gpurun_out/bquick.json
exit $rc
