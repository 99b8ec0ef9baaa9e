#!/bin/bash
# selected GPU tests: tools/gpu_quick.sh FILE_OR_K_EXPR...  (pytest args)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > gpurun_out/gpu_quick.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_quick.log; exit $rc
