#!/bin/bash
# the whole GPU suite, then the round's evidence (tools/round_evidence.sh <tag>)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_gpu_tests.log
bash tools/round_evidence.sh "$tag"
