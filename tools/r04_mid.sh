#!/bin/bash
# the k-means / sharded / container GPU tests, then tools/r04_quick.sh's measurements
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-m}
timeout -k 10 900 python -u -m pytest tests/test_multiproc_gpu.py tests/test_multi_gpu.py tests/test_dist_gpu.py -v -x --timeout 300 \
    --timeout-method thread > gpurun_out/${tag}_mtests.log 2>&1 || { tail -30 gpurun_out/${tag}_mtests.log; exit 1; }
tail -2 gpurun_out/${tag}_mtests.log
bash tools/r04_quick.sh ${tag}
