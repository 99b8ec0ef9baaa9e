#!/bin/bash
# the whole GPU suite and smoke() on the current tree (the round-end driver's two steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 880 python -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread > gpurun_out/r05_suite.log 2>&1 \
  || { tail -60 gpurun_out/r05_suite.log; exit 1; }
tail -3 gpurun_out/r05_suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r05_smoke.log 2>&1 \
  || { tail -20 gpurun_out/r05_smoke.log; exit 1; }
cat gpurun_out/r05_smoke.log
