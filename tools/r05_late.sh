#!/bin/bash
# the late Morton / texture order as the default: the GPU suite, smoke() and one default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/r05_suite.sh && \
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r05_late_bench.log 2>&1 \
  || { tail -30 gpurun_out/r05_late_bench.log; exit 1; }
tail -1 gpurun_out/r05_late_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d.get('sog_stages'))[:900])"
