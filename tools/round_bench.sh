#!/bin/bash
# the round's evidence: full bench line (with the CPU baseline) + rocprofv3 kernel summary
# of the same command; outputs under gpurun_out/<tag>_*
set -o pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${tag}_prof.json 2> gpurun_out/${tag}_prof.err || { tail -20 gpurun_out/${tag}_prof.err; exit 1; }
echo profiled
