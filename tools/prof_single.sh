#!/bin/bash
# kernel trace of the single-device headline step (1 warmup + 1 timed + 1 staged step)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/prof_single -o single -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > $R/gpurun_out/ps.json 2> $R/gpurun_out/ps.err
echo rc=$?
