#!/bin/bash
# kernel trace of the single-device headline step (1 timed + 1 stage-marked step, no warmup,
# no verification) and its per-step breakdown (tools/step_breakdown.py)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_single
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/prof_single -o single -- python3 $R/bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline --no-e2e --no-paths > $R/gpurun_out/ps.json 2> $R/gpurun_out/ps.err || { echo fail; tail -5 $R/gpurun_out/ps.err; exit 1; }
python3 $R/tools/step_breakdown.py $R/gpurun_out/prof_single 2 | tee $R/gpurun_out/ps_breakdown.txt
