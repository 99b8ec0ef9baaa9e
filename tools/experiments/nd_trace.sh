#!/bin/bash
# kernel trace of one bench step: per-kernel totals (tools/trace_agg.py)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_nd
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_nd -o nd -- python3 $R/bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline --no-e2e --no-paths > $R/gpurun_out/nd.json 2> $R/gpurun_out/nd.err || { echo prof fail; tail $R/gpurun_out/nd.err; exit 1; }
python3 $R/tools/trace_agg.py $R/gpurun_out/prof_nd 60 > $R/gpurun_out/nd_agg.txt
head -30 $R/gpurun_out/nd_agg.txt
