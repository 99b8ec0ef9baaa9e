#!/bin/bash
# kernel-trace summaries of one step through the sharded path (world 1, RCCL) and the
# single-device path, for the per-rank overhead of splat_dist
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dist -o dist -- python3 $R/bench.py --dist --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pd.json 2> $R/gpurun_out/pd.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_single -o single -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-paths > $R/gpurun_out/ps.json 2> $R/gpurun_out/ps.err
echo rc=$?
