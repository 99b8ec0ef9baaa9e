#!/bin/bash
# kernel traces of one step through the sharded path (st_dev_sog_sharded at world 1, RCCL) and
# the single-device path (st_dev_sog), each with its per-step breakdown (tools/step_breakdown.py):
# the per-rank overhead of the multi-GPU code
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_dist $R/gpurun_out/prof_single
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/prof_dist -o dist -- python3 $R/bench.py --dist --steps 1 --warmup 1 --no-verify --no-cpu-baseline > $R/gpurun_out/pd.json 2> $R/gpurun_out/pd.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/prof_single -o single -- python3 $R/bench.py --steps 1 --warmup 1 --no-verify --no-cpu-baseline --no-e2e --no-paths > $R/gpurun_out/ps.json 2> $R/gpurun_out/ps.err && \
python3 $R/tools/step_breakdown.py $R/gpurun_out/prof_dist 3 > $R/gpurun_out/pd_breakdown.txt && \
python3 $R/tools/step_breakdown.py $R/gpurun_out/prof_single 3 > $R/gpurun_out/ps_breakdown.txt
echo rc=$?
