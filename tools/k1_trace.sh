#!/bin/bash
# kernel trace of one bench step (no ST_DEBUG): the 1-D block's timeline
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_k1b
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_k1b -o k1 -- python3 $R/bench.py --steps 1 --warmup 1 --no-verify --no-cpu-baseline --no-e2e --no-paths > $R/gpurun_out/k1b.json 2> $R/gpurun_out/k1b.err || { echo prof fail; tail $R/gpurun_out/k1b.err; exit 1; }
python3 $R/tools/trace_block.py $R/gpurun_out/prof_k1b k_iota k_sweep 1 > $R/gpurun_out/k1b_block.txt
tail -3 $R/gpurun_out/k1b_block.txt
python3 $R/tools/trace_block.py $R/gpurun_out/prof_k1b k_nd_combine ZZZ -1 > $R/gpurun_out/k1b_tail.txt
tail -3 $R/gpurun_out/k1b_tail.txt
