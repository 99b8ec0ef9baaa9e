#!/bin/bash
# kernel + memory-copy + HIP runtime trace of the headline step after one warmup step, for the
# GPU's idle gaps inside a steady-state step (tools/step_gaps.py)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_gaps
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d $R/gpurun_out/prof_gaps -o gaps -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-verify --no-cpu-baseline --no-e2e --no-paths > $R/gpurun_out/pg.json 2> $R/gpurun_out/pg.err \
    || { echo fail; tail -5 $R/gpurun_out/pg.err; exit 1; }
echo traced
