#!/bin/bash
# 1-D k-means of the headline step: uncertified clusters per iteration (ST_DEBUG) and the kernel
# trace of the cluster1d chain (one bench step)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ST_DEBUG=1 timeout -k 10 300 python3 $R/bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline --no-e2e --no-paths > $R/gpurun_out/k1d.json 2> $R/gpurun_out/k1d.err || { tail -5 $R/gpurun_out/k1d.err; exit 1; }
grep "st k1" $R/gpurun_out/k1d.err | head -80 > $R/gpurun_out/k1_flags.txt
rm -rf $R/gpurun_out/prof_k1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_k1 -o k1 -- python3 $R/bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline --no-e2e --no-paths > /dev/null 2>&1 || { echo prof fail; exit 1; }
echo done
