#!/bin/bash
# round 5 (late): the single-device 1-D block with the colours' cluster1d beside the scales' (side
# context, speculative from draw 0) against after them on the main stream (ST_C1_SERIAL=1):
# interleaved bench steps, then a kernel trace of the serial form's block
set -o pipefail
mkdir -p gpurun_out/c1
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2 3; do
  for v in 0 1; do
    ST_C1_SERIAL=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-paths --no-extra --no-verify > gpurun_out/c1/s$v$i.json 2> gpurun_out/c1/s$v$i.err || { echo "fail $v $i"; tail gpurun_out/c1/s$v$i.err; exit 1; }
    python3 -c "import json; b=json.load(open('gpurun_out/c1/s$v$i.json')); print('serial=$v', $i, round(b['ms_per_step'], 2), b['textures_sha256'][:12])"
  done
done
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/c1/prof
ST_C1_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/c1/prof -o k1 -- python3 $R/bench.py --steps 1 --warmup 1 --no-verify --no-cpu-baseline --no-e2e --no-paths --no-extra > /dev/null 2> $R/gpurun_out/c1/prof.err || { tail $R/gpurun_out/c1/prof.err; exit 1; }
python3 $R/tools/trace_block.py $R/gpurun_out/c1/prof k_iota k_sweep 1 > $R/gpurun_out/c1/block.txt
tail -2 $R/gpurun_out/c1/block.txt
