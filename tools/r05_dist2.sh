#!/bin/bash
# round 5 (late): the sharded path at world 1 against st_dev_sog at an 8-way rank's size (1.25M)
# and at 10M, interleaved, no profiler: wall time per step of each
set -o pipefail
mkdir -p gpurun_out/dist2
R=$GRAFT_REPO_ROOT
cd $R
for n in 1250000 10000000; do
  for i in 1 2; do
    for m in single dist; do
      f=""; [ $m = dist ] && f="--dist"
      timeout -k 10 300 python3 bench.py $f --total-splats $n --steps 6 --warmup 1 --no-verify --no-cpu-baseline --no-e2e --no-paths --no-extra > gpurun_out/dist2/$m$n$i.json 2> gpurun_out/dist2/$m$n$i.err || { echo "fail $m $n"; tail gpurun_out/dist2/$m$n$i.err; exit 1; }
      python3 -c "import json; r=json.load(open('gpurun_out/dist2/$m$n$i.json')); print('$m', $n, $i, round(r['ms_per_step'], 2))"
    done
  done
done
