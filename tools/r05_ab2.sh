#!/bin/bash
# round 5 (late): interleaved same-box A/B of the headline step, base (the committed library) against
# new (grouping with one reservation per code per workgroup, the large-cluster check deferred to
# the next sync): bench.py with ST_LIB, 4 alternations of 10 timed steps each
set -o pipefail
mkdir -p gpurun_out/ab2
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2 3 4; do
  for v in base new; do
    ST_LIB=tools/var/$v.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-paths --no-extra --no-verify > gpurun_out/ab2/$v$i.json 2> gpurun_out/ab2/$v$i.err || { echo "fail $v $i"; tail gpurun_out/ab2/$v$i.err; exit 1; }
    python3 -c "import json; b=json.load(open('gpurun_out/ab2/$v$i.json')); print('$v', $i, round(b['ms_per_step'], 2), b['textures_sha256'][:12] if isinstance(b.get('textures_sha256'), str) else '')"
  done
done
