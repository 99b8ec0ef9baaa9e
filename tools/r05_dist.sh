#!/bin/bash
# round 5: the sharded path's per-rank cost at the per-rank size of the 8-way 10M job (1.25M
# splats): kernel traces of st_dev_sog_sharded at world 1 (RCCL) and st_dev_sog, their per-step
# kernel sums (tools/step_breakdown.py) beside each run's wall time per step
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
rm -rf $R/gpurun_out/pdist $R/gpurun_out/psing
C="--total-splats 1250000 --steps 4 --warmup 0 --no-verify --no-cpu-baseline --no-e2e --no-paths --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/pdist -o dist -- python3 $R/bench.py --dist $C > $R/gpurun_out/pdist.json 2> $R/gpurun_out/pdist.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/psing -o single -- python3 $R/bench.py $C > $R/gpurun_out/psing.json 2> $R/gpurun_out/psing.err && \
python3 $R/tools/step_breakdown.py $R/gpurun_out/pdist 4 > $R/gpurun_out/pdist_breakdown.txt && \
python3 $R/tools/step_breakdown.py $R/gpurun_out/psing 5 > $R/gpurun_out/psing_breakdown.txt || { tail -20 $R/gpurun_out/pdist.err $R/gpurun_out/psing.err; exit 1; }
python3 -c "
import json
for t in ('pdist', 'psing'):
    r = json.load(open('$R/gpurun_out/' + t + '.json')); print(t, r['config']['parallelism'], round(r['ms_per_step'], 2))"
head -45 $R/gpurun_out/pdist_breakdown.txt; head -45 $R/gpurun_out/psing_breakdown.txt
