#!/bin/bash
# round 5 evidence on the committed tree, one call: (1) the driver's bench command; (2) the same
# command under rocprofv3 --kernel-trace --stats (without the extra records, whose 50M launches
# would mix into the sweep's average, and without the CPU baseline); (3) the sweep's HBM traffic
# and utilisation passes; (4) the fused fix-up's counter passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err \
  || { tail -30 gpurun_out/r05_bench.err; exit 1; }
python3 -c "
import json; r=json.load(open('gpurun_out/r05_bench.json')); print(r['value'], r['ms_per_step'], r['verified'], r['roofline']['avg_launch_ms'], r['roofline']['frac'])"
rm -rf gpurun_out/r05_prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof -o bench --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/r05_prof.json 2> gpurun_out/r05_prof.err \
  || { tail -30 gpurun_out/r05_prof.err; exit 1; }
echo profiled
bash tools/pmc_traffic.sh && bash tools/pmc.sh util --n 10000000 --iters 1 > gpurun_out/util.log && bash tools/pmc_fix.sh \
  && python3 tools/pmc_fix.py gpurun_out gpurun_out/pmc_fixup.json > /dev/null && echo pmc done
