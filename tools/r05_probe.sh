#!/bin/bash
# round 5: (1) the fix-up's memory pattern alone (tools/experiments/gather_probe: 10M random 192-B
# rows); (2) where the streamed .sog file's time goes (ST_DEBUG phase stamps); (3) the bench line
# with the Node host's end-to-end leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/experiments/gather_probe > gpurun_out/gather_probe.log 2>&1 || { cat gpurun_out/gather_probe.log; exit 1; }
cat gpurun_out/gather_probe.log
ST_DEBUG=1 timeout -k 10 300 python3 tools/experiments/sog_file_probe.py > gpurun_out/sog_file_probe.log 2> gpurun_out/sog_file_probe.err \
  || { tail -30 gpurun_out/sog_file_probe.err; exit 1; }
cat gpurun_out/sog_file_probe.log; grep "st sog file" gpurun_out/sog_file_probe.err | tail -4
timeout -k 10 500 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05_bench3.json 2> gpurun_out/r05_bench3.err \
  || { tail -40 gpurun_out/r05_bench3.err; exit 1; }
python3 -c "
import json; r=json.load(open('gpurun_out/r05_bench3.json')); e=r['end_to_end_file']
print(r['value'], r['ms_per_step'], r['verified'], r['kernels']['kn.fixrow'])
print('e2e', e['ms'], e['split_ms'], e['separate_calls']['ms'], e['separate_calls']['split_ms'])
print('node', json.dumps(e['node_host']))"
