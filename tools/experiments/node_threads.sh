#!/bin/bash
# the Node drop-in's writeSogFile with 2 / 4 / 8 compare threads (ST_MIRROR_THREADS) and with the
# resident-column reuse off (ST_HOST_MIRROR=0): per-rep readPly / writeSogFile ms
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for cfg in "ST_MIRROR_THREADS=8" "ST_MIRROR_THREADS=4" "ST_MIRROR_THREADS=2" "ST_HOST_MIRROR=0"; do
  env $cfg timeout -k 10 300 python3 -u tools/node_probe.py > gpurun_out/nt_$cfg.log 2>&1 || { tail -5 gpurun_out/nt_$cfg.log; exit 1; }
  python3 -c "
import json,sys
ln=[l for l in open('gpurun_out/nt_$cfg.log') if l.startswith('{')][-1]
r=json.loads(ln)['runs']
print('$cfg', [(round(x['readPly'],1), round(x['writeSogFile'],1)) for x in r])"
done
