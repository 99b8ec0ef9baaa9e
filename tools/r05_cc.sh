#!/bin/bash
# round 5: (1) the Node drop-in's job (staged-copy rates, addon timings, streamed-file phases) with
# readPly's columns in huge-page external buffers; (2) the colour cache: the .sog container with
# (libsplat_hip.so) and without it (libsplat_hip_nocc.so, -DST_NO_CCACHE), per-texture sizes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=splat-transform_amd/lib
timeout -k 10 300 python3 tools/node_probe.py > gpurun_out/node_probe2.log 2>&1 || { tail -30 gpurun_out/node_probe2.log; exit 1; }
cat gpurun_out/node_probe2.log
for v in cc nocc cc; do
  lib=$L/libsplat_hip.so; [ $v = nocc ] && lib=$L/libsplat_hip_nocc.so
  ST_LIB=$lib timeout -k 10 300 python3 tools/bench_bundle.py 10000000 --no-pil > gpurun_out/cc_$v.log 2>&1 || { tail -20 gpurun_out/cc_$v.log; exit 1; }
  python3 -c "
import json; r=json.loads(open('gpurun_out/cc_$v.log').read().strip().splitlines()[-1]); print('$v', round(r['bundle_wall_ms'],2), round(r['device_kernel_ms'],2), r['archive_bytes'], r['entries'])"
done
