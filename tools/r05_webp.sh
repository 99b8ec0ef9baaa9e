#!/bin/bash
# round 5: the container with the colour cache on the means textures only -- the WebP / .sog / file
# tests, the container measurement, the Node drop-in job
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_webp_gpu.py tests/test_sog_file_gpu.py tests/test_js_host.py tests/test_ply_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r05_webp_tests.log 2>&1 || { tail -40 gpurun_out/r05_webp_tests.log; exit 1; }
tail -2 gpurun_out/r05_webp_tests.log
timeout -k 10 300 python3 tools/bench_bundle.py 10000000 --no-pil > gpurun_out/cc_gated.log 2>&1 || { tail -20 gpurun_out/cc_gated.log; exit 1; }
python3 -c "
import json; r=json.loads(open('gpurun_out/cc_gated.log').read().strip().splitlines()[-1]); print('gated', round(r['bundle_wall_ms'],2), round(r['device_kernel_ms'],2), r['archive_bytes'], r['entries'])"
timeout -k 10 300 python3 tools/node_probe.py > gpurun_out/node_probe3.log 2>&1 || { tail -30 gpurun_out/node_probe3.log; exit 1; }
head -2 gpurun_out/node_probe3.log
