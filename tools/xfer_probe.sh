#!/bin/bash
# staged host copies: rates under a few thread / chunk settings (tools/xfer_probe.py)
set -o pipefail
mkdir -p gpurun_out
for cfg in "8 16" "16 16" "8 64" "4 16" "16 4"; do
  set -- $cfg
  echo "== threads $1 chunk ${2} MiB"
  ST_XFER_THREADS=$1 ST_XFER_CHUNK_MB=$2 timeout -k 10 120 python3 tools/xfer_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
