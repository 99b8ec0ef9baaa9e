#!/bin/bash
# one bench step with ST_DEBUG: the 1-D k-means' flagged clusters, members and replay candidates
set -o pipefail
mkdir -p gpurun_out
ST_DEBUG=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-verify --no-cpu-baseline --no-e2e --no-paths > gpurun_out/k1dbg.json 2> gpurun_out/k1dbg.err || { tail -20 gpurun_out/k1dbg.err; exit 1; }
grep "st k1" gpurun_out/k1dbg.err | sort | uniq -c | sort -rn | head -40
