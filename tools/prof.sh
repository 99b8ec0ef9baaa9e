#!/bin/bash
# rocprofv3 kernel-trace summary of one bench step (+1 warmup); output under gpurun_out/prof_<tag>
set -o pipefail
tag=${1:-run}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o bench --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 "$@" > gpurun_out/prof_${tag}.json 2> gpurun_out/prof_${tag}.err || { tail -20 gpurun_out/prof_${tag}.err; exit 1; }
f=$(find gpurun_out/prof_${tag} -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -40
