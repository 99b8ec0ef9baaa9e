#!/bin/bash
# rocprofv3 kernel-trace summary of the config-3 HBM-bound path (tools/bench_paths.py)
set -o pipefail
tag=${1:-paths}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o paths --output-format csv -- python3 tools/bench_paths.py > gpurun_out/prof_${tag}.json 2> gpurun_out/prof_${tag}.err || { tail -20 gpurun_out/prof_${tag}.err; exit 1; }
f=$(find gpurun_out/prof_${tag} -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | sed 's/(.*)"/"/' | head -40
