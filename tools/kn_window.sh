#!/bin/bash
# the assign's decision window on Gaussian vs heavy-tailed correlated SH (tools/kn_bench.py
# --dist): per-iteration kernel times, then (ST_DEBUG=1, separate run: it adds syncs) the pair /
# ambiguous counts of every assign.  tools/kn_window.sh <tag> [n]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-win}; n=${2:-10000000}
for dist in gauss t3; do
  timeout -k 10 170 python3 tools/kn_bench.py --n $n --iters 3 --dist $dist > gpurun_out/${tag}_${dist}.log 2>&1 || { tail -20 gpurun_out/${tag}_${dist}.log; exit 1; }
  ST_DEBUG=1 timeout -k 10 170 python3 tools/kn_bench.py --n $n --iters 3 --dist $dist > gpurun_out/${tag}_${dist}_dbg.log 2>&1 || { tail -20 gpurun_out/${tag}_${dist}_dbg.log; exit 1; }
  echo "== $dist"; cat gpurun_out/${tag}_${dist}.log; grep "pairs=" gpurun_out/${tag}_${dist}_dbg.log
done
