#!/bin/bash
# round 5 (late): the fused fix-up's sums reading a half batch's values into registers at once
# (ST_FL_RA=1) -- the k-means parity tests with it, then interleaved kn_bench runs at 10M
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
ST_FL_RA=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_sog65k.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ra_tests.log 2>&1 || { tail -30 gpurun_out/ra_tests.log; exit 1; }
tail -1 gpurun_out/ra_tests.log
for rep in 1 2 3; do
  for ra in 0 1; do
    ST_FL_RA=$ra timeout -k 10 120 python3 tools/kn_bench.py --n 10000000 --iters 3 > gpurun_out/ra_kn_$ra.txt 2>&1 || { tail gpurun_out/ra_kn_$ra.txt; exit 1; }
    echo "ra=$ra $(grep -E 'kn.fixrow|kmeans total' gpurun_out/ra_kn_$ra.txt | tr '\n' ' ') $(grep sha256 gpurun_out/ra_kn_$ra.txt | cut -c1-40)"
  done
done
