#!/bin/bash
# round 5: the decided points' grouping, k_code_scatter (4,096-point rounds, ST_CS_WG=0) against
# k_code_scatter_run (one reservation per code per workgroup) at several workgroup counts, on the
# SH palette shape at 10M: kernel times under rocprofv3 (tools/kstats.py) and the k-means result
# hash of each
set -o pipefail
mkdir -p gpurun_out/cs
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for W in 0 256 512 128 0 256; do
  rm -rf $R/gpurun_out/cs/p$W
  ST_CS_WG=$W timeout -k 10 240 rocprofv3 --kernel-trace -d $R/gpurun_out/cs/p$W -o cs -- python3 $R/tools/kn_bench.py --n 10000000 --iters 3 > $R/gpurun_out/cs/w$W.txt 2>&1 || { echo "fail $W"; tail $R/gpurun_out/cs/w$W.txt; exit 1; }
  echo "W=$W $(grep sha256 $R/gpurun_out/cs/w$W.txt)"
  python3 $R/tools/kstats.py $R/gpurun_out/cs/p$W 'code_scatter|fixrow_lp|k_sweep<3, 0>'
done
