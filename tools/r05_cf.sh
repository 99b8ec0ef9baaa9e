#!/bin/bash
# round 5 (late): k_centroid_frags with four lanes per row -- the k-means parity tests, then its
# time per launch at K = 65,536 (kernel trace of kn_bench at 10M, 3 iterations)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_sog65k.py tests/test_multi_gpu.py tests/test_multiproc_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cf_tests.log 2>&1 || { tail -30 gpurun_out/cf_tests.log; exit 1; }
tail -1 gpurun_out/cf_tests.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/cf_prof
timeout -k 10 240 rocprofv3 --kernel-trace -d $R/gpurun_out/cf_prof -o cf -- python3 $R/tools/kn_bench.py --n 10000000 --iters 3 > $R/gpurun_out/cf_kn.txt 2>&1 || { tail $R/gpurun_out/cf_kn.txt; exit 1; }
grep sha256 $R/gpurun_out/cf_kn.txt
python3 $R/tools/kstats.py $R/gpurun_out/cf_prof 'centroid_frags|norm_table|half_max|nd_combine|nd_partials|k_sweep<3, 0>'
