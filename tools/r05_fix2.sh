#!/bin/bash
# round 5: the lane-per-point fix-up at four waves per SIMD -- k-means parity tests, then kn_bench
# against the 16-lane-group form (libsplat_hip_g16.so), interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=splat-transform_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sog65k.py tests/test_config2_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r05_fix2_tests.log 2>&1 || { tail -40 gpurun_out/r05_fix2_tests.log; exit 1; }
tail -2 gpurun_out/r05_fix2_tests.log
for rep in 1 2 3; do
  for v in lp g16; do
    lib=$L/libsplat_hip.so; [ $v = g16 ] && lib=$L/libsplat_hip_g16.so
    ST_LIB=$lib timeout -k 10 170 python3 tools/kn_bench.py --n 10000000 --iters 3 --dist gauss > gpurun_out/f2_${v}_$rep.log 2>&1 \
      || { tail -20 gpurun_out/f2_${v}_$rep.log; exit 1; }
    echo "$v $rep: $(grep -h 'kmeans total\|kn.fixrow' gpurun_out/f2_${v}_$rep.log | tr '\n' ' ')"
  done
done
# the Node drop-in's PLY -> .sog job: staged-copy rates and the streamed file's phases
timeout -k 10 300 python3 tools/node_probe.py > gpurun_out/node_probe.log 2>&1 || { tail -30 gpurun_out/node_probe.log; exit 1; }
cat gpurun_out/node_probe.log
