#!/bin/bash
# round 5: what bounds the lane-per-point fix-up -- timing-only variants without the row gathers
# (every batch reads one row), without the screen, without the sums (kn_bench 10M, 3 iterations)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=splat-transform_amd/lib
for rep in 1 2; do
  for v in base NOGATHER NOSCREEN NOACC; do
    lib=$L/libsplat_hip.so; [ $v != base ] && lib=$L/libsplat_hip_$v.so
    ST_LIB=$lib timeout -k 10 170 python3 tools/kn_bench.py --n 10000000 --iters 3 --dist gauss > gpurun_out/fv_${v}_$rep.log 2>&1 \
      || { tail -20 gpurun_out/fv_${v}_$rep.log; exit 1; }
    echo "$v $rep: $(grep -h 'kn.fixrow' gpurun_out/fv_${v}_$rep.log | tr '\n' ' ')"
  done
done
