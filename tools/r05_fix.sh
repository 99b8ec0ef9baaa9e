#!/bin/bash
# round 5: the lane-per-point fused fix-up (k_fixrow_lp) -- the k-means parity tests, then an
# interleaved A/B against the 16-lane-group form (libsplat_hip_g16.so, -DST_FIX_GROUP16) and the
# window A/B (libsplat_hip_wr3.so, -DST_WINDOW_R3), 10M x 45, K = 65,536; then the per-rank work of
# an 8-way 10M job (1.25M splats, sharded path at world 1 and st_dev_sog)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=splat-transform_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_sog65k.py tests/test_config2_gpu.py \
  tests/test_full_verify_gpu.py tests/test_multiproc_gpu.py tests/test_process_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_fix_tests.log 2>&1 \
  || { tail -40 gpurun_out/r05_fix_tests.log; exit 1; }
tail -3 gpurun_out/r05_fix_tests.log
for rep in 1 2 3; do
  for v in lp g16 wr3; do
    lib=$L/libsplat_hip.so; [ $v = g16 ] && lib=$L/libsplat_hip_g16.so; [ $v = wr3 ] && lib=$L/libsplat_hip_wr3.so
    ST_LIB=$lib timeout -k 10 170 python3 tools/kn_bench.py --n 10000000 --iters 3 --dist gauss > gpurun_out/fx_${v}_$rep.log 2>&1 \
      || { tail -20 gpurun_out/fx_${v}_$rep.log; exit 1; }
    echo "$v gauss $rep: $(grep -h 'kmeans total\|kn.sweep\|kn.fixrow' gpurun_out/fx_${v}_$rep.log | tr '\n' ' ')"
  done
done
timeout -k 10 170 python3 tools/kn_bench.py --n 10000000 --iters 3 --dist t3 > gpurun_out/fx_lp_t3.log 2>&1 || { tail -20 gpurun_out/fx_lp_t3.log; exit 1; }
echo "lp t3: $(grep -h 'kmeans total\|kn.sweep\|kn.fixrow' gpurun_out/fx_lp_t3.log | tr '\n' ' ')"
for m in "--dist" ""; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --total-splats 1250000 --no-extra --no-cpu-baseline --no-e2e --no-paths $m \
    > gpurun_out/r05_rank8$m.json 2> gpurun_out/r05_rank8$m.err || { tail -30 gpurun_out/r05_rank8$m.err; exit 1; }
  python3 -c "
import json; r=json.load(open('gpurun_out/r05_rank8$m.json')); print('1.25M $m', r['config']['parallelism'], round(r['ms_per_step'],2), r['verified'], r['kernels']['kn.sweep'], r['kernels']['kn.fixrow'])"
done
# chunk pack: SH bytes staged through LDS (libsplat_hip.so) against direct lane stores (libsplat_hip_cp0.so)
for rep in 1 2; do
  for v in cp0 new; do
    lib=$L/libsplat_hip.so; [ $v = cp0 ] && lib=$L/libsplat_hip_cp0.so
    ST_LIB=$lib timeout -k 10 200 python3 tools/bench_paths.py > gpurun_out/cp_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/cp_${v}_$rep.log; exit 1; }
    python3 -c "
import json; r=json.loads(open('gpurun_out/cp_${v}_$rep.log').read().strip().splitlines()[-1]); print('$v $rep', {k: (round(v['ms'], 3), round(v.get('frac_hbm', 0), 3)) for k, v in r['stages'].items()})"
  done
done
