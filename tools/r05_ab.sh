#!/bin/bash
# round 5: (1) the default bench line with its extra records; (2) the assign window A/B --
# round 4's reachable-norm window (libsplat_hip.so) against round 3's palette-wide one
# (libsplat_hip_wr3.so, -DST_WINDOW_R3), interleaved on one box, 10M x 45, K = 65,536, Gaussian
# and heavy-tailed SH; (3) the per-rank work of an 8-way 10M job: 1.25M splats through the
# sharded path at world 1 and through st_dev_sog
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=splat-transform_amd/lib
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05_bench2.json 2> gpurun_out/r05_bench2.err \
  || { tail -40 gpurun_out/r05_bench2.err; exit 1; }
python3 -c "
import json; r=json.load(open('gpurun_out/r05_bench2.json'))
print(r['value'], r['ms_per_step'], r['config']['workload'], r['verified'])
print(json.dumps(r['extra_records'], indent=1))
print(r['end_to_end_file']['ms'], r['kernels']['kn.sweep'], r['kernels']['kn.fixrow'])"
for rep in 1 2 3; do
  for v in r4 r3; do
    lib=$L/libsplat_hip.so; [ $v = r3 ] && lib=$L/libsplat_hip_wr3.so
    for dist in gauss t3; do
      ST_LIB=$lib timeout -k 10 170 python3 tools/kn_bench.py --n 10000000 --iters 3 --dist $dist > gpurun_out/ab_${v}_${dist}_$rep.log 2>&1 \
        || { tail -20 gpurun_out/ab_${v}_${dist}_$rep.log; exit 1; }
      echo "$v $dist $rep: $(grep -h 'kmeans total\|kn.sweep' gpurun_out/ab_${v}_${dist}_$rep.log | tr '\n' ' ')"
    done
  done
done
for m in "--dist" ""; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --total-splats 1250000 --no-extra --no-cpu-baseline --no-e2e --no-paths $m \
    > gpurun_out/r05_rank8$m.json 2> gpurun_out/r05_rank8$m.err || { tail -30 gpurun_out/r05_rank8$m.err; exit 1; }
  python3 -c "
import json; r=json.load(open('gpurun_out/r05_rank8$m.json')); print('1.25M $m', r['config']['parallelism'], round(r['ms_per_step'],2), r['verified'], r['kernels']['kn.sweep'])"
done
