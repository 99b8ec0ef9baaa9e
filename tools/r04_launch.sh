#!/bin/bash
# bench.py's own N-rank launch on one GPU (--backend gloo: st_dev_sog_sharded in N processes over
# the library's host shared-memory transport) against the one-GPU sharded run of the same table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-10000000}
for n in 2 3; do
  timeout -k 10 600 python3 bench.py --gpus $n --backend gloo --total-splats $T --steps 2 --warmup 1 --no-weak \
      > gpurun_out/launch_n${n}.json 2> gpurun_out/launch_n${n}.err || { tail -30 gpurun_out/launch_n${n}.err; exit 1; }
  echo "n=$n done"
done
timeout -k 10 600 python3 bench.py --gpus 1 --total-splats $T --steps 2 --warmup 1 \
    > gpurun_out/launch_n1.json 2> gpurun_out/launch_n1.err || { tail -30 gpurun_out/launch_n1.err; exit 1; }
python3 - <<'PY'
import json
r = {n: json.load(open(f'gpurun_out/launch_n{n}.json')) for n in (1, 2, 3)}
for n, v in r.items():
    print(n, v['config']['parallelism'], v.get('transport'), v['ms_per_step'], v['value'], v['verified'], v['textures_sha256'][:16])
print('same textures:', len({v['textures_sha256'] for v in r.values()}) == 1)
PY
