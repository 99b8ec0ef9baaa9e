#!/bin/bash
# BASELINE configs 4 and 5 at their full sizes through the multi-process sharded path on one GPU
# (bench.py --gpus N --backend gloo: st_dev_sog_sharded in N processes, host shared memory),
# each against the one-GPU run of the same table (equal textures_sha256)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 900 python3 bench.py --steps 1 --warmup 0 --no-weak "$@" > gpurun_out/c45_${tag}.json 2> gpurun_out/c45_${tag}.err \
    || { tail -30 gpurun_out/c45_${tag}.err; return 1; }
  python3 -c "import json; r=json.load(open('gpurun_out/c45_${tag}.json')); print('${tag}', r['n_gpus'], r['config']['parallelism'], r.get('transport'), round(r['ms_per_step'],1), round(r['value'],2), r['verified'], r['textures_sha256'][:16])"
}
run c4_n1 --total-splats 50000000 && run c4_n4 --gpus 4 --backend gloo --total-splats 50000000 \
 && run c5_n1 --merge 4 && run c5_n3 --gpus 3 --backend gloo --merge 4 || exit 1
python3 - <<'PY'
import json
r = {t: json.load(open(f'gpurun_out/c45_{t}.json')) for t in ('c4_n1', 'c4_n4', 'c5_n1', 'c5_n3')}
print('config 4 same textures:', r['c4_n1']['textures_sha256'] == r['c4_n4']['textures_sha256'])
print('config 5 same textures:', r['c5_n1']['textures_sha256'] == r['c5_n3']['textures_sha256'])
PY
