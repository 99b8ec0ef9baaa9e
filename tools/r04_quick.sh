#!/bin/bash
# k-means parity tests (+ the container and config-2 tests) + the window / heavy-tailed
# measurement + a headline bench with the end-to-end file leg.  tools/r04_quick.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-q}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_sog65k.py tests/test_webp_gpu.py tests/test_config2_gpu.py \
    -v -x --timeout 300 --timeout-method thread \
    -k "kmeans or argmin or sog65k or sog_golden or bundle or config2 or cluster1d" > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
bash tools/kn_window.sh ${tag} || exit 1
timeout -k 10 600 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-paths > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "
import json; r=json.load(open('gpurun_out/${tag}_bench.json'))
print('value', r['value'], 'ms', r['ms_per_step'], 'sweep', r['roofline']['avg_launch_ms'], 'verified', r['verified'])
print({k: round(v['avg_ms'], 3) for k, v in r['kernels'].items()})
print(r['stages_ms'])
e = r['end_to_end_file']; print('e2e', e['ms'], e['Msplats_per_s'], e['split_ms'], e['archive_equals_in_memory_step'])
print('container', r['container']['ms'])"
