#!/bin/bash
# L2 hit rate of the assign sweep (TCC_HIT / TCC_MISS, one --pmc pass, kernel trace only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-l2}; shift || true
rm -rf gpurun_out/${tag}
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/${tag} -o pmc --output-format csv -- \
    python3 tools/kn_bench.py --n 10000000 --iters 1 "$@" > gpurun_out/${tag}.log 2>&1 || { tail -20 gpurun_out/${tag}.log; exit 1; }
f=$(find gpurun_out/${tag} -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0]
    acc[n][r['Counter_Name']] += float(r['Counter_Value'])
for n, c in acc.items():
    if 'sweep' in n or 'sumnd' in n or 'fixrow' in n:
        h, m = c.get('TCC_HIT_sum', 0), c.get('TCC_MISS_sum', 0)
        print(f'{n}: hit {h:.3e} miss {m:.3e} hit-rate {h / max(h + m, 1):.3f}')
PY
