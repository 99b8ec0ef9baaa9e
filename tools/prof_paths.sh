#!/bin/bash
# rocprofv3 kernel-trace summary of the config-3 HBM-bound path (tools/bench_paths.py)
set -o pipefail
tag=${1:-paths}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o paths --output-format csv -- python3 tools/bench_paths.py > gpurun_out/prof_${tag}.json 2> gpurun_out/prof_${tag}.err || { tail -20 gpurun_out/prof_${tag}.err; exit 1; }
f=$(find gpurun_out/prof_${tag} -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, re, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:25]:
    n = x["Name"]; m = re.search(r"(k_\w+(<[^>]*>)?|__amd\w+|onesweep\w+|partition_kernel)", n)
    print(f"{(m.group(1) if m else n[:50]):40s} {x['Calls']:>5} {float(x['AverageNs'])/1e3:10.1f}us {float(x['TotalDurationNs'])/1e6:9.2f}ms")
PY
