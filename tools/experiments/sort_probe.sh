#!/bin/bash
# rocPRIM radix_sort_pairs probe next to the library's Morton stage (kernel split by rocprofv3)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 tools/var/probe_sort 10000000 30 && timeout -k 10 60 tools/var/probe_sort 10000000 16 &&
timeout -k 10 120 python3 tools/morton_prof.py &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_morton -o mo --output-format csv -- python3 tools/morton_prof.py > gpurun_out/prof_morton.log 2>&1 || exit 1
f=$(find gpurun_out/prof_morton -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, re, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:20]:
    n = x["Name"]; m = re.search(r"(k_\w+(<[^>]*>)?|__amd\w+|elementwise\w*|\w+_kernel)", n)
    print(f"{(m.group(1) if m else n[:50]):40s} {x['Calls']:>5} {float(x['AverageNs'])/1e3:10.1f}us {float(x['TotalDurationNs'])/1e6:9.2f}ms")
PY
