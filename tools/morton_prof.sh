#!/bin/bash
# kernel split of the Morton stage on one input kind: tools/morton_prof.sh gauss|clustered|grid
set -o pipefail
k=${1:-clustered}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_mo_$k
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mo_$k -o mo --output-format csv -- python3 tools/morton_prof.py 10000000 $k > gpurun_out/prof_mo_$k.log 2>&1 || { tail -5 gpurun_out/prof_mo_$k.log; exit 1; }
grep morton gpurun_out/prof_mo_$k.log
f=$(find gpurun_out/prof_mo_$k -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, re, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:16]:
    n = x["Name"]; m = re.search(r"(k_\w+(<[^>]*>)?|__amd\w+|\w+_kernel)", n)
    print(f"{(m.group(1) if m else n[:50]):40s} {int(x['Calls'])/12:7.1f}/call {float(x['AverageNs'])/1e3:10.1f}us {float(x['TotalDurationNs'])/1e6/12:9.3f}ms/call")
PY
