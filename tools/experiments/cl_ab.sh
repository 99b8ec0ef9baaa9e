#!/bin/bash
# one-workgroup chunk list A/B on the 1-D k-means (kernel stats of tools/k1_dup_bench.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base ss256; do
  rm -rf gpurun_out/prof_cl_$v
  ST_LIB=tools/var/$v.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cl_$v -o cl --output-format csv -- python3 tools/k1_dup_bench.py 10000000 0 > gpurun_out/cl_$v.log 2>&1 || { tail -5 gpurun_out/cl_$v.log; exit 1; }
  grep cluster1d gpurun_out/cl_$v.log | tail -1
  f=$(find gpurun_out/prof_cl_$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'chunk_list' in x['Name']:
        print('  chunk_list', x['Calls'], float(x['AverageNs']) / 1e3, 'us avg', float(x['MaxNs']) / 1e3, 'max')
PY
done
