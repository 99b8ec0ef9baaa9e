#!/bin/bash
# k_small_sort thread-count A/B on the 1-D k-means (kernel stats of tools/k1_dup_bench.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base ss256; do
  rm -rf gpurun_out/prof_ss_$v
  ST_LIB=tools/var/$v.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ss_$v -o ss --output-format csv -- python3 tools/k1_dup_bench.py 10000000 0 > gpurun_out/ss_$v.log 2>&1 || { tail -5 gpurun_out/ss_$v.log; exit 1; }
  grep cluster1d gpurun_out/ss_$v.log | tail -1
  f=$(find gpurun_out/prof_ss_$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'small_sort' in x['Name']:
        print('  k_small_sort', x['Calls'], float(x['AverageNs']) / 1e3, 'us avg', float(x['MinNs']) / 1e3, 'min')
PY
done
