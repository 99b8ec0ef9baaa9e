#!/bin/bash
# 1-D kernel times of library variants (tools/var/<name>.so) on cluster1d over 3 x 10M values
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  rm -rf $R/gpurun_out/k1v_$v
  ST_LIB=$R/tools/var/$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/k1v_$v -o k --output-format csv -- python3 $R/tools/k1_dup_bench.py 10000000 > $R/gpurun_out/k1v_$v.log 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/k1v_$v.log; exit 1; }
  f=$(find $R/gpurun_out/k1v_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"
  python3 - "$f" <<'P'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_kd1' in r['Name'] or 'k_ff_' in r['Name']:
        print(f"  {r['Name'][:50]:50s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:9.1f} us")
P
done
