#!/bin/bash
# k_fixrow_acc time of library variants (tools/var/<name>.so) on the N-D micro-bench (10M x 45, K=65,536)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  rm -rf $R/gpurun_out/fab_$v
  ST_LIB=$R/tools/var/$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fab_$v -o k --output-format csv -- python3 $R/tools/kn_bench.py --n 10000000 --iters 3 > $R/gpurun_out/fab_$v.log 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/fab_$v.log; exit 1; }
  f=$(find $R/gpurun_out/fab_$v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'P'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if any(x in n for x in ['k_fixrow_acc','k_sweep<3, 0>','k_nd_combine','k_nd_seq','k_code_scatter','k_fixpair','k_others','k_exact']):
        print(f"  {n[:50]:50s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:9.1f} us")
P
done
