#!/bin/bash
# config-3 stage table of several library builds (ST_LIB=tools/var/<v>.so; timing only)
for v in "$@"; do
  echo "== $v"
  ST_LIB=tools/var/$v.so timeout -k 10 300 python3 tools/bench_paths.py 2>/dev/null | python3 -c "
import json,sys; d=json.load(sys.stdin)
print('config3', round(d['config3']['ms'],3), 'one_call', round(d['config3_one_call']['ms'],3))
for k,v in d['stages'].items(): print(' ', k, round(v['ms'],3), round(v['frac_hbm'],3))
" || exit 1
done
