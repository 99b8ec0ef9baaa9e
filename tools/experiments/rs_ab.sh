set -o pipefail
for v in base rs8 rs24 rs32; do
  echo "== $v"; ST_LIB=tools/var/$v.so timeout -k 10 120 python3 tools/morton_prof.py || exit 1
done
for v in rs8 rs24 rs32; do ST_LIB=tools/var/$v.so timeout -k 10 300 python3 tools/radix_check.py > gpurun_out/rc_$v.log 2>&1 || { tail -5 gpurun_out/rc_$v.log; exit 1; }; tail -1 gpurun_out/rc_$v.log; done
