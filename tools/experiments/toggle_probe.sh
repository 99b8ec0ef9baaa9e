#!/bin/bash
# operand-data experiments on the assign sweep (variants built by tools/experiments/mkvar.sh; results of
# the variants are not labels, only the sweep's time is read)
mkdir -p gpurun_out
for v in ${@:-base tileconst allsame allzero base}; do
  if [ $v = base ]; then L=""; else L=tools/var/$v.so; fi
  echo "== $v"
  ST_LIB=$L timeout -k 10 120 python tools/kn_bench.py --n 10000000 --iters 2 > gpurun_out/tg_$v.log 2>&1
  rc=$?
  grep -E "kn.sweep" gpurun_out/tg_$v.log || { echo "rc=$rc"; tail -3 gpurun_out/tg_$v.log; }
  [ $rc -ge 124 ] && exit 1
done
exit 0
