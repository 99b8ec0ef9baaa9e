#!/bin/bash
# sweep utilisation counters for the baseline library (tools/var/base.so) and the current one:
# two --pmc passes each (kernel trace only), summarised by tools/experiments/pmc_ab.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${PMC_LIBS:-base cur}; do
  if [ $v = cur ]; then unset ST_LIB; else export ST_LIB=tools/var/$v.so; fi
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    rm -rf gpurun_out/pab_${v}_$i
    timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pab_${v}_$i -o pmc --output-format csv -- python3 tools/kn_bench.py --n 10000000 --iters 1 > gpurun_out/pab_${v}_$i.log 2>&1 || { tail -20 gpurun_out/pab_${v}_$i.log; exit 1; }
  done
done
python3 tools/experiments/pmc_ab.py ${PMC_LIBS:-base cur}
