#!/bin/bash
# What bounds the fused fix-up (k_fixrow_lp) and the grouping (k_code_scatter): wave-state and
# LDS counters, then FETCH_SIZE / WRITE_SIZE, each in its own --pmc pass over kn_bench at 10M
# (kernel trace only).  Summarise with tools/pmc_fix.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmcf_$i -o pmc --output-format csv -- \
      python3 tools/kn_bench.py --n 10000000 --iters 2 > gpurun_out/pmcf_$i.log 2>&1 || { tail -20 gpurun_out/pmcf_$i.log; exit 1; }
  echo "pass $i done"
done
echo done
