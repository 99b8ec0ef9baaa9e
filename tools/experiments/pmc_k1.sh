#!/bin/bash
# what bounds the 1-D k-means kernels (k_kd1_assign_acc, k_ff_*): wave-state / LDS counters and
# FETCH / WRITE passes over tools/experiments/k1_bench.py (kernel trace only); summarise with
# tools/pmc_fix.py gpurun_out/k1 out.json k_kd1_assign_acc,k_kd1_final,k_ff_batch,k_ff_finish
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/k1
timeout -k 10 120 python3 tools/experiments/k1_bench.py colours > gpurun_out/k1/time.log 2>&1 && \
timeout -k 10 120 python3 tools/experiments/k1_bench.py scales >> gpurun_out/k1/time.log 2>&1 || { tail gpurun_out/k1/time.log; exit 1; }
cat gpurun_out/k1/time.log
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/k1/pmcf_$i -o pmc --output-format csv -- \
      python3 tools/experiments/k1_bench.py colours > gpurun_out/k1/pmcf_$i.log 2>&1 || { tail -20 gpurun_out/k1/pmcf_$i.log; exit 1; }
  echo "pass $i done"
done
