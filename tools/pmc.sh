#!/bin/bash
# PMC counters of the k-means sweep (separate --pmc passes, kernel trace only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-pmc}; shift || true
timeout -k 10 300 python3 tools/kn_bench.py "$@" > gpurun_out/${tag}_plain.log 2>&1 || exit 1
cat gpurun_out/${tag}_plain.log
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_COUNT" \
           "SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/${tag}_$i -o pmc --output-format csv -- python3 tools/kn_bench.py "$@" > gpurun_out/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_$i.log; exit 1; }
done
echo done
