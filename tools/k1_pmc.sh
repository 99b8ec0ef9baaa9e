#!/bin/bash
# 1-D assign (k_kd1_assign_acc) utilisation counters on tools/k1_dup_bench.py (3 x 10M values,
# K = 256, 10 iterations): two --pmc passes, kernel trace only
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf gpurun_out/k1pmc_$i
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/k1pmc_$i -o pmc --output-format csv -- python3 tools/k1_dup_bench.py ${K1N:-10000000} > gpurun_out/k1pmc_$i.log 2>&1 || { tail -20 gpurun_out/k1pmc_$i.log; exit 1; }
done
python3 - <<'P'
import collections, csv, glob
for kern in ('k_kd1_assign_acc', 'k_kd1_final', 'k_ff_batch'):
    c = collections.defaultdict(float); dur = {}
    for i in (1, 2):
        fs = glob.glob(f'gpurun_out/k1pmc_{i}/**/*counter_collection.csv', recursive=True)
        for r in csv.DictReader(open(fs[0])):
            if kern not in r['Kernel_Name']:
                continue
            c[(i, r['Counter_Name'])] += float(r['Counter_Value'])
            dur[(i, r['Dispatch_Id'])] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    nd = sum(1 for (i, _) in dur if i == 1)
    if not nd:
        continue
    ns = sum(v for (i, _), v in dur.items() if i == 1) / nd
    wc = c[(1, 'SQ_WAVE_CYCLES')] or 1
    print(f'{kern}: {nd} launches, {ns / 1e3:.1f} us avg; per launch: valu {c[(1, "SQ_INSTS_VALU")] / nd:.3e} salu {c[(1, "SQ_INSTS_SALU")] / nd:.3e} '
          f'lds {c[(1, "SQ_INSTS_LDS")] / nd:.3e} lds_bank_conflict {c[(1, "SQ_LDS_BANK_CONFLICT")] / nd:.3e} vmem_rd {c[(2, "SQ_INSTS_VMEM_RD")] / nd:.3e} '
          f'waves {c[(1, "SQ_WAVES")] / nd:.0f} busy {c[(1, "SQ_BUSY_CYCLES")] / nd:.3e}')
    print(f'   of wave cycles: wait_any {c[(2, "SQ_WAIT_ANY")] / wc:.3f} wait_inst_any {c[(2, "SQ_WAIT_INST_ANY")] / wc:.3f} '
          f'wait_inst_lds {c[(2, "SQ_WAIT_INST_LDS")] / wc:.3f} active_any {c[(2, "SQ_ACTIVE_INST_ANY")] / wc:.3f} '
          f'active_valu {c[(2, "SQ_ACTIVE_INST_VALU")] / wc:.3f} active_lds {c[(2, "SQ_ACTIVE_INST_LDS")] / wc:.3f}')
P
