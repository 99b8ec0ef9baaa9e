#!/usr/bin/env python3
"""Summary of tools/experiments/pmc_ab.sh: per library, the sweep launch's clock, matrix-pipe busy and
wave-cycle split.   python tools/experiments/pmc_ab.py base cur"""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for v in sys.argv[1:]:
    c = collections.defaultdict(float)
    dur = {}
    for i in (1, 2):
        fs = glob.glob(os.path.join(ROOT, 'gpurun_out', f'pab_{v}_{i}', '**', '*counter_collection.csv'), recursive=True)
        if not fs:
            continue
        for r in csv.DictReader(open(fs[0])):
            if 'k_sweep<3, 0>' not in r['Kernel_Name']:
                continue
            c[(i, r['Counter_Name'])] += float(r['Counter_Value'])
            dur[(i, r['Dispatch_Id'])] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    ns = sum(v_ for (i, _), v_ in dur.items() if i == 1) / max(1, sum(1 for (i, _) in dur if i == 1))
    gui = c[(1, 'GRBM_GUI_ACTIVE')] / 8
    wc = c[(1, 'SQ_WAVE_CYCLES')]
    print(f'{v}: {ns / 1e6:.2f} ms  clock {gui / ns:.3f} GHz  mfma insts {c[(1, "SQ_INSTS_MFMA")]:.3e}  '
          f'mfma busy {c[(1, "SQ_VALU_MFMA_BUSY_CYCLES")] / (gui * 1024):.3f}  valu insts {c[(1, "SQ_INSTS_VALU")]:.3e}  '
          f'salu {c[(2, "SQ_INSTS_SALU")]:.3e}  lds {c[(2, "SQ_INSTS_LDS")]:.3e}  waves {c[(1, "SQ_WAVES")]:.0f}')
    if wc:
        print(f'   of wave cycles: wait_any {c[(2, "SQ_WAIT_ANY")] / wc:.3f}  wait_inst_any {c[(2, "SQ_WAIT_INST_ANY")] / wc:.3f}  '
              f'active_any {c[(2, "SQ_ACTIVE_INST_ANY")] / wc:.3f}  active_valu {c[(1, "SQ_ACTIVE_INST_VALU")] / wc:.3f}  '
              f'active_lds {c[(2, "SQ_ACTIVE_INST_LDS")] / wc:.3f}  busy_cycles {c[(1, "SQ_BUSY_CYCLES")]:.3e}')
