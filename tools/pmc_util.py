#!/usr/bin/env python3
"""Summarise the sweep's utilisation counters (tools/pmc.sh util --n 10000000 --iters 1: three
separate --pmc passes, kernel trace only) into profiles/<round>/pmc_sweep_util.json: the
engine clock the chip held during the launch, matrix-pipe busy and wave wait fractions.
    python tools/pmc_util.py [tag] [round]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else 'util'
rnd = sys.argv[2] if len(sys.argv) > 2 else 'r01'
XCDS, SIMDS, CUS = 8, 1024, 256
FLOP_PER_CLK_PER_CU = 2.5e15 / (CUS * 2.4e9)  # dense fp16 MFMA at the 2.4 GHz peak clock

c = collections.defaultdict(float)
dur = []
for i in (1, 2, 3):
    f = glob.glob(os.path.join(ROOT, 'gpurun_out', f'{tag}_{i}', '**', '*counter_collection.csv'), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if 'k_sweep<3, 0>' in r['Kernel_Name']]
    disp = {}
    for r in rows:
        c[(i, r['Counter_Name'])] += float(r['Counter_Value'])
        disp[r['Dispatch_Id']] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    dur += list(disp.values())
ns = sum(dur) / len(dur)
gui = c[(1, 'GRBM_GUI_ACTIVE')] / XCDS  # cycles per XCD
clock = gui / ns  # GHz
busy = c[(1, 'SQ_VALU_MFMA_BUSY_CYCLES')] / (gui * SIMDS)
out = {
    'kernel': 'k_sweep<3, 0>',
    'workload': 'tools/kn_bench.py --n 10000000 --iters 1 (the bench launch shape)',
    'passes': 'tools/pmc.sh: three rocprofv3 --pmc passes (8 SQ + GRBM each), kernel trace only',
    'launch_ns': ns,
    'GRBM_GUI_ACTIVE_per_xcd': gui,
    'engine_clock_GHz': clock,
    'SQ_INSTS_MFMA': c[(1, 'SQ_INSTS_MFMA')],
    'SQ_VALU_MFMA_BUSY_CYCLES': c[(1, 'SQ_VALU_MFMA_BUSY_CYCLES')],
    'mfma_busy_frac': busy,
    'SQ_WAVE_CYCLES': c[(1, 'SQ_WAVE_CYCLES')],
    'wait_any_frac_of_wave_cycles': c[(2, 'SQ_WAIT_ANY')] / c[(1, 'SQ_WAVE_CYCLES')],
    'SQ_LDS_BANK_CONFLICT': c[(2, 'SQ_LDS_BANK_CONFLICT')],
    'dense_fp16_peak_at_this_clock_TFLOPs': FLOP_PER_CLK_PER_CU * CUS * clock * 1e9 / 1e12,
    'note': 'the chip holds this clock under the sweep (power-limited); the 2.5 PF headline peak assumes 2.4 GHz',
}
os.makedirs(os.path.join(ROOT, 'profiles', rnd), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, 'profiles', rnd, 'pmc_sweep_util.json'), 'w'), indent=1)
print(json.dumps(out, indent=1))
