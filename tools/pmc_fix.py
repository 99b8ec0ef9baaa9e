#!/usr/bin/env python3
"""Summarise tools/pmc_fix.sh: per kernel of interest, the mean over its launches of each
counter (SQ_* per launch, FETCH_SIZE x2 + WRITE_SIZE in bytes), with the wave-state shares.
    python tools/pmc_fix.py [gpurun_out] [out.json]"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

KEYS = ('k_fixrow_lp', 'k_code_scatter', 'k_fixpair_b', 'k_sweep<3, 0>', 'k_sweep<3, 1>', 'k_nd_seq', 'k_nd_combine')
if len(sys.argv) > 3:  # other kernels: comma-separated name prefixes
    KEYS = tuple(sys.argv[3].split(','))


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out'
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, 'pmcf_*', 'pmc_counter_collection.csv'))):
        per = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            name = re.sub(r'\(.*', '', r['Kernel_Name'].replace('st::(anonymous namespace)::', '').replace('void ', ''))
            key = next((k for k in KEYS if name.startswith(k)), None)
            if key is None:
                continue
            d = per[(key, r['Dispatch_Id'])]
            d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
            d['_ns'] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        for (key, _), d in per.items():
            for c, v in d.items():
                acc[key][c].append(v)
    out = {}
    for key, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items() if c != '_ns'}
        m['launches'] = len(cs.get('SQ_WAVES', cs.get('FETCH_SIZE', [0])))
        if 'FETCH_SIZE' in m:
            m['read_bytes'] = 2 * m['FETCH_SIZE'] * 1024  # KiB units, gfx950 half count of 16-B reads
        if 'WRITE_SIZE' in m:
            m['write_bytes'] = m['WRITE_SIZE'] * 1024
        wc = m.get('SQ_WAVE_CYCLES')
        if wc:
            for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS',
                      'SQ_ACTIVE_INST_VMEM', 'SQ_WAIT_INST_LDS'):
                if c in m:
                    m['share_' + c] = m[c] / wc
        if m.get('SQ_LDS_IDX_ACTIVE'):
            m['lds_conflict_share'] = m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']
        out[key] = {c: (round(v, 4) if isinstance(v, float) else v) for c, v in sorted(m.items())}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], 'w'), indent=1)


if __name__ == '__main__':
    main()
