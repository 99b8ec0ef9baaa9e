#!/usr/bin/env python3
"""Idle gaps of the GPU inside one steady-state headline step (tools/prof_gaps.sh trace): the
step is the second group of ten k_sweep<3, 0> launches (the first is the warmup step), widened
to the kernels that run before and after them without a gap of more than 5 ms; prints the busy
time (union of kernels and copies over every stream), the idle time and the largest gaps with
the HIP runtime calls that ran on the host meanwhile.
    python tools/step_gaps.py gpurun_out/prof_gaps [step_index=1]"""
import glob
import os
import sqlite3
import sys
from collections import Counter


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof_gaps'
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    f = glob.glob(os.path.join(d, '**', '*.db'), recursive=True)[0]
    c = sqlite3.connect(f)
    ks = list(c.execute('select name, start, end from kernels order by start'))
    mc = list(c.execute('select name, start, end from memory_copies order by start'))
    try:
        api = list(c.execute('select name, start, end from regions order by start'))
    except sqlite3.Error:
        api = []
    sw = [i for i, k in enumerate(ks) if 'k_sweep<3, 0>' in k[0]]
    first, last = sw[10 * step], sw[10 * step + 9]
    i = first
    while i > 0 and ks[i][1] - ks[i - 1][2] < 5e6:
        i -= 1
    j = last
    while j + 1 < len(ks) and ks[j + 1][1] - ks[j][2] < 5e6 and 'sweep' not in ks[j + 1][0]:
        j += 1
    start, end = ks[i][1], ks[j][2]
    ev = sorted([(a, b, n) for n, a, b in ks if start <= a <= end] + [(a, b, n) for n, a, b in mc if start <= a <= end])
    gaps, busy = [], 0
    cs, ce, cn = ev[0][0], ev[0][1], ev[0][2]
    for a, b, n in ev[1:]:
        if a > ce:
            gaps.append((a - ce, ce, a, cn, n))
            busy += ce - cs
            cs = a
        if b > ce:
            ce, cn = b, n
    busy += ce - cs
    print(f'step window {(end - start) / 1e6:.2f} ms: busy {busy / 1e6:.2f} ms, idle {(end - start - busy) / 1e6:.2f} ms '
          f'in {len(gaps)} gaps')
    hist = Counter()
    for g in gaps:
        hist['<10us' if g[0] < 1e4 else '<50us' if g[0] < 5e4 else '<200us' if g[0] < 2e5 else '>=200us'] += g[0]
    print('idle by gap size (ms):', {k: round(v / 1e6, 2) for k, v in hist.items()})
    for dur, a, b, n0, n1 in sorted(gaps, reverse=True)[:20]:
        during = Counter(n.split('(')[0] for n, s, e in api if s < b and e > a)
        top = ', '.join(f'{k} x{v}' for k, v in during.most_common(4))
        print(f'{dur / 1e3:8.1f} us at +{(a - start) / 1e6:7.2f} ms  after {n0[:38]:38s} before {n1[:38]:38s} | {top}')


if __name__ == '__main__':
    main()
