#!/usr/bin/env python3
"""Per-step kernel time of the library from a rocprofv3 trace directory (sqlite .db or csv) of
`bench.py --steps 1 --warmup 0 --no-verify ...` (the timed step plus the stage-marked step =
2 steps).  Prints the top kernels (ms per step) and the memory-copy totals.
    python tools/step_breakdown.py gpurun_out/prof_single [steps=2]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def rows(d):
    for f in glob.glob(os.path.join(d, '**', '*.db'), recursive=True):
        c = sqlite3.connect(f)
        for name, dur in c.execute('select name, duration from kernels'):
            yield 'k', name, dur
        for name, dur, size in c.execute('select name, duration, size from memory_copies'):
            yield 'm', f'{name} ({size >> 20} MiB)' if size >= (1 << 20) else name, dur


def main():
    d = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    tot, cnt = defaultdict(float), defaultdict(int)
    mt, mc = defaultdict(float), defaultdict(int)
    for kind, name, dur in rows(d):
        if kind == 'k':
            if 'st::' not in name and 'rocclr' not in name:
                continue
            short = name.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
            tot[short] += dur / 1e6
            cnt[short] += 1
        else:
            mt[name] += dur / 1e6
            mc[name] += 1
    print(f'library kernels: {sum(tot.values()) / steps:.2f} ms per step')
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:70]:
        print(f'{v / steps:9.3f} ms {cnt[k] / steps:7.1f}x  {k}')
    for k, v in sorted(mt.items(), key=lambda x: -x[1])[:8]:
        print(f'copy {v / steps:9.3f} ms {mc[k] / steps:7.1f}x  {k}')


if __name__ == '__main__':
    main()
