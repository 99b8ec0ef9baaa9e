#!/usr/bin/env python3
"""Mean duration per launch of the kernels matching a regex in a rocprofv3 --kernel-trace
directory (sqlite .db):  kstats.py DIR REGEX"""
import glob
import re
import sqlite3
import sys
from collections import defaultdict

d, rx = sys.argv[1], re.compile(sys.argv[2])
db = glob.glob(d + '/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
ks = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
kd = [t for t in tabs if t.startswith('rocpd_kernel_dispatch')][0]
tot = defaultdict(list)
for n, s, e in c.execute(f'select s.display_name, d.start, d.end from {kd} d join {ks} s on d.kernel_id = s.id'):
    n = re.sub(r'\(.*', '', n.replace('void ', '').replace('(anonymous namespace)::', ''))
    if rx.search(n):
        tot[n].append((e - s) / 1e3)
for k, v in sorted(tot.items()):
    print(f'{k:50s} {sum(v) / len(v):10.1f} us x{len(v)}')
