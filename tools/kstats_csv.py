#!/usr/bin/env python3
"""the top kernels of a rocprofv3 --stats kernel_stats.csv: name, calls, total ms, mean us
  python tools/kstats_csv.py <kernel_stats.csv> [rows]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    nm = r['Name'].replace('void ', '').replace('st::(anonymous namespace)::', '').split('(')[0]
    print(f"{nm[:70]:70s} {r['Calls']:>6} {float(r['TotalDurationNs']) / 1e6:9.2f} ms {float(r['AverageNs']) / 1e3:9.1f} us")
