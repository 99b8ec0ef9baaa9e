"""Kernel timeline of one window of a rocprofv3 kernel trace (sqlite): every dispatch between
the first kernel matching START and the first matching END after it, with its queue/stream,
start offset, duration and the idle gap on its stream.  Usage: trace_block.py DIR START END [NTH]"""
import glob
import re
import sqlite3
import sys


def main():
    d, start, end = sys.argv[1], sys.argv[2], sys.argv[3]
    nth = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    db = glob.glob(d + '/**/*.db', recursive=True)[0]
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    ks = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
    kd = [t for t in tabs if t.startswith('rocpd_kernel_dispatch')][0]
    rows = list(c.execute(f'select s.display_name, d.start, d.end, d.queue_id, d.grid_size_x, d.workgroup_size_x '
                          f'from {kd} d join {ks} s on d.kernel_id = s.id order by d.start'))

    def short(n):
        n = n.replace('(anonymous namespace)::', '').replace('void ', '')
        return re.sub(r'\(.*', '', n)[:48]
    starts = [i for i, r in enumerate(rows) if re.search(start, r[0])]
    i0 = starts[nth]
    i1 = next((i for i in range(i0, len(rows)) if re.search(end, rows[i][0])), len(rows) - 1)
    t0 = rows[i0][1]
    last = {}
    for i in range(i0, i1 + 1):
        n, s, e, q, g, w = rows[i]
        gap = (s - last[q]) / 1e3 if q in last else 0.0
        last[q] = e
        print(f'{(s - t0) / 1e3:9.1f} q{q} dur {(e - s) / 1e3:8.1f} gap {gap:7.1f} wg {g // max(w, 1):6d} {short(n)}')
    print('window us', (rows[i1][2] - t0) / 1e3)


main()
