"""Main-stream occupancy of one writeSog step from a rocprofv3 kernel trace (sqlite): the queue
that runs the SH k-means' sweeps is the main stream; between the NTH dispatch matching START and
the next matching END it sums that queue's kernel time and its idle gaps, and lists the largest
gaps with the kernels on either side (host round trips, waits on side streams).
Usage: stream_gaps.py DIR START|#INDEX END [NTH] [TOP]"""
import glob
import re
import sqlite3
import sys


def main():
    d, start, end = sys.argv[1], sys.argv[2], sys.argv[3]
    nth = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    top = int(sys.argv[5]) if len(sys.argv) > 5 else 25
    db = glob.glob(d + '/**/*.db', recursive=True)[0]
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    ks = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
    kd = [t for t in tabs if t.startswith('rocpd_kernel_dispatch')][0]
    rows = list(c.execute(f'select s.display_name, d.start, d.end, d.queue_id from {kd} d join {ks} s '
                          f'on d.kernel_id = s.id order by d.start'))

    def short(n):
        n = n.replace('(anonymous namespace)::', '').replace('void ', '')
        return re.sub(r'\(.*', '', n.replace('(anonymous namespace)::', ''))[:44]
    # START '#I': the dispatch at index I of the trace (what a step-boundary search printed)
    i0 = int(start[1:]) if start.startswith('#') else [i for i, r in enumerate(rows) if re.search(start, r[0])][nth]
    i1 = next((i for i in range(i0 + 1, len(rows)) if re.search(end, rows[i][0])), len(rows) - 1)
    win = rows[i0:i1 + 1]
    mq = next(r[3] for r in win if 'k_sweep<3, 0>' in r[0])
    main_q = [r for r in win if r[3] == mq]
    t0, t1 = win[0][1], win[-1][2]
    busy = sum(e - s for _, s, e, _ in main_q)
    sweep = sum(e - s for n, s, e, _ in main_q if 'k_sweep<3, 0>' in n)
    gaps = []
    for a, b in zip(main_q, main_q[1:]):
        g = b[1] - a[2]
        if g > 0:
            gaps.append((g, short(a[0]), short(b[0]), (a[2] - t0) / 1e3))
    print(f'window {(t1 - t0) / 1e6:.2f} ms; main queue q{mq}: {len(main_q)} kernels, busy {busy / 1e6:.2f} ms '
          f'(sweep {sweep / 1e6:.2f}, other {(busy - sweep) / 1e6:.2f}), idle {sum(g for g, *_ in gaps) / 1e6:.2f} ms '
          f'({len(gaps)} gaps; before its first kernel {(main_q[0][1] - t0) / 1e6:.2f} ms)')
    byk = {}
    for n, s, e, _ in main_q:
        if 'k_sweep<3, 0>' in n:
            continue
        k = short(n)
        byk[k] = byk.get(k, 0) + (e - s)
    print('main-queue kernels other than the sweep (ms):')
    for k, v in sorted(byk.items(), key=lambda x: -x[1])[:top]:
        print(f'  {v / 1e6:7.3f}  {k}')
    print(f'largest idle gaps on the main queue (us, at ms into the window):')
    for g, a, b, at in sorted(gaps, reverse=True)[:top]:
        print(f'  {g / 1e3:8.1f}  at {at:8.2f}  {a} -> {b}')
    pairs = {}
    for g, a, b, _ in gaps:
        pairs.setdefault((a, b), [0, 0])
        pairs[(a, b)][0] += g
        pairs[(a, b)][1] += 1
    print('idle by (before -> after) pair (ms, count):')
    for (a, b), (g, n) in sorted(pairs.items(), key=lambda x: -x[1][0])[:top]:
        print(f'  {g / 1e6:7.3f} x{n:4d}  {a} -> {b}')


main()
