#!/usr/bin/env python3
"""Summarise tools/pmc_paths.sh (FETCH_SIZE / WRITE_SIZE passes over tools/bench_paths.py at 10M
and over one headline bench step) into profiles/<round>/pmc_paths.json: per HBM-bound kernel, the
HBM bytes per launch the counters report against the kernel's algorithmic bytes per launch.
    python tools/pmc_paths.py [round]

Counter units and corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads, so the
streamed read bytes are 2 x FETCH_SIZE; WRITE_SIZE is exact for streaming stores.  Other access
widths are uncalibrated: for kernels whose reads are random gathers both the raw and the doubled
figure are listed."""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1] if len(sys.argv) > 1 else 'r04'
G = os.path.join(ROOT, 'gpurun_out')
N = 10_000_000
HBM = 8.0e12


def short(k):
    m = re.search(r'(k_\w+(?:<[^()]*?>)?)\(', k)
    return m.group(1) if m else k[:60]


def load(run, counter):
    f = glob.glob(os.path.join(G, f'pmcp_{run}_{counter}', '**', '*counter_collection.csv'), recursive=True)[0]
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for r in csv.DictReader(open(f)):
        if r['Counter_Name'] != counter:
            continue
        a = agg[(short(r['Kernel_Name']), int(r['Grid_Size']))]
        a[0] += 1
        a[1] += float(r['Counter_Value']) * 1024.0
        a[2] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
    return agg


# (run, kernel, grid size) -> (algorithmic read bytes, written bytes, read pattern, what) per launch at 10M
SPEC = [
    ('paths', 'k_transform<15, true, true, true>', 2097152, 220 * N, 220 * N, 'stream',
     'transform -r 0,45,0 (a3/a4): x y z, rot_0..3, scale_0..2, f_rest_0..44 read and written (55 f32)'),
    ('paths', 'k_finite_flags4', 2097152, 248 * N, 4 * N, 'stream',
     'filterNaN flags (a6): 62 f32 columns read, one flag word written'),
    ('paths', 'k_gather_cols4', 2097152, 252 * N, 248 * N, 'stream (index ascending)',
     'filterNaN row gather (a6): kept index + 62 columns read, 62 columns written'),
    ('paths', 'k_ext<float>', 624384, 12 * N, 0, 'stream', 'Morton level-0 extents (a8): x y z read'),
    ('paths', 'k_keys0<float>', 624384, 16 * N, 4 * N, 'stream',
     'Morton level-0 keys (a8): idx + x y z read, 30-bit key written (+ first-digit tile counts)'),
    ('paths', 'k_rs_hist<unsigned int>', 624384, 4 * N, 0, 'stream', 'Morton radix pass histogram (a8): keys read'),
    ('paths', 'k_rs_scatter<unsigned int>', 624384, 8 * N, 8 * N, 'stream read, digit-run writes',
     'Morton radix pass scatter (a8): (key, idx) read and written'),
    ('paths', 'k_pack_rows<45, false>', 9990144, 236 * N, 96 * N, 'stream',
     'chunk pack, rows (a9/a10): 14 member + 45 SH f32 columns read, one 96-B packed row written'),
    ('paths', 'k_pack_rows_chunk<45>', 2497536, 100 * N, 61 * N + 72 * (N // 256), 'random 96-B row gathers',
     'chunk pack, chunks (a9/a10): Morton order + the 96-B packed row gathered, vertex 16 B + SH 45 B + chunk 72 B/256'),
    ('step', 'k_kd1_assign_acc<true>', 234496, 4 * 3 * N, 3 * N, 'stream',
     'cluster1d assign (a16) over the 30M scale / colour values: value read, byte label written'),
]


def main():
    out = {'what': 'HBM traffic of the HBM-bound kernels: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes '
                   '(kernel trace only) over tools/bench_paths.py 10000000 (config 3 stages) and one headline '
                   'bench step (tools/pmc_paths.sh); per-launch averages',
           'correction': 'gfx950 FETCH_SIZE counts half the bytes of 16-B/lane streaming reads (MI355X_MICROARCH.md): '
                         'read bytes = 2 x FETCH_SIZE for streamed reads; random gathers are uncalibrated (raw and '
                         'doubled both listed)',
           'kernels': {}}
    data = {run: (load(run, 'FETCH_SIZE'), load(run, 'WRITE_SIZE')) for run in ('paths', 'step')}
    for run, k, grid, rd, wr, pattern, what in SPEC:
        f, w = data[run]
        if (k, grid) not in f or (k, grid) not in w:
            out['kernels'][k] = {'missing': True}
            continue
        fc, fb, ft = f[(k, grid)]
        wc, wb, wt = w[(k, grid)]
        fetch, write = fb / fc, wb / wc
        secs = (ft + wt) / (fc + wc)  # launch time under counter collection (kernels serialised)
        traffic = 2 * fetch + write
        out['kernels'][k] = {
            'what': what, 'read_pattern': pattern, 'launches': fc,
            'alg_read_bytes': rd, 'alg_write_bytes': wr, 'alg_bytes': rd + wr,
            'FETCH_SIZE_bytes': fetch, 'WRITE_SIZE_bytes': write,
            'hbm_bytes_corrected': traffic, 'traffic_over_alg': traffic / (rd + wr),
            'read_raw_over_alg': fetch / rd if rd else None, 'write_over_alg': write / wr if wr else None,
            'launch_ms_under_pmc': secs * 1e3,
            'alg_frac_hbm_under_pmc': (rd + wr) / secs / HBM,
        }
    os.makedirs(os.path.join(ROOT, 'profiles', rnd), exist_ok=True)
    dst = os.path.join(ROOT, 'profiles', rnd, 'pmc_paths.json')
    json.dump(out, open(dst, 'w'), indent=1)
    for k, v in out['kernels'].items():
        if 'missing' in v:
            print(f'{k:36s} missing')
            continue
        print(f"{k:36s} alg {v['alg_bytes'] / 1e9:6.3f} GB  fetch(raw) {v['FETCH_SIZE_bytes'] / 1e9:6.3f}  "
              f"write {v['WRITE_SIZE_bytes'] / 1e9:6.3f}  corrected/alg {v['traffic_over_alg']:.2f}  "
              f"{v['launch_ms_under_pmc']:.3f} ms  alg {v['alg_frac_hbm_under_pmc']:.2f} of HBM")


if __name__ == '__main__':
    main()
