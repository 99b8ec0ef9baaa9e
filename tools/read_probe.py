#!/usr/bin/env python3
"""readPly's host form (st_ply_read) at the bench shape (10M SH-3 splats, 248 B rows) into
pre-touched host columns (as the Node addon's pooled column blocks are) and into fresh ones,
with and without its host twins; beside it the device form (st_dev_ply_read).
  python tools/read_probe.py [n]      (run with ST_DEBUG=1 for the phase stamps)
Writes gpurun_out/read_probe.json."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
sys.path.insert(0, ROOT)

import numpy as np
import torch

import bench
import splat_hip as sh


def main(n=10_000_000):
    dev = torch.device('cuda', 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx = sh.Context(0)
    ctx.set_stream(s.cuda_stream)
    names = bench.PLY_ORDER
    head = ('ply\nformat binary_little_endian 1.0\n' + f'element vertex {n}\n' +
            ''.join(f'property float {k}\n' for k in names) + 'end_header\n').encode()
    path = os.path.join(os.environ.get('TMPDIR', '/tmp'), 'st_read_probe.ply')
    rng = np.random.default_rng(1)
    with open(path, 'wb') as f:
        f.write(head)
        for a in range(0, n, 1_000_000):
            f.write(rng.standard_normal((min(1_000_000, n - a), len(names)), dtype=np.float32).tobytes())
    cols = [np.ones(n, np.float32) for _ in names]  # touched once, reused (the addon's column pool)
    ptrs = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
    out = {'splats': n, 'file_bytes': os.path.getsize(path), 'runs': {}}
    fd = os.open(path, os.O_RDONLY)
    try:
        h = sh.PlyHeader()
        sh.check(sh.lib().st_ply_read_header(ctypes.c_int32(fd), ctypes.byref(h)))
        variants = [('default', {}), ('no_mirror', {'ST_HOST_MIRROR': '0'})]
        for rnd in range(2):
            for name, env in variants:
                os.environ.pop('ST_HOST_MIRROR', None)
                os.environ.update(env)
                ts = []
                for r in range(4):
                    t0 = time.perf_counter()
                    sh.check(sh.lib().st_ply_read(ctx.h, ctypes.c_int32(fd), ctypes.byref(h), ctypes.c_int32(0), ptrs))
                    ts.append((time.perf_counter() - t0) * 1e3)
                out['runs'].setdefault(name, []).extend(ts[1:])
                print(name, [f'{t:.1f}' for t in ts], file=sys.stderr, flush=True)
        os.environ.pop('ST_HOST_MIRROR', None)
        # fresh columns every rep (a CLI process's one read): new pages, faulted in by the read
        for name in ('fresh_columns',):
            ts = []
            for r in range(3):
                fresh = [np.empty(n, np.float32) for _ in names]
                fp = (ctypes.c_void_p * len(fresh))(*[c.ctypes.data for c in fresh])
                t0 = time.perf_counter()
                sh.check(sh.lib().st_ply_read(ctx.h, ctypes.c_int32(fd), ctypes.byref(h), ctypes.c_int32(0), fp))
                ts.append((time.perf_counter() - t0) * 1e3)
                del fresh, fp
            out['runs'][name] = ts
            print(name, [f'{t:.1f}' for t in ts], file=sys.stderr, flush=True)
        # the columns hold the file's values
        want = np.frombuffer(open(path, 'rb').read()[len(head):], np.float32).reshape(n, len(names))
        out['columns_equal_file'] = all(np.array_equal(cols[j], want[:, j]) for j in range(len(names)))
        del want
        ts = []
        for r in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.read_ply_dev(path)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        out['runs']['device_form'] = ts[1:]
        print('device form', [f'{t:.1f}' for t in ts], file=sys.stderr, flush=True)
    finally:
        os.close(fd)
        os.remove(path)
    out['median_ms'] = {k: float(np.median(v)) for k, v in out['runs'].items()}
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, 'gpurun_out', 'read_probe.json'), 'w'), indent=1)
    print(json.dumps(out['median_ms']))


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000)
