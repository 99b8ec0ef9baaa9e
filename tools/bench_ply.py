#!/usr/bin/env python3
"""PLY ingest and compressed-PLY decode at the bench shape (10M SH-3 splats, 248 B rows).

  ingest       st_dev_ply_read: file (page cache) -> pinned 32 MiB chunks -> HBM -> k_ply_cols
               end-to-end GB/s and the transpose kernel's HBM rate (2 x 248 B per row)
  decompress   k_decompress + k_decompress_sh: read 16 B (+ chunk rows) + 45 B, write 59 x 4 B per splat

Writes gpurun_out/ply.json."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))

import numpy as np
import torch

import splat_hip as sh


def main(n=10_000_000):
    dev = torch.device('cuda', 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx = sh.Context(0)
    ctx.set_stream(s.cuda_stream)
    names = ['x', 'y', 'z', 'nx', 'ny', 'nz', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] + \
        ['opacity', 'scale_0', 'scale_1', 'scale_2'] + [f'rot_{i}' for i in range(4)]
    head = ('ply\nformat binary_little_endian 1.0\n' + f'element vertex {n}\n' +
            ''.join(f'property float {k}\n' for k in names) + 'end_header\n').encode()
    d = os.environ.get('TMPDIR', '/tmp')
    path = os.path.join(d, 'st_bench.ply')
    rng = np.random.default_rng(1)
    with open(path, 'wb') as f:
        f.write(head)
        step = 1_000_000
        for a in range(0, n, step):
            m = min(step, n - a)
            f.write(rng.standard_normal((m, len(names)), dtype=np.float32).tobytes())
    size = os.path.getsize(path)
    out = {'splats': n, 'file_bytes': size}
    try:
        ctx.read_ply_dev(path)  # warm: workspace, pinned chunks
        ctx.set_profiling(True)
        ctx.reset_kernel_stats()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            _, els = ctx.read_ply_dev(path)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        kms, kc = ctx.kernel_stats('ply.cols')
        out['ingest'] = {'wall_ms': wall * 1e3, 'file_GBps': size / wall / 1e9,
                         'transpose_ms': kms / reps, 'transpose_launches': kc // reps,
                         'transpose_hbm_GBps': 2 * 248 * n / (kms / reps / 1e3) / 1e9}
        cols = dict(els)['vertex']
    finally:
        os.remove(path)
    # decompress: pack the table on the device first (Morton + chunk pack), then decode
    tab = {k: cols[k] for k in names if not k.startswith('n')}
    order = torch.arange(n, dtype=torch.int32, device=dev)
    ctx.dev_morton_order(tab['x'], tab['y'], tab['z'], order)
    chunk = torch.empty((n + 255) // 256 * 18, device=dev)
    vertex = torch.empty(n * 4, dtype=torch.int32, device=dev)
    shb = torch.empty(n * 45, dtype=torch.uint8, device=dev)
    ctx.dev_pack_compressed(tab, order, chunk, vertex, shb)
    ch = chunk.view(-1, 18)
    chd = {k: ch[:, i].contiguous() for i, k in enumerate(sh.CHUNK_COLS)}
    vx = vertex.view(-1, 4)
    vxd = {k: vx[:, i].contiguous() for i, k in enumerate(sh.VERTEX_COLS)}
    sv = shb.view(n, 45)
    shd = [sv[:, i].contiguous() for i in range(45)]
    dec = {k: torch.empty(n, device=dev) for k in sh.DECOMP_COLS + [f'f_rest_{i}' for i in range(45)]}
    ctx.dev_decompress_ply(chd, vxd, shd, dec)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(s)
    for _ in range(5):
        ctx.dev_decompress_ply(chd, vxd, shd, dec)
    ev[1].record(s)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / 5
    alg = 16 + 45 + 59 * 4  # bytes per splat (chunk rows amortised)
    out['decompress'] = {'ms': ms, 'Msplats_per_s': n / (ms / 1e3) / 1e6, 'alg_bytes_per_splat': alg,
                         'hbm_GBps': alg * n / (ms / 1e3) / 1e9}
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(ROOT, 'gpurun_out', 'ply.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000)
