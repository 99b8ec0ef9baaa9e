#!/usr/bin/env python3
"""HBM-bound stages of the path at BASELINE config 3 (10M SH-3 splats, -r 0,45,0,
--filterNaN -> .compressed.ply), each timed with HIP events on the library's stream
and priced against the 8 TB/s HBM peak with its ALGORITHMIC bytes per splat:

  transform (a3/a4)       440 B  read+write x,y,z, rot_0..3, scale_0..2, f_rest_0..44 (f32)
  filter_finite (a6)      252 B  read 62 columns + write the kept index
  permute_rows (a6)       496 B  gather 62 columns + write them
  morton_order (a8)        92 B  SURVEY 8d: extents 12 + keys 12+4 + 4-pass 8-bit LSD on 8-B pairs 64
                                 (+ morton_order_clumped: the same over clumped positions, priced
                                 the same way; not part of the config-3 pipeline)
  pack_compressed (a9/10) 301 B  gather 14+45 columns, write vertex 16 B + sh 45 B + chunk

Prints one JSON object (also written to gpurun_out/paths.json)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))

import torch

import splat_hip as sh

HBM = 8.0e12


def main(n=10_000_000, reps=5):
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = sh.Context(0)
    ctx.set_stream(stream.cuda_stream)
    out = measure(ctx, stream, dev, n, reps)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(ROOT, 'gpurun_out', 'paths.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


def measure(ctx, stream, dev, n=10_000_000, reps=5):
    """the stage table and the whole config-3 pipeline; ctx runs on `stream`"""
    g = torch.Generator(device=dev)
    g.manual_seed(1003)
    names = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] + \
        ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3', 'nx', 'ny', 'nz']
    cols = {k: torch.randn(n, generator=g, device=dev) for k in names}
    # 0.1% of rows get a NaN/Inf in a random column
    bad = torch.randperm(n, generator=g, device=dev)[: n // 1000]
    which = torch.randint(0, len(names), (bad.numel(),), generator=g, device=dev)
    for j, k in enumerate(names):
        rows = bad[which == j]
        cols[k][rows[: rows.numel() // 2]] = float('nan')
        cols[k][rows[rows.numel() // 2:]] = float('inf')
    torch.cuda.synchronize()

    def timed(fn):
        fn()  # warm
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        best = []
        for _ in range(reps):
            ev[0].record(stream)
            fn()
            ev[1].record(stream)
            torch.cuda.synchronize()
            best.append(ev[0].elapsed_time(ev[1]))
        return sorted(best)[len(best) // 2]

    out = {'splats': n, 'hbm_peak_GBps': HBM / 1e9, 'stages': {}}

    def report(name, ms, bytes_per_splat, rows=n):
        gbs = bytes_per_splat * rows / (ms / 1e3) / 1e9
        out['stages'][name] = {'ms': ms, 'alg_bytes_per_splat': bytes_per_splat, 'achieved_GBps': gbs,
                               'frac_hbm': gbs / (HBM / 1e9)}

    params = sh.action_params('rotate', (0, 45, 0))
    report('transform', timed(lambda: ctx.dev_transform(cols, params)), 440)
    idx = torch.empty(n, dtype=torch.int32, device=dev)
    kept = [0]

    def filt():
        kept[0] = ctx.dev_filter_finite(cols, idx)
    report('filter_finite', timed(filt), 62 * 4 + 4)
    m = kept[0]
    dst = {k: torch.empty(m, device=dev) for k in names}
    report('permute_rows', timed(lambda: ctx.dev_permute_rows(cols, idx, m, dst)), 62 * 8, rows=m)
    order = torch.empty(m, dtype=torch.int32, device=dev)

    def morton():
        order.copy_(torch.arange(m, dtype=torch.int32, device=dev))
        ctx.dev_morton_order(dst['x'], dst['y'], dst['z'], order)
    report('morton_order', timed(morton), 92, rows=m)
    # the same ordering over clumped positions (80% of the splats in 20,000 clumps of ~400 at
    # one point each): the recursion levels real scenes reach (ordering.ts:90-104), not in config3
    gc = torch.Generator(device=dev)
    gc.manual_seed(1004)
    cid = torch.randint(0, 20000, (m,), generator=gc, device=dev)
    inclump = torch.rand(m, generator=gc, device=dev) < 0.8
    cxyz = []
    for a in ('x', 'y', 'z'):
        cc = torch.randn(20000, generator=gc, device=dev)
        cxyz.append(torch.where(inclump, cc[cid] + dst[a] * 1e-6, dst[a]).contiguous())

    def morton_clumped():
        order.copy_(torch.arange(m, dtype=torch.int32, device=dev))
        ctx.dev_morton_order(cxyz[0], cxyz[1], cxyz[2], order)
    report('morton_order_clumped', timed(morton_clumped), 92, rows=m)
    out['stages']['morton_order_clumped']['what'] = ('not a config-3 stage: positions in 20,000 clumps, '
                                                      'so the ordering recurses (deeper levels)')
    del cxyz, cid, inclump
    chunk = torch.empty((m + 255) // 256 * 18, device=dev)
    vertex = torch.empty(m * 4, dtype=torch.int32, device=dev)
    shb = torch.empty(m * 45, dtype=torch.uint8, device=dev)
    pack_cols = {k: v for k, v in dst.items() if not k.startswith('n')}
    report('pack_compressed', timed(lambda: ctx.dev_pack_compressed(pack_cols, order, chunk, vertex, shb)), 301,
           rows=m)

    # the whole config-3 device pipeline (inputs resident, outputs in HBM)
    def pipeline():
        ctx.dev_transform(cols, params)
        mm = ctx.dev_filter_finite(cols, idx)
        ctx.dev_permute_rows(cols, idx, mm, dst)
        morton()
        ctx.dev_pack_compressed(pack_cols, order, chunk, vertex, shb)
    ms = timed(pipeline)
    out['config3'] = {'ms': ms, 'Msplats_per_s': n / (ms / 1e3) / 1e6, 'kept': m}

    # the same chain as ONE library call (st_dev_compressed_ply: processDataTable's actions, then
    # writeCompressedPly's ordering + chunk loop), and its host form (st_compressed_ply: the table
    # uploaded from pageable host arrays, the packed arrays downloaded -- the Node CLI's path,
    # PCIe-inclusive)
    acts = [{'kind': 'rotate', 'value': (0, 45, 0)}, {'kind': 'filterNaN'}]
    items = list(cols.items())
    dchunk = torch.empty((n + 255) // 256 * 18, device=dev)
    dvertex = torch.empty(n * 4, dtype=torch.int32, device=dev)
    dsh = torch.empty(n * 45, dtype=torch.uint8, device=dev)
    ms1 = timed(lambda: ctx.dev_compressed_ply(items, acts, dchunk, dvertex, dsh))
    out['config3_one_call'] = {'ms': ms1, 'Msplats_per_s': n / (ms1 / 1e3) / 1e6,
                               'what': 'st_dev_compressed_ply (rotate 0,45,0 + filterNaN + Morton + chunk pack)'}
    host = [(k, v.cpu().numpy()) for k, v in items]
    ref = ctx.compressed_ply(host, acts)  # warm (workspace)
    t0 = time.perf_counter()
    for _ in range(2):
        ctx.compressed_ply(host, acts)
    ms2 = (time.perf_counter() - t0) / 2 * 1e3
    out['config3_host_one_call'] = {'ms': ms2, 'Msplats_per_s': n / (ms2 / 1e3) / 1e6,
                                    'what': 'st_compressed_ply from pageable host columns (62 x 4 B/splat up, '
                                            '16 + 45 B/splat + chunks down): the PCIe-inclusive rate of the Node path'}
    out['config3_file'] = file_path(ctx, host, acts, ref)
    return out


CHUNK_PROPS = ['min_x', 'min_y', 'min_z', 'max_x', 'max_y', 'max_z', 'min_scale_x', 'min_scale_y', 'min_scale_z',
               'max_scale_x', 'max_scale_y', 'max_scale_z', 'min_r', 'min_g', 'min_b', 'max_r', 'max_g', 'max_b']
VERTEX_PROPS = ['packed_position', 'packed_rotation', 'packed_scale', 'packed_color']


def compressed_ply_header(m, C, version='0.10.1'):
    """write-compressed-ply.ts:35-54's header text"""
    lines = ['ply', 'format binary_little_endian 1.0', f'comment Generated by splat-transform {version}',
             f'element chunk {(m + 255) // 256}'] + [f'property float {p}' for p in CHUNK_PROPS] + \
        [f'element vertex {m}'] + [f'property uint {p}' for p in VERTEX_PROPS]
    if C:
        lines += [f'element sh {m}'] + [f'property uchar f_rest_{i}' for i in range(3 * C)]
    return ('\n'.join(lines + ['end_header']) + '\n').encode()


def file_path(ctx, host, acts, ref, reps=3):
    """the CLI's `in.ply -r 0,45,0 --filterNaN out.compressed.ply` from the file to the file:
    st_ply_compressed_ply_file (page cache -> pinned -> HBM, the chain, the arrays written at their
    offsets as they leave HBM), each rep into a FRESH output file (the reference's CLI writes a new
    'wx' file, index.ts:107-112); and the same job through the Node drop-in host
    (tools/bench_node_c3.js: compressPlyFile(inHandle, outHandle, actions) over the addon).  The
    table is written once as a binary PLY (untimed); every output file must equal the reference's
    header + the host one-call arrays byte for byte"""
    import hashlib
    import shutil
    import subprocess
    import tempfile

    import numpy as np
    n = len(host[0][1])
    m, chunk, vertex, shb = ref
    C = shb.size // max(1, 3 * m)
    want = compressed_ply_header(m, C) + chunk.tobytes() + vertex.tobytes() + shb.tobytes()
    want_sha = hashlib.sha256(want).hexdigest()
    d = tempfile.mkdtemp(prefix='st_c3_', dir=os.environ.get('TMPDIR', '/tmp'))
    src = os.path.join(d, 'in.ply')
    try:
        head = ('ply\nformat binary_little_endian 1.0\n' + f'element vertex {n}\n' +
                ''.join(f'property float {k}\n' for k, _ in host) + 'end_header\n').encode()
        with open(src, 'wb') as f:
            f.write(head)
            step = 1 << 22
            for a in range(0, n, step):
                f.write(np.stack([v[a:a + step] for _, v in host], 1).tobytes())
        times, same = [], True
        for r in range(reps + 1):  # rep 0 warms the page cache and the buffers
            dst = os.path.join(d, f'out{r}.compressed.ply')
            t0 = time.perf_counter()
            mm, CC, size = ctx.ply_compressed_ply_file(src, acts, dst)
            t1 = time.perf_counter()
            if r:
                times.append(t1 - t0)
            same = same and mm == m and CC == C and size == len(want) and \
                hashlib.sha256(open(dst, 'rb').read()).hexdigest() == want_sha
            os.remove(dst)
        ms = sorted(times)[len(times) // 2] * 1e3
        out = {'ms': ms, 'Msplats_per_s': n / (ms / 1e3) / 1e6, 'reps': reps, 'ply_bytes': os.path.getsize(src),
               'out_bytes': len(want), 'equals_host_one_call': same,
               'what': 'st_ply_compressed_ply_file: PLY file (page cache) -> HBM -> rotate + filterNaN + Morton + '
                       'chunk pack -> a fresh .compressed.ply written at offsets as the arrays leave HBM'}
        node = shutil.which('node')
        addon = os.path.join(ROOT, 'splat-transform_amd', 'napi', 'build', 'addon.node')
        if node and os.path.exists(addon):
            r = subprocess.run([node, os.path.join(ROOT, 'tools', 'bench_node_c3.js'), src, d, str(reps)],
                               capture_output=True, text=True, timeout=600)
            if os.environ.get('ST_DEBUG'):  # the addon's phase stamps
                sys.stderr.write(r.stderr)
            if r.returncode != 0:
                out['node_host'] = {'error': r.stderr[-2000:]}
            else:
                res = json.loads(r.stdout.strip().splitlines()[-1])
                nms = sorted(res['ms'])[len(res['ms']) // 2]
                out['node_host'] = {'ms': nms, 'Msplats_per_s': n / (nms / 1e3) / 1e6, 'reps': len(res['ms']),
                                    'split_ms': res.get('split'),
                                    'equals_host_one_call': all(h == want_sha for h in res['sha256']),
                                    'what': 'node tools/bench_node_c3.js: compressPlyFile(inHandle, outHandle '
                                            "('wx', fresh), [rotate 0,45,0, filterNaN]) over napi/addon.node"}
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000)
