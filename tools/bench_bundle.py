#!/usr/bin/env python3
"""The .sog container stage at the bench shape (10M SH-3 splats): WebP lossless encode
of the seven textures + CRC-32 + ZIP (st_dev_sog_bundle), timed with HIP events per
kernel and end to end, beside libwebp (Pillow, 1 thread, lossless, method 4 -- what the
reference's WebPEncodeLosslessRGBA runs as wasm) on the same textures.

Algorithmic bytes per pixel of the encoder: predict reads 4 B (+ neighbours, L2) and
writes 4 B; hist reads 4 B; bits reads 4 B; emit reads 4 B and writes the stream.

Writes gpurun_out/bundle.json."""
import io
import json
import os
import sys
import time
import zipfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))

import numpy as np
import torch

import splat_hip as sh
from bench import synth_table


def main(n=10_000_000, reps=3, pil=True):
    dev = torch.device('cuda', 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx = sh.Context(0)
    ctx.set_stream(s.cuda_stream)
    cols = synth_table(n, 1002, dev)
    draws = np.random.default_rng(42).random(2 * 65536 * 12)
    W, H, pal, cw, ch = sh.sog_geometry(n, 15)
    u8 = dict(device=dev, dtype=torch.uint8)
    tex = {k: torch.empty(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
    tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
    meta, _ = ctx.dev_sog(cols, 10, draws, tex)
    torch.cuda.synchronize()
    z = ctx.dev_sog_bundle(meta, n, tex, 0, 0)  # warm (workspace + pinned archive allocation)
    ctx.set_profiling(True)
    ctx.reset_kernel_stats()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.dev_sog_bundle_view(meta, n, tex, 0, 0)  # archive lands in pinned host memory, no copy
    wall = (time.perf_counter() - t0) / reps
    kern = {}
    for k in ('webp.predict', 'webp.hist', 'webp.cache', 'webp.bits', 'webp.emit', 'crc32'):
        ms, cnt = ctx.kernel_stats(k)
        kern[k] = {'ms_per_bundle': ms / reps, 'launches_per_bundle': cnt // reps}
    ctx.set_profiling(False)
    zf = zipfile.ZipFile(io.BytesIO(z))
    entries = {i.filename: i.file_size for i in zf.infolist()}
    npix = {k: W * H for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
    npix['shN_centroids'] = cw * ch
    total_pix = sum(npix.values())
    dev_ms = sum(v['ms_per_bundle'] for v in kern.values())
    out = {'splats': n, 'texture': [W, H], 'shN_centroids': [cw, ch], 'pixels': total_pix,
           'bundle_wall_ms': wall * 1e3, 'device_kernel_ms': dev_ms, 'kernels': kern,
           'archive_bytes': len(z), 'entries': entries,
           'encoder_alg_bytes_per_pixel': 20,
           'encoder_achieved_GBps': 20 * total_pix / (dev_ms / 1e3) / 1e9}
    if pil:
        from PIL import Image
        ref = {}
        for name, key, (w, h) in [('means_l', 'means_l', (W, H)), ('means_u', 'means_u', (W, H)),
                                  ('quats', 'quats', (W, H)), ('scales', 'scales', (W, H)), ('sh0', 'sh0', (W, H)),
                                  ('shN_centroids', 'shN_centroids', (cw, ch)),
                                  ('shN_labels', 'shN_labels', (W, H))]:
            img = Image.fromarray(tex[key].cpu().numpy().reshape(h, w, 4), 'RGBA')
            b = io.BytesIO()
            t0 = time.perf_counter()
            img.save(b, 'WEBP', lossless=True, quality=70, method=4)
            dt = time.perf_counter() - t0
            ref[name + '.webp'] = {'bytes': len(b.getvalue()), 'ms': dt * 1e3,
                                   'ours_bytes': entries[name + '.webp']}
            print(name, ref[name + '.webp'], flush=True)
        out['libwebp_1thread'] = ref
        out['libwebp_total_ms'] = sum(v['ms'] for v in ref.values())
        out['libwebp_total_bytes'] = sum(v['bytes'] for v in ref.values())
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    if '--crops' in sys.argv:  # the first 256 rows of each texture, for encoder experiments on the host
        for key, (w, h) in [(k, (W, H)) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')] + \
                [('shN_centroids', (cw, ch))]:
            a = tex[key].cpu().numpy().reshape(h, w, 4)[:256]
            np.save(os.path.join(ROOT, 'gpurun_out', f'crop_{key}.npy'), a)
    with open(os.path.join(ROOT, 'gpurun_out', 'bundle.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000, pil='--no-pil' not in sys.argv)
