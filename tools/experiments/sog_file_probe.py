#!/usr/bin/env python3
"""Where the streamed writeSog-to-file (st_dev_sog_file) spends its time at 10M SH-3 against the
separate calls (st_dev_sog, st_dev_sog_bundle_view, one write(2)): 3 reps each after a warm-up,
wall clock per call and the step's stage marks (ST_TIMING)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
os.environ['ST_TIMING'] = '1'
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import splat_hip as sh  # noqa: E402

n = 10_000_000
dev = torch.device('cuda', 0)
ctx = sh.Context(0)
ctx.bind_torch_stream(dev)
cols = bench.synth_table(n, 1002, dev)
W, H, pal, cw, ch = sh.sog_geometry(n, 15)
u8 = dict(device=dev, dtype=torch.uint8)
tex = {k: torch.empty(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
draws = np.random.default_rng(42).random(2 * 65536 * 12)
d = tempfile.mkdtemp(dir=os.environ.get('TMPDIR', '/tmp'))
path = os.path.join(d, 'out.sog')
for rep in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.dev_sog_file(cols, 10, draws, tex, path)
    t1 = time.perf_counter()
    st = json.loads(ctx.timings())
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    meta, _ = ctx.dev_sog(cols, 10, draws, tex)
    t3 = time.perf_counter()
    addr, size = ctx.dev_sog_bundle_view(meta, n, tex, 0, 0)
    t4 = time.perf_counter()
    with open(path + '.2', 'wb') as f:
        f.write((bench.ctypes_char_array(size)).from_address(addr))
    t5 = time.perf_counter()
    st2 = json.loads(ctx.timings())
    if rep:
        print(f'streamed {1e3 * (t1 - t0):.1f} ms | separate: step {1e3 * (t3 - t2):.1f} + bundle '
              f'{1e3 * (t4 - t3):.1f} + write {1e3 * (t5 - t4):.1f} = {1e3 * (t5 - t2):.1f} ms', flush=True)
        print('  streamed stages', {k: round(v, 1) for k, v in st.items() if isinstance(v, (int, float))}, flush=True)
        print('  separate stages', {k: round(v, 1) for k, v in st2.items() if isinstance(v, (int, float))}, flush=True)
os.remove(path)
os.remove(path + '.2')
os.rmdir(d)
