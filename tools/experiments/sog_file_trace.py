#!/usr/bin/env python3
"""st_dev_sog_file against st_dev_sog at 10M SH-3, alternated (3 reps each after a warm-up), wall
clock per call; meant to run under rocprofv3 --kernel-trace so the sweeps of the two can be
compared (where the streamed archive's early entries slow the step)."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
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
    ta = time.perf_counter()
    if os.path.exists(path):  # the previous rep's file, truncated apart (what os.open(O_TRUNC) costs)
        os.close(os.open(path, os.O_WRONLY | os.O_TRUNC))
    t0 = time.perf_counter()
    ctx.dev_sog_file(cols, 10, draws, tex, path)
    t1 = time.perf_counter()
    print(f'  truncate of the previous file {1e3 * (t0 - ta):.1f} ms', flush=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ctx.dev_sog(cols, 10, draws, tex)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(f'rep {rep}: sog_file {1e3 * (t1 - t0):.1f} ms, sog step {1e3 * (t3 - t2):.1f} ms', flush=True)
os.remove(path)
os.rmdir(d)
