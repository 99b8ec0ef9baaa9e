#!/usr/bin/env python3
"""How many Math.random draws the two cluster1d of writeSog take on the bench's table (re-seeds of
empty clusters, write-sog.ts:245-268 -> k-means.ts:164-192): the draws the SH palette k-means
starts after.  python tools/k1_draws.py [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
sys.path.insert(0, ROOT)

import numpy as np
import torch

import bench
import splat_hip as sh

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
dev = torch.device('cuda', 0)
ctx = sh.Context(0)
ctx.bind_torch_stream(dev)
draws = np.random.default_rng(42).random(2 * 65536 * 12)
for name, make in (('gauss', lambda: bench.synth_table(n, bench.SEED, dev)),
                   ('realistic', lambda: bench.realistic_table(n, bench.SEED + 77, dev))):
    t = make()
    out = {}
    for grp, cols in (('scales', ['scale_0', 'scale_1', 'scale_2']), ('colours', ['f_dc_0', 'f_dc_1', 'f_dc_2'])):
        cen = torch.empty(256, device=dev)
        lab = torch.empty(3 * n, dtype=torch.uint8, device=dev)
        used = ctx.dev_cluster1d([t[k] for k in cols], 10, draws, cen, lab)
        out[grp] = used
    print(name, n, out, flush=True)
