#!/usr/bin/env python3
"""cluster1d (write-sog.ts:56-99) timing on 3 columns of n values with few distinct values
(quantised inputs: empty clusters, re-seeds onto existing values, coinciding centroids, ties).
    python tools/k1_dup_bench.py [n] [distinct]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
import numpy as np
import torch

import splat_hip as sh

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
distinct = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dev = torch.device('cuda', 0)
g = torch.Generator(device=dev)
g.manual_seed(3)
cols = [torch.randn(n, generator=g, device=dev) for _ in range(3)]
if distinct:
    for c in cols:
        c.copy_(torch.floor(torch.rand(n, generator=g, device=dev) * distinct) * 0.25 - 5)
ctx = sh.Context(0)
ctx.bind_torch_stream(dev)
draws = np.random.default_rng(1).random(1 << 16)
cen = torch.empty(256, device=dev)
lab = torch.empty(3 * n, dtype=torch.int32, device=dev)
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    used = ctx.dev_cluster1d(cols, 10, draws, cen, lab)
    torch.cuda.synchronize()
    print(f'cluster1d n={n} x 3 distinct={distinct or "all"}: {(time.perf_counter() - t0) * 1e3:.1f} ms, draws {used}',
          flush=True)
