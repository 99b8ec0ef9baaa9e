#!/usr/bin/env python3
"""N-D k-means micro-bench (SH palette shape): n points x D=45, K=65536, a few iterations.
Used under rocprofv3 --pmc to read the assign sweep's counters without the whole SOG step."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))

import numpy as np
import torch

import splat_hip as sh

ap = argparse.ArgumentParser()
ap.add_argument('--n', type=int, default=2_000_000)
ap.add_argument('--d', type=int, default=45)
ap.add_argument('--k', type=int, default=65536)
ap.add_argument('--iters', type=int, default=2)
ap.add_argument('--zero-frac', type=float, default=0.0, help='fraction of all-zero rows (duplicate points)')
a = ap.parse_args()
dev = torch.device('cuda', 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
cols = [torch.randn(a.n, generator=g, device=dev) * 0.1 for _ in range(a.d)]
if a.zero_frac > 0:  # exact duplicates: identical init rows -> identical centroids -> exact ties
    z = torch.rand(a.n, generator=g, device=dev) < a.zero_frac
    for c in cols:
        c[z] = 0.0
ctx = sh.Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
cen = torch.empty(a.d * a.k, device=dev)
lab = torch.empty(a.n, dtype=torch.int32, device=dev)
draws = np.random.default_rng(1).random(a.k * (a.iters + 2) * 2)
ctx.set_profiling(True)
import time
t0 = time.perf_counter()
used = ctx.dev_kmeans(cols, a.k, a.iters, draws, cen, lab)
torch.cuda.synchronize()
print(f'kmeans total {(time.perf_counter() - t0) * 1e3:.1f} ms ({a.iters} iters, zero-frac {a.zero_frac})')
for name in ('kn.sweep', 'kn.collect', 'kn.fixrow', 'kn.exact', 'kn.groups', 'kn.ties', 'kn.sumnd'):
    ms, cnt = ctx.kernel_stats(name)
    print(f'{name}: {ms / max(cnt, 1):.3f} ms x {cnt}')
