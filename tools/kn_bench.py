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
ap.add_argument('--dist', default='gauss', choices=['gauss', 't3'],
                help='gauss: iid N(0, 0.1^2) (the bench); t3: heavy-tailed and correlated, Student-t nu=3 x 0.1 '
                     'through a fixed mixing matrix (what trained scenes carry)')
a = ap.parse_args()
dev = torch.device('cuda', 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
if a.dist == 'gauss':
    cols = [torch.randn(a.n, generator=g, device=dev) * 0.1 for _ in range(a.d)]
else:
    # t_3 = N(0,1) / sqrt(chi2_3 / 3), then x = 0.1 t M^T with M = I + 0.5 G / sqrt(d) (G fixed N(0,1))
    gm = torch.Generator(device='cpu')
    gm.manual_seed(3)
    M = (torch.eye(a.d) + 0.5 * torch.randn(a.d, a.d, generator=gm) / a.d ** 0.5).to(dev)
    cols = [None] * a.d
    for s in range(0, a.n, 1 << 21):
        e = min(a.n, s + (1 << 21))
        z = torch.randn(e - s, a.d, generator=g, device=dev)
        chi = (torch.randn(e - s, 3, generator=g, device=dev) ** 2).sum(1, keepdim=True)
        x = (z / torch.sqrt(chi / 3)) @ M.T * 0.1
        for j in range(a.d):
            cols[j] = x[:, j].contiguous() if cols[j] is None else torch.cat([cols[j], x[:, j]])
    cols = [c.float().contiguous() for c in cols]
if a.zero_frac > 0:  # exact duplicates: identical init rows -> identical centroids -> exact ties
    z = torch.rand(a.n, generator=g, device=dev) < a.zero_frac
    for c in cols:
        c[z] = 0.0
ctx = sh.Context(0)
ctx.bind_torch_stream(dev)
cen = torch.empty(a.d * a.k, device=dev)
lab = torch.empty(a.n, dtype=torch.int32, device=dev)
draws = np.random.default_rng(1).random(a.k * (a.iters + 2) * 2)
ctx.set_profiling(True)
import time
t0 = time.perf_counter()
used = ctx.dev_kmeans(cols, a.k, a.iters, draws, cen, lab)
torch.cuda.synchronize()
print(f'kmeans total {(time.perf_counter() - t0) * 1e3:.1f} ms ({a.iters} iters, zero-frac {a.zero_frac}, dist {a.dist}, n {a.n})')
for name in ('kn.sweep', 'kn.collect', 'kn.fixrow', 'kn.fixpair', 'kn.exact', 'kn.groups', 'kn.ties', 'kn.sumnd'):
    ms, cnt = ctx.kernel_stats(name)
    print(f'{name}: {ms / max(cnt, 1):.3f} ms x {cnt}')
import hashlib
print('result sha256', hashlib.sha256(cen.cpu().numpy().tobytes() + lab.cpu().numpy().tobytes()).hexdigest()[:16],
      'draws used', used)
print('assign classification', ctx.kmeans_stats())
