#!/usr/bin/env python3
"""How much would the N-D fix-up gain if the points were stored grouped by their tile-half?
One exact assign (st_dev_kmeans_assign: sweep + k_fixrow_b) of n x 45 points against the
centroids after one update, (a) in the original order, (b) permuted by the codes of those same
centroids (the best case), (c) permuted by the previous iteration's codes (one iteration stale,
what a reorder between iterations would give).  Prints kn.fixrow per call.
    python tools/experiments/locality_probe.py [n]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
import torch  # noqa: E402

import splat_hip as sh  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
d, k = 45, 65536
dev = torch.device('cuda', 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
X = torch.randn(d, n, generator=g, device=dev) * 0.1
ctx = sh.Context(0)
ctx.bind_torch_stream(dev)


def assign(Xc, cen):
    t0 = time.time()
    cols = [Xc[j].contiguous() for j in range(d)]
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.dev_kmeans_prepare(cols)
    ctx.dev_kmeans_assign(cols, k, cen, lab)  # warm
    ctx.set_profiling(True)
    ctx.reset_kernel_stats()
    for _ in range(3):
        ctx.dev_kmeans_assign(cols, k, cen, lab)
    torch.cuda.synchronize()
    ms, cnt = ctx.kernel_stats('kn.fixrow')
    sw, scnt = ctx.kernel_stats('kn.sweep')
    ctx.set_profiling(False)
    print(f'  assign x4: {time.time() - t0:.1f} s', flush=True)
    return lab.long(), ms / cnt, sw / scnt


def update(Xc, lab):
    s = torch.zeros(d, k, dtype=torch.float64, device=dev)
    s.index_add_(1, lab, Xc.double())
    cnt = torch.bincount(lab, minlength=k).clamp(min=1)
    return (s / cnt).float().contiguous()


def code(lab):
    return (lab >> 5) * 2 + ((lab >> 2) & 1)


rows = torch.randperm(n, generator=g, device=dev)[:k]
C0 = X[:, rows].contiguous()
L0, f0, s0 = assign(X, C0)
C1 = update(X, L0)
L1, f1, s1 = assign(X, C1)
print(f'original order, centroids C1: fixrow {f1:.3f} ms, sweep {s1:.2f} ms', flush=True)
p = torch.argsort(code(L1), stable=True)
Xp = X[:, p].contiguous()
_, fb, _ = assign(Xp, C1)
print(f'grouped by C1 codes (best case): fixrow {fb:.3f} ms', flush=True)
C2 = update(X, L1)
L2, f2, _ = assign(X, C2)
_, fs, _ = assign(Xp, C2)
print(f'C2 in original order: fixrow {f2:.3f} ms; grouped by the previous (C1) codes: {fs:.3f} ms', flush=True)
same = (code(L2) == code(L1)).float().mean().item()
print(f'points keeping their tile-half C1 -> C2: {same:.3f}', flush=True)
