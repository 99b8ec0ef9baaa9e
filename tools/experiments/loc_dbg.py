#!/usr/bin/env python3
"""debug aid (tools/experiments/locality_probe.py's sequence at a small size): assigns of the
same points in the original order and grouped by tile-half, against centroids after one update"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                'splat-transform_amd', 'py'))
import torch  # noqa: E402

import splat_hip as sh  # noqa: E402

n = int(sys.argv[1])
d, k = 45, int(sys.argv[2])
dev = torch.device('cuda', 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
X = torch.randn(d, n, generator=g, device=dev) * 0.1
ctx = sh.Context(0)
ctx.bind_torch_stream(dev)


def assign(Xc, cen, tag):
    cols = [Xc[j].contiguous() for j in range(d)]
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    print(f'{tag}: start', flush=True)
    t0 = time.time()
    ctx.dev_kmeans_prepare(cols)
    torch.cuda.synchronize()
    t1 = time.time()
    ctx.dev_kmeans_assign(cols, k, cen, lab)
    torch.cuda.synchronize()
    t2 = time.time()
    print(f'{tag}: prepare {t1 - t0:.3f} s assign {t2 - t1:.3f} s', flush=True)
    return lab.long()


def update(Xc, lab):
    s = torch.zeros(d, k, dtype=torch.float64, device=dev)
    s.index_add_(1, lab, Xc.double())
    cnt = torch.bincount(lab, minlength=k)
    print('empty clusters', int((cnt == 0).sum()), flush=True)
    return (s / cnt.clamp(min=1)).float().contiguous()


rows = torch.randperm(n, generator=g, device=dev)[:k]
C0 = X[:, rows].contiguous()
L0 = assign(X, C0, 'orig C0')
C1 = update(X, L0)
L1 = assign(X, C1, 'orig C1')
code = (L1 >> 5) * 2 + ((L1 >> 2) & 1)
p = torch.argsort(code, stable=True)
print('perm min', int(p.min()), 'max', int(p.max()), 'distinct', int(torch.unique(p).numel()), flush=True)
Xp = X[:, p].contiguous()
print('absmax X', float(X.abs().max()), 'Xp', float(Xp.abs().max()), 'finite', bool(torch.isfinite(Xp).all()), flush=True)
ps = p.sort().values
print('perm is a permutation', bool((ps == torch.arange(n, device=dev)).all()), flush=True)
assign(Xp, C1, 'grouped C1')
