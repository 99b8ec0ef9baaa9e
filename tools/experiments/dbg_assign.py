#!/usr/bin/env python3
"""One device assign (st_dev_kmeans_assign) against the oracle's KdTree assign on a golden
k-means case's points and final centroids; mismatching points with their exact distances
(debugging aid).  ST_DEBUG=1 adds the library's pair / ambiguous counts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ('splat-transform_amd/py', 'oracle', 'tests'):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import torch

import oracle
import splat_hip as sh
from golden_io import Golden

name = sys.argv[1] if len(sys.argv) > 1 else 'd3_grid'
g = Golden('kmeans')
case = [c for c in g.meta['cases'] if c['name'] == name][0]
d, k = case['d'], case['k']
cols = [g[f'{name}_p{j}'] for j in range(d)]
cen = np.stack([g[f'{name}_c{j}'] for j in range(d)])  # (d, k)
n = len(cols[0])
_, want = oracle.kmeans_assign(cols, cen)
dev = torch.device('cuda', 0)
ctx = sh.Context(0)
ctx.bind_torch_stream(dev)
tcols = [torch.from_numpy(c).to(dev) for c in cols]
tcen = torch.from_numpy(cen.reshape(-1).copy()).to(dev)
lab = torch.empty(n, dtype=torch.int32, device=dev)
ctx.dev_kmeans_prepare(tcols)
ctx.dev_kmeans_assign(tcols, k, tcen, lab)
torch.cuda.synchronize()
got = lab.cpu().numpy().astype(np.uint32)
bad = np.nonzero(got != want)[0]
print(f'{name}: {len(bad)} of {n} labels differ', flush=True)
P = np.stack(cols).astype(np.float64)
C = cen.astype(np.float64)
for i in bad[:6]:
    dist = ((C - P[:, i:i + 1]) ** 2).sum(0)
    o = np.argsort(dist, kind='stable')[:4]
    print(f'  point {i} {P[:, i]} want {want[i]} got {got[i]}; nearest {list(o)} dists {dist[o]}; '
          f'want-dist {dist[want[i]]} got-dist {dist[got[i]]}; cen want {C[:, want[i]]} got {C[:, got[i]]}')

# iteration by iteration: the first kmeans() iteration whose labels differ from the oracle's,
# then the device assign against the oracle's centroids before that iteration
draws = oracle.mulberry32(case['seed'], case['draws'] + 16)
for it in range(1, case['iters'] + 1):
    _, ocen, olab, _ = oracle.kmeans(cols, k, it, draws)
    gcen, glab, _ = ctx.kmeans(cols, k, it, draws)
    nb = int((np.asarray(glab) != olab).sum())
    print(f'iters={it}: labels differ at {nb} points', flush=True)
    if nb:
        _, pcen, _, _ = oracle.kmeans(cols, k, it - 1, draws) if it > 1 else (0, None, None, 0)
        if pcen is None:
            break
        pc = np.asarray(pcen, np.float32).reshape(d, k)
        _, want = oracle.kmeans_assign(cols, pc)
        tcen = torch.from_numpy(pc.reshape(-1).copy()).to(dev)
        ctx.dev_kmeans_prepare(tcols)
        ctx.dev_kmeans_assign(tcols, k, tcen, lab)
        torch.cuda.synchronize()
        got = lab.cpu().numpy().astype(np.uint32)
        bad = np.nonzero(got != want)[0]
        print(f'  assign on the centroids after {it - 1} iterations: {len(bad)} differ', flush=True)
        C = pc.astype(np.float64)
        for i in bad[:6]:
            dist = ((C - P[:, i:i + 1]) ** 2).sum(0)
            o = np.argsort(dist, kind='stable')[:4]
            print(f'  point {i} {P[:, i]} want {want[i]} got {got[i]}; nearest {list(o)} dists {dist[o]}; '
                  f'cen want {C[:, want[i]]} got {C[:, got[i]]}')
        break
