"""How many points could skip the SH assign between k-means iterations?

Measures, on the bench's synthetic SH data (10M x 45, K = 65,536), the fraction of points
whose label provably cannot change at assign t+2 under three classic bounds, given the
exact distances of assign t+1:
  hamerly: d1 + drift[a] < d2 - max(drift)
  yinyang: d1 + drift[a] < min over groups g of (d_g - max drift in g), G groups of
           consecutive centroid indices (d_g = nearest distance within g, own centroid
           excluded)
  elkan:   d1 + drift[a] < min over c != a of (d_c - drift[c])   (the best single-centroid bound)
Distances in f64 on a point subsample (torch on the GPU).  Research probe only: it reads
centroids produced by the library's own k-means (st_dev_kmeans, iters = t and t + 1)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
import splat_hip as sh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=10_000_000)
    ap.add_argument('--k', type=int, default=65536)
    ap.add_argument('--sample', type=int, default=20000)
    ap.add_argument('--iters', default='1,2,4,8')
    ap.add_argument('--groups', type=int, default=1024)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = sh.Context(0)
    ctx.set_stream(stream.cuda_stream)
    g = torch.Generator(device=dev)
    g.manual_seed(1002)
    D, K, n = 45, args.k, args.n
    cols = [torch.randn(n, generator=g, device=dev) * 0.1 for _ in range(D)]
    draws = np.random.default_rng(42).random(2 * K * 12)
    pts = torch.stack(cols, 1)
    sel = torch.randperm(n, generator=g, device=dev)[:args.sample]
    P = pts[sel].double()
    del pts
    out = {}
    for t in [int(x) for x in args.iters.split(',')]:
        cen = []
        for it in (t, t + 1):
            c = torch.empty(D * K, device=dev)
            lab = torch.empty(n, dtype=torch.int32, device=dev)
            ctx.dev_kmeans(cols, K, it, draws, c, lab)
            torch.cuda.synchronize()
            cen.append(c.view(D, K).t().double())
        C0, C1 = cen  # centroids used by assign t+1 and assign t+2
        drift = (C1 - C0).norm(dim=1)
        dmax = drift.max()
        stats = dict(drift_max=float(dmax), drift_med=float(drift.median()),
                     drift_p99=float(drift.quantile(0.99)))
        ham = yin = elk = 0
        gap, d1s = [], []
        for b in range(0, P.shape[0], 2000):
            p = P[b:b + 2000]
            d = torch.cdist(p, C0)  # f64 distances to the centroids of assign t+1
            d1, a = d.min(1)
            d[torch.arange(p.shape[0], device=dev), a] = float('inf')
            d2 = d.min(1).values
            gap.append(d2 - d1)
            d1s.append(d1)
            u = d1 + drift[a]
            ham += int((u < d2 - dmax).sum())
            G = args.groups
            dg = d.view(p.shape[0], G, K // G).min(2).values
            gmax = drift.view(G, K // G).max(1).values
            yin += int((u < (dg - gmax[None, :]).min(1).values).sum())
            d -= drift[None, :]
            elk += int((u < d.min(1).values).sum())
            del d, dg
        m = P.shape[0]
        gap = torch.cat(gap)
        stats.update(gap_med=float(gap.median()), d1_med=float(torch.cat(d1s).median()), hamerly=ham / m,
                     yinyang=yin / m, elkan=elk / m)
        out[t] = stats
        print(t, json.dumps(stats), flush=True)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, 'gpurun_out', 'prune_probe.json'), 'w'), indent=1)


if __name__ == '__main__':
    main()
