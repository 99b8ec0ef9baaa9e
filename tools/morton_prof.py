#!/usr/bin/env python3
"""Morton ordering (generateOrdering) of 10M Gaussian device columns, repeated: run under
rocprofv3 --kernel-trace --stats for the per-kernel split of one config-3 Morton stage."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
import torch

import splat_hip as sh

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
kind = sys.argv[2] if len(sys.argv) > 2 else 'gauss'  # gauss | clustered | clumps | grid
dev = torch.device('cuda', 0)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
ctx = sh.Context(0)
ctx.set_stream(stream.cuda_stream)
g = torch.Generator(device=dev)
g.manual_seed(7)
x, y, z = (torch.randn(n, generator=g, device=dev) for _ in range(3))
if kind == 'clustered':
    # half the splats in 64 tight blobs (1e-5 of the extent): deep equal-key runs, many segments
    m = torch.rand(n, generator=g, device=dev) < 0.5
    centre = torch.randint(0, 64, (n,), generator=g, device=dev).float()
    for a in (x, y, z):
        a[m] = centre[m] * 0.05 + a[m] * 1e-5
elif kind == 'clumps':
    # 80% of the splats in 20,000 small clumps (~400 each): one deeper level of many segments
    m = torch.rand(n, generator=g, device=dev) < 0.8
    cid = torch.randint(0, 20000, (n,), generator=g, device=dev)
    cx, cy, cz = (torch.randn(20000, generator=g, device=dev) for _ in range(3))
    for a, cc in ((x, cx), (y, cy), (z, cz)):
        a[m] = cc[cid[m]] + a[m] * 1e-6
elif kind == 'grid':
    # coordinates on a coarse lattice: many exactly equal points (runs that never split)
    for a in (x, y, z):
        a.copy_(torch.round(a * 4) / 4)
order = torch.empty(n, dtype=torch.int32, device=dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
best = 1e9
for r in range(12):
    order.copy_(torch.arange(n, dtype=torch.int32, device=dev))
    ev[0].record(stream)
    ctx.dev_morton_order(x, y, z, order)
    ev[1].record(stream)
    stream.synchronize()
    if r >= 2:
        best = min(best, ev[0].elapsed_time(ev[1]))
print(f'morton n={n} {kind}: {best * 1e3:.1f} us per call (best of 10)')
