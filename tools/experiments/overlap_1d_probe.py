#!/usr/bin/env python3
"""Is the latency-bound 1-D block free when it runs beside the SH sweep?  The SH palette k-means
(10M x 45, K = 65,536, 2 iterations) on one context and the colours' cluster1d (3 x 10M values,
10 iterations) on another, alone and together (two host threads, two streams)."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import splat_hip as sh  # noqa: E402

dev = torch.device('cuda', 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
n = 10_000_000
X = [torch.randn(n, generator=g, device=dev) * 0.1 for _ in range(45)]
C = [torch.randn(n, generator=g, device=dev) for _ in range(3)]
torch.cuda.synchronize()
a, b = sh.Context(0), sh.Context(0)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
a.set_stream(sa.cuda_stream)
b.set_stream(sb.cuda_stream)
cen = torch.empty(45 * 65536, device=dev)
lab = torch.empty(n, dtype=torch.int32, device=dev)
cb = torch.empty(256, device=dev)
lab8 = torch.empty(3 * n, dtype=torch.uint8, device=dev)
draws = np.random.default_rng(1).random(65536 * 8)


def sh_km():
    a.dev_kmeans(X, 65536, 2, draws, cen, lab)
    a.synchronize()


def one_d():
    b.dev_cluster1d(C, 10, draws, cb, lab8)
    b.synchronize()


def t(fn):
    t0 = time.perf_counter()
    fn()
    return (time.perf_counter() - t0) * 1e3


for f in (sh_km, one_d):
    f()  # warm
for rep in range(3):
    ta, tb = t(sh_km), t(one_d)
    th = threading.Thread(target=one_d)
    t0 = time.perf_counter()
    th.start()
    sh_km()
    th.join()
    tt = (time.perf_counter() - t0) * 1e3
    print(f'SH k-means alone {ta:.1f} ms, 1-D alone {tb:.1f} ms, together {tt:.1f} ms '
          f'(saved {ta + tb - tt:.1f} of {tb:.1f})', flush=True)
