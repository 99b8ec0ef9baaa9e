#!/usr/bin/env python3
"""1-D k-means micro-bench (cluster1d's shape: 3 x 10M values, K = 256, 10 iterations) on the
bench's synthetic scales (uniform in [-7, -2)) or colours (N(0, 1)); for rocprofv3 passes over
the 1-D kernels (tools/experiments/pmc_k1.sh)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__file__), '..', '..', 'splat-transform_amd', 'py'))
import splat_hip as sh  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else 'colours'
n = 30_000_000
dev = torch.device('cuda', 0)
g = torch.Generator(device=dev)
g.manual_seed(5)
x = (torch.rand(n, generator=g, device=dev) * 5 - 7) if kind == 'scales' else torch.randn(n, generator=g, device=dev)
ctx = sh.Context(0)
ctx.bind_torch_stream(dev)
cen = torch.empty(256, device=dev)
lab = torch.empty(n, dtype=torch.int32, device=dev)
draws = np.random.default_rng(1).random(256 * 12)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    used = ctx.dev_kmeans([x], 256, 10, draws, cen, lab)
    torch.cuda.synchronize()
    print(f'{kind}: 1-D k-means {1e3 * (time.perf_counter() - t0):.2f} ms (draws {used})', flush=True)
