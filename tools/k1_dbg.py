"""cluster1d on N(0,1) colours at the bench size, ST_DEBUG counts of uncertified / fallback clusters"""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'splat-transform_amd', 'py'))
import splat_hip as sh
dev = torch.device('cuda', 0)
g = torch.Generator(device=dev); g.manual_seed(1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
cols = [torch.randn(n, generator=g, device=dev) for _ in range(3)]
ctx = sh.Context(0)
ctx.set_profiling(True)
cb = torch.empty(256, device=dev); lab = torch.empty(3 * n, dtype=torch.uint8, device=dev)
ctx.dev_cluster1d(cols, 10, np.random.default_rng(1).random(4096), cb, lab)
torch.cuda.synchronize()
ms, cnt = ctx.kernel_stats('k1.sum')
print('k1.sum avg ms', ms / cnt, cnt)
