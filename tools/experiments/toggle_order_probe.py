#!/usr/bin/env python3
"""Does the order of the centroids change the sweep's time?  The sweep is power-limited and the
centroid fragments are the operand that changes from one MFMA to the next, so centroids ordered
so that neighbouring tiles are alike toggle fewer bits.  One prepare, then assigns of the same
n x 45 points against the same 65,536 centroids in several orders (labels are discarded: only
kn.sweep's time is read).
    python tools/experiments/toggle_order_probe.py [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
import torch  # noqa: E402

import splat_hip as sh  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
d, k = 45, 65536
dev = torch.device('cuda', 0)
ctx = sh.Context(0)
ctx.bind_torch_stream(dev)
g = torch.Generator(device=dev)
g.manual_seed(7)
X = torch.randn(d, n, generator=g, device=dev) * 0.1
cols = [X[j].contiguous() for j in range(d)]
lab = torch.empty(n, dtype=torch.int32, device=dev)
rows = torch.randperm(n, generator=g, device=dev)[:k]
C = X[:, rows].contiguous()
ctx.dev_kmeans_prepare(cols)


def sweep_ms(cen, reps=4):
    ctx.dev_kmeans_assign(cols, k, cen.contiguous(), lab)  # warm
    ctx.set_profiling(True)
    ctx.reset_kernel_stats()
    for _ in range(reps):
        ctx.dev_kmeans_assign(cols, k, cen.contiguous(), lab)
    torch.cuda.synchronize()
    ms, cnt = ctx.kernel_stats('kn.sweep')
    ctx.set_profiling(False)
    return ms / cnt


# principal direction of the centroids
Cc = C - C.mean(1, keepdim=True)
u = torch.linalg.svd(Cc.double(), full_matrices=False)[0][:, :3].float()
proj = u.t() @ Cc  # [3, k]
orders = {
    'random (draw order)': torch.arange(k, device=dev),
    'by coordinate 0': torch.argsort(C[0]),
    'by first principal component': torch.argsort(proj[0]),
}
# 3-D Morton of the first three principal components, 10 bits each
q = ((proj - proj.min(1, keepdim=True).values) / (proj.max(1, keepdim=True).values - proj.min(1, keepdim=True).values)
     * 1023).long().clamp(0, 1023)
code = torch.zeros(k, dtype=torch.long, device=dev)
for b in range(10):
    for a in range(3):
        code |= ((q[a] >> b) & 1) << (3 * b + a)
orders['Morton of 3 principal components'] = torch.argsort(code)
orders['random (draw order), again'] = torch.arange(k, device=dev)
for name, o in orders.items():
    print(f'{name:36s} sweep {sweep_ms(C[:, o]):.3f} ms per launch ({n} points)', flush=True)
