"""debug: splat_dist kmeans / cluster1d (world 1, gloo) vs the single-device entry points"""
import os, sys, socket
import numpy as np, torch, torch.distributed as dist
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'splat-transform_amd', 'py'), os.path.join(ROOT, 'tests')]
import splat_hip as sh, splat_dist
from test_dist_gpu import _table
s = socket.socket(); s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
dist.init_process_group('gloo', rank=0, world_size=1)
dev = torch.device('cuda', 0)
n = 24000
full = _table(n, 5)
cols = {k: torch.from_numpy(v).to(dev) for k, v in full.items()}
draws = np.random.default_rng(6).random(1 << 20)
ctx = sh.Context(0)
ops = splat_dist.HipOps(ctx, dev)
comm = splat_dist.Comm()
shard = splat_dist.Shard(comm, n)
for name, cl in (('scales', [cols[f'scale_{i}'] for i in range(3)]), ('fdc', [cols[f'f_dc_{i}'] for i in range(3)])):
    cb, lab8, used = splat_dist.cluster1d(ops, comm, shard, cl, 3, draws)
    cb2 = torch.empty(256, device=dev); lab2 = torch.empty(3 * n, dtype=torch.uint8, device=dev)
    used2 = ctx.dev_cluster1d(cl, 3, draws, cb2, lab2)
    torch.cuda.synchronize()
    print(name, 'used', used, used2, 'cb eq', torch.equal(cb, cb2), 'lab eq', torch.equal(lab8, lab2))
pts = [cols[f'f_rest_{i}'] for i in range(45)]
for k in (1024, 16384):
    cen, lab, used = splat_dist.kmeans(ops, comm, shard, pts, k, 3, draws)
    cen2 = torch.empty(45 * k, device=dev); lab2 = torch.empty(n, dtype=torch.int32, device=dev)
    used2 = ctx.dev_kmeans(pts, k, 3, draws, cen2, lab2)
    torch.cuda.synchronize()
    print('kmeans', k, 'used', used, used2, 'cen eq', torch.equal(cen.reshape(-1), cen2), 'lab eq', torch.equal(lab, lab2),
          'nlab diff', (lab != lab2).sum().item())
