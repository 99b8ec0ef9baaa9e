"""debug: 1-D splat_dist kmeans step by step vs st_dev_kmeans (world 1)"""
import os, sys, socket
import numpy as np, torch, torch.distributed as dist
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'splat-transform_amd', 'py'), os.path.join(ROOT, 'tests')]
import splat_hip as sh, splat_dist
s = socket.socket(); s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
dist.init_process_group('gloo', rank=0, world_size=1)
dev = torch.device('cuda', 0)
n = 6000
x = torch.from_numpy((np.random.default_rng(3).random(n) * 5 - 7).astype(np.float32)).to(dev)
draws = np.random.default_rng(6).random(1 << 16)
ctx = sh.Context(0)
ops = splat_dist.HipOps(ctx, dev)
comm = splat_dist.Comm()
shard = splat_dist.Shard(comm, n)
for iters in (0, 1, 2):
    cen, lab, used = splat_dist.kmeans(ops, comm, shard, [x], 256, iters, draws)
    cen2 = torch.empty(256, device=dev); lab2 = torch.zeros(n, dtype=torch.int32, device=dev)
    used2 = ctx.dev_kmeans([x], 256, iters, draws, cen2, lab2)
    torch.cuda.synchronize()
    c1, c2 = cen.reshape(-1).cpu().numpy(), cen2.cpu().numpy()
    bad = np.nonzero(c1.view(np.uint32) != c2.view(np.uint32))[0]
    print('iters', iters, 'used', used, used2, 'cen diff idx', bad[:8], c1[bad[:3]], c2[bad[:3]],
          'lab diff', (lab != lab2).sum().item() if iters else '-')
# one assign on the same centroids
cen2 = torch.empty(256, device=dev); lab2 = torch.zeros(n, dtype=torch.int32, device=dev)
ctx.dev_kmeans([x], 256, 1, draws, cen2, lab2)
lab3 = torch.zeros(n, dtype=torch.int32, device=dev)
c0 = torch.empty(256, device=dev); ctx.dev_kmeans([x], 256, 0, draws, c0, lab3)
ops.prepare([x]); ops.assign([x], 256, c0.reshape(1, 256).contiguous(), lab3)
torch.cuda.synchronize()
print('assign on init centroids: label diff', (lab3 != lab2).sum().item())
sums, sabs, emin, counts = ops.partials([x], 1, 256, lab3)
torch.cuda.synchronize()
l = lab3.cpu().numpy(); xv = x.cpu().numpy()
ref_counts = np.bincount(l, minlength=256)
print('counts ok', np.array_equal(counts.cpu().numpy()[0], ref_counts), counts.cpu().numpy()[0][:8], ref_counts[:8])
ref_sums = np.array([np.float64(xv[l == c].astype(np.float64).sum()) for c in range(256)])
print('sums close', np.allclose(sums.cpu().numpy()[0, 0], ref_sums), sums.cpu().numpy()[0, 0][:4], ref_sums[:4])
print('emin', emin.cpu().numpy()[0, 0][:8], 'sabs', sabs.cpu().numpy()[0, 0][:4])
