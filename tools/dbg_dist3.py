"""debug: manual 1-D distributed loop, 2 iterations, checking every intermediate"""
import os, sys, socket
import numpy as np, torch, torch.distributed as dist
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'splat-transform_amd', 'py')]
import splat_hip as sh, splat_dist
s = socket.socket(); s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
dist.init_process_group('gloo', rank=0, world_size=1)
dev = torch.device('cuda', 0)
n, k = 6000, 256
xv = (np.random.default_rng(3).random(n) * 5 - 7).astype(np.float32)
x = torch.from_numpy(xv).to(dev)
ctx = sh.Context(0)
ops = splat_dist.HipOps(ctx, dev)
c0 = torch.empty(k, device=dev); l0 = torch.zeros(n, dtype=torch.int32, device=dev)
ctx.dev_kmeans([x], k, 0, np.zeros(4), c0, l0)
cen = c0.reshape(1, k).clone()
ops.prepare([x])
lab = torch.empty(n, dtype=torch.int32, device=dev)
for it in range(2):
    ops.assign([x], k, cen, lab)
    sums, sabs, emin, counts = ops.partials([x], 1, k, lab)
    torch.cuda.synchronize()
    l = lab.cpu().numpy()
    ref = np.array([xv[l == c].astype(np.float64).sum() for c in range(k)])
    print(it, 'partials ok', np.allclose(sums.cpu().numpy()[0, 0], ref), 'counts', counts.cpu().numpy()[0][:4],
          'emin', emin.cpu().numpy()[0,0][:3])
    S, A = sums.sum(0), sabs.sum(0)
    E, C = emin.min(0).values.contiguous(), counts.sum(0, dtype=torch.int32)
    print('   S', S.shape, S.is_contiguous(), S.cpu().numpy()[0][:3], 'C', C.cpu().numpy()[:3], 'E', E.cpu().numpy()[0][:3])
    pend = ops.finish(1, k, S, A, E, C, cen)
    torch.cuda.synchronize()
    print('   pending', pend.numel(), 'cen', cen.cpu().numpy()[0][:4], 'ref', (ref / np.maximum(np.bincount(l, minlength=k), 1))[:4])
