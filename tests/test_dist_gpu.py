"""Multi-process writeSog on the GPU: two or four ranks (uneven shards) on cuda:0 over gloo,
product step API (splat_dist.HipOps), must reproduce the single-device st_dev_sog of
the whole table bit for bit.  (On an 8-GPU node the same code runs one rank per GPU
over RCCL; bench.py --gpus N.)"""
import os
import socket
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'splat-transform_amd', 'py'), os.path.join(ROOT, 'oracle')):
    if p not in sys.path:
        sys.path.insert(0, p)

NAMES = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] + \
    ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3']


def _table(n, seed):
    rng = np.random.default_rng(seed)
    cols = {}
    cube = rng.random(n) < 0.05
    for a, off in zip('xyz', (1.0, -2.0, 3.0)):
        cols[a] = np.where(cube, off + rng.random(n) * 1e-3, rng.normal(0, 10, n)).astype(np.float32)
    for i in range(3):
        cols[f'f_dc_{i}'] = rng.normal(0, 1, n).astype(np.float32)
    for i in range(45):
        cols[f'f_rest_{i}'] = (rng.normal(0, 0.1, n)).astype(np.float32)
    cols['opacity'] = rng.normal(0, 2, n).astype(np.float32)
    for i in range(3):
        cols[f'scale_{i}'] = (rng.random(n) * 5 - 7).astype(np.float32)
    for i in range(4):
        cols[f'rot_{i}'] = rng.normal(0, 1, n).astype(np.float32)
    return cols


def _rank(rank, world, port, n, seed, iters, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import splat_hip as sh
    import splat_dist
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    full = _table(n, seed)
    cuts = {2: [0, n * 3 // 7, n], 4: [0, n // 7, n * 3 // 7, n * 6 // 7, n]}[world]  # uneven shards
    lo, hi = cuts[rank], cuts[rank + 1]
    cols = {k: torch.from_numpy(v[lo:hi].copy()).to(dev) for k, v in full.items()}
    draws = np.random.default_rng(seed + 1).random(1 << 20)
    ctx = sh.Context(0)
    ops = splat_dist.HipOps(ctx, dev)
    comm = splat_dist.Comm()
    tex, meta, used = splat_dist.write_sog(ops, comm, cols, iters, draws)
    torch.cuda.synchronize()
    if rank == 0:
        # the .sog archive of the gathered textures (WebP + CRC + ZIP on rank 0's device)
        z = ctx.dev_sog_bundle(splat_dist.meta_struct(meta), meta['count'], tex, 0x6a2b, 0x58b1)
        q.put(dict(tex={k: v.cpu().numpy() for k, v in tex.items()}, meta=meta, used=used, zip=z))
    dist.destroy_process_group()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 4])
def test_multi_rank_write_sog_matches_single_device(world):
    import torch.multiprocessing as mp
    import splat_hip as sh
    n, seed, iters = 24000, 5, 3
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    mctx = mp.get_context('spawn')
    q = mctx.Queue()
    procs = [mctx.Process(target=_rank, args=(r, world, port, n, seed, iters, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0

    dev = torch.device('cuda', 0)
    full = _table(n, seed)
    cols = {k: torch.from_numpy(v).to(dev) for k, v in full.items()}
    W, H, pal, cw, ch = sh.sog_geometry(n, 15)
    u8 = dict(device=dev, dtype=torch.uint8)
    tex = {k: torch.zeros(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
    tex['shN_centroids'] = torch.zeros(cw * ch * 4, **u8)
    draws = np.random.default_rng(seed + 1).random(1 << 20)
    ctx = sh.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    meta, used = ctx.dev_sog(cols, iters, draws, tex)
    torch.cuda.synchronize()
    assert res['used'] == used
    for k, v in tex.items():
        assert np.array_equal(res['tex'][k], v.cpu().numpy()), k
    m = res['meta']
    assert list(m['means_min']) == list(meta.means_min) and list(m['means_max']) == list(meta.means_max)
    for k in ('scales_codebook', 'sh0_codebook', 'shn_codebook'):
        assert np.array_equal(np.asarray(m[k]).view(np.uint32), np.array(getattr(meta, k), np.float32).view(np.uint32)), k
    # identical .sog archive
    assert ctx.dev_sog_bundle(meta, n, tex, 0x6a2b, 0x58b1) == res['zip']
    ctx.close()
