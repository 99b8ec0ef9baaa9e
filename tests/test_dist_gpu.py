"""Multi-process writeSog on the GPU: two or four ranks (uneven shards) on cuda:0 over gloo,
and the RCCL code path at world size 1;
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


def _table(n, seed, C=15):
    rng = np.random.default_rng(seed)
    cols = {}
    cube = rng.random(n) < 0.05
    for a, off in zip('xyz', (1.0, -2.0, 3.0)):
        cols[a] = np.where(cube, off + rng.random(n) * 1e-3, rng.normal(0, 10, n)).astype(np.float32)
    for i in range(3):
        cols[f'f_dc_{i}'] = rng.normal(0, 1, n).astype(np.float32)
    for i in range(3 * C):
        cols[f'f_rest_{i}'] = (rng.normal(0, 0.1, n)).astype(np.float32)
    cols['opacity'] = rng.normal(0, 2, n).astype(np.float32)
    for i in range(3):
        cols[f'scale_{i}'] = (rng.random(n) * 5 - 7).astype(np.float32)
    for i in range(4):
        cols[f'rot_{i}'] = rng.normal(0, 1, n).astype(np.float32)
    return cols


def _rank(rank, world, backend, port, n, seed, iters, q, C=15, empty=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)  # before the process group: RCCL binds the rank to this device
    dist.init_process_group(backend, rank=rank, world_size=world)
    import splat_hip as sh
    import splat_dist
    full = _table(n, seed, C)
    cuts = {1: [0, n], 3: [0, n // 5, n * 3 // 5, n], 2: [0, n * 3 // 7, n], 4: [0, n // 7, n * 3 // 7, n * 6 // 7, n]}[world]  # uneven shards
    if empty:  # rank 0 holds no rows
        cuts = [0, 0] + cuts[2:]
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


def _collect(q, procs, count, timeout=600):
    """count results from the rank processes; fails at once when a rank dies (the others would
    wait in a collective until gloo's timeout)"""
    import queue
    import time
    out, t0 = [], time.time()
    while len(out) < count:
        try:
            out.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.time() - t0 > timeout:
                for p in procs:
                    if p.is_alive():
                        p.kill()
                raise AssertionError(f'rank process failed (exit codes {[p.exitcode for p in procs]})')
    return out


def _adversarial_1d(n, seed):
    """three columns whose cluster sums defeat the order-free certificate: values over 15
    decades (tiny members under large sums: replay candidates, and past CAND_MAX the
    sequential chain), zeros and -0"""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(3):
        u = rng.random(n)
        v = rng.normal(0, 1, n)
        v = np.where(u < 0.3, v * 1e-9, v)
        v = np.where((u >= 0.7) & (u < 0.9), v * 1e3, v)
        v = np.where(u >= 0.9, np.sign(v) * rng.uniform(1e5, 1e6, n), v)
        v[rng.random(n) < 0.01] = 0.0
        v[rng.random(n) < 0.01] = -0.0
        out.append(v.astype(np.float32))
    return out


def _c1d_rank(rank, world, port, n, seed, iters, q, cap):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    if cap is not None:
        os.environ['ST_REPLAY_CAP'] = str(cap)
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import splat_hip as sh
    import splat_dist
    full = _adversarial_1d(n, seed)
    cuts = [0] + [n * (r + 1) * (r + 2) // (world * (world + 1)) for r in range(world)]  # uneven shards
    lo, hi = cuts[rank], cuts[rank + 1]
    cols = [torch.from_numpy(c[lo:hi].copy()).to(dev) for c in full]
    draws = np.random.default_rng(seed + 1).random(1 << 16)
    ctx = sh.Context(0)
    ops = splat_dist.HipOps(ctx, dev)
    comm = splat_dist.Comm()
    shard = splat_dist.Shard(comm, hi - lo)
    cb, lab8, used = splat_dist.cluster1d(ops, comm, shard, cols, iters, draws)
    torch.cuda.synchronize()
    q.put(dict(rank=rank, cb=cb.cpu().numpy(), lab=lab8.cpu().numpy().reshape(3, hi - lo), used=used, lo=lo, hi=hi))
    dist.destroy_process_group()
    ctx.close()


def _single_c1d(q, n, seed, iters, cap):
    if cap is not None:
        os.environ['ST_REPLAY_CAP'] = str(cap)
    import splat_hip as sh
    dev = torch.device('cuda', 0)
    ctx = sh.Context(0)
    ctx.bind_torch_stream(dev)  # before the inputs are made: they are ordered on the same stream
    full = _adversarial_1d(n, seed)
    cols = [torch.from_numpy(c).to(dev) for c in full]
    cb = torch.empty(256, dtype=torch.float32, device=dev)
    lab = torch.empty(3 * n, dtype=torch.uint8, device=dev)
    draws = np.random.default_rng(seed + 1).random(1 << 16)
    used = ctx.dev_cluster1d(cols, iters, draws, cb, lab)
    torch.cuda.synchronize()
    q.put(dict(cb=cb.cpu().numpy(), lab=lab.cpu().numpy().reshape(3, n), used=used))
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize('world,cap', [(1, None), (3, None), (3, 0)])
def test_dist_cluster1d_adversarial_matches_single_device(world, cap):
    """cluster1d over sharded columns (segments = rank x column) where 1-D cluster sums are
    uncertified: the chunked replay from each segment's running start must give the
    single-device codebook and labels bit for bit.  cap = 0 (ST_REPLAY_CAP) sends every
    uncertified sum down the sequential chain instead, on both sides.  The single-device
    reference result is computed in its own process under the same cap."""
    import torch.multiprocessing as mp
    n, seed, iters = 90000, 11, 4
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    mctx = mp.get_context('spawn')
    q = mctx.Queue()
    procs = [mctx.Process(target=_c1d_rank, args=(r, world, port, n, seed, iters, q, cap)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(_collect(q, procs, world), key=lambda r: r['rank'])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    p = mctx.Process(target=_single_c1d, args=(q, n, seed, iters, cap))
    p.start()
    one = _collect(q, [p], 1)[0]
    p.join(timeout=120)
    assert p.exitcode == 0
    for r in res:
        assert r['used'] == one['used']
        assert np.array_equal(r['cb'].view(np.uint32), one['cb'].view(np.uint32))
        assert np.array_equal(r['lab'], one['lab'][:, r['lo']:r['hi']])


@pytest.mark.gpu
@pytest.mark.parametrize('backend,world,C,empty', [('gloo', 2, 15, False), ('gloo', 4, 15, False),
                                                   ('nccl', 1, 15, False), ('gloo', 2, 0, False),
                                                   ('gloo', 3, 3, False), ('gloo', 2, 8, False),
                                                   ('gloo', 3, 15, True)])
def test_multi_rank_write_sog_matches_single_device(backend, world, C, empty):
    """gloo: 2 to 4 ranks sharing cuda:0.  nccl: RCCL refuses two ranks on one GPU, so the
    RCCL leg runs the same sharded code path at world size 1 (device-tensor collectives,
    every dtype / reduce op the 8-GPU job issues).  C: SH coefficients per channel (bands
    3, 0, 1, 2; write-sog.ts:296).  empty: rank 0 holds no rows."""
    import torch.multiprocessing as mp
    import splat_hip as sh
    n, seed, iters = 24000, 5, 3
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    mctx = mp.get_context('spawn')
    q = mctx.Queue()
    procs = [mctx.Process(target=_rank, args=(r, world, backend, port, n, seed, iters, q, C, empty))
             for r in range(world)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 1)[0]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0

    dev = torch.device('cuda', 0)
    ctx = sh.Context(0)
    ctx.bind_torch_stream(dev)  # before the inputs are made: they are ordered on the same stream
    full = _table(n, seed, C)
    cols = {k: torch.from_numpy(v).to(dev) for k, v in full.items()}
    W, H, pal, cw, ch = sh.sog_geometry(n, C)
    u8 = dict(device=dev, dtype=torch.uint8)
    keys = ('means_l', 'means_u', 'quats', 'scales', 'sh0') + (('shN_labels',) if C else ())
    tex = {k: torch.zeros(W * H * 4, **u8) for k in keys}
    if C:
        tex['shN_centroids'] = torch.zeros(cw * ch * 4, **u8)
    draws = np.random.default_rng(seed + 1).random(1 << 20)
    meta, used = ctx.dev_sog(cols, iters, draws, tex)
    torch.cuda.synchronize()
    assert res['used'] == used
    for k, v in tex.items():
        assert np.array_equal(res['tex'][k], v.cpu().numpy()), k
    m = res['meta']
    assert list(m['means_min']) == list(meta.means_min) and list(m['means_max']) == list(meta.means_max)
    assert set(res['tex']) == set(tex)
    for k in ('scales_codebook', 'sh0_codebook') + (('shn_codebook',) if C else ()):
        assert np.array_equal(np.asarray(m[k]).view(np.uint32), np.array(getattr(meta, k), np.float32).view(np.uint32)), k
    # identical .sog archive
    assert ctx.dev_sog_bundle(meta, n, tex, 0x6a2b, 0x58b1) == res['zip']
    ctx.close()
