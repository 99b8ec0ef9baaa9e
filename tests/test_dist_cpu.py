"""Multi-GPU exchange logic on CPU: splat_dist's k-means / cluster1d with world_size 2
over gloo, per-rank steps by the oracle stand-in (tests/dist_oracle_ops.py), must equal
the single-process oracle bit for bit -- including uncertified sums (the
segment-ordered sequential chain) and empty-cluster re-seeds."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'splat-transform_amd', 'py'), os.path.join(ROOT, 'oracle'), os.path.dirname(__file__)):
    if p not in sys.path:
        sys.path.insert(0, p)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data(seed):
    rng = np.random.default_rng(seed)
    n, d = 420, 4
    x = rng.normal(0, 1, (d, n)).astype(np.float32)
    tiny = rng.random((d, n)) < 0.15          # wide exponent range: uncertified sums
    x[tiny] *= np.float32(1e-12)
    x[:, 200:260] = x[:, 199:200]             # duplicates: coincident centroids -> empty clusters
    return x


def _worker(rank, world, port, seed, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import oracle
    import splat_dist
    from dist_oracle_ops import OracleOps
    x = _data(seed)
    n = x.shape[1]
    cut = [0, 170, n] if world == 2 else None
    lo, hi = cut[rank], cut[rank + 1]
    comm = splat_dist.Comm()
    shard = splat_dist.Shard(comm, hi - lo)
    cols = [torch.from_numpy(x[j, lo:hi].copy()) for j in range(x.shape[0])]
    draws = oracle.mulberry32(seed, 4096)
    ops = OracleOps()
    cen, lab, used = splat_dist.kmeans(ops, comm, shard, cols, 40, 4, draws)
    labs = comm.allgather(lab)
    cb, lab8, used1 = splat_dist.cluster1d(ops, comm, shard, cols[:3], 3, draws)
    lab8s = comm.allgather(lab8.reshape(3, -1).t().contiguous())
    # fewer points than clusters (k-means.ts:139-144): the points are the centroids
    cen2, lab2, used2 = splat_dist.kmeans(ops, comm, shard, cols, n + 80, 2, draws)
    lab2s = comm.allgather(lab2)
    if rank == 0:
        out.put(dict(cen=cen.numpy().copy(), lab=torch.cat(labs).numpy().copy(), used=used,
                     cb=cb.numpy().copy(), lab8=torch.cat(lab8s).t().numpy().copy(), used1=used1,
                     cen2=cen2.numpy().copy(), lab2=torch.cat(lab2s).numpy().copy(), used2=used2))
    dist.destroy_process_group()


def test_distributed_kmeans_matches_single_process():
    import oracle
    seed = 11
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, seed, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x = _data(seed)
    draws = oracle.mulberry32(seed, 4096)
    rc, cen, lab, used = oracle.kmeans([x[j] for j in range(x.shape[0])], 40, 4, draws)
    assert rc == 0
    assert res['used'] == used and used > 40, 'empty-cluster re-seeds exercised'
    assert np.array_equal(res['lab'], lab)
    assert np.array_equal(res['cen'].view(np.uint32), cen.view(np.uint32))
    rc, cb, lab8, used1 = oracle.cluster1d([x[j] for j in range(3)], 3, draws)
    assert rc == 0 and res['used1'] == used1
    assert np.array_equal(res['cb'].view(np.uint32), cb.view(np.uint32))
    assert np.array_equal(res['lab8'], lab8)
    rc, cen2, lab2, used2 = oracle.kmeans([x[j] for j in range(x.shape[0])], x.shape[1] + 80, 2, draws)
    assert rc == 0 and res['used2'] == used2 == 0
    assert np.array_equal(res['lab2'], lab2) and np.array_equal(lab2, np.arange(x.shape[1]))
    assert np.array_equal(res['cen2'].view(np.uint32), cen2.view(np.uint32))


def _texel_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import splat_dist
    counts = [5, 9, 0][:world]  # uneven shards, one empty
    N, size = sum(counts), 20
    g = torch.Generator().manual_seed(3)
    pos_all = torch.randperm(N, generator=g).to(torch.int32)  # a global Morton order
    rows = torch.arange(N, dtype=torch.int32)
    comm = splat_dist.Comm()
    shard = splat_dist.Shard(comm, counts[rank])
    off = sum(counts[:rank])
    # texel of global row r: its index + 1 (non-zero), 4 bytes
    loc = {'a': (rows[off:off + counts[rank]] + 1).view(torch.uint8).clone(),
           'b': (rows[off:off + counts[rank]] * 7 + 3).view(torch.uint8).clone()}
    tex = splat_dist.gather_texels(comm, shard, loc, pos_all if rank == 0 else None, size)
    if rank == 0:
        out.put({k: v.view(torch.int32).numpy().copy() for k, v in tex.items()})
    else:
        assert tex is None
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_gather_texels_places_rows_at_morton_positions(world):
    """rank 0 assembles each texture from the ranks' row-ordered texels: global row r lands
    at pos_all[r], the rest of the W*H texture stays zero (splat_dist.gather_texels)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_texel_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    counts = [5, 9, 0][:world]
    N = sum(counts)
    pos_all = torch.randperm(N, generator=torch.Generator().manual_seed(3)).numpy()
    for key, f in (('a', lambda r: r + 1), ('b', lambda r: r * 7 + 3)):
        want = np.zeros(20, np.int32)
        want[pos_all] = f(np.arange(N))
        assert np.array_equal(res[key], want)
