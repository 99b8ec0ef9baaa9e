"""World 8 -- the N of the driver's first RCCL run -- rehearsed as eight rank processes on one GPU
over the library's host shared-memory transport (st_comm_init_host), the calls and the program
order of the 8-GPU job with host memory carrying the bytes RCCL would
(write-sog.ts:245-258,313: the palette k-means whose centroid sums are all-reduced every
iteration; the two cluster1d on ranks 0 and 1, shared with the other six).

* north_star's table (one 10M-splat SH-3 table, 1.25M rows per rank) through `bench.py --gpus 8
  --backend gloo`: every label of every shard an exact f64 argmin, the same centroids on every
  rank, the seven textures and meta equal to st_dev_sog of the whole table on one device, and the
  collective sequences of the eight ranks identical (ST_SIDE_INLINE=1: both channels issued from
  the main thread at RCCL's program points, ST_COLL_TRACE logs them);
* a ragged 8-way split of the multi-process tests' table (tests/mp_table.py: sums that fail the
  order-free certificate, so the sequential hand-off crosses all eight ranks) with one rank of 0
  rows and one of 1 row, against the single-device writeSog, traces identical too."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import test_configs_full_gpu as full  # noqa: E402
import test_multiproc_gpu as mp  # noqa: E402

pytestmark = pytest.mark.gpu

WORLD = 8
ref = mp.ref  # the single-device writeSog fixture of the multi-process tests


def _traces(d):
    tr = [open(d / f'coll_rank{r}.txt').read().splitlines() for r in range(WORLD)]
    assert tr[0] and all(t == tr[0] for t in tr), [len(t) for t in tr]
    ops = {ln.split()[1] for ln in tr[0]}
    assert {'allreduce_sum_f64', 'gatherv'} <= ops, ops
    return tr[0]


def test_north_star_10m_in_eight_processes_matches_one_gpu(tmp_path, monkeypatch):
    T = 10_000_000
    d = tmp_path / 'trace'
    d.mkdir()
    monkeypatch.setenv('ST_SIDE_INLINE', '1')
    monkeypatch.setenv('ST_COLL_TRACE', str(d))
    eight = full._bench(['--gpus', str(WORLD), '--backend', 'gloo'])
    monkeypatch.delenv('ST_COLL_TRACE')
    monkeypatch.delenv('ST_SIDE_INLINE')
    full._check_sharded(eight, WORLD, T)
    assert eight['config']['splats_rank0'] == T // WORLD
    assert eight['config']['workload'].startswith('north_star: ')
    _traces(d)
    import torch

    import bench
    table = bench.table_rows(T, 0, T, torch.device('cuda', 0))
    sha, ver = full._one_device(table)
    del table
    full._check_one_device(ver, T)
    assert sha == eight['textures_sha256']


def test_ragged_eight_way_split_with_empty_and_one_row_ranks(tmp_path, ref):
    n = mp.N
    cuts = [0, 1, n // 9, n // 9, n // 3, n // 3 + 77_777, n // 2, n * 7 // 8, n]
    assert len(cuts) == WORLD + 1
    d = tmp_path / 'trace'
    d.mkdir()
    mp.check(*mp.run_job(tmp_path, cuts, env={'ST_SIDE_INLINE': '1', 'ST_COLL_TRACE': str(d)}), ref(n))
    _traces(d)
