"""Native multi-GPU writeSog (st_multi.hip: st_group_* / st_comm_* / st_dev_sog_sharded /
st_set_devices) against the single-device writeSog of the global table, bit for bit.

On the one-GPU test box several ranks share cuda:0 through the host-staged exchange (the same
orchestration code as RCCL, a different transport); the RCCL transport runs at world size 1
(in-process ncclCommInitAll, and the one-process-per-GPU ncclCommInitRank form).  Config 5's
combine of several inputs (index.ts:158-210) is covered by tables with different schemas."""
import numpy as np
import pytest

import oracle
import splat_hip as sh

pytestmark = pytest.mark.gpu

NAMES = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] + \
    ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3']


def _table(n, seed, C=15, adversarial=False):
    rng = np.random.default_rng(seed)
    cols = {}
    cube = rng.random(n) < 0.05
    for a, off in zip('xyz', (1.0, -2.0, 3.0)):
        cols[a] = np.where(cube, off + rng.random(n) * 1e-3, rng.normal(0, 10, n)).astype(np.float32)
    for i in range(3):
        cols[f'f_dc_{i}'] = rng.normal(0, 1, n).astype(np.float32)
    for i in range(3 * C):
        cols[f'f_rest_{i}'] = rng.normal(0, 0.1, n).astype(np.float32)
    cols['opacity'] = rng.normal(0, 2, n).astype(np.float32)
    for i in range(3):
        v = rng.random(n) * 5 - 7
        if adversarial:  # cluster sums that fail the order-free certificate (values over 15 decades)
            u = rng.random(n)
            v = np.where(u < 0.3, v * 1e-9, np.where(u > 0.9, v * 1e5, v))
        cols[f'scale_{i}'] = v.astype(np.float32)
    for i in range(4):
        cols[f'rot_{i}'] = rng.normal(0, 1, n).astype(np.float32)
    return cols


@pytest.fixture(scope='module')
def ctx():
    import torch  # noqa: F401
    c = sh.Context(0)
    yield c
    c.close()


def _same(got, want):
    tex, meta, used = got
    wtex, wmeta, wused = want
    assert used == wused
    assert sorted(tex) == sorted(wtex)
    for k in wtex:
        assert np.array_equal(tex[k], wtex[k]), k
    for f in ('width', 'height', 'sh_bands', 'palette_size', 'shn_width', 'shn_height'):
        assert getattr(meta, f) == getattr(wmeta, f), f
    assert list(meta.means_min) == list(wmeta.means_min) and list(meta.means_max) == list(wmeta.means_max)
    for f in ('scales_codebook', 'sh0_codebook', 'shn_codebook'):
        assert np.array_equal(np.array(getattr(meta, f), np.float32).view(np.uint32),
                              np.array(getattr(wmeta, f), np.float32).view(np.uint32)), f


def test_group_duplicated_rows_and_clumps_equal_single_device(ctx):
    """Inputs real scenes bring, sharded 3 ways: 20% of the splats share one all-zero SH row
    (coinciding palette centroids, exact ties resolved by the KdTree walk on every rank) and
    half sit in 40 clumps of identical positions (rank 0's Morton recursion)."""
    n = 30_011
    cols = _table(n, 77)
    rng = np.random.default_rng(78)
    dup = rng.random(n) < 0.2
    for i in range(45):
        cols[f'f_rest_{i}'][dup] = 0.0
    clump = rng.random(n) < 0.5
    cid = rng.integers(0, 40, n)
    for a in 'xyz':
        centre = rng.normal(0, 10, 40).astype(np.float32)
        cols[a][clump] = centre[cid[clump]]
    draws = np.random.default_rng(9).random(1 << 18)
    want = ctx.sog(cols, 2, draws)
    g = sh.Group([0] * 3, host_staged=True)
    try:
        _same(g.sog([cols], 2, draws, [0, 9000, 20000, n]), want)
    finally:
        g.close()


@pytest.mark.parametrize('who', ['scales', 'colours', 'neither'])
def test_group_cluster1d_reseeds_equal_single_device(ctx, who):
    """The two cluster1d run over the gathered columns, the scales on rank 0 and the colours on
    rank 1 from draw 0 (kept only when the scales took no draw, rerun after them otherwise;
    re-seeds of empty clusters, k-means.ts:174-178).  A far outlier in a column leaves most
    linspace centroids (k-means.ts:23-39) without members, so that cluster1d takes draws; shards
    of 3 ranks (rank 1's empty: it still runs the colours), and every rank must continue from the
    draws ranks 0 and 1 report."""
    n = 20_011
    cols = _table(n, 91, C=3)
    rng = np.random.default_rng(92)
    for k in {'scales': ['scale_0', 'scale_2'], 'colours': ['f_dc_1'], 'neither': []}[who]:
        cols[k] = (rng.integers(0, 4, n) * 0.25 - 5).astype(np.float32)
        cols[k][17] = 40.0
    draws = np.random.default_rng(93).random(1 << 17)
    want = ctx.sog(cols, 2, draws)
    g = sh.Group([0] * 3, host_staged=True)
    try:
        _same(g.sog([cols], 2, draws, [0, 7000, 7000, n]), want)
    finally:
        g.close()


@pytest.mark.parametrize('world,splits,adv,heavy', [(2, None, False, False), (3, 'empty0', False, False),
                                                     (4, 'ragged', True, False), (4, 'ragged', True, True)])
def test_group_host_staged_equals_single_device(ctx, monkeypatch, world, splits, adv, heavy):
    """heavy: ST_OTHERS_SPLIT / _CHUNK send every cluster with more than 2 pair / ambiguous points
    through the chip-wide others sums (k_heavy), in the single-device
    update and in the sharded partials"""
    if heavy:
        monkeypatch.setenv('ST_OTHERS_SPLIT', '2')
        monkeypatch.setenv('ST_OTHERS_CHUNK', '3')
    n = 30_011
    cols = _table(n, 40 + world, adversarial=adv)
    draws = np.random.default_rng(7).random(1 << 18)
    want = ctx.sog(cols, 2, draws)
    sp = None
    if splits == 'empty0':
        sp = [0, 0, n // 2, n]
    elif splits == 'ragged':
        sp = [0, 7, 9000, 9001, n]
    g = sh.Group([0] * world, host_staged=True)
    try:
        _same(g.sog([cols], 2, draws, sp), want)
    finally:
        g.close()


def test_group_combine_inputs_equals_single_device_on_combined(ctx):
    """config 5 in small: three input tables (SH-3, SH-3, SH-0) concatenated by combine() --
    the SH-0 table's f_rest rows are zero -- sharded over 3 ranks that cut across table bounds"""
    tabs = [_table(9_000, 1), _table(12_345, 2), _table(7_000, 3, C=0)]
    draws = np.random.default_rng(9).random(1 << 18)
    combined = oracle.combine([list(t.items()) for t in tabs])
    want = ctx.sog(dict(combined), 2, draws)
    g = sh.Group([0, 0, 0], host_staged=True)
    try:
        _same(g.sog(tabs, 2, draws), want)
        _same(g.sog(tabs, 2, draws, [0, 15_000, 15_001, 28_345]), want)
    finally:
        g.close()


def test_group_rccl_world1_and_bundle(ctx):
    cols = _table(20_000, 5)
    draws = np.random.default_rng(11).random(1 << 18)
    want = ctx.sog(cols, 2, draws)
    g = sh.Group([0], host_staged=False)
    try:
        _same(g.sog([cols], 2, draws), want)
        z, used = g.sog_bundle([cols], 2, draws, 0x6a2b, 0x58b1)
        zw, usedw = ctx.sog_bundle(cols, 2, draws, 0x6a2b, 0x58b1)
        assert used == usedw and z == zw
    finally:
        g.close()


def test_comm_rank_world1_dev_sog_sharded(ctx):
    """the one-process-per-GPU form (ncclCommInitRank) at world size 1: st_dev_sog_sharded of two
    local tables == st_dev_sog of their concatenation"""
    import torch
    a, b = _table(11_000, 6), _table(6_000, 7)
    full = {k: np.concatenate([a[k], b[k]]) for k in a}
    draws = np.random.default_rng(13).random(1 << 18)
    dev = lambda t: {k: torch.from_numpy(v).cuda() for k, v in t.items()}  # noqa: E731
    W, H, pal, cw, ch = sh.sog_geometry(17_000, 15)
    mk = lambda: {**{k: torch.zeros(W * H * 4, dtype=torch.uint8, device='cuda') for k in  # noqa: E731
                     ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')},
                  'shN_centroids': torch.zeros(cw * ch * 4, dtype=torch.uint8, device='cuda')}
    t1, t2 = mk(), mk()
    m1, u1 = ctx.dev_sog(dev(full), 2, draws, t1)
    comm = sh.Comm(ctx, 1, 0, sh.comm_unique_id())
    try:
        m2, u2 = ctx.dev_sog_sharded(comm, [dev(a), dev(b)], 2, draws, t2)
    finally:
        comm.close()
    torch.cuda.synchronize()
    assert u1 == u2
    for k in t1:
        assert torch.equal(t1[k], t2[k]), k
    assert list(m1.means_min) == list(m2.means_min)


def test_set_devices(ctx):
    assert sh.get_devices() == 1
    sh.set_devices(1)
    with pytest.raises(sh.StError):
        sh.set_devices(sh.device_count() + 1)
    assert sh.get_devices() == 1


def test_st_num_gpus_env():
    """ST_NUM_GPUS=<n> selects the writeSog device count on first use (st_set_devices); more GPUs
    than the box has fails loudly"""
    import os
    import subprocess
    import sys
    py = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'splat-transform_amd', 'py')
    code = ('import ctypes, sys; sys.path.insert(0, %r); import splat_hip as sh; L = sh.lib(); '
            'n = ctypes.c_int32(); rc = L.st_get_devices(ctypes.byref(n)); print(rc, n.value)' % py)
    for value, want in (('1', '0 1'), (str(sh.device_count() + 1), '-1 0')):
        r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, ST_NUM_GPUS=value))
        assert r.returncode == 0, r.stderr
        assert r.stdout.strip() == want, (value, r.stdout)


@pytest.mark.parametrize('world,splits', [(2, None), (3, [0, 5_000, 5_001, 23_345])])
def test_group_bundle_with_input_actions_equals_single_device(ctx, world, splits):
    """`a.ply -r 0,45,0 --filterNaN b.ply -s 2 --filterByValue opacity,gt,0 --filterBands 1 out.sog` on
    `world` ranks: each input's actions run on the ranks' parts of it (transform / filters sharded,
    SURVEY 8e row 1), then combine + writeSog; the .sog bytes equal processDataTable per input ->
    combine -> writeSog on one device"""
    a, b = _table(11_000, 21), _table(12_345, 22)
    for k, r in (('x', 3), ('f_rest_7', 4_000), ('opacity', 10_999)):
        a[k][r] = np.nan
    b['opacity'][5] = np.nan  # filterByValue opacity > 0 drops it (NaN compares false)
    acts = [[{'kind': 'rotate', 'value': (0, 45, 0)}, {'kind': 'filterNaN'}],
            [{'kind': 'scale', 'value': 2.0}, {'kind': 'filterByValue', 'columnName': 'opacity', 'comparator': 'gt',
                                               'value': 0.0}, {'kind': 'filterBands', 'value': 1}]]
    draws = np.random.default_rng(13).random(1 << 18)
    # (copies: processDataTable's leading transforms mutate their input, as the reference's do)
    pa = ctx.process([(k, v.copy()) for k, v in a.items()], acts[0])
    pb = ctx.process([(k, v.copy()) for k, v in b.items()], acts[1])
    combined = dict(oracle.combine([pa, pb]))
    want, wused = ctx.sog_bundle(combined, 2, draws, 0x6000, 0x5a21)
    g = sh.Group([0] * world, host_staged=True)
    try:
        got, used = g.sog_bundle_process([a, b], acts, 2, draws, 0x6000, 0x5a21, splits)
    finally:
        g.close()
    assert used == wused and got == want


@pytest.mark.parametrize('host_staged,world', [(True, 3), (False, 1)])
def test_group_usable_after_a_failed_call(ctx, host_staged, world):
    """a recoverable error inside a group call (draws exhausted on one rank's init) aborts that
    call's collectives; the group rebuilds them, and the next call succeeds bit for bit"""
    cols = _table(20_000, 15)
    draws = np.random.default_rng(17).random(1 << 18)
    want = ctx.sog(cols, 2, draws)
    g = sh.Group([0] * world, host_staged=host_staged)
    try:
        with pytest.raises(sh.StError) as e:
            g.sog([cols], 2, draws[:100])  # too few draws for the 1-D and palette inits
        assert 'another rank failed' not in str(e.value)
        _same(g.sog([cols], 2, draws), want)
        with pytest.raises(sh.StError):
            g.sog([cols], 2, draws[:100])
        _same(g.sog([cols], 2, draws), want)
    finally:
        g.close()


def test_comm_count(ctx):
    comm = sh.Comm(ctx, 1, 0, sh.comm_unique_id())
    try:
        assert comm.count() == 1
    finally:
        comm.close()


@pytest.mark.parametrize('host_staged,world', [(True, 3), (False, 1)])
def test_group_one_rank_fails_the_others_are_released(ctx, host_staged, world, monkeypatch):
    """ST_FAULT_RANK: the last rank throws after the first exchange while the others wait in the
    next collective; the abort releases them, the caller gets the injected error (not the abort),
    and the rebuilt group's next call is exact"""
    cols = _table(20_000, 16)
    draws = np.random.default_rng(18).random(1 << 18)
    want = ctx.sog(cols, 2, draws)
    g = sh.Group([0] * world, host_staged=host_staged)
    try:
        monkeypatch.setenv('ST_FAULT_RANK', str(world - 1))
        with pytest.raises(sh.StError) as e:
            g.sog([cols], 2, draws)
        assert 'injected failure' in str(e.value)
        monkeypatch.delenv('ST_FAULT_RANK')
        _same(g.sog([cols], 2, draws), want)
    finally:
        g.close()
