"""filterNaN / permuteRows / combine over every column type (process.ts:47-61,84-95,
data-table.ts:135-149, index.ts:158-210) against the reference's own vectors
(tests/golden/filter_combine.*: make_golden.js filter_combine)."""
import numpy as np
import pytest

import oracle
import splat_hip as sh
from golden_io import Golden

TYPES = {'int8': np.int8, 'uint8': np.uint8, 'int16': np.int16, 'uint16': np.uint16, 'int32': np.int32,
         'uint32': np.uint32, 'float32': np.float32, 'float64': np.float64}


def _c4(g):
    tables = []
    for i in range(4):
        names = g.meta[f'c4_{i}_names']
        tables.append([(nm, g[f'c4_{i}_i{j}']) for j, nm in enumerate(names)])
    return tables


def _same(a, b):
    assert a.dtype == b.dtype and a.shape == b.shape
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


def test_oracle_combine_matches_reference():
    g = Golden('filter_combine')
    out = oracle.combine(_c4(g))
    assert [n for n, _ in out] == g.meta['c4_out_names']
    assert [a.dtype for _, a in out] == [np.dtype(TYPES[t]) for t in g.meta['c4_out_types']]
    for j, (_, a) in enumerate(out):
        _same(a, g[f'c4_out_i{j}'])
    abc = [g.table(f'cmb_{t}_').items() for t in 'abc']
    out = oracle.combine([list(t) for t in abc])
    assert [n for n, _ in out] == g.meta['cmb_out_columns']
    for j, (_, a) in enumerate(out):
        _same(a, g[f'cmb_out_i{j}'])


def test_oracle_typed_filter_nan_matches_reference():
    g = Golden('filter_combine')
    src = list(g.table('typed_in_').items())
    out, _ = oracle.filter_nan(src)
    want = g.table('typed_out_')
    for name, a in out:
        _same(a, want[name])


def test_combine_layout_matches_reference():
    """st_combine_layout (host half of st_dev_combine, no device needed)"""
    g = Golden('filter_combine')
    tables = _c4(g)
    lay = sh.combine_layout(tables)
    assert [tables[t][c][0] for t, c in lay] == g.meta['c4_out_names']
    assert [tables[t][c][1].dtype for t, c in lay] == [np.dtype(TYPES[x]) for x in g.meta['c4_out_types']]
    abc = [list(g.table(f'cmb_{t}_').items()) for t in 'abc']
    lay = sh.combine_layout(abc)
    assert [abc[t][c][0] for t, c in lay] == g.meta['cmb_out_columns']


# ---- device ---------------------------------------------------------------------------
@pytest.fixture(scope='module')
def ctx():
    import torch  # noqa: F401
    c = sh.Context(0)
    yield c
    c.close()


def _dev(items):
    import torch
    return [(n, torch.from_numpy(np.ascontiguousarray(a)).cuda()) for n, a in items]


def _host(items):
    return [(n, t.cpu().numpy()) for n, t in items]


@pytest.mark.gpu
def test_dev_combine_matches_reference(ctx):
    import torch
    g = Golden('filter_combine')
    for tables, names_key, want_key in ((_c4(g), 'c4_out_names', 'c4_out_i'),
                                        ([list(g.table(f'cmb_{t}_').items()) for t in 'abc'], 'cmb_out_columns',
                                         'cmb_out_i')):
        lay = sh.combine_layout(tables)
        total = sum(len(t[0][1]) for t in tables)
        # garbage-filled: the zero fill of absent rows is part of the contract
        dst = [(tables[t][c][0], torch.from_numpy(np.full(total, 7, tables[t][c][1].dtype)).cuda()) for t, c in lay]
        ctx.dev_combine([_dev(t) for t in tables], dst)
        ctx.synchronize()
        assert [n for n, _ in dst] == g.meta[names_key]
        for j, (_, a) in enumerate(_host(dst)):
            _same(a, g[f'{want_key}{j}'])


@pytest.mark.gpu
@pytest.mark.parametrize('host', [False, True])
def test_typed_filter_nan_matches_reference(ctx, host):
    import torch
    g = Golden('filter_combine')
    src = list(g.table('typed_in_').items())
    want = g.table('typed_out_')
    if host:
        out = ctx.filter_nan(src)
    else:
        d = _dev(src)
        idx = torch.empty(len(src[0][1]), dtype=torch.int32, device='cuda')
        m = ctx.dev_filter_finite_t(d, idx)
        dst = [(n, torch.empty(m, dtype=a.dtype, device='cuda')) for n, a in d]
        ctx.dev_permute_rows_t(d, idx, m, dst)
        ctx.synchronize()
        out = _host(dst)
    for name, a in out:
        _same(a, want[name])


@pytest.mark.gpu
def test_filter_nan_then_permute_golden(ctx):
    """the float32 splat table: st_dev_filter_finite -> st_dev_permute_rows (the config-3 device
    path, k_gather_cols4) against the reference's filterNaN output"""
    import torch
    g = Golden('filter_combine')
    src = g.table('in_')
    want = g.table('out_')
    d = {k: torch.from_numpy(v).cuda() for k, v in src.items()}
    idx = torch.empty(len(src['x']), dtype=torch.int32, device='cuda')
    m = ctx.dev_filter_finite(d, idx)
    dst = {k: torch.empty(m, dtype=torch.float32, device='cuda') for k in d}
    ctx.dev_permute_rows(d, idx, m, dst)
    ctx.synchronize()
    for k in src:
        _same(dst[k].cpu().numpy(), want[k])


@pytest.mark.gpu
@pytest.mark.parametrize('n,m,shift', [(100_003, 70_001, 0), (4097, 4097, 1), (1_000_000, 999_999, 3), (5, 3, 0),
                                       (64, 0, 0)])
def test_permute_rows_every_type_vs_numpy(ctx, n, m, shift):
    """dst[c][j] = src[c][idx[j]] for the eight types; m % 4 != 0 tails; shift > 0 offsets every
    column (and the index array) by `shift` elements so the 16-byte wide path is not taken"""
    import torch
    rng = np.random.default_rng(n + m)
    src = []
    for t, dt in TYPES.items():
        raw = rng.integers(0, 256, (n + shift) * np.dtype(dt).itemsize, dtype=np.uint8).view(dt)
        src.append((f'c_{t}', raw))
    for j in range(70):  # > 64 four-byte columns: the wide kernel runs in groups
        src.append((f'f{j}', rng.normal(0, 1, n + shift).astype(np.float32)))
    idx = np.concatenate([np.zeros(shift, np.uint32), rng.integers(0, n, m).astype(np.uint32)])
    d_src = [(k, torch.from_numpy(a).cuda()[shift:]) for k, a in src]
    d_idx = torch.from_numpy(idx.view(np.int32)).cuda()[shift:]
    dst = [(k, torch.empty(m + shift, dtype=a.dtype, device='cuda')[shift:]) for k, a in d_src]
    ctx.dev_permute_rows_t(d_src, d_idx, m, dst)
    ctx.synchronize()
    for (k, a), (_, b) in zip(src, dst):
        _same(b.cpu().numpy(), a[shift:][idx[shift:]])
    if shift == 0:  # the float32 entry point (k_gather_cols4 directly) on the f32 columns
        f = {k: t for k, t in d_src if t.dtype == torch.float32}
        out = {k: torch.empty(m, dtype=torch.float32, device='cuda') for k in f}
        ctx.dev_permute_rows(f, d_idx, m, out)
        ctx.synchronize()
        for k, a in src:
            if a.dtype == np.float32:
                _same(out[k].cpu().numpy(), a[idx])


@pytest.mark.gpu
def test_filter_nan_f64_and_int_columns_vs_oracle(ctx):
    import torch
    rng = np.random.default_rng(5)
    n = 300_001
    cols = [('x', rng.normal(0, 1, n).astype(np.float32)), ('d', rng.normal(0, 1, n)),
            ('u', rng.integers(0, 255, n).astype(np.uint8)), ('i', rng.integers(-9, 9, n).astype(np.int32))]
    cols[0][1][rng.integers(0, n, 500)] = np.nan
    cols[1][1][rng.integers(0, n, 500)] = np.inf
    cols[1][1][rng.integers(0, n, 500)] = np.nan
    want, _ = oracle.filter_nan(cols)
    got = ctx.filter_nan(cols)
    for (k, a), (_, b) in zip(want, got):
        _same(b, a)
