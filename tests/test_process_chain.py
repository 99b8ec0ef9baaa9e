"""processDataTable (process.ts:64-145) and the CLI's `in.ply [actions] out.compressed.ply`
(index.ts:463-496 -> writeCompressedPly, write-compressed-ply.ts:31-115) as one call
(st_process / st_compressed_ply / st_dev_compressed_ply), against the reference's own vectors
(tests/golden/process_chain.*: make_golden.js process_chain -- every action kind, NaN/-0 edges,
an unknown comparator, a missing column, an empty result) and, at 1M splats, the oracle chain.
Compressed-PLY outputs are compared as file bytes (NaN bit patterns included)."""
import numpy as np
import pytest

import oracle
import splat_hip as sh
from golden_io import Golden

TYPES = {'int8': np.int8, 'uint8': np.uint8, 'int16': np.int16, 'uint16': np.uint16, 'int32': np.int32,
         'uint32': np.uint32, 'float32': np.float32, 'float64': np.float64}


def _bytes_equal(a, b, what):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    assert a.dtype == b.dtype and a.shape == b.shape, (what, a.dtype, b.dtype, a.shape, b.shape)
    bad = np.nonzero(a.view(np.uint8) != b.view(np.uint8))[0]
    assert bad.size == 0, f'{what}: {bad.size} bytes differ, first at byte {bad[:4]}'


def _case(g, c):
    src = [(k, g[f'{c}_in_{k}']) for k in g.meta[f'{c}_in_columns']]
    want = [(k, g[f'{c}_out_{k}']) for k in g.meta[f'{c}_out_columns']]
    return src, g.meta[f'{c}_actions'], want


G = Golden('process_chain')
CASES = G.meta['cases']


# ---- CPU: the oracle and the host-side schema logic against the reference --------------
@pytest.mark.parametrize('case', CASES)
def test_oracle_chain_matches_reference(case):
    src, acts, want = _case(G, case)
    out, chunk, vertex, shb = oracle.compressed_ply(src, acts)
    assert [k for k, _ in out] == [k for k, _ in want]
    assert [str(a.dtype) for _, a in out] == [str(np.dtype(TYPES[t])) for t in G.meta[f'{case}_out_types']]
    for (k, a), (_, b) in zip(out, want):
        _bytes_equal(a, b, k)
    for nm, a in (('chunk', chunk), ('vertex', vertex), ('sh', shb)):
        _bytes_equal(a, G[f'{case}_{nm}'], nm)


@pytest.mark.parametrize('case', CASES)
def test_process_schema_matches_reference(case):
    src, acts, want = _case(G, case)
    assert [k for k, _ in sh.process_schema(src, acts)] == [k for k, _ in want]


# ---- GPU: the one-call chain --------------------------------------------------------------
@pytest.fixture(scope='module')
def ctx():
    import torch  # noqa: F401
    c = sh.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_compressed_ply_matches_reference(ctx, case):
    src, acts, want = _case(G, case)
    m, chunk, vertex, shb = ctx.compressed_ply(src, acts)
    assert m == len(want[0][1])
    for nm, a in (('chunk', chunk), ('vertex', vertex), ('sh', shb)):
        _bytes_equal(a, G[f'{case}_{nm}'], nm)


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_process_matches_reference(ctx, case):
    src, acts, want = _case(G, case)
    out = ctx.process(src, acts)
    assert [k for k, _ in out] == [k for k, _ in want]
    for (k, a), (_, b) in zip(out, want):
        _bytes_equal(a, b, k)


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_process_mutates_input_like_reference(ctx, case):
    """the transforms before the first filter change the caller's columns in place (process.ts:65-83,
    filterBands' renamed columns included): the input afterwards equals the reference's"""
    src, acts, want = _case(G, case)
    src = [(k, a.copy()) for k, a in src]
    out = ctx.process(src, acts)
    for k, a in src:
        _bytes_equal(a, G[f'{case}_after_{k}'], k)
    for (k, a), (_, b) in zip(out, want):
        _bytes_equal(a, b, k)
    if not any(a['kind'] in ('filterNaN', 'filterByValue') for a in acts):
        srcs = {id(a) for _, a in src}
        assert all(id(a) in srcs for _, a in out), 'without a filter the result shares the input arrays'


@pytest.mark.gpu
@pytest.mark.parametrize('case', ['config3', 'bands2_lte', 'empty'])
def test_dev_compressed_ply_matches_reference(ctx, case):
    import torch
    src, acts, want = _case(G, case)
    n = len(src[0][1])
    d = [(k, torch.from_numpy(np.ascontiguousarray(a)).cuda()) for k, a in src]
    chunk = torch.full(((n + 255) // 256 * 18 + 1,), 7.0, device='cuda')
    vertex = torch.zeros(n * 4 + 1, dtype=torch.int32, device='cuda')
    shb = torch.zeros(n * 45 + 1, dtype=torch.uint8, device='cuda')
    m, C = ctx.dev_compressed_ply(d, acts, chunk, vertex, shb)
    ctx.synchronize()
    assert m == len(want[0][1])
    _bytes_equal(chunk[:(m + 255) // 256 * 18].cpu().numpy(), G[f'{case}_chunk'], 'chunk')
    _bytes_equal(vertex[:m * 4].cpu().numpy().view(np.uint32), G[f'{case}_vertex'], 'vertex')
    _bytes_equal(shb[:m * 3 * C].cpu().numpy(), G[f'{case}_sh'], 'sh')


@pytest.mark.gpu
def test_compressed_ply_config3_1m_vs_oracle(ctx):
    """BASELINE config 3's chain at 1M SH-3 splats, one call: -r 0,45,0 --filterNaN then the
    Morton order and chunk pack, 0.1% of rows non-finite, 5% in a 1e-3 cube (Morton runs > 256)"""
    n = 1_000_000
    rng = np.random.default_rng(2003)
    names = ['x', 'y', 'z', 'nx', 'ny', 'nz', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] + \
        ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3']
    cols = {k: rng.normal(0, 1, n).astype(np.float32) for k in names}
    cols['x'] *= 10
    cube = rng.random(n) < 0.05
    cols['x'][cube] = 1 + rng.random(cube.sum()).astype(np.float32) * 1e-3
    bad = rng.choice(n, n // 1000, replace=False)
    for j, r in enumerate(bad):
        cols[names[j % len(names)]][r] = [np.nan, np.inf, -np.inf][j % 3]
    acts = [{'kind': 'rotate', 'value': [0, 45, 0]}, {'kind': 'filterNaN'}]
    src = list(cols.items())
    m, chunk, vertex, shb = ctx.compressed_ply(src, acts)
    out, ochunk, overtex, osh = oracle.compressed_ply(src, acts)
    assert m == len(out[0][1])
    _bytes_equal(chunk, ochunk, 'chunk')
    _bytes_equal(vertex, overtex, 'vertex')
    _bytes_equal(shb, osh, 'sh')


@pytest.mark.gpu
def test_process_typed_filter_by_value_vs_oracle(ctx):
    """filterByValue on integer and float64 columns (compared as JS numbers), then filterNaN,
    over the reference's all-types table"""
    g = Golden('filter_combine')
    src = list(g.table('typed_in_').items())
    for acts in ([{'kind': 'filterByValue', 'columnName': 'c_uint8', 'comparator': 'gt', 'value': 100}],
                 [{'kind': 'filterByValue', 'columnName': 'c_int32', 'comparator': 'lte', 'value': -1.5e9},
                  {'kind': 'filterNaN'}],
                 [{'kind': 'filterByValue', 'columnName': 'c_float64', 'comparator': 'neq', 'value': 0},
                  {'kind': 'filterByValue', 'columnName': 'c_int16', 'comparator': 'gte', 'value': 0}],
                 [{'kind': 'filterByValue', 'columnName': 'c_uint32', 'comparator': 'eq', 'value': 0}]):
        out = ctx.process(src, acts)
        want = oracle.process(src, acts)
        assert [k for k, _ in out] == [k for k, _ in want]
        for (k, a), (_, b) in zip(out, want):
            _bytes_equal(a, b, k)


@pytest.mark.gpu
def test_chain_errors(ctx):
    """the reference's own failures only: a bad filterBands value and a missing chunk member (its
    other column types are accepted, tests/test_typed_columns.py)"""
    src, acts, _ = _case(G, 'config3')
    with pytest.raises(sh.StError) as e:
        ctx.compressed_ply([(k, a) for k, a in src if k != 'opacity'], [])
    assert e.value.code == sh.ST_ERR_ARG and 'opacity' in str(e.value)
    with pytest.raises(sh.StError) as e:
        ctx.compressed_ply(src, [{'kind': 'filterBands', 'value': 4}])
    assert e.value.code == sh.ST_ERR_ARG


# ---- GPU: the same chain straight from the PLY file (st_ply_compressed_ply / st_ply_sog_bundle) --
def _write_ply(path, items):
    """binary little-endian PLY of one 'vertex' element (float32 / uchar / double columns as given)"""
    code = {np.dtype(np.float32): 'float', np.dtype(np.float64): 'double', np.dtype(np.uint8): 'uchar',
            np.dtype(np.int32): 'int'}
    n = len(items[0][1])
    rows = np.zeros(n, np.dtype([(k, a.dtype.newbyteorder('<')) for k, a in items]))
    for k, a in items:
        rows[k] = a
    head = 'ply\nformat binary_little_endian 1.0\ncomment test\n' + f'element vertex {n}\n' + ''.join(
        f'property {code[np.dtype(a.dtype)]} {k}\n' for k, a in items) + 'end_header\n'
    with open(path, 'wb') as f:
        f.write(head.encode() + rows.tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_ply_compressed_ply_matches_reference(ctx, case, tmp_path):
    src, acts, want = _case(G, case)
    p = str(tmp_path / 'in.ply')
    _write_ply(p, src)
    m, chunk, vertex, shb = ctx.ply_compressed_ply(p, acts)
    assert m == len(want[0][1])
    for nm, a in (('chunk', chunk), ('vertex', vertex), ('sh', shb)):
        _bytes_equal(a, G[f'{case}_{nm}'], nm)


@pytest.mark.gpu
def test_ply_sog_bundle_equals_host_one_call(ctx, tmp_path):
    """in.ply -r 0,45,0 --filterNaN out.sog from the file, resident: the archive equals writeSog's
    bundle of the processed table computed through the host entry points"""
    src, acts, _ = _case(G, 'config3')
    p = str(tmp_path / 'in.ply')
    _write_ply(p, src)
    draws = oracle.mulberry32(5, 200_000)
    got, used = ctx.ply_sog_bundle(p, acts, 3, draws, 0x6000, 0x5a21)
    proc = dict(ctx.process(src, acts))
    want, used2 = ctx.sog_bundle({k: v for k, v in proc.items() if k not in ('nx', 'ny', 'nz')}, 3, draws, 0x6000,
                                 0x5a21)
    assert used == used2 and got == want


@pytest.mark.gpu
@pytest.mark.parametrize('n', [262_145, 4_194_305 + 7])
def test_process_staged_copies_vs_oracle(ctx, n):
    """The one-call host forms move columns of 1 MiB and more through the pinned slots that host
    threads fill and drain (staged_h2d / staged_d2h; smaller ones go straight through the
    runtime): a typed table whose columns fall on both sides of that line and across several
    16 MiB slots, through processDataTable (filterByValue, filterNaN, a transform) and back."""
    rng = np.random.default_rng(n)
    src = [('x', rng.normal(0, 5, n).astype(np.float32)), ('y', rng.normal(0, 5, n).astype(np.float32)),
           ('z', rng.normal(0, 5, n).astype(np.float32)),
           ('c_f64', rng.normal(0, 1, n)), ('c_u8', rng.integers(0, 256, n).astype(np.uint8)),
           ('c_i16', rng.integers(-30000, 30000, n).astype(np.int16))]
    src[3][1][rng.random(n) < 0.01] = np.nan
    acts = [{'kind': 'filterByValue', 'columnName': 'c_u8', 'comparator': 'gte', 'value': 3},
            {'kind': 'filterNaN'},
            {'kind': 'translate', 'value': (1.0, -2.0, 0.5)}]
    out = ctx.process(src, acts)
    want = oracle.process(src, acts)
    assert [k for k, _ in out] == [k for k, _ in want]
    for (k, a), (_, b) in zip(out, want):
        _bytes_equal(a, b, k)
