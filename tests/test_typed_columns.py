"""Columns that are not float32 (a PLY with `double` properties, and integer ones) on the writers'
path: the reference reads every column through getRow as JS numbers and stores through setRow
(data-table.ts:63-76), so transform (transform.ts:24-64), the ordering (ordering.ts:32-47), the
compressed-PLY writer (write-compressed-ply.ts:56-109, members through CompressedChunk's
Float32Arrays, SH bytes from the numbers) and writeSog (write-sog.ts:110-370: positions,
rotations and opacity as numbers, cluster1d and the k-means points as Float32Arrays, calcAverage
summing the numbers) all take them.

Parity is pinned to the reference itself: tests/golden/typed_columns.* holds the reference's own
processDataTable / writeCompressedPly / writeSog outputs on such tables (make_golden.js
typed_columns): the processed table, the input table afterwards (transforms before the first
filter mutate it), the four file writes, and writeSog's textures, meta and Math.random draws."""

import numpy as np
import pytest

import oracle
import splat_hip as sh
from golden_io import Golden

G = Golden('typed_columns')
CASES = G.meta['cases']
SOG_CASES = [c for c in CASES if f'{c}_sog' in G.meta]
DT = {'int8': np.int8, 'uint8': np.uint8, 'int16': np.int16, 'uint16': np.uint16, 'int32': np.int32,
      'uint32': np.uint32, 'float32': np.float32, 'float64': np.float64}


def _bytes_equal(a, b, what):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    assert a.dtype == b.dtype and a.shape == b.shape, (what, a.dtype, b.dtype, a.shape, b.shape)
    bad = np.nonzero(a.view(np.uint8) != b.view(np.uint8))[0]
    assert bad.size == 0, f'{what}: {bad.size} bytes differ, first at byte {bad[:4]}'


def _table(prefix):
    return [(k, G[f'{prefix}{k}']) for k in G.meta[f'{prefix}columns']]


def _actions(case):
    return G.meta[f'{case}_actions']


# ---- CPU: the fixture itself -------------------------------------------------------------
@pytest.mark.parametrize('case', CASES)
def test_fixture_holds_non_float32_columns(case):
    """the cases really exercise other types (float64 everywhere, or a mix with integers)"""
    types = G.meta[f'{case}_in_types']
    assert any(t != 'float32' for t in types)
    for (k, a), t in zip(_table(f'{case}_in_'), types):
        assert a.dtype == np.dtype(DT[t]), k


@pytest.mark.parametrize('case', CASES)
def test_process_schema_typed(case):
    src = _table(f'{case}_in_')
    got = sh.process_schema(src, _actions(case))
    assert [k for k, _ in got] == G.meta[f'{case}_out_columns']
    assert [str(t) for _, t in got] == [str(np.dtype(DT[t])) for t in G.meta[f'{case}_out_types']]


# ---- GPU -------------------------------------------------------------------------------------
@pytest.fixture(scope='module')
def ctx():
    import torch  # noqa: F401
    c = sh.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_process_typed_matches_reference(ctx, case):
    """processDataTable on the typed table: the processed table (types kept) and the input table
    afterwards, byte for byte"""
    src = [(k, a.copy()) for k, a in _table(f'{case}_in_')]
    out = ctx.process(src, _actions(case))
    assert [k for k, _ in out] == G.meta[f'{case}_out_columns']
    for (k, a), (_, b) in zip(out, _table(f'{case}_out_')):
        _bytes_equal(a, b, k)
    for (k, a), (_, b) in zip(src, _table(f'{case}_after_')):
        _bytes_equal(a, b, 'after ' + k)


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_compressed_ply_typed_matches_reference(ctx, case):
    """processDataTable + writeCompressedPly in one call: chunk / vertex / sh bytes"""
    src = _table(f'{case}_in_')
    m, chunk, vertex, shb = ctx.compressed_ply(src, _actions(case))
    assert m == len(_table(f'{case}_out_')[0][1])
    for nm, a in (('chunk', chunk), ('vertex', vertex), ('sh', shb)):
        _bytes_equal(a, G[f'{case}_{nm}'], nm)


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_compressed_ply_from_typed_file(ctx, case, tmp_path):
    """the same straight from a PLY whose properties have these types (double, short, int, ...)"""
    src = _table(f'{case}_in_')
    ptype = {np.dtype(np.int8): 'char', np.dtype(np.uint8): 'uchar', np.dtype(np.int16): 'short',
             np.dtype(np.uint16): 'ushort', np.dtype(np.int32): 'int', np.dtype(np.uint32): 'uint',
             np.dtype(np.float32): 'float', np.dtype(np.float64): 'double'}
    n = len(src[0][1])
    head = ('ply\nformat binary_little_endian 1.0\n' + f'element vertex {n}\n' +
            ''.join(f'property {ptype[a.dtype]} {k}\n' for k, a in src) + 'end_header\n').encode()
    rows = np.zeros(n, dtype=[(k, a.dtype.newbyteorder('<')) for k, a in src])
    for k, a in src:
        rows[k] = a
    p = str(tmp_path / 'typed.ply')
    with open(p, 'wb') as f:
        f.write(head)
        f.write(rows.tobytes())
    m, chunk, vertex, shb = ctx.ply_compressed_ply(p, _actions(case))
    for nm, a in (('chunk', chunk), ('vertex', vertex), ('sh', shb)):
        _bytes_equal(a, G[f'{case}_{nm}'], nm)


@pytest.mark.gpu
def test_transform_typed_in_place(ctx):
    """transform() alone on a typed host table (st_transform_t) equals the reference's first
    action of the f64 case (the input afterwards: the rotate ran before the filter)"""
    cols = dict((k, a.copy()) for k, a in _table('f64_in_'))
    act = _actions('f64')[0]
    ctx.transform(cols, sh.action_params(act['kind'], act['value']))
    for k, b in _table('f64_after_'):
        _bytes_equal(cols[k], b, k)


@pytest.mark.gpu
def test_morton_typed_matches_float64_sort(ctx):
    """generateOrdering of float64 / integer positions (st_morton_order_t) against the same keys
    computed in numpy from the numbers (single level: no run of > 256 equal keys)"""
    rng = np.random.default_rng(5)
    n = 50_000
    x = rng.normal(0, 10, n)  # float64, not float32-representable
    y = (rng.normal(0, 1000, n)).astype(np.int32)
    z = rng.normal(0, 10, n).astype(np.float32)
    got = ctx.morton_order(x, y, z)
    vals = [x, y.astype(np.float64), z.astype(np.float64)]
    q = []
    for v in vals:
        mn, mx = v.min(), v.max()
        mul = 1024 / (mx - mn)
        q.append(np.minimum(1023, (v - mn) * mul).astype(np.uint32))

    def part1by2(a):
        a = a & 0x3ff
        a = (a ^ (a << 16)) & 0xff0000ff
        a = (a ^ (a << 8)) & 0x0300f00f
        a = (a ^ (a << 4)) & 0x030c30c3
        return (a ^ (a << 2)) & 0x09249249
    key = (part1by2(q[2]) << 2) + (part1by2(q[1]) << 1) + part1by2(q[0])
    assert np.bincount(key).max() <= 256
    want = np.argsort(key, kind='stable').astype(np.uint32)
    _bytes_equal(got, want, 'order')


def _check_sog(tex, meta, used, case):
    ref = G.meta[f'{case}_sog']
    assert used == ref['draws']
    for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels'):
        _bytes_equal(tex[k], G[f'{case}_sog_{k}'], k)
    m = ref['meta']
    assert list(meta.means_min) == m['means']['mins']
    assert list(meta.means_max) == m['means']['maxs']
    _bytes_equal(np.array(meta.scales_codebook, np.float32), np.array(m['scales']['codebook'], np.float32), 'scales')
    _bytes_equal(np.array(meta.sh0_codebook, np.float32), np.array(m['sh0']['codebook'], np.float32), 'sh0')
    _bytes_equal(np.array(meta.shn_codebook, np.float32), np.array(m['shN']['codebook'], np.float32), 'shN')
    assert meta.palette_size == m['shN']['count'] and meta.sh_bands == m['shN']['bands']


@pytest.mark.gpu
@pytest.mark.parametrize('case', SOG_CASES)
def test_sog_typed_matches_reference(ctx, case):
    """writeSog of the typed table: textures, meta and the draws consumed"""
    ref = G.meta[f'{case}_sog']
    tex, meta, used = ctx.sog_process(_table(f'{case}_sog_in_'), [], ref['iters'],
                                      oracle.mulberry32(ref['seed'], ref['draws'] + 64))
    _check_sog(tex, meta, used, case)


@pytest.mark.gpu
@pytest.mark.parametrize('case', SOG_CASES)
def test_sog_bundle_typed_equals_textures(ctx, case):
    """the .sog archive of the typed table (st_sog_bundle_process) holds the same pixels: it
    equals the archive the library builds from the reference's own textures and meta"""
    import torch
    ref = G.meta[f'{case}_sog']
    draws = oracle.mulberry32(ref['seed'], ref['draws'] + 64)
    got, used = ctx.sog_bundle_process(_table(f'{case}_sog_in_'), [], ref['iters'], draws, 0x6000, 0x5a21)
    assert used == ref['draws']
    tex, meta, _ = ctx.sog_process(_table(f'{case}_sog_in_'), [], ref['iters'], draws)
    dev = {k: torch.from_numpy(np.ascontiguousarray(G[f'{case}_sog_{k}']).reshape(-1)).cuda()
           for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels')}
    want = ctx.dev_sog_bundle(meta, ref['n'], dev, 0x6000, 0x5a21)
    assert got == want
