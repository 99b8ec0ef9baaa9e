"""PLY ingest (st_ply_read / st_dev_ply_read: file -> pinned chunks -> HBM -> k_ply_cols)
and the compressed-PLY reader (st_decompress_ply / st_dev_decompress_ply, k_decompress)
against the reference's outputs (tests/golden/ply_io.*) and the oracle restatements.
Every value bit-exact."""
import os

import numpy as np
import pytest
import torch

import oracle
import ply
import splat_hip as sh
from golden_io import Golden
from test_ply_cpu import CP, G, compressed_file, same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    c = sh.Context(0)
    c.set_stream(s.cuda_stream)
    return c


def test_read_ply_mixed_matches_reference(ctx, tmp_path):
    p = tmp_path / 'mixed.ply'
    p.write_bytes(G['mixed_file'].tobytes())
    comments, els = ctx.read_ply(str(p))
    assert comments == G.meta['mixed']['comments']
    for name, cols in els:
        for k, v in cols.items():
            assert same(v, G[f'mixed_{name}_{k}']), (name, k)
    comments, els = ctx.read_ply_dev(str(p))
    for name, cols in els:
        for k, v in cols.items():
            assert same(v.cpu().numpy(), G[f'mixed_{name}_{k}']), (name, k)


def _gs_file(n, shc, seed, extra_byte=False):
    rng = np.random.default_rng(seed)
    names = ['x', 'y', 'z', 'nx', 'ny', 'nz', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + \
        [f'f_rest_{i}' for i in range(3 * shc)] + ['opacity', 'scale_0', 'scale_1', 'scale_2'] + \
        [f'rot_{i}' for i in range(4)]
    fields = [(k, '<f4') for k in names] + ([('flag', 'u1')] if extra_byte else [])
    rows = np.zeros(n, np.dtype(fields))
    for k, t in fields:
        rows[k] = rng.normal(0, 1, n).astype(t) if t == '<f4' else rng.integers(0, 256, n)
    head = 'ply\nformat binary_little_endian 1.0\n' + f'element vertex {n}\n' + ''.join(
        f"property {'float' if t == '<f4' else 'uchar'} {k}\n" for k, t in fields) + 'end_header\n'
    return head.encode() + rows.tobytes()


@pytest.mark.parametrize('n,shc,odd,chunk', [(300_000, 15, False, None), (100_003, 3, True, None),
                                             (50_001, 0, True, 40_000), (9, 15, True, 64)])
def test_read_ply_vs_oracle(ctx, tmp_path, monkeypatch, n, shc, odd, chunk):
    if chunk:
        monkeypatch.setenv('ST_PLY_CHUNK', str(chunk))  # many pinned chunks through the double buffer
    data = _gs_file(n, shc, n, odd)
    p = tmp_path / 'gs.ply'
    p.write_bytes(data)
    _, want = ply.read_ply(data)
    _, got = ctx.read_ply_dev(str(p))
    for (wn, wc), (gn, gc) in zip(want, got):
        assert wn == gn and list(wc) == list(gc)
        for k in wc:
            assert same(gc[k].cpu().numpy(), wc[k]), k
    # the host form: the pinned chunks transposed on the host (AVX2 8 x 8 blocks for float-only
    # rows, value by value otherwise) beside the device ingest, with and without the columns'
    # host twins -- every byte as the oracle's
    for env in (None, 'ST_HOST_MIRROR'):
        if env:
            monkeypatch.setenv(env, '0')
        _, got = ctx.read_ply(str(p))
        if env:
            monkeypatch.delenv(env)
        for (wn, wc), (gn, gc) in zip(want, got):
            assert wn == gn and list(wc) == list(gc)
            for k in wc:
                assert same(gc[k], wc[k]), (k, env)


def test_read_ply_truncated_file_raises(ctx, tmp_path):
    data = _gs_file(1000, 0, 3)
    p = tmp_path / 'cut.ply'
    p.write_bytes(data[:-5])
    with pytest.raises(sh.StError):
        ctx.read_ply(str(p))


@pytest.mark.parametrize('name', [c['name'] for c in G.meta['compressed']])
def test_decompress_matches_reference(ctx, tmp_path, name):
    p = tmp_path / 'c.ply'
    p.write_bytes(compressed_file(name))
    _, els = ctx.read_ply(str(p))
    el = dict(els)
    shc = [el['sh'][f'f_rest_{i}'] for i in range(len(el['sh']))] if 'sh' in el else []
    out = ctx.decompress_ply(el['chunk'], el['vertex'], shc)
    assert list(out) == G.meta[f'{name}_columns']
    for k, v in out.items():
        assert same(v, G[f'{name}_dec_{k}']), k


def test_pack_then_decompress_large_vs_oracle(ctx):
    # the device chunk pack output of 1M SH3 splats, decompressed on the device
    rng = np.random.default_rng(44)
    n = 1_000_000
    names = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2', 'opacity', 'scale_0', 'scale_1', 'scale_2',
             'rot_0', 'rot_1', 'rot_2', 'rot_3'] + [f'f_rest_{i}' for i in range(45)]
    cols = {k: rng.normal(0, 1, n).astype(np.float32) for k in names}
    order = ctx.morton_order(cols['x'], cols['y'], cols['z'])
    chunk, vertex, shb = ctx.pack_compressed(cols, order, 45)
    chunk = chunk.reshape(-1, 18)
    ch = {k: np.ascontiguousarray(chunk[:, i]) for i, k in enumerate(sh.CHUNK_COLS)}
    vertex = vertex.reshape(-1, 4)
    vx = {k: np.ascontiguousarray(vertex[:, i]) for i, k in enumerate(sh.VERTEX_COLS)}
    shb = shb.reshape(n, 45)
    shc = [np.ascontiguousarray(shb[:, i]) for i in range(45)]
    want = oracle.decompress_ply(ch, vx, shc)
    d = lambda a: torch.from_numpy(a).cuda()
    out = {k: torch.empty(n, dtype=torch.float32, device='cuda') for k in want}
    ctx.dev_decompress_ply({k: d(v) for k, v in ch.items()}, {k: d(v) for k, v in vx.items()}, [d(a) for a in shc],
                           out)
    for k in want:
        assert same(out[k].cpu().numpy(), want[k]), k


@pytest.mark.parametrize('slot_mb', [None, '1'])
def test_compressed_ply_file_equals_the_arrays(ctx, tmp_path, monkeypatch, slot_mb):
    """st_ply_compressed_ply_file / st_compressed_ply_file (the CLI's `in.ply -r 0,45,0 --filterNaN
    out.compressed.ply`, write-compressed-ply.ts:31-115): the file is the reference's header + the
    chunk / vertex / sh arrays of the one-call form, byte for byte -- into a file that held longer
    content, with 1 MiB slots too (many pieces through the ring)"""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools'))
    import bench_paths
    if slot_mb:
        monkeypatch.setenv('ST_CPF_SLOT_MB', slot_mb)
    n = 300_001
    data = bytearray(_gs_file(n, 15, 11))
    src = tmp_path / 'in.ply'
    src.write_bytes(bytes(data))
    _, els = ctx.read_ply(str(src))
    cols = dict(els)['vertex']
    cols['x'][::997] = np.nan  # rows filterNaN drops
    src.write_bytes(data[:data.index(b'end_header\n') + 11] + np.stack(list(cols.values()), 1).astype('<f4').tobytes())
    acts = [{'kind': 'rotate', 'value': (0, 45, 0)}, {'kind': 'filterNaN'}]
    m, chunk, vertex, shb = ctx.ply_compressed_ply(str(src), acts)
    want = bench_paths.compressed_ply_header(m, 15) + chunk.tobytes() + vertex.tobytes() + shb.tobytes()
    out = tmp_path / 'out.compressed.ply'
    out.write_bytes(b'\x07' * (len(want) + 12345))
    mm, C, size = ctx.ply_compressed_ply_file(str(src), acts, str(out))
    assert (mm, C, size) == (m, 15, len(want)) and m < n
    assert out.read_bytes() == want
    mm, C, size = ctx.compressed_ply_file(list(cols.items()), acts, str(out), version='9.9.9')
    assert out.read_bytes() == want.replace(b'splat-transform 0.10.1', b'splat-transform 9.9.9')


def test_compressed_ply_file_refuses_append(ctx, tmp_path):
    src = tmp_path / 'in.ply'
    src.write_bytes(_gs_file(1000, 0, 3))
    out = tmp_path / 'o.ply'
    out.write_bytes(b'keep')
    import ctypes
    fd, ofd = os.open(str(src), os.O_RDONLY), os.open(str(out), os.O_WRONLY | os.O_APPEND)
    try:
        h = sh.PlyHeader()
        sh.check(sh.lib().st_ply_read_header(ctypes.c_int32(fd), ctypes.byref(h)))
        m, C, size = ctypes.c_uint64(), ctypes.c_int32(), ctypes.c_uint64()
        rc = sh.lib().st_ply_compressed_ply_file(ctx.h, ctypes.c_int32(fd), ctypes.byref(h), ctypes.c_int32(-1), None,
                                                 ctypes.c_int32(0), ctypes.c_int32(ofd), None, ctypes.byref(m),
                                                 ctypes.byref(C), ctypes.byref(size))
    finally:
        os.close(fd)
        os.close(ofd)
    assert rc == sh.ST_ERR_ARG and b'O_APPEND' in sh.lib().st_last_error()
    assert out.read_bytes() == b'keep'
