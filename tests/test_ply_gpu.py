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
