"""The writeSog host forms on resident columns (st_ctx::HostMirror, st_host_api.hip run_host_sog).

st_ply_read_resident (the Node host's readPly): the host columns stay unfilled and the values live
in HBM until st_ply_materialize -- writeSog reads them on the device, every other host form copies
them down first, and a second read of the element copies them down before it reuses their slots.

st_ply_read: readPly -> writeSog (index.ts:433-510 -> write-sog.ts:110-370)
without uploading a table the device already holds, and only while the caller's columns are
byte for byte what st_ply_read wrote.

Every output is compared with the same call under ST_HOST_MIRROR=0 (always uploaded): unchanged
columns run from the resident copy (st_ctx_last_host_reuse reports 59 columns); a column changed
anywhere -- one value in the middle of an SH column, the first x, the last opacity -- sends the
call back to an upload, and the output is the changed table's."""
import os

import numpy as np
import pytest
import torch

import splat_hip as sh

pytestmark = pytest.mark.gpu

N = 300_000
ITERS = 3


@pytest.fixture(scope='module')
def ctx():
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    c = sh.Context(0)
    c.set_stream(s.cuda_stream)
    yield c
    c.close()


def _ply(path, n, seed):
    import bench
    rng = np.random.default_rng(seed)
    names = bench.PLY_ORDER
    rows = np.zeros(n, np.dtype([(k, '<f4') for k in names]))
    for k in names:
        rows[k] = rng.normal(0, 0.1 if k.startswith('f_rest') else 1, n)
    rows['scale_0'] = rng.random(n) * 5 - 7
    head = ('ply\nformat binary_little_endian 1.0\n' + f'element vertex {n}\n' +
            ''.join(f'property float {k}\n' for k in names) + 'end_header\n').encode()
    with open(path, 'wb') as f:
        f.write(head + rows.tobytes())


def _draws():
    return np.random.default_rng(9).random(2 * 65536 * (ITERS + 2))


def _file(ctx, cols, path, monkeypatch, mirror):
    if mirror:
        monkeypatch.delenv('ST_HOST_MIRROR', raising=False)
    else:
        monkeypatch.setenv('ST_HOST_MIRROR', '0')
    used, size = ctx.sog_file(cols, ITERS, _draws(), path, 0x1234, 0x5678)
    data = open(path, 'rb').read()
    assert len(data) == size
    monkeypatch.delenv('ST_HOST_MIRROR', raising=False)
    return data, used, ctx.host_reuse()


def _read(ctx, path):
    _, els = ctx.read_ply(path)
    return dict(els)['vertex']


@pytest.mark.parametrize('change', [None, ('f_rest_17', N // 2), ('x', 0), ('opacity', N - 1)])
def test_sog_file_on_resident_columns_equals_upload(ctx, tmp_path, monkeypatch, change):
    src = str(tmp_path / 'in.ply')
    _ply(src, N, 4)
    cols = _read(ctx, src)  # a fresh read: its mirrors are the ones registered
    if change:
        k, i = change
        cols[k][i] = np.float32(cols[k][i] + 0.75)
    out = str(tmp_path / 'out.sog')
    got, used, reuse = _file(ctx, cols, out, monkeypatch, True)
    if change:
        assert reuse == (0, 0), reuse
    else:
        assert reuse == (59, 59 * N * 4), reuse
    want, wused, wreuse = _file(ctx, cols, out, monkeypatch, False)
    assert wreuse == (0, 0)
    assert got == want and used == wused


def test_sog_and_bundle_on_resident_columns(ctx, tmp_path, monkeypatch):
    src = str(tmp_path / 'in.ply')
    _ply(src, N, 5)
    cols = _read(ctx, src)
    draws = _draws()
    b1 = ctx.sog_bundle(cols, ITERS, draws, 1, 2)
    assert ctx.host_reuse()[0] == 59
    t1 = ctx.sog(cols, ITERS, draws)
    assert ctx.host_reuse()[0] == 59
    monkeypatch.setenv('ST_HOST_MIRROR', '0')
    b0 = ctx.sog_bundle(cols, ITERS, draws, 1, 2)
    t0 = ctx.sog(cols, ITERS, draws)
    assert ctx.host_reuse() == (0, 0)
    monkeypatch.delenv('ST_HOST_MIRROR')
    assert b1 == b0
    assert t1[2] == t0[2] and list(t1[0]) == list(t0[0])
    for k in t0[0]:
        assert np.array_equal(t1[0][k], t0[0][k]), k


def test_a_second_read_replaces_the_mirrors(ctx, tmp_path, monkeypatch):
    """mirrors belong to the last st_ply_read: the first read's columns are uploaded after a second
    read (their device slots were overwritten), and still give their own output"""
    a, b = str(tmp_path / 'a.ply'), str(tmp_path / 'b.ply')
    _ply(a, N, 6)
    _ply(b, N, 7)
    ca = _read(ctx, a)
    cb = _read(ctx, b)
    out = str(tmp_path / 'o.sog')
    ga, _, ra = _file(ctx, ca, out, monkeypatch, True)
    assert ra == (0, 0)
    gb, _, rb = _file(ctx, cb, out, monkeypatch, True)
    assert rb[0] == 59
    wa, _, _ = _file(ctx, ca, out, monkeypatch, False)
    wb, _, _ = _file(ctx, cb, out, monkeypatch, False)
    assert ga == wa and gb == wb and ga != gb


def _read_resident(ctx, path):
    _, els = ctx.read_ply(path, resident=True)
    return dict(els)['vertex']


def test_resident_read_sog_file_runs_on_the_device_copy(ctx, tmp_path, monkeypatch):
    """st_ply_read_resident + st_sog_file: no column copied down or uploaded (59 reused), the
    archive equal to the eager read's uploaded one; the unfilled host columns stay untouched"""
    src = str(tmp_path / 'in.ply')
    _ply(src, N, 11)
    ref = _read(ctx, src)
    cols = _read_resident(ctx, src)
    mark = np.float32(-12345.5)
    for v in cols.values():
        v[:] = mark  # the library must never read these bytes
    out = str(tmp_path / 'out.sog')
    got, used, reuse = _file(ctx, cols, out, monkeypatch, True)
    assert reuse == (59, 59 * N * 4), reuse
    assert all(np.all(v == mark) for v in cols.values())
    want, wused, _ = _file(ctx, ref, out, monkeypatch, False)
    assert got == want and used == wused


def test_resident_read_materialize_and_forget(ctx, tmp_path, monkeypatch):
    """st_ply_materialize fills a column with the read's values (then an ordinary host column:
    uploaded, so a change to it shows in the output); st_ply_forget drops one without copying"""
    src = str(tmp_path / 'in.ply')
    _ply(src, N, 12)
    ref = _read(ctx, src)
    cols = _read_resident(ctx, src)
    ctx.materialize(cols['f_rest_5'])
    ctx.materialize(cols['f_rest_5'])  # no-op the second time
    assert np.array_equal(cols['f_rest_5'].view(np.uint32), ref['f_rest_5'].view(np.uint32))
    ctx.forget(cols['y'])
    cols['y'][:] = ref['y']  # the caller's own values now
    cols['f_rest_5'][3] += np.float32(0.25)
    ref['f_rest_5'][3] += np.float32(0.25)
    out = str(tmp_path / 'out.sog')
    got, _, reuse = _file(ctx, cols, out, monkeypatch, True)
    assert reuse[0] == 57, reuse
    want, _, _ = _file(ctx, ref, out, monkeypatch, False)
    assert got == want


def test_resident_read_other_host_forms_copy_down_first(ctx, tmp_path, monkeypatch):
    """a host form other than writeSog's (st_transform in place, st_filter_nan) given unfilled
    resident columns reads the read's values (copied down first); the columns it wrote are the
    caller's afterwards, the untouched ones stay resident"""
    src = str(tmp_path / 'in.ply')
    _ply(src, N, 13)
    ref = _read(ctx, src)
    cols = _read_resident(ctx, src)
    kept = ctx.filter_nan([('opacity', cols['opacity'])])
    assert np.array_equal(kept[0][1].view(np.uint32), ref['opacity'].view(np.uint32))
    p = sh.transform_params((1.0, -2.0, 0.5), (0.0, 0.0, 0.0, 1.0), 2.0)
    moved = ('x', 'y', 'z', 'rot_0', 'rot_1', 'rot_2', 'rot_3', 'scale_0', 'scale_1', 'scale_2')
    ctx.transform({k: cols[k] for k in moved}, p)
    ctx.transform({k: ref[k] for k in moved}, p)
    for k in moved + ('opacity',):
        assert np.array_equal(cols[k].view(np.uint32), ref[k].view(np.uint32)), k
    out = str(tmp_path / 'out.sog')
    got, _, reuse = _file(ctx, cols, out, monkeypatch, True)
    assert reuse[0] == 59 - 11, reuse  # the ten transformed columns and the filtered opacity came down
    want, _, _ = _file(ctx, ref, out, monkeypatch, False)
    assert got == want


def test_resident_reads_keep_their_own_device_copies(ctx, tmp_path, monkeypatch):
    """each resident read's columns hold device blocks of their own: a second read (same element,
    another file) leaves the first table resident -- both run from HBM and give their own output;
    a forgotten table's blocks serve the next read"""
    a, b = str(tmp_path / 'a.ply'), str(tmp_path / 'b.ply')
    _ply(a, N, 14)
    _ply(b, N, 15)
    ra, rb = _read(ctx, a), _read(ctx, b)
    ca = _read_resident(ctx, a)
    cb = _read_resident(ctx, b)
    out = str(tmp_path / 'o.sog')
    ga, _, xa = _file(ctx, ca, out, monkeypatch, True)
    gb, _, xb = _file(ctx, cb, out, monkeypatch, True)
    assert xa[0] == 59 and xb[0] == 59, (xa, xb)
    wa, _, _ = _file(ctx, ra, out, monkeypatch, False)
    wb, _, _ = _file(ctx, rb, out, monkeypatch, False)
    assert ga == wa and gb == wb and ga != gb
    for k in ra:
        assert np.array_equal(ctx.materialize(ca[k]).view(np.uint32), ra[k].view(np.uint32)), k
    del cb  # its finalizers forget the columns: their blocks go to the pool
    cc = _read_resident(ctx, b)
    gc, _, xc = _file(ctx, cc, out, monkeypatch, True)
    assert xc[0] == 59 and gc == wb
