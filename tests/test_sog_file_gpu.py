"""writeSog into a file with the archive streamed (st_dev_sog_file; write-sog.ts:110-370 and the
CLI's write of the .sog): the file holds exactly the archive st_dev_sog_bundle builds from the
same step's textures, the textures equal st_dev_sog's, for SH-3 and SH-0 tables; a failing write
(a descriptor opened read-only) is reported, not hung on."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    import torch

    import splat_hip as sh
    c = sh.Context(0)
    c.bind_torch_stream(torch.device('cuda', 0))
    yield c
    c.close()


def _textures(sh, n, C, dev):
    import torch
    W, H, pal, cw, ch = sh.sog_geometry(n, C)
    u8 = dict(device=dev, dtype=torch.uint8)
    tex = {k: torch.zeros(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0')}
    if C:
        tex['shN_labels'] = torch.zeros(W * H * 4, **u8)
        tex['shN_centroids'] = torch.zeros(cw * ch * 4, **u8)
    return tex


@pytest.mark.parametrize('n,C', [(300_000, 15), (70_000, 0)])
def test_sog_file_equals_the_bundle(ctx, tmp_path, n, C):
    import torch

    import bench
    import splat_hip as sh
    dev = torch.device('cuda', 0)
    cols = bench.synth_table(n, 31 + C, dev)
    if not C:
        cols = {k: v for k, v in cols.items() if not k.startswith('f_rest')}
    draws = np.random.default_rng(3).random(2 * 65536 * 8)
    tex = _textures(sh, n, C, dev)
    path = str(tmp_path / 'out.sog')
    meta, used, size = ctx.dev_sog_file(cols, 5, draws, tex, path, 0x6a2b, 0x58b1)
    data = open(path, 'rb').read()
    assert len(data) == size
    assert ctx.dev_sog_bundle(meta, n, tex, 0x6a2b, 0x58b1) == data
    ref = _textures(sh, n, C, dev)
    meta2, used2 = ctx.dev_sog(cols, 5, draws, ref)
    assert used2 == used and meta2.palette_size == meta.palette_size
    for k in tex:
        assert torch.equal(tex[k], ref[k]), k


def test_sog_file_write_error_is_reported(ctx, tmp_path):
    """a descriptor that takes writes but fails them (/dev/full: ENOSPC) ends the call with
    ST_ERR_ARG 'write failed' after the step, and the context still works afterwards"""
    import torch

    import bench
    import splat_hip as sh
    if not os.path.exists('/dev/full'):
        pytest.skip('no /dev/full')
    dev = torch.device('cuda', 0)
    n = 70_000
    cols = bench.synth_table(n, 5, dev)
    tex = _textures(sh, n, 15, dev)
    draws = np.random.default_rng(3).random(2 * 65536 * 8)
    fd = os.open('/dev/full', os.O_WRONLY)
    try:
        rc, _ = _sog_file_fd(ctx, cols, tex, draws, fd)
    finally:
        os.close(fd)
    assert rc == sh.ST_ERR_ARG and b'write failed' in sh.lib().st_last_error()
    meta, used, size = ctx.dev_sog_file(cols, 2, draws, tex, str(tmp_path / 'ok.sog'))
    assert size == os.path.getsize(str(tmp_path / 'ok.sog'))


@pytest.mark.parametrize('flags,msg', [(os.O_RDONLY, b'open for writing'),
                                       (os.O_WRONLY | os.O_APPEND, b'O_APPEND')], ids=['rdonly', 'append'])
def test_sog_file_refuses_unusable_descriptors_up_front(ctx, tmp_path, flags, msg):
    """pwrite on an O_APPEND descriptor ignores the offset (Linux) and a read-only one fails only
    at the first write: both are refused with ST_ERR_ARG before any work, the file untouched"""
    import torch

    import bench
    import splat_hip as sh
    dev = torch.device('cuda', 0)
    n = 20_000
    cols = bench.synth_table(n, 5, dev)
    tex = _textures(sh, n, 15, dev)
    draws = np.random.default_rng(3).random(2 * 65536 * 8)
    path = str(tmp_path / 'x.sog')
    open(path, 'wb').write(b'keep')
    fd = os.open(path, flags)
    try:
        rc, _ = _sog_file_fd(ctx, cols, tex, draws, fd)
    finally:
        os.close(fd)
    assert rc == sh.ST_ERR_ARG and msg in sh.lib().st_last_error()
    assert open(path, 'rb').read() == b'keep'


def _sog_file_fd(ctx, cols, tex, draws, fd, iters=2):
    import ctypes

    import splat_hip as sh
    t = sh.make_table(cols)
    out = sh.SogTextures(*[(tex[k].data_ptr() if k in tex else None) for k in
                           ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels')])
    meta, used, size = sh.SogMeta(), ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = sh.lib().st_dev_sog_file(ctx.h, ctypes.byref(t), ctypes.c_int32(iters), sh._vp(draws),
                                  ctypes.c_uint64(len(draws)), ctypes.byref(used), ctypes.byref(meta),
                                  ctypes.byref(out), ctypes.c_int32(fd), ctypes.c_uint16(0), ctypes.c_uint16(0),
                                  ctypes.byref(size))
    return rc, size.value


def test_sog_file_needs_a_seekable_descriptor(ctx, tmp_path):
    """the archive goes out at absolute offsets: a pipe is refused before any work (ST_ERR_ARG,
    'seekable'), as a negative descriptor is"""
    import torch

    import bench
    import splat_hip as sh
    dev = torch.device('cuda', 0)
    n = 70_000
    cols = bench.synth_table(n, 5, dev)
    tex = _textures(sh, n, 15, dev)
    draws = np.random.default_rng(3).random(2 * 65536 * 8)
    r, w = os.pipe()
    try:
        rc, _ = _sog_file_fd(ctx, cols, tex, draws, w)
    finally:
        os.close(r)
        os.close(w)
    assert rc == sh.ST_ERR_ARG and b'seekable' in sh.lib().st_last_error()
    rc, _ = _sog_file_fd(ctx, cols, tex, draws, -1)
    assert rc == sh.ST_ERR_ARG


def test_sog_file_over_a_longer_file_is_cut_to_the_archive(ctx, tmp_path):
    """a descriptor opened without O_TRUNC on a longer file: the file ends where the archive does
    (a zip reader looks for the end record from the end of the file)"""
    import io
    import zipfile

    import torch

    import bench
    import splat_hip as sh
    dev = torch.device('cuda', 0)
    n = 70_000
    cols = bench.synth_table(n, 5, dev)
    tex = _textures(sh, n, 15, dev)
    draws = np.random.default_rng(3).random(2 * 65536 * 8)
    path = str(tmp_path / 'old.sog')
    with open(path, 'wb') as f:
        f.write(b'\xab' * (8 << 20))  # longer than the archive
    fd = os.open(path, os.O_WRONLY)
    try:
        rc, size = _sog_file_fd(ctx, cols, tex, draws, fd)
    finally:
        os.close(fd)
    assert rc == 0 and os.path.getsize(path) == size < (8 << 20)
    data = open(path, 'rb').read()
    assert len(zipfile.ZipFile(io.BytesIO(data)).namelist()) == 8


_GROUP_FILE = r'''
import ctypes, io, os, sys, zipfile
import numpy as np
sys.path.insert(0, sys.argv[1])
import splat_hip as sh
n = 30_011
rng = np.random.default_rng(8)
cols = {k: rng.normal(0, 1, n).astype(np.float32) for k in
        ['x', 'y', 'z', 'scale_0', 'scale_1', 'scale_2', 'f_dc_0', 'f_dc_1', 'f_dc_2', 'opacity',
         'rot_0', 'rot_1', 'rot_2', 'rot_3'] + ['f_rest_%d' % i for i in range(9)]}
draws = np.random.default_rng(9).random(1 << 18)
ctx = sh.Context(0)
path = sys.argv[2]
with open(path, 'wb') as f:
    f.write(b'\xee' * (8 << 20))  # a longer earlier file: no O_TRUNC below
fd = os.open(path, os.O_WRONLY)
t = sh.make_table(cols)
used, size = ctypes.c_uint64(0), ctypes.c_uint64(0)
try:
    sh.check(sh.lib().st_sog_file(ctx.h, ctypes.byref(t), ctypes.c_int32(2), sh._vp(draws), ctypes.c_uint64(len(draws)),
                                  ctypes.byref(used), ctypes.c_int32(fd), ctypes.c_uint16(0), ctypes.c_uint16(0),
                                  ctypes.byref(size)))
finally:
    os.close(fd)
got = open(path, 'rb').read()
assert len(got) == size.value, (len(got), size.value)
assert len(zipfile.ZipFile(io.BytesIO(got)).namelist()) == 8
n_dev = ctypes.c_int32(0)
sh.check(sh.lib().st_get_devices(ctypes.byref(n_dev)))
print('ranks', n_dev.value, 'bytes', size.value, 'used', used.value, 'digest', __import__('hashlib').sha256(got).hexdigest())
'''


def test_sog_file_group_branch_cuts_a_longer_file(tmp_path):
    """st_sog_file's multi-GPU branch (the default group; ST_DEFAULT_GROUP_RANKS=2 makes it two
    host-staged ranks on this one GPU): the group's archive written over a longer existing file
    opened without O_TRUNC is cut to its length, a valid 8-entry zip, the same bytes as the one-GPU
    branch writes"""
    import subprocess
    import sys
    py = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'splat-transform_amd', 'py')
    out = {}
    for ranks in ('2', ''):
        env = dict(os.environ, ST_DEFAULT_GROUP_RANKS=ranks)
        r = subprocess.run([sys.executable, '-c', _GROUP_FILE, py, str(tmp_path / f'g{ranks}.sog')],
                           capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        out[ranks] = r.stdout.split()
    assert out['2'][1] == '2' and out[''][1] == '1'
    assert out['2'][3:] == out[''][3:]  # bytes, draws used and digest
