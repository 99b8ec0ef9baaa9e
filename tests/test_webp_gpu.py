"""The device WebP lossless encoder, CRC-32 and the .sog bundle.

WebP parity is at the decoded-pixel level: every stream must be a
valid lossless WebP that libwebp (Pillow) decodes to exactly the input RGBA.  The
bundle is compared with the reference's own .sog (tests/golden/sog_bundle.*):
same entries, order, flags, clock and meta.json bytes; each texture decodes to
the pixels the reference wrote (its payload in the fixture is the raw RGBA).
"""
import io
import struct
import zipfile
import zlib

import numpy as np
import pytest
import torch
from PIL import Image

import oracle
import sog_container as oc
import splat_hip as sh
from golden_io import Golden
from test_sog_container_cpu import _images

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    # one real stream shared by torch and the library (a NULL handle would select the
    # context's own stream, unordered with torch's copies)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    c = sh.Context(0)
    c.set_stream(s.cuda_stream)
    return c


def _decode(b):
    return np.array(Image.open(io.BytesIO(b)).convert('RGBA'))


def _dev_encode(ctx, img):
    d = torch.from_numpy(np.ascontiguousarray(img, np.uint8)).cuda()
    h, w = img.shape[:2]
    out = torch.empty(sh.webp_max_size(w, h), dtype=torch.uint8, device='cuda')
    n = ctx.dev_webp_lossless(d, out)
    return out[:n].cpu().numpy().tobytes()


@pytest.mark.parametrize('kind', list(_images().keys()))
def test_webp_roundtrip_small(ctx, kind):
    img = _images()[kind].astype(np.uint8)
    b = _dev_encode(ctx, img)
    assert b[:4] == b'RIFF' and b[8:16] == b'WEBPVP8L'
    assert struct.unpack('<I', b[4:8])[0] == len(b) - 8
    assert np.array_equal(_decode(b), img)
    # host form: identical stream
    assert ctx.webp_lossless(img) == b


def test_webp_roundtrip_sog_fixture_textures(ctx):
    g = Golden('sog')
    for case in g.meta['cases']:
        for f in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels'):
            key = f"{case['name']}_{f}"
            if key in g:
                img = g[key]
                assert np.array_equal(_decode(_dev_encode(ctx, img)), img), key


@pytest.mark.parametrize('shape', [(1, 16384), (16384, 2), (1531, 2049), (3164, 3164)])
def test_webp_roundtrip_large(ctx, shape):
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    h, w = shape
    # smooth high bytes + noisy low bytes, like the means textures
    y, x = np.mgrid[0:h, 0:w]
    img = np.stack([(x * 255 // max(w - 1, 1)), (y * 255 // max(h - 1, 1)), rng.integers(0, 256, (h, w)),
                    np.where(rng.random((h, w)) < 0.01, 0, 255)], -1).astype(np.uint8)
    assert np.array_equal(_decode(_dev_encode(ctx, img)), img)


def test_webp_rejects_bad_geometry(ctx):
    d = torch.zeros((4, 4, 4), dtype=torch.uint8, device='cuda')
    out = torch.empty(16, dtype=torch.uint8, device='cuda')  # below st_webp_max_size
    with pytest.raises(sh.StError):
        ctx.dev_webp_lossless(d, out)
    assert sh.webp_max_size(16385, 1) == 0


@pytest.mark.parametrize('n', [0, 1, 15, 16, 17, 4095, 4096, 4097, 1 << 20, 3_000_007])
def test_crc32_vs_zlib(ctx, n):
    rng = np.random.default_rng(n)
    a = rng.integers(0, 256, n + 1, dtype=np.uint8)
    d = torch.from_numpy(a).cuda()
    assert ctx.dev_crc32(d, n) == zlib.crc32(a[:n].tobytes())
    # unaligned start, and continuing from a running value (crc.ts update() twice)
    assert ctx.dev_crc32(d[1:], n) == zlib.crc32(a[1:n + 1].tobytes())
    c0 = zlib.crc32(b'splat')
    assert ctx.dev_crc32(d, n, crc_in=c0) == zlib.crc32(a[:n].tobytes(), c0)


def test_crc32_small_vs_oracle(ctx):
    a = np.frombuffer(b'The quick brown fox jumps over the lazy dog', np.uint8)
    assert ctx.dev_crc32(torch.from_numpy(a.copy()).cuda()) == oc.crc32(a.tobytes()) == 0x414FA339


def _payload_rgba(p):
    # the identity WebP stand-in of the fixture generator: 'RGBA', width, height, length, pixels
    assert p[:4] == b'RGBA'
    w, h, n = struct.unpack('<III', p[4:16])
    return np.frombuffer(p[16:16 + n], np.uint8).reshape(h, w, 4)


@pytest.mark.parametrize('name', ['b_sh1', 'b_sh0'])
def test_sog_bundle_vs_reference(ctx, name):
    g = Golden('sog_bundle')
    c = next(c for c in g.meta['cases'] if c['name'] == name)
    ref = zipfile.ZipFile(io.BytesIO(g[name + '_zip'].tobytes()))
    cols = g.table(name + '_in_')
    draws = oracle.mulberry32(c['seed'], c['draws'] + 64)
    t, d = oc.dos_clock(*c['clock'])
    z, used = ctx.sog_bundle(cols, c['iters'], draws, t, d)
    assert used == c['draws']
    got = zipfile.ZipFile(io.BytesIO(z))
    assert got.testzip() is None  # every CRC checks
    gi, ri = got.infolist(), ref.infolist()
    assert [i.filename for i in gi] == [i.filename for i in ri]
    for a, b in zip(gi, ri):
        assert (a.flag_bits, a.compress_type, a.date_time) == (b.flag_bits, b.compress_type, b.date_time)
    assert got.read('meta.json') == ref.read('meta.json')
    for i in ri:
        if i.filename.endswith('.webp'):
            assert np.array_equal(_decode(got.read(i.filename)), _payload_rgba(ref.read(i.filename))), i.filename
    # the archive is the reference's layout around our entries
    entries = [(i.filename, got.read(i.filename)) for i in gi]
    assert oc.zip_store(entries, t, d) == z


def test_sog_bundle_device_view_matches_copy(ctx):
    g = Golden('sog_bundle')
    c = next(c for c in g.meta['cases'] if c['name'] == 'b_sh1')
    cols = {k: torch.from_numpy(v).cuda() for k, v in g.table('b_sh1_in_').items()}
    draws = oracle.mulberry32(c['seed'], c['draws'] + 64)
    W, H, pal, cw, ch = sh.sog_geometry(c['n'], 3)
    u8 = dict(device='cuda', dtype=torch.uint8)
    tex = {k: torch.empty(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
    tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
    meta, used = ctx.dev_sog(cols, c['iters'], draws, tex)
    assert used == c['draws']
    t, d = oc.dos_clock(*c['clock'])
    z = ctx.dev_sog_bundle(meta, c['n'], tex, t, d)
    addr, size = ctx.dev_sog_bundle_view(meta, c['n'], tex, t, d)
    import ctypes
    assert ctypes.string_at(addr, size) == z
    host, _ = ctx.sog_bundle(g.table('b_sh1_in_'), c['iters'], draws, t, d)
    assert host == z


def _harness_encode(img, tmp_path):
    """the scalar emulation of the device kernels around the product's header code
    (tests/native/vp8l_cpu_check.cpp), choosing the colour cache the same way"""
    import subprocess
    from test_sog_container_cpu import _harness
    h, w = img.shape[:2]
    src, dst = tmp_path / 'in.rgba', tmp_path / 'out.webp'
    np.ascontiguousarray(img, np.uint8).tofile(src)
    r = subprocess.run([_harness(), str(src), str(w), str(h), str(dst)], capture_output=True, text=True, check=True)
    return dst.read_bytes(), int(r.stderr.split('cache_bits ')[1].split()[0])


def _palette_scene(h, w, seed):
    """runs of a few hundred repeating colours with smooth stretches between them: colour-cache
    hits whose last writer lies many 4,096-pixel groups (and scan chunks) back"""
    rng = np.random.default_rng(seed)
    pal = rng.integers(0, 256, (300, 4)).astype(np.uint8)
    pal[:, 3] = 255
    img = pal[rng.integers(0, 300, (h, w))]
    y, x = np.mgrid[0:h, 0:w]
    band = (y // 37) % 3 == 0
    img[band, 0] = (x[band] * 3) % 256
    img[band, 1] = (y[band] * 2) % 256
    rare = rng.random((h, w)) < 0.0005  # colours seen once, then again far later
    img[rare] = pal[0]
    return img


def test_webp_matches_scalar_emulation_with_colour_cache(ctx, tmp_path):
    """the device stream equals the scalar emulation byte for byte (the same predictors, copies,
    colour-cache hits across groups and scan chunks, cache size and prefix codes), and a cache is
    taken where colours repeat"""
    cases = dict(_images())
    cases['palette_scene'] = _palette_scene(700, 1000, 3)
    g = Golden('sog')
    for case in g.meta['cases']:
        for f in ('means_l', 'means_u', 'scales', 'shN_labels'):
            key = f"{case['name']}_{f}"
            if key in g:
                cases[key] = g[key]
    used = 0
    for name, img in cases.items():
        img = np.ascontiguousarray(img, np.uint8)
        want, bits = _harness_encode(img, tmp_path)
        got = _dev_encode(ctx, img)
        assert got == want, name
        assert np.array_equal(_decode(got), img), name
        used += bits > 0
    assert used >= 3
