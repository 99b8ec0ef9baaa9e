"""The Node host side (splat-transform_amd/js + napi/addon.node): the reference's
function signatures over the C-ABI.  CPU: the addon loads, exports the entry
points, and fails loudly without a GPU (no CPU fallback).  GPU: the host module
driven like the reference's writers reproduces the oracle bit for bit."""
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADDON = os.path.join(ROOT, 'splat-transform_amd', 'napi', 'build', 'addon.node')
NODE = shutil.which('node')

pytestmark = pytest.mark.skipif(NODE is None, reason='node not installed')


@pytest.fixture(scope='module')
def addon_built():
    import splat_hip as sh
    if not os.path.exists(sh.LIB_PATH):
        sh.build()
    if not os.path.exists(ADDON):
        subprocess.check_call(['make', '-s', '-C', os.path.join(ROOT, 'splat-transform_amd', 'napi')])
    return ADDON


def node(script):
    return subprocess.run([NODE, '-e', script], cwd=ROOT, capture_output=True, text=True, timeout=120)


def test_addon_exports(addon_built):
    r = node("const h=require('./splat-transform_amd/js'); console.log(JSON.stringify(Object.keys(h.addon).sort()),"
             " h.addon.version())")
    assert r.returncode == 0, r.stderr
    keys, ver = r.stdout.strip().rsplit(' ', 1)
    assert json.loads(keys) == sorted(['version', 'deviceCount', 'quatFromEuler', 'transform', 'filterFinite',
                                       'filterNaN', 'combineLayout', 'setDevices', 'getDevices', 'mortonOrder', 'packCompressed', 'kmeans', 'cluster1d', 'sog',
                                       'webpLossless', 'sogBundle', 'readPly', 'decompressPly', 'compressedPly',
                                       'process', 'compressedPlyFromFile', 'sogBundleFromFile',
                                       'sogProcess', 'sogBundleProcess', 'transformTyped', 'mortonOrderTyped',
                                       'sogFile', 'rcclInfo', 'lastHostReuse', 'compressedPlyToFile',
                                       'compressedPlyTableToFile', 'materialize'])
    assert ver == '1'


def test_quat_from_euler_matches_oracle(addon_built):
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    r = node("const h=require('./splat-transform_amd/js'); console.log(JSON.stringify(h.quatFromEuler(10, 45, -30)))")
    assert r.returncode == 0, r.stderr
    q = json.loads(r.stdout)
    want = oracle.transform_params(euler=(10, 45, -30))['quat']
    assert [q['x'], q['y'], q['z'], q['w']] == list(want)


@pytest.mark.skipif(os.path.exists('/dev/kfd') and os.access('/dev/kfd', os.R_OK), reason='a GPU is present')
def test_no_cpu_fallback(addon_built):
    r = node("const h=require('./splat-transform_amd/js'); const t=new h.DataTable([new h.Column('x', new Float32Array(4))]);"
             " try { h.transform(t, {x:0,y:0,z:0}, {x:0,y:0,z:0,w:1}, 2); console.log('RAN') }"
             " catch (e) { console.log('THREW ' + e.message) }")
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith('THREW splat-hip:'), r.stdout


def _table_ops(what):
    r = subprocess.run([NODE, os.path.join(ROOT, 'tests', 'js', 'table_ops.js'), what], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout)


def test_js_combine_matches_reference(addon_built):
    """combine() (index.ts:158-210) through the addon's st_combine_layout: union by (name, type),
    duplicates of the first table kept, zero fill (host-only, no device)"""
    out = _table_ops('combine')
    assert out['names'] == ['x', 'id', 'x', 'w', 'id', 'q', 'w', 'b']
    assert all(out['same']) and all(out['same3']), out


@pytest.mark.gpu
def test_js_typed_columns_match_reference(addon_built):
    """columns that are not float32 through the Node host (processDataTable, writeCompressedPly,
    transform, writeSog's textures / meta / draws) against the reference's own outputs
    (tests/golden/typed_columns.*)"""
    r = subprocess.run([NODE, os.path.join(ROOT, 'tests', 'js', 'typed_columns.js')], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout)
    assert out.pop('transform_f64') is True
    bad = {c: [k for k, ok in v.items() if not ok] for c, v in out.items() if not all(v.values())}
    assert not bad, bad


@pytest.mark.gpu
def test_js_filter_nan_every_type_matches_reference(addon_built):
    """filterNaN through the addon (st_filter_nan): float64 columns tested, integer columns kept,
    each column's type preserved; the splat table too"""
    out = _table_ops('filter')
    assert all(out['same']) and all(out['same2']), out


@pytest.mark.gpu
def test_js_process_and_compressed_ply_match_reference(addon_built):
    """processDataTable (process.ts:64-145) and writeCompressedPly (write-compressed-ply.ts:31-115),
    alone and with the action list in the same device call, against the reference's writes:
    every action kind, header text included"""
    r = subprocess.run([NODE, os.path.join(ROOT, 'tests', 'js', 'process_chain.js')], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout)
    bad = {c: [k for k, ok in v.items() if not ok] for c, v in out.items() if not all(v.values())}
    assert not bad, bad


@pytest.mark.gpu
def test_js_set_devices(addon_built):
    """setDevices (st_set_devices): the GPU count writeSog shards over"""
    out = _table_ops('devices')
    assert out == {'before': 1, 'after': 1, 'threw': True}, out


@pytest.mark.gpu
def test_host_roundtrip_matches_oracle(addon_built, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    rng = np.random.default_rng(77)
    n, k, iters, seed = 20000, 256, 2, 91
    names = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] + \
        ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3']
    cols = {c: rng.normal(0, 1, n).astype(np.float32) for c in names}
    for i in range(45):
        cols[f'f_rest_{i}'] *= np.float32(0.1)
    for c in names:
        cols[c].tofile(tmp_path / f'{c}.f32')
    (tmp_path / 'manifest.json').write_text(json.dumps(
        {'columns': names, 'euler': [0, 45, 0], 'k': k, 'iters': iters, 'seed': seed}))
    r = subprocess.run([NODE, os.path.join(ROOT, 'tests', 'js', 'host_roundtrip.js'), str(tmp_path)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr

    ref = {c: v.copy() for c, v in cols.items()}
    oracle.transform(ref, oracle.transform_params(euler=(0, 45, 0)), 15)
    for c in names:
        got = np.fromfile(tmp_path / f't_{c}.f32', np.float32)
        assert np.array_equal(got.view(np.uint32), ref[c].view(np.uint32)), c
    order = oracle.morton_order(ref['x'], ref['y'], ref['z'])
    chunk, vertex, shb = oracle.pack_compressed(ref, order, 45)
    assert np.array_equal(np.fromfile(tmp_path / 'chunk.f32', np.float32).view(np.uint32), chunk.view(np.uint32))
    assert np.array_equal(np.fromfile(tmp_path / 'vertex.u32', np.uint32), vertex)
    assert np.array_equal(np.fromfile(tmp_path / 'sh.u8', np.uint8), shb)
    pts = [ref[f'f_rest_{i}'] for i in range(45)]
    rc, cen, labels, used = oracle.kmeans(pts, k, iters, oracle.mulberry32(seed, 1 << 16))
    assert rc == 0
    assert np.array_equal(np.fromfile(tmp_path / 'labels.u32', np.uint32), labels)
    assert np.array_equal(np.fromfile(tmp_path / 'centroids.f32', np.float32).view(np.uint32),
                          cen.reshape(-1).view(np.uint32))


@pytest.mark.gpu
def test_js_sog_bundle_matches_reference(addon_built, tmp_path):
    import io
    import struct
    import zipfile
    from PIL import Image
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import sog_container as oc
    from golden_io import Golden
    g = Golden('sog_bundle')
    c = next(c for c in g.meta['cases'] if c['name'] == 'b_sh1')
    cols = g.table('b_sh1_in_')
    for k, v in cols.items():
        v.astype(np.float32).tofile(tmp_path / f'{k}.f32')
    img = np.random.default_rng(3).integers(0, 256, (45, 67, 4), dtype=np.uint8)
    img.tofile(tmp_path / 'img.rgba')
    (tmp_path / 'manifest.json').write_text(json.dumps(
        {'columns': list(cols), 'seed': c['seed'], 'iters': c['iters'], 'clock': c['clock'], 'w': 67, 'h': 45}))
    r = subprocess.run([NODE, os.path.join(ROOT, 'tests', 'js', 'sog_bundle.js'), str(tmp_path)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    z = (tmp_path / 'out.sog').read_bytes()
    ref = zipfile.ZipFile(io.BytesIO(g['b_sh1_zip'].tobytes()))
    got = zipfile.ZipFile(io.BytesIO(z))
    assert got.testzip() is None
    assert [i.filename for i in got.infolist()] == [i.filename for i in ref.infolist()]
    assert [i.date_time for i in got.infolist()] == [i.date_time for i in ref.infolist()]
    assert got.read('meta.json') == ref.read('meta.json')
    for i in ref.infolist():
        if i.filename.endswith('.webp'):
            p = ref.read(i.filename)
            w, h, n = struct.unpack('<III', p[4:16])
            want = np.frombuffer(p[16:16 + n], np.uint8).reshape(h, w, 4)
            assert np.array_equal(np.array(Image.open(io.BytesIO(got.read(i.filename))).convert('RGBA')), want)
    t, d = oc.dos_clock(*c['clock'])
    assert oc.zip_store([(i.filename, got.read(i.filename)) for i in got.infolist()], t, d) == z
    dec = np.array(Image.open(tmp_path / 'img.webp').convert('RGBA'))
    assert np.array_equal(dec, img)


@pytest.mark.gpu
@pytest.mark.parametrize('resident', ['1', '0'])
def test_js_read_ply_and_decompress_match_reference(addon_built, tmp_path, resident):
    """readPly (resident columns copied down as JS reads them, or -- ST_READ_RESIDENT=0 -- filled by
    the read) and decompressPly against the reference's readers' outputs"""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from golden_io import Golden
    from test_ply_cpu import compressed_file
    g = Golden('ply_io')
    (tmp_path / 'mixed.ply').write_bytes(g['mixed_file'].tobytes())
    (tmp_path / 'comp.ply').write_bytes(compressed_file('sh3'))
    r = subprocess.run([NODE, os.path.join(ROOT, 'tests', 'js', 'ply_read.js'), str(tmp_path)],
                       capture_output=True, text=True, timeout=600, env=dict(os.environ, ST_READ_RESIDENT=resident))
    assert r.returncode == 0, r.stdout + r.stderr
    summ = json.loads((tmp_path / 'summary.json').read_text())
    assert summ['mixed']['comments'] == g.meta['mixed']['comments']
    assert not summ['mixed']['compressed'] and summ['comp']['compressed']
    for e in g.meta['mixed']['elements']:
        for k, _ in e['columns']:
            ref = g[f"mixed_{e['name']}_{k}"]
            got = np.fromfile(tmp_path / f"mixed_{e['name']}_{k}.bin", ref.dtype)
            assert np.array_equal(got.view(f'u{ref.dtype.itemsize}'), ref.view(f'u{ref.dtype.itemsize}')), k
    assert summ['comp']['decoded'] == g.meta['sh3_columns']
    for k in g.meta['sh3_columns']:
        ref = g[f'sh3_dec_{k}']
        got = np.fromfile(tmp_path / f'comp_dec_{k}.bin', np.float32)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k


@pytest.mark.gpu
def test_js_sog_file_equals_bundle(addon_built, tmp_path):
    """writeSogFile (st_sog_file: the .sog streamed into an open FileHandle while the SH k-means
    runs) writes exactly writeSogBundle's archive for the same table, draws and clock"""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from golden_io import Golden
    g = Golden('sog_bundle')
    c = next(c for c in g.meta['cases'] if c['name'] == 'b_sh1')
    cols = g.table('b_sh1_in_')
    for k, v in cols.items():
        v.astype(np.float32).tofile(tmp_path / f'{k}.f32')
    (tmp_path / 'manifest.json').write_text(json.dumps(
        {'columns': list(cols), 'seed': c['seed'], 'iters': c['iters'], 'clock': c['clock']}))
    for mode in ('file', 'bundle'):
        r = subprocess.run([NODE, os.path.join(ROOT, 'tests', 'js', 'sog_file.js'), str(tmp_path), mode],
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout + r.stderr
        assert f'sog {mode} ok' in r.stdout
    assert (tmp_path / 'out_file.sog').read_bytes() == (tmp_path / 'out_bundle.sog').read_bytes()


@pytest.mark.gpu
def test_js_resident_read_columns_through_write_sog_file(addon_built, tmp_path):
    """readPly leaves the columns in HBM (st_ply_read_resident) until JS reads a column's `data`:
    writeSogFile of an untouched table reads all 59 writeSog columns where they are, a table whose
    columns JS read or changed uploads exactly those columns -- every archive equal to the upload
    path's for the same values; two tables read from one file each keep their own device copy
    (tests/js/resident_read.js: same draws, pinned clock)"""
    sys.path.insert(0, ROOT)
    import bench
    n = 300_000
    cols = {k: v.numpy() for k, v in bench.synth_table(n, 4242, 'cpu').items()}
    src = tmp_path / 'in.ply'
    head = ('ply\nformat binary_little_endian 1.0\n' + f'element vertex {n}\n' +
            ''.join(f'property float {k}\n' for k in bench.PLY_ORDER) + 'end_header\n').encode()
    rows = np.stack([cols[k] if k in cols else np.zeros(n, np.float32) for k in bench.PLY_ORDER], 1)
    src.write_bytes(head + rows.astype('<f4').tobytes())
    r = subprocess.run([NODE, os.path.join(ROOT, 'tests', 'js', 'resident_read.js'), str(src), str(tmp_path), '3'],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    sha = out['untouched']['sha']
    assert out['untouched']['reused'] == 59, out
    assert out['read'] == {'sha': sha, 'reused': 0, 'finite': True}, out
    assert out['changed']['reused'] == 58 and out['changed_ref']['reused'] == 0, out
    assert out['changed']['sha'] == out['changed_ref']['sha'] != sha, out
    assert out['first'] == {'sha': sha, 'reused': 59} and out['second'] == {'sha': sha, 'reused': 59}, out
    assert out['meta'] == {'sha': sha, 'reused': 59} and out['numRows'] == n and out['columns'] == 62, out
    assert out['bundle'] == {'sha': sha, 'reused': 59}, out
    assert out['hasRot'], out
    got = np.fromfile(tmp_path / 'first_f_rest_44.bin', np.float32)
    assert np.array_equal(got.view(np.uint32), cols['f_rest_44'].view(np.uint32))
    got = np.fromfile(tmp_path / 'meta_x.bin', np.float32)
    assert np.array_equal(got.view(np.uint32), cols['x'].view(np.uint32))
