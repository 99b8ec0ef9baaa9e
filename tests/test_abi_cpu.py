"""CPU-side checks of the product library: it loads, exports every symbol the
C-ABI header declares, and its host-only constants (PlayCanvas math restated,
RotateSH matrices, SOG geometry) match the reference's golden vectors.
No compute call that needs a GPU is made here."""
import os
import re

import numpy as np
import pytest

import splat_hip as sh
from golden_io import Golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, 'include', 'st_abi.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(st_[a-z0-9_]+)\s*\(', src)))


@pytest.fixture(scope='module')
def L():
    if not os.path.exists(sh.LIB_PATH):
        sh.build()
    return sh.lib()


def test_library_exports_every_declared_symbol(L):
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(sh.EXPORTS)
    assert L.st_abi_version() == 1


def test_library_is_gfx950_code_object(L):
    blob = open(sh.LIB_PATH, 'rb').read()
    assert b'amdgcn-amd-amdhsa--gfx950' in blob


def test_quat_and_transform_params_match_reference(L):
    g = Golden('transform')
    for li, acts in enumerate(g.meta['actions']):
        for ai, act in enumerate(acts):
            p = sh.action_params(act['kind'], act['value'])
            q = np.array(p.r[:])
            assert np.array_equal(q.view(np.uint64), g[f'p{li}_{ai}_quat'].view(np.uint64))
            assert np.array_equal(np.array(p.m4[:], np.float32).view(np.uint32), g[f'p{li}_{ai}_mat4'].view(np.uint32))
            rot = g[f'p{li}_{ai}_shrot']
            assert np.array_equal(np.array(p.sh1[:]), rot[0:3, 0:3].ravel())
            assert np.array_equal(np.array(p.sh2[:]), rot[3:8, 3:8].ravel())
            assert np.array_equal(np.array(p.sh3[:]), rot[8:15, 8:15].ravel())


def test_sog_geometry_matches_reference(L):
    g = Golden('sog')
    for case in g.meta['cases']:
        n = case['n']
        name = case['name']
        C = {'sh0': 0, 'sh1': 3, 'sh2': 8, 'sh3': 15}[name]
        W, H, pal, cw, ch = sh.sog_geometry(n, C)
        assert g[f'{name}_means_l'].shape == (H, W, 4)
        if C:
            assert pal == case['meta']['shN']['count']
            assert g[f'{name}_shN_centroids'].shape == (ch, cw, 4)
    # paletteSize = min(64, 2^floor(log2(n/1024))) * 1024
    for n, want in [(1024, 1024), (2047, 1024), (2048, 2048), (65535, 32768), (65536, 65536), (10**7, 65536),
                    (700, 512), (1, 1)]:
        assert sh.sog_geometry(n, 15)[2] == want, n


def test_context_without_gpu_fails_loudly(L):
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(sh.StError):
        sh.Context(0)


def test_set_stream_refuses_handle_zero():
    """torch's legacy default stream has handle 0, which the C ABI reads as NULL (the context's own
    non-blocking stream): the wrapper refuses it rather than silently unordering the library
    against the caller's torch work (a race found when the inputs were made on the default stream)"""
    c = object.__new__(sh.Context)
    for h in (0, None):
        with pytest.raises(ValueError, match='own stream'):
            c.set_stream(h)


def _get_devices_with_env(value):
    """st_get_devices in a fresh process with ST_NUM_GPUS set (the switch applies once per process)"""
    import subprocess
    import sys
    code = ('import ctypes, sys; sys.path.insert(0, %r); import splat_hip as sh; L = sh.lib(); '
            'n = ctypes.c_int32(); rc = L.st_get_devices(ctypes.byref(n)); '
            'print(rc, n.value, L.st_last_error().decode())' % os.path.join(ROOT, 'splat-transform_amd', 'py'))
    env = dict(os.environ, ST_NUM_GPUS=value)
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    rc, n, msg = r.stdout.strip().split(' ', 2) + [''] * (3 - len(r.stdout.strip().split(' ', 2)))
    return int(rc), int(n), msg


def test_st_num_gpus_rejects_a_bad_value():
    """ST_NUM_GPUS: a value that is not a device count fails loudly, before any device call"""
    rc, n, msg = _get_devices_with_env('two')
    assert rc == sh.ST_ERR_ARG and n == 0 and 'ST_NUM_GPUS' in msg
    rc, _, msg = _get_devices_with_env('0')
    assert rc == sh.ST_ERR_ARG and 'ST_NUM_GPUS' in msg


def _rccl_python(env_value=None, torch_first=True):
    """st_rccl_info in a fresh Python process (torch imported first, as the bench does)"""
    import json
    import subprocess
    import sys
    code = (('import torch; ' if torch_first else '') +
            'import json, sys; sys.path.insert(0, %r); import splat_hip as sh; '
            'print(json.dumps(sh.rccl_info()))' % os.path.join(ROOT, 'splat-transform_amd', 'py'))
    env = dict(os.environ)
    env.pop('ST_RCCL', None)
    if env_value is not None:
        env['ST_RCCL'] = env_value
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return tuple(json.loads(r.stdout.strip().splitlines()[-1]))


def test_rccl_is_the_same_file_under_python_and_node():
    """the library binds RCCL at run time by path (st_rccl.h): under the Python host -- where torch
    has already mapped its own librccl.so.1 (2.26.x) -- and under the Node host (no torch) the
    collectives run on the same file, /opt/rocm/lib/librccl.so.1, and report the same version"""
    import shutil
    import subprocess
    v, path = _rccl_python()
    assert os.path.realpath(path) == os.path.realpath('/opt/rocm/lib/librccl.so.1'), path
    assert v >= 22700, v
    node = shutil.which('node')
    addon = os.path.join(ROOT, 'splat-transform_amd', 'napi', 'build', 'addon.node')
    if not node or not os.path.exists(addon):
        pytest.skip('node or the N-API addon absent')
    js = ("const h = require(%r); console.log(JSON.stringify(h.rcclInfo()));" %
          os.path.join(ROOT, 'splat-transform_amd', 'js'))
    env = dict(os.environ)
    env.pop('ST_RCCL', None)
    r = subprocess.run([node, '-e', js], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    nj = json.loads(r.stdout.strip().splitlines()[-1])
    assert (nj['version'], nj['path']) == (v, path)


def test_rccl_process_mode_binds_the_loaded_copy():
    """ST_RCCL=process: the copy of soname librccl.so.1 already in the process (torch's), the
    binding before round 6 -- a different version than the ROCm install's"""
    import torch
    v, path = _rccl_python('process')
    assert os.path.realpath(path) == os.path.realpath(os.path.join(os.path.dirname(torch.__file__), 'lib',
                                                                   'librccl.so'))
    assert v != _rccl_python()[0]


def test_rccl_bad_path_fails_loudly():
    import subprocess
    import sys
    code = ('import sys; sys.path.insert(0, %r); import splat_hip as sh\n'
            'try:\n    sh.rccl_info(); print("loaded")\nexcept sh.StError as e:\n    print("error", e)'
            % os.path.join(ROOT, 'splat-transform_amd', 'py'))
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True,
                       env=dict(os.environ, ST_RCCL='/nonexistent/librccl.so.1'), timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith('error') and 'ST_RCCL' in r.stdout, r.stdout
