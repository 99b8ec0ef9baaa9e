"""ctypes binding of oracle/build/libst_oracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference path (st_oracle.c) is the parity checker
for the MI355X product.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('ST_ORACLE_LIB') or os.path.join(HERE, 'build', 'libst_oracle.so')

_f32p = np.ctypeslib.ndpointer(np.float32, flags='C')
_lib = None


def build():
    subprocess.check_call(['make', '-s', '-C', HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c_d, c_u64, c_i = ctypes.c_double, ctypes.c_uint64, ctypes.c_int
        vp = ctypes.c_void_p
        L.st_o_exp.restype = c_d
        L.st_o_exp.argtypes = [c_d]
        L.st_o_log.restype = c_d
        L.st_o_log.argtypes = [c_d]
        for f in ('st_o_quat_from_euler', 'st_o_mat4_trs', 'st_o_mat3_from_quat', 'st_o_rotate_sh',
                  'st_o_transform', 'st_o_filter_finite', 'st_o_morton_order', 'st_o_pack_compressed',
                  'st_o_kmeans', 'st_o_cluster1d', 'st_o_sog', 'st_o_kmeans_assign_mt'):
            getattr(L, f).restype = c_i
        L.st_o_filter_finite.restype = c_u64
        L.st_o_quat_from_euler.argtypes = [c_d, c_d, c_d, vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def mulberry32(seed, n):
    """The Math.random replacement stream used by tests/golden/gen/make_golden.js."""
    i = np.arange(1, n + 1, dtype=np.uint64)
    a = ((np.uint64(seed) + i * np.uint64(0x6D2B79F5)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    with np.errstate(over='ignore'):
        t = (a ^ (a >> np.uint32(15))) * (a | np.uint32(1))
        t = t ^ (t + (t ^ (t >> np.uint32(7))) * (t | np.uint32(61)))
    return (t ^ (t >> np.uint32(14))).astype(np.float64) / 4294967296.0


def set_threads(threads):
    """OpenMP threads for the k-means assign loop (labels are those of the sequential loop)."""
    lib().st_o_set_threads(ctypes.c_int(threads))


def exp(x):
    return lib().st_o_exp(float(x))


def log(x):
    return lib().st_o_log(float(x))


def transform_params(t=(0.0, 0.0, 0.0), euler=None, quat=None, s=1.0):
    """PlayCanvas Mat4.setTRS / Mat3.setFromQuat / RotateSH as transform() builds them."""
    L = lib()
    q = np.array([0, 0, 0, 1], np.float64) if quat is None else np.asarray(quat, np.float64).copy()
    if euler is not None:
        L.st_o_quat_from_euler(float(euler[0]), float(euler[1]), float(euler[2]), _p(q))
    m4 = np.zeros(16, np.float32)
    m3 = np.zeros(9, np.float32)
    L.st_o_mat4_trs(_p(np.asarray(t, np.float64)), _p(q), ctypes.c_double(s), _p(m4))
    L.st_o_mat3_from_quat(_p(q), _p(m3))
    sh1, sh2, sh3 = np.zeros(9), np.zeros(25), np.zeros(49)
    L.st_o_rotate_sh(_p(m3), _p(sh1), _p(sh2), _p(sh3))
    return dict(quat=q, mat4=m4, mat3=m3, sh1=sh1, sh2=sh2, sh3=sh3, s=float(s))


def transform(cols, params, sh_coeffs):
    """In-place transform of a dict of float32 columns (transform.ts:12-65)."""
    L = lib()
    g = lambda k: cols.get(k)
    has = lambda ks: all(k in cols for k in ks)
    x = _p(g('x')) if has(('x', 'y', 'z')) else None
    y = _p(g('y')) if x else None
    z = _p(g('z')) if x else None
    rot = _ptrs([cols[f'rot_{i}'] for i in range(4)]) if has([f'rot_{i}' for i in range(4)]) else None
    sc = _ptrs([cols[f'scale_{i}'] for i in range(3)]) if has([f'scale_{i}' for i in range(3)]) else None
    sh = _ptrs([cols[f'f_rest_{i}'] for i in range(sh_coeffs * 3)]) if sh_coeffs else None
    n = len(next(iter(cols.values())))
    L.st_o_transform(ctypes.c_uint64(n), x, y, z, rot, sc, sh, ctypes.c_int(sh_coeffs), _p(params['mat4']),
                     _p(params['quat']), ctypes.c_double(params['s']), _p(params['sh1']), _p(params['sh2']),
                     _p(params['sh3']))


def filter_finite(col_list):
    n = len(col_list[0])
    out = np.zeros(n, np.uint32)
    m = lib().st_o_filter_finite(ctypes.c_uint64(n), ctypes.c_int(len(col_list)), _ptrs(col_list), _p(out))
    return out[:m]


def morton_order(x, y, z, indices=None):
    n = len(x)
    idx = np.arange(n, dtype=np.uint32) if indices is None else np.ascontiguousarray(indices, np.uint32).copy()
    lib().st_o_morton_order(_p(x), _p(y), _p(z), _p(idx), ctypes.c_uint64(len(idx)))
    return idx


MEMBERS = ['x', 'y', 'z', 'scale_0', 'scale_1', 'scale_2', 'f_dc_0', 'f_dc_1', 'f_dc_2', 'opacity',
           'rot_0', 'rot_1', 'rot_2', 'rot_3']


def pack_compressed(cols, order, nsh):
    n = len(order)
    nch = (n + 255) // 256
    chunk = np.zeros(nch * 18, np.float32)
    vertex = np.zeros(n * 4, np.uint32)
    sh = np.zeros(n * nsh, np.uint8)
    shc = [cols[f'f_rest_{k}'] for k in range(nsh)]
    lib().st_o_pack_compressed(ctypes.c_uint64(n), _ptrs([cols[m] for m in MEMBERS]),
                               _ptrs(shc) if nsh else None, ctypes.c_int(nsh), _p(order), _p(chunk),
                               _p(vertex), _p(sh))
    return chunk, vertex, sh


def kmeans(col_list, k, iters, draws):
    d = len(col_list)
    n = len(col_list[0])
    kk = k if n >= k else n
    cent = np.zeros(d * kk, np.float32)
    labels = np.zeros(n, np.uint32)
    used = ctypes.c_uint64(0)
    rc = lib().st_o_kmeans(_ptrs(col_list), ctypes.c_int(d), ctypes.c_uint64(n), ctypes.c_int(k),
                           ctypes.c_int(iters), _p(draws), ctypes.c_uint64(len(draws)), ctypes.byref(used),
                           _p(cent), _p(labels))
    return rc, cent.reshape(d, kk), labels, used.value


def kmeans_assign(col_list, centroids, threads=1):
    """centroids: (d, k) float32; threads > 1 splits the points over OpenMP threads"""
    d, n = len(col_list), len(col_list[0])
    cen = np.ascontiguousarray(centroids, np.float32)
    labels = np.zeros(n, np.uint32)
    if threads > 1:
        rc = lib().st_o_kmeans_assign_mt(_ptrs(col_list), ctypes.c_int(d), ctypes.c_uint64(n), _p(cen),
                                         ctypes.c_int(cen.shape[1]), _p(labels), ctypes.c_int(threads))
    else:
        rc = lib().st_o_kmeans_assign(_ptrs(col_list), ctypes.c_int(d), ctypes.c_uint64(n), _p(cen),
                                      ctypes.c_int(cen.shape[1]), _p(labels))
    return rc, labels


def cluster1d(col_list, iters, draws):
    n = len(col_list[0])
    cent = np.zeros(256, np.float32)
    labels = np.zeros(n * len(col_list), np.uint8)
    used = ctypes.c_uint64(0)
    rc = lib().st_o_cluster1d(_ptrs(col_list), ctypes.c_int(len(col_list)), ctypes.c_uint64(n),
                              ctypes.c_int(iters), _p(draws), ctypes.c_uint64(len(draws)), ctypes.byref(used),
                              _p(cent), _p(labels))
    return rc, cent, labels.reshape(len(col_list), n), used.value


class SogMeta(ctypes.Structure):
    _fields_ = [('width', ctypes.c_int), ('height', ctypes.c_int),
                ('means_min', ctypes.c_double * 3), ('means_max', ctypes.c_double * 3),
                ('scales_codebook', ctypes.c_float * 256), ('sh0_codebook', ctypes.c_float * 256),
                ('sh_bands', ctypes.c_int), ('palette_size', ctypes.c_int),
                ('shn_codebook', ctypes.c_float * 256), ('shn_width', ctypes.c_int), ('shn_height', ctypes.c_int)]


def sog(cols, sh_coeffs, iters, draws):
    n = len(cols['x'])
    w = int(np.ceil(np.sqrt(n) / 4) * 4)
    h = int(np.ceil(n / w / 4) * 4)
    tex = {k: np.zeros(w * h * 4, np.uint8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
    pal = 65536
    cent = np.zeros(64 * max(sh_coeffs, 1) * ((pal + 63) // 64) * 4, np.uint8)
    meta = SogMeta()
    used = ctypes.c_uint64(0)
    shc = [cols[f'f_rest_{k}'] for k in range(3 * sh_coeffs)]
    rc = lib().st_o_sog(ctypes.c_uint64(n), _ptrs([cols[m] for m in MEMBERS]), _ptrs(shc) if sh_coeffs else None,
                        ctypes.c_int(sh_coeffs), ctypes.c_int(iters), _p(draws), ctypes.c_uint64(len(draws)),
                        ctypes.byref(used), ctypes.byref(meta), _p(tex['means_l']), _p(tex['means_u']),
                        _p(tex['quats']), _p(tex['scales']), _p(tex['sh0']), _p(cent), _p(tex['shN_labels']))
    out = {k: v.reshape(h, w, 4) for k, v in tex.items()}
    if sh_coeffs:
        out['shN_centroids'] = cent[:meta.shn_width * meta.shn_height * 4].reshape(meta.shn_height, meta.shn_width, 4)
    else:
        del out['shN_labels']
    return rc, out, meta, used.value


CHUNK_COLS = ['min_x', 'min_y', 'min_z', 'max_x', 'max_y', 'max_z', 'min_scale_x', 'min_scale_y', 'min_scale_z',
              'max_scale_x', 'max_scale_y', 'max_scale_z', 'min_r', 'min_g', 'min_b', 'max_r', 'max_g', 'max_b']
VERTEX_COLS = ['packed_position', 'packed_rotation', 'packed_scale', 'packed_color']
DECOMP_COLS = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2', 'opacity', 'rot_0', 'rot_1', 'rot_2', 'rot_3',
               'scale_0', 'scale_1', 'scale_2']


def decompress_ply(chunk, vertex, sh):
    """decompressPly (decompress-ply.ts:82-232) -> dict of float32 columns"""
    n = len(vertex['packed_position'])
    ch = [np.ascontiguousarray(chunk[k], np.float32) for k in CHUNK_COLS]
    vx = [np.ascontiguousarray(vertex[k], np.uint32) for k in VERTEX_COLS]
    sv = [np.ascontiguousarray(a, np.uint8) for a in sh]
    names = DECOMP_COLS + [f'f_rest_{i}' for i in range(len(sv))]
    out = {k: np.empty(n, np.float32) for k in names}
    lib().st_o_decompress_ply(ctypes.c_uint64(n), _ptrs(ch), _ptrs(vx), _ptrs(sv) if sv else None,
                              ctypes.c_int(len(sv)), _ptrs([out[k] for k in names]))
    return out



# ---- whole-table row operations on typed columns (numpy restatement) -----------------
def combine(tables):
    """combine (index.ts:158-210): tables are lists of (name, array).  Result columns: the first
    table's, then each later column whose (name, dtype) is not yet present; rows appended in
    table order; each source column lands in the FIRST result column of its (name, dtype);
    the rest stays zero."""
    if len(tables) == 1:
        return list(tables[0])
    cols = list(tables[0])
    for t in tables[1:]:
        for name, a in t:
            if not any(n == name and b.dtype == a.dtype for n, b in cols):
                cols.append((name, a))
    total = sum(len(t[0][1]) for t in tables)
    out = [(name, np.zeros(total, a.dtype)) for name, a in cols]
    off = 0
    for t in tables:
        for name, a in t:
            tgt = next(b for n, b in out if n == name and b.dtype == a.dtype)
            tgt[off:off + len(a)] = a
        off += len(t[0][1])
    return out


def filter_nan(cols):
    """filterNaN (process.ts:84-95 -> filter :47-61 -> permuteRows data-table.ts:135-149): keep a row
    iff isFinite holds for every column value (always for integer columns)"""
    n = len(cols[0][1])
    keep = np.ones(n, bool)
    for _, a in cols:
        if a.dtype.kind == 'f':
            keep &= np.isfinite(a)
    idx = np.nonzero(keep)[0].astype(np.uint32)
    return [(name, a[idx]) for name, a in cols], idx


def _band_coeffs(names):
    """{ '9': 1, '24': 2, '-1': 3 }[index of the first missing f_rest_i] ?? 0, as coefficients"""
    first_missing = next((i for i in range(45) if f'f_rest_{i}' not in names), -1)
    return {9: 3, 24: 8, -1: 15}.get(first_missing, 0)


def process(cols, actions):
    """processDataTable (process.ts:64-145) over a list of (name, array): actions are dicts with
    'kind' translate / rotate (Euler degrees) / scale / filterNaN / filterByValue (columnName,
    comparator, value) / filterBands (value) / param.  transform() runs in the C restatement on
    the float32 columns; the filters are numpy predicates + the permuteRows gather; filterBands
    renames / drops f_rest columns against the ORIGINAL table's band (process.ts:111)."""
    cols = [(k, np.array(a, copy=True)) for k, a in cols]
    in_coeffs = _band_coeffs([k for k, _ in cols])
    for act in actions:
        kind = act['kind']
        if kind in ('translate', 'rotate', 'scale'):
            v = act['value']
            p = (transform_params(t=v) if kind == 'translate' else
                 transform_params(euler=v) if kind == 'rotate' else transform_params(s=float(v)))
            f32 = {k: a for k, a in cols if a.dtype == np.float32}
            if f32:
                transform(f32, p, _band_coeffs(list(f32)))
        elif kind == 'filterNaN':
            cols, _ = filter_nan(cols)
        elif kind == 'filterByValue':
            n = len(cols[0][1]) if cols else 0
            col = next((a for k, a in cols if k == act['columnName']), None)
            x = np.full(n, np.nan) if col is None else col.astype(np.float64)
            v = float(act['value'])
            with np.errstate(invalid='ignore'):
                keep = {'lt': lambda: x < v, 'lte': lambda: x <= v, 'gt': lambda: x > v, 'gte': lambda: x >= v,
                        'eq': lambda: x == v, 'neq': lambda: ~(x == v)}.get(act['comparator'],
                                                                          lambda: np.ones(n, bool))()
            idx = np.nonzero(keep)[0]
            cols = [(k, a[idx]) for k, a in cols]
        elif kind == 'filterBands':
            out_coeffs = [0, 3, 8, 15][act['value']]
            if out_coeffs < in_coeffs:
                mp = {}
                for i in range(in_coeffs):
                    for j in range(3):
                        mp[f'f_rest_{i + j * in_coeffs}'] = f'f_rest_{i + j * out_coeffs}' if i < out_coeffs else None
                cols = [(mp.get(k, k), a) for k, a in cols if k not in mp or mp[k] is not None]
        elif kind != 'param':
            raise ValueError(kind)
    return cols


def compressed_ply(cols, actions):
    """processDataTable then writeCompressedPly's arrays (write-compressed-ply.ts:31-115):
    (processed table, chunk, vertex, sh)"""
    out = process(cols, actions)
    d = dict(out)
    nsh = 3 * _band_coeffs([k for k, _ in out])
    order = morton_order(d['x'], d['y'], d['z'])
    return (out,) + tuple(pack_compressed(d, order, nsh))
