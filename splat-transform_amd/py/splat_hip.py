"""ctypes binding of libsplat_hip.so (the C-ABI in include/st_abi.h).

Used by the tests, bench.py and __graft_entry__.  Host-array entry points take
numpy arrays; ``dev_*`` entry points take torch CUDA (HIP) tensors and pass
their device pointers, running on torch's current stream.  There is no CPU
fallback: constructing a Context without a gfx950 device raises.
"""
import ctypes
import weakref
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
# ST_LIB overrides the library path (kernel-variant experiments under tools/)
LIB_PATH = os.environ.get('ST_LIB') or os.path.join(PKG, 'lib', 'libsplat_hip.so')

ST_OK = 0
ST_ERR_ARG, ST_ERR_HIP, ST_ERR_NONFINITE, ST_ERR_DRAWS = -1, -2, -3, -4
_lib = None


class StError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f'st error {code}: {msg}')
        self.code = code


class Table(ctypes.Structure):
    _fields_ = [('n', ctypes.c_uint64), ('ncol', ctypes.c_int32),
                ('names', ctypes.POINTER(ctypes.c_char_p)), ('cols', ctypes.POINTER(ctypes.c_void_p))]


class TTable(ctypes.Structure):
    _fields_ = [('n', ctypes.c_uint64), ('ncol', ctypes.c_int32), ('names', ctypes.POINTER(ctypes.c_char_p)),
                ('types', ctypes.POINTER(ctypes.c_int32)), ('cols', ctypes.POINTER(ctypes.c_void_p))]


class TransformParams(ctypes.Structure):
    _fields_ = [('m4', ctypes.c_float * 16), ('r', ctypes.c_double * 4), ('s', ctypes.c_double),
                ('sh1', ctypes.c_double * 9), ('sh2', ctypes.c_double * 25), ('sh3', ctypes.c_double * 49)]


class SogMeta(ctypes.Structure):
    _fields_ = [('width', ctypes.c_int32), ('height', ctypes.c_int32),
                ('means_min', ctypes.c_double * 3), ('means_max', ctypes.c_double * 3),
                ('scales_codebook', ctypes.c_float * 256), ('sh0_codebook', ctypes.c_float * 256),
                ('sh_bands', ctypes.c_int32), ('palette_size', ctypes.c_int32),
                ('shn_codebook', ctypes.c_float * 256), ('shn_width', ctypes.c_int32), ('shn_height', ctypes.c_int32)]


class SogTextures(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in
                ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shn_centroids', 'shn_labels')]


class Action(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('compare', ctypes.c_int32), ('column', ctypes.c_char_p),
                ('value', ctypes.c_double), ('bands', ctypes.c_int32), ('transform', TransformParams)]


ACTION_TRANSFORM, ACTION_FILTER_NAN, ACTION_FILTER_VALUE, ACTION_FILTER_BANDS, ACTION_PARAM = 1, 2, 3, 4, 5
COMPARE = {'lt': 0, 'lte': 1, 'gt': 2, 'gte': 3, 'eq': 4, 'neq': 5}


PLY_TYPES = {1: ('char', np.int8), 2: ('uchar', np.uint8), 3: ('short', np.int16), 4: ('ushort', np.uint16),
             5: ('int', np.int32), 6: ('uint', np.uint32), 7: ('float', np.float32), 8: ('double', np.float64)}


class PlyProperty(ctypes.Structure):
    _fields_ = [('name', ctypes.c_char * 64), ('type', ctypes.c_int32)]


class PlyElement(ctypes.Structure):
    _fields_ = [('name', ctypes.c_char * 64), ('count', ctypes.c_uint64), ('nprops', ctypes.c_int32),
                ('props', PlyProperty * 256)]


class PlyHeader(ctypes.Structure):
    _fields_ = [('header_bytes', ctypes.c_uint64), ('nelements', ctypes.c_int32), ('ncomments', ctypes.c_int32),
                ('comments', ctypes.c_char * 8192), ('elements', PlyElement * 16)]

    def layout(self):
        """[(element name, count, [(prop name, numpy dtype)])]"""
        out = []
        for e in self.elements[:self.nelements]:
            out.append((e.name.decode(), e.count,
                        [(p.name.decode(), PLY_TYPES[p.type][1]) for p in e.props[:e.nprops]]))
        return out

    def comment_list(self):
        return self.comments.decode().split('\n') if self.ncomments else []


EXPORTS = [
    'st_abi_version', 'st_last_error', 'st_device_count', 'st_ctx_create', 'st_ctx_destroy', 'st_ctx_set_stream',
    'st_ctx_synchronize', 'st_ctx_last_timings', 'st_ctx_last_kmeans_stats', 'st_ctx_set_profiling', 'st_ctx_reset_kernel_stats',
    'st_ctx_kernel_stats', 'st_ctx_set_verify', 'st_ctx_verify_snapshot', 'st_quat_from_euler', 'st_transform_params_make', 'st_sog_geometry',
    'st_transform', 'st_filter_finite', 'st_morton_order', 'st_pack_compressed', 'st_kmeans', 'st_cluster1d', 'st_sog',
    'st_dev_transform', 'st_dev_filter_finite', 'st_dev_permute_rows', 'st_dev_concat_rows', 'st_dev_morton_order',
    'st_dev_pack_compressed', 'st_dev_kmeans', 'st_dev_cluster1d', 'st_dev_sog',
    'st_set_devices', 'st_get_devices', 'st_comm_unique_id', 'st_comm_init_rank', 'st_comm_init_host', 'st_comm_destroy',
    'st_comm_count', 'st_rccl_info', 'st_ctx_last_host_reuse', 'st_ply_compressed_ply_file',
    'st_compressed_ply_file',
    'st_dev_sog_sharded', 'st_group_create', 'st_group_destroy', 'st_group_sog', 'st_group_sog_bundle',
    'st_filter_nan', 'st_dev_filter_finite_t', 'st_dev_permute_rows_t', 'st_combine_layout', 'st_dev_combine',
    'st_dev_minmax', 'st_dev_kmeans_init_rows', 'st_dev_gather_rows', 'st_dev_kmeans_prepare',
    'st_dev_kmeans_assign', 'st_dev_kmeans_partials',
    'st_dev_kmeans_seqsum', 'st_dev_kmeans_finish', 'st_dev_kmeans_average', 'st_dev_cluster1d_codebook',
    'st_dev_sog_scatter', 'st_dev_sog_shn_centroids',
    'st_webp_max_size', 'st_dev_webp_lossless', 'st_webp_lossless', 'st_dev_crc32', 'st_zip_store',
    'st_sog_meta_json', 'st_dev_sog_bundle', 'st_dev_sog_bundle_view', 'st_dev_sog_file', 'st_sog_file', 'st_sog_bundle',
    'st_free',
    'st_ply_parse_header', 'st_ply_read_header', 'st_ply_row_bytes', 'st_dev_ply_transpose', 'st_dev_ply_read',
    'st_ply_read', 'st_ply_read_resident', 'st_ply_materialize', 'st_ply_forget', 'st_dev_decompress_ply', 'st_decompress_ply',
    'st_process', 'st_compressed_ply', 'st_dev_compressed_ply', 'st_ply_compressed_ply', 'st_ply_sog_bundle',
    'st_group_sog_bundle_process',
    'st_transform_t', 'st_dev_transform_t', 'st_morton_order_t', 'st_dev_morton_order_t', 'st_sog_process',
    'st_sog_bundle_process', 'st_dev_sog_t',
]


def _forget_column(ctx_ref, ptr):
    """a resident read's column is being freed: the context (if still open) drops it (st_ply_forget)"""
    c = ctx_ref()
    if c is not None and c.h:
        lib().st_ply_forget(c.h, ctypes.c_void_p(ptr))


def build(jobs=8):
    subprocess.check_call(['make', '-s', '-C', PKG, f'-j{jobs}'])


def lib():
    """Load libsplat_hip.so (fails loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'{LIB_PATH} missing: build it with `make -C {PKG}` (hipcc, gfx950)')
        L = ctypes.CDLL(LIB_PATH)
        for name in EXPORTS:
            getattr(L, name)
        L.st_last_error.restype = ctypes.c_char_p
        L.st_ctx_last_timings.restype = ctypes.c_char_p
        L.st_ctx_last_kmeans_stats.restype = ctypes.c_char_p
        L.st_ctx_destroy.restype = None
        L.st_comm_destroy.restype = None
        L.st_group_destroy.restype = None
        L.st_free.restype = None
        L.st_webp_max_size.restype = ctypes.c_uint64
        L.st_ply_row_bytes.restype = ctypes.c_uint64
        for name in EXPORTS:
            if name not in ('st_last_error', 'st_ctx_last_timings', 'st_ctx_last_kmeans_stats', 'st_ctx_destroy', 'st_free', 'st_webp_max_size',
                            'st_ply_row_bytes', 'st_comm_destroy', 'st_group_destroy'):
                getattr(L, name).restype = ctypes.c_int
        _lib = L
    return _lib


def check(rc):
    if rc != ST_OK:
        raise StError(rc, lib().st_last_error().decode())


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _ptr(t):
    """device pointer of a torch tensor or numpy host array"""
    if t is None:
        return None
    if hasattr(t, 'data_ptr'):
        return ctypes.c_void_p(t.data_ptr())
    return ctypes.c_void_p(t.ctypes.data)


def make_table(cols):
    """st_table over a dict name -> float32 array (numpy host or torch device); keeps refs alive"""
    names = list(cols.keys())
    n = len(cols[names[0]]) if names else 0
    c_names = (ctypes.c_char_p * len(names))(*[s.encode() for s in names])
    c_cols = (ctypes.c_void_p * len(names))(*[_ptr(cols[k]).value for k in names])
    t = Table(n, len(names), ctypes.cast(c_names, ctypes.POINTER(ctypes.c_char_p)),
              ctypes.cast(c_cols, ctypes.POINTER(ctypes.c_void_p)))
    t._keep = (c_names, c_cols, cols)
    return t


_NP_TO_PLY = {np.dtype(v[1]): k for k, v in PLY_TYPES.items()}


def ply_type_of(a):
    """st_ply_type code of a numpy array or torch tensor's element type"""
    if hasattr(a, 'data_ptr'):
        import torch
        tmap = {torch.int8: 1, torch.uint8: 2, torch.int16: 3, torch.uint16: 4, torch.int32: 5, torch.uint32: 6,
                torch.float32: 7, torch.float64: 8}
        return tmap[a.dtype]
    return _NP_TO_PLY[np.dtype(a.dtype)]


def make_ttable(cols, n=None):
    """st_ttable over a list of (name, array) or a dict (numpy host or torch device, any of the eight
    types); keeps refs alive"""
    items = list(cols.items()) if isinstance(cols, dict) else list(cols)
    names = [k for k, _ in items]
    if n is None:
        n = len(items[0][1]) if items else 0
    c_names = (ctypes.c_char_p * len(items))(*[k.encode() for k in names])
    c_types = (ctypes.c_int32 * len(items))(*[ply_type_of(a) for _, a in items])
    c_cols = (ctypes.c_void_p * len(items))(*[_ptr(a).value for _, a in items])
    t = TTable(n, len(items), ctypes.cast(c_names, ctypes.POINTER(ctypes.c_char_p)),
               ctypes.cast(c_types, ctypes.POINTER(ctypes.c_int32)), ctypes.cast(c_cols, ctypes.POINTER(ctypes.c_void_p)))
    t._keep = (c_names, c_types, c_cols, items)
    return t


def combine_layout(tables):
    """combine()'s result columns (index.ts:164-178): [(table index, column index)]; tables are lists
    of (name, array)"""
    tts = [make_ttable(t) for t in tables]
    arr = (ctypes.POINTER(TTable) * len(tts))(*[ctypes.pointer(t) for t in tts])
    ncol = ctypes.c_int32()
    check(lib().st_combine_layout(arr, ctypes.c_int32(len(tts)), None, None, ctypes.byref(ncol)))
    ct = (ctypes.c_int32 * max(ncol.value, 1))()
    ci = (ctypes.c_int32 * max(ncol.value, 1))()
    check(lib().st_combine_layout(arr, ctypes.c_int32(len(tts)), ct, ci, ctypes.byref(ncol)))
    return [(ct[i], ci[i]) for i in range(ncol.value)]


def set_devices(n):
    """st_set_devices: st_sog / st_sog_bundle shard their rows over GPUs 0..n-1 (RCCL)"""
    check(lib().st_set_devices(ctypes.c_int32(n)))


def get_devices():
    n = ctypes.c_int32()
    check(lib().st_get_devices(ctypes.byref(n)))
    return n.value


def comm_unique_id():
    """128-byte RCCL unique id (rank 0 creates it; the launcher hands it to every rank)"""
    buf = (ctypes.c_uint8 * 128)()
    check(lib().st_comm_unique_id(buf))
    return bytes(buf)


def _tables_arg(tables):
    ts = [make_table(t) for t in tables]
    arr = (ctypes.POINTER(Table) * len(ts))(*[ctypes.pointer(t) for t in ts])
    return ts, arr


def _sog_out(N, C, host=True, device=None):
    W, H, pal, cw, ch = sog_geometry(N, C)
    names = ['means_l', 'means_u', 'quats', 'scales', 'sh0'] + (['shN_labels'] if C else [])
    if host:
        tex = {k: np.zeros(W * H * 4, np.uint8) for k in names}
        if C:
            tex['shN_centroids'] = np.zeros(cw * ch * 4, np.uint8)
    else:
        import torch
        tex = {k: torch.empty(W * H * 4, dtype=torch.uint8, device=device) for k in names}
        if C:
            tex['shN_centroids'] = torch.empty(cw * ch * 4, dtype=torch.uint8, device=device)
    out = SogTextures(*[(_ptr(tex[k]).value if k in tex else None) for k in
                        ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels')])
    return tex, out, (W, H, cw, ch)


def _union_coeffs(tables):
    names = set()
    for t in tables:
        names.update(t.keys())
    miss = next((i for i in range(45) if f'f_rest_{i}' not in names), -1)
    return [0, 3, 8, 15][{9: 1, 24: 2, -1: 3}.get(miss, 0)]


class Group:
    """st_group: several ranks in this process (one context + host thread each).  host_staged: the
    exchange goes through host memory, so ranks may share a GPU (the multi-rank tests)"""

    def __init__(self, devices, host_staged=False):
        self.h = ctypes.c_void_p()
        arr = (ctypes.c_int32 * len(devices))(*devices)
        check(lib().st_group_create(arr, ctypes.c_int32(len(devices)), ctypes.c_int32(1 if host_staged else 0),
                                    ctypes.byref(self.h)))
        self.world = len(devices)

    def close(self):
        if self.h:
            lib().st_group_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sog(self, tables, iters, draws, splits=None):
        """writeSog of the concatenated host tables (dicts name -> float32 array)"""
        N = sum(len(next(iter(t.values()))) for t in tables)
        C = _union_coeffs(tables)
        tex, out, (W, H, cw, ch) = _sog_out(N, C)
        ts, arr = _tables_arg(tables)
        sp = (ctypes.c_uint64 * (self.world + 1))(*splits) if splits is not None else None
        meta = SogMeta()
        used = ctypes.c_uint64()
        check(lib().st_group_sog(self.h, arr, ctypes.c_int32(len(ts)), sp, ctypes.c_int32(iters), _vp(draws),
                                 ctypes.c_uint64(len(draws)), ctypes.byref(used), ctypes.byref(meta),
                                 ctypes.byref(out)))
        res = {k: v.reshape(H, W, 4) for k, v in tex.items() if k != 'shN_centroids'}
        if C:
            res['shN_centroids'] = tex['shN_centroids'].reshape(ch, cw, 4)
        return res, meta, used.value

    def sog_bundle(self, tables, iters, draws, dos_time, dos_date, splits=None):
        ts, arr = _tables_arg(tables)
        sp = (ctypes.c_uint64 * (self.world + 1))(*splits) if splits is not None else None
        out, size = ctypes.c_void_p(), ctypes.c_uint64(0)
        used = ctypes.c_uint64()
        check(lib().st_group_sog_bundle(self.h, arr, ctypes.c_int32(len(ts)), sp, ctypes.c_int32(iters),
                                        _vp(draws), ctypes.c_uint64(len(draws)), ctypes.byref(used),
                                        ctypes.c_uint16(dos_time), ctypes.c_uint16(dos_date), ctypes.byref(out),
                                        ctypes.byref(size)))
        return _take(out, size), used.value


    def sog_bundle_process(self, tables, actions, iters, draws, dos_time, dos_date, splits=None):
        """writeSog -> .sog bytes of the combine of `tables` after each table's processDataTable
        `actions` (one list per table) ran on the ranks' parts (st_group_sog_bundle_process)"""
        ts, arr = _tables_arg(tables)
        acts = [make_actions(a) for a in actions]
        aptr = (ctypes.POINTER(Action) * len(ts))(*[ctypes.cast(a, ctypes.POINTER(Action)) for a in acts])
        nact = (ctypes.c_int32 * len(ts))(*[len(a) for a in actions])
        sp = (ctypes.c_uint64 * (self.world + 1))(*splits) if splits is not None else None
        out, size = ctypes.c_void_p(), ctypes.c_uint64(0)
        used = ctypes.c_uint64()
        check(lib().st_group_sog_bundle_process(self.h, arr, ctypes.c_int32(len(ts)), sp, aptr, nact,
                                                ctypes.c_int32(iters), _vp(draws), ctypes.c_uint64(len(draws)),
                                                ctypes.byref(used), ctypes.c_uint16(dos_time),
                                                ctypes.c_uint16(dos_date), ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size), used.value


class Comm:
    """st_comm: this process's rank of a one-rank-per-process job: over RCCL (one GPU per rank,
    `uid` from comm_unique_id on rank 0) or, with Comm.host, over host shared memory (any number
    of ranks on one GPU)"""

    def __init__(self, ctx, world, rank, uid=None, _host=None):
        self.h = ctypes.c_void_p()
        self.world, self.rank = world, rank
        if _host is not None:
            name, slot_bytes, timeout_s = _host
            check(lib().st_comm_init_host(ctx.h, ctypes.c_int32(world), ctypes.c_int32(rank), name.encode(),
                                          ctypes.c_uint64(slot_bytes), ctypes.c_double(timeout_s),
                                          ctypes.byref(self.h)))
            self.transport = 'host-shm'
            return
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(lib().st_comm_init_rank(ctx.h, ctypes.c_int32(world), ctypes.c_int32(rank), buf, ctypes.byref(self.h)))
        self.transport = 'rccl'

    @classmethod
    def host(cls, ctx, world, rank, name, slot_bytes=0, timeout_s=600.0):
        """st_comm_init_host: every rank passes the same job `name` (unique per job)"""
        return cls(ctx, world, rank, _host=(name, slot_bytes, timeout_s))

    def count(self):
        """ranks in the communicator (ncclCommCount for RCCL)"""
        n = ctypes.c_int32()
        check(lib().st_comm_count(self.h, ctypes.byref(n)))
        return n.value

    def close(self):
        if self.h:
            lib().st_comm_destroy(self.h)
            self.h = ctypes.c_void_p()


def quat_from_euler(ex, ey, ez):
    q = (ctypes.c_double * 4)()
    check(lib().st_quat_from_euler(ctypes.c_double(ex), ctypes.c_double(ey), ctypes.c_double(ez), q))
    return np.array(q[:])


def transform_params(t=(0.0, 0.0, 0.0), r=(0.0, 0.0, 0.0, 1.0), s=1.0):
    p = TransformParams()
    check(lib().st_transform_params_make((ctypes.c_double * 3)(*t), (ctypes.c_double * 4)(*r), ctypes.c_double(s),
                                         ctypes.byref(p)))
    return p


def action_params(kind, value):
    """process.ts:71-83: translate / rotate (Euler degrees) / scale"""
    if kind == 'translate':
        return transform_params(t=value)
    if kind == 'rotate':
        return transform_params(r=quat_from_euler(*value))
    if kind == 'scale':
        return transform_params(s=float(value))
    raise ValueError(kind)


def make_actions(actions):
    """processDataTable's ProcessAction list (process.ts:6-42) as st_action[]: dicts with 'kind' in
    translate / rotate / scale (value as in action_params), filterNaN, filterByValue (columnName,
    comparator, value), filterBands (value), param"""
    arr = (Action * max(1, len(actions)))()
    keep = []
    for a, act in zip(arr, actions):
        k = act['kind']
        if k in ('translate', 'rotate', 'scale'):
            a.kind, a.transform = ACTION_TRANSFORM, action_params(k, act['value'])
        elif k == 'filterNaN':
            a.kind = ACTION_FILTER_NAN
        elif k == 'filterByValue':
            col = act['columnName'].encode()
            keep.append(col)
            a.kind, a.column, a.value = ACTION_FILTER_VALUE, col, float(act['value'])
            a.compare = COMPARE.get(act['comparator'], -1)
        elif k == 'filterBands':
            a.kind, a.bands = ACTION_FILTER_BANDS, int(act['value'])
        elif k == 'param':
            a.kind = ACTION_PARAM
        else:
            raise ValueError(k)
    arr._keep = keep
    return arr


def process_schema(items, actions, with_source=False):
    """the (name, dtype) columns processDataTable leaves (filterBands renames / drops f_rest
    columns against the ORIGINAL table's band, process.ts:110-134); with_source: (name, dtype,
    index of the input column it is)"""
    names = [k for k, _ in items]
    first_missing = next((i for i in range(45) if f'f_rest_{i}' not in names), -1)
    in_coeffs = {9: 3, 24: 8, -1: 15}.get(first_missing, 0)
    cols = [(k, np.dtype(a.dtype), i) for i, (k, a) in enumerate(items)]
    for act in actions:
        if act['kind'] != 'filterBands':
            continue
        out_coeffs = [0, 3, 8, 15][act['value']]
        if out_coeffs >= in_coeffs:
            continue
        mp = {}
        for i in range(in_coeffs):
            for j in range(3):
                mp[f'f_rest_{i + j * in_coeffs}'] = f'f_rest_{i + j * out_coeffs}' if i < out_coeffs else None
        cols = [(mp[k], t, i) if k in mp else (k, t, i) for k, t, i in cols if k not in mp or mp[k] is not None]
    return cols if with_source else [(k, t) for k, t, _ in cols]


TRANSFORM_KINDS = ('translate', 'rotate', 'scale')
FILTER_KINDS = ('filterNaN', 'filterByValue')


def sog_geometry(n, sh_coeffs):
    v = [ctypes.c_int32() for _ in range(5)]
    check(lib().st_sog_geometry(ctypes.c_uint64(n), ctypes.c_int32(sh_coeffs), *[ctypes.byref(x) for x in v]))
    return tuple(x.value for x in v)


def _take(buf, size):
    """copy a malloc'd library buffer into bytes and release it"""
    try:
        return ctypes.string_at(buf, size.value)
    finally:
        lib().st_free(buf)


def webp_max_size(w, h):
    return lib().st_webp_max_size(ctypes.c_int32(w), ctypes.c_int32(h))


def zip_store(entries, dos_time, dos_date):
    """store-only ZIP of [(name, bytes, crc)] in the layout of serialize/zip-writer.ts (host)"""
    n = len(entries)
    names = (ctypes.c_char_p * n)(*[e[0].encode() for e in entries])
    bufs = [ctypes.create_string_buffer(bytes(e[1]), len(e[1]) or 1) for e in entries]
    data = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in bufs])
    sizes = (ctypes.c_uint64 * n)(*[len(e[1]) for e in entries])
    crcs = (ctypes.c_uint32 * n)(*[e[2] for e in entries])
    out, size = ctypes.c_void_p(), ctypes.c_uint64(0)
    check(lib().st_zip_store(names, data, sizes, crcs, ctypes.c_int32(n), ctypes.c_uint16(dos_time),
                             ctypes.c_uint16(dos_date), ctypes.byref(out), ctypes.byref(size)))
    return _take(out, size)


def sog_meta_json(meta, count):
    """meta.json text of writeSog for an SogMeta (host)"""
    out, size = ctypes.c_void_p(), ctypes.c_uint64(0)
    check(lib().st_sog_meta_json(ctypes.byref(meta), ctypes.c_uint64(count), ctypes.byref(out), ctypes.byref(size)))
    return _take(out, size)


CHUNK_COLS = ['min_x', 'min_y', 'min_z', 'max_x', 'max_y', 'max_z', 'min_scale_x', 'min_scale_y', 'min_scale_z',
              'max_scale_x', 'max_scale_y', 'max_scale_z', 'min_r', 'min_g', 'min_b', 'max_r', 'max_g', 'max_b']
VERTEX_COLS = ['packed_position', 'packed_rotation', 'packed_scale', 'packed_color']
DECOMP_COLS = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2', 'opacity', 'rot_0', 'rot_1', 'rot_2', 'rot_3',
               'scale_0', 'scale_1', 'scale_2']


def ply_parse_header(data):
    """readPly's header (read-ply.ts:54-137) from the first bytes of a file (host)"""
    h = PlyHeader()
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    check(lib().st_ply_parse_header(buf, ctypes.c_uint64(len(data)), ctypes.byref(h)))
    return h


def rccl_info():
    """(version, path) of the RCCL the library's collectives run on (st_rccl_info: loaded by path,
    /opt/rocm/lib/librccl.so.1 unless ST_RCCL says otherwise; no GPU needed)"""
    v = ctypes.c_int32(0)
    buf = ctypes.create_string_buffer(4096)
    check(lib().st_rccl_info(ctypes.byref(v), buf, ctypes.c_uint64(len(buf))))
    return v.value, buf.value.decode()


def device_count():
    n = ctypes.c_int32(0)
    check(lib().st_device_count(ctypes.byref(n)))
    return n.value


class Context:
    def __init__(self, device=0):
        # PyTorch-ROCm ships its own HIP runtime next to the one this library links; when both
        # live in one process, torch's must initialise first (the other order leaves torch
        # without a device).  Device tensors are still shared through plain pointers.
        if 'torch' in sys.modules:
            try:
                sys.modules['torch'].cuda.init()
            except RuntimeError:
                pass  # no device: st_ctx_create reports it
        self.h = ctypes.c_void_p()
        check(lib().st_ctx_create(ctypes.c_int32(device), ctypes.byref(self.h)))

    def close(self):
        if self.h:
            lib().st_ctx_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle):
        """run on a caller-owned hipStream_t.  Handle 0 is refused: torch's legacy default stream
        has handle 0, which the C ABI reads as NULL = the context's own (non-blocking) stream, so
        the library would silently stop ordering against the caller's torch work."""
        if not stream_handle:
            raise ValueError('set_stream(0): handle 0 selects the context\'s own stream, not the legacy '
                             'default stream; use bind_torch_stream() or use_own_stream()')
        check(lib().st_ctx_set_stream(self.h, ctypes.c_void_p(stream_handle)))

    def use_own_stream(self):
        check(lib().st_ctx_set_stream(self.h, None))

    def bind_torch_stream(self, device):
        """one real stream for the library and the caller's torch work on `device`: torch's
        current stream when it is not the legacy default stream, else a new stream made
        current, ordered after what the default stream already holds.  Returns the torch stream."""
        import torch
        s = torch.cuda.current_stream(device)
        if s.cuda_stream == 0:
            prev, s = s, torch.cuda.Stream(device)
            s.wait_stream(prev)  # work already queued on the default stream comes first
            torch.cuda.set_stream(s)
        self.set_stream(s.cuda_stream)
        return s

    def synchronize(self):
        check(lib().st_ctx_synchronize(self.h))

    def timings(self):
        return lib().st_ctx_last_timings(self.h).decode()

    def host_reuse(self):
        """(columns, bytes) the last writeSog host form ran from st_ply_read's resident copy
        (st_ctx_last_host_reuse; (0, 0): it uploaded them)"""
        cols, nb = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(lib().st_ctx_last_host_reuse(self.h, ctypes.byref(cols), ctypes.byref(nb)))
        return cols.value, nb.value

    def sog_file(self, cols, iters, draws, path, dos_time=0, dos_date=0):
        """writeSog of a host table into a file (st_sog_file): (used, size).  The file is opened
        without O_TRUNC (st_sog_file cuts it to the archive's length)"""
        keep = {k: np.ascontiguousarray(v, np.float32) for k, v in cols.items()}
        t = make_table(keep)
        used, size = ctypes.c_uint64(0), ctypes.c_uint64(0)
        fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
        try:
            check(lib().st_sog_file(self.h, ctypes.byref(t), ctypes.c_int32(iters), _vp(draws),
                                    ctypes.c_uint64(len(draws)), ctypes.byref(used), ctypes.c_int32(fd),
                                    ctypes.c_uint16(dos_time), ctypes.c_uint16(dos_date), ctypes.byref(size)))
        finally:
            os.close(fd)
        return used.value, size.value

    def kmeans_stats(self):
        """the last N-D k-means' assign classification (st_ctx_last_kmeans_stats) as a dict"""
        import json
        return json.loads(lib().st_ctx_last_kmeans_stats(self.h).decode())

    def set_profiling(self, on=True):
        check(lib().st_ctx_set_profiling(self.h, ctypes.c_int32(1 if on else 0)))

    def reset_kernel_stats(self):
        check(lib().st_ctx_reset_kernel_stats(self.h))

    def kernel_stats(self, name):
        """(total_ms, launches) of a named library kernel since the last reset (HIP events, ctx stream)"""
        ms = ctypes.c_double(0)
        cnt = ctypes.c_uint64(0)
        check(lib().st_ctx_kernel_stats(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(cnt)))
        return ms.value, cnt.value

    def set_verify(self, on=True):
        check(lib().st_ctx_set_verify(self.h, ctypes.c_int32(1 if on else 0)))

    def verify_snapshot(self, device='cuda'):
        """(prev_centroids [d, k], centroids [d, k], labels [n]) torch tensors of the last N-D
        k-means run while verification was on (st_ctx_verify_snapshot)"""
        import torch
        d, k, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_uint64()
        check(lib().st_ctx_verify_snapshot(self.h, None, None, None, ctypes.byref(d), ctypes.byref(k),
                                           ctypes.byref(n)))
        prev = torch.empty((d.value, k.value), dtype=torch.float32, device=device)
        cen = torch.empty_like(prev)
        lab = torch.empty(n.value, dtype=torch.int32, device=device)
        check(lib().st_ctx_verify_snapshot(self.h, _ptr(prev), _ptr(cen), _ptr(lab), ctypes.byref(d),
                                           ctypes.byref(k), ctypes.byref(n)))
        self.synchronize()
        return prev, cen, lab

    # ---- host-memory seams ----------------------------------------------------
    def transform(self, cols, params):
        """transform() in place on host columns (dict name -> array); columns that are not float32
        take st_transform_t (the reference's getRow / setRow on any type)"""
        if any(np.dtype(a.dtype) != np.float32 for a in cols.values()):
            t = make_ttable(cols)
            check(lib().st_transform_t(self.h, ctypes.byref(t), ctypes.byref(params)))
            return
        t = make_table(cols)
        check(lib().st_transform(self.h, ctypes.byref(t), ctypes.byref(params)))

    def filter_finite(self, cols):
        t = make_table(cols)
        out = np.zeros(t.n, np.uint32)
        m = ctypes.c_uint64(0)
        check(lib().st_filter_finite(self.h, ctypes.byref(t), _vp(out), ctypes.byref(m)))
        return out[:m.value]

    def morton_order(self, x, y, z, indices=None):
        n = len(x)
        idx = np.arange(n, dtype=np.uint32) if indices is None else np.ascontiguousarray(indices, np.uint32).copy()
        if any(np.dtype(a.dtype) != np.float32 for a in (x, y, z)):  # ordering.ts reads any type's numbers
            xyz = [np.ascontiguousarray(a) for a in (x, y, z)]
            ptrs = (ctypes.c_void_p * 3)(*[a.ctypes.data for a in xyz])
            types = (ctypes.c_int32 * 3)(*[ply_type_of(a) for a in xyz])
            check(lib().st_morton_order_t(self.h, ptrs, types, _vp(idx), ctypes.c_uint64(n)))
            return idx
        check(lib().st_morton_order(self.h, _vp(x), _vp(y), _vp(z), _vp(idx), ctypes.c_uint64(n)))
        return idx

    def pack_compressed(self, cols, order, nsh):
        t = make_table(cols)
        n = t.n
        chunk = np.zeros(((n + 255) // 256) * 18, np.float32)
        vertex = np.zeros(n * 4, np.uint32)
        sh = np.zeros(max(n * nsh, 1), np.uint8)
        check(lib().st_pack_compressed(self.h, ctypes.byref(t), _vp(np.ascontiguousarray(order, np.uint32)),
                                       _vp(chunk), _vp(vertex), _vp(sh)))
        return chunk, vertex, sh[:n * nsh]

    def kmeans(self, col_list, k, iters, draws):
        d, n = len(col_list), len(col_list[0])
        kk = min(k, n)
        cent = np.zeros(d * kk, np.float32)
        labels = np.zeros(n, np.uint32)
        used = ctypes.c_uint64(0)
        ptrs = (ctypes.c_void_p * d)(*[c.ctypes.data for c in col_list])
        check(lib().st_kmeans(self.h, ptrs, ctypes.c_int32(d), ctypes.c_uint64(n), ctypes.c_int32(k),
                              ctypes.c_int32(iters), _vp(draws), ctypes.c_uint64(len(draws)), ctypes.byref(used),
                              _vp(cent), _vp(labels)))
        return cent.reshape(d, kk), labels, used.value

    def cluster1d(self, col_list, iters, draws):
        n = len(col_list[0])
        cent = np.zeros(256, np.float32)
        labels = np.zeros(n * len(col_list), np.uint8)
        used = ctypes.c_uint64(0)
        ptrs = (ctypes.c_void_p * len(col_list))(*[c.ctypes.data for c in col_list])
        check(lib().st_cluster1d(self.h, ptrs, ctypes.c_int32(len(col_list)), ctypes.c_uint64(n),
                                 ctypes.c_int32(iters), _vp(draws), ctypes.c_uint64(len(draws)), ctypes.byref(used),
                                 _vp(cent), _vp(labels)))
        return cent, labels.reshape(len(col_list), n), used.value

    def sog(self, cols, iters, draws):
        t = make_table(cols)
        C = sum(1 for k in cols if k.startswith('f_rest_')) // 3
        C = {9: 3, 24: 8, 45: 15}.get(3 * C, 0) if C else 0
        W, H, pal, cw, ch = sog_geometry(t.n, C)
        tex = {k: np.zeros(W * H * 4, np.uint8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0')}
        if C:
            tex['shN_labels'] = np.zeros(W * H * 4, np.uint8)
            tex['shN_centroids'] = np.zeros(cw * ch * 4, np.uint8)
        out = SogTextures(tex['means_l'].ctypes.data, tex['means_u'].ctypes.data, tex['quats'].ctypes.data,
                          tex['scales'].ctypes.data, tex['sh0'].ctypes.data,
                          tex['shN_centroids'].ctypes.data if C else None,
                          tex['shN_labels'].ctypes.data if C else None)
        meta = SogMeta()
        used = ctypes.c_uint64(0)
        check(lib().st_sog(self.h, ctypes.byref(t), ctypes.c_int32(iters), _vp(draws), ctypes.c_uint64(len(draws)),
                           ctypes.byref(used), ctypes.byref(meta), ctypes.byref(out)))
        res = {k: v.reshape(H, W, 4) for k, v in tex.items() if k != 'shN_centroids'}
        if C:
            res['shN_centroids'] = tex['shN_centroids'].reshape(ch, cw, 4)
        return res, meta, used.value

    def sog_process(self, cols, actions, iters, draws):
        """processDataTable then writeSog's textures + meta on a host table of any column types
        (list of (name, array) or dict): (textures, meta, draws used) as sog()"""
        items = list(cols.items()) if isinstance(cols, dict) else list(cols)
        names = [k for k, _ in items]
        first_missing = next((i for i in range(45) if f'f_rest_{i}' not in names), -1)
        C = {9: 3, 24: 8, -1: 15}.get(first_missing, 0)
        t = make_ttable(items)
        tex, out, _ = _sog_out(t.n, C)
        meta = SogMeta()
        used = ctypes.c_uint64(0)
        acts = make_actions(actions)
        check(lib().st_sog_process(self.h, ctypes.byref(t), acts, ctypes.c_int32(len(actions)), ctypes.c_int32(iters),
                                   _vp(draws), ctypes.c_uint64(len(draws)), ctypes.byref(used), ctypes.byref(meta),
                                   ctypes.byref(out)))
        W, H, cw, ch = meta.width, meta.height, meta.shn_width, meta.shn_height
        res = {k: v[:W * H * 4].reshape(H, W, 4) for k, v in tex.items() if k != 'shN_centroids'}
        if meta.sh_bands:
            res['shN_centroids'] = tex['shN_centroids'][:cw * ch * 4].reshape(ch, cw, 4)
        else:
            res.pop('shN_labels', None)
        return res, meta, used.value

    def sog_bundle_process(self, cols, actions, iters, draws, dos_time, dos_date):
        """processDataTable then writeSog to a .sog bundle, any column types: (archive, draws used)"""
        items = list(cols.items()) if isinstance(cols, dict) else list(cols)
        t = make_ttable(items)
        acts = make_actions(actions)
        used = ctypes.c_uint64(0)
        out, size = ctypes.c_void_p(), ctypes.c_uint64(0)
        check(lib().st_sog_bundle_process(self.h, ctypes.byref(t), acts, ctypes.c_int32(len(actions)),
                                          ctypes.c_int32(iters), _vp(draws), ctypes.c_uint64(len(draws)),
                                          ctypes.byref(used), ctypes.c_uint16(dos_time), ctypes.c_uint16(dos_date),
                                          ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size), used.value

    def webp_lossless(self, rgba):
        """WebPEncodeLosslessRGBA of a host (H, W, 4) uint8 array -> .webp bytes"""
        rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
        h, w = rgba.shape[:2]
        out, size = ctypes.c_void_p(), ctypes.c_uint64(0)
        check(lib().st_webp_lossless(self.h, _vp(rgba), ctypes.c_int32(w), ctypes.c_int32(h), ctypes.c_int32(w * 4),
                                     ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size)

    def read_ply(self, path, resident=False):
        """readPly (read-ply.ts:111-191) -> (comments, [(element, {prop: numpy column})]); rows go through HBM.
        resident: st_ply_read_resident -- the numpy columns stay unfilled (the values live in HBM) until
        materialize(column) or a host form other than writeSog's reads them; keep them alive until then,
        or forget() them"""
        fd = os.open(path, os.O_RDONLY)
        try:
            h = PlyHeader()
            check(lib().st_ply_read_header(ctypes.c_int32(fd), ctypes.byref(h)))
            out = []
            read = lib().st_ply_read_resident if resident else lib().st_ply_read
            for ei, (name, count, props) in enumerate(h.layout()):
                cols = {pn: np.empty(count, dt) for pn, dt in props}
                ptrs = (ctypes.c_void_p * max(len(props), 1))(*[cols[pn].ctypes.data for pn, _ in props])
                check(read(self.h, ctypes.c_int32(fd), ctypes.byref(h), ctypes.c_int32(ei), ptrs))
                if resident:  # st_ply_read_resident's contract: forgotten before the memory goes away
                    for a in cols.values():
                        weakref.finalize(a, _forget_column, weakref.ref(self), a.ctypes.data)
                out.append((name, cols))
            return h.comment_list(), out
        finally:
            os.close(fd)

    def materialize(self, col):
        """a resident read's column filled from HBM (st_ply_materialize); no-op for any other array"""
        check(lib().st_ply_materialize(self.h, ctypes.c_void_p(col.ctypes.data)))
        return col

    def forget(self, col):
        """drop a resident or mirrored column without copying it (st_ply_forget)"""
        check(lib().st_ply_forget(self.h, ctypes.c_void_p(col.ctypes.data)))

    def decompress_ply(self, chunk, vertex, sh):
        """decompressPly (decompress-ply.ts:82-232): chunk/vertex dicts of numpy columns, sh list of uint8
        columns -> dict of float32 columns in the reference's order"""
        n = len(vertex['packed_position'])
        keep = [np.ascontiguousarray(chunk[k], np.float32) for k in CHUNK_COLS]
        cp = (ctypes.c_void_p * 18)(*[a.ctypes.data for a in keep])
        vk = [np.ascontiguousarray(vertex[k], np.uint32) for k in VERTEX_COLS]
        vp = (ctypes.c_void_p * 4)(*[a.ctypes.data for a in vk])
        sk = [np.ascontiguousarray(a, np.uint8) for a in sh]
        sp = (ctypes.c_void_p * max(len(sk), 1))(*[a.ctypes.data for a in sk])
        names = DECOMP_COLS + [f'f_rest_{i}' for i in range(len(sk))]
        out = {k: np.empty(n, np.float32) for k in names}
        op = (ctypes.c_void_p * len(names))(*[out[k].ctypes.data for k in names])
        check(lib().st_decompress_ply(self.h, ctypes.c_uint64(n), cp, vp, sp, ctypes.c_int32(len(sk)), op))
        return out

    def sog_bundle(self, cols, iters, draws, dos_time, dos_date):
        """writeSog to a .sog bundle: (archive bytes, draws used)"""
        t = make_table(cols)
        used = ctypes.c_uint64(0)
        out, size = ctypes.c_void_p(), ctypes.c_uint64(0)
        check(lib().st_sog_bundle(self.h, ctypes.byref(t), ctypes.c_int32(iters), _vp(draws),
                                  ctypes.c_uint64(len(draws)), ctypes.byref(used), ctypes.c_uint16(dos_time),
                                  ctypes.c_uint16(dos_date), ctypes.byref(out), ctypes.byref(size)))
        return _take(out, size), used.value

    # ---- device-memory seams (torch tensors) --------------------------------------
    def dev_webp_lossless(self, rgba, out):
        """rgba: device uint8 (H, W, 4) tensor; out: device uint8 tensor of >= webp_max_size bytes"""
        h, w = rgba.shape[:2]
        size = ctypes.c_uint64(0)
        check(lib().st_dev_webp_lossless(self.h, _ptr(rgba), ctypes.c_int32(w), ctypes.c_int32(h),
                                         ctypes.c_int32(rgba.stride(0)), _ptr(out), ctypes.c_uint64(out.numel()),
                                         ctypes.byref(size)))
        return size.value

    def dev_crc32(self, data, n=None, crc_in=0):
        out = ctypes.c_uint32(0)
        n = data.numel() if n is None else n
        check(lib().st_dev_crc32(self.h, _ptr(data), ctypes.c_uint64(n), ctypes.c_uint32(crc_in),
                                 ctypes.byref(out)))
        return out.value

    def dev_sog_bundle_view(self, meta, count, tex, dos_time, dos_date):
        """as dev_sog_bundle without the copy: (address, size) of the context's pinned archive"""
        t = SogTextures(*[(tex[k].data_ptr() if k in tex else None) for k in
                          ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels')])
        out, size = ctypes.c_void_p(), ctypes.c_uint64(0)
        check(lib().st_dev_sog_bundle_view(self.h, ctypes.byref(meta), ctypes.c_uint64(count), ctypes.byref(t),
                                           ctypes.c_uint16(dos_time), ctypes.c_uint16(dos_date), ctypes.byref(out),
                                           ctypes.byref(size)))
        return out.value, size.value

    def dev_sog_bundle(self, meta, count, tex, dos_time, dos_date):
        """the .sog archive bytes of device textures (dict as for dev_sog) and their SogMeta"""
        t = SogTextures(*[(tex[k].data_ptr() if k in tex else None) for k in
                          ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels')])
        out, size = ctypes.c_void_p(), ctypes.c_uint64(0)
        check(lib().st_dev_sog_bundle(self.h, ctypes.byref(meta), ctypes.c_uint64(count), ctypes.byref(t),
                                      ctypes.c_uint16(dos_time), ctypes.c_uint16(dos_date), ctypes.byref(out),
                                      ctypes.byref(size)))
        return _take(out, size)

    def read_ply_dev(self, path, device='cuda'):
        """readPly into device columns: (comments, [(element, {prop: torch tensor})])"""
        import torch
        tmap = {np.int8: torch.int8, np.uint8: torch.uint8, np.int16: torch.int16, np.uint16: torch.uint16,
                np.int32: torch.int32, np.uint32: torch.uint32, np.float32: torch.float32, np.float64: torch.float64}
        fd = os.open(path, os.O_RDONLY)
        try:
            h = PlyHeader()
            check(lib().st_ply_read_header(ctypes.c_int32(fd), ctypes.byref(h)))
            out = []
            for ei, (name, count, props) in enumerate(h.layout()):
                cols = {pn: torch.empty(count, dtype=tmap[dt], device=device) for pn, dt in props}
                ptrs = (ctypes.c_void_p * max(len(props), 1))(*[cols[pn].data_ptr() for pn, _ in props])
                check(lib().st_dev_ply_read(self.h, ctypes.c_int32(fd), ctypes.byref(h), ctypes.c_int32(ei), ptrs))
                out.append((name, cols))
            return h.comment_list(), out
        finally:
            os.close(fd)

    def dev_decompress_ply(self, chunk, vertex, sh, out):
        """device form of decompress_ply: torch tensors in, `out` dict of float32 tensors (DECOMP_COLS + f_rest_*)"""
        n = vertex['packed_position'].numel()
        cp = (ctypes.c_void_p * 18)(*[chunk[k].data_ptr() for k in CHUNK_COLS])
        vp = (ctypes.c_void_p * 4)(*[vertex[k].data_ptr() for k in VERTEX_COLS])
        sp = (ctypes.c_void_p * max(len(sh), 1))(*[a.data_ptr() for a in sh])
        names = DECOMP_COLS + [f'f_rest_{i}' for i in range(len(sh))]
        op = (ctypes.c_void_p * len(names))(*[out[k].data_ptr() for k in names])
        check(lib().st_dev_decompress_ply(self.h, ctypes.c_uint64(n), cp, vp, sp, ctypes.c_int32(len(sh)), op))

    def dev_transform(self, cols, params):
        t = make_table(cols)
        check(lib().st_dev_transform(self.h, ctypes.byref(t), ctypes.byref(params)))

    def dev_morton_order(self, x, y, z, idx):
        check(lib().st_dev_morton_order(self.h, _ptr(x), _ptr(y), _ptr(z), _ptr(idx), ctypes.c_uint64(len(idx))))

    def dev_pack_compressed(self, cols, order, chunk, vertex, sh):
        t = make_table(cols)
        check(lib().st_dev_pack_compressed(self.h, ctypes.byref(t), _ptr(order), _ptr(chunk), _ptr(vertex),
                                           _ptr(sh)))

    def dev_filter_finite(self, cols, out_idx):
        t = make_table(cols)
        m = ctypes.c_uint64(0)
        check(lib().st_dev_filter_finite(self.h, ctypes.byref(t), _ptr(out_idx), ctypes.byref(m)))
        return m.value

    def filter_nan(self, cols):
        """filterNaN on host columns (list of (name, numpy array), any type) -> the surviving rows"""
        items = list(cols.items()) if isinstance(cols, dict) else list(cols)
        out = [(k, np.empty_like(a)) for k, a in items]
        ts, td = make_ttable(items), make_ttable(out)
        m = ctypes.c_uint64()
        check(lib().st_filter_nan(self.h, ctypes.byref(ts), ctypes.byref(td), ctypes.byref(m)))
        return [(k, a[:m.value].copy()) for k, a in out]

    def process(self, cols, actions):
        """processDataTable (process.ts:64-145) on host columns (list of (name, numpy array) or a
        dict) in one upload -> the processed table as a list of (name, array).  As in the
        reference, the transforms before the first filter mutate the input arrays (`result` is
        the input table until a filter copies it; filterBands renames its columns without copying
        them): that region runs first and is written back, the rest runs on the mutated columns.
        Without a filter the result's arrays ARE the input's."""
        items = list(cols.items()) if isinstance(cols, dict) else list(cols)
        first = next((i for i, a in enumerate(actions) if a['kind'] in FILTER_KINDS), len(actions))
        region = actions[:first]
        rs = process_schema(items, region, with_source=True)
        if any(a['kind'] in TRANSFORM_KINDS for a in region):
            for (_, a), (_, _, src) in zip(self._process(items, region), rs):
                np.copyto(items[src][1], a)
        if first == len(actions):
            return [(k, items[src][1]) for k, _, src in rs]
        return self._process(items, [a for i, a in enumerate(actions) if i >= first or a['kind'] not in TRANSFORM_KINDS])

    def _process(self, items, actions):
        """st_process: the action list in one upload, the input untouched"""
        n = len(items[0][1]) if items else 0
        out = [(k, np.empty(n, t)) for k, t in process_schema(items, actions)]
        ts, td = make_ttable(items), make_ttable(out, n)
        acts = make_actions(actions)
        m = ctypes.c_uint64()
        check(lib().st_process(self.h, ctypes.byref(ts), acts, ctypes.c_int32(len(actions)), ctypes.byref(td),
                               ctypes.byref(m)))
        return [(k, a[:m.value].copy()) for k, a in out]

    def compressed_ply(self, cols, actions):
        """processDataTable then writeCompressedPly's device part, one upload: (m, chunk, vertex, sh)"""
        items = list(cols.items()) if isinstance(cols, dict) else list(cols)
        n = len(items[0][1]) if items else 0
        chunk = np.zeros(max(1, (n + 255) // 256 * 18), np.float32)
        vertex = np.zeros(max(1, n * 4), np.uint32)
        sh = np.zeros(max(1, n * 45), np.uint8)
        ts = make_ttable(items, n)
        acts = make_actions(actions)
        m, C = ctypes.c_uint64(), ctypes.c_int32()
        check(lib().st_compressed_ply(self.h, ctypes.byref(ts), acts, ctypes.c_int32(len(actions)), _vp(chunk),
                                      _vp(vertex), _vp(sh), ctypes.byref(m), ctypes.byref(C)))
        m, C = m.value, C.value
        return m, chunk[:(m + 255) // 256 * 18], vertex[:m * 4], sh[:m * 3 * C]

    def dev_compressed_ply(self, cols, actions, chunk, vertex, sh):
        """the same over device columns (list of (name, tensor)) into device outputs sized for n rows"""
        ts = make_ttable(cols)
        acts = make_actions(actions)
        m, C = ctypes.c_uint64(), ctypes.c_int32()
        check(lib().st_dev_compressed_ply(self.h, ctypes.byref(ts), acts, ctypes.c_int32(len(actions)), _ptr(chunk),
                                          _ptr(vertex), _ptr(sh), ctypes.byref(m), ctypes.byref(C)))
        return m.value, C.value

    def ply_compressed_ply(self, path, actions, element=-1):
        """readPly + processDataTable + writeCompressedPly's arrays from the file, resident in HBM
        (st_ply_compressed_ply): (m, chunk, vertex, sh)"""
        fd = os.open(path, os.O_RDONLY)
        try:
            h = PlyHeader()
            check(lib().st_ply_read_header(ctypes.c_int32(fd), ctypes.byref(h)))
            ei = element if element >= 0 else [e[0] for e in h.layout()].index('vertex')
            n = h.layout()[ei][1]
            chunk = np.zeros(max(1, (n + 255) // 256 * 18), np.float32)
            vertex = np.zeros(max(1, n * 4), np.uint32)
            sh = np.zeros(max(1, n * 45), np.uint8)
            acts = make_actions(actions)
            m, C = ctypes.c_uint64(), ctypes.c_int32()
            check(lib().st_ply_compressed_ply(self.h, ctypes.c_int32(fd), ctypes.byref(h), ctypes.c_int32(element),
                                              acts, ctypes.c_int32(len(actions)), _vp(chunk), _vp(vertex), _vp(sh),
                                              ctypes.byref(m), ctypes.byref(C)))
        finally:
            os.close(fd)
        m, C = m.value, C.value
        return m, chunk[:(m + 255) // 256 * 18], vertex[:m * 4], sh[:m * 3 * C]

    def ply_compressed_ply_file(self, path, actions, out_path, version=None, element=-1):
        """readPly + processDataTable + writeCompressedPly into out_path (st_ply_compressed_ply_file:
        the arrays written at offsets as they leave HBM; the file opened without O_TRUNC, cut to
        length by the library): (m, sh_coeffs, file bytes)"""
        fd = os.open(path, os.O_RDONLY)
        try:
            h = PlyHeader()
            check(lib().st_ply_read_header(ctypes.c_int32(fd), ctypes.byref(h)))
            acts = make_actions(actions)
            m, C, size = ctypes.c_uint64(), ctypes.c_int32(), ctypes.c_uint64()
            ofd = os.open(out_path, os.O_WRONLY | os.O_CREAT, 0o644)
            try:
                check(lib().st_ply_compressed_ply_file(self.h, ctypes.c_int32(fd), ctypes.byref(h),
                                                       ctypes.c_int32(element), acts, ctypes.c_int32(len(actions)),
                                                       ctypes.c_int32(ofd), version.encode() if version else None,
                                                       ctypes.byref(m), ctypes.byref(C), ctypes.byref(size)))
            finally:
                os.close(ofd)
        finally:
            os.close(fd)
        return m.value, C.value, size.value

    def compressed_ply_file(self, cols, actions, out_path, version=None):
        """processDataTable + writeCompressedPly of a host table into out_path (st_compressed_ply_file):
        (m, sh_coeffs, file bytes)"""
        items = list(cols.items()) if isinstance(cols, dict) else list(cols)
        n = len(items[0][1]) if items else 0
        ts = make_ttable(items, n)
        acts = make_actions(actions)
        m, C, size = ctypes.c_uint64(), ctypes.c_int32(), ctypes.c_uint64()
        ofd = os.open(out_path, os.O_WRONLY | os.O_CREAT, 0o644)
        try:
            check(lib().st_compressed_ply_file(self.h, ctypes.byref(ts), acts, ctypes.c_int32(len(actions)),
                                               ctypes.c_int32(ofd), version.encode() if version else None,
                                               ctypes.byref(m), ctypes.byref(C), ctypes.byref(size)))
        finally:
            os.close(ofd)
        return m.value, C.value, size.value

    def ply_sog_bundle(self, path, actions, iters, draws, dos_time, dos_date, element=-1):
        """readPly + processDataTable + writeSog to .sog bytes from the file (st_ply_sog_bundle):
        (archive bytes, draws used)"""
        fd = os.open(path, os.O_RDONLY)
        try:
            h = PlyHeader()
            check(lib().st_ply_read_header(ctypes.c_int32(fd), ctypes.byref(h)))
            acts = make_actions(actions)
            draws = np.ascontiguousarray(draws, np.float64)
            used, size = ctypes.c_uint64(), ctypes.c_uint64()
            out = ctypes.c_void_p()
            check(lib().st_ply_sog_bundle(self.h, ctypes.c_int32(fd), ctypes.byref(h), ctypes.c_int32(element), acts,
                                          ctypes.c_int32(len(actions)), ctypes.c_int32(iters), _vp(draws),
                                          ctypes.c_uint64(len(draws)), ctypes.byref(used), ctypes.c_uint16(dos_time),
                                          ctypes.c_uint16(dos_date), ctypes.byref(out), ctypes.byref(size)))
        finally:
            os.close(fd)
        return _take(out, size), used.value

    def dev_filter_finite_t(self, cols, out_idx):
        t = make_ttable(cols)
        m = ctypes.c_uint64()
        check(lib().st_dev_filter_finite_t(self.h, ctypes.byref(t), _ptr(out_idx), ctypes.byref(m)))
        return m.value

    def dev_permute_rows_t(self, src, idx, m, dst):
        ts, td = make_ttable(src), make_ttable(dst, m)
        check(lib().st_dev_permute_rows_t(self.h, ctypes.byref(ts), _ptr(idx), ctypes.c_uint64(m), ctypes.byref(td)))

    def dev_combine(self, tables, dst):
        """tables: lists of (name, device tensor); dst: list of (name, tensor) in combine_layout order"""
        tts = [make_ttable(t) for t in tables]
        arr = (ctypes.POINTER(TTable) * len(tts))(*[ctypes.pointer(t) for t in tts])
        td = make_ttable(dst)
        check(lib().st_dev_combine(self.h, arr, ctypes.c_int32(len(tts)), ctypes.byref(td)))

    def dev_permute_rows(self, src, idx, m, dst):
        ts, td = make_table(src), make_table(dst)
        check(lib().st_dev_permute_rows(self.h, ctypes.byref(ts), _ptr(idx), ctypes.c_uint64(m), ctypes.byref(td)))

    def dev_kmeans(self, col_list, k, iters, draws, centroids, labels):
        d, n = len(col_list), len(col_list[0])
        used = ctypes.c_uint64(0)
        ptrs = (ctypes.c_void_p * d)(*[c.data_ptr() for c in col_list])
        check(lib().st_dev_kmeans(self.h, ptrs, ctypes.c_int32(d), ctypes.c_uint64(n), ctypes.c_int32(k),
                                  ctypes.c_int32(iters), _vp(draws), ctypes.c_uint64(len(draws)), ctypes.byref(used),
                                  _ptr(centroids), _ptr(labels)))
        return used.value

    def dev_cluster1d(self, col_list, iters, draws, centroids, labels):
        n = len(col_list[0])
        used = ctypes.c_uint64(0)
        ptrs = (ctypes.c_void_p * len(col_list))(*[c.data_ptr() for c in col_list])
        check(lib().st_dev_cluster1d(self.h, ptrs, ctypes.c_int32(len(col_list)), ctypes.c_uint64(n),
                                     ctypes.c_int32(iters), _vp(draws), ctypes.c_uint64(len(draws)),
                                     ctypes.byref(used), _ptr(centroids), _ptr(labels)))
        return used.value

    def dev_sog_sharded(self, comm, locals_, iters, draws, tex=None):
        """this rank's part of a sharded writeSog; locals_: list of dicts name -> device column (this
        rank's tables in global order); tex (rank 0): dict of device outputs as dev_sog's"""
        ts, arr = _tables_arg(locals_)
        meta = SogMeta()
        used = ctypes.c_uint64()
        out = None
        if tex is not None:
            out = SogTextures(*[(_ptr(tex[k]).value if k in tex else None) for k in
                                ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels')])
        check(lib().st_dev_sog_sharded(self.h, comm.h, arr, ctypes.c_int32(len(ts)), ctypes.c_int32(iters),
                                       _vp(draws), ctypes.c_uint64(len(draws)), ctypes.byref(used),
                                       ctypes.byref(meta) if tex is not None else None,
                                       ctypes.byref(out) if out is not None else None))
        return meta, used.value

    def dev_sog(self, cols, iters, draws, tex):
        """tex: dict of device uint8 tensors (see sog_geometry for sizes)"""
        t = make_table(cols)
        out = SogTextures(*[(tex[k].data_ptr() if k in tex else None) for k in
                            ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels')])
        meta = SogMeta()
        used = ctypes.c_uint64(0)
        check(lib().st_dev_sog(self.h, ctypes.byref(t), ctypes.c_int32(iters), _vp(draws),
                               ctypes.c_uint64(len(draws)), ctypes.byref(used), ctypes.byref(meta),
                               ctypes.byref(out)))
        return meta, used.value

    def dev_sog_file(self, cols, iters, draws, tex, path, dos_time=0, dos_date=0):
        """writeSog into the file at `path` (st_dev_sog_file: the step, the archive streamed to the
        file while the SH k-means runs): (meta, draws used, file bytes)"""
        t = make_table(cols)
        out = SogTextures(*[(tex[k].data_ptr() if k in tex else None) for k in
                            ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels')])
        meta = SogMeta()
        used, size = ctypes.c_uint64(0), ctypes.c_uint64(0)
        import time
        t0 = time.perf_counter()
        # no O_TRUNC: st_dev_sog_file cuts the file to the archive's length itself, and a file
        # truncated to zero and rewritten is flushed at close on ext4 (replace-via-truncate), and
        # frees its old pages first -- 10-14 ms each for a 157 MB archive
        fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
        t1 = time.perf_counter()
        try:
            check(lib().st_dev_sog_file(self.h, ctypes.byref(t), ctypes.c_int32(iters), _vp(draws),
                                        ctypes.c_uint64(len(draws)), ctypes.byref(used), ctypes.byref(meta),
                                        ctypes.byref(out), ctypes.c_int32(fd), ctypes.c_uint16(dos_time),
                                        ctypes.c_uint16(dos_date), ctypes.byref(size)))
        finally:
            t2 = time.perf_counter()
            os.close(fd)
            if os.environ.get('ST_DEBUG'):
                print(f'[splat_hip] dev_sog_file: open {1e3 * (t1 - t0):.1f} ms, call {1e3 * (t2 - t1):.1f} ms, '
                      f'close {1e3 * (time.perf_counter() - t2):.1f} ms', file=sys.stderr)
        return meta, used.value, size.value

    # ---- multi-GPU building blocks (device tensors; see splat_dist.py) ----------------
    def dev_minmax(self, cols):
        m = len(cols)
        lo, hi = (ctypes.c_double * m)(), (ctypes.c_double * m)()
        ptrs = (ctypes.c_void_p * m)(*[c.data_ptr() for c in cols])
        check(lib().st_dev_minmax(self.h, ptrs, ctypes.c_int32(m), ctypes.c_uint64(len(cols[0])), lo, hi))
        return list(lo), list(hi)

    def dev_kmeans_prepare(self, col_list):
        d, n = len(col_list), len(col_list[0])
        ptrs = (ctypes.c_void_p * d)(*[c.data_ptr() for c in col_list])
        check(lib().st_dev_kmeans_prepare(self.h, ptrs, ctypes.c_int32(d), ctypes.c_uint64(n)))

    def dev_kmeans_assign(self, col_list, k, centroids, labels):
        d, n = len(col_list), len(col_list[0])
        ptrs = (ctypes.c_void_p * d)(*[c.data_ptr() for c in col_list])
        check(lib().st_dev_kmeans_assign(self.h, ptrs, ctypes.c_int32(d), ctypes.c_uint64(n), ctypes.c_int32(k),
                                         _ptr(centroids), _ptr(labels)))

    def dev_kmeans_partials(self, col_list, nseg, k, labels, sums, sabs, emin, counts):
        d, n = len(col_list), len(col_list[0])
        ptrs = (ctypes.c_void_p * d)(*[c.data_ptr() for c in col_list])
        check(lib().st_dev_kmeans_partials(self.h, ptrs, ctypes.c_int32(d), ctypes.c_uint64(n), ctypes.c_int32(nseg),
                                           ctypes.c_int32(k), _ptr(labels), _ptr(sums), _ptr(sabs), _ptr(emin),
                                           _ptr(counts)))

    def dev_kmeans_seqsum(self, d, k, seg, pairs, running, emin, sabs):
        check(lib().st_dev_kmeans_seqsum(self.h, ctypes.c_int32(d), ctypes.c_int32(k), ctypes.c_int32(seg),
                                         _ptr(pairs), ctypes.c_uint32(len(pairs)), _ptr(running), _ptr(emin),
                                         _ptr(sabs)))

    def dev_kmeans_init_rows(self, draws, n, k, rows):
        """initializeCentroids over n global rows: rows (device uint32/int32, k) filled; returns draws used"""
        used = ctypes.c_uint64(0)
        draws = np.ascontiguousarray(draws, dtype=np.float64)
        check(lib().st_dev_kmeans_init_rows(self.h, _vp(draws), ctypes.c_uint64(len(draws)), ctypes.c_uint64(n),
                                            ctypes.c_int32(k), _ptr(rows), ctypes.byref(used)))
        return used.value

    def dev_gather_rows(self, col_list, offset, rows, out):
        """out (device f32, d*k) = the rows this rank holds, bit pattern 0 elsewhere"""
        d, k = len(col_list), len(rows)
        ptrs = (ctypes.c_void_p * d)(*[c.data_ptr() for c in col_list])
        check(lib().st_dev_gather_rows(self.h, ptrs, ctypes.c_int32(d), ctypes.c_uint64(len(col_list[0])),
                                       ctypes.c_uint64(offset), _ptr(rows), ctypes.c_int32(k), _ptr(out)))

    def dev_kmeans_finish(self, d, k, sums, sabs, emin, counts, centroids, pending):
        np_ = ctypes.c_uint32(0)
        check(lib().st_dev_kmeans_finish(self.h, ctypes.c_int32(d), ctypes.c_int32(k), _ptr(sums), _ptr(sabs),
                                         _ptr(emin), _ptr(counts), _ptr(centroids), _ptr(pending), ctypes.byref(np_)))
        return np_.value

    def dev_kmeans_average(self, d, k, pairs, running, counts, centroids):
        check(lib().st_dev_kmeans_average(self.h, ctypes.c_int32(d), ctypes.c_int32(k), _ptr(pairs),
                                          ctypes.c_uint32(len(pairs)), _ptr(running), _ptr(counts), _ptr(centroids)))

    def dev_cluster1d_codebook(self, centroids, labels, codebook, labels8):
        check(lib().st_dev_cluster1d_codebook(self.h, _ptr(centroids), _ptr(labels), ctypes.c_uint64(len(labels)),
                                              _ptr(codebook), _ptr(labels8)))

    def dev_sog_scatter(self, cols, pos, lo, hi, scale_labels, color_labels, shn_labels, tex):
        t = make_table(cols)
        out = SogTextures(*[(tex[k].data_ptr() if tex.get(k) is not None else None) for k in
                            ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels')])
        meta = SogMeta()
        check(lib().st_dev_sog_scatter(self.h, ctypes.byref(t), _ptr(pos), (ctypes.c_double * 3)(*lo),
                                       (ctypes.c_double * 3)(*hi), _ptr(scale_labels), _ptr(color_labels),
                                       _ptr(shn_labels), ctypes.byref(meta), ctypes.byref(out)))
        return meta

    def dev_sog_shn_centroids(self, codebook_labels, sh_coeffs, palette, out):
        check(lib().st_dev_sog_shn_centroids(self.h, _ptr(codebook_labels), ctypes.c_int32(sh_coeffs),
                                             ctypes.c_int32(palette), _ptr(out)))
