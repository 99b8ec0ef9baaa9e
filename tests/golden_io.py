"""Loader for the committed golden fixtures (tests/golden/<set>.{json,bin})."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


class Golden:
    def __init__(self, name):
        with open(os.path.join(GOLDEN, name + '.json')) as f:
            self.manifest = json.load(f)
        with open(os.path.join(GOLDEN, name + '.bin'), 'rb') as f:
            self.blob = f.read()
        self.meta = self.manifest['meta']

    def keys(self):
        return self.manifest['arrays'].keys()

    def __contains__(self, k):
        return k in self.manifest['arrays']

    def __getitem__(self, k):
        a = self.manifest['arrays'][k]
        arr = np.frombuffer(self.blob, dtype='<' + a['dtype'], count=a['nbytes'] // np.dtype(a['dtype']).itemsize,
                            offset=a['offset'])
        return arr.reshape(a['shape']).copy()

    def table(self, prefix):
        return {c: self[prefix + c] for c in self.meta[prefix + 'columns']}


def mulberry32(seed, n):
    """The Math.random stand-in of tests/golden/gen/make_golden.js (uniform k / 2^32)."""
    i = np.arange(1, n + 1, dtype=np.uint64)
    a = ((np.uint64(seed) + i * np.uint64(0x6D2B79F5)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    with np.errstate(over='ignore'):
        t = (a ^ (a >> np.uint32(15))) * (a | np.uint32(1))
        t = t ^ (t + (t ^ (t >> np.uint32(7))) * (t | np.uint32(61)))
    return (t ^ (t >> np.uint32(14))).astype(np.float64) / 4294967296.0


def gs_column_names(sh_coeffs):
    return (['x', 'y', 'z', 'nx', 'ny', 'nz', 'f_dc_0', 'f_dc_1', 'f_dc_2'] +
            [f'f_rest_{i}' for i in range(3 * sh_coeffs)] +
            ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3'])


def bell_splats(n, sh_coeffs, seed, cube_frac):
    """numpy restatement of make_golden.js makeBellSplats: the same draws in the same order with
    the same f64 + - * sequence, stored to float32 (round to nearest), so the table is bit-identical
    to the one the reference ran on (the fixture's input_sha256 digests check that)."""
    names = gs_column_names(sh_coeffs)
    per_row = 1 + 4 * 3 + 4 * 3 + 4 * 3 * sh_coeffs + 4 + 3 + 4 * 4
    u = mulberry32(seed, n * per_row).reshape(n, per_row)
    cols = {k: np.zeros(n, np.float32) for k in names}
    pos = [0]

    def take(w):
        s = u[:, pos[0]:pos[0] + w]
        pos[0] += w
        return s

    def bell(sigma):
        d = take(4)
        return ((((d[:, 0] + d[:, 1]) + d[:, 2]) + d[:, 3]) - 2.0) * sigma

    cube = take(1)[:, 0] < cube_frac
    for a, off in zip('xyz', (1.0, -2.0, 3.0)):
        v = bell(17.32)
        cols[a] = np.where(cube, off + (v + 34.64) * 1e-5, v).astype(np.float32)
    for c in range(3):
        cols[f'f_dc_{c}'] = bell(1.732).astype(np.float32)
    for c in range(3 * sh_coeffs):
        cols[f'f_rest_{c}'] = bell(0.1732).astype(np.float32)
    cols['opacity'] = bell(3.464).astype(np.float32)
    for c in range(3):
        cols[f'scale_{c}'] = (-7.0 + 5.0 * take(1)[:, 0]).astype(np.float32)
    for c in range(4):
        cols[f'rot_{c}'] = bell(1.732).astype(np.float32)
    assert pos[0] == per_row
    return names, cols


def sha256(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
