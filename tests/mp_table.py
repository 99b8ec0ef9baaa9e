"""The deterministic SH-3 splat table of the multi-process tests (tests/test_multiproc_gpu.py and
its rank processes, tests/mp_sog_rank.py): the bench's distributions plus values
that make the order-free sum certificate fail, so the sequential hand-off between ranks runs:
  * scales spread over ~15 decades (1-D cluster sums: the cluster1d pending chain);
  * 0.05% of the SH coefficients scaled by 1e-9 (N-D cluster sums whose members span many
    binades: the SH k-means pending chain).
Not collected by pytest."""
import numpy as np

NAMES = ['x', 'y', 'z', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] + \
    ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3']


def table(n, seed):
    rng = np.random.default_rng(seed)
    cols = {}
    cube = rng.random(n) < 0.05
    for a, off in zip('xyz', (1.0, -2.0, 3.0)):
        cols[a] = np.where(cube, off + rng.random(n) * 1e-3, rng.normal(0, 10, n)).astype(np.float32)
    for i in range(3):
        cols[f'f_dc_{i}'] = rng.normal(0, 1, n).astype(np.float32)
    for i in range(45):
        v = rng.normal(0, 0.1, n)
        tiny = rng.random(n) < 5e-4
        cols[f'f_rest_{i}'] = np.where(tiny, v * 1e-9, v).astype(np.float32)
    cols['opacity'] = rng.normal(0, 2, n).astype(np.float32)
    for i in range(3):
        v = rng.random(n) * 5 - 7
        u = rng.random(n)
        cols[f'scale_{i}'] = np.where(u < 0.3, v * 1e-9, np.where(u > 0.9, v * 1e5, v)).astype(np.float32)
    for i in range(4):
        cols[f'rot_{i}'] = rng.normal(0, 1, n).astype(np.float32)
    return cols


def draws(seed):
    """the host's Math.random stream (the same on every rank)"""
    return np.random.default_rng(seed + 1).random(1 << 20)
