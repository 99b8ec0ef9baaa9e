#!/usr/bin/env python3
"""Radix sort stress on the device: stable (key, index) sorts of several sizes and key widths
through the Morton and k-means entry points are checked against numpy's stable argsort."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import numpy as np
import torch

import oracle
import splat_hip as sh

ctx = sh.Context(0)
for n in (1, 5, 4095, 4096, 4097, 100_000, 3_000_001, 10_000_000):
    rng = np.random.default_rng(n)
    x, y, z = (rng.normal(0, 5, n).astype(np.float32) for _ in range(3))
    t0 = time.time()
    got = ctx.morton_order(x, y, z)
    dt = time.time() - t0
    ok = True
    if n <= 3_000_001:
        ok = np.array_equal(got, oracle.morton_order(x, y, z))
    print(f'morton n={n}: {"ok" if ok else "MISMATCH"} {dt * 1e3:.1f} ms', flush=True)
    if not ok:
        sys.exit(1)

# clumped inputs: deeper recursion levels (segmented extents, small-segment sorts, compaction)
for kind, n in (('clumps', 3_000_000), ('clumps_dup', 2_000_000), ('lattice', 3_000_000), ('blobs', 3_000_000),
                ('mixed', 3_000_000)):
    rng = np.random.default_rng(len(kind) * 7 + n)
    x, y, z = (rng.normal(0, 5, n).astype(np.float32) for _ in range(3))
    if kind.startswith('clumps') or kind == 'mixed':
        m = rng.random(n) < 0.8
        size = 600 if kind != 'mixed' else int(rng.integers(300, 9000))
        cid = rng.integers(0, max(1, int(n * 0.8) // size), n)
        cx, cy, cz = (rng.normal(0, 5, cid.max() + 1).astype(np.float32) for _ in range(3))
        jit = 0.0 if kind == 'clumps_dup' else 1e-5
        for a, cc in ((x, cx), (y, cy), (z, cz)):
            a[m] = (cc[cid[m]] + a[m] * jit).astype(np.float32)
        if kind == 'clumps_dup':
            x[m & (rng.random(n) < 0.5)] += np.float32(1e-4)
        if kind == 'mixed':  # some big clumps too, NaNs, a flat axis in part of them
            big = rng.random(n) < 0.1
            for a in (x, y, z):
                a[big] = (3.0 + a[big] * 1e-6).astype(np.float32)
            z[m & (cid % 7 == 0)] = 2.0
            y[rng.random(n) < 0.001] = np.nan
    elif kind == 'lattice':
        for a in (x, y, z):
            a[:] = np.round(a * 0.8) / 0.8
    else:
        m = rng.random(n) < 0.6
        centre = rng.integers(0, 300, n).astype(np.float32)
        for a in (x, y, z):
            a[m] = (centre[m] * 0.03 + a[m] * 1e-5).astype(np.float32)
    perm = rng.permutation(n).astype(np.uint32)
    for ix in (None, perm):
        t0 = time.time()
        got = ctx.morton_order(x, y, z, ix)
        dt = time.time() - t0
        ok = np.array_equal(got, oracle.morton_order(x, y, z, ix))
        print(f'morton {kind} n={n} {"perm" if ix is not None else "iota"}: {"ok" if ok else "MISMATCH"} {dt * 1e3:.1f} ms',
              flush=True)
        if not ok:
            sys.exit(1)
