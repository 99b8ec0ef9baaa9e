#!/usr/bin/env python3
"""Host one-call transfer rates: st_filter_nan over a 10M x 62-column float32 table in pageable
numpy arrays (2.48 GB up, the survivors down), with ST_XFER_PRINT=1 reporting each staged copy.
    ST_XFER_THREADS=.. ST_XFER_CHUNK_MB=.. python tools/xfer_probe.py [n]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
os.environ.setdefault('ST_XFER_PRINT', '1')
import numpy as np
import torch  # noqa: F401  (HIP runtime first, as the tests do)

import splat_hip as sh

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
rng = np.random.default_rng(3)
cols = {f'c{i}': rng.random(n, dtype=np.float32) for i in range(62)}
ctx = sh.Context(0)
for rep in range(3):
    t0 = time.perf_counter()
    m = len(ctx.filter_nan(cols)[0][1])
    print(f'filter_nan call {1e3 * (time.perf_counter() - t0):.1f} ms (kept {m})', flush=True)
