#!/usr/bin/env python3
"""Which k-means golden cases does the library (ST_LIB) miss, and where (debugging aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ('splat-transform_amd/py', 'oracle', 'tests'):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import torch  # noqa: F401

import oracle
import splat_hip as sh
from golden_io import Golden

ctx = sh.Context(0)
g = Golden('kmeans')
for case in g.meta['cases']:
    name = case['name']
    cols = [g[f'{name}_p{j}'] for j in range(case['d'])]
    draws = oracle.mulberry32(case['seed'], case['draws'] + 16)
    cent, labels, used = ctx.kmeans(cols, case['k'], case['iters'], draws)
    bad_c = sum(int((cent[j].view(np.uint32) != g[f'{name}_c{j}'].view(np.uint32)).sum()) for j in range(case['d']))
    bad_l = np.nonzero(labels != g[f'{name}_labels'])[0]
    print(f"{name}: n={len(cols[0])} d={case['d']} k={case['k']} iters={case['iters']} used {used} vs {case['draws']}"
          f" centroid mismatches {bad_c} label mismatches {len(bad_l)} first {bad_l[:5]}", flush=True)
    for i in bad_l[:3]:
        p = np.array([c[i] for c in cols], np.float64)
        gl, ml = g[f'{name}_labels'][i], labels[i]
        print('   point', i, 'golden label', gl, 'ours', ml)
