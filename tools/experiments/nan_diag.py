import sys, numpy as np
sys.path.insert(0, 'splat-transform_amd/py'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
import torch
import splat_hip as sh
from golden_io import Golden
ctx = sh.Context(0)
for gname in ('typed_columns', 'process_chain'):
    G = Golden(gname)
    for c in G.meta['cases']:
        src = [(k, G[f'{c}_in_{k}'].copy()) for k in G.meta[f'{c}_in_columns']]
        out = ctx.process(src, G.meta[f'{c}_actions'])
        for tag, got in (('after', src), ('out', out)):
            for k, a in got:
                b = G[f'{c}_{tag}_{k}']
                if a.tobytes() != b.tobytes():
                    av, bv = a.view(np.uint8).reshape(len(a), -1), b.view(np.uint8).reshape(len(b), -1)
                    bad = np.nonzero((av != bv).any(1))[0]
                    fa = a.astype(np.float64) if a.dtype.kind == 'f' else None
                    nanonly = fa is not None and np.isnan(a[bad]).all() and np.isnan(b[bad]).all()
                    print(gname, c, tag, k, a.dtype, 'rows', bad[:6], 'nan-only' if nanonly else 'VALUES',
                          [hex(int(x)) for x in a[bad[:3]].view(np.uint64 if a.dtype == np.float64 else np.uint32 if a.dtype == np.float32 else a.dtype)] if a.dtype.kind=='f' else a[bad[:3]],
                          [hex(int(x)) for x in b[bad[:3]].view(np.uint64 if b.dtype == np.float64 else np.uint32 if b.dtype == np.float32 else b.dtype)] if b.dtype.kind=='f' else b[bad[:3]])
print('done')
