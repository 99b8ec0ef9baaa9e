#!/usr/bin/env python3
"""One rank of a sharded writeSog job of separate processes on one GPU (test helper for
tests/test_multiproc_gpu.py; not collected by pytest).  The library's own one-rank-per-process
path -- st_comm_init_host + st_dev_sog_sharded, the same calls bench.py --gpus N makes, with
host shared memory carrying the bytes instead of RCCL -- over rows [cuts[rank], cuts[rank+1])
of the deterministic table tests/mp_table.py builds.  Writes <out>/rank<r>.json: the draws
consumed, and on rank 0 the sha256 of the seven textures and the meta fields."""
import argparse
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
sys.path.insert(0, HERE)

TEX = ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels', 'shN_centroids')


def digest(tex, meta):
    import numpy as np
    h = hashlib.sha256()
    for k in TEX:
        if k in tex:
            h.update(tex[k].cpu().numpy().tobytes())
    for f in ('width', 'height', 'sh_bands', 'palette_size', 'shn_width', 'shn_height'):
        h.update(int(getattr(meta, f)).to_bytes(8, 'little'))
    for f in ('means_min', 'means_max', 'scales_codebook', 'sh0_codebook', 'shn_codebook'):
        h.update(np.array(list(getattr(meta, f)), np.float64).tobytes())
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--world', type=int, required=True)
    ap.add_argument('--rank', type=int, required=True)
    ap.add_argument('--name', required=True)
    ap.add_argument('--n', type=int, required=True)
    ap.add_argument('--cuts', required=True, help='comma-separated row bounds, world + 1 of them')
    ap.add_argument('--seed', type=int, default=11)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--slot', type=int, default=0)
    ap.add_argument('--out', required=True)
    ap.add_argument('--repeat', type=int, default=1, help='calls of the sharded step (the result of each must agree)')
    a = ap.parse_args()
    import numpy as np
    import torch

    import mp_table
    import splat_hip as sh
    cuts = [int(x) for x in a.cuts.split(',')]
    lo, hi = cuts[a.rank], cuts[a.rank + 1]
    dev = torch.device('cuda', 0)
    full = mp_table.table(a.n, a.seed)
    cols = {k: torch.from_numpy(v[lo:hi].copy()).to(dev) for k, v in full.items()}
    del full
    draws = mp_table.draws(a.seed)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = sh.Context(0)
    ctx.set_stream(stream.cuda_stream)
    comm = sh.Comm.host(ctx, a.world, a.rank, a.name, slot_bytes=a.slot, timeout_s=300)
    tex = None
    if a.rank == 0:
        W, H, pal, cw, ch = sh.sog_geometry(a.n, 15)
        u8 = dict(device=dev, dtype=torch.uint8)
        tex = {k: torch.empty(W * H * 4, **u8) for k in TEX[:6]}
        tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
    res = {'rank': a.rank, 'rows': hi - lo, 'used': [], 'sha256': []}
    for _ in range(a.repeat):
        meta, used = ctx.dev_sog_sharded(comm, [cols], a.iters, draws, tex)
        torch.cuda.synchronize()
        res['used'].append(used)
        if a.rank == 0:
            res['sha256'].append(digest(tex, meta))
    comm.close()
    ctx.close()
    with open(os.path.join(a.out, f'rank{a.rank}.json'), 'w') as f:
        json.dump(res, f)


if __name__ == '__main__':
    main()
