#!/usr/bin/env python3
"""Where the realistic table's step goes (bench.py realistic_table: heavy-tailed correlated SH,
all-zero SH rows, clumped positions), one ingredient at a time against the Gaussian table:
per-step wall time, the stage marks (ST_TIMING) and the named kernels' totals of one step.
  python tools/realistic_probe.py [n]      -> gpurun_out/realistic_probe.json"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))
sys.path.insert(0, ROOT)

import numpy as np
import torch

import bench
import splat_hip as sh

KERNELS = ('kn.sweep', 'kn.collect', 'kn.fixrow', 'kn.fixpair', 'kn.exact', 'kn.sumnd', 'k1.assign', 'k1.sum')


def main(n=10_000_000, only=None):
    dev = torch.device('cuda', 0)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    ctx = sh.Context(0)
    ctx.set_stream(s.cuda_stream)
    draws = np.random.default_rng(42).random(2 * 65536 * 12)
    W, H, pal, cw, ch = sh.sog_geometry(n, 15)
    u8 = dict(device=dev, dtype=torch.uint8)
    tex = {k: torch.empty(W * H * 4, **u8) for k in bench.TEX_ORDER[:6]}
    tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
    cases = {
        'gauss': lambda: bench.synth_table(n, bench.SEED + 77, dev),
        'realistic': lambda: bench.realistic_table(n, bench.SEED + 77, dev),
        'no_zero_rows': lambda: bench.realistic_table(n, bench.SEED + 77, dev, zero_frac=0.0),
        'no_clumps': lambda: bench.realistic_table(n, bench.SEED + 77, dev, clump_frac=0.0),
        'zero_rows_only': lambda: zero_only(n, dev),
    }
    out = {}
    for name, make in cases.items():
        if only and name not in only:
            continue
        cols = make()
        torch.cuda.synchronize()
        ctx.dev_sog(cols, 10, draws, tex)  # warm
        torch.cuda.synchronize()
        ts = []
        for _ in range(2):
            t0 = time.perf_counter()
            ctx.dev_sog(cols, 10, draws, tex)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        os.environ['ST_TIMING'] = '1'
        ctx.set_profiling(True)
        ctx.reset_kernel_stats()
        ctx.dev_sog(cols, 10, draws, tex)
        torch.cuda.synchronize()
        stages = json.loads(ctx.timings())
        kern = {k: ctx.kernel_stats(k) for k in KERNELS}
        ctx.set_profiling(False)
        os.environ.pop('ST_TIMING')
        out[name] = {'ms': ts, 'stages': stages, 'kernels_ms_launches': kern, 'assign': ctx.kmeans_stats()}
        print(name, [round(t, 1) for t in ts], json.dumps(stages), json.dumps(kern), json.dumps(out[name]['assign']),
              flush=True)
        del cols
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, 'gpurun_out', 'realistic_probe.json'), 'w'), indent=1)


def zero_only(n, dev):
    cols = bench.synth_table(n, bench.SEED + 77, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    zero = torch.rand(n, generator=g, device=dev) < 0.3
    for i in range(45):
        cols[f'f_rest_{i}'][zero] = 0
    return cols


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000, sys.argv[2].split(',') if len(sys.argv) > 2 else None)
