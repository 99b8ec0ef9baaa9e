#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY: pin the oracle at paletteSize 65,536, then extend the fixture.

1. Rebuild the sog65k table (tests/golden_io.bell_splats) and check it against the input
   digests the reference run recorded (tests/golden/sog65k.json, make_golden.js sog65k).
2. Run the oracle's writeSog (oracle/st_oracle.c st_o_sog) with the reference's 2 iterations
   and the same Math.random stream: every texture digest, meta value, draw count and the SH
   palette labels must equal the reference's -- this pins the oracle at K = 65,536.
3. Run it with 10 iterations (the reference's default, write-sog.ts:241 shIterations) and
   write tests/golden/sog65k_i10.json: texture digests, meta and draws, the fixture for
   the same table at the bench's iteration count (the reference itself would need ~1 h).

    python3 tests/golden/gen/make_sog65k_oracle.py [--threads 8] [--golden DIR]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'oracle')]
import golden_io  # noqa: E402
import oracle  # noqa: E402

TEX = ['means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_centroids', 'shN_labels']


def sog_digests(cols, iters, draws):
    rc, tex, meta, used = oracle.sog(cols, 15, iters, draws)
    assert rc == 0, rc
    out = {k: {'w': int(tex[k].shape[1]), 'h': int(tex[k].shape[0]), 'sha256': golden_io.sha256(tex[k])} for k in TEX}
    m = {'means_min': list(meta.means_min), 'means_max': list(meta.means_max),
         'scales': [float(v) for v in meta.scales_codebook], 'sh0': [float(v) for v in meta.sh0_codebook],
         'shN': [float(v) for v in meta.shn_codebook], 'palette_size': meta.palette_size, 'bands': meta.sh_bands}
    labels = (tex['shN_labels'][..., 0].astype(np.uint32) | (tex['shN_labels'][..., 1].astype(np.uint32) << 8))
    return out, m, used, labels.reshape(-1)


def ref_meta(meta):
    return {'means_min': meta['means']['mins'], 'means_max': meta['means']['maxs'],
            'scales': meta['scales']['codebook'], 'sh0': meta['sh0']['codebook'], 'shN': meta['shN']['codebook'],
            'palette_size': meta['shN']['count'], 'bands': meta['shN']['bands']}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--threads', type=int, default=os.cpu_count() or 1)
    ap.add_argument('--golden', default=os.path.join(ROOT, 'tests', 'golden'))
    ap.add_argument('--iters', type=int, default=10)
    a = ap.parse_args()
    oracle.set_threads(a.threads)
    fx = golden_io.Golden.__new__(golden_io.Golden)
    with open(os.path.join(a.golden, 'sog65k.json')) as f:
        fx.manifest = json.load(f)
    with open(os.path.join(a.golden, 'sog65k.bin'), 'rb') as f:
        fx.blob = f.read()
    fx.meta = m = fx.manifest['meta']
    names, cols = golden_io.bell_splats(m['n'], m['sh_coeffs'], m['seed'], m['cube_frac'])
    bad = [k for k in names if golden_io.sha256(cols[k]) != m['input_sha256'][k]]
    assert not bad, f'table differs from the reference run: {bad}'
    cols = {k: v for k, v in cols.items() if not k.startswith('n')}
    draws = golden_io.mulberry32(m['draw_seed'], 4 * 65536 * (a.iters + 2))

    t0 = time.time()
    tex, meta, used, labels = sog_digests(cols, m['iters'], draws)
    t2 = time.time() - t0
    assert used == m['draws'], (used, m['draws'])
    assert meta == ref_meta(m['meta']), 'meta differs from the reference'
    order = oracle.morton_order(cols['x'], cols['y'], cols['z'])  # texel i holds row order[i]
    assert np.array_equal(labels[:m['n']], fx['sh_labels'][order]), 'SH palette labels differ'
    for k in TEX:
        assert tex[k] == m['textures'][k], f'{k} differs from the reference'
    print(f'oracle == reference at {m["iters"]} iterations, palette {meta["palette_size"]} ({t2:.0f} s)')

    t0 = time.time()
    tex, meta, used, _ = sog_digests(cols, a.iters, draws)
    t10 = time.time() - t0
    out = {
        'generator': 'tests/golden/gen/make_sog65k_oracle.py (oracle/st_oracle.c st_o_sog, pinned to '
                     'sog65k.json at 2 iterations by the same script)',
        'meta': {'table': 'sog65k.json (makeBellSplats)', 'n': m['n'], 'iters': a.iters, 'draw_seed': m['draw_seed'],
                 'draws': int(used), 'textures': tex, 'meta': meta, 'oracle_threads': a.threads, 'seconds': t10,
                 'pinned': {'iters': m['iters'], 'seconds': t2}},
        'arrays': {},
    }
    with open(os.path.join(a.golden, f'sog65k_i{a.iters}.json'), 'w') as f:
        json.dump(out, f, indent=1)
    open(os.path.join(a.golden, f'sog65k_i{a.iters}.bin'), 'wb').close()
    print(f'wrote sog65k_i{a.iters}.json ({t10:.0f} s)')


if __name__ == '__main__':
    main()
