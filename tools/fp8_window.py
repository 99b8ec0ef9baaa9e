#!/usr/bin/env python3
"""The fp8 question, measured: how wide would the assign's certified score
window be if the sweep's operands were e4m3 (block-scaled) instead of fp16?

The sweep (st_kmeans_nd.hip, k_sweep) scores every centroid c against a point p as
|c|^2 - 2 p.c from low-precision operands, then certifies its top candidates with an error bound:
every centroid whose approximate score is within (its bound + the best one's bound) of the best
approximate score may be the exact f64 argmin (kd-tree.ts:26-35 order) and has to be settled
exactly.  A point whose window holds more than 3 centroids leaves the fast path (the sweep keeps
the top 3 per tile; beyond that the point is re-collected).

This script, on the container CPU (numpy, f64 exact scores), takes a 20k-point sample of the
bench's SH data (45 dims; Gaussian N(0, 0.1^2) as bench.py, and the heavy-tailed t3 rows of
tests/test_gpu_parity.py) against K = 65,536 centroids -- the data rows the reference's init
draws (iteration 0) and the means after two Lloyd iterations over a 655k-row sample (later
iterations) -- and counts, per operand format, the points whose window holds > 1, > 3 centroids:
  fp16   : IEEE half (u = 2^-11), what the kernel runs on (v_mfma_f32_32x32x16_f16)
  e4m3   : OCP fp8 e4m3 with one power-of-two scale per 32-element block (MX-style), u = 2^-4
  e5m2   : the same with e5m2 (u = 2^-3)
The bound is the one an implementable kernel has: Cauchy-Schwarz on the quantisation errors,
2 (|dp| |c| + |p| |dc| + |dp| |dc|) + the f32 accumulation, per (point, centroid); the 'tight'
column uses the elementwise 2 (|dp|.|c| + |p|.|dc| + |dp|.|dc|) (three more GEMMs per pass --
a lower bound on any certified window).  The exact argmin lies in every window (checked).

  python tools/fp8_window.py [points] [--lloyd-sample N]   -> gpurun_out/fp8_window.json"""
import argparse
import json
import os
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K, D = 65536, 45


def heavy_tailed(rng, n, d, scale=0.1):
    m = np.eye(d) + 0.5 * np.random.default_rng(3).normal(0, 1, (d, d)) / np.sqrt(d)
    t = rng.normal(0, 1, (n, d)) / np.sqrt((rng.normal(0, 1, (n, 3)) ** 2).sum(1, keepdims=True) / 3)
    return (t @ m.T * scale).astype(np.float32)


def data(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == 'gauss':
        return (rng.normal(0, 1, (n, D)) * 0.1).astype(np.float32)
    return heavy_tailed(rng, n, D)


def quant_minifloat(x, mbits, emin, emax_val):
    """round-to-nearest-even onto a minifloat with `mbits` mantissa bits, normal exponents >= emin
    (subnormal spacing 2^(emin - mbits)) and largest finite value emax_val (saturating)"""
    a = np.abs(x).astype(np.float64)
    e = np.floor(np.log2(np.maximum(a, np.finfo(np.float64).tiny)))
    e = np.maximum(e, emin)
    sp = np.exp2(e - mbits)
    q = np.minimum(np.round(a / sp) * sp, emax_val)
    return np.sign(x) * q


def quant(x, fmt):
    """x [rows, D] f32 -> the value the kernel's operand represents (f64)"""
    if fmt == 'fp16':
        return x.astype(np.float16).astype(np.float64)
    mbits, emin, vmax = {'e4m3': (3, -6, 448.0), 'e5m2': (2, -14, 57344.0)}[fmt]
    out = np.empty(x.shape, np.float64)
    for b0 in range(0, x.shape[1], 32):  # MX-style: one power-of-two scale per 32-element block
        blk = x[:, b0:b0 + 32].astype(np.float64)
        amax = np.abs(blk).max(1, keepdims=True)
        scale = np.exp2(np.ceil(np.log2(np.maximum(amax, 1e-30) / vmax)))
        out[:, b0:b0 + 32] = quant_minifloat(blk / scale, mbits, emin, vmax) * scale
    return out


def lloyd(pts, cen, iters, block=4096):
    """plain Lloyd iterations (f32 GEMM argmin; the means of the members in f64)"""
    for _ in range(iters):
        cn = (cen.astype(np.float64) ** 2).sum(1)
        lab = np.empty(len(pts), np.int64)
        for a in range(0, len(pts), block):
            s = cn[None, :] - 2.0 * (pts[a:a + block] @ cen.T)
            lab[a:a + block] = s.argmin(1)
        sums = np.zeros((len(cen), D))
        np.add.at(sums, lab, pts.astype(np.float64))
        cnt = np.bincount(lab, minlength=len(cen))
        keep = cnt > 0
        cen = cen.copy()
        cen[keep] = (sums[keep] / cnt[keep, None]).astype(np.float32)
    return cen


def windows(pts, cen, fmt, block=512):
    """per point: centroids in the certified window (Cauchy-Schwarz bound, tight bound)"""
    c64 = cen.astype(np.float64)
    cn = (c64 ** 2).sum(1)
    cq = quant(cen, fmt)
    dc = cq - c64
    ncen, ndc, ncq = np.linalg.norm(c64, axis=1), np.linalg.norm(dc, axis=1), np.linalg.norm(cq, axis=1)
    cqf, adc, ac64 = cq.astype(np.float32), np.abs(dc).astype(np.float32), np.abs(c64).astype(np.float32)
    acc = 2 * D * 2.0 ** -24  # f32 accumulation of the D products (relative to |pq| |cq|)
    n_cs, n_tight, lost = [], [], 0
    for a in range(0, len(pts), block):
        p64 = pts[a:a + block].astype(np.float64)
        pq = quant(pts[a:a + block], fmt)
        dp = pq - p64
        exact = cn[None, :] - 2.0 * (p64 @ c64.T)
        approx = cn[None, :] - 2.0 * (pq.astype(np.float32) @ cqf.T).astype(np.float64)
        npn, ndp, npq = np.linalg.norm(p64, axis=1), np.linalg.norm(dp, axis=1), np.linalg.norm(pq, axis=1)
        acc_t = acc * np.outer(npq, ncq)
        b_cs = 2 * (np.outer(ndp, ncen) + np.outer(npn, ndc) + np.outer(ndp, ndc)) + acc_t
        b_t = 2 * ((np.abs(dp).astype(np.float32) @ ac64.T) + (np.abs(p64).astype(np.float32) @ adc.T) +
                   (np.abs(dp).astype(np.float32) @ adc.T)).astype(np.float64) * (1 + 1e-6) + acc_t
        best = exact.argmin(1)
        for b, out in ((b_cs, n_cs), (b_t, n_tight)):
            top = (approx + b).min(1, keepdims=True)
            inwin = (approx - b) <= top
            out.append(inwin.sum(1))
            lost += int((~inwin[np.arange(len(best)), best]).sum())
    n_cs, n_tight = np.concatenate(n_cs), np.concatenate(n_tight)

    def summary(v):
        return {'mean_candidates': float(v.mean()), 'frac_gt1': float((v > 1).mean()),
                'frac_gt3': float((v > 3).mean()), 'frac_gt64': float((v > 64).mean()),
                'p99_candidates': float(np.percentile(v, 99)), 'max_candidates': int(v.max())}
    return {'cauchy_schwarz': summary(n_cs), 'tight': summary(n_tight), 'exact_argmin_outside_window': lost}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('points', type=int, nargs='?', default=20_000)
    ap.add_argument('--lloyd-sample', type=int, default=655_360)
    ap.add_argument('--kinds', default='gauss,t3')
    a = ap.parse_args()
    out = {'K': K, 'D': D, 'points': a.points, 'lloyd_sample': a.lloyd_sample, 'cases': {}}
    for kind in a.kinds.split(','):
        t0 = time.time()
        pool = data(kind, K + a.points + a.lloyd_sample, 1002 if kind == 'gauss' else 3003)
        cen0 = pool[:K]  # initializeCentroids: data rows (k-means.ts:8-20)
        pts = pool[K:K + a.points]
        cen2 = lloyd(pool[K + a.points:], cen0, 2)
        for stage, cen in (('iteration0_data_rows', cen0), ('after_2_lloyd', cen2)):
            for fmt in ('fp16', 'e4m3', 'e5m2'):
                r = windows(pts, cen, fmt)
                out['cases'][f'{kind}/{stage}/{fmt}'] = r
                print(kind, stage, fmt, json.dumps(r), flush=True)
        print(kind, f'{time.time() - t0:.0f} s', flush=True)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(ROOT, 'gpurun_out', 'fp8_window.json'), 'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
