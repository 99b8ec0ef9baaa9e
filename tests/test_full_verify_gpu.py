"""The headline workload checked whole: 10M synthetic SH-3 splats, palette 65,536, 10 k-means
iterations (BASELINE.json configs[1]; write-sog.ts:296-359).  Every one of the 10M labels of the
last assign is the exact f64 argmin over the centroids it used (kd-tree.ts:22-70; an f64 GEMM in
torch decides all but near-ties, which take the reference's sequential distance), 1,024 sampled
centroids are the sequential f64 means of their members (k-means.ts:41-63), and every shN_labels
texel sits at its Morton position -- bench.py's verify_step with all_labels."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_headline_step_every_label_exact():
    import torch

    import bench
    import splat_hip as sh
    dev = torch.device('cuda', 0)
    ctx = sh.Context(0)
    ctx.bind_torch_stream(dev)
    n = 10_000_000
    cols = bench.synth_table(n, 1002, dev)
    W, H, pal, cw, ch = sh.sog_geometry(n, 15)
    assert pal == 65536
    u8 = dict(device=dev, dtype=torch.uint8)
    tex = {k: torch.empty(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
    tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
    draws = np.random.default_rng(42).random(2 * 65536 * 12)

    def step():
        return ctx.dev_sog(cols, 10, draws, tex)
    step()
    v = bench.verify_step(ctx, cols, tex, step, n_clusters=1024, all_labels=True)
    assert v['ok'], v
    assert v['labels_checked'] == n and v['labels_wrong'] == 0
    assert v['centroid_values_wrong'] == 0 and v['texel_labels_wrong'] == 0
    ctx.close()


def test_heavy_tailed_scene_every_label_exact():
    """a 2M-splat SH-3 table whose SH rows are heavy-tailed and correlated (Student-t nu = 3
    through a fixed mixing matrix, what trained scenes carry; tests/test_gpu_parity.py
    heavy_tailed), 5% of the positions in a 1e-3 cube: writeSog's palette k-means at 65,536 with 10 iterations,
    every label and 512 sampled centroids checked against the reference's definitions"""
    import torch

    import bench
    import splat_hip as sh
    from test_gpu_parity import heavy_tailed
    dev = torch.device('cuda', 0)
    ctx = sh.Context(0)
    ctx.bind_torch_stream(dev)
    n = 2_000_000
    cols = bench.synth_table(n, 77, dev)
    rng = np.random.default_rng(77)
    for i, c in enumerate(heavy_tailed(rng, n, 45)):
        cols[f'f_rest_{i}'] = torch.from_numpy(c).to(dev)
    W, H, pal, cw, ch = sh.sog_geometry(n, 15)
    assert pal == 65536
    u8 = dict(device=dev, dtype=torch.uint8)
    tex = {k: torch.empty(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
    tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
    draws = np.random.default_rng(5).random(2 * 65536 * 12)

    def step():
        return ctx.dev_sog(cols, 10, draws, tex)
    step()
    v = bench.verify_step(ctx, cols, tex, step, n_clusters=512, all_labels=True)
    assert v['ok'], v
    assert v['labels_checked'] == n and v['labels_wrong'] == 0 and v['centroid_values_wrong'] == 0
    ctx.close()
