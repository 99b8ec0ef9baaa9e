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
