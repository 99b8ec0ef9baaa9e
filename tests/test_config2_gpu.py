"""BASELINE config 2 at its size: a 1M-splat SH-3 table -> .sog with 10 k-means iterations
(write-sog.ts:110-370; the palette k-means at paletteSize 65,536, write-sog.ts:296-359), on the
device and from a PLY file.

No fixture covers 1M splats (the reference's --no-gpu path would take days), so the output is
checked through the reference's definitions on every label and texel and on sampled centroids
(bench.py's verify_step: the verified step IS the computed one):
  * all 1M SH labels are exact f64 argmins over the centroids the last assign used
    (kd-tree.ts:26-35 order); exact ties, which the KdTree order decides, are counted;
  * 256 sampled centroids (and the largest cluster's) are the f32-rounded sequential f64 means
    of their members in ascending point order (calcAverage, k-means.ts:41-63);
  * all 1M shN_labels texels hold the label of the row at their Morton position;
and the PLY file -> .sog file path (read-ply.ts:111-191 -> writeSog -> ZIP) gives the same
archive bytes as the in-memory step."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'splat-transform_amd', 'py'))

pytestmark = pytest.mark.gpu

N = 1_000_000


def test_config2_1M_sh3_10_iterations():
    import torch

    import bench
    import splat_hip as sh
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = sh.Context(0)
    try:
        ctx.set_stream(stream.cuda_stream)
        cols = bench.synth_table(N, 2002, dev)
        W, H, pal, cw, ch = sh.sog_geometry(N, 15)
        assert pal == 65536  # write-sog.ts:296: min(64, 2^floor(log2(n / 1024))) * 1024
        u8 = dict(device=dev, dtype=torch.uint8)
        tex = {k: torch.empty(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
        tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
        draws = np.random.default_rng(42).random(2 * 65536 * 12)

        def step():
            return ctx.dev_sog(cols, 10, draws, tex)
        meta, used = step()
        torch.cuda.synchronize()
        assert meta.palette_size == 65536 and meta.sh_bands == 3 and used >= 65536
        v = bench.verify_step(ctx, cols, tex, step, n_clusters=256, all_labels=True)
        assert v['ok'], v
        assert v['labels_checked'] == N and v['clusters_checked'] == 256 and v['texel_labels_checked'] == N
        # the CLI's in.ply -> out.sog: the file path gives the in-memory step's archive
        addr, size = ctx.dev_sog_bundle_view(meta, N, tex, 0, 0)
        ref = bytes(bench.ctypes_char_array(size).from_address(addr))
        e2e = bench.end_to_end(ctx, cols, 10, draws, tex, ref, meta, reps=1)
        assert e2e['archive_equals_in_memory_step'], e2e
        # the Node drop-in (readPly -> writeSogFile over the addon, Math.random = the same draws,
        # Date pinned): every rep's file is the library's archive of this step
        nh = e2e['node_host']
        if nh is not None:
            assert nh.get('archive_equals_library') and nh['resident_columns_reused'] == 59, nh
    finally:
        ctx.close()
