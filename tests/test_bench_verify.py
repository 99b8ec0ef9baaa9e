"""bench.py checks its own output (verify_step): the check passes on the library's step and fails
when the step's output is wrong -- a texel label moved, or a step that is not deterministic."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def env():
    import torch

    import bench
    import splat_hip as sh
    dev = torch.device('cuda', 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = sh.Context(0)
    ctx.set_stream(stream.cuda_stream)
    n = 70_000  # paletteSize 65,536 from 65,536 splats (write-sog.ts:310)
    cols = bench.synth_table(n, 1234, dev)
    W, H, pal, cw, ch = sh.sog_geometry(n, 15)
    assert pal == 65536
    u8 = dict(device=dev, dtype=torch.uint8)
    tex = {k: torch.empty(W * H * 4, **u8) for k in ('means_l', 'means_u', 'quats', 'scales', 'sh0', 'shN_labels')}
    tex['shN_centroids'] = torch.empty(cw * ch * 4, **u8)
    draws = np.random.default_rng(42).random(2 * 65536 * 5)
    yield bench, ctx, cols, tex, draws
    ctx.close()


def test_verify_passes_on_the_library_step(env):
    bench, ctx, cols, tex, draws = env

    def step():
        return ctx.dev_sog(cols, 3, draws, tex)
    step()
    v = bench.verify_step(ctx, cols, tex, step, n_labels=1024, n_clusters=16)
    assert v['ok'], v
    assert v['labels_wrong'] == 0 and v['texel_labels_wrong'] == 0 and v['centroid_values_wrong'] == 0


def test_verify_fails_on_a_wrong_texel(env):
    bench, ctx, cols, tex, draws = env

    def step():
        out = ctx.dev_sog(cols, 3, draws, tex)
        tex['shN_labels'][4 * 17] ^= 1  # one palette label off by one
        return out
    step()
    v = bench.verify_step(ctx, cols, tex, step, n_labels=256, n_clusters=4)
    assert not v['ok'] and v['texel_labels_wrong'] == 1, v


def test_verify_fails_when_the_step_is_not_reproducible(env):
    bench, ctx, cols, tex, draws = env
    calls = [0]

    def step():
        calls[0] += 1
        return ctx.dev_sog(cols, 3, draws[calls[0]:], tex)  # another Math.random stream each call
    step()
    v = bench.verify_step(ctx, cols, tex, step, n_labels=256, n_clusters=4)
    assert not v['ok'] and not v['textures_equal_timed_step'], v
