"""Parity of the HIP path (through the C-ABI) against the reference's golden
vectors and the pinned CPU restatement.  Integer / byte / index outputs must
be bit-exact; float outputs of the transform are compared bit-exactly too
(NaN as NaN), which is stricter than the 1e-5 relative bound north_star states.
"""
import numpy as np
import pytest

import oracle
import splat_hip as sh
from golden_io import Golden
from test_oracle_golden import same_bits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    import torch  # noqa: F401  (initialised before the library's runtime: see splat_hip.Context)
    return sh.Context(0)


@pytest.mark.parametrize('band', [0, 1, 2, 3])
def test_transform_golden(ctx, band):
    g = Golden('transform')
    for li, acts in enumerate(g.meta['actions']):
        cols = g.table(f'b{band}_in_')
        for act in acts:
            ctx.transform(cols, sh.action_params(act['kind'], act['value']))
        for k in cols:
            key = f'b{band}_a{li}_{k}'
            if key in g:
                same_bits(cols[k], g[key])


def test_transform_large_vs_oracle(ctx):
    rng = np.random.default_rng(1003)
    n = 200_000
    names = ['x', 'y', 'z'] + [f'f_rest_{i}' for i in range(45)] + ['scale_0', 'scale_1', 'scale_2'] + \
        [f'rot_{i}' for i in range(4)]
    cols = {k: rng.normal(0, 1, n).astype(np.float32) for k in names}
    ref = {k: v.copy() for k, v in cols.items()}
    op = oracle.transform_params(euler=(0, 45, 0))
    oracle.transform(ref, op, 15)
    ctx.transform(cols, sh.action_params('rotate', (0, 45, 0)))
    for k in names:
        same_bits(cols[k], ref[k])


def test_morton_golden(ctx):
    g = Golden('ordering')
    for name in g.meta['cases']:
        got = ctx.morton_order(g[f'{name}_x'], g[f'{name}_y'], g[f'{name}_z'])
        same_bits(got, g[f'{name}_order'])


@pytest.mark.parametrize('n,frac', [(300_000, 0.05), (1_000_000, 0.2)])
def test_morton_large_vs_oracle(ctx, n, frac):
    rng = np.random.default_rng(1000 + n)
    x, y, z = (rng.normal(0, 10, n).astype(np.float32) for _ in range(3))
    m = rng.random(n) < frac
    for a in (x, y, z):
        a[m] = (1 + rng.random(m.sum()) * 1e-3).astype(np.float32)
    got = ctx.morton_order(x, y, z)
    want = oracle.morton_order(x, y, z)
    same_bits(got, want)


def test_compressed_ply_golden(ctx):
    g = Golden('compressed_ply')
    for name in g.meta['cases']:
        cols = g.table(f'{name}_in_')
        nsh = sum(1 for c in cols if c.startswith('f_rest_'))
        order = ctx.morton_order(cols['x'], cols['y'], cols['z'])
        chunk, vertex, shb = ctx.pack_compressed(cols, order, nsh)
        same_bits(chunk, g[f'{name}_chunk'])
        same_bits(vertex, g[f'{name}_vertex'])
        same_bits(shb, g[f'{name}_sh'])


def test_filter_nan_golden(ctx):
    g = Golden('filter_combine')
    cols = g.table('in_')
    keep = ctx.filter_finite(cols)
    out = g.table('out_')
    for k in cols:
        same_bits(cols[k][keep], out[k])


def test_kmeans_golden(ctx):
    g = Golden('kmeans')
    for case in g.meta['cases']:
        name = case['name']
        cols = [g[f'{name}_p{j}'] for j in range(case['d'])]
        draws = oracle.mulberry32(case['seed'], case['draws'] + 16)
        cent, labels, used = ctx.kmeans(cols, case['k'], case['iters'], draws)
        assert used == case['draws'], name
        for j in range(case['d']):
            same_bits(cent[j], g[f'{name}_c{j}'])
        same_bits(labels, g[f'{name}_labels'])


def test_cluster1d_golden(ctx):
    g = Golden('kmeans')
    m = g.meta['cluster1d']
    cols = [g[f'cluster1d_p{j}'] for j in range(3)]
    cent, labels, used = ctx.cluster1d(cols, m['iters'], oracle.mulberry32(m['seed'], 1000))
    assert used == m['draws']
    same_bits(cent, g['cluster1d_centroids'])
    for j in range(3):
        same_bits(labels[j], g[f'cluster1d_l{j}'])


def test_sog_golden(ctx):
    g = Golden('sog')
    for case in g.meta['cases']:
        name = case['name']
        cols = g.table(f'{name}_in_')
        tex, meta, used = ctx.sog(cols, case['iters'], oracle.mulberry32(case['seed'], case['draws'] + 64))
        assert used == case['draws'], name
        for k, v in tex.items():
            same_bits(v, g[f'{name}_{k}'])
        ref = case['meta']
        assert list(meta.means_min) == ref['means']['mins']
        assert list(meta.means_max) == ref['means']['maxs']
        same_bits(np.array(meta.scales_codebook, np.float32), np.array(ref['scales']['codebook'], np.float32))
        same_bits(np.array(meta.sh0_codebook, np.float32), np.array(ref['sh0']['codebook'], np.float32))
        if 'shN' in ref:
            same_bits(np.array(meta.shn_codebook, np.float32), np.array(ref['shN']['codebook'], np.float32))


@pytest.mark.parametrize('mode', ['', 'ST_ND_SORT'])
@pytest.mark.parametrize('n,d,k,tiny', [(30_000, 9, 256, 0.002), (40_000, 9, 8, 0.002), (20_000, 45, 1024, 0.0005)])
def test_kmeans_nd_uncertified_sums_vs_oracle(ctx, n, d, k, tiny, mode, monkeypatch):
    """N-D k-means whose cluster sums fail the exactness certificate in some dimensions (tiny
    members): the fused fix-up's partials are discarded for those clusters and their members
    are summed in point order (k_nd_seq); with K = 8 the flagged clusters hold more members
    than that kernel takes and the iteration falls back to the member sort.  ST_ND_SORT: the
    member-sort update every iteration."""
    if mode:
        monkeypatch.setenv(mode, '1')
    rng = np.random.default_rng(n + k)
    cols = [rng.normal(0, 0.1, n).astype(np.float32) for _ in range(d)]
    for c in cols:
        m = rng.random(n) < tiny
        c[m] *= np.float32(1e-9)
    draws = oracle.mulberry32(n + k + 1, 4 * k * 4 + 64)
    cent, labels, used = ctx.kmeans(cols, k, 3, draws)
    rc, ocent, olabels, oused = oracle.kmeans(cols, k, 3, draws)
    assert rc == 0 and used == oused
    same_bits(labels, olabels)
    same_bits(cent, ocent)


def heavy_tailed(rng, n, d, scale=0.1):
    """Student-t (nu = 3) coordinates through a fixed mixing matrix: heavy-tailed, correlated SH
    rows like trained scenes carry (outlying rows become outlying centroids)"""
    m = np.eye(d) + 0.5 * np.random.default_rng(3).normal(0, 1, (d, d)) / np.sqrt(d)
    t = rng.normal(0, 1, (n, d)) / np.sqrt((rng.normal(0, 1, (n, 3)) ** 2).sum(1, keepdims=True) / 3)
    return [np.ascontiguousarray(c) for c in (t @ m.T * scale).astype(np.float32).T]


@pytest.mark.parametrize('n,d,k,iters,dist', [(20_000, 45, 1024, 2, 'gauss'), (30_000, 9, 2048, 2, 'gauss'),
                                              (60_000, 1, 256, 4, 'gauss'), (20_000, 45, 1024, 3, 't3'),
                                              # row widths the SH palettes share (12, 48) at other d:
                                              # the fused fix-up is for d = 9 / 24 / 45 only
                                              (20_000, 12, 1024, 2, 'gauss'), (20_000, 48, 1024, 2, 'gauss'),
                                              (20_000, 10, 1024, 2, 'gauss'), (20_000, 22, 1024, 2, 'gauss')])
def test_kmeans_vs_oracle(ctx, n, d, k, iters, dist):
    rng = np.random.default_rng(n + d)
    cols = ([rng.normal(0, 0.1, n).astype(np.float32) for _ in range(d)] if dist == 'gauss'
            else heavy_tailed(rng, n, d))
    draws = oracle.mulberry32(n + k, 4 * k * (iters + 1) + 64)
    cent, labels, used = ctx.kmeans(cols, k, iters, draws)
    rc, ocent, olabels, oused = oracle.kmeans(cols, k, iters, draws)
    assert rc == 0 and used == oused
    same_bits(labels, olabels)
    same_bits(cent, ocent)
    if d > 1:  # how the assigns decided the points (st_ctx_last_kmeans_stats), summed over iterations
        st = ctx.kmeans_stats()
        assert st['assigns'] == iters and st['points'] == n * iters
        assert st['ambiguous'] >= st['overflow'] >= st['walked_overflow'] >= 0
        assert st['pairs'] + st['ambiguous'] <= st['points']


@pytest.mark.parametrize('n,d,k,iters,dist,split,chunk', [(20_000, 45, 1024, 3, 'gauss', 4, 16),
                                                         (20_000, 45, 1024, 3, 't3', 1, 1),
                                                         (30_000, 24, 2048, 2, 'gauss', 8, 5),
                                                         (30_000, 9, 2048, 2, 't3', 2, 64)])
def test_kmeans_heavy_others_vs_oracle(ctx, monkeypatch, n, d, k, iters, dist, split, chunk):
    """clusters with many pair / ambiguous points (a cluster of all-zero rows on a near-tie: millions
    at 10M) are summed over the chip in chunks (k_heavy): ST_OTHERS_SPLIT /
    ST_OTHERS_CHUNK lower the threshold (8,192) and the chunk (4,096) so every such cluster here
    takes that path; labels, centroids and draws equal the reference's"""
    monkeypatch.setenv('ST_OTHERS_SPLIT', str(split))
    monkeypatch.setenv('ST_OTHERS_CHUNK', str(chunk))
    rng = np.random.default_rng(n + d + 7)
    cols = ([rng.normal(0, 0.1, n).astype(np.float32) for _ in range(d)] if dist == 'gauss'
            else heavy_tailed(rng, n, d))
    draws = oracle.mulberry32(n + k + 1, 4 * k * (iters + 1) + 64)
    cent, labels, used = ctx.kmeans(cols, k, iters, draws)
    rc, ocent, olabels, oused = oracle.kmeans(cols, k, iters, draws)
    assert rc == 0 and used == oused
    same_bits(labels, olabels)
    same_bits(cent, ocent)


K1_MODES = ['', 'ST_K1_SYNC', 'ST_K1_TILES', 'ST_K1_SORT', 'ST_K1_FF_MAX=0', 'ST_REPLAY_CAP=0',
            'ST_REPLAY_CAP=2']


def set_mode(monkeypatch, mode):
    if mode:
        name, _, val = mode.partition('=')
        monkeypatch.setenv(name, val or '1')


@pytest.mark.parametrize('mode', K1_MODES)
@pytest.mark.parametrize('tiny_frac', [0.0, 2e-5, 0.02])
def test_cluster1d_uncertified_sums_vs_oracle(ctx, tiny_frac, mode, monkeypatch, capfd):
    """1-D k-means whose cluster sums fail the exactness certificate: clusters straddling 0
    hold tiny members, so the sequential f64 sum rounds -- a few events (the replay) or many
    (the sequential fallback).  mode: the iteration queued without read-backs, the flagged
    clusters updated by the three-pass flagged update (default); the flagged count read back
    each iteration (ST_K1_SYNC), the flagged clusters' members gathered by the tile kernels (ST_K1_TILES),
    every iteration's member sort (ST_K1_SORT), the queued run abandoned at the first flagged
    cluster and rerun synchronised (ST_K1_FF_MAX=0), or the replay capped at 0 / 2 candidates so
    that the sequential chain takes over (ST_REPLAY_CAP; ST_DEBUG's counts show that it did)."""
    set_mode(monkeypatch, mode)
    capped = mode.startswith('ST_REPLAY_CAP') and (tiny_frac > 0 if mode.endswith('=0') else tiny_frac >= 0.02)
    if capped:
        monkeypatch.setenv('ST_DEBUG', '1')
        capfd.readouterr()
    rng = np.random.default_rng(77)
    n = 300_000
    cols = [rng.normal(0, 1, n).astype(np.float32) for _ in range(3)]
    for c in cols:
        tiny = rng.random(n) < tiny_frac
        c[tiny] *= np.float32(1e-9)
    draws = oracle.mulberry32(5, 1 << 14)
    cent, labels, used = ctx.cluster1d(cols, 4, draws)
    if capped:  # the capped replay sent clusters down the sequential chain
        import re
        err = capfd.readouterr().err
        seq = sum(int(x) for x in re.findall(r'sequential-fallback=(\d+)', err)) + len(re.findall(r',seq=1', err))
        assert seq > 0, err[-2000:]
    rc, ocent, olabels, oused = oracle.cluster1d(cols, 4, draws)
    assert rc == 0 and used == oused
    assert np.array_equal(cent.view(np.uint32), ocent.view(np.uint32))
    assert np.array_equal(labels, olabels)


@pytest.mark.parametrize('mode', ['', 'ST_K1_SYNC'])
@pytest.mark.parametrize('tiny_frac', [0.0, 2e-5, 0.02])
def test_cluster1d_uncertified_many_tiles_vs_oracle(ctx, tiny_frac, mode, monkeypatch):
    """The sort-free 1-D iteration at a size where every accumulating workgroup takes several
    4,096-point tiles and the flagged clusters' members are gathered from hundreds of tiles
    (1.5M points per column, 4.5M values, 4,395 look-back chunks); 0.02 drives sums with many
    rounding events into the sequential chain."""
    set_mode(monkeypatch, mode)
    rng = np.random.default_rng(78)
    n = 1_500_000
    cols = [rng.normal(0, 1, n).astype(np.float32) for _ in range(3)]
    for c in cols:
        tiny = rng.random(n) < tiny_frac
        c[tiny] *= np.float32(1e-9)
    draws = oracle.mulberry32(6, 1 << 14)
    cent, labels, used = ctx.cluster1d(cols, 3, draws)
    rc, ocent, olabels, oused = oracle.cluster1d(cols, 3, draws)
    assert rc == 0 and used == oused
    assert np.array_equal(cent.view(np.uint32), ocent.view(np.uint32))
    assert np.array_equal(labels, olabels)


@pytest.mark.parametrize('mode', ['', 'ST_K1_SYNC'])
def test_cluster1d_sorted_columns_vs_oracle(ctx, mode, monkeypatch):
    """Sorted columns (ascending, descending, ascending): every cluster's members are one
    contiguous run of points, so the flagged cluster straddling 0 fills a few hundred chunks
    and every other chunk of the one-pass update's look-back holds none of its members."""
    set_mode(monkeypatch, mode)
    rng = np.random.default_rng(79)
    n = 2_000_000
    cols = []
    for j in range(3):
        c = rng.normal(0, 1, n).astype(np.float32)
        tiny = rng.random(n) < 2e-4
        c[tiny] *= np.float32(1e-9)
        c.sort()
        cols.append(np.ascontiguousarray(c[::-1]) if j == 1 else c)
    draws = oracle.mulberry32(7, 1 << 14)
    cent, labels, used = ctx.cluster1d(cols, 3, draws)
    rc, ocent, olabels, oused = oracle.cluster1d(cols, 3, draws)
    assert rc == 0 and used == oused
    assert np.array_equal(cent.view(np.uint32), ocent.view(np.uint32))
    assert np.array_equal(labels, olabels)


@pytest.mark.parametrize('n,k,dup,dist', [(40_000, 65536, 0.0, 'gauss'), (30_000, 65536, 0.3, 'gauss'),
                                          (20_000, 131072, 0.0, 'gauss'), (40_000, 65536, 0.0, 't3'),
                                          (30_000, 65536, 0.3, 't3')])
def test_nd_assign_full_palette_argmin(ctx, n, k, dup, dist):
    """One assign pass at the SOG palette size (K = 65,536 / 131,072, D = 45) against a
    brute-force f64 distance computed on the device in the reference's own order
    (kd-tree.ts:26-35: l += (c - p)^2 sequentially over the dimensions, each op rounded
    like a JS number): every label must reach the exact minimum.  dup > 0 makes a share of
    the points copies of centroids (distance 0 and near-ties between neighbouring rows).
    t3: heavy-tailed correlated points, the centroids data rows of the same distribution
    (outlying centroids: the decision window must not widen for every point)."""
    import torch
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev)
    g.manual_seed(n + k)
    d = 45
    if dist == 'gauss':
        cen = (torch.randn(d, k, generator=g, device=dev) * 0.05).contiguous()
        pts = torch.randn(d, n, generator=g, device=dev) * 0.1
    else:
        rows = heavy_tailed(np.random.default_rng(n + k), n + k, d)
        cen = torch.from_numpy(np.stack([r[:k] for r in rows])).to(dev).contiguous()
        pts = torch.from_numpy(np.stack([r[k:] for r in rows])).to(dev)
    if dup:
        m = int(n * dup)
        pick = torch.randint(0, k, (m,), generator=g, device=dev)
        pts[:, :m] = cen[:, pick] + torch.randn(d, m, generator=g, device=dev) * 1e-4
    cols = [pts[j].contiguous() for j in range(d)]
    labels = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.dev_kmeans_prepare(cols)
    ctx.dev_kmeans_assign(cols, k, cen, labels)
    ctx.synchronize()
    torch.cuda.synchronize()
    lab = labels.long()
    cd = cen.double()
    bad = 0
    for s in range(0, n, 512):
        e = min(n, s + 512)
        pd = torch.stack([c[s:e] for c in cols]).double()
        dist = torch.zeros(e - s, k, dtype=torch.float64, device=dev)
        for j in range(d):
            v = cd[j][None, :] - pd[j][:, None]
            dist += v * v
        mn = dist.min(1).values
        got = dist.gather(1, lab[s:e, None]).squeeze(1)
        bad += int((got != mn).sum().item())
    assert bad == 0, f'{bad} labels miss the exact f64 minimum'


@pytest.mark.parametrize('levels', [7, 50, 300])
def test_cluster1d_ties_and_duplicates_vs_oracle(ctx, levels):
    """1-D k-means on integer-valued columns: many points lie exactly midway between two
    centroids (equal rounded distances), empty clusters are re-seeded onto existing values
    (duplicate centroids), so the assign must fall back to the KdTree walk's tie-break."""
    rng = np.random.default_rng(levels)
    n = 40_000
    cols = [rng.integers(-levels, levels, n).astype(np.float32) for _ in range(3)]
    cols[1] *= np.float32(0.5)
    draws = oracle.mulberry32(levels, 1 << 15)
    cent, labels, used = ctx.cluster1d(cols, 5, draws)
    rc, ocent, olabels, oused = oracle.cluster1d(cols, 5, draws)
    assert rc == 0 and used == oused
    assert np.array_equal(cent.view(np.uint32), ocent.view(np.uint32))
    assert np.array_equal(labels, olabels)


def test_kmeans_bench_size_first_assign_and_update(ctx):
    """The bench's SH k-means at full size (10M x 45, K = 65,536; SURVEY 8d data): one
    iteration, checked through size-independent properties.  The init rows are the first K
    distinct floor(draw * n) (k-means.ts:8-20); every sampled label must reach the exact f64
    minimum over those K centroids (kd-tree.ts:26-35 order), and sampled centroids must equal
    the sequential f64 mean of their members (calcAverage, k-means.ts:41-63)."""
    import torch
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1002)
    n, d, k = 10_000_000, 45, 65536
    cols = [torch.randn(n, generator=g, device=dev) * 0.1 for _ in range(d)]
    draws = np.random.default_rng(42).random(4 * k)
    cen = torch.empty(d * k, device=dev)
    labels = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # the context runs on its own stream
    used = ctx.dev_kmeans(cols, k, 1, draws, cen, labels)
    ctx.synchronize()
    torch.cuda.synchronize()
    # the init rows, as the reference draws them
    rows, seen, cur = [], set(), 0
    while len(rows) < k:
        r = int(np.floor(draws[cur] * n))
        cur += 1
        if r not in seen:
            seen.add(r)
            rows.append(r)
    assert used >= cur  # the init consumed exactly cur draws; re-seeds may add more
    ridx = torch.tensor(rows, device=dev)
    c0 = torch.stack([c[ridx] for c in cols]).double()  # (d, k) init centroids
    sample = torch.randint(0, n, (4096,), generator=g, device=dev)
    lab = labels[sample].long()
    bad = 0
    for s in range(0, sample.numel(), 512):
        idx = sample[s:s + 512]
        dist = torch.zeros(idx.numel(), k, dtype=torch.float64, device=dev)
        for j in range(d):
            v = c0[j][None, :] - cols[j][idx].double()[:, None]
            dist += v * v
        got = dist.gather(1, lab[s:s + 512, None]).squeeze(1)
        bad += int((got != dist.min(1).values).sum().item())
    assert bad == 0, f'{bad} of 4096 sampled labels miss the exact f64 minimum'
    # the update: sequential f64 means of a few clusters' members (ascending point order)
    lab_all = labels.long()
    cen = cen.view(d, k)
    for cl in torch.randint(0, k, (6,), generator=g, device=dev).tolist():
        members = torch.nonzero(lab_all == cl).flatten()
        if members.numel() == 0:
            continue  # re-seeded
        vals = torch.stack([c[members] for c in cols]).cpu().numpy().astype(np.float64)
        for j in range(d):
            acc = 0.0
            for v in vals[j]:
                acc += float(v)
            want = np.float32(acc / members.numel())
            assert np.float32(cen[j, cl].item()).view(np.uint32) == want.view(np.uint32), (cl, j)


def test_config3_chain_vs_oracle(ctx):
    """BASELINE config 3 as one device chain (-r 0,45,0 -> filterNaN -> permuteRows ->
    generateOrdering -> writeCompressedPly's chunk pack), inputs resident in HBM, 1M SH-3 splats
    with 0.1% of rows holding NaN/Inf; every output array bit-exact against the oracle chain
    (process.ts:64-145, data-table.ts:135-149, ordering.ts:4-110, write-compressed-ply.ts:56-109)"""
    import torch
    n = 1_000_000
    rng = np.random.default_rng(1003)
    names = ['x', 'y', 'z', 'nx', 'ny', 'nz', 'f_dc_0', 'f_dc_1', 'f_dc_2'] + [f'f_rest_{i}' for i in range(45)] + \
        ['opacity', 'scale_0', 'scale_1', 'scale_2', 'rot_0', 'rot_1', 'rot_2', 'rot_3']
    cols = {k: rng.normal(0, 1, n).astype(np.float32) for k in names}
    cols['x'] *= 10
    cube = rng.random(n) < 0.05  # equal-key Morton runs > 256
    cols['x'][cube] = 1 + rng.random(cube.sum()).astype(np.float32) * 1e-3
    bad = rng.choice(n, n // 1000, replace=False)
    for j, r in enumerate(bad):
        cols[names[j % len(names)]][r] = [np.nan, np.inf, -np.inf][j % 3]
    ref = {k: v.copy() for k, v in cols.items()}
    d = {k: torch.from_numpy(v).cuda() for k, v in cols.items()}
    # device chain
    ctx.dev_transform(d, sh.action_params('rotate', (0, 45, 0)))
    idx = torch.empty(n, dtype=torch.int32, device='cuda')
    m = ctx.dev_filter_finite(d, idx)
    kept = {k: torch.empty(m, device='cuda') for k in names}
    ctx.dev_permute_rows(d, idx, m, kept)
    order = torch.arange(m, dtype=torch.int32, device='cuda')
    ctx.dev_morton_order(kept['x'], kept['y'], kept['z'], order)
    chunk = torch.empty((m + 255) // 256 * 18, device='cuda')
    vertex = torch.empty(m * 4, dtype=torch.int32, device='cuda')
    shb = torch.empty(m * 45, dtype=torch.uint8, device='cuda')
    ctx.dev_pack_compressed({k: v for k, v in kept.items() if not k.startswith('n')}, order, chunk, vertex, shb)
    ctx.synchronize()
    # oracle chain
    oracle.transform(ref, oracle.transform_params(euler=(0, 45, 0)), 15)
    oidx = oracle.filter_finite([ref[k] for k in names])
    assert m == len(oidx)
    same_bits(idx[:m].cpu().numpy().view(np.uint32), oidx)
    oref = {k: v[oidx] for k, v in ref.items()}
    for k in names:
        same_bits(kept[k].cpu().numpy(), oref[k])
    oorder = oracle.morton_order(oref['x'], oref['y'], oref['z'])
    same_bits(order.cpu().numpy().view(np.uint32), oorder)
    want = oracle.pack_compressed(oref, oorder, 45)
    for got, w in zip((chunk, vertex, shb), want):
        same_bits(got.cpu().numpy().view(w.dtype), w)
