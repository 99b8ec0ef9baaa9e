"""Edge cases of the HIP path against the pinned CPU restatement (oracle/): degenerate and
non-finite inputs, ragged sizes around the 256-splat chunk and the 1,024-row tile, and
the whole writeSog pipeline for every SH band.  Integer / byte / index outputs bit-exact,
floats bit-exact (NaN as NaN)."""
import numpy as np
import pytest

import oracle
import splat_hip as sh
from test_oracle_golden import same_bits

pytestmark = pytest.mark.gpu

MEMBERS = ['x', 'y', 'z', 'scale_0', 'scale_1', 'scale_2', 'f_dc_0', 'f_dc_1', 'f_dc_2', 'opacity',
           'rot_0', 'rot_1', 'rot_2', 'rot_3']


@pytest.fixture(scope='module')
def ctx():
    import torch  # noqa: F401  (torch's HIP runtime first: see splat_hip.Context)
    return sh.Context(0)


def _table(n, C, seed, spice=False):
    rng = np.random.default_rng(seed)
    cols = {k: rng.normal(0, 1, n).astype(np.float32) for k in MEMBERS}
    for i in range(3):
        cols[f'scale_{i}'] = (rng.random(n) * 5 - 7).astype(np.float32)
    for i in range(3 * C):
        cols[f'f_rest_{i}'] = (rng.normal(0, 0.1, n)).astype(np.float32)
    if spice and n:
        # +-Inf / NaN members, scales past the +-20 clamp, zero and negative-dominant quaternions,
        # SH bytes past both saturation ends, -0
        k = max(1, n // 50)
        idx = rng.choice(n, size=min(n, 6 * k), replace=False)
        a, b, c_, d, e, f = np.array_split(idx, 6)
        cols['x'][a] = np.inf
        cols['y'][b] = -np.inf
        cols['z'][c_] = np.nan
        cols['scale_0'][d] = 100.0
        cols['scale_1'][d] = -100.0
        for i in range(4):
            cols[f'rot_{i}'][e] = 0.0
        cols['rot_2'][f] = -5.0
        cols['opacity'][a] = np.nan
        cols['f_dc_1'][b] = -0.0
        if C:
            cols['f_rest_0'][c_] = 50.0
            cols['f_rest_1'][d] = -50.0
            cols['f_rest_2'][e] = np.nan
    return cols


@pytest.mark.parametrize('n', [0, 1, 2, 3, 255, 256, 257, 1023, 1025])
def test_morton_ragged_vs_oracle(ctx, n):
    rng = np.random.default_rng(n)
    x, y, z = (rng.normal(0, 5, n).astype(np.float32) for _ in range(3))
    same_bits(ctx.morton_order(x, y, z), oracle.morton_order(x, y, z))


@pytest.mark.parametrize('case', ['all_equal', 'nan_coords', 'inf_extent', 'one_axis_flat', 'big_equal_run',
                                  'neg_zero', 'lattice', 'blobs', 'blobs_flat', 'clumps', 'clumps_dup'])
@pytest.mark.parametrize('n', [5000, 70001, 1_000_003])
def test_morton_degenerate_vs_oracle(ctx, case, n):
    """ordering.ts:53-65: zero-length extents, non-finite extents (ordering skipped), NaN
    coordinates (key 0), equal-key runs longer than 256 (recursion with their own extents)."""
    rng = np.random.default_rng(7)
    x, y, z = (rng.normal(0, 5, n).astype(np.float32) for _ in range(3))
    if case == 'all_equal':
        x[:], y[:], z[:] = 1.5, -2.0, 3.25
    elif case == 'nan_coords':
        x[rng.random(n) < 0.1] = np.nan
        z[rng.random(n) < 0.05] = np.nan
    elif case == 'inf_extent':
        y[17] = np.inf
    elif case == 'one_axis_flat':
        z[:] = 4.0
    elif case == 'big_equal_run':
        m = rng.random(n) < 0.4
        for a in (x, y, z):
            a[m] = 0.5
        x[m] += (rng.integers(0, 3, m.sum()) * 1e-6).astype(np.float32)
    elif case == 'neg_zero':
        x[::2] = -0.0
        x[1::2] = 0.0
    elif case == 'lattice':  # many exactly equal points: runs whose own extents are all zero
        for a in (x, y, z):
            a[:] = np.round(a * 0.8) / 0.8
    elif case in ('blobs', 'blobs_flat'):  # tight blobs: several recursion levels, many segments
        m = rng.random(n) < 0.6
        centre = rng.integers(0, 300, n).astype(np.float32)
        for a in (x, y, z):
            a[m] = (centre[m] * 0.03 + a[m] * 1e-5).astype(np.float32)
        if case == 'blobs_flat':  # some blobs flat on one axis, NaN members in others
            z[m & (centre < 100)] = 1.0
            x[m & (centre > 250) & (rng.random(n) < 0.01)] = np.nan
    elif case in ('clumps', 'clumps_dup'):
        # ~600-member clumps: deeper-level segments small enough for the one-workgroup sort;
        # with duplicates, runs inside them recurse once more (and stop: equal coordinates)
        m = rng.random(n) < 0.8
        cid = rng.integers(0, max(1, int(n * 0.8) // 600), n)
        cx, cy, cz = (rng.normal(0, 5, cid.max() + 1).astype(np.float32) for _ in range(3))
        jit = 1e-5 if case == 'clumps' else 0.0
        for a, cc in ((x, cx), (y, cy), (z, cz)):
            a[m] = (cc[cid[m]] + a[m] * jit).astype(np.float32)
        if case == 'clumps_dup':
            half = m & (rng.random(n) < 0.5)
            x[half] += np.float32(1e-4)
    same_bits(ctx.morton_order(x, y, z), oracle.morton_order(x, y, z))


@pytest.mark.parametrize('n', [2048, 2049, 4095, 65535, 65536, 65537, 4096 * 25 + 1, 4096 * 37, 1_500_007])
def test_morton_onesweep_sizes_vs_oracle(ctx, n):
    """Level-0 sorts of whole and ragged 4,096-key tiles, and a caller-supplied permutation of
    the indices (the values carried through the passes are idx[j]: ordering.ts:4-20 sorts the
    indices it is given)."""
    rng = np.random.default_rng(n)
    x, y, z = (rng.normal(0, 10, n).astype(np.float32) for _ in range(3))
    m = rng.random(n) < 0.05
    for a in (x, y, z):
        a[m] = (2 + rng.random(m.sum()) * 1e-3).astype(np.float32)
    perm = rng.permutation(n).astype(np.uint32)
    same_bits(ctx.morton_order(x, y, z, perm), oracle.morton_order(x, y, z, perm))
    same_bits(ctx.morton_order(x, y, z), oracle.morton_order(x, y, z))


@pytest.mark.parametrize('n,m', [(3000, 2000), (100_000, 70_001), (50_000, 200_003)])
def test_morton_index_subsets_vs_oracle(ctx, n, m):
    """generateOrdering over an index list that is not a permutation (a subset with repeated
    rows, shorter or longer than the table): extents, keys and the stable order all follow
    the given indices (ordering.ts:4-20); level 0 sorts idx in place as its own values."""
    import torch
    dev = torch.device('cuda', 0)
    rng = np.random.default_rng(m)
    x, y, z = (rng.normal(0, 3, n).astype(np.float32) for _ in range(3))
    x[rng.random(n) < 0.01] = np.nan
    idx = rng.integers(0, n, m).astype(np.uint32)
    tx, ty, tz = (torch.from_numpy(a).to(dev) for a in (x, y, z))
    tidx = torch.from_numpy(idx.view(np.int32).copy()).to(dev)
    ctx.dev_morton_order(tx, ty, tz, tidx)
    ctx.synchronize()
    same_bits(tidx.cpu().numpy().view(np.uint32), oracle.morton_order(x, y, z, idx))


@pytest.mark.parametrize('n,C', [(1, 0), (255, 3), (256, 15), (257, 8), (1000, 15), (4097, 3)])
def test_pack_compressed_edges_vs_oracle(ctx, n, C):
    """compressed-chunk.ts:44-180: NaN-propagating chunk min/max, the +-20 scale clamp, zero
    quaternions, the padded last chunk (write-compressed-ply.ts:90-93), SH byte saturation."""
    cols = _table(n, C, 100 + n, spice=True)
    order = np.random.default_rng(n).permutation(n).astype(np.uint32)
    got = ctx.pack_compressed(cols, order, 3 * C)
    want = oracle.pack_compressed(cols, order, 3 * C)
    for g, w in zip(got, want):
        same_bits(np.asarray(g).view(np.uint8), np.asarray(w).view(np.uint8))


@pytest.mark.parametrize('n,C,kind', [(70_001, 15, 'perm'), (70_001, 15, 'repeats'), (1000, 8, 'repeats'),
                                      (300_000, 3, 'perm')])
def test_pack_compressed_orders_vs_oracle(ctx, n, C, kind):
    """Chunk packing over a permutation and over an index list that repeats rows (the
    reference's chunk loop, write-compressed-ply.ts:56-109, accepts any list of row indices)."""
    cols = _table(n, C, 300 + n + C, spice=True)
    rng = np.random.default_rng(n + C)
    order = rng.permutation(n).astype(np.uint32)
    if kind == 'repeats':
        order[rng.integers(0, n, max(1, n // 100))] = order[0]
    got = ctx.pack_compressed(cols, order, 3 * C)
    want = oracle.pack_compressed(cols, order, 3 * C)
    for g, w in zip(got, want):
        same_bits(np.asarray(g).view(np.uint8), np.asarray(w).view(np.uint8))


@pytest.mark.parametrize('kind', ['none', 'all', 'sparse', 'last_row', 'inf_only'])
def test_filter_finite_edges_vs_oracle(ctx, kind):
    n = 3001
    cols = _table(n, 3, 5)
    names = list(cols)
    rng = np.random.default_rng(9)
    if kind == 'all':
        for r in range(n):
            cols[names[r % len(names)]][r] = np.nan
    elif kind == 'sparse':
        for r in rng.choice(n, 40, replace=False):
            cols[names[rng.integers(len(names))]][r] = np.nan if r % 2 else -np.inf
    elif kind == 'last_row':
        cols['rot_3'][n - 1] = np.inf
    elif kind == 'inf_only':
        cols['x'][::7] = np.inf
    got = ctx.filter_finite(cols)
    want = oracle.filter_finite([cols[k] for k in names])
    same_bits(np.asarray(got, np.uint32), np.asarray(want, np.uint32))


@pytest.mark.parametrize('action', [('scale', 0.0), ('scale', 1e30), ('translate', (1e38, -1e38, 0.0)),
                                    ('rotate', (90, 0, 180)), ('rotate', (0.0, 0.0, 0.0))])
def test_transform_extremes_vs_oracle(ctx, action):
    """transform.ts:12-65 with a zero / huge scale (log(0) = -inf, overflow), huge
    translations and exact-angle rotations over NaN / Inf / -0 inputs."""
    kind, value = action
    cols = _table(2000, 15, 11, spice=True)
    ref = {k: v.copy() for k, v in cols.items()}
    if kind == 'scale':
        op = oracle.transform_params(s=float(value))
    elif kind == 'translate':
        op = oracle.transform_params(t=value)
    else:
        op = oracle.transform_params(euler=value)
    oracle.transform(ref, op, 15)
    ctx.transform(cols, sh.action_params(kind, value))
    for k in cols:
        same_bits(cols[k], ref[k])


@pytest.mark.parametrize('C', [0, 3, 8, 15])
def test_sog_all_bands_vs_oracle(ctx, C):
    """writeSog (write-sog.ts:110-370) end to end for every SH band: textures, meta and the
    Math.random draws consumed (paletteSize 4,096 at n = 5,000)."""
    n = 5000
    cols = _table(n, C, 40 + C)
    draws = oracle.mulberry32(C + 1, 1 << 15)
    tex, meta, used = ctx.sog(cols, 3, draws)
    rc, otex, ometa, oused = oracle.sog(cols, C, 3, draws)
    assert rc == 0 and used == oused
    assert set(tex) == set(otex)
    for k in tex:
        same_bits(tex[k], otex[k])
    for f in ('width', 'height', 'sh_bands', 'palette_size', 'shn_width', 'shn_height'):
        assert getattr(meta, f) == getattr(ometa, f), f
    for f in ('means_min', 'means_max', 'scales_codebook', 'sh0_codebook', 'shn_codebook'):
        same_bits(np.array(getattr(meta, f)[:]), np.array(getattr(ometa, f)[:]))


@pytest.mark.parametrize('n,d,k,zero_frac,protos,mode', [(20_000, 45, 1024, 0.05, 0, ''), (20_000, 45, 1024, 0.3, 0, ''),
                                                         (30_000, 24, 2048, 0.5, 0, ''), (8_000, 9, 256, 0.02, 0, ''),
                                                         (30_000, 45, 1024, 0.4, 40, ''),
                                                         (20_000, 45, 1024, 0.3, 0, 'signed_zeros'),
                                                         (20_000, 45, 4096, 0.3, 3, 'signed_zeros'),
                                                         (20_000, 45, 1024, 0.3, 0, 'no_groups'),
                                                         (30_000, 45, 1024, 0.4, 40, 'no_groups')])
def test_kmeans_duplicated_rows_vs_oracle(ctx, monkeypatch, n, d, k, zero_frac, protos, mode):
    """Many exactly duplicated points (all-zero rows): the init draws pick several of them, so
    several centroids coincide and every point whose nearest row is theirs is equidistant from
    all of them.  The assign sweeps one representative per distinct centroid row and settles such
    a point with a descent of the reference's tree (the member KdTree.findNearest meets first,
    kd-tree.ts:39-68); exact ties between distinct rows go to the walk.  protos > 0: the
    duplicated rows are copies of that many random rows instead of zeros; signed_zeros: the
    duplicated rows' zeros carry random signs (-0 and +0 are one coordinate to the distance and
    the tree); no_groups: every centroid swept (ST_NO_CEN_GROUPS), the ties walked.  Labels,
    centroids and draws match the reference."""
    rng = np.random.default_rng(n + d + k)
    cols = [rng.normal(0, 0.1, n).astype(np.float32) for _ in range(d)]
    z = rng.random(n) < zero_frac
    which = rng.integers(0, max(protos, 1), n)
    for c in cols:
        if mode == 'signed_zeros':
            c[:protos][rng.random(protos) < 0.3] = 0.0
        c[z] = c[:protos][which[z]] if protos else 0.0
        if mode == 'signed_zeros':
            c[z & (c == 0) & (rng.random(n) < 0.5)] = np.float32(-0.0)
    if mode == 'no_groups':
        monkeypatch.setenv('ST_NO_CEN_GROUPS', '1')
    draws = oracle.mulberry32(n + k, 8 * k * 4 + 64)
    cent, labels, used = ctx.kmeans(cols, k, 3, draws)
    rc, ocent, olabels, oused = oracle.kmeans(cols, k, 3, draws)
    assert rc == 0 and used == oused
    same_bits(labels, olabels)
    same_bits(cent, ocent)


@pytest.mark.parametrize('big,tiny,zero', [(24, 0.0, 0.0), (24, 0.02, 0.0), (1, 0.0, 0.0), (24, 0.02, 0.3),
                                           (1, 0.02, 0.3), (24, 0.02, -0.3)])
def test_kmeans_split_cluster_sums_vs_oracle(ctx, monkeypatch, big, tiny, zero):
    """calcAverage (k-means.ts:41-63) for clusters above the split threshold (ST_SUMND_BIG lowers
    the default 16,384): slices summed in parallel under the exactness certificate, and the
    sequential chain where tiny members break the certificate -- which walks the members' rows
    that are not all zero (adding +-0 leaves the running sum as it is): zero = the fraction of
    all-zero rows (negative: their zeros are -0.0 and +0.0 at random).  big = 1 splits every
    cluster with more than one member."""
    n, d, k = 6000, 9, 64
    rng = np.random.default_rng(big + int(tiny * 100) + int(abs(zero) * 1000) + (7 if zero < 0 else 0))
    cols = [rng.normal(0, 1, n).astype(np.float32) for _ in range(d)]
    zr = rng.random(n) < abs(zero)
    for c in cols:
        t = rng.random(n) < tiny
        c[t] *= np.float32(1e-12)
        c[zr] = 0.0
        if zero < 0:
            c[zr & (rng.random(n) < 0.5)] = np.float32(-0.0)
    draws = oracle.mulberry32(9, 1 << 12)
    monkeypatch.setenv('ST_SUMND_BIG', str(big))
    cent, labels, used = ctx.kmeans(cols, k, 3, draws)
    monkeypatch.delenv('ST_SUMND_BIG')
    rc, ocent, olabels, oused = oracle.kmeans(cols, k, 3, draws)
    assert rc == 0 and used == oused
    same_bits(labels, olabels)
    same_bits(cent, ocent)


@pytest.mark.parametrize('n,C', [(1, 3), (2, 0), (17, 8), (85, 0), (86, 0), (300, 15), (1023, 3), (1025, 15),
                                 (2049, 8)])
def test_sog_small_tables_vs_oracle(ctx, n, C):
    """writeSog on tables smaller than the default palette (write-sog.ts:310 paletteSize from n:
    256 at n = 300, 512 at n = 1,023 ...), textures barely larger than the table.  Below 86
    splats the scales' cluster1d has fewer than 256 values: the reference's kmeans returns a
    plain Array there (k-means.ts:139-144) and the `.subarray` of write-sog.ts throws, so both
    the product and the oracle report an error."""
    cols = _table(n, C, 500 + n)
    draws = oracle.mulberry32(n, 1 << 14)
    rc, otex, ometa, oused = oracle.sog(cols, C, 3, draws)
    if 3 * n < 256:
        assert rc != 0
        with pytest.raises(sh.StError):
            ctx.sog(cols, 3, draws)
        return
    tex, meta, used = ctx.sog(cols, 3, draws)
    assert rc == 0 and used == oused
    assert set(tex) == set(otex)
    for k in tex:
        same_bits(tex[k], otex[k])
    for f in ('width', 'height', 'sh_bands', 'palette_size', 'shn_width', 'shn_height'):
        assert getattr(meta, f) == getattr(ometa, f), f
    for f in ('means_min', 'means_max', 'scales_codebook', 'sh0_codebook', 'shn_codebook'):
        same_bits(np.array(getattr(meta, f)[:]), np.array(getattr(ometa, f)[:]))


@pytest.mark.parametrize('kind', ['clumps', 'lattice'])
def test_sog_clumped_positions_vs_oracle(ctx, kind):
    """writeSog over positions whose Morton order recurses (ordering.ts:90-104): clumps of
    ~600 splats at one point each (segments sorted inside one workgroup, their runs stopping on
    all-equal extents), or a coarse lattice (runs whose extents are all zero) -- the means
    textures place every row at its Morton position."""
    n, C = 6000, 3
    cols = _table(n, C, 91)
    rng = np.random.default_rng(3)
    if kind == 'clumps':
        cid = rng.integers(0, 8, n)
        for i, a in enumerate(('x', 'y', 'z')):
            cen = rng.normal(0, 4, 8).astype(np.float32)
            cols[a] = (cen[cid] + (rng.random(n) < 0.5) * np.float32(1e-3) * (i == 0)).astype(np.float32)
    else:
        for a in ('x', 'y', 'z'):
            cols[a] = (np.round(cols[a] * 0.5) / 0.5).astype(np.float32)
    draws = oracle.mulberry32(11, 1 << 15)
    tex, meta, used = ctx.sog(cols, 3, draws)
    rc, otex, ometa, oused = oracle.sog(cols, C, 3, draws)
    assert rc == 0 and used == oused
    for k in tex:
        same_bits(tex[k], otex[k])
    same_bits(np.array(meta.means_min[:]), np.array(ometa.means_min[:]))
    same_bits(np.array(meta.means_max[:]), np.array(ometa.means_max[:]))


@pytest.mark.parametrize('who', ['scales', 'colours', 'both', 'neither'])
def test_sog_reseeding_cluster1d_vs_oracle(ctx, who):
    """The colours' cluster1d runs beside the scales' on a side context from draw 0 and is kept
    only when the scales' k-means took no draw (re-seeds of empty clusters, k-means.ts:174-178);
    otherwise it reruns after them.  Columns with a far outlier leave most linspace centroids
    (k-means.ts:23-39) without members, so that cluster1d consumes draws."""
    n, C = 5000, 3
    cols = _table(n, C, 77)
    rng = np.random.default_rng(5)
    outlier = {'scales': ['scale_0', 'scale_1', 'scale_2'], 'colours': ['f_dc_0', 'f_dc_1', 'f_dc_2'],
               'both': ['scale_0', 'f_dc_2'], 'neither': []}[who]
    for k in outlier:
        cols[k] = (rng.integers(0, 4, n) * 0.25 - 5).astype(np.float32)
        cols[k][17] = 40.0
    draws = oracle.mulberry32(123, 1 << 15)
    s_cols = [cols[f'scale_{i}'] for i in range(3)]
    _, _, _, s_used = oracle.cluster1d(s_cols, 3, draws)
    assert (s_used > 0) == (who in ('scales', 'both'))
    tex, meta, used = ctx.sog(cols, 3, draws)
    rc, otex, ometa, oused = oracle.sog(cols, C, 3, draws)
    assert rc == 0 and used == oused
    for k in tex:
        same_bits(tex[k], otex[k])
    for f in ('scales_codebook', 'sh0_codebook', 'shn_codebook'):
        same_bits(np.array(getattr(meta, f)[:]), np.array(getattr(ometa, f)[:]))


@pytest.mark.parametrize('case', ['n_eq_4k', 'repeats', 'host_env'])
def test_kmeans_device_init_vs_oracle(ctx, case, monkeypatch):
    """initializeCentroids (k-means.ts:8-20) on the device (n >= 4k): first occurrences of
    floor(draw * n) in draw order over a window of the draws.  'repeats' fills the window
    with a few rows so it holds fewer than k distinct ones (the call reruns with the host's
    loop); 'host_env' forces the host loop (ST_KM_HOST_INIT)."""
    k, d, iters = 1024, 9, 2
    n = 4 * k if case == 'n_eq_4k' else 20_000
    rng = np.random.default_rng(3)
    cols = [rng.normal(0, 0.1, n).astype(np.float32) for _ in range(d)]
    draws = oracle.mulberry32(99, 8 * k * (iters + 2))
    if case == 'repeats':
        draws[:k + k // 4 + 4000] = (rng.integers(0, 7, k + k // 4 + 4000) + 0.5) / n
    if case == 'host_env':
        monkeypatch.setenv('ST_KM_HOST_INIT', '1')
    cent, labels, used = ctx.kmeans(cols, k, iters, draws)
    rc, ocent, olabels, oused = oracle.kmeans(cols, k, iters, draws)
    assert rc == 0 and used == oused
    same_bits(labels, olabels)
    same_bits(cent, ocent)


def test_kmeans_draw_outside_unit_interval_fails(ctx):
    k, n = 256, 4096
    rng = np.random.default_rng(4)
    cols = [rng.normal(0, 1, n).astype(np.float32) for _ in range(3)]
    draws = rng.random(4 * k * 4)
    draws[10] = 1.0
    with pytest.raises(sh.StError):
        ctx.kmeans(cols, k, 2, draws)


@pytest.mark.parametrize('case', ['device', 'short_window', 'small_n'])
def test_step_api_init_rows_and_gather(ctx, case):
    """st_dev_kmeans_init_rows (the sharded k-means init): the reference's rejection loop
    (k-means.ts:8-20) over the global n -- on the device when n >= 4k, by the host when the
    draw window is short or n < 4k -- and st_dev_gather_rows' owned-row assembly."""
    import torch
    dev = torch.device('cuda', 0)
    k = 4096
    n = 3 * k if case == 'small_n' else 100_000
    rng = np.random.default_rng(21)
    draws = rng.random(8 * k)
    if case == 'short_window':
        draws[:k + k // 4 + 5000] = (rng.integers(0, 9, k + k // 4 + 5000) + 0.5) / n
    want, seen, cur = [], set(), 0
    while len(want) < k:
        r = int(np.floor(draws[cur] * n))
        cur += 1
        if r not in seen:
            seen.add(r)
            want.append(r)
    rows = torch.empty(k, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    used = ctx.dev_kmeans_init_rows(draws, n, k, rows)
    ctx.synchronize()
    assert used == cur
    assert rows.cpu().numpy().tolist() == want
    # owned-row gather: two shards of the table, assembled by an integer sum of the bit patterns
    d = 5
    cols = [torch.from_numpy(rng.normal(0, 1, n).astype(np.float32)).to(dev) for _ in range(d)]
    cols[0][int(want[0])] = -0.0
    cut = n // 3
    parts = []
    for lo, hi in ((0, cut), (cut, n)):
        out = torch.empty((d, k), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        ctx.dev_gather_rows([c[lo:hi].contiguous() for c in cols], lo, rows, out)
        ctx.synchronize()
        parts.append(out.view(torch.int32))
    got = (parts[0] + parts[1]).view(torch.float32).cpu().numpy()
    ref = np.stack([c.cpu().numpy()[want] for c in cols])
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize('swap', [False, True])
def test_assign_pair_ties_without_ambiguous_points(ctx, swap):
    """Exact ties found by the pair fix-up (two tile-halves) when no point is ambiguous: the
    KdTree walk (kd-tree.ts:39-68) must still decide them.  Points at (3,0,0) are exactly 1 from
    centroids (2,0,0) and (3,1,0), which sit in different halves of tile 0; every other centroid is
    far away, so no point needs the collect sweep."""
    import torch
    dev = torch.device('cuda', 0)
    k, n = 64, 3000
    cen = np.zeros((3, k), np.float32)
    for i in range(k):
        cen[:, i] = (40 + i, 40, 40)
    a, b = (28, 1) if swap else (1, 28)  # rows 1 and 28 of tile 0: lane-halves 0 and 1
    cen[:, a] = (2, 0, 0)
    cen[:, b] = (3, 1, 0)
    pts = np.zeros((3, n), np.float32)
    pts[:, : n // 2] = np.array([[3], [0], [0]], np.float32)
    pts[:, n // 2:] = np.array([[2], [0], [0]], np.float32)
    cols = [np.ascontiguousarray(pts[j]) for j in range(3)]
    _, want = oracle.kmeans_assign(cols, cen)
    tcols = [torch.from_numpy(c).to(dev) for c in cols]
    tcen = torch.from_numpy(cen.reshape(-1).copy()).to(dev)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.dev_kmeans_prepare(tcols)
    ctx.dev_kmeans_assign(tcols, k, tcen, lab)
    ctx.synchronize()
    same_bits(lab.cpu().numpy().astype(np.uint32), want)


def test_sync_check_mode_vs_oracle(monkeypatch):
    """ST_SYNC_CHECK=1 (read when a context is created) synchronizes the device after every
    launch check, so a fault is reported at the launch that caused it; results are unchanged."""
    n, C = 5000, 3
    cols = _table(n, C, 61)
    draws = oracle.mulberry32(5, 1 << 15)
    monkeypatch.setenv('ST_SYNC_CHECK', '1')
    c1 = sh.Context(0)
    tex, meta, used = c1.sog(cols, 2, draws)
    monkeypatch.delenv('ST_SYNC_CHECK')
    c1.close()
    sh.Context(0).close()  # a context created without it turns the checks off again
    rc, otex, ometa, oused = oracle.sog(cols, C, 2, draws)
    assert rc == 0 and used == oused
    for k in tex:
        same_bits(tex[k], otex[k])


def test_kmeans_labels_buffer_unaligned(ctx):
    """The decided points' grouping reads the labels 16 bytes at a time (k_code_scatter_run); a
    caller's labels buffer that is not 16-byte aligned takes the 4,096-point rounds instead
    (k_code_scatter).  Both give the reference's labels and centroids."""
    import torch
    n, d, k, iters = 40_000, 9, 256, 2
    rng = np.random.default_rng(61)
    cols = [rng.normal(0, 0.1, n).astype(np.float32) for _ in range(d)]
    draws = oracle.mulberry32(n + k + 3, 4 * k * (iters + 1) + 64)
    rc, ocent, olabels, oused = oracle.kmeans(cols, k, iters, draws)
    assert rc == 0
    dev = torch.device('cuda', 0)
    tcols = [torch.from_numpy(c).to(dev) for c in cols]
    for off in (0, 1):
        cen = torch.empty(d * k, device=dev)
        lab_buf = torch.empty(n + 4, dtype=torch.int32, device=dev)
        lab = lab_buf[off:off + n]
        assert (lab.data_ptr() % 16 == 0) == (off == 0)
        used = ctx.dev_kmeans(tcols, k, iters, draws, cen, lab)
        torch.cuda.synchronize()
        assert used == oused
        same_bits(lab.cpu().numpy().astype(np.uint32), np.asarray(olabels, dtype=np.uint32))
        same_bits(cen.cpu().numpy(), np.asarray(ocent, dtype=np.float32).reshape(-1))


@pytest.mark.parametrize('who', ['scales', 'colours', 'both', 'neither'])
def test_sog_cluster1d_draws_move_the_sh_cursor_vs_oracle(ctx, who):
    """writeSog's SH palette k-means starts at draw 0 beside the two cluster1d (a 1-D k-means
    takes draws only to re-seed empty clusters) and reruns at the cursor they leave when they did
    take draws (write-sog.ts:245-313): columns of four distinct values leave 252 of 256 clusters
    empty, so the scales' / the colours' cluster1d (or both) take draws; textures, codebooks and
    the draws used equal the reference's"""
    n, C = 20_011, 3
    cols = _table(n, C, 4242)
    rng = np.random.default_rng(77)
    groups = {'scales': ['scale_0', 'scale_1', 'scale_2'], 'colours': ['f_dc_0', 'f_dc_1', 'f_dc_2'],
              'both': ['scale_0', 'scale_1', 'scale_2', 'f_dc_0', 'f_dc_1', 'f_dc_2'], 'neither': []}[who]
    for k in groups:
        cols[k] = (rng.integers(0, 4, n) * 0.25 - 5).astype(np.float32)
    draws = oracle.mulberry32(31, 1 << 16)
    tex, meta, used = ctx.sog(cols, 3, draws)
    rc, otex, ometa, oused = oracle.sog(cols, C, 3, draws)
    assert rc == 0 and used == oused
    for k in otex:
        same_bits(tex[k], otex[k])
    for f in ('scales_codebook', 'sh0_codebook', 'shn_codebook'):
        same_bits(np.array(getattr(meta, f)[:]), np.array(getattr(ometa, f)[:]))
