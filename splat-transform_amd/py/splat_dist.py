"""splat_dist.py -- multi-GPU kmeans / cluster1d / writeSog over a row-sharded table.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI, "gloo"
works too).  Rank r holds rows [off_r, off_r + n_r) of every column, ranks in
order, so the global table is the concatenation of the shards.  The results are
the single-device results on that global table, bit for bit:

* k-means (k-means.ts:137-201): assign is row-local; the update needs the
  per-cluster f64 sums of calcAverage, which the reference adds in ascending
  global point order.  Each rank computes exact partials; where the global
  certificate sum|x| < 2^(emin+53) holds (almost everywhere) the allreduced sum
  is the reference's, the remaining (cluster, dim) pairs replay the sequential
  sum by handing the running value from segment to segment in global order
  (st_dev_kmeans_seqsum on the owner, a broadcast between ranks).
  Math.random: every rank holds the same draws and consumes them identically
  (init rows, empty-cluster re-seeds in ascending cluster order); the owner of a
  drawn row supplies its values.
* Morton order (ordering.ts:4-110) is a global sort: x/y/z are all-gathered and
  every rank orders the whole table (one exchange of 12 B/splat).  Each rank writes
  the texels of its own rows in row order; rank 0 gathers them (4 B per splat and
  texture) and places them at their global Morton positions.

`HipOps` is the product backend (the C-ABI step API on device tensors).  Any object
with the same methods can stand in (tests/dist_oracle_ops.py checks the exchange
logic on CPU with gloo).
"""
import math

import numpy as np
import torch
import torch.distributed as dist

import splat_hip as sh


class Comm:
    """torch.distributed collectives; gloo runs on host copies of device tensors."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.host = dist.get_backend(group) == 'gloo'
        self.dev = torch.device('cpu') if self.host else torch.device('cuda', torch.cuda.current_device())

    def _io(self, t):
        return t if t.device == self.dev else t.to(self.dev)

    def allreduce(self, t, op=dist.ReduceOp.SUM):
        x = self._io(t)
        dist.all_reduce(x, op=op, group=self.group)
        if x is not t:
            t.copy_(x)
        return t

    def broadcast(self, t, src):
        x = self._io(t)
        dist.broadcast(x, src=src, group=self.group)
        if x is not t:
            t.copy_(x)
        return t

    def gather_async(self, t, dst=0):
        """every rank's tensor (equal shapes) gathered on rank dst, issued without waiting: returns
        wait() -> the list on rank dst, None elsewhere.  `t` must stay untouched until wait() returns."""
        x = self._io(t)
        out = [torch.empty_like(x) for _ in range(self.world)] if self.rank == dst else None
        work = dist.gather(x, out, dst=dst, group=self.group, async_op=True)

        def wait():
            work.wait()
            return None if out is None else [o.to(t.device) for o in out]
        return wait

    def allgather(self, t):
        """list of every rank's tensor (shapes may differ in dim 0)"""
        x = self._io(t)
        n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(sizes, n, group=self.group)
        m = int(max(s.item() for s in sizes))
        pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        pad[:x.shape[0]] = x
        out = [torch.zeros_like(pad) for _ in range(self.world)]
        dist.all_gather(out, pad, group=self.group)
        return [o[:int(s.item())].to(t.device) for o, s in zip(out, sizes)]


class Shard:
    """row ranges of every rank"""

    def __init__(self, comm, n_local):
        self.comm = comm
        counts = comm.allgather(torch.tensor([n_local], dtype=torch.int64))
        self.counts = [int(c.item()) for c in counts]
        self.offsets = [sum(self.counts[:r]) for r in range(comm.world)]
        self.n = n_local
        self.off = self.offsets[comm.rank]
        self.N = sum(self.counts)

    def owner(self, row):
        for r in range(self.comm.world):
            if self.offsets[r] <= row < self.offsets[r] + self.counts[r]:
                return r
        raise IndexError(row)


class HipOps:
    """the product backend: libsplat_hip step API on device tensors"""

    def __init__(self, ctx, device):
        self.ctx = ctx
        self.device = device
        # library kernels and the torch glue between them share one stream.  It must be a
        # real stream: st_ctx_set_stream(NULL) selects the context's own stream, so torch's
        # legacy default stream (handle 0) would not order against the library.  The entry
        # points below run their torch glue on it (`_on_stream`); the caller's current stream
        # is left as it was.
        cur = torch.cuda.current_stream(device)
        if cur.cuda_stream == 0:
            cur = torch.cuda.Stream(device)
        self.stream = cur
        ctx.set_stream(cur.cuda_stream)

    def empty(self, shape, dtype):
        return torch.empty(shape, dtype=dtype, device=self.device)

    def zeros(self, shape, dtype):
        return torch.zeros(shape, dtype=dtype, device=self.device)

    # an empty shard (a rank with no rows) skips the library calls over its rows: their
    # contributions are the identities of the collectives that follow
    def minmax(self, cols):
        if cols[0].numel() == 0:
            return [math.inf] * len(cols), [-math.inf] * len(cols)
        return self.ctx.dev_minmax(cols)

    def init_rows(self, draws, n, k):
        rows = self.empty((k,), torch.int32)
        used = self.ctx.dev_kmeans_init_rows(draws, n, k, rows)
        return rows, used

    def gather_rows(self, pts, offset, rows):
        out = self.empty((len(pts), rows.shape[0]), torch.float32)
        self.ctx.dev_gather_rows(pts, offset, rows, out)
        return out

    def prepare(self, pts):
        self.rows = pts[0].numel()
        if self.rows:
            self.ctx.dev_kmeans_prepare(pts)

    def assign(self, pts, k, cen, labels):
        if pts[0].numel():
            self.ctx.dev_kmeans_assign(pts, k, cen, labels)

    def partials(self, pts, nseg, k, labels):
        d = len(pts)
        sums = self.empty((nseg, d, k), torch.float64)
        sabs = self.empty((nseg, d, k), torch.float64)
        emin = self.empty((nseg, d, k), torch.int32)
        counts = self.empty((nseg, k), torch.int32)
        if pts[0].numel() == 0:  # st_dist.hip k_partials: sums 0, ulp exponent 2^20 for no members
            return sums.zero_(), sabs.zero_(), emin.fill_(1 << 20), counts.zero_()
        self.ctx.dev_kmeans_partials(pts, nseg, k, labels, sums, sabs, emin, counts)
        return sums, sabs, emin, counts

    def seqsum(self, d, k, seg, pairs, running, emin, sabs):
        if self.rows:  # an empty shard adds nothing to the running sums
            self.ctx.dev_kmeans_seqsum(d, k, seg, pairs, running, emin, sabs)

    def finish(self, d, k, sums, sabs, emin, counts, cen):
        pending = self.empty((d * k,), torch.int32)
        npend = self.ctx.dev_kmeans_finish(d, k, sums, sabs, emin, counts, cen, pending)
        return pending[:npend]

    def average(self, d, k, pairs, running, counts, cen):
        self.ctx.dev_kmeans_average(d, k, pairs, running, counts, cen)

    def codebook(self, cen, labels):
        cb = self.empty((256,), torch.float32)
        lab8 = self.empty((labels.shape[0],), torch.uint8)
        self.ctx.dev_cluster1d_codebook(cen, labels, cb, lab8)
        return cb, lab8

    def morton(self, x, y, z):
        idx = torch.arange(x.shape[0], dtype=torch.int32, device=self.device)
        self.ctx.dev_morton_order(x, y, z, idx)
        return idx

    def cluster1d_local(self, cols, iters, draws):
        """replicated cluster1d (identical input on every rank): the single-device path"""
        n = cols[0].shape[0]
        cb = self.empty((256,), torch.float32)
        lab = self.empty((len(cols) * n,), torch.uint8)
        used = self.ctx.dev_cluster1d(cols, iters, np.ascontiguousarray(draws), cb, lab)
        return cb, lab, used

    def scatter(self, cols, pos, lo, hi, scale_lab, color_lab, shn_lab, tex):
        return self.ctx.dev_sog_scatter(cols, pos, lo, hi, scale_lab, color_lab, shn_lab, tex)

    def shn_centroids(self, cl, C, pal, out):
        self.ctx.dev_sog_shn_centroids(cl, C, pal, out)


# ---- k-means ---------------------------------------------------------------------------
class _Points:
    """the k-means point set of one rank and its place in the global order"""

    def __init__(self, shard, cols, concat):
        self.shard = shard
        self.concat = concat  # cluster1d: columns concatenated (column-major over the global table)
        if concat:
            self.pts = [torch.cat([c.reshape(-1) for c in cols])] if len(cols) > 1 else [cols[0]]
            self.nseg = len(cols)
            self.d = 1
            self.N = shard.N * len(cols)
        else:
            self.pts = list(cols)
            self.nseg = 1
            self.d = len(cols)
            self.N = shard.N
        self.n = self.pts[0].shape[0]

    def segments(self):
        """(owner rank, local segment) in global order"""
        world = self.shard.comm.world
        return [(r, s) for s in range(self.nseg) for r in range(world)]

    def locate(self, g):
        """global point indices (array) -> (owner ranks, local point indices)"""
        g = np.asarray(g, dtype=np.int64)
        offs = np.asarray(self.shard.offsets, dtype=np.int64)
        cnts = np.asarray(self.shard.counts, dtype=np.int64)
        if self.concat:
            col, row = np.divmod(g, self.shard.N)
            r = np.searchsorted(offs, row, side='right') - 1
            return r, col * cnts[r] + (row - offs[r])
        r = np.searchsorted(offs, g, side='right') - 1
        return r, g - offs[r]


def _on_stream(f):
    """run an entry point's torch glue on the library's stream (ops.stream), then restore the
    caller's current stream"""
    import functools

    @functools.wraps(f)
    def wrap(ops, *a, **kw):
        if getattr(ops, 'stream', None) is None:  # a host backend (the tests' CPU stand-in)
            return f(ops, *a, **kw)
        caller = torch.cuda.current_stream(ops.device)
        ops.stream.wait_stream(caller)  # the inputs were produced on the caller's stream
        with torch.cuda.stream(ops.stream):
            out = f(ops, *a, **kw)
        caller.wait_stream(ops.stream)  # and the outputs are read there
        return out
    return wrap


def _gather_rows(ops, comm, P, rows):
    """values (d, len(rows)) of global points `rows`, supplied by their owners"""
    m = len(rows)
    owners, local = P.locate(rows)
    vals = ops.zeros((max(m, 1), P.d), torch.float32)
    mine = np.nonzero(owners == comm.rank)[0]
    if mine.size:
        ii = torch.from_numpy(mine).to(vals.device)
        li = torch.from_numpy(local[mine]).to(vals.device)
        for j in range(P.d):
            vals[ii, j] = P.pts[j][li]
    parts = comm.allgather(vals)
    out = ops.zeros((P.d, max(m, 1)), torch.float32)
    for r in range(comm.world):
        sel = torch.from_numpy(np.nonzero(owners == r)[0]).to(vals.device)
        if sel.numel():
            out[:, sel] = parts[r][sel].t()
    return out[:, :m]


@_on_stream
def kmeans(ops, comm, shard, cols, k, iters, draws, concat=False):
    """kmeans over the global table (k-means.ts:137-201, --no-gpu results).

    cols: local device columns; concat=True clusters cluster1d's 1-D concatenation
    of the columns.  Returns (centroids (d, k) float32, local labels, draws used)."""
    P = _Points(shard, cols, concat)
    if P.N < k:
        # k-means.ts:139-144: the points themselves are the centroids, point i is labelled i
        cen = _gather_rows(ops, comm, P, np.arange(P.N))
        r = comm.rank
        cnt, off = shard.counts[r], shard.offsets[r]
        j = np.arange(P.n, dtype=np.int64)
        g = (j // max(cnt, 1)) * shard.N + off + j % max(cnt, 1) if concat else off + j
        return cen, torch.from_numpy(g.astype(np.int32)).to(P.pts[0].device), 0
    d, n = P.d, P.n
    ops.prepare(P.pts)
    cursor = 0
    if d == 1:
        lo, hi = ops.minmax(P.pts)
        t = torch.tensor([lo[0], -hi[0]], dtype=torch.float64)
        comm.allreduce(t, dist.ReduceOp.MIN)
        m, M = t[0].item(), -t[1].item()
        i = np.arange(k, dtype=np.float64)
        cen_np = (m + (M - m) * i / (k - 1)).astype(np.float32)  # initializeCentroids1D (k-means.ts:23-39)
        cen = torch.from_numpy(cen_np).to(P.pts[0].device).reshape(1, k)
    else:
        # initializeCentroids: the same k global rows on every rank (st_dev_kmeans_init_rows); each
        # rank supplies the rows it holds, the others' bit patterns are 0, an integer SUM assembles them
        rows, used = ops.init_rows(draws[cursor:], P.N, k)
        cursor += used
        cen = ops.gather_rows(P.pts, shard.off, rows).contiguous()
        comm.allreduce(cen.view(torch.int32))
    labels = ops.empty((n,), torch.int32)
    for _ in range(iters):
        ops.assign(P.pts, k, cen, labels)
        sums, sabs, emin, counts = ops.partials(P.pts, P.nseg, k, labels)
        # one SUM allreduce for the f64 sums, sum|x| and the counts (exact in f64 below 2^53),
        # one MIN allreduce for the ulp exponents
        SAC = torch.cat([sums.sum(0).reshape(-1), sabs.sum(0).reshape(-1),
                         counts.sum(0, dtype=torch.float64).reshape(-1)])
        E = emin.min(0).values.contiguous()
        comm.allreduce(SAC)
        comm.allreduce(E, dist.ReduceOp.MIN)
        S = SAC[:d * k].reshape(d, k)
        A = SAC[d * k:2 * d * k].reshape(d, k)
        C = SAC[2 * d * k:].to(torch.int32)
        pending = ops.finish(d, k, S, A, E, C, cen)
        if pending.numel():
            running = ops.zeros((pending.numel(),), torch.float64)
            for r, seg in P.segments():
                if r == comm.rank:
                    ops.seqsum(d, k, seg, pending, running, E, A)
                comm.broadcast(running, r)
            ops.average(d, k, pending, running, C, cen)
        empty = (C == 0).nonzero().flatten().tolist()
        if empty:  # re-seed (k-means.ts:174-178): ascending clusters, one draw each
            rows = []
            for _ in empty:
                if cursor >= len(draws):
                    raise sh.StError(sh.ST_ERR_DRAWS, 'kmeans: Math.random draws exhausted while re-seeding')
                if not 0.0 <= draws[cursor] < 1.0:  # the row would fall outside the table
                    raise sh.StError(sh.ST_ERR_ARG, 'kmeans: a re-seed draw outside [0, 1)')
                rows.append(math.floor(draws[cursor] * P.N))
                cursor += 1
            vals = _gather_rows(ops, comm, P, rows)
            cen[:, torch.tensor(empty, dtype=torch.int64, device=cen.device)] = vals
    return cen, labels, cursor


@_on_stream
def cluster1d(ops, comm, shard, cols, iters, draws):
    """cluster1d (write-sog.ts:56-99) over the global table: codebook (256) + byte labels
    of the local rows, one column block per input column"""
    cen, labels, used = kmeans(ops, comm, shard, cols, 256, iters, draws, concat=True)
    cb, lab8 = ops.codebook(cen.reshape(-1), labels)
    return cb, lab8, used


# ---- writeSog ------------------------------------------------------------------------------
@_on_stream
def write_sog(ops, comm, cols, iters, draws):
    """writeSog's textures + meta (write-sog.ts:110-370) for the global table.
    cols: dict name -> local device column.  Returns (textures, meta) on rank 0 (None elsewhere)
    and the number of draws consumed."""
    shard = Shard(comm, cols['x'].shape[0])
    N = shard.N
    C = _sh_coeffs(cols)
    W, H, pal, cw, ch = sh.sog_geometry(N, C)
    dev = cols['x'].device
    # global Morton order: every rank orders the whole table, keeps its rows' positions
    xyz = [torch.cat(comm.allgather(cols[a])) for a in ('x', 'y', 'z')]
    idx = ops.morton(*xyz)
    del xyz
    pos_all = torch.empty(N, dtype=torch.int32, device=dev)
    pos_all[idx.long()] = torch.arange(N, dtype=torch.int32, device=dev)
    del idx
    if comm.rank != 0:
        pos_all = None  # rank 0 places every rank's texels
    lo, hi = ops.minmax([cols['x'], cols['y'], cols['z']])
    t = torch.tensor(list(lo) + [-v for v in hi], dtype=torch.float64)
    comm.allreduce(t, dist.ReduceOp.MIN)
    lo, hi = t[:3].tolist(), [-v for v in t[3:].tolist()]

    cursor = 0
    meta = {}
    scb, slab, u = cluster1d(ops, comm, shard, [cols[f'scale_{i}'] for i in range(3)], iters, draws[cursor:])
    cursor += u
    ccb, clab, u = cluster1d(ops, comm, shard, [cols[f'f_dc_{i}'] for i in range(3)], iters, draws[cursor:])
    cursor += u
    meta['scales_codebook'] = scb.cpu().numpy()
    meta['sh0_codebook'] = ccb.cpu().numpy()
    # texels of this rank's rows in local row order (4 B per row and texture); rank 0
    # gathers them and places them at their global Morton positions.  The five textures
    # that do not wait for the SH k-means go out now, their gathers overlapping it.
    rows = torch.arange(shard.n, dtype=torch.int32, device=dev)
    early = ('means_l', 'means_u', 'quats', 'scales', 'sh0')
    loc = {k: torch.zeros(shard.n * 4, dtype=torch.uint8, device=dev) for k in early}
    m = ops.scatter(cols, rows, lo, hi, slab, clab, None, loc)
    pending = gather_texels_start(comm, shard, loc)
    shn_cent = None
    if C:
        D = 3 * C
        cen, shn_lab, u = kmeans(ops, comm, shard, [cols[f'f_rest_{i}'] for i in range(D)], pal, iters,
                                 draws[cursor:])
        cursor += u
        ncb, ncl, u = ops.cluster1d_local([cen[i].contiguous() for i in range(D)], iters, draws[cursor:])
        cursor += u
        meta['shn_codebook'] = ncb.cpu().numpy()
        if comm.rank == 0:
            shn_cent = torch.zeros(cw * ch * 4, dtype=torch.uint8, device=dev)
            ops.shn_centroids(ncl, C, pal, shn_cent)
        late = {'shN_labels': torch.zeros(shard.n * 4, dtype=torch.uint8, device=dev)}
        ops.scatter(cols, rows, lo, hi, None, None, shn_lab, late)
        pending.update(gather_texels_start(comm, shard, late))
    tex = gather_texels_finish(comm, shard, pending, pos_all, W * H)
    if comm.rank != 0:
        return None, None, cursor
    if shn_cent is not None:
        tex['shN_centroids'] = shn_cent
    meta.update(width=W, height=H, count=N, means_min=list(m.means_min), means_max=list(m.means_max),
                sh_bands={0: 0, 3: 1, 8: 2, 15: 3}[C], palette_size=pal, shn_width=cw, shn_height=ch)
    return tex, meta, cursor


def gather_texels(comm, shard, loc, pos_all, size):
    """The textures of the global table on rank 0 (None elsewhere): every rank holds the RGBA
    texels of its own rows in local row order (`loc`, 4 B per row); rank 0 gathers them (one
    point-to-point transfer per rank, N x 4 B per texture in total, instead of a sum-reduce of
    whole textures) and places global row r at pos_all[r], its position in the Morton order.
    Texels past the table stay zero, as in the single-device writer."""
    return gather_texels_finish(comm, shard, gather_texels_start(comm, shard, loc), pos_all, size)


def gather_texels_start(comm, shard, loc):
    """issue the (asynchronous) gathers of gather_texels; returns the pending transfers"""
    m = max(shard.counts)
    pending = {}
    for key, t in loc.items():
        v = t.view(torch.int32)
        pad = torch.zeros(m, dtype=torch.int32, device=v.device)
        pad[:v.numel()] = v
        pending[key] = comm.gather_async(pad, 0)
    return pending


def gather_texels_finish(comm, shard, pending, pos_all, size):
    """wait for the gathers and place the rows on rank 0 (see gather_texels)"""
    out = {}
    for key, wait in pending.items():
        parts = wait()
        if parts is None:
            continue
        full = torch.cat([p[:c] for p, c in zip(parts, shard.counts)])
        tex = torch.zeros(size, dtype=torch.int32, device=full.device)
        tex[pos_all.long()] = full
        out[key] = tex.view(torch.uint8)
    return out if comm.rank == 0 else None


def _sh_coeffs(cols):
    # band rule of transform.ts:20 / write-sog.ts:296
    miss = next((i for i in range(45) if f'f_rest_{i}' not in cols), -1)
    return [0, 3, 8, 15][{9: 1, 24: 2, -1: 3}.get(miss, 0)]


def meta_struct(meta):
    """the SogMeta (st_abi.h) of write_sog's meta dict, for the .sog bundle on rank 0"""
    m = sh.SogMeta()
    m.width, m.height = meta['width'], meta['height']
    for k in range(3):
        m.means_min[k] = meta['means_min'][k]
        m.means_max[k] = meta['means_max'][k]
    for k in range(256):
        m.scales_codebook[k] = float(meta['scales_codebook'][k])
        m.sh0_codebook[k] = float(meta['sh0_codebook'][k])
        if meta['sh_bands']:
            m.shn_codebook[k] = float(meta['shn_codebook'][k])
    m.sh_bands, m.palette_size = meta['sh_bands'], meta['palette_size']
    m.shn_width, m.shn_height = meta['shn_width'], meta['shn_height']
    return m


@_on_stream
def write_sog_bundle(ops, comm, cols, iters, draws, dos_time, dos_date):
    """writeSog to a .sog archive (write-sog.ts:110-370 + zip-writer.ts) for the global table:
    the textures of write_sog, then WebP + CRC + ZIP on rank 0's device.  Returns the archive
    bytes on rank 0 (None elsewhere) and the draws consumed."""
    tex, meta, used = write_sog(ops, comm, cols, iters, draws)
    if tex is None:
        return None, used
    return ops.ctx.dev_sog_bundle(meta_struct(meta), meta['count'], tex, dos_time, dos_date), used

