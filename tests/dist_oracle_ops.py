"""CPU stand-in for splat_dist.HipOps -- TEST INFRASTRUCTURE ONLY.

Implements the per-rank step API of the multi-GPU k-means (assign, partials,
seqsum, finish, average, codebook) with the oracle restatement and plain
Python floats on CPU tensors, so the exchange logic of splat_dist (certificate,
segment-ordered chain, re-seed ownership, Math.random bookkeeping) runs under
gloo on a machine without a GPU and can be compared with the single-process
oracle."""
import numpy as np
import torch

import oracle
import splat_hip as sh


def _ulp_exp(x):
    e = (np.float32(x).view(np.uint32) >> 23) & 0xff
    return -149 if e == 0 else int(e) - 150


class OracleOps:
    device = torch.device('cpu')

    def empty(self, shape, dtype):
        return torch.empty(shape, dtype=dtype)

    def zeros(self, shape, dtype):
        return torch.zeros(shape, dtype=dtype)

    def minmax(self, cols):
        lo, hi = [], []
        for c in cols:
            a = c.numpy()
            a = a[~np.isnan(a)]
            lo.append(float(a.min()) if a.size else float('inf'))
            hi.append(float(a.max()) if a.size else float('-inf'))
        return lo, hi

    def init_rows(self, draws, n, k):
        """initializeCentroids (k-means.ts:8-20): the reference's rejection loop over the global n"""
        rows, chosen, cur = [], set(), 0
        while len(rows) < k:
            if cur >= len(draws):
                raise sh.StError(sh.ST_ERR_DRAWS, 'kmeans: Math.random draws exhausted during initialisation')
            r = int(np.floor(draws[cur] * n))
            cur += 1
            if r not in chosen:
                chosen.add(r)
                rows.append(r)
        return torch.tensor(rows, dtype=torch.int64), cur

    def gather_rows(self, pts, offset, rows):
        n = pts[0].shape[0]
        out = torch.zeros((len(pts), rows.shape[0]), dtype=torch.float32)
        for i, r in enumerate(rows.tolist()):
            if offset <= r < offset + n:
                for j, p in enumerate(pts):
                    out[j, i] = p[r - offset]
        return out

    def prepare(self, pts):
        if not all(np.isfinite(p.numpy()).all() for p in pts):
            raise sh.StError(sh.ST_ERR_NONFINITE, 'kmeans: non-finite point')

    def assign(self, pts, k, cen, labels):
        rc, lab = oracle.kmeans_assign([p.numpy() for p in pts], cen.numpy())
        assert rc == 0
        labels.copy_(torch.from_numpy(lab.astype(np.int32)))

    def partials(self, pts, nseg, k, labels):
        d, n = len(pts), pts[0].shape[0]
        seg_len = n // nseg
        vals = np.stack([p.numpy() for p in pts])
        lab = labels.numpy().astype(np.int64)
        self.members = {}
        sums = np.zeros((nseg, d, k))
        sabs = np.zeros((nseg, d, k))
        emin = np.full((nseg, d, k), 1 << 20, np.int32)
        counts = np.zeros((nseg, k), np.int32)
        for s in range(nseg):
            for c in range(k):
                m = [i for i in range(s * seg_len, (s + 1) * seg_len) if lab[i] == c]
                self.members[(s, c)] = m
                counts[s, c] = len(m)
                for j in range(d):
                    acc = 0.0
                    sa = 0.0
                    for i in m:
                        v = float(vals[j, i])
                        acc += v
                        sa += abs(v)
                        if v != 0.0:
                            emin[s, j, c] = min(emin[s, j, c], _ulp_exp(v))
                    sums[s, j, c] = acc
                    sabs[s, j, c] = sa
        self.vals, self.d = vals, d
        return (torch.from_numpy(sums), torch.from_numpy(sabs), torch.from_numpy(emin), torch.from_numpy(counts))

    def seqsum(self, d, k, seg, pairs, running, emin=None, sabs=None):
        for p, pair in enumerate(pairs.tolist()):
            c, j = divmod(pair, d)
            acc = float(running[p])
            for i in self.members[(seg, c)]:
                acc += float(self.vals[j, i])
            running[p] = acc

    def finish(self, d, k, sums, sabs, emin, counts, cen):
        pend = []
        for c in range(k):
            cnt = int(counts[c])
            for j in range(d):
                if not cnt:
                    continue
                sa, em = float(sabs[j, c]), int(emin[j, c])
                if sa == 0.0 or sa * (1.0 + 1.0e-6) < 2.0 ** (em + 53):
                    cen[j, c] = float(np.float32(float(sums[j, c]) / cnt))
                else:
                    pend.append(c * d + j)
        return torch.tensor(pend, dtype=torch.int32)

    def average(self, d, k, pairs, running, counts, cen):
        for p, pair in enumerate(pairs.tolist()):
            c, j = divmod(pair, d)
            cen[j, c] = float(np.float32(float(running[p]) / int(counts[c])))

    def codebook(self, cen, labels):
        cv = cen.numpy()
        key = np.where(cv == 0, np.float32(0), cv)
        order = np.argsort(key, kind='stable')
        inv = np.empty(256, np.int64)
        inv[order] = np.arange(256)
        return torch.from_numpy(cv[order].copy()), torch.from_numpy(inv[labels.numpy().astype(np.int64)].astype(np.uint8))
