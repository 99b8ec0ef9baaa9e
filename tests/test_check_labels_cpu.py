"""bench.check_all_labels (the headline's every-label check) on CPU tensors: it accepts exact
argmins, counts a wrong label, settles near-ties with the sequential f64 distance and leaves
exact ties unchecked."""
import numpy as np
import torch

import bench


def _exact(sh, cen):
    p = sh.double().numpy()
    c = cen.double().numpy()
    d = np.zeros((p.shape[1], c.shape[1]))
    for j in range(p.shape[0]):  # the reference's order: dimension by dimension
        d += (c[j][None, :] - p[j][:, None]) ** 2
    return d


def test_check_all_labels_exact_wrong_and_ties():
    rng = np.random.default_rng(3)
    d, k, n = 7, 50, 3000
    cen = torch.from_numpy(rng.normal(size=(d, k)).astype(np.float32))
    sh = torch.from_numpy(rng.normal(size=(d, n)).astype(np.float32))
    # points exactly on centroid 3, and a duplicate of centroid 3 at 9: exact ties
    cen[:, 9] = cen[:, 3]
    sh[:, :5] = cen[:, 3:4]
    # a near-tie: a point halfway (in f32) between centroids 11 and 12 along one axis
    cen[:, 12] = cen[:, 11]
    cen[0, 12] = cen[0, 11] + 2.0 ** -10
    sh[:, 10] = cen[:, 11]
    sh[0, 10] = cen[0, 11] + 2.0 ** -11
    dist = _exact(sh, cen)
    lab = torch.from_numpy(dist.argmin(1).astype(np.int32))
    bad, ties, slow = bench.check_all_labels(sh, cen, lab, tile=512)
    assert bad == 0 and ties >= 6 and slow >= ties
    lab[100] = (lab[100] + 1) % k
    bad, _, _ = bench.check_all_labels(sh, cen, lab, tile=512)
    assert bad == 1


def test_check_all_labels_many_exact_ties_vectorised():
    """30% of the points sit on a centroid that has a duplicate (what the reference's KdTree
    order decides): every one is counted as a tie, in one pass"""
    import time
    rng = np.random.default_rng(4)
    d, k, n = 9, 64, 20000
    cen = torch.from_numpy(rng.normal(size=(d, k)).astype(np.float32))
    cen[:, 20] = cen[:, 5]
    sh = torch.from_numpy(rng.normal(size=(d, n)).astype(np.float32))
    dup = rng.random(n) < 0.3
    sh[:, torch.from_numpy(dup)] = cen[:, 5:6]
    dist = _exact(sh, cen)
    lab = torch.from_numpy(dist.argmin(1).astype(np.int32))
    want_ties = int(((dist == dist.min(1, keepdims=True)).sum(1) > 1).sum())  # also points nearest to 5 anyway
    assert want_ties >= int(dup.sum())
    t0 = time.time()
    bad, ties, slow = bench.check_all_labels(sh, cen, lab, tile=4096)
    assert bad == 0 and ties == want_ties and slow >= ties
    assert time.time() - t0 < 60
