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
