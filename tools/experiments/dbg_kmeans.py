import sys, os, numpy as np
sys.path.insert(0, 'splat-transform_amd/py'); sys.path.insert(0, 'oracle')
import splat_hip as sh, oracle
os.environ['ST_DEBUG'] = '1'
ctx = sh.Context(0)
rng = np.random.default_rng(3)
n, d, k = 20000, 45, 1024
cols = [rng.normal(0, 0.1, n).astype(np.float32) for _ in range(d)]
draws = oracle.mulberry32(5, 10000)
cent, labels, used = ctx.kmeans(cols, k, 2, draws)
rc, oc, ol, ou = oracle.kmeans(cols, k, 2, draws)
print('match', np.array_equal(labels, ol), np.array_equal(cent.view(np.uint32), oc.view(np.uint32)))
