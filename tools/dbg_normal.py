import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from oracle import tpe_oracle as O
from hyperopt_amd.engine import Engine, LevelProblem
from hyperopt_amd import parzen
import test_gpu_kernels as T
engine = Engine(precision='fp32')
rs = np.random.RandomState(31)
n = 20000
dist, args = 'normal', dict(mu=1.0, sigma=3.0)
obs = rs.normal(1.0, 3.0, n)
rs.shuffle(obs)
bidx = np.sort(rs.choice(n, 25, replace=False)).astype(np.int32)
m = np.zeros(n, bool); m[bidx] = True
host = parzen.fit_posterior(dist, args, obs[m], obs[~m], 1.0)
dev, _ = T._device_post(engine, dist, args, obs, bidx)
above = O.adaptive_parzen_normal(obs[~m], 1.0, 1.0, 3.0)
C = 1 << 16
for name, post in (('dev', dev), ('host', host)):
    for ex in (True, False):
        engine.expand = ex
        res, cand, l, g = engine.run([LevelProblem(post, 0, [3])], C, seed=9, want_lg=True, return_cand=True)
        ref = O.gmm1_lpdf(cand[0], *above)
        err = np.abs(g[0] - ref) / np.maximum(np.abs(ref), 1)
        i = int(np.argmax(err))
        print(name, 'expand', ex, 'max err %.3g at %d x=%r g=%r ref=%r' % (err.max(), i, cand[0][i], g[0][i], ref[i]), 'n>1e-6:', int((err > 1e-6).sum()))
