"""Diagnostic: above-lpdf error distribution of test_device_fit_matches_oracle's
uniform case under batch flags (argv: flags values)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from oracle import tpe_oracle as O  # noqa: E402
from hyperopt_amd import parzen  # noqa: E402
from hyperopt_amd.engine import Engine, LevelProblem  # noqa: E402


def main():
    eng = Engine(precision='fp32')
    rs = np.random.RandomState(31)
    n = 20000
    obs = np.clip(np.concatenate([rs.normal(-2, 0.05, n // 2), rs.uniform(-5, 5, n // 2 - 3),
                                  [-4.9, 4.95, 0.0]]), -5, 5)
    rs.shuffle(obs)
    bidx = np.sort(rs.choice(n, 25, replace=False)).astype(np.int32)
    m = np.zeros(n, bool)
    m[bidx] = True
    args = dict(low=-5.0, high=5.0)
    host = parzen.fit_posterior('uniform', args, obs[m], obs[~m], 1.0)
    above = O.adaptive_parzen_normal(obs[~m], 1.0, 0.0, 10.0)
    C = 1 << 16
    sub = np.random.RandomState(0).choice(C, 6000, replace=False)
    for fl in sys.argv[1:]:
        os.environ['TPE_DEBUG_FLAGS'] = fl
        res, cand, l, g = eng.run([LevelProblem(host, 0, [3])], C, seed=9, want_lg=True, return_cand=True)
        ref = O.gmm1_lpdf(cand[0][sub], *above, low=-5.0, high=5.0)
        err = np.abs(g[0][sub] - ref) / np.maximum(np.abs(ref), 1.0)
        o = np.argsort(err)[::-1][:5]
        print('flags %s: max %.3g p99 %.3g mean %.3g; worst x %s err %s' % (
            fl, err.max(), np.percentile(err, 99), err.mean(), cand[0][sub][o], err[o]))
        sys.stdout.flush()


if __name__ == '__main__':
    main()
