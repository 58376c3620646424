"""Where the headline suggest's Python time goes on the real device: each
Python step of tpe.suggest timed by thin wrappers (history extract, below
split, tree records, the native call, the result documents) over a steady
loop, medians in us; the native call's own host phases beside."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
from hyperopt_amd import _native as N, history as H, rand, tpe  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    acc = {}

    def wrap(mod, name, key):
        f = getattr(mod, name)

        def g(*a, **k):
            t = time.perf_counter()
            r = f(*a, **k)
            acc.setdefault(key, []).append(time.perf_counter() - t)
            return r
        setattr(mod, name, g)

    wrap(tpe._history, 'extract', 'extract')
    wrap(tpe._history, 'split_below', 'split_below')
    wrap(tpe, '_tree_labels', 'tree_labels')
    wrap(tpe, '_native_tree', 'native_tree')
    wrap(rand, 'docs_from_choices', 'docs')
    lib = N.load()
    buf = (ctypes.c_double * len(N.PHASES))()
    walls, ret = [], []
    for i in range(n + 50):
        lib.tpe_host_phases(1, None, 0)
        t = time.perf_counter()
        tpe.suggest([bench.N_HISTORY], domain, trials, 100 + i, n_EI_candidates=bench.C_PER_GPU)
        w = time.perf_counter() - t
        lib.tpe_host_phases(1, buf, len(N.PHASES))
        if i >= 50:
            walls.append(w)
            ret.append(buf[N.PHASES.index('return')])
    for k in acc:
        acc[k] = acc[k][-n:]
    print('suggest wall p50 %.1f us; native call (phase clock, entry to return) p50 %.1f us' %
          (1e6 * np.median(walls), np.median(ret)))
    for k, v in acc.items():
        print('  %-12s %6.1f us' % (k, 1e6 * np.median(v)))
    med = {k: 1e6 * np.median(v) for k, v in acc.items()}
    print('  glue (wall - extract - split - native_tree - docs) %.1f us' %
          (1e6 * np.median(walls) - med['extract'] - med['split_below'] - med['native_tree'] - med['docs']))
    print('  native_tree besides tree_labels and the native call %.1f us' %
          (med['native_tree'] - med['tree_labels'] - np.median(ret)))


if __name__ == '__main__':
    main()
