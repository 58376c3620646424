"""Wall-time split of the headline suggest without a profiler: time spent in
the Parzen fits, in the native level runner (pack + device round trip), and in
everything else, from perf_counter wrappers around those calls."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import engine as E, history as H, tpe  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    eng = E.get_engine(torch.device('cuda', 0))
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    acc = {}

    def wrap(obj, name, key):
        fn = getattr(obj, name)

        def w(*a, **k):
            t0 = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                acc[key] = acc.get(key, 0.0) + time.perf_counter() - t0
        setattr(obj, name, w)
    wrap(tpe._Fits, 'get', 'fits')
    wrap(eng, 'run_level', 'run_level')
    wrap(eng, 'suggest_tree', 'suggest_tree (native fits+levels)')
    wrap(tpe, '_tree_labels', 'suggest_tree/_tree_labels')
    wrap(H, 'extract', 'extract')
    wrap(H, 'split_below', 'split_below')
    wrap(tpe.rand, 'docs_from_choices', 'docs')
    wrap(tpe, '_predict_activity', 'predict(+gate fits)')
    wrap(eng, '_labels', 'run_level/_labels')
    for i in range(5):
        tpe.suggest([bench.N_HISTORY], domain, trials, i, n_EI_candidates=bench.C_PER_GPU)
    acc.clear()
    lat = []
    for i in range(steps):
        t0 = time.perf_counter()
        tpe.suggest([bench.N_HISTORY], domain, trials, 100 + i, n_EI_candidates=bench.C_PER_GPU)
        lat.append(time.perf_counter() - t0)
    tot = sum(lat)
    print('suggest p50 %.3f ms, mean %.3f ms' % (1e3 * np.median(lat), 1e3 * tot / steps))
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print('  %-12s %7.1f us/suggest' % (k, 1e6 * v / steps))
    nested = [k for k in acc if '/' in k or k.startswith('predict')]
    print('  %-12s %7.1f us/suggest' % ('other', 1e6 * (tot - sum(v for k, v in acc.items() if k not in nested))
                                       / steps))
    # the C packer alone on this host (the level runner's host share)
    import ctypes
    from hyperopt_amd import _native as N
    from hyperopt_amd.engine import LevelProblem
    hist = H.extract(domain, trials)
    fits = tpe._Fits(domain.table, hist, H.split_below(hist, 0.25), 1.0, eng)
    T = domain.table
    probs = [LevelProblem(fits.get(T.by_label[l]), T.by_label[l].index, [bench.N_HISTORY])
             for l in ['svm_C', 'svm_kernel', 'svm_rbf_gamma', 'model']]
    labels, keep = eng._labels(probs)
    info = N.PackInfo()
    pin = eng._pinned
    best = 1e9
    for _ in range(20):
        t0 = time.perf_counter()
        for _ in range(20):
            eng.lib.tpe_host_pack_level(labels, len(probs), bench.C_PER_GPU, 5, 0, 0, 0, pin.data_ptr(), pin.numel(),
                                        ctypes.byref(info))
        best = min(best, (time.perf_counter() - t0) / 20)
    print('  tpe_host_pack_level alone (4 labels, min of 20x20): %.1f us' % (1e6 * best))


if __name__ == '__main__':
    main()
