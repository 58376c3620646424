"""CPU timing of the native host phases of the config-3 suggest (no GPU):
the svm/rbf branch's label fits (tpe_host_fit_split / tpe_host_cat_split) and
tpe_host_pack_level of its fused level, each repeated; prints microseconds per
call (median of repeats).  Usage: python tools/pack_time.py [N_HISTORY] [REPS]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import _native as N, history as H, tpe  # noqa: E402
from hyperopt_amd.engine import Engine, LevelProblem  # noqa: E402


def main():
    n_hist = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    lib = N.load()
    domain, trials = bench.make_history(n_hist, bench.SEED)
    T = domain.table
    hist = H.extract(domain, trials)
    below = H.split_below(hist, 0.25)
    fits = tpe._Fits(T, hist, below, 1.0, None)
    labels = ['model', 'svm_kernel', 'svm_C', 'svm_rbf_gamma']
    rows = [T.by_label[k] for k in labels]
    ids = np.array([n_hist], dtype=np.int64)
    t0 = time.perf_counter()
    for _ in range(50):
        fits.cache.clear()
        for r in rows:
            fits.get(r)
    t_fit = (time.perf_counter() - t0) / 50 * 1e6
    problems = [LevelProblem(fits.get(r), r.index, ids) for r in rows]
    recs, keep = Engine._labels(problems)
    info = N.PackInfo()
    cap = 64 << 20
    NC = int(sys.argv[3]) if len(sys.argv) > 3 else bench.C_PER_GPU
    blob = np.empty(cap, dtype=np.uint8)
    ts = []
    for _ in range(reps):
        s = time.perf_counter()
        rc = lib.tpe_host_pack_level(recs, len(problems), NC, 7, 0, 0, N.PREC_F32, blob.ctypes.data, cap,
                                     ctypes.byref(info))
        ts.append(time.perf_counter() - s)
        assert rc == 0, rc
    ks = [int(p.post.above[0].shape[0]) if p.post.above is not None else 0 for p in problems]
    print('history %d, labels %s, above K %s' % (n_hist, labels, ks))
    print('python _Fits (4 labels, incl. ctypes): %.1f us' % t_fit)
    print('tpe_host_pack_level: p50 %.1f us, p10 %.1f us (blob %d B, %d tab jobs, %d tab units)'
          % (1e6 * np.median(ts), 1e6 * np.percentile(ts, 10), info.blob_bytes, info.n_tab_jobs, info.tab_units))


if __name__ == '__main__':
    main()
