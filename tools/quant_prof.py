"""cProfile of the config-3 tree's rf-branch suggest (quantized labels at 2^20
candidates): where the host time of a quantized suggest goes."""
import cProfile
import ctypes
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED, loss=bench.rf_loss)
    for i in range(10):
        tpe.suggest([bench.N_HISTORY], domain, trials, i, n_EI_candidates=bench.C_PER_GPU)
    torch.cuda.synchronize()
    lat = []
    for i in range(n):
        t0 = time.perf_counter()
        tpe.suggest([bench.N_HISTORY], domain, trials, 100 + i, n_EI_candidates=bench.C_PER_GPU)
        lat.append(time.perf_counter() - t0)
    print('rf-branch suggest p50 %.1f us' % (1e6 * np.median(lat)))
    from hyperopt_amd.engine import get_engine
    eng = get_engine()
    eng.profile = {}
    for i in range(20):
        tpe.suggest([bench.N_HISTORY], domain, trials, 500 + i, n_EI_candidates=bench.C_PER_GPU)
    prof, eng.profile = eng.profile, None
    for k, v in prof.items():
        print('  device stage %-10s %7.1f us (%d launches)' % (k, 1e3 * np.median([a[0] for a in v]), len(v)))
    # host phases of the native call (tpe_host_phases) and numpy's argsort of
    # the quantized labels' columns (the caller's part of their fits)
    from hyperopt_amd import _native as N, history as H
    buf = (ctypes.c_double * len(N.PHASES))()
    eng.lib.tpe_host_phases(1, None, 0)
    ph = []
    for i in range(50):
        tpe.suggest([bench.N_HISTORY], domain, trials, 700 + i, n_EI_candidates=bench.C_PER_GPU)
        eng.lib.tpe_host_phases(1, buf, len(N.PHASES))
        ph.append(list(buf))
    eng.lib.tpe_host_phases(0, None, 0)
    med = np.median(np.array(ph), axis=0)
    print('  host phases (us since entry): ' + '  '.join('%s %.1f' % (k, v) for k, v in zip(N.PHASES, med)))
    hist = H.extract(domain, trials)
    for r in domain.table.rows:
        if r.dist.startswith('q'):
            x = np.asarray(hist.obs[r.label][1], dtype=np.float64)
            ts = []
            for _ in range(50):
                s0 = time.perf_counter()
                np.argsort(x)
                ts.append(time.perf_counter() - s0)
            print('  np.argsort %-16s n %6d: %6.1f us' % (r.label, len(x), 1e6 * np.median(ts)))
    pr = cProfile.Profile()
    pr.enable()
    for i in range(n):
        tpe.suggest([bench.N_HISTORY], domain, trials, 1000 + i, n_EI_candidates=bench.C_PER_GPU)
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
