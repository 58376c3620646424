"""cProfile of the config-3 tree's rf-branch suggest (quantized labels at 2^20
candidates): where the host time of a quantized suggest goes."""
import cProfile
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
    pr = cProfile.Profile()
    pr.enable()
    for i in range(n):
        tpe.suggest([bench.N_HISTORY], domain, trials, 1000 + i, n_EI_candidates=bench.C_PER_GPU)
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
