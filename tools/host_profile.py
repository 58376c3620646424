"""cProfile of the bench workload's suggest calls (host-side cost breakdown)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402
from hyperopt_amd.engine import get_engine  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    get_engine(torch.device('cuda', 0))
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    C = bench.C_PER_GPU
    for i in range(3):
        tpe.suggest([bench.N_HISTORY], domain, trials, i, n_EI_candidates=C)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for i in range(steps):
        tpe.suggest([bench.N_HISTORY], domain, trials, 100 + i, n_EI_candidates=C)
    pr.disable()
    dt = time.perf_counter() - t0
    print('ms/suggest under cProfile: %.3f' % (1e3 * dt / steps))
    st = pstats.Stats(pr)
    st.sort_stats('tottime').print_stats(35)
    st.sort_stats('cumulative').print_stats(30)


if __name__ == '__main__':
    main()
