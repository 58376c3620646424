"""cProfile of the headline tpe.suggest on the real device (host-side Python
and native-call costs; the profiler inflates per-call overheads)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import torch  # noqa: E402,F401

import bench  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    for i in range(10):
        tpe.suggest([bench.N_HISTORY], domain, trials, i, n_EI_candidates=bench.C_PER_GPU)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(n):
        tpe.suggest([bench.N_HISTORY], domain, trials, 100 + i, n_EI_candidates=bench.C_PER_GPU)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats('tottime').print_stats(35)


if __name__ == '__main__':
    main()
