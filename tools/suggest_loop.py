"""The headline tpe.suggest in a loop (no bench bookkeeping): a clean target
for rocprofv3 API / kernel / copy traces (tools/api_timeline.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import torch  # noqa: E402,F401

import bench  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    for i in range(n):
        tpe.suggest([bench.N_HISTORY], domain, trials, 100 + i, n_EI_candidates=bench.C_PER_GPU)
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
