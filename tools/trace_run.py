"""Runs headline suggests on the library named by TPE_HIP_LIB (a build with
TPE_SAMPLE_TRACE / TPE_TABLES_TRACE: per-workgroup phase times printed by the
kernels) — the last suggest's lines are the steady state."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    for i in range(n):
        print('=== suggest %d' % i, flush=True)
        tpe.suggest([bench.N_HISTORY], domain, trials, 100 + i, n_EI_candidates=bench.C_PER_GPU)
        torch.cuda.synchronize()


if __name__ == '__main__':
    main()
