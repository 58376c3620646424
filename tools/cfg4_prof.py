"""Where config 4's step goes outside the native call (VERDICT round 5, next
2: the per-rank Python the label axis leaves unsharded).  Runs bench.py's
config-4 step (4096 ids x 4096 candidates x 20 dims, columnar results) and
prints the step wall, the native call's host phases (tpe_host_phases) and a
cProfile of the Python by cumulative and own time.

  python tools/cfg4_prof.py [--steps 10] [--config 4|5]"""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--config', type=int, default=4)
    ap.add_argument('--dims', type=int, default=1000)
    ap.add_argument('--history5', type=int, default=100000)
    ap.add_argument('--appending', action='store_true')
    ap.add_argument('--axis4', default='labels')
    ap.add_argument('--warmup', type=int, default=2)
    args = ap.parse_args()
    from hyperopt_amd import _native as N
    from hyperopt_amd.engine import get_engine
    eng = get_engine(torch.device('cuda', 0))
    desc, step, _ = bench.config_workload(args.config, 0, 1, args)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    buf = (ctypes.c_double * len(N.PHASES))()
    eng.lib.tpe_host_phases(1, None, 0)
    walls, ph = [], []
    for i in range(args.steps):
        s0 = time.perf_counter()
        step(10 + i)
        walls.append(1e6 * (time.perf_counter() - s0))
        eng.lib.tpe_host_phases(1, buf, len(N.PHASES))
        ph.append(list(buf))
    eng.lib.tpe_host_phases(0, None, 0)
    med = np.median(np.array(ph), 0)
    w = float(np.median(walls))
    print('%s\nstep wall p50 %.1f us; native phases (us since entry) %s; outside the native call %.1f us'
          % (desc, w, dict(zip(N.PHASES, [round(float(x), 1) for x in med])), w - med[N.PHASES.index('return')]))
    pr = cProfile.Profile()
    pr.enable()
    for i in range(args.steps):
        step(100 + i)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats('cumulative').print_stats(30)
    st.sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
