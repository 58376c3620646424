"""cProfile of config 5's appending step (bench.py --config 5 --appending: one
evaluated suggestion appended to the 1000-label columnar history before every
suggest).  Usage: python tools/cfg5_app_prof.py [STEPS]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd.engine import get_engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    args = argparse.Namespace(dims=1000, history5=100000, appending=True, steps=n + 3, warmup=0)
    get_engine(torch.device('cuda', 0))
    _, step, _ = bench.config_workload(5, 0, 1, args)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    lat = []
    for i in range(n):
        pr.enable()
        t0 = time.perf_counter()
        step(10 + i)
        lat.append(time.perf_counter() - t0)
        pr.disable()
    print('config-5 appending step p50 %.2f ms (profiled)' % (1e3 * np.median(lat)))
    st = pstats.Stats(pr)
    rows = sorted(st.stats.items(), key=lambda kv: -kv[1][2])[:30]
    print('%8s %10s %10s  %s' % ('calls', 'own ms', 'cum ms', 'function (per step)'))
    for (f, line, name), (cc, nc, tt, ct, _) in rows:
        print('%8.1f %10.3f %10.3f  %s:%d(%s)' % (nc / n, 1e3 * tt / n, 1e3 * ct / n, os.path.basename(f), line, name))


if __name__ == '__main__':
    main()
