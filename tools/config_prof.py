"""cProfile of one BASELINE config's step (bench.config_workload) on the device."""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('config', type=int)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--dims', type=int, default=1000)
    ap.add_argument('--history5', type=int, default=100000)
    args = ap.parse_args()
    from hyperopt_amd.engine import get_engine
    get_engine(torch.device('cuda', 0))
    desc, step, _ = bench.config_workload(args.config, 0, 1, args)
    step(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(1 + i)
    torch.cuda.synchronize()
    print('%s: %.2f ms per step' % (desc, 1e3 * (time.perf_counter() - t0) / args.steps))
    pr = cProfile.Profile()
    pr.enable()
    for i in range(args.steps):
        step(100 + i)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
