"""The Python around the native call of a batched suggest, on the CPU (no
GPU): config 4's or config 5's step (bench.config_workload) with
Engine.suggest_tree replaced by a stub that returns at once — what is left
is the per-rank host work a label / grid shard does not divide (history
view, below split, tree records, result columns).  Diagnostic only.

  python tools/py_overhead_cpu.py [--config 4|5] [--steps 50] [--appending]"""
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
from hyperopt_amd import _native as N, engine as E  # noqa: E402


class _StubEngine(E.Engine):
    def __init__(self):                      # (no device: the fields suggest() reads)
        self.lib = N.load()
        self.device = torch.device('cpu')
        self._dev_index = 0
        self.device_fit_min = E.DEVICE_FIT_MIN
        self.tree_calls = 0
        self.precision = 'fp32'
        self.profile = None
        self.expand = self.fuse = True
        self.last_tree_path = None

    def suggest_tree(self, labels, below_sorted, prior_weight, lf, ids, n_cand, seed, min_draws, flags=0,
                     shard=None, exchange=None, labels_ptr=None):
        n, nl = len(ids), len(labels)
        io = getattr(self, '_io', None)
        if io is None or io[0].shape != (n, nl):
            io = self._io = (np.zeros((n, nl)), np.ones((n, nl), dtype=np.int8))
        return io


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=4)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--dims', type=int, default=1000)
    ap.add_argument('--history5', type=int, default=100000)
    ap.add_argument('--appending', action='store_true')
    ap.add_argument('--warmup', type=int, default=2)
    args = ap.parse_args()
    args.axis4 = 'labels'
    eng = _StubEngine()
    E._ENGINES['cpu'] = eng
    E.get_engine = lambda device=None, precision='fp32': eng
    from hyperopt_amd import tpe
    tpe.get_engine = E.get_engine
    desc, step, _ = bench.config_workload(args.config, 0, 1, args)
    for i in range(3):
        step(i)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(10 + i)
    dt = (time.perf_counter() - t0) / args.steps
    print('%s\nPython around a stubbed native call: %.1f us per step' % (desc, 1e6 * dt))
    pr = cProfile.Profile()
    pr.enable()
    for i in range(args.steps):
        step(100 + i)
    pr.disable()
    pstats.Stats(pr).sort_stats('cumulative').print_stats(25)


if __name__ == '__main__':
    main()
