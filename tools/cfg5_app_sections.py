"""Where config 5's appended step spends its time outside the native call:
bench.py's --config 5 --appending step with light perf_counter wrappers
around the Python functions on its path (median per step over --steps).
Diagnostic only.  python tools/cfg5_app_sections.py [--steps 30]"""
import argparse
import collections
import functools
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import devhist, engine as E, history, tpe  # noqa: E402

ACC = collections.defaultdict(float)


def wrap(obj, name, key=None):
    f = getattr(obj, name)
    key = key or '%s.%s' % (getattr(obj, '__name__', type(obj).__name__), name)

    @functools.wraps(f)
    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            ACC[key] += time.perf_counter() - t0
    setattr(obj, name, g)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=30)
    args = ap.parse_args()
    ns = argparse.Namespace(dims=1000, history5=100000, steps=args.steps + 5, warmup=2, appending=True, axis4='labels')
    E.get_engine(torch.device('cuda', 0))
    for obj, name in ((tpe, '_tree_labels'), (tpe, '_native_tree'), (tpe, '_suggest_local'), (E.Engine, 'suggest_tree'),
                      (devhist.DeviceColumns, 'upload_rows'), (devhist._Orders, 'ptrs_many'),
                      (devhist._Orders, 'commit_many'), (history, 'split_below'), (history.History, '__init__'),
                      (tpe, '_result_dicts'), (devhist.DeviceColumns, '_scatter'), (devhist._Staging, 'get'),
                      (devhist._Staging, 'used'), (devhist, '_positions'), (devhist.DeviceColumns, 'upload'),
                      (devhist.DeviceColumns, 'addresses'), (tpe, '_tree_groups'), (tpe, '_tree_static')):
        if hasattr(obj, name):
            wrap(obj, name)
    desc, step, _ = bench.config_workload(5, 0, 1, ns)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    rows = []
    for i in range(args.steps):
        ACC.clear()
        t0 = time.perf_counter()
        step(100 + i)
        wall = time.perf_counter() - t0
        r = dict(ACC)
        r['step'] = wall
        rows.append(r)
    keys = sorted(set(k for r in rows for k in r))
    print(desc)
    for k in keys:
        print('%-34s median %8.1f us' % (k, 1e6 * float(np.median([r.get(k, 0.0) for r in rows]))))


if __name__ == '__main__':
    main()
