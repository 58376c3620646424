#!/usr/bin/env python3
"""Time the CPU oracle against the reference itself (build container only).

bench.py's cpu_baseline times ``oracle/tpe_oracle.py`` (kind "port") on the GPU
box's host, where the reference cannot run.  This script checks, here, that
the port is a faithful stand-in for the reference's speed: both run the same
``tpe.suggest`` calls (same history, seed and n_EI_candidates, one thread),
the outputs are compared for equality, and the wall times are recorded in
profiles/r02_oracle_vs_reference.json (tests/test_oracle_golden.py asserts the
ratio stays within +-15 %).

Usage:  oracle/make_refpy3.sh && python tools/oracle_vs_reference.py
"""
import json
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, '..')
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import gen_golden as G  # noqa: E402  (imports the reference from /tmp/refpy3)
from oracle import tpe_oracle as O  # noqa: E402
from oracle.spacedesc import params_from_desc  # noqa: E402

# (space, history size, n_EI_candidates, seeds): config 2 (10-dim mixed, 1k
# history, 10k candidates) and bench.py's cpu_baseline sample (the config-3
# tree, 10k history, C = 16384)
WORKLOADS = [('mixed10', 1000, 10000, [101, 102, 103]), ('tree', 10000, 16384, [201, 202, 203])]


def main():
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)
    except Exception:  # pragma: no cover
        pass
    out = dict(host=platform.processor() or platform.machine(), python=platform.python_version(),
               numpy=np.__version__, generator='tools/oracle_vs_reference.py', runs=[])
    for name, n, C, seeds in WORKLOADS:
        domain, trials = G.make_history(G.SPACES[name], n, seed=7 + n)
        hist = G.history_to_json(trials)
        params = params_from_desc(G.SPACES[name])
        t_ref, t_orc, same = [], [], True
        for s in seeds:
            t0 = time.perf_counter()
            docs = G.tpe.suggest([n], domain, trials, s, n_EI_candidates=C)
            t_ref.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            mine = O.tpe_suggest(params, hist, s, n_EI_candidates=C)
            t_orc.append(time.perf_counter() - t0)
            want = G.doc_vals(docs)
            same = same and set(want) == set(mine) and all(float(want[k]) == float(mine[k]) for k in want)
        r = dict(space=name, history=n, n_EI_candidates=C, seeds=seeds, reference_s=t_ref, oracle_s=t_orc,
                 ratio=float(np.median(t_orc) / np.median(t_ref)), identical_outputs=bool(same))
        print(json.dumps(r))
        out['runs'].append(r)
    with open(os.path.join(ROOT, 'profiles', 'r02_oracle_vs_reference.json'), 'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
