"""cProfile of the headline suggest in bench.py's appending (FMinIter) loop:
one evaluated document inserted and trials.refresh() before every suggest; only
the suggest itself is profiled.  Usage: python tools/append_prof.py [N]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import tpe  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    tid = bench.N_HISTORY
    pr = cProfile.Profile()
    lat = []
    for i in range(n + 5):
        on = i >= 5
        if on:
            pr.enable()
        s0 = time.perf_counter()
        docs = tpe.suggest([tid], domain, trials, bench.SEED + 20000 + i, n_EI_candidates=bench.C_PER_GPU)
        dt = time.perf_counter() - s0
        if on:
            pr.disable()
            lat.append(dt)
        trials.insert_trial_docs(docs)
        trials.refresh()
        bench.evaluate(domain, trials, trials.trials[-1])      # (as FMinIter stores the result)
        tid += 1
    torch.cuda.synchronize()
    print('appending suggest p50 %.1f us (profiled)' % (1e6 * np.median(lat)))
    st = pstats.Stats(pr)
    rows = sorted(st.stats.items(), key=lambda kv: -kv[1][2])[:30]
    print('%8s %10s %10s  %s' % ('calls', 'own us', 'cum us', 'function (per suggest)'))
    for (f, line, name), (cc, nc, tt, ct, _) in rows:
        print('%8.1f %10.2f %10.2f  %s:%d(%s)' % (nc / len(lat), 1e6 * tt / len(lat), 1e6 * ct / len(lat),
                                                  os.path.basename(f), line, name))


if __name__ == '__main__':
    main()
