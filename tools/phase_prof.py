"""Where one tpe.suggest of a workload spends its time: p50 wall, the native
call's host phases (tpe_host_phases: us since its entry) and the Python rest.
Run under `rocprofv3 --kernel-trace --stats` for the device kernels' times.
Usage: python tools/phase_prof.py WORKLOAD [STEPS]
WORKLOAD: svm (config 3 headline), rf (config 3 rf-steered: quantized labels),
cfg2 (config 2: 10-dim mixed space, 1k trials, C = 10^4), app (config 3 with one
evaluated document appended before every suggest, FMinIter's flow)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import _native as N, tpe  # noqa: E402
from hyperopt_amd.engine import get_engine  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else 'svm'
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    eng = get_engine(torch.device('cuda', 0))
    if wl == 'cfg2':
        domain, trials = bench.mixed10_history(1000, bench.SEED)
        new_id, C = 1000, 10000
    else:
        domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED,
                                            loss=bench.rf_loss if wl == 'rf' else None)
        new_id, C = bench.N_HISTORY, bench.C_PER_GPU
    buf = (ctypes.c_double * len(N.PHASES))()
    tid = new_id

    def one(i):
        nonlocal tid
        docs = tpe.suggest([tid], domain, trials, 1000 + i, n_EI_candidates=C)
        if wl == 'app':
            trials.insert_trial_docs(docs)
            trials.refresh()
            bench.evaluate(domain, trials, trials.trials[-1])
            tid += 1
        return docs
    for i in range(20):
        one(i)
    torch.cuda.synchronize()
    eng.lib.tpe_host_phases(1, None, 0)
    wall, ph = [], []
    for i in range(steps):
        t0 = time.perf_counter()
        docs = tpe.suggest([tid], domain, trials, 5000 + i, n_EI_candidates=C)
        wall.append(1e6 * (time.perf_counter() - t0))
        eng.lib.tpe_host_phases(1, buf, len(N.PHASES))
        ph.append(list(buf))
        if wl == 'app':
            trials.insert_trial_docs(docs)
            trials.refresh()
            bench.evaluate(domain, trials, trials.trials[-1])
            tid += 1
    eng.lib.tpe_host_phases(0, None, 0)
    med = np.median(np.array(ph), axis=0)
    print('%s: suggest p50 %.1f us  p10 %.1f  p90 %.1f' % (wl, np.median(wall), np.percentile(wall, 10),
                                                           np.percentile(wall, 90)))
    print('  native phases (median us since entry): ' +
          '  '.join('%s %.1f' % (k, v) for k, v in zip(N.PHASES, med)))
    print('  outside the native call (Python): %.1f us' % (np.median(wall) - med[N.PHASES.index('return')]))
    print('  active labels:', sorted(k for k, v in docs[0]['misc']['vals'].items() if v))


if __name__ == '__main__':
    main()
