"""Steady-state per-stage device time of the headline suggest's levels: every
stage re-issued back to back (Engine.profile_repeat), HIP events on the
launch stream.  Prints one line per (level, stage)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import history as H, tpe  # noqa: E402
from hyperopt_amd.engine import LevelProblem, get_engine  # noqa: E402


def main():
    rep = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    eng = get_engine(torch.device('cuda', 0))
    eng.fuse = os.environ.get('TPE_NO_FUSE') is None
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    hist = H.extract(domain, trials)
    fits = tpe._Fits(domain.table, hist, H.split_below(hist, 0.25), 1.0, eng)
    T = domain.table
    for lv in (['model'], ['svm_C', 'svm_kernel'], ['svm_rbf_gamma'], ['svm_C'], ['svm_C', 'svm_kernel', 'svm_rbf_gamma', 'model']):
        probs = [LevelProblem(fits.get(T.by_label[l]), T.by_label[l].index, [bench.N_HISTORY]) for l in lv]
        eng.run(probs, bench.C_PER_GPU, 5)
        eng.profile, eng.profile_repeat = {}, rep
        eng.run(probs, bench.C_PER_GPU, 5)
        torch.cuda.synchronize()
        for k, v in eng.profile.items():
            extra = ''
            if k == 'k_above_f32':
                a = v[0]
                extra = '  algorithmic CE %.3g, exact CE %.3g, expanded components %.3g' % (a[1], a[2], a[3])
                ce = eng.last_ce[:, 0].astype(np.float64)
                extra += '; exact CE per work item: mean %.3g p99 %.3g max %.3g (%d items)' % (
                    ce.mean(), np.percentile(ce, 99), ce.max(), len(ce))
                os.makedirs('gpurun_out', exist_ok=True)
                np.save('gpurun_out/ce_%s.npy' % '+'.join(lv), eng.last_ce)
            print('%-28s %-16s %8.1f us%s' % ('+'.join(lv), k, 1e3 * float(np.mean([a[0] for a in v])), extra))
        eng.profile, eng.profile_repeat = None, 1


if __name__ == '__main__':
    main()
