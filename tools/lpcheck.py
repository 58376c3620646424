import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import bench
from hyperopt_amd import history as H, tpe, _native as N
from hyperopt_amd.engine import LevelProblem, get_engine
eng = get_engine(torch.device('cuda', 0))
domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
hist = H.extract(domain, trials)
fits = tpe._Fits(domain.table, hist, H.split_below(hist, 0.25), 1.0, eng)
T = domain.table
for lab in ('svm_C', 'svm_rbf_gamma'):
    post = fits.get(T.by_label[lab])
    res = eng.run([LevelProblem(post, T.by_label[lab].index, [10000])], 1 << 20, 5)
    torch.cuda.synchronize()
    prob, _ = eng.device_tables()
    p = prob[0]
    tab = eng._bufs['tab'].view(torch.float32).cpu().numpy()
    off, n = int(p['tab_off'][0]), int(p['tab_n'][0])
    rows = tab[4 * off: 4 * (off + 3 * n)].reshape(n, 12)
    print(lab, 'flags', int(p['flags']), 'n', n, 'nan below', np.isnan(rows[:, 0]).mean(), 'nan above', np.isnan(rows[:, 6]).mean())
    print(' below first rows', rows[:3, :6], '\n above', rows[n//2:n//2+2, 6:])
    # timing
    eng.profile = {}
    for i in range(5): eng.run([LevelProblem(post, T.by_label[lab].index, [10000])], 1 << 20, 5)
    torch.cuda.synchronize()
    print(' stages', {k: np.mean([a[0] for a in v]) for k, v in eng.profile.items()})
    eng.profile = None
