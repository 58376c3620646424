import ctypes, os, sys, time
sys.path.insert(0, '/root/repo')
import numpy as np, torch
import bench
from hyperopt_amd import _native as N, dist as D, tpe
from hyperopt_amd.engine import get_engine
eng = get_engine(torch.device('cuda', 0))
labels = ['x%02d' % i for i in range(20)]
hist = bench.soa_history(labels, 10000, bench.SEED, lambda v: sum((x - 0.3) ** 2 for x in v.values()))
table = bench.flat_uniform_table(labels)
ids = np.arange(10000, 10000 + 4096)
for N8, tag in ((1, 'unsharded'), (8, 'labels8')):
    owner = D.label_owners(table, N8)
    remote = tuple(ix for ix, o in enumerate(owner) if o >= 0 and o != 0)
    for i in range(3):
        tpe._suggest_local(table, hist, ids, i, 1.0, 4096, 0.25, 'philox', 'fp32', None, None, True, remote)
    torch.cuda.synchronize()
    eng.lib.tpe_host_phases(1, None, 0)
    sys.stderr.write('=== %s\n' % tag)
    for i in range(3):
        tpe._suggest_local(table, hist, ids, 10 + i, 1.0, 4096, 0.25, 'philox', 'fp32', None, None, True, remote)
    eng.lib.tpe_host_phases(0, None, 0)
