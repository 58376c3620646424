"""Where the time of one native config-3 suggest (tpe_suggest_tree) goes:
the native fits of the four labels the svm/rbf branch needs, timed by calling
tpe_host_cat_split / tpe_host_fit_split directly; the packer alone; the whole
tpe_suggest_tree call; and the device stages of the same call (stage profiler).
Run on the GPU box: python tools/native_split.py [reps]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import _native as N, engine as E, history as H, tpe  # noqa: E402


def best_of(fn, reps=200, inner=10):
    b = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(inner):
            fn()
        b = min(b, (time.perf_counter() - t0) / inner)
    return 1e6 * b


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    eng = E.get_engine(torch.device('cuda', 0))
    lib = N.load()
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    hist = H.extract(domain, trials)
    table = domain.table
    below = np.sort(H.split_below(hist, 0.25)).astype(np.int64)
    arr, keep = tpe._tree_labels(table, hist)[:2]
    tot_fit = 0.0
    for lab in ('model', 'svm_kernel', 'svm_C', 'svm_rbf_gamma'):
        r = arr[table.by_label[lab].index]
        n = int(r['n_obs'])
        if r['family'] == N.FAM_CATEGORICAL:
            up = int(r['upper'])
            out = np.empty(2 * up)
            p = int(r['p_prior']) or None

            def f():
                lib.tpe_host_cat_split(int(r['values']), int(r['tids']), n, below.ctypes.data, len(below), up, p,
                                       1.0, 25, out.ctypes.data, out.ctypes.data + 8 * up)
        else:
            out = np.empty(6 * (n + 1))
            k = np.empty(2, dtype=np.int64)

            def f():
                lib.tpe_host_fit_split(int(r['values']), int(r['tids']), int(r['order']), n, below.ctypes.data,
                                       len(below), 1.0, float(r['prior_mu']), float(r['prior_sigma']), 25,
                                       out.ctypes.data, k.ctypes.data)
        t = best_of(f, reps)
        tot_fit += t
        print('  fit %-14s n_obs %6d  %7.1f us' % (lab, n, t))
    print('  fits total                     %7.1f us' % tot_fit)
    # the packer alone on the four labels' native fits (what tpe_suggest_tree packs)
    from hyperopt_amd.engine import LevelProblem
    fits = tpe._Fits(table, hist, H.split_below(hist, 0.25), 1.0, eng)
    probs = [LevelProblem(fits.get(table.by_label[l]), table.by_label[l].index, [bench.N_HISTORY])
             for l in ('model', 'svm_C', 'svm_kernel', 'svm_rbf_gamma')]
    labels_in, keep_in = eng._labels(probs)
    ids = np.array([bench.N_HISTORY], dtype=np.int64)
    C = bench.C_PER_GPU

    def sug():
        eng.suggest_tree(arr, below, 1.0, 25, ids, C, 5, tpe.SPECULATE_MIN_DRAWS)
    for _ in range(20):
        sug()
    torch.cuda.synchronize()
    lat = []
    for i in range(reps):
        t0 = time.perf_counter()
        sug()
        lat.append(time.perf_counter() - t0)
    print('  tpe_suggest_tree (Engine.suggest_tree)  p50 %7.1f us  min %7.1f us' %
          (1e6 * np.median(lat), 1e6 * np.min(lat)))
    # host phases of the same call (tpe_host_phases: us since the call's entry)
    ph = []
    buf = (ctypes.c_double * len(N.PHASES))()
    lib.tpe_host_phases(1, None, 0)
    for i in range(reps):
        sug()
        lib.tpe_host_phases(1, buf, len(N.PHASES))
        ph.append(list(buf))
    lib.tpe_host_phases(0, None, 0)
    med = np.median(np.array(ph), axis=0)
    print('  host phases (median us since entry): ' +
          '  '.join('%s %.1f' % (k, v) for k, v in zip(N.PHASES, med)))
    info = N.PackInfo()
    pin = eng._pinned
    if pin is not None:
        t = best_of(lambda: lib.tpe_host_pack_level(labels_in, len(probs), bench.C_PER_GPU, 5, 0, 0, 0,
                                                    pin.data_ptr(), pin.numel(), ctypes.byref(info)), reps)
        print('  tpe_host_pack_level (4 labels)  %7.1f us' % t)
    eng.profile = {}
    for _ in range(20):
        sug()
    prof = eng.profile
    eng.profile = None
    for k, v in prof.items():
        print('  device stage %-10s %7.1f us' % (k, 1e3 * np.median([a[0] for a in v])))
    if '--exchange' in sys.argv:
        exchange_overhead(eng, lib, arr, below, ids, C, reps, sug)


def exchange_overhead(eng, lib, arr, below, ids, C, reps, sug):
    """The candidate-shard exchange forced on a one-rank RCCL group (the
    device combine: run records reduced, all-gathered and combined on the
    device, one synchronise per level) against the plain call, alternating."""
    import torch.distributed as dist
    from hyperopt_amd import dist as D
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29533')
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    ex = D.exchange_for(eng, always=True)

    def sug_x():
        eng.suggest_tree(arr, below, 1.0, 25, ids, C, 5, tpe.SPECULATE_MIN_DRAWS, shard=(0, 1), exchange=ex)
    for _ in range(20):
        sug_x()
    a, b = [], []
    for i in range(reps):
        t0 = time.perf_counter()
        sug()
        a.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        sug_x()
        b.append(time.perf_counter() - t0)
    mode = 'host' if os.environ.get('TPE_DEVICE_COMBINE', '1') == '0' else 'device'
    print('  exchange forced (RCCL, world 1, %s combine): p50 %7.1f us vs plain %7.1f us: +%.1f us'
          % (mode, 1e6 * np.median(b), 1e6 * np.median(a), 1e6 * (np.median(b) - np.median(a))))
    # RCCL's own latency: one small in-place all-gather on the stream, synchronised
    t = torch.zeros(256, dtype=torch.uint8, device='cuda')
    out = torch.empty(256, dtype=torch.uint8, device='cuda')
    lat = []
    for i in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dist.all_gather_into_tensor(out, t)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    print('  torch.distributed all_gather_into_tensor (256 B, world 1, synchronised): p50 %.1f us' %
          (1e6 * np.median(lat)))
    ph = []
    buf = (ctypes.c_double * len(N.PHASES))()
    lib.tpe_host_phases(1, None, 0)
    for i in range(reps):
        sug_x()
        lib.tpe_host_phases(1, buf, len(N.PHASES))
        ph.append(list(buf))
    lib.tpe_host_phases(0, None, 0)
    med = np.median(np.array(ph), axis=0)
    print('  exchange host phases (median us since entry): ' +
          '  '.join('%s %.1f' % (k, v) for k, v in zip(N.PHASES, med)))
    ex.close()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
