"""Measured per-rank work of the sharded batched suggests (VERDICT round 5,
next 2), on ONE GPU: for each axis and rank count N, the part of config 4's
or config 5's step that the most loaded rank runs — its labels
(TPE_F_REMOTE for the others) for its block of ids, exactly the
``_suggest_local`` call ``tpe._suggest_sharded`` makes on that rank — timed
end to end (Python, fits, pack, device, results), p50 over ``--steps``.  The
one thing not measured is the all-gather of the chosen values (no multi-GPU
box): modelled as (N - 1) ring hops of ``--hop-us`` plus the gathered bytes
at ``--bw-gbs``, both ASSUMED.  Prints T1, each (axis, N) rank time, T(N)
and the efficiency T1 / (N * T(N)); ``--json`` writes them.

  python tools/rank_share.py [--config 4|5] [--steps 10] [--json out.json]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


PH = {}


def timed(fn, steps, key=None):
    """(p50, mean) wall of fn over steps; the median native host phases
    (tpe_host_phases) kept under PH[key]."""
    import ctypes
    from hyperopt_amd import _native as N
    from hyperopt_amd.engine import get_engine
    lib = get_engine().lib
    for i in range(2):
        fn(i)
    torch.cuda.synchronize()
    w, ph = [], []
    buf = (ctypes.c_double * len(N.PHASES))()
    lib.tpe_host_phases(1, None, 0)
    for i in range(steps):
        s0 = time.perf_counter()
        fn(100 + i)
        w.append(1e6 * (time.perf_counter() - s0))
        lib.tpe_host_phases(1, buf, len(N.PHASES))
        ph.append(list(buf))
    lib.tpe_host_phases(0, None, 0)
    if key is not None:
        PH[key] = dict(zip(N.PHASES, [round(float(x), 1) for x in np.median(np.array(ph), 0)]))
    return float(np.median(w)), float(np.mean(w))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=4)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--hop-us', type=float, default=3.0)
    ap.add_argument('--bw-gbs', type=float, default=50.0)
    ap.add_argument('--json', default=None)
    ap.add_argument('--only-n', type=int, default=0, help='one rank count only (and no unsharded run)')
    args = ap.parse_args()
    from hyperopt_amd import dist as D, tpe
    from hyperopt_amd.engine import get_engine
    get_engine(torch.device('cuda', 0))
    if args.config == 4:
        labels = ['x%02d' % i for i in range(20)]
        hist = bench.soa_history(labels, 10000, bench.SEED, lambda v: sum((x - 0.3) ** 2 for x in v.values()))
        table = bench.flat_uniform_table(labels)
        ids = np.arange(10000, 10000 + 4096)
        C = 4096
    else:
        labels = ['x%04d' % i for i in range(1000)]
        N5 = 100000
        hist = bench.soa_history(labels, N5, bench.SEED, lambda v: np.zeros(N5))
        hist.losses[:] = np.random.RandomState(bench.SEED + 1).uniform(size=N5) + 1e-9 * np.arange(N5)
        table = bench.flat_uniform_table(labels)
        ids = np.array([N5])
        C = 4096
    L, n = len(table.rows), len(ids)

    def local(ids_blk, remote):
        def f(i):
            tpe._suggest_local(table, hist, ids_blk, bench.SEED + i, 1.0, C, 0.25, 'philox', 'fp32', None, None,
                               True, remote)
        return f

    t1, t1m = timed(local(ids, ()), args.steps, 'unsharded') if not args.only_n else (float('nan'), float('nan'))
    rows = [dict(axis='unsharded', N=1, shape=[1, 1], rank_us=t1, rank_mean_us=t1m, x_us=0.0, T_us=t1, eff=1.0,
                 phases_us=PH.get('unsharded'))]
    axes = [('labels', None), ('ids', None), ('grid', None)] if args.config == 4 else [('labels', None)]
    if args.config == 4:
        axes += [('grid', 2), ('grid', 4)]
    for N in (args.only_n,) if args.only_n else (2, 4, 8):
        for axis, G in axes:
            if axis == 'labels':
                shape = (N, 1)
            elif axis == 'ids':
                shape = (1, N)
            elif G is None:
                shape = D.grid_shape(L, n, N, D.label_cost(len(hist), C))
            else:
                if N % G or G == N or G == 1:
                    continue
                shape = (G, N // G)
            owner = D.label_owners(table, shape[0])
            # the most loaded rank: label group 0 (round-robin: the first groups
            # hold the extra labels), id block 0 (shard_range: the larger blocks last)
            g, b = 0, shape[1] - 1
            remote = tuple(ix for ix, o in enumerate(owner) if o >= 0 and o != g)
            lo, hi = D.shard_range(n, b, shape[1])
            name = axis if G is None else 'grid %dx%d' % shape
            t, tm = timed(local(ids[lo:hi], remote), args.steps, (name, N))
            blk = max(hi2 - lo2 for lo2, hi2 in (D.shard_range(n, bb, shape[1]) for bb in range(shape[1])))
            if shape[1] == 1:                           # (the label axis: each rank's columns, padded)
                nbytes = n * max(owner.count(o) for o in range(shape[0])) * 8 * N
            else:                                       # (a block's rows: values and activity)
                nbytes = blk * L * 9 * N
            x = args.hop_us * (N - 1) + nbytes * (N - 1) / N / (args.bw_gbs * 1e3)
            T = t + x
            rows.append(dict(axis=name, N=N, shape=list(shape), rank_us=t, rank_mean_us=tm, x_us=x, T_us=T,
                             eff=t1 / (N * T), phases_us=PH.get((name, N))))
    print('config %d: T1 (unsharded suggest, p50) %.1f us; all-gather modelled: %.1f us a hop, %.0f GB/s (ASSUMED)'
          % (args.config, t1, args.hop_us, args.bw_gbs))
    print('%-10s %3s %8s %10s %8s %10s %6s' % ('axis', 'N', 'G x B', 'rank us', 'x us', 'T(N) us', 'eff'))
    for r in rows:
        print('%-10s %3d %8s %10.1f %8.1f %10.1f %6.2f   %s' % (r['axis'], r['N'], '%dx%d' % tuple(r['shape']),
                                                                  r['rank_us'], r['x_us'], r['T_us'], r['eff'],
                                                                  r['phases_us']))
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(dict(config=args.config, T1_us=t1, hop_us=args.hop_us, bw_gbs=args.bw_gbs, rows=rows), f)


if __name__ == '__main__':
    main()
