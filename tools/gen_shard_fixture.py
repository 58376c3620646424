#!/usr/bin/env python3
"""Record real engine outputs for the CPU combine test (tests/test_dist.py):
the config-3 tree's fused level (4 labels, 3000-trial history) run unsharded
and as two candidate shards (tpe_level_run over [0, C/2) and [C/2, C) with the
global counter base).  Run on the GPU box:
    python tools/gen_shard_fixture.py gpurun_out/shard_results.json
then copy the file to tests/golden/."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
from hyperopt_amd import dist as D, history as H, tpe  # noqa: E402
from hyperopt_amd.engine import LevelProblem, get_engine  # noqa: E402

FIELDS = ('score', 'l', 'g', 'value', 'idx', 'global_idx')


def rec(res):
    return {f: [float(x) if f not in ('idx', 'global_idx') else int(x) for x in res[f]] for f in FIELDS}


def main(path):
    eng = get_engine()
    domain, trials = bench.make_history(3000, 0)
    hist = H.extract(domain, trials)
    fits = tpe._Fits(domain.table, hist, H.split_below(hist, 0.25), 1.0, eng)
    T = domain.table
    cases = []
    for C, seed in ((1 << 16, 21), (1 << 18, 22), (12345, 23)):
        labels = ['model', 'svm_C', 'svm_kernel', 'svm_rbf_gamma']
        probs = [LevelProblem(fits.get(T.by_label[l]), T.by_label[l].index, [3000]) for l in labels]
        full = eng.run_level(probs, C, seed)
        shards = []
        for r in range(2):
            lo, hi = D.shard_range(C, r, 2)
            shards.append(eng.run_level(probs, hi - lo, seed, cand_base=lo, n_cand_global=C))
        comb = D.combine_results(np.stack(shards))
        assert np.array_equal(comb['global_idx'], full['global_idx']), (C, seed)
        cases.append(dict(C=C, seed=seed, labels=labels, full=rec(full), shards=[rec(s) for s in shards]))
    with open(path, 'w') as f:
        json.dump({'generator': 'tools/gen_shard_fixture.py (engine outputs on an MI355X)', 'data': cases}, f)
    print('wrote', path)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/shard_results.json')
