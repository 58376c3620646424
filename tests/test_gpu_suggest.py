"""End-to-end GPU tests of tpe.suggest / fmin against the reference.

Replay mode (the reference's RandomState candidate draws, float64 scoring on
the GPU) must reproduce the reference's suggestions and whole fmin
trajectories exactly; the default Philox mode is checked for determinism,
batching semantics and optimisation quality.
"""
import functools

import numpy as np
import pytest

from oracle.spacedesc import params_from_desc, synthetic_loss
from tests.helpers import amd_space, trials_from_history, doc_values

pytestmark = pytest.mark.gpu


def _domain(desc):
    from hyperopt_amd import base
    return base.Domain(lambda x: 0.0, amd_space(desc))


def test_replay_suggest_matches_reference(golden):
    from hyperopt_amd import tpe
    g = golden('suggest_vectors.json')
    for case in g['cases']:
        if case.get('kind') == 'rand':
            continue
        d = _domain(g['spaces'][case['space']])
        trials = trials_from_history(case['history'], d)
        docs = tpe.suggest_replay([case['n']], d, trials, case['seed'],
                                  n_EI_candidates=case['n_EI_candidates'])
        got = doc_values(docs)
        want = case['result']
        assert set(got) == set(want), (case['space'], case['seed'])
        for k in want:
            assert float(got[k]) == float(want[k]), (case['space'], case['seed'], k, got[k], want[k])
        trials.assert_valid_trial(docs[0])


def test_fmin_config1_trajectories_exact(golden):
    """Config 1: fmin(tpe.suggest) on hp.uniform('x',-10,10), (x-3)^2, 100
    evals, seeds 0..9 — identical x and loss sequences to the reference."""
    from hyperopt_amd import fmin, hp, tpe, Trials
    g = golden('fmin_traj.json')
    for run in g['runs']:
        if run['space'] != 'u1':
            continue
        t = Trials()
        fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -10, 10), algo=tpe.suggest_replay,
             max_evals=run['max_evals'], trials=t, rstate=np.random.RandomState(run['seed']))
        assert [float(d['misc']['vals']['x'][0]) for d in t.trials] == run['x'], run['seed']
        assert [float(d['result']['loss']) for d in t.trials] == run['loss']


def test_fmin_conditional_trajectories_exact(golden):
    from hyperopt_amd import fmin, tpe, Trials
    g = golden('fmin_traj.json')
    for run in g['runs']:
        if run['space'] == 'u1':
            continue
        t = Trials()

        def objective(_cfg, _t=t):
            d = _t._dynamic_trials[-1]
            vals = {k: (v[0] if v else None) for k, v in d['misc']['vals'].items()}
            return synthetic_loss(vals, d['tid'])
        fmin(objective, amd_space(g['spaces'][run['space']]), algo=tpe.suggest_replay,
             max_evals=run['max_evals'], trials=t, rstate=np.random.RandomState(run['seed']))
        got = [{k: float(v[0]) for k, v in d['misc']['vals'].items() if v} for d in t.trials]
        want = [{k: float(v) for k, v in d.items()} for d in run['vals']]
        assert got == want, run['space']


def test_philox_batched_equals_single(golden):
    from hyperopt_amd import tpe
    g = golden('suggest_vectors.json')
    case = [c for c in g['cases'] if c['space'] == 'tree' and c.get('kind') != 'rand'][-1]
    d = _domain(g['spaces']['tree'])
    trials = trials_from_history(case['history'], d)
    ids = list(range(case['n'], case['n'] + 12))
    batch = tpe.suggest(ids, d, trials, 77, n_EI_candidates=512)
    assert [doc['tid'] for doc in batch] == ids
    for j, new_id in enumerate(ids):
        single = tpe.suggest([new_id], d, trials, 77, n_EI_candidates=512)
        assert doc_values(single) == doc_values([batch[j]])
        trials.assert_valid_trial(batch[j])
    again = tpe.suggest(ids, d, trials, 77, n_EI_candidates=512)
    assert [doc_values([a]) for a in again] == [doc_values([b]) for b in batch]


def test_philox_suggest_respects_space(golden):
    from hyperopt_amd import tpe
    g = golden('suggest_vectors.json')
    for case in g['cases']:
        if case.get('kind') == 'rand':
            continue
        params = {p['label']: p for p in params_from_desc(g['spaces'][case['space']])}
        d = _domain(g['spaces'][case['space']])
        trials = trials_from_history(case['history'], d)
        for precision in ('fp32', 'fp64'):
            docs = tpe.suggest([case['n'], case['n'] + 1], d, trials, case['seed'],
                               n_EI_candidates=case['n_EI_candidates'], precision=precision)
            for doc in docs:
                vals = doc_values([doc])
                for k, v in vals.items():
                    p = params[k]
                    a = p['args']
                    if p['dist'] in ('randint', 'categorical'):
                        assert isinstance(v, np.integer) and 0 <= v < a['upper']
                    elif p['dist'] in ('uniform',):
                        assert a['low'] <= v < a['high']
                    elif p['dist'] == 'loguniform':
                        assert np.exp(a['low']) <= v <= np.exp(a['high'])
                    if 'q' in a:
                        assert abs(np.round(v / a['q']) * a['q'] - v) == 0
                # conditional activity is consistent with the chosen parents
                for k, p in params.items():
                    if p['parent'] is not None:
                        pl, pv = p['parent']
                        assert (k in vals) == (pl in vals and int(vals[pl]) == pv), (k, vals)


def test_philox_fmin_quality():
    """fmin with the default device sampler optimises config 1 as well as the
    reference does (reference best losses at seeds 0-2: 9.5e-4, 3.2e-5, 2.7e-4)."""
    from hyperopt_amd import fmin, hp, tpe, Trials
    best = []
    for s in range(5):
        t = Trials()
        fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -10, 10), algo=tpe.suggest, max_evals=100,
             trials=t, rstate=np.random.RandomState(s))
        best.append(min(t.losses()))
    assert np.median(best) < 1e-2, best


def test_partial_kwargs_and_startup():
    from hyperopt_amd import fmin, hp, tpe, Trials
    algo = functools.partial(tpe.suggest, n_EI_candidates=4096, n_startup_jobs=5, gamma=0.3)
    t = Trials()
    argmin = fmin(lambda d: (d['a'] - 1) ** 2 + d['b'], {'a': hp.uniform('a', -3, 3), 'b': hp.randint('b', 4)},
                  algo=algo, max_evals=40, trials=t, rstate=np.random.RandomState(0))
    assert len(t) == 40 and set(argmin) == {'a', 'b'}


def _tree_history(n, seed=0):
    """bench.py's config-3 tree space with an n-trial synthetic history."""
    import bench
    return bench.make_history(n, seed)


def test_fused_levels_match_level_by_level():
    """Speculative level fusion (one device batch for every tree level, gates
    verified afterwards) chooses what the level-by-level evaluation chooses:
    exactly at fp64 (unpruned, no near-tie flips), gates exactly at fp32."""
    from hyperopt_amd import tpe
    domain, trials = _tree_history(3000)
    C = 1 << 16
    for precision in ('fp64', 'fp32'):
        for seed in (3, 4):
            fused = doc_values(tpe.suggest([3000], domain, trials, seed, n_EI_candidates=C, precision=precision))
            tpe.SPECULATE = False
            try:
                seq = doc_values(tpe.suggest([3000], domain, trials, seed, n_EI_candidates=C, precision=precision))
            finally:
                tpe.SPECULATE = True
            assert set(fused) == set(seq), (fused, seq)
            for k in seq:
                if precision == 'fp64' or k in domain.table.parent_labels:
                    assert fused[k] == seq[k], (precision, seed, k, fused[k], seq[k])


def test_fused_levels_misprediction_falls_back():
    """A wrong gate prediction is detected on the device results and the
    suggest falls back to level-by-level evaluation."""
    from hyperopt_amd import history as H, tpe
    from hyperopt_amd.engine import get_engine
    domain, trials = _tree_history(3000)
    hist = H.extract(domain, trials)
    eng = get_engine()
    fits = tpe._Fits(domain.table, hist, H.split_below(hist, 0.25), 1.0, eng)
    pred = tpe._predict_activity(domain.table, fits, 1 << 16)
    assert pred is not None and pred['model'] >= 0
    good = tpe._choices_fused(domain.table, fits, [3000], 5, 1 << 16, eng, None)
    assert good is not None and int(good[0]['model']) == pred['model']
    wrong = dict(pred)
    wrong['model'] = (pred['model'] + 1) % 3
    orig = tpe._predict_activity
    tpe._predict_activity = lambda *a: wrong
    try:
        assert tpe._choices_fused(domain.table, fits, [3000], 5, 1 << 16, eng, None) is None
        got = tpe._choices_philox(domain.table, fits, [3000], 5, 1 << 16, eng, None)
    finally:
        tpe._predict_activity = orig
    tpe.SPECULATE = False
    try:
        ref = tpe._choices_philox(domain.table, fits, [3000], 5, 1 << 16, eng, None)
    finally:
        tpe.SPECULATE = True
    assert got == ref


def _resume_space():
    from hyperopt_amd import hp
    return {'x': hp.uniform('x', -5, 5), 'q': hp.quniform('q', 0, 10, 1),
            'c': hp.choice('c', [0, {'y': hp.loguniform('y', -2, 1)}])}


def _resume_obj(d):
    return (d['x'] - 1) ** 2 + 0.05 * abs(d['q'] - 4) + (0.1 if d['c'] == 0 else float(d['c']['y']))


def test_fmin_resume_through_tpe_matches_uninterrupted():
    """Checkpoint / resume through TPE (fmin.py:147-175): 30 evals, pickle,
    reload (the SoA history cache is rebuilt from the documents), 30 more with
    the same RandomState stream == one uninterrupted 60-eval run — replay mode
    (reference-exact) and the default Philox device sampler (deterministic)."""
    import pickle
    from hyperopt_amd import fmin, tpe, Trials
    for algo in (tpe.suggest_replay, functools.partial(tpe.suggest, n_EI_candidates=4096)):
        rs = np.random.RandomState(21)
        t = Trials()
        fmin(_resume_obj, _resume_space(), algo=algo, max_evals=30, trials=t, rstate=rs)
        t2 = pickle.loads(pickle.dumps(t))
        fmin(_resume_obj, _resume_space(), algo=algo, max_evals=60, trials=t2, rstate=rs)
        ref = Trials()
        fmin(_resume_obj, _resume_space(), algo=algo, max_evals=60, trials=ref, rstate=np.random.RandomState(21))
        got = [d['misc']['vals'] for d in t2.trials]
        want = [d['misc']['vals'] for d in ref.trials]
        assert got == want and t2.losses() == ref.losses(), algo


def test_fmin_path_resumes_through_tpe(tmp_path, monkeypatch):
    """fmin_path: 25 evaluations (20 start-up + 5 TPE), dump, reload, 10 more
    TPE evaluations; the first 25 documents survive unchanged."""
    import importlib
    F = importlib.import_module('hyperopt_amd.fmin')
    monkeypatch.setenv('HYPEROPT_FMIN_SEED', '7')
    path = str(tmp_path / 'trials.pkl')
    t1 = F.fmin_path(_resume_obj, _resume_space(), 25, path)
    first = [d['misc']['vals'] for d in t1.trials]
    t2 = F.fmin_path(_resume_obj, _resume_space(), 10, path)
    assert len(t2) == 35 and [d['misc']['vals'] for d in t2.trials][:25] == first
    assert [d['tid'] for d in t2.trials] == list(range(35))
    for d in t2.trials:
        t2.assert_valid_trial(d)
