"""Checkpoint / resume (reference fmin.py:147-175) and the Trials SoA cache.

``fmin_path`` unpickles a ``Trials`` when the file exists (any unreadable file
starts fresh, as the reference's bare ``except``), runs ``max_evals`` more
evaluations with TPE and dumps the trials again.  ``Trials`` pickles without
its SoA history cache (history.py), which is rebuilt from the documents after
a reload.  These CPU tests stay inside the start-up phase (rand.suggest), so
no device is needed; tests/test_gpu_suggest.py resumes through TPE itself.
"""
import importlib
import pickle

import numpy as np

from hyperopt_amd import base, history as H, hp, rand

F = importlib.import_module("hyperopt_amd.fmin")      # the package exports the fmin function under that name


def _space():
    return {'x': hp.uniform('x', -5, 5), 'c': hp.choice('c', [0, {'y': hp.loguniform('y', -2, 1)}])}


def _obj(d):
    return (d['x'] - 1) ** 2 + (0.1 if d['c'] == 0 else float(d['c']['y']))


def _hist_equal(a, b):
    np.testing.assert_array_equal(a.tids, b.tids)
    np.testing.assert_array_equal(a.losses, b.losses)
    assert set(a.obs) == set(b.obs)
    for k in a.obs:
        np.testing.assert_array_equal(a.obs[k][0], b.obs[k][0])
        np.testing.assert_array_equal(a.obs[k][1], b.obs[k][1])


def _vals(trials):
    return [{k: v for k, v in d['misc']['vals'].items()} for d in trials.trials]


def test_fmin_path_resumes_and_appends(tmp_path, monkeypatch):
    monkeypatch.setenv('HYPEROPT_FMIN_SEED', '3')
    path = str(tmp_path / 'trials.pkl')
    t1 = F.fmin_path(_obj, _space(), 8, path)
    assert len(t1) == 8
    first = _vals(t1)
    t2 = F.fmin_path(_obj, _space(), 6, path)          # loads the 8, runs 6 more, dumps 14
    assert len(t2) == 14 and _vals(t2)[:8] == first
    assert [d['tid'] for d in t2.trials] == list(range(14))
    with open(path, 'rb') as f:
        t3 = pickle.load(f)
    assert _vals(t3) == _vals(t2)
    assert all(d['state'] == base.JOB_STATE_DONE for d in t3.trials)


def test_fmin_path_unreadable_file_starts_fresh(tmp_path, monkeypatch):
    monkeypatch.setenv('HYPEROPT_FMIN_SEED', '4')
    path = tmp_path / 'trials.pkl'
    path.write_bytes(b'not a pickle')
    t = F.fmin_path(_obj, _space(), 5, str(path))
    assert len(t) == 5


def test_fmin_path_dumps_on_error(tmp_path, monkeypatch):
    monkeypatch.setenv('HYPEROPT_FMIN_SEED', '5')
    path = str(tmp_path / 'trials.pkl')
    calls = []

    def bad(d):
        calls.append(1)
        if len(calls) == 4:
            raise RuntimeError('objective failed')
        return _obj(d)
    try:
        F.fmin_path(bad, _space(), 6, path)
    except RuntimeError:
        pass
    else:
        raise AssertionError('the objective error must propagate')
    with open(path, 'rb') as f:
        t = pickle.load(f)
    assert len(t._dynamic_trials) == 4
    assert t._dynamic_trials[-1]['state'] == base.JOB_STATE_ERROR and len(t) == 3


def test_resume_trajectory_matches_uninterrupted_run():
    """30 evals, pickle, reload, 30 more with the same RandomState stream ==
    one 60-eval run (start-up phase: rand.suggest)."""
    space = _space()
    rs = np.random.RandomState(11)
    t = base.Trials()
    F.fmin(_obj, space, algo=rand.suggest, max_evals=30, trials=t, rstate=rs)
    t2 = pickle.loads(pickle.dumps(t))
    F.fmin(_obj, space, algo=rand.suggest, max_evals=60, trials=t2, rstate=rs)
    ref = base.Trials()
    F.fmin(_obj, space, algo=rand.suggest, max_evals=60, trials=ref, rstate=np.random.RandomState(11))
    assert _vals(t2) == _vals(ref)
    assert t2.losses() == ref.losses()


def test_history_cache_rebuilds_after_pickle_and_error_drop():
    space = _space()
    t = base.Trials()
    F.fmin(_obj, space, algo=rand.suggest, max_evals=40, trials=t, rstate=np.random.RandomState(2))
    domain = base.Domain(_obj, space)
    h1 = H.extract(domain, t)                          # builds the incremental cache
    assert '_tpe_history' not in pickle.loads(pickle.dumps(t)).__dict__
    t2 = pickle.loads(pickle.dumps(t))
    _hist_equal(h1, H.extract(domain, t2))             # rebuilt from the documents
    _hist_equal(h1, H._generic(domain, t.trials, domain.table))
    # a middle document turns ERROR: refresh() drops it, the cache must follow
    t._dynamic_trials[17]['state'] = base.JOB_STATE_ERROR
    t.refresh()
    assert len(t) == 39
    _hist_equal(H.extract(domain, t), H._generic(domain, t.trials, domain.table))
    # appended documents extend the cache incrementally
    F.fmin(_obj, space, algo=rand.suggest, max_evals=45, trials=t, rstate=np.random.RandomState(9))
    _hist_equal(H.extract(domain, t), H._generic(domain, t.trials, domain.table))
