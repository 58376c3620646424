"""Host-side logic (no GPU): space flattening, start-up path, history SoA,
Parzen fit and posterior tables against the reference's golden vectors."""
import numpy as np
import pytest

from oracle import tpe_oracle as O
from oracle.spacedesc import params_from_desc
from tests.helpers import amd_space, trials_from_history, doc_values

import hyperopt_amd as H
from hyperopt_amd import base, history, parzen, rand, space


def _domain(desc):
    return base.Domain(lambda x: 0.0, amd_space(desc))


def test_param_table_matches_desc(golden):
    g = golden('suggest_vectors.json')
    for name, desc in g['spaces'].items():
        d = _domain(desc)
        ref = {p['label']: p for p in params_from_desc(desc)}
        assert d.table.labels == sorted(ref)
        for r in d.table.rows:
            p = ref[r.label]
            assert r.dist == p['dist']
            assert r.parents == [None if p['parent'] is None else tuple(p['parent'])]
        # RNG order == the oracle's (pinned by the reference's fixtures)
        assert [r.label for r in d.table.rng_order()] == O._resolve_order(list(ref.values()))


def test_rand_suggest_exact(golden):
    g = golden('suggest_vectors.json')
    for case in g['cases']:
        if case.get('kind') != 'rand':
            continue
        d = _domain(g['spaces'][case['space']])
        docs = rand.suggest([case['n']], d, base.Trials(), case['seed'])
        got = doc_values(docs)
        assert {k: float(v) for k, v in got.items()} == {k: float(v) for k, v in case['result'].items()}
        assert docs[0]['tid'] == case['n'] and docs[0]['misc']['tid'] == case['n']
        base.Trials().assert_valid_trial(docs[0])


def test_history_matches_reference_walk(golden):
    g = golden('suggest_vectors.json')
    for case in g['cases'][:6]:
        if case.get('kind') == 'rand':
            continue
        d = _domain(g['spaces'][case['space']])
        trials = trials_from_history(case['history'], d)
        h = history.extract(d, trials)
        tids, losses, docs = O.history_arrays([dict(tid=x['tid'], loss=x['loss'], vals=x['vals'])
                                               for x in case['history']])
        assert list(h.tids) == tids and list(h.losses) == losses
        # incremental path: extend by a document and compare again
        h2 = history.extract(d, trials)
        assert h2.tids is not None and list(h2.tids) == tids
        gen = history._generic(d, trials.trials, d.table)
        for k in d.table.labels:
            assert list(gen.obs[k][0]) == list(h.obs[k][0])
            assert list(map(float, gen.obs[k][1])) == list(map(float, h.obs[k][1]))


def test_history_cache_tracks_loss_updates():
    d = base.Domain(lambda x: 0.0, {'x': H.hp.uniform('x', 0, 1)})
    t = base.Trials()
    docs = rand.suggest([0, 1, 2], d, t, 1)
    t.insert_trial_docs(docs)
    t.refresh()
    h = history.extract(d, t)
    assert np.all(np.isinf(h.losses))
    for i, doc in enumerate(t.trials):
        doc['state'] = base.JOB_STATE_DONE
        doc['result'] = {'status': 'ok', 'loss': float(i)}
    h = history.extract(d, t)
    assert list(h.losses) == [0.0, 1.0, 2.0]


def _same_as_walk(d, t):
    h = history.extract(d, t)
    gen = history._generic(d, t.trials, d.table)
    assert list(h.tids) == list(gen.tids) and list(h.losses) == list(gen.losses)
    for k in d.table.labels:
        assert list(h.obs[k][0]) == list(gen.obs[k][0]), k
        assert list(map(float, h.obs[k][1])) == list(map(float, gen.obs[k][1])), k
    return h


def _done_trials(d, n, seed=3, tracked=False):
    """``n`` random-search documents, DONE; their results the caller's plain
    dicts (loss-watched documents), or with ``tracked`` Domain.new_result()
    dicts updated in place (tracked documents, as fmin's)."""
    t = base.Trials()
    rs = np.random.RandomState(seed)
    for tid in range(n):
        doc = rand.suggest([tid], d, t, rs.randint(2 ** 31 - 1))[0]
        doc['state'] = base.JOB_STATE_DONE
        if tracked:
            doc['result'] = d.new_result()
            doc['result'].update(status='ok', loss=float(rs.uniform()))
        else:
            doc['result'] = {'status': 'ok', 'loss': float(rs.uniform())}
        t.insert_trial_docs([doc])
    t.refresh()
    return t


def test_history_cache_rebuilds_on_view_changes():
    """Changes to a Trials view that are not appends rebuild the SoA cache:
    a middle document replaced by one with other values, a middle document
    dropped (ERROR) at refresh, a pending document's values edited in place
    — each gives the reference walk's history (tpe.py:820-842)."""
    import copy
    d = base.Domain(lambda x: 0.0, {'x': H.hp.uniform('x', 0, 1), 'c': H.hp.choice('c', [0, 1, 2])})
    t = _done_trials(d, 200)
    h0 = _same_as_walk(d, t)
    # replaced in the middle (off the sampled positions), then refreshed
    i = 37
    new = copy.deepcopy(t._dynamic_trials[i])
    new['misc']['vals']['x'] = [0.123456]
    t._dynamic_trials[i] = new
    t.refresh()
    h1 = _same_as_walk(d, t)
    assert h1 is not h0 and 0.123456 in list(h1.obs['x'][1])
    # dropped in the middle: its state turns ERROR, refresh removes it from the view
    t._dynamic_trials[101]['state'] = base.JOB_STATE_ERROR
    t.refresh()
    h2 = _same_as_walk(d, t)
    assert len(h2) == 199 and 101 not in list(h2.tids)
    # a pending document's values edited in place (the running trial's doc)
    doc = rand.suggest([500], d, t, 5)[0]
    t.insert_trial_docs([doc])
    t.refresh()
    _same_as_walk(d, t)
    t.trials[-1]['misc']['vals']['x'] = [0.654321]
    h3 = _same_as_walk(d, t)
    assert 0.654321 in list(h3.obs['x'][1])
    # plain appends keep the cache (no rebuild: the same value columns, extended)
    t.trials[-1]['state'] = base.JOB_STATE_DONE
    t.trials[-1]['result'] = {'status': 'ok', 'loss': 0.5}
    h4 = _same_as_walk(d, t)
    more = rand.suggest([501], d, t, 6)[0]
    more['state'] = base.JOB_STATE_DONE
    more['result'] = {'status': 'ok', 'loss': 0.25}
    t.insert_trial_docs([more])
    t.refresh()
    cache = history._CACHES[t]
    h5 = _same_as_walk(d, t)
    assert history._CACHES[t] is cache and len(h5) == len(h4) + 1


@pytest.mark.parametrize('tracked', [False, True])
def test_history_cache_sees_in_place_edits_of_completed_documents(tracked):
    """Completed documents the cache has consumed, edited in place at any
    depth (values, loss, state), through a view edit without refresh, after
    a pickle round trip, or through the caller's own inserted list: each
    extract equals the reference walk (tpe.py:820-842); edits of bookkeeping
    keys and of pending documents keep the cache.  Results the caller's
    plain dicts (loss-watched documents) or tracked ones."""
    import copy
    import pickle
    d = base.Domain(lambda x: 0.0, {'x': H.hp.uniform('x', 0, 1), 'c': H.hp.choice('c', [0, 1, 2])})
    t = _done_trials(d, 300, tracked=tracked)
    _same_as_walk(d, t)
    cache = history._CACHES[t]
    assert len(cache.watch_res) == (0 if tracked else 300) and not cache.watch
    t.trials[150]['refresh_time'] = 1.0             # bookkeeping: no rebuild
    _same_as_walk(d, t)
    assert history._CACHES[t] is cache
    t.trials[151]['misc']['vals']['x'][0] = 0.987654  # a value, two levels down
    h = _same_as_walk(d, t)
    assert 0.987654 in list(h.obs['x'][1]) and history._CACHES[t] is not cache
    t.trials[77]['result']['loss'] = -5.0             # a loss
    h = _same_as_walk(d, t)
    assert -5.0 in list(h.losses)
    t.trials[78]['result'] = {'status': 'ok', 'loss': -6.0}    # a new result dict, then edited
    _same_as_walk(d, t)
    t.trials[78]['result']['loss'] = -7.0
    h = _same_as_walk(d, t)
    assert -7.0 in list(h.losses) and -6.0 not in list(h.losses)
    t.trials[79]['state'] = base.JOB_STATE_RUNNING    # back to pending, then its loss edited
    _same_as_walk(d, t)
    t.trials[79]['result']['loss'] = -8.0
    h = _same_as_walk(d, t)
    assert h.losses[79] == -8.0
    k = 'c' if t.trials[80]['misc']['vals']['c'] else 'x'
    del t.trials[80]['misc']['vals'][k][:]            # an observation removed
    t.trials[80]['misc']['idxs'][k].clear()
    _same_as_walk(d, t)
    new = copy.deepcopy(t.trials[90])                 # the view edited without refresh
    new['misc']['vals']['x'] = [0.5555]
    t.trials[90] = new
    h = _same_as_walk(d, t)
    assert 0.5555 in list(h.obs['x'][1])
    t._dynamic_trials[90] = t.trials[90]
    t.refresh()                                       # a deep copy: tracked from the refresh on
    _same_as_walk(d, t)
    t.trials[90]['misc']['vals']['x'][0] = 0.6666
    h = _same_as_walk(d, t)
    assert 0.6666 in list(h.obs['x'][1])
    t2 = pickle.loads(pickle.dumps(t))                 # a pickle round trip stays tracked
    _same_as_walk(d, t2)
    t2.trials[200]['misc']['vals']['x'] = [0.1234]
    h = _same_as_walk(d, t2)
    assert 0.1234 in list(h.obs['x'][1])
    docs = rand.suggest([1000], d, t2, 9)             # the caller's list names the held documents
    docs[0]['state'] = base.JOB_STATE_DONE
    docs[0]['result'] = {'status': 'ok', 'loss': 0.5}
    t2.insert_trial_docs(docs)
    t2.refresh()
    _same_as_walk(d, t2)
    docs[0]['result']['loss'] = -9.0
    h = _same_as_walk(d, t2)
    assert h.losses[-1] == -9.0
    plain = rand.suggest([1001], d, t2, 10)[0]
    plain.update(state=base.JOB_STATE_DONE, result={'status': 'ok', 'loss': 0.5})
    t2._dynamic_trials.append(plain)
    t2.refresh()                                      # put in directly: tracked at refresh
    _same_as_walk(d, t2)
    t2.trials[-1]['result']['loss'] = -11.0
    h = _same_as_walk(d, t2)
    assert h.losses[-1] == -11.0


def _fresh_trials_like(d, t):
    """A new Trials holding plain copies of ``t``'s view (the reference's
    state after the same edits)."""
    import copy
    t2 = base.Trials()
    t2.insert_trial_docs([copy.deepcopy(dict(x)) for x in t.trials])
    t2.refresh()
    return t2


def test_trials_store_the_callers_objects():
    """insert_trial_docs stores the caller's documents and an assignment into
    a document stores the assigned object (reference base.py:295-307, 315-331):
    edits made later through the caller's own handles — the document after
    insert_trial_docs, a result dict after assignment, a misc held before the
    insertion, a values list assigned into it, a plain dict document — are the
    Trials' state, and the history equals the reference walk and a Trials
    built afresh from that state."""
    d = base.Domain(lambda x: 0.0, {'x': H.hp.uniform('x', 0, 1), 'c': H.hp.choice('c', [0, 1, 2])})
    for tracked in (False, True):
        tr = _done_trials(d, 60, tracked=tracked)
        _same_as_walk(d, tr)
        # 1. the verdict's pattern: edit after insert_trial_docs([doc]), then refresh
        doc = rand.suggest([60], d, tr, 11)[0]
        lst = [doc]
        tr.insert_trial_docs(lst)
        assert lst[0] is doc and tr._dynamic_trials[-1] is doc
        doc['state'] = base.JOB_STATE_DONE
        doc['result'] = {'status': 'ok', 'loss': 0.125}
        tr.refresh()
        assert tr.trials[-1] is doc and tr.losses()[-1] == 0.125
        h = _same_as_walk(d, tr)
        assert h.losses[-1] == 0.125
        # 2. a result dict assigned, then mutated through the caller's handle
        r = {'status': 'ok', 'loss': 2.0}
        tr.trials[0]['result'] = r
        assert tr.trials[0]['result'] is r
        _same_as_walk(d, tr)
        r['loss'] = 3.0
        assert tr.losses()[0] == 3.0
        h = _same_as_walk(d, tr)
        assert h.losses[0] == 3.0
        r['loss'] = -1.0                                  # twice: the loss-watch follows the object
        assert _same_as_walk(d, tr).losses[0] == -1.0
        # 3. a misc held before the insertion, edited after it
        doc2 = rand.suggest([61], d, tr, 12)[0]
        m = doc2['misc']
        doc2['state'] = base.JOB_STATE_DONE
        doc2['result'] = {'status': 'ok', 'loss': 0.75}
        tr.insert_trial_docs([doc2])
        tr.refresh()
        _same_as_walk(d, tr)
        m['vals']['x'] = [0.4242]
        m['idxs']['x'] = [61]
        assert tr.trials[-1]['misc'] is m
        h = _same_as_walk(d, tr)
        assert 0.4242 in list(h.obs['x'][1])
        # 4. a values list of the caller's assigned into a document, then edited
        L = [0.31]
        tr.trials[5]['misc']['vals']['x'] = L
        tr.trials[5]['misc']['idxs']['x'] = [tr.trials[5]['tid']]
        _same_as_walk(d, tr)
        L[0] = 0.32
        h = _same_as_walk(d, tr)
        assert 0.32 in list(h.obs['x'][1]) and 0.31 not in list(h.obs['x'][1])
        # 5. a plain dict document of the caller's: stored as it is, edits seen
        plain = dict(rand.suggest([62], d, tr, 13)[0])
        plain['misc'] = {'tid': 62, 'cmd': None, 'workdir': None, 'idxs': {'x': [62], 'c': []},
                         'vals': {'x': [0.5], 'c': []}}
        plain['state'] = base.JOB_STATE_DONE
        plain['result'] = {'status': 'ok', 'loss': 0.01}
        tr.insert_trial_docs([plain])
        tr.refresh()
        assert tr.trials[-1] is plain and type(plain) is dict
        _same_as_walk(d, tr)
        plain['misc']['vals']['x'][0] = 0.55
        plain['result']['loss'] = 0.02
        h = _same_as_walk(d, tr)
        assert h.losses[-1] == 0.02 and 0.55 in list(h.obs['x'][1])
        plain['state'] = base.JOB_STATE_ERROR             # a plain document leaves the view at refresh
        tr.refresh()
        assert plain not in tr.trials
        _same_as_walk(d, tr)
        plain['state'] = base.JOB_STATE_DONE              # ... and comes back
        tr.refresh()
        assert tr.trials[-1] is plain
        # the same history as a Trials built afresh from the final state
        h = _same_as_walk(d, tr)
        h2 = history.extract(d, _fresh_trials_like(d, tr))
        assert list(h.losses) == list(h2.losses) and list(h.tids) == list(h2.tids)
        for k in d.table.labels:
            assert list(map(float, h.obs[k][1])) == list(map(float, h2.obs[k][1]))


def test_fmin_documents_are_tracked():
    """fmin's own documents (rand / tpe suggestions, Domain.evaluate results)
    are tracked: the history cache re-reads none of them per suggest, and a
    result edited through the Trials afterwards is still seen."""
    from hyperopt_amd.fmin import fmin
    t = base.Trials()
    fmin(lambda x: (x - 0.3) ** 2, H.hp.uniform('x', 0, 1), algo=rand.suggest, max_evals=40, trials=t,
         rstate=np.random.RandomState(0))
    d = base.Domain(lambda x: 0.0, H.hp.uniform('x', 0, 1))
    _same_as_walk(d, t)
    c = history._CACHES[t]
    assert not c.watch and not c.watch_res
    t.trials[10]['result']['loss'] = -4.0
    assert _same_as_walk(d, t).losses[10] == -4.0


def test_view_append_is_dropped_at_refresh():
    """A document appended to ``trials.trials`` alone is gone after the next
    refresh, which rebuilds the view from the documents (base.py:231-242)."""
    d = base.Domain(lambda x: 0.0, {'x': H.hp.uniform('x', 0, 1)})
    t = _done_trials(d, 30, tracked=True)
    _same_as_walk(d, t)
    extra = rand.suggest([99], d, t, 3)[0]
    extra['state'] = base.JOB_STATE_DONE
    extra['result'] = {'status': 'ok', 'loss': 0.5}
    t.trials.append(extra)
    assert _same_as_walk(d, t).tids[-1] == 99       # (the view as it stands)
    t.refresh()
    assert extra not in t.trials and len(t.trials) == 30
    assert 99 not in list(_same_as_walk(d, t).tids)


def test_incremental_refresh_equals_full_filter():
    """Trials.refresh extends the view in place after appends and rebuilds it
    after any other change: over a random sequence of appends, state edits
    (into and out of ERROR), direct _dynamic_trials edits and view edits the
    view always equals the reference's filter of every document
    (base.py:183-194), and the history equals the reference walk."""
    rs = np.random.RandomState(7)
    d = base.Domain(lambda x: 0.0, {'x': H.hp.uniform('x', 0, 1)})
    t = base.Trials()
    tid = 0
    for step in range(300):
        op = rs.randint(6)
        if op <= 2 or len(t._dynamic_trials) < 5:
            docs = rand.suggest(list(range(tid, tid + rs.randint(1, 4))), d, t, rs.randint(1000))
            tid += len(docs)
            for doc in docs:
                doc['state'] = base.JOB_STATE_DONE
                doc['result'] = {'status': 'ok', 'loss': float(rs.uniform())}
            t.insert_trial_docs(docs)
            if rs.rand() < 0.2:          # an appended document failing before the refresh
                docs[-1]['state'] = base.JOB_STATE_ERROR
        elif op == 3:                    # a seen document into or out of ERROR
            doc = t._dynamic_trials[rs.randint(len(t._dynamic_trials))]
            doc['state'] = base.JOB_STATE_ERROR if doc['state'] != base.JOB_STATE_ERROR else base.JOB_STATE_DONE
        elif op == 4 and rs.rand() < 0.3:   # a direct edit of the document list
            i = rs.randint(len(t._dynamic_trials))
            t._dynamic_trials[i] = dict(t._dynamic_trials[i])
        elif op == 5 and rs.rand() < 0.3 and len(t.trials):    # a view edit
            del t.trials[rs.randint(len(t.trials))]
        t.refresh()
        want = [x for x in t._dynamic_trials if x['state'] != base.JOB_STATE_ERROR]
        assert len(t.trials) == len(want) and all(a is b for a, b in zip(t.trials, want)), step
        if step % 10 == 0 and len(t.trials):
            _same_as_walk(d, t)


def test_appended_documents_update_tree_records_in_place():
    """FMinIter's flow — one or a few finished documents appended before each
    suggest: the tree records updated in place (tpe._tree_refill), the merged
    value orders and the below set kept incrementally (one-document fast
    paths) equal a rebuild from scratch and the reference's argsort below set
    (tpe.py:625-636) — including tied losses."""
    import bench
    from hyperopt_amd import tpe
    domain, trials = bench.make_history(600, 3)
    table = domain.table
    rs = np.random.RandomState(0)
    tid = 10 ** 6
    in_place = 0
    for i in range(40):
        hist = history.extract(domain, trials)
        below = history.split_below(hist, 0.25)
        memo = getattr(hist._cache, 'tree_memo', None)
        tl = tpe._tree_labels(table, hist, None)
        in_place += memo is not None and memo[3][0] is tl[0]
        # a rebuild from scratch gives the same records
        cache = hist._cache
        kept = cache.tree_memo
        cache.tree_memo = None
        assert tpe._tree_labels(table, hist, None)[0].tobytes() == tl[0].tobytes(), i
        cache.tree_memo = kept[:3] + (tl,) + kept[4:]
        n_below = min(int(np.ceil(0.25 * np.sqrt(len(hist)))), 25)
        L = hist.losses
        order = np.argsort(L)
        if L[order[n_below - 1]] != L[order[n_below]]:
            assert sorted(below.tolist()) == sorted(hist.tids[order[:n_below]].tolist()), i
        for k in table.labels:
            o = hist.value_order(k)
            if o is not None:
                v = np.asarray(hist.obs[k][1], dtype=np.float64)
                assert len(o) == len(v) and np.all(np.diff(v[o]) >= 0), (i, k)
                assert sorted(o.tolist()) == list(range(len(v)))
        for _ in range(rs.randint(1, 4)):
            d = rand.suggest([tid], domain, trials, rs.randint(2 ** 31 - 1))[0]
            d['state'] = base.JOB_STATE_DONE
            d['result'] = {'status': 'ok', 'loss': float(rs.choice([0.0, 0.5, rs.uniform()]))}
            tid += 1
            trials.insert_trial_docs([d])
        trials.refresh()
    assert in_place >= 30


def test_fit_posterior_exact(golden):
    for case in golden('kernel_vectors.json'):
        post = parzen.fit_posterior(case['dist'], case['args'], np.asarray(case['below']),
                                    np.asarray(case['above']), 1.0)
        for got, want in ((post.below, case['b_params']), (post.above, case['a_params'])):
            for g_, w_ in zip(got, want):
                assert list(np.asarray(g_, dtype=float)) == [float(v) for v in w_], case['dist']


def test_parzen_unit_vectors_exact(golden):
    for case in golden('unit_vectors.json')['adaptive_parzen_normal']:
        w, m, s = parzen.fit_parzen(case['mus'], case['prior_weight'], case['prior_mu'], case['prior_sigma'])
        assert list(w) == case['w'] and list(m) == case['mu'] and list(s) == case['sigma']
    for case in golden('unit_vectors.json')['linear_forgetting_weights']:
        assert list(parzen.linear_forgetting_weights(case['N'], case['LF'])) == case['w']


def test_split_matches_ap_filter_trials(golden):
    for case in golden('unit_vectors.json')['ap_filter_trials']:
        h = history.History(np.asarray(case['l_idxs']), np.asarray(case['l_vals']), {})
        bt = history.split_below(h, case['gamma'])
        m = history.below_mask(np.asarray(case['o_idxs']), bt)
        ov = np.asarray(case['o_vals'])
        assert list(ov[m]) == case['below'] and list(ov[~m]) == case['above']


def test_gauss_table_reproduces_lpdf(golden):
    """The folded (mu, a, c, base) table evaluated in float64 on the host
    reproduces GMM1_lpdf / LGMM1_lpdf — checks the table algebra the kernels use."""
    for case in golden('kernel_vectors.json'):
        if case['dist'] not in ('uniform', 'loguniform', 'normal', 'lognormal'):
            continue
        post = parzen.fit_posterior(case['dist'], case['args'], np.asarray(case['below']),
                                    np.asarray(case['above']), 1.0)
        logf = post.family == 1
        x = np.asarray(case['cand'])
        t = np.log(x) if logf else x
        for mix, ref in ((post.below, case['l']), (post.above, case['g'])):
            mu, a, c, b = parzen.gauss_table(*mix, post, logf)
            v = c[None, :] - (a[None, :] * (t[:, None] - mu[None, :])) ** 2
            m = v.max(axis=1)
            lp = (m + np.log2(np.exp2(v - m[:, None]).sum(axis=1))) * np.log(2) + b - (t if logf else 0)
            np.testing.assert_allclose(lp, ref, rtol=1e-10, atol=1e-10)


def test_space_evaluate_and_duplicate_label():
    sp = {'a': H.hp.choice('c', [H.hp.uniform('u', 0, 1), {'k': H.hp.randint('r', 3)}]),
          'b': H.scope.int(H.hp.quniform('q', 0, 10, 1)) + 1}
    assert space.evaluate(sp, {'c': 1, 'r': np.int64(2), 'q': 4.0}) == {'a': {'k': 2}, 'b': 5}
    assert space.evaluate(sp, {'c': 0, 'u': np.float64(0.5), 'q': 3.0}) == {'a': 0.5, 'b': 4}
    with pytest.raises(H.exceptions.DuplicateLabel):
        base.Domain(lambda x: 0, [H.hp.uniform('x', 0, 1), H.hp.uniform('x', 0, 2)])
    with pytest.raises(TypeError):
        H.hp.uniform(3, 0, 1)


def test_tree_memo_follows_the_table_object():
    """The native tree records are memoised per (table object, document
    count): a second Domain with the same labels and other bounds on the same
    Trials gets its own records (its bounds and priors), never the first's."""
    from hyperopt_amd import base, hp, history as H, rand, tpe
    d1 = base.Domain(lambda d: 0.0, {'x': hp.uniform('x', -5, 5), 'c': hp.choice('c', [0, 1])})
    trials = base.Trials()
    rs = np.random.RandomState(0)
    for tid in range(30):
        doc = rand.suggest([tid], d1, trials, rs.randint(2 ** 31 - 1))[0]
        doc['state'] = base.JOB_STATE_DONE
        doc['result'] = {'status': 'ok', 'loss': float(tid)}
        trials.insert_trial_docs([doc])
    trials.refresh()
    a1 = tpe._tree_labels(d1.table, H.extract(d1, trials))[0]
    assert tpe._tree_labels(d1.table, H.extract(d1, trials))[0] is a1          # memo hit
    d2 = base.Domain(lambda d: 0.0, {'x': hp.uniform('x', -1, 2), 'c': hp.choice('c', [0, 1])})
    a2 = tpe._tree_labels(d2.table, H.extract(d2, trials))[0]
    ix = d2.table.by_label['x'].index
    assert (a2[ix]['low'], a2[ix]['high'], a2[ix]['prior_mu']) == (-1.0, 2.0, 0.5)
    assert (a1[ix]['low'], a1[ix]['high']) == (-5.0, 5.0)


def test_plain_history_below_split_from_sampled_bound():
    """A History without a Trials cache takes its n_below smallest losses from
    a strided sample's bound (history._smallest_plain) instead of an O(N)
    argpartition: the same positions, ordered by (loss, position), as a stable
    argsort (NaN last) — ties at the boundary, NaN and +inf losses included —
    and split_below gives the reference's below set."""
    from hyperopt_amd import history as H
    rs = np.random.RandomState(5)
    checked = 0
    for trial in range(200):
        n = int(rs.randint(2000, 60000))
        L = rs.uniform(size=n)
        if trial % 3 == 0:
            L = np.round(L * rs.randint(5, 400)) / 7.0           # heavy ties
        if trial % 5 == 0:
            L[rs.choice(n, rs.randint(1, 40))] = np.nan
        if trial % 7 == 0:
            L[rs.choice(n, rs.randint(1, 40))] = np.inf
        m = int(rs.randint(1, 27))
        got = H._smallest_plain(L, m)
        if got is None:
            continue
        checked += 1
        np.testing.assert_array_equal(got, np.argsort(L, kind='stable')[:m])
        tids = np.arange(n, dtype=np.int64) * 3
        hist = H.History(tids, L, {})
        b = H.split_below(hist, 0.25)
        nb = min(int(np.ceil(0.25 * np.sqrt(n))), 25)
        ref = tids[np.argsort(L, kind='stable')[:nb]]
        Ls = np.sort(np.where(np.isnan(L), np.inf, L))
        if nb < n and Ls[nb - 1] != Ls[nb]:                     # (a boundary tie: the reference's argsort order decides)
            assert set(np.asarray(b).tolist()) == set(ref.tolist())
    assert checked > 150


def test_plain_history_ranking_kept_across_appends():
    """Columnar Histories over one append-only loss buffer (a History per
    suggest over growing views, sharing ``dev``: bench.py config 5
    --appending) keep their loss ranking incrementally (history._TopState):
    after every append of 1-3 losses (ties, +inf, an occasional NaN and a
    jump of 50 that rebuilds) the m smallest are a stable argsort's, and
    split_below gives the reference's below set; a History reused as it is
    returns the same below set object."""
    from hyperopt_amd import history as H
    rs = np.random.RandomState(11)
    cap = 30000
    L = np.round(rs.uniform(size=cap) * 20000) / 7.0          # (ties, the boundary mostly untied)
    L[rs.choice(cap, 30)] = np.inf
    tids = np.arange(cap, dtype=np.int64) * 2
    dev = {}
    n = 12000
    checked = 0
    for step in range(300):
        n += 50 if step % 97 == 0 else int(rs.randint(1, 4))
        if step == 150:
            L[n - 1] = np.nan
        hist = H.History(tids[:n], L[:n], {}, dev=dev)
        m = int(rs.randint(1, 27))
        got = hist.smallest(m)
        ref = np.argsort(L[:n], kind='stable')[:m]
        np.testing.assert_array_equal(np.asarray(got), ref)
        b = H.split_below(hist, 0.25)
        nb = min(int(np.ceil(0.25 * np.sqrt(n))), 25)
        Ls = np.sort(np.where(np.isnan(L[:n]), np.inf, L[:n]))
        if Ls[nb - 1] != Ls[nb]:
            assert set(np.asarray(b).tolist()) == set(tids[np.argsort(L[:n], kind='stable')[:nb]].tolist())
            checked += 1
        assert H.split_below(hist, 0.25) is b or Ls[nb - 1] == Ls[nb]
    assert checked > 100
    assert isinstance(dev['_top'], H._TopState)
