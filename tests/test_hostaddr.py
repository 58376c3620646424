"""The _hostaddr CPython extension (hyperopt_amd/csrc/hostaddr.c): each
function against the Python it replaces."""
import ctypes

import numpy as np
import pytest

_ha = pytest.importorskip('hyperopt_amd._hostaddr')


def test_addresses_and_tails():
    arrs = [np.arange(5, dtype=np.float64) + k for k in range(4)]
    assert _ha.addresses(arrs).tolist() == [a.ctypes.data for a in arrs]
    got = _ha.tails(arrs, np.array([1, 0, 3, 5]), np.array([3, 2, 5, 5]))
    np.testing.assert_array_equal(got, np.concatenate([arrs[0][1:3], arrs[1][0:2], arrs[2][3:5]]))


@pytest.mark.parametrize('n_ids', [1, 4, 5, 300])
def test_result_dicts_keep_numpy_types(n_ids):
    """A suggest's per-id dicts (tpe._result_dicts, _hostaddr.typed_dicts): level
    order, None for an inactive label, np.int64 categories and np.float64
    values — the reference's types whatever the id count."""
    from hyperopt_amd import hp, tpe
    from hyperopt_amd.space import ParamTable
    table = ParamTable({'c': hp.choice('c', [{'x': hp.uniform('x', 0, 1)}, {'y': hp.normal('y', 0, 1)}]),
                        'z': hp.loguniform('z', -1, 1)})
    order = table.level_order()
    rs = np.random.RandomState(n_ids)
    L = len(table.rows)
    values = rs.uniform(size=(n_ids, L))
    active = np.ones((n_ids, L), dtype=np.int8)
    ci = table.by_label['c'].index
    values[:, ci] = rs.randint(0, 2, n_ids)
    for j in range(n_ids):                 # (the branch the choice did not take: inactive)
        active[j, table.by_label['y' if values[j, ci] == 0 else 'x'].index] = 0
    got = tpe._result_dicts(table, values, active)
    assert len(got) == n_ids
    for j, d in enumerate(got):
        assert list(d) == list(order)
        for k, v in d.items():
            r = table.by_label[k]
            if not active[j, r.index]:
                assert v is None
            elif r.categorical:
                assert type(v) is np.int64 and v == int(values[j, r.index])
            else:
                assert type(v) is np.float64 and v == values[j, r.index]


def test_tracked_misc_matches_python():
    """The native misc of a suggested id has the Python version's contents,
    key order, types and parent links (tracked lists under tracked dicts
    under the misc, misc._up None, misc._fx False)."""
    from hyperopt_amd import base
    chosen = {'m': 1, 'a': None, 'b': 2.5, 'c': None, 'd': np.float64(0.25)}
    nat = base.tracked_misc(7, ('cmd',), 'wd', chosen)
    saved = base._ha_misc
    base._ha_misc = None
    try:
        ref = base.tracked_misc(7, ('cmd',), 'wd', chosen)
    finally:
        base._ha_misc = saved
    assert saved is not None
    for m in (nat, ref):
        assert type(m) is base._Part and m._up is None and m._fx is False
        assert list(m) == ['tid', 'cmd', 'workdir', 'idxs', 'vals']
        for k in ('idxs', 'vals'):
            assert type(m[k]) is base._Part and m[k]._up() is m
            assert list(m[k]) == list(chosen)
            for lab, lst in m[k].items():
                assert type(lst) is base._PartList and lst._up() is m[k]
    assert nat == ref
    assert type(nat['vals']['d'][0]) is np.float64
    # the lists are tracked: an edit reaches the misc's log like the Python ones'
    nat['vals']['b'].append(3.0)
    assert nat['vals']['b'] == [2.5, 3.0]


def test_call_tree_matches_ctypes_on_refused_arguments():
    """The trampoline passes the same arguments through: a refused call (a
    negative label count) returns what the ctypes call returns."""
    from hyperopt_amd import _native as N
    lib = N.load()
    fn = ctypes.cast(lib.tpe_suggest_tree, ctypes.c_void_p).value
    ws, need, path = N.LevelWS(), N.LevelNeed(), (ctypes.c_int32 * 2)()
    rc_ct = lib.tpe_suggest_tree(0, -1, 0, 0, 1.0, 25, 0, 1, 2048, 0, 0, None, 5, 64.0, 0, 0, ctypes.byref(ws),
                                 ctypes.byref(need), 0, 0, 0, path, 0)
    rc_tr = _ha.call_tree(fn, 0, -1, 0, 0, 1.0, 25, 0, 1, 2048, 0, 0, 0, 5, 64.0, 0, 0, ctypes.addressof(ws),
                          ctypes.addressof(need), 0, 0, 0, ctypes.addressof(path), 0)
    assert rc_ct == rc_tr == -1                    # TPE_E_ARG
    with pytest.raises(ValueError):
        _ha.call_tree(0, 0, -1, 0, 0, 1.0, 25, 0, 1, 2048, 0, 0, 0, 5, 64.0, 0, 0, 0, 0, 0, 0, 0, 0, 0)


def test_insert_sorted_matches_numpy():
    """One value into a sorting permutation and its sorted values: numpy's
    searchsorted(side='right') position (ties: after the equal ones; NaN after
    every number) and np.insert's arrays."""
    rs = np.random.RandomState(1)
    for _ in range(500):
        m = rs.randint(0, 40)
        col = np.sort(np.concatenate([rs.choice([0.5, 1.0, 2.0, np.nan], m // 2), rs.uniform(0, 3, m - m // 2)]))
        v = float(rs.choice([0.5, 1.0, 2.0, np.nan, rs.uniform(0, 3)]))
        perm = np.zeros(m + 1, dtype=np.int64)
        perm[:m] = np.arange(m)
        sv = np.zeros(m + 1)
        sv[:m] = col
        at_ref = int(np.searchsorted(col, v, side='right'))
        assert _ha.insert_sorted(perm, sv, m, v, m) == at_ref
        np.testing.assert_array_equal(sv, np.insert(col, at_ref, v))
        np.testing.assert_array_equal(perm, np.insert(np.arange(m), at_ref, m))
    with pytest.raises(ValueError):
        _ha.insert_sorted(np.zeros(3, dtype=np.int64), np.zeros(3), 3, 1.0, 3)     # no room


def test_obs_append_matches_python_loop():
    """History._Cache.extend's per-label loop in C: the same columns, counts and
    changed labels as the Python loop, and the first full column handed back
    with nothing of its label written."""
    from hyperopt_amd.history import _Grow
    rs = np.random.RandomState(2)
    labels = ['a', 'b', 'c', 'd']
    kinds = {'a': np.float64, 'b': np.int64, 'c': np.float64, 'd': np.float64}

    def cols():
        return {k: _Grow(np.int64) for k in labels}, {k: _Grow(kinds[k]) for k in labels}

    ct, cv = cols()
    pt, pv = cols()
    for tid in range(200):
        vals = {}
        for k in labels:
            r = rs.randint(4)
            if r == 1:
                vals[k] = []
            elif r >= 2:
                vals[k] = [int(rs.randint(5)) if k == 'b' else (np.float64(rs.uniform()) if r == 3 else rs.uniform())]
        ch_c, ch_p = set(), set()
        j = _ha.obs_append(labels, vals, tid, [ct[k] for k in labels], [cv[k] for k in labels], ch_c)
        for k in (labels[j:] if j >= 0 else []):     # (a full column: Python from there, as extend goes on)
            v = vals.get(k)
            if v:
                ct[k].append(tid); cv[k].append(v[0]); ch_c.add(k)
        for k in labels:
            v = vals.get(k)
            if v:
                pt[k].append(tid); pv[k].append(v[0]); ch_p.add(k)
        assert ch_c == ch_p
    for k in labels:
        assert ct[k].n == pt[k].n and cv[k].n == pv[k].n
        np.testing.assert_array_equal(ct[k].view(), pt[k].view())
        np.testing.assert_array_equal(cv[k].view(), pv[k].view())
        assert cv[k].view().dtype == pv[k].view().dtype
    # a full column comes back untouched
    g_t, g_v = _Grow(np.int64), _Grow(np.float64)
    g_t.n = g_v.n = g_t.a.shape[0]
    assert _ha.obs_append(['x'], {'x': [1.5]}, 7, [g_t], [g_v], set()) == 0
    assert g_t.n == g_t.a.shape[0]


def test_suggestion_documents_hold_no_reference_cycles():
    """A suggestion's document (tracked misc, result, the doc itself) is freed
    by reference counting: the parent links are weak, and the tree walk of
    ParamTable.rng_order is no recursive closure — nothing per suggest is
    left for the cyclic collector (whose collections were the headline
    suggest's latency tail)."""
    import gc
    import bench
    from hyperopt_amd import base, rand
    domain, trials = bench.make_history(60, 3)
    T0 = 7_000_000                                 # (tids no other test's documents carry)
    d = rand.suggest([500], domain, trials, 1)     # (first call: caches)
    del d
    gc.collect()
    gc.disable()
    gc.set_debug(gc.DEBUG_SAVEALL)
    try:
        for i in range(40):
            d = rand.suggest([T0 + i], domain, trials, i)
            # the links still lead up to the document, for the mutation logs
            lst = d[0]['misc']['vals']['model']
            assert lst._up() is d[0]['misc']['vals'] and d[0]['misc']['vals']._up() is d[0]['misc']
            del d, lst
        gc.collect()
        # (other tests' objects may be collected here too — a Trials' cache is a
        # cycle — so only this loop's documents count: their tids are unique)
        ours = [o for o in gc.garbage if type(o) in (base._Doc, base._Part) and T0 <= o.get('tid', -1) < T0 + 40]
    finally:
        gc.set_debug(0)
        gc.garbage.clear()
        gc.enable()
    assert not ours, len(ours)
