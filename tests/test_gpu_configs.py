"""Full-size GPU parity of BASELINE.json configs 3, 4 and 5 against the oracle.

The production path (``tpe.suggest`` / ``tpe.suggest_choices`` -> the one-call
level runner) runs at the configs' full sizes; every winner it returns is then
checked against the CPU oracle (oracle/tpe_oracle.py, pinned to the
reference's golden vectors):

  * the oracle splits and fits the history itself (ap_filter_trials,
    adaptive_parzen_normal: tpe.py:613-641, 398-475);
  * the winner's candidates are re-drawn through the engine (Philox counters
    depend only on (seed, label, new_id, candidate index), so a re-run draws
    exactly the production candidates) with per-candidate l and g;
  * l and g agree with the oracle's GMM1_lpdf / LGMM1_lpdf within the
    north_star tolerance (1e-5 relative, fp32; 1e-9 for quantized families,
    which are scored in float64), and categorical choices are exact;
  * the production winner lies in the oracle's eps-tie set.  The oracle scores
    a random subset plus the best candidates by GPU score; every candidate it
    does not score is shown unable to reach that set (its GPU score plus its
    own tolerance bound stays below the set), so the check covers all C
    candidates without an O(C*K) CPU pass.
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

TOL32 = 1e-5
TOL64 = 1e-9


def _chunked(fn, x, n_comp):
    """fn over x in chunks whose C x K temporaries stay near 160 MB."""
    step = max(1, int(2e7 // max(n_comp, 1)))
    if not len(x):
        return np.zeros(0)
    return np.concatenate([np.asarray(fn(x[i:i + step]), dtype=np.float64) for i in range(0, len(x), step)])


def _check_lpdf(got, ref, tol, what):
    fin = np.isfinite(ref)
    err = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1.0)
    assert err.size == 0 or err.max() <= tol, (what, float(err.max()), int(np.argmax(err)))
    assert np.all((got[~fin] == ref[~fin]) | (got[~fin] < -700)), what


def check_winner(values, cand, l, g, lpdf_b, lpdf_a, n_comp, tol, rs, what, k_top=1024, n_rand=1024):
    """Each value in ``values`` (the production winners of one problem's
    candidate set) is a candidate in the oracle's eps-tie set; l and g of the
    checked candidates agree with the oracle.  Returns the number of
    candidates the oracle scored."""
    s = l - g
    C = len(s)
    assert not np.isnan(s).any(), what
    # per-candidate bound of |s_gpu - s_ref| implied by the lpdf tolerance
    bound = 1.001 * tol * (np.maximum(np.abs(l), 1.0) + np.maximum(np.abs(g), 1.0))
    u, inv = np.unique(cand, return_inverse=True)
    if len(u) <= max(C // 4, 1):
        # few distinct values (quantized lattice, categories): the oracle scores
        # each distinct value once, which covers every candidate exactly
        lr = _chunked(lpdf_b, u, 32)[inv]
        gr = _chunked(lpdf_a, u, n_comp)[inv]
        _check_lpdf(l, lr, tol, what + ' l')
        _check_lpdf(g, gr, tol, what + ' g')
        sr = lr - gr
        fin = np.isfinite(sr)
        M = np.max(sr[fin])
        eps = 4 * tol * max(1.0, float(np.max(np.abs(lr[fin]))), float(np.max(np.abs(gr[fin]))))
        ties = np.nonzero(sr >= M - eps)[0]
        for v in np.atleast_1d(values):
            assert np.isin(np.nonzero(cand == v)[0], ties).any(), (what, v, float(M))
        return C
    rnd = rs.choice(C, min(n_rand, C), replace=False)
    while True:
        k = min(k_top, C)
        top = np.argpartition(-s, k - 1)[:k] if k < C else np.arange(C)
        chk = np.union1d(top, rnd)
        lr = _chunked(lpdf_b, cand[chk], 32)
        gr = _chunked(lpdf_a, cand[chk], n_comp)
        _check_lpdf(l[chk], lr, tol, what + ' l')
        _check_lpdf(g[chk], gr, tol, what + ' g')
        sr = lr - gr
        fin = np.isfinite(sr)
        M = np.max(sr[fin])
        eps = 4 * tol * max(1.0, float(np.max(np.abs(lr[fin]))), float(np.max(np.abs(gr[fin]))))
        if k == C:
            break
        unchecked = np.ones(C, dtype=bool)
        unchecked[chk] = False
        if not unchecked.any() or np.max((s + bound)[unchecked]) < M - eps:
            break
        k_top *= 8                   # a wide near-tie plateau: score more candidates
    ties = chk[sr >= M - eps]
    for v in np.atleast_1d(values):
        at = np.nonzero(cand == v)[0]
        assert len(at), (what, 'winner is not one of the candidates', v)
        assert np.isin(at, ties).any(), (what, v, at[:5], float(M), float(np.max(s)), ties[:10])
    return len(chk)


def _oracle_fits(row, hist, gamma=0.25):
    """The oracle's below/above posteriors of one label from a History."""
    otids, ovals = hist.obs[row.label]
    below, above = O.ap_filter_trials(otids, ovals, hist.tids, hist.losses, gamma)
    args = dict(row.args)
    return O.fit_posterior(row.dist, args, below, 1.0), O.fit_posterior(row.dist, args, above, 1.0)


def _check_problem(eng, fits, row, hist, ids, C, seed, winners, rs, what, **kw):
    """Re-draw the candidates of (row, id) for every id in ``ids`` and check
    the production ``winners`` (one value per id) against the oracle."""
    from hyperopt_amd.engine import LevelProblem
    pb, pa = _oracle_fits(row, hist)
    res, cand, l, g = eng.run([LevelProblem(fits.get(row), row.index, ids)], C, seed, want_lg=True,
                              return_cand=True)
    for i, (nid, win) in enumerate(zip(ids, winners)):
        tag = '%s id %d' % (what, nid)
        if row.categorical:
            c = cand[i].astype(np.int64)
            lr, gr = O.categorical_lpdf(c, pb.params[0]), O.categorical_lpdf(c, pa.params[0])
            np.testing.assert_allclose(l[i], lr, rtol=1e-12, atol=1e-12, err_msg=tag)
            np.testing.assert_allclose(g[i], gr, rtol=1e-12, atol=1e-12, err_msg=tag)
            assert int(win) == int(c[int(np.argmax(lr - gr))]), tag          # exact (np.argmax)
            continue
        q = pb.q
        tol = TOL64 if q is not None else TOL32
        check_winner([win], cand[i], l[i], g[i], pb.lpdf, pa.lpdf, len(pa.params[0]), tol, rs, tag, **kw)
    return cand


# ----------------------------------------------------------------- config 3
def _tree_loss_rf(v, tid):
    import bench
    return bench.rf_loss(v, tid)


@pytest.mark.parametrize('branch', ['svm', 'rf'])
def test_config3_suggest_full_size(branch):
    """Config 3: tpe.suggest on the conditional tree, 10k-trial history,
    2^20 candidates — the bench workload (svm/rbf branch) and a history that
    steers the tree to the rf branch (quantized labels qU(10,500,10) and
    qU(2,30,1) at 2^20 candidates)."""
    import bench
    from hyperopt_amd import history as H, tpe
    from hyperopt_amd.engine import get_engine
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED,
                                        loss=None if branch == 'svm' else _tree_loss_rf)
    C = bench.C_PER_GPU
    new_id = bench.N_HISTORY
    seed = 4242
    doc = tpe.suggest([new_id], domain, trials, seed, n_EI_candidates=C)[0]
    trials.assert_valid_trial(doc)
    vals = {k: v[0] for k, v in doc['misc']['vals'].items() if v}
    assert vals['model'] == {'svm': 0, 'rf': 1}[branch], vals
    eng = get_engine()
    hist = H.extract(domain, trials)
    fits = tpe._Fits(domain.table, hist, H.split_below(hist, 0.25), 1.0, eng)
    rs = np.random.RandomState(3)
    for label, v in sorted(vals.items()):
        _check_problem(eng, fits, domain.table.by_label[label], hist, [new_id], C, seed, [v], rs,
                       'config3/%s %s' % (branch, label))
    again = tpe.suggest([new_id], domain, trials, seed, n_EI_candidates=C)[0]
    assert again['misc']['vals'] == doc['misc']['vals']                      # deterministic
    # the stage profiler (bench.py's roofline) times the production flow and
    # changes nothing: tables + tabulated sampling with early selection, no
    # select stage
    eng.profile = {}
    try:
        prof_doc = tpe.suggest([new_id], domain, trials, seed, n_EI_candidates=C)[0]
        prof = eng.profile
    finally:
        eng.profile = None
    assert prof_doc['misc']['vals'] == doc['misc']['vals']
    assert 'k_tables' in prof and 'k_sample' in prof and 'k_select' not in prof, sorted(prof)
    ms, units, ce = prof['k_sample'][0][:3]
    if branch == 'svm':                        # (the log-polynomial pass, timed by its own launch events)
        assert 0 < prof['k_sample'][0][3] <= ms, prof['k_sample'][0]
    # units: the candidates the sample kernels draw (lazy categoricals are scanned by the table stage)
    n_cont = sum(1 for k in vals if not domain.table.by_label[k].categorical)
    assert ms > 0 and n_cont * C <= units <= len(vals) * C and ce > 0, prof['k_sample']


# ----------------------------------------------------------------- config 4
def test_config4_batched_full_size():
    """Config 4: one batched suggest of 4096 new_ids x 4096 candidates over a
    20-dim U(-5,5) space and a 10k-trial history (pooled labels, u64
    atomicMax winners).  Every id: 20 in-bounds values, identical on a re-run
    and identical to the id's single-id suggest for a sample of ids; 64
    seeded (id, dim) pairs against the oracle."""
    import bench
    from hyperopt_amd import history as H, tpe
    from hyperopt_amd.engine import get_engine
    labels = ['x%02d' % i for i in range(20)]
    hist = bench.soa_history(labels, 10000, bench.SEED, lambda v: sum((x - 0.3) ** 2 for x in v.values()))
    table = bench.flat_uniform_table(labels)
    ids = np.arange(10000, 10000 + 4096)
    C, seed = 4096, 777
    got = tpe.suggest_choices(table, hist, ids, seed, n_EI_candidates=C)
    assert len(got) == len(ids)
    arr = np.array([[d[k] for k in labels] for d in got], dtype=np.float64)
    assert np.all(np.isfinite(arr)) and np.all(arr >= -5) and np.all(arr < 5)
    assert len(np.unique(arr[:, 0])) > 3000             # ids draw from their own streams
    again = tpe.suggest_choices(table, hist, ids, seed, n_EI_candidates=C)
    assert [[d[k] for k in labels] for d in again] == arr.tolist()
    eng = get_engine()
    fits = tpe._Fits(table, hist, H.split_below(hist, 0.25), 1.0, eng)
    rs = np.random.RandomState(5)
    pick = rs.choice(len(ids) * len(labels), 64, replace=False)
    by_label = {}
    for p in pick:
        by_label.setdefault(labels[p % len(labels)], []).append(p // len(labels))
    for label, rows in sorted(by_label.items()):
        rows = sorted(rows)
        _check_problem(eng, fits, table.by_label[label], hist, ids[rows], C, seed,
                       [got[r][label] for r in rows], rs, 'config4 %s' % label, k_top=256, n_rand=256)
    from hyperopt_amd.engine import LevelProblem
    for r in rs.choice(len(ids), 3, replace=False):
        # a single-id suggest of the same id draws the same candidates; its
        # winner scores like the pooled one (both in the eps-tie set)
        one = tpe.suggest_choices(table, hist, [ids[r]], seed, n_EI_candidates=C)[0]
        for k in labels:
            row = table.by_label[k]
            _, cand, l, g = eng.run([LevelProblem(fits.get(row), row.index, [ids[r]])], C, seed, want_lg=True,
                                    return_cand=True)
            s = l[0] - g[0]
            i1, i2 = np.nonzero(cand[0] == one[k])[0], np.nonzero(cand[0] == got[r][k])[0]
            assert len(i1) and len(i2), (k, r)
            assert abs(s[i1[0]] - s[i2[0]]) <= 4 * TOL32 * max(1.0, abs(s[i2[0]])), (k, r)


# ----------------------------------------------------------------- config 5
def test_config5_device_fit_full_size():
    """Config 5: 1000-dim U(-5,5) space, 100k-trial history, C = 4096, one
    native call: every below side fitted on the host, every above mixture on
    the device (resident value order: chunk sort + merges on the first call,
    compaction, chunked build).  For 20 sampled
    dims the device-fitted rows (mu, sigma, weights, wide list) match the
    oracle's adaptive_parzen_normal, and the production winner is checked
    against the oracle's lpdf / eps-tie set."""
    import bench
    from hyperopt_amd import history as H, tpe
    from hyperopt_amd.engine import LevelProblem, get_engine
    D, N, C, seed = 1000, 100000, 4096, 99
    labels = ['x%04d' % i for i in range(D)]
    hist = bench.soa_history(labels, N, bench.SEED, lambda v: np.zeros(N))
    hist.losses[:] = np.random.RandomState(bench.SEED + 1).uniform(size=N) + 1e-9 * np.arange(N)
    table = bench.flat_uniform_table(labels)
    eng = get_engine()
    assert N >= eng.device_fit_min
    eng.last_tree_path = None
    got = tpe.suggest_choices(table, hist, [N], seed, n_EI_candidates=C)[0]
    assert eng.last_tree_path == (0, 1)                         # one native call, one level
    v = np.array([got[k] for k in labels])
    assert np.all(np.isfinite(v)) and np.all(v >= -5) and np.all(v < 5)
    rs = np.random.RandomState(8)
    sample = sorted(rs.choice(D, 20, replace=False))
    fits = tpe._Fits(table, hist, H.split_below(hist, 0.25), 1.0, eng)
    rows = [table.by_label[labels[i]] for i in sample]
    posts = [fits.get(r) for r in rows]
    assert all(p.above_dev is not None for p in posts)          # the device fit is what runs
    eng.run([LevelProblem(p, r.index, [N]) for p, r in zip(posts, rows)], C, seed)
    prob, comp32 = eng.device_tables()
    for j, r in enumerate(rows):
        pb, pa = _oracle_fits(r, hist)
        w_o, mu_o, sg_o = pa.params
        p = prob[j]
        K = int(p['above_len'])
        assert K == len(mu_o), (r.label, K, len(mu_o))
        rw = comp32[int(p['above_off']):int(p['above_off']) + K].astype(np.float64)
        mu = rw[:, 0] + rw[:, 1]
        np.testing.assert_allclose(mu, mu_o, rtol=1e-12, atol=1e-12, err_msg=r.label)
        np.testing.assert_allclose(O_A_SCALE / rw[:, 2], np.maximum(sg_o, O.EPS), rtol=2e-7, err_msg=r.label)
        # c_k = log2(w_k / sigma_k) - shift: a constant offset from the oracle's
        lw = np.log2(w_o) - np.log2(np.maximum(sg_o, O.EPS))
        narrow = np.isfinite(rw[:, 3])
        d = rw[narrow, 3] - lw[narrow]
        assert d.max() - d.min() <= 4e-6, (r.label, d.max() - d.min())
        nw = int(p['wide_len'])
        assert 1 <= nw <= 16 and np.count_nonzero(~narrow) == nw
        wide = comp32[int(p['wide_off']):int(p['wide_off']) + nw].astype(np.float64)
        for wr in wide:                                          # each wide row is a sorted row
            at = np.nonzero((rw[:, 0] == wr[0]) & (rw[:, 1] == wr[1]) & (rw[:, 2] == wr[2]) & ~narrow)[0]
            assert len(at) == 1, r.label
            assert abs(wr[3] - lw[at[0]] - np.median(d)) <= 4e-6, r.label
        _check_problem(eng, fits, r, hist, [N], C, seed, [got[r.label]], rs, 'config5 %s' % r.label,
                       k_top=64, n_rand=256)


O_A_SCALE = float(np.sqrt(0.5 / np.log(2.0)))      # sqrt(log2(e) / 2): a_k = A / max(sigma_k, EPS)


def test_device_value_order_incremental():
    """The resident device value order of device-fitted labels (tpe_fit_above:
    chunk sort -> merge passes -> merge into the resident order, or DELTA MODE:
    at most TPE_FIT_DELTA_MAX new observations read beside the order as one
    virtual order, no merge) over suggests that append 200, 1, 1, 10, 5, 16
    and 1 observations (FMinIter appends one per suggest): after every suggest
    each label's order is np.argsort(kind='stable') of the kernel coordinate of
    the observations it holds (ties by tid order; repeated values included) —
    all of them after a merge, the last merged prefix in delta mode — the
    suggestion equals a from-scratch fit's (a full sort and merge) bit for bit,
    and at the end the device rows match the oracle's adaptive_parzen_normal."""
    from hyperopt_amd import _native as N, base, devhist, hp, history as H, tpe
    from hyperopt_amd.engine import LevelProblem, get_engine
    eng = get_engine()
    N0, C, seed = 20000, 4096, 17
    steps = [0, 200, 1, 1, 10, 5, 16, 1]
    Nt = N0 + sum(steps)
    assert N0 - 25 >= eng.device_fit_min and N.FIT_DELTA_MAX == 16
    table = base.Domain(lambda d: 0.0, {'u': hp.uniform('u', -5, 5), 'l': hp.loguniform('l', -3, 2)}).table
    rs = np.random.RandomState(3)
    u = rs.uniform(-5, 5, Nt)
    u[::7] = np.round(u[::7], 1)                     # repeated values: ties broken by tid order
    u[N0 + 200:N0 + 202] = u[5]                      # new observations equal to resident ones
    lv = np.exp(rs.uniform(-3, 2, Nt))
    lv[::13] = np.round(lv[::13], 2)
    tids = np.arange(Nt, dtype=np.int64)
    losses = rs.uniform(size=Nt) + 1e-9 * tids
    losses[N0 + 210] = -1.0                          # a new observation in the below set (delta mode)
    dev = {}                                         # the Trials cache's device state, kept across suggests
    vals = {'u': u, 'l': lv}

    def hist_of(n, d):
        return H.History(tids[:n], losses[:n].copy(), {k: (tids[:n], v[:n]) for k, v in vals.items()}, dev=d)
    n, held, deltas = N0, N0, 0
    for s, inc in enumerate(steps):
        n += inc
        if n - held > N.FIT_DELTA_MAX:
            held = n                                 # a merge: the order holds all of them
        else:
            deltas += n > held
        hist = hist_of(n, dev)
        got = tpe.suggest_choices(table, hist, [n], seed + s, n_EI_candidates=C)[0]
        dc = devhist.columns(hist, eng.device)
        for label, v in vals.items():
            o = dc.order(label)
            assert o.n == held, (label, s, o.n, held)
            t = np.log(v[:held]) if label == 'l' else v[:held]
            keys, idx = o.host()
            want = np.argsort(t, kind='stable')
            np.testing.assert_array_equal(idx, want, err_msg='%s step %d' % (label, s))
            np.testing.assert_array_equal(keys, t[want], err_msg='%s step %d' % (label, s))
        fresh = tpe.suggest_choices(table, hist_of(n, {}), [n], seed + s, n_EI_candidates=C)[0]
        assert got == fresh, (s, n, got, fresh)
    assert deltas == 4 and n == Nt == held
    # the device rows of the final history against the oracle
    hist = hist_of(Nt, dev)
    fits = tpe._Fits(table, hist, H.split_below(hist, 0.25), 1.0, eng)
    rows = [table.by_label[k] for k in ('l', 'u')]
    posts = [fits.get(r) for r in rows]
    assert all(p.above_dev is not None and p.above_dev[3].n == Nt for p in posts)
    eng.run([LevelProblem(p, r.index, [Nt]) for p, r in zip(posts, rows)], C, seed)
    prob, comp32 = eng.device_tables()
    for j, r in enumerate(rows):
        w_o, mu_o, sg_o = _oracle_fits(r, hist)[1].params
        p = prob[j]
        K = int(p['above_len'])
        assert K == len(mu_o), (r.label, K, len(mu_o))
        rw = comp32[int(p['above_off']):int(p['above_off']) + K].astype(np.float64)
        np.testing.assert_allclose(rw[:, 0] + rw[:, 1], mu_o, rtol=1e-12, atol=1e-12, err_msg=r.label)
        np.testing.assert_allclose(O_A_SCALE / rw[:, 2], np.maximum(sg_o, O.EPS), rtol=2e-7, err_msg=r.label)


# ----------------------------------------------------------------- config 2
@pytest.mark.parametrize('seed', [2024, 77])
def test_config2_suggest_full_size(seed):
    """Config 2: tpe.suggest on the 10-dim mixed space (3 uniform, 3
    loguniform, 2 quniform, 2 choice) with the bench's 1000-trial history and
    C = 10,000 (the native tree path with caller-made fits of the quantized
    labels): every one of the 10 winners against the oracle — lpdf within
    1e-5 (continuous, fp32) / 1e-9 (quantized, f64), the winner in the eps-tie
    set, categorical choices exact."""
    import bench
    from hyperopt_amd import history as H, hp, tpe
    from hyperopt_amd.engine import get_engine
    domain, trials = bench.mixed10_history(1000, bench.SEED)
    C, new_id = 10000, 1000
    eng = get_engine()
    eng.last_tree_path = None
    doc = tpe.suggest([new_id], domain, trials, seed, n_EI_candidates=C)[0]
    trials.assert_valid_trial(doc)
    assert eng.last_tree_path is not None                    # the production (native tree) path ran
    vals = {k: v[0] for k, v in doc['misc']['vals'].items() if v}
    assert sorted(vals) == sorted(bench.mixed10_space(hp)), vals
    hist = H.extract(domain, trials)
    fits = tpe._Fits(domain.table, hist, H.split_below(hist, 0.25), 1.0, eng)
    rs = np.random.RandomState(seed)
    for label, v in sorted(vals.items()):
        _check_problem(eng, fits, domain.table.by_label[label], hist, [new_id], C, seed, [v], rs,
                       'config2 %s' % label, k_top=2048, n_rand=2048)
