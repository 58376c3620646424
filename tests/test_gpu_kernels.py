"""GPU parity of the HIP kernels (through the C-ABI) against the reference's
golden vectors and the CPU oracle.

Tolerances (north_star):
  fp32 lpdf:  |gpu - ref| <= 1e-5 * max(|ref|, 1)
  fp64 lpdf:  |gpu - ref| <= 1e-9 * max(|ref|, 1)
  argmax:     the GPU index lies in the reference's eps-tie set
              {i : score_ref[i] >= max - eps}, eps = 4 * lpdf bound; equal when
              that set has one element.  Categorical choices are bit-exact.
"""
import numpy as np
import pytest

from oracle import tpe_oracle as O

pytestmark = pytest.mark.gpu

TOL = {'fp32': 1e-5, 'fp64': 1e-9}


@pytest.fixture(scope='module')
def engine():
    from hyperopt_amd.engine import Engine
    return Engine(precision='fp32')


@pytest.fixture(params=['tables', 'per_candidate'])
def scoring(request, monkeypatch):
    """Tabulated scoring (include/tpe_hip.h "Tabulated scoring", the default for
    large candidate sets) and the per-candidate path it replaces (TPE_TABLES=0:
    sorted candidates, pruned above kernel, finalize) — both must hold parity."""
    if request.param == 'per_candidate':
        monkeypatch.setenv('TPE_TABLES', '0')
    return request.param


def _post(case):
    from hyperopt_amd import parzen
    return parzen.fit_posterior(case['dist'], case['args'], np.asarray(case['below']),
                                np.asarray(case['above']), 1.0)


def _check_lpdf(got, ref, tol, what):
    ref = np.asarray(ref)
    fin = np.isfinite(ref)
    err = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1.0)
    assert err.max() <= tol, (what, float(err.max()), int(np.argmax(err)))
    # reference -inf (log of an underflowed mass): GPU gives -inf or a huge negative
    assert np.all((got[~fin] == ref[~fin]) | (got[~fin] < -700)), what


def _check_argmax(idx, l_ref, g_ref, tol, what):
    score = np.asarray(l_ref) - np.asarray(g_ref)
    eps = 4 * tol * max(1.0, float(np.max(np.abs(l_ref))), float(np.max(np.abs(g_ref))))
    m = np.nanmax(score)
    ties = np.nonzero(score >= m - eps)[0]
    assert idx in ties, (what, idx, int(np.argmax(score)), ties[:10])
    if len(ties) == 1:
        assert idx == int(np.argmax(score))


@pytest.mark.parametrize('precision', ['fp32', 'fp64'])
def test_kernel_vectors_injected(golden, engine, precision):
    """Reference-fitted mixtures, reference-drawn candidates -> l, g, argmax."""
    from hyperopt_amd.engine import LevelProblem
    engine.set_precision(precision)
    for case in golden('kernel_vectors.json'):
        post = _post(case)
        cand = np.asarray(case['cand'], dtype=np.float64)
        lp = LevelProblem(post, 3, [7], inject=cand[None, :])
        res, l, g = engine.run([lp], len(cand), seed=5, want_lg=True)
        tol = TOL[precision] if post.family in (0, 1) else 1e-9
        _check_lpdf(l[0], case['l'], tol, (case['dist'], precision, 'l'))
        _check_lpdf(g[0], case['g'], tol, (case['dist'], precision, 'g'))
        _check_argmax(int(res[0]['idx']), case['l'], case['g'], tol, (case['dist'], precision))
        assert res[0]['value'] == cand[int(res[0]['idx'])]
        if post.family == 4:
            assert int(res[0]['idx']) == case['best']
    engine.set_precision('fp32')


def test_lpdf_unit_vectors(golden, engine):
    """Every GMM1_lpdf / LGMM1_lpdf golden case (bounded, unbounded, q) at fp64
    and fp32, using the case's mixture as both below and above."""
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    for precision in ('fp64', 'fp32'):
        engine.set_precision(precision)
        for case in golden('unit_vectors.json')['lpdf']:
            if case['fn'] == 'categorical_lpdf':
                continue
            log = case['fn'] == 'LGMM1_lpdf'
            q = case['q']
            fam = (3 if q else 1) if log else (2 if q else 0)
            mix = (np.asarray(case['w']), np.asarray(case['mu']), np.asarray(case['sigma']))
            post = parzen.Posterior('x', fam, case['low'], case['high'], q, mix, mix)
            x = np.asarray(case['x'])
            res, l, g = engine.run([LevelProblem(post, 0, [0], inject=x[None, :])], len(x), 1, want_lg=True)
            tol = TOL[precision] if not q else 1e-9
            _check_lpdf(l[0], case['out'], tol, (case['fn'], q, case['low'], precision))
            # below (exact two-pass) and above (split partial sums) paths agree
            np.testing.assert_allclose(l[0], g[0], rtol=tol, atol=tol)
    engine.set_precision('fp32')


def test_philox_sampler_distribution(engine):
    """Device draws follow the below mixture: bounds, quantisation, and the
    exact mixture CDF (Kolmogorov distance), incl. truncation (the rejection
    loop of tpe.py:82-87 is sampled by inversion)."""
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    from scipy.special import erf
    rs = np.random.RandomState(3)
    C = 1 << 18
    for dist, args in (('uniform', dict(low=-2.0, high=3.0)), ('normal', dict(mu=0.5, sigma=2.0)),
                       ('loguniform', dict(low=-4.0, high=1.0)), ('quniform', dict(low=0.0, high=10.0, q=0.5)),
                       ('randint', dict(upper=5)), ('categorical', dict(p=[0.1, 0.5, 0.4], upper=3))):
        if dist in ('randint', 'categorical'):
            below = rs.randint(0, args['upper'], 9)
            above = rs.randint(0, args['upper'], 50)
        else:
            lo, hi = (args['low'], args['high']) if 'low' in args else (-3.0, 4.0)
            below = rs.uniform(lo, hi, 9)
            above = rs.uniform(lo, hi, 50)
            if dist == 'loguniform':
                below, above = np.exp(below), np.exp(above)
        post = parzen.fit_posterior(dist, args, below, above, 1.0)
        for precision in ('fp32', 'fp64'):
            engine.set_precision(precision)
            res, cand = engine.run([LevelProblem(post, 1, [0])], C, seed=99, return_cand=True)
            x = cand[0]
            assert np.all(np.isfinite(x))
            if post.family == 4:
                freq = np.bincount(x.astype(int), minlength=post.upper) / C
                np.testing.assert_allclose(freq, post.below[0], atol=5e-3)
                continue
            w, mu, sg = post.below
            if post.low is not None:
                t = np.log(x) if post.family in (1, 3) else x
                if post.q is None:
                    assert t.min() >= post.low and t.max() < post.high, dist
            if post.q is not None:
                np.testing.assert_allclose(np.round(x / post.q) * post.q, x, rtol=0, atol=0)
                continue
            t = np.sort(np.log(x) if post.family == 1 else x)
            grid = t[:: C // 512]
            Phi = lambda z: 0.5 * (1 + erf(z / np.sqrt(2)))
            if post.low is None:
                F = (w[None, :] * Phi((grid[:, None] - mu) / sg)).sum(1)
            else:
                mass = Phi((post.high - mu) / sg) - Phi((post.low - mu) / sg)
                F = (w * (Phi((grid[:, None] - mu) / sg) - Phi((post.low - mu) / sg))).sum(1) / (w * mass).sum()
            Femp = (np.arange(0, C, C // 512) + 1) / C
            assert np.max(np.abs(F - Femp)) < 6e-3, (dist, precision, float(np.max(np.abs(F - Femp))))
    engine.set_precision('fp32')


def test_ordered_draws_distribution(engine, monkeypatch):
    """TPE_BATCH_ORDERED_DRAWS: pruned (sorted) problems draw ordered
    candidates (uniform order statistics through the mixture, include/tpe_hip.h
    "Ordered draws") instead of i.i.d. draws + sort: the draws follow the exact
    below-mixture CDF, stay in bounds, come out sorted inside each component's
    run, are identical for every shard count, and pick a winner of the same
    quality as the default i.i.d. draws."""
    import os
    from hyperopt_amd import _native as N
    from hyperopt_amd import parzen
    from hyperopt_amd.dist import combine_results, shard_range
    from hyperopt_amd.engine import LevelProblem
    from scipy.special import erf
    monkeypatch.setenv('TPE_TABLES', '0')          # ordered draws replace the sort of per-candidate scoring
    rs = np.random.RandomState(8)
    C = 1 << 18
    Phi = lambda z: 0.5 * (1 + erf(z / np.sqrt(2)))
    for dist, args in (('uniform', dict(low=-2.0, high=3.0)), ('normal', dict(mu=0.5, sigma=2.0)),
                       ('loguniform', dict(low=-4.0, high=1.0)), ('lognormal', dict(mu=0.0, sigma=1.0))):
        lo, hi = (args['low'], args['high']) if 'low' in args else (-3.0, 4.0)
        below, above = rs.uniform(lo, hi, 20), rs.uniform(lo, hi, 3000)
        if dist.startswith('log'):
            below, above = np.exp(below), np.exp(above)
        post = parzen.fit_posterior(dist, args, below, above, 1.0)
        res_iid = engine.run([LevelProblem(post, 1, [0])], C, seed=99)
        os.environ['TPE_DEBUG_FLAGS'] = str(N.BATCH_ORDERED_DRAWS)
        try:
            res, cand, l, g = engine.run([LevelProblem(post, 1, [0])], C, seed=99, want_lg=True, return_cand=True)
            if dist == 'uniform':          # shard-invariant draws (global 64-index prefix blocks)
                parts, cands = [], []
                for r in range(3):
                    a0, a1 = shard_range(C, r, 3)
                    pr, cr = engine.run([LevelProblem(post, 1, [0])], a1 - a0, seed=99, cand_base=a0,
                                        n_cand_global=C, return_cand=True)
                    parts.append(pr)
                    cands.append(cr)
                np.testing.assert_array_equal(np.concatenate(cands, axis=1), cand)
                comb = combine_results(np.stack(parts))
                np.testing.assert_allclose(comb['score'], res['score'], rtol=1e-6, atol=1e-6)
        finally:
            os.environ.pop('TPE_DEBUG_FLAGS', None)
        x = cand[0]
        assert np.all(np.isfinite(x)) and np.all(np.isfinite(l[0])) and np.all(np.isfinite(g[0])), dist
        t = np.log(x) if post.family == 1 else x
        if post.low is not None:
            assert t.min() >= post.low and t.max() < post.high, dist
        # sorted inside runs: one descent per component boundary at most
        assert np.count_nonzero(np.diff(t) < -1e-4 * (t.max() - t.min())) <= len(post.below[0]), dist
        w, mu, sg = post.below
        grid = np.sort(t)[:: C // 512]
        if post.low is None:
            F = (w[None, :] * Phi((grid[:, None] - mu) / sg)).sum(1)
        else:
            mass = Phi((post.high - mu) / sg) - Phi((post.low - mu) / sg)
            F = (w * (Phi((grid[:, None] - mu) / sg) - Phi((post.low - mu) / sg))).sum(1) / (w * mass).sum()
        Femp = (np.arange(0, C, C // 512) + 1) / C
        assert np.max(np.abs(F - Femp)) < 6e-3, (dist, float(np.max(np.abs(F - Femp))))
        score = l[0] - g[0]
        assert int(res[0]['idx']) == int(np.argmax(score)) and res[0]['value'] == x[int(res[0]['idx'])]
        # same law as the i.i.d. draws: the best score agrees up to sampling noise
        assert abs(res_iid[0]['score'] - res[0]['score']) <= 0.05 * max(1.0, abs(res[0]['score'])), dist


def test_pooled_label_matches_single_problems(engine, scoring):
    """A pruned label active for several ids is pooled (one sort for all its
    problems, per-problem winners by atomicMax): every id draws what it draws
    alone, its winner lies in the oracle's eps-tie set of those draws, the
    reported l and g are the oracle's at the winner, and a rerun is
    bit-identical."""
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    rs = np.random.RandomState(17)
    for dist, args in (('uniform', dict(low=-5.0, high=5.0)), ('loguniform', dict(low=-4.0, high=3.0))):
        below, above = rs.uniform(-4, 3, 20), rs.uniform(-4, 3, 3000)
        if dist == 'loguniform':
            below, above = np.exp(below), np.exp(above)
        post = parzen.fit_posterior(dist, args, below, above, 1.0)
        lpdf = O.lgmm1_lpdf if dist == 'loguniform' else O.gmm1_lpdf
        ids = list(range(40, 49))
        C = 3000
        res, cand, l, g = engine.run([LevelProblem(post, 2, ids)], C, seed=5, want_lg=True, return_cand=True)
        again = engine.run([LevelProblem(post, 2, ids)], C, seed=5)
        np.testing.assert_array_equal(again, res)
        for i, nid in enumerate(ids):
            one, cand1 = engine.run([LevelProblem(post, 2, [nid])], C, seed=5, return_cand=True)
            np.testing.assert_array_equal(cand1[0], cand[i])               # the id's own Philox stream
            lb = lpdf(cand[i], *post.below, low=post.low, high=post.high)
            la = lpdf(cand[i], *post.above, low=post.low, high=post.high)
            _check_lpdf(l[i], lb, 1e-5, (dist, 'pooled l'))
            _check_lpdf(g[i], la, 1e-5, (dist, 'pooled g'))
            k = int(res[i]['idx'])
            _check_argmax(k, lb, la, 1e-5, (dist, 'pooled'))
            assert res[i]['value'] == cand[i][k] and res[i]['global_idx'] == k
            assert abs(res[i]['l'] - lb[k]) <= 1e-5 * max(1.0, abs(lb[k]))
            assert abs(res[i]['g'] - la[k]) <= 1e-5 * max(1.0, abs(la[k]))
            assert abs(res[i]['score'] - one[0]['score']) <= 4e-5 * max(1.0, abs(one[0]['score']))


def test_lazy_categorical_matches_full_scan(engine):
    """TPE_F_CAT_LAZY: the select stage scans draws in index order until no
    undrawn category can win; the result equals the full per-candidate path
    (forced by asking for the candidates) — common, rare-but-lazy (several
    rounds), too-rare (not lazy), undrawable and all-tied categories."""
    from hyperopt_amd import _native as N
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    cases = [([0.2, 0.5, 0.3], [0.4, 0.3, 0.3]),
             ([0.9997, 0.0003], [0.9999999, 1e-7]),
             ([0.99999, 0.00001], [0.99999999, 1e-8]),
             ([0.5, 0.0, 0.5], [0.3, 0.4, 0.3]),
             ([0.25, 0.25, 0.5], [0.25, 0.25, 0.5])]
    for pb, pa in cases:
        post = parzen.Posterior('categorical', N.FAM_CATEGORICAL, None, None, None, (np.array(pb),),
                                (np.array(pa),), len(pb))
        for C in (1000, 1 << 18):
            lazy = engine.run_level([LevelProblem(post, 4, [0, 1, 2])], C, seed=3)
            full, cand = engine.run([LevelProblem(post, 4, [0, 1, 2])], C, seed=3, return_cand=True)
            np.testing.assert_array_equal(lazy, full)
            for k in range(3):
                assert full[k]['value'] == cand[k][int(full[k]['idx'])]


def test_sharding_matches_single_device(engine, scoring):
    """Philox counters are global candidate indices, so every shard count draws
    the same candidate set.  Scores agree to fp32 rounding (pruned windows and
    split groupings follow the shard's own sorted waves), the argmax agrees up
    to ties within that rounding, and a repeated run is bit-identical."""
    from hyperopt_amd import parzen
    from hyperopt_amd.dist import combine_results, shard_range
    from hyperopt_amd.engine import LevelProblem
    rs = np.random.RandomState(5)
    post = parzen.fit_posterior('uniform', dict(low=-5.0, high=5.0), rs.uniform(-5, 5, 20),
                                rs.uniform(-5, 5, 3000), 1.0)
    C = 100000
    full, cand, l, g = engine.run([LevelProblem(post, 2, [0, 1, 2])], C, seed=123, want_lg=True, return_cand=True)
    again = engine.run([LevelProblem(post, 2, [0, 1, 2])], C, seed=123)
    np.testing.assert_array_equal(again, full)
    for world in (2, 3, 4, 8):
        parts, cands = [], []
        for r in range(world):
            lo, hi = shard_range(C, r, world)
            res_r, cand_r = engine.run([LevelProblem(post, 2, [0, 1, 2])], hi - lo, seed=123, cand_base=lo,
                                       n_cand_global=C, return_cand=True)
            parts.append(res_r)
            cands.append(cand_r)
        np.testing.assert_array_equal(np.concatenate(cands, axis=1), cand)      # identical draws
        comb = combine_results(np.stack(parts))
        np.testing.assert_allclose(comb['score'], full['score'], rtol=1e-6, atol=1e-6)
        for p in range(3):
            score = l[p] - g[p]
            ties = np.nonzero(score >= score.max() - 1e-5)[0]
            assert comb['global_idx'][p] in ties
            assert comb['value'][p] == cand[p][comb['global_idx'][p]]


def test_large_config3_shaped_problem(engine, scoring):
    """Config-3-sized problem (C = 2^20 candidates, 10k-trial history):
    size-independent checks — lpdf of a random subset vs the oracle, argmax is
    the max of all returned scores, and a rerun is bit-identical."""
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    rs = np.random.RandomState(11)
    obs = np.exp(rs.uniform(-5, 5, 10000))
    post = parzen.fit_posterior('loguniform', dict(low=-5.0, high=5.0), obs[:25], obs[25:], 1.0)
    C = 1 << 20
    res, cand, l, g = engine.run([LevelProblem(post, 0, [0])], C, seed=7, want_lg=True, return_cand=True)
    score = l[0] - g[0]
    assert int(res[0]['idx']) == int(np.argmax(score))
    sub = rs.choice(C, 2000, replace=False)
    lb = O.lgmm1_lpdf(cand[0][sub], *post.below, low=-5.0, high=5.0)
    la = O.lgmm1_lpdf(cand[0][sub], *post.above, low=-5.0, high=5.0)
    _check_lpdf(l[0][sub], lb, 1e-5, 'l')
    _check_lpdf(g[0][sub], la, 1e-5, 'g')
    res2 = engine.run([LevelProblem(post, 0, [0])], C, seed=7)
    assert res2[0]['idx'] == res[0]['idx'] and res2[0]['score'] == res[0]['score']


def test_pruning_and_underflow_extremes(engine, scoring):
    """Above mixtures large enough to be pruned, clustered observations plus
    isolated wide components, and candidates far in the tails (the fixed-shift
    sum underflows there and the max-shifted fallback takes over)."""
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    rs = np.random.RandomState(21)
    obs = np.concatenate([rs.normal(0.0, 0.05, 3000), rs.normal(3.0, 0.01, 500), [-40.0, 25.0]])
    rs.shuffle(obs)
    for dist, args in (('normal', dict(mu=0.0, sigma=5.0)), ('uniform', dict(low=-50.0, high=50.0))):
        post = parzen.fit_posterior(dist, args, obs[:20], obs[20:], 1.0)
        x = np.concatenate([rs.uniform(-1, 4, 3000), [-49.9, -40.0, -20.0, 0.0, 3.0, 24.9, 49.9],
                            np.linspace(-45, 45, 1000)])
        if dist == 'normal':
            x = np.concatenate([x, [-300.0, 300.0, 1e4]])
        low, high = (post.low, post.high)
        lb = O.gmm1_lpdf(x, *post.below, low=low, high=high)
        la = O.gmm1_lpdf(x, *post.above, low=low, high=high)
        res, l, g = engine.run([LevelProblem(post, 0, [0], inject=x[None, :])], len(x), 1, want_lg=True)
        _check_lpdf(l[0], lb, 1e-5, (dist, 'l'))
        _check_lpdf(g[0], la, 1e-5, (dist, 'g'))
        _check_argmax(int(res[0]['idx']), lb, la, 1e-5, dist)


def _device_post(engine, dist, args, obs, bidx):
    """Posterior whose above mixture is fitted on the device (tpe_fit_above)."""
    from hyperopt_amd import devhist, history, parzen
    hist = history.History(np.arange(len(obs)), np.zeros(len(obs)), {'x': (np.arange(len(obs)), obs)})
    dc = devhist.columns(hist, engine.device)
    col = dc.column('x', np.log(obs) if dist in ('loguniform', 'lognormal') else obs)   # kernel coordinate
    return parzen.fit_posterior(dist, args, obs[bidx], None, 1.0,
                                above_dev=(col, len(obs), bidx, dc.order('x'))), col


@pytest.mark.parametrize('dist,args', [('uniform', dict(low=-5.0, high=5.0)),
                                       ('loguniform', dict(low=-4.0, high=3.0)),
                                       ('normal', dict(mu=1.0, sigma=3.0)),
                                       ('lognormal', dict(mu=0.0, sigma=1.0))])
def test_device_fit_matches_oracle(engine, dist, args, scoring):
    """Device Parzen fit of the above mixture (gather -> segmented sort ->
    build) against the oracle's adaptive_parzen_normal + GMM1/LGMM1 lpdf, on
    sampled and injected candidates; the below side stays the host fit, so the
    draws equal the host-fit run's and the argmax lies in its eps-tie set."""
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    rs = np.random.RandomState(31)
    n = 20000
    if dist == 'uniform':     # clustered + isolated observations: wide components
        obs = np.clip(np.concatenate([rs.normal(-2, 0.05, n // 2), rs.uniform(-5, 5, n // 2 - 3),
                                      [-4.9, 4.95, 0.0]]), -5, 5)
    elif dist == 'loguniform':
        obs = np.exp(rs.uniform(-4, 3, n))
    elif dist == 'normal':
        obs = rs.normal(1.0, 3.0, n)
    else:
        obs = np.exp(rs.normal(0, 1, n))
    rs.shuffle(obs)
    bidx = np.sort(rs.choice(n, 25, replace=False)).astype(np.int32)
    m = np.zeros(n, bool)
    m[bidx] = True
    host = parzen.fit_posterior(dist, args, obs[m], obs[~m], 1.0)
    dev, _ = _device_post(engine, dist, args, obs, bidx)
    logf = dist in ('loguniform', 'lognormal')
    tr = np.log if logf else (lambda v: v)
    pmu = 0.5 * (args['low'] + args['high']) if 'low' in args else args['mu']
    psig = (args['high'] - args['low']) if 'low' in args else args['sigma']
    above = O.adaptive_parzen_normal(tr(obs[~m]), 1.0, pmu, psig)
    lpdf = O.lgmm1_lpdf if logf else O.gmm1_lpdf
    low, high = host.low, host.high
    C = 1 << 16
    res_d, cand_d, l_d, g_d = engine.run([LevelProblem(dev, 0, [3])], C, seed=9, want_lg=True, return_cand=True)
    res_h, cand_h, l_h, g_h = engine.run([LevelProblem(host, 0, [3])], C, seed=9, want_lg=True, return_cand=True)
    np.testing.assert_array_equal(cand_d, cand_h)
    # the same below fit: equal l (bit for bit when both runs score the same way;
    # a device-fitted label needs more candidates per table row before tables pay)
    _check_lpdf(l_d[0], l_h[0], 1e-5, (dist, 'l'))
    sub = rs.choice(C, 3000, replace=False)
    _check_lpdf(g_d[0][sub], lpdf(cand_d[0][sub], *above, low=low, high=high), 1e-5, (dist, 'g'))
    _check_argmax(int(res_d[0]['idx']), l_h[0], g_h[0], 1e-5, dist)
    # injected tails (wide components, fixed-shift underflow fallback)
    lo_x = tr(np.min(obs)) - 3 * psig
    hi_x = tr(np.max(obs)) + 3 * psig
    if low is not None:
        lo_x, hi_x = low, high
    x = np.linspace(lo_x, hi_x, 4001)[:-1]
    x = np.exp(x) if logf else x
    res_i, l_i, g_i = engine.run([LevelProblem(dev, 0, [3], inject=x[None, :])], len(x), 1, want_lg=True)
    _check_lpdf(g_i[0], lpdf(x, *above, low=low, high=high), 1e-5, (dist, 'g inj'))
    # repeatable bit for bit
    res_d2 = engine.run([LevelProblem(dev, 0, [3])], C, seed=9)
    assert res_d2[0]['idx'] == res_d[0]['idx'] and res_d2[0]['score'] == res_d[0]['score']


@pytest.mark.parametrize('case', ['uniform_dense', 'clustered', 'loguniform'])
def test_box_moment_tables_match_direct_tables(engine, monkeypatch, case):
    """Box-moment cells (include/tpe_hip.h "Box moments": Hermite moments per
    box of the narrowest width, translated to each cell's Taylor moments) of a
    device-fitted above mixture against the same cells built directly from
    every component within reach (TPE_FGT=0 with tables forced): the same
    draws, the above lpdf within 2e-6 relative of each other on every sampled
    candidate and both within the fp32 tolerance of the oracle; the argmax
    inside the eps-tie set.  'clustered' mixes narrow clusters with isolated
    points, so boxes hold components of other widths (summed directly)."""
    from hyperopt_amd import _native as N
    from hyperopt_amd.engine import LevelProblem
    rs = np.random.RandomState(77)
    n = 40000
    if case == 'uniform_dense':          # config 5's shape: every bandwidth at the clip
        dist, args, obs = 'uniform', dict(low=-5.0, high=5.0), rs.uniform(-5, 5, n)
    elif case == 'clustered':
        dist, args = 'uniform', dict(low=-5.0, high=5.0)
        obs = np.clip(np.concatenate([rs.normal(-2, 0.05, n // 2), rs.uniform(-5, 5, n // 2 - 3),
                                      [-4.9, 4.95, 0.0]]), -5, 5)
    else:
        dist, args, obs = 'loguniform', dict(low=-4.0, high=3.0), np.exp(rs.uniform(-4, 3, n))
    rs.shuffle(obs)
    bidx = np.sort(rs.choice(n, 25, replace=False)).astype(np.int32)
    m = np.zeros(n, bool)
    m[bidx] = True
    dev, _ = _device_post(engine, dist, args, obs, bidx)
    logf = dist == 'loguniform'
    tr = np.log if logf else (lambda v: v)
    pmu, psig = 0.5 * (args['low'] + args['high']), args['high'] - args['low']
    above = O.adaptive_parzen_normal(tr(obs[~m]), 1.0, pmu, psig)
    lpdf = O.lgmm1_lpdf if logf else O.gmm1_lpdf
    C = 1 << 16
    monkeypatch.setenv('TPE_TAB_DEVFIT_RATIO', '1')
    monkeypatch.setenv('TPE_LOGPOLY', '0')          # direct cells: moment rows, as the boxes give
    out = {}
    for fgt in ('1', '0'):
        monkeypatch.setenv('TPE_FGT', fgt)
        res, cand, l, g = engine.run([LevelProblem(dev, 0, [3])], C, seed=9, want_lg=True, return_cand=True)
        prob, _ = engine.device_tables()
        assert prob[0]['tab_mode'] == N.TAB_CELLS
        assert bool(prob[0]['flags'] & N.F_FGT) == (fgt == '1')
        out[fgt] = (res, cand[0], l[0], g[0])
    np.testing.assert_array_equal(out['1'][1], out['0'][1])
    np.testing.assert_array_equal(out['1'][2], out['0'][2])        # the below side: the same cells
    gf, gd = out['1'][3], out['0'][3]
    assert np.all(np.abs(gf - gd) <= 2e-6 * np.maximum(1.0, np.abs(gd))), np.max(np.abs(gf - gd))
    x = out['1'][1]
    sub = rs.choice(C, 3000, replace=False)
    _check_lpdf(gf[sub], lpdf(x[sub], *above, low=dev.low, high=dev.high), 1e-5, (case, 'g'))
    _check_argmax(int(out['1'][0][0]['idx']), out['1'][2], gd, 1e-5, case)


def test_device_fit_batched_labels_and_suggest():
    """Several device-fitted labels (and host-fitted ones) in one level, through
    tpe.suggest_choices: identical to suggest_choices with every fit on the host
    up to the eps-tie set, and the column upload is incremental."""
    from hyperopt_amd import hp, tpe
    from hyperopt_amd.engine import get_engine
    from hyperopt_amd.history import History
    from hyperopt_amd.space import ParamTable
    rs = np.random.RandomState(41)
    N = 6000
    labels = {'a': hp.uniform('a', -5, 5), 'b': hp.loguniform('b', -3, 2), 'c': hp.normal('c', 0, 2),
              'd': hp.quniform('d', 0, 10, 1)}
    vals = {'a': rs.uniform(-5, 5, N), 'b': np.exp(rs.uniform(-3, 2, N)), 'c': rs.normal(0, 2, N),
            'd': np.round(rs.uniform(0, 10, N))}
    tids = np.arange(N)
    losses = (vals['a'] - 1) ** 2 + rs.uniform(0, 1e-3, N)
    hist = History(tids, losses, {k: (tids, v) for k, v in vals.items()})
    table = ParamTable(labels)
    engine = get_engine()
    old = engine.device_fit_min
    try:
        engine.device_fit_min = 1000
        got = tpe.suggest_choices(table, hist, [N, N + 1], 5, n_EI_candidates=4096)
        dc = hist.dev[str(engine.device)]
        assert set(dc.slot) == {'a', 'b', 'c'} and all(dc.count(k) == N for k in dc.slot)
        engine.device_fit_min = 10 ** 9
        ref = tpe.suggest_choices(table, hist, [N, N + 1], 5, n_EI_candidates=4096)
    finally:
        engine.device_fit_min = old
    for g, r in zip(got, ref):
        assert g['d'] == r['d']
        for k in 'abc':
            assert abs(g[k] - r[k]) <= 1e-3 * max(1.0, abs(r[k])), (k, g[k], r[k])


@pytest.mark.parametrize('early', ['1', '0'])
def test_device_fit_more_than_64_ids(monkeypatch, early):
    """A device-fitted label active for 130 ids in one batched level (260 problems: an expanded level where the labels tabulate; ADVICE r5:
    k_fit_wide wrote the problem fields of the first 64 ids only), with the fit
    launched from inside the pack (early fit, k_fit_patch) and after the upload:
    every id's choice equals the host-fitted suggest's (eps-tie set) and the
    device-fitted labels' values are the same for a 1-id suggest of that id."""
    from hyperopt_amd import hp, tpe
    from hyperopt_amd.engine import get_engine
    from hyperopt_amd.history import History
    from hyperopt_amd.space import ParamTable
    monkeypatch.setenv('TPE_EARLY_FIT', early)
    rs = np.random.RandomState(43)
    N, n_ids = 5000, 130
    labels = {'a': hp.uniform('a', -5, 5), 'b': hp.loguniform('b', -3, 2)}
    vals = {'a': rs.uniform(-5, 5, N), 'b': np.exp(rs.uniform(-3, 2, N))}
    tids = np.arange(N)
    losses = (vals['a'] - 1) ** 2 + 0.1 * np.log(vals['b']) ** 2 + rs.uniform(0, 1e-3, N)
    hist = History(tids, losses, {k: (tids, v) for k, v in vals.items()})
    table = ParamTable(labels)
    ids = list(range(N, N + n_ids))
    engine = get_engine()
    old = engine.device_fit_min
    try:
        engine.device_fit_min = 1000
        got = tpe.suggest_choices(table, hist, ids, 7, n_EI_candidates=1024)
        one = tpe.suggest_choices(table, hist, [ids[-1]], 7, n_EI_candidates=1024)
        engine.device_fit_min = 10 ** 9
        ref = tpe.suggest_choices(table, hist, ids, 7, n_EI_candidates=1024)
    finally:
        engine.device_fit_min = old
    assert len(got) == len(ref) == n_ids
    for g, r in zip(got, ref):
        for k in 'ab':
            assert np.isfinite(g[k]) and abs(g[k] - r[k]) <= 1e-3 * max(1.0, abs(r[k])), (k, g[k], r[k])
    assert got[-1] == one[0]


def test_local_expansion_matches_exact_and_is_used(engine, monkeypatch):
    """The pruned f32 kernel's local (Taylor) expansion: above-lpdf of 2^20
    sampled candidates within 1e-5 of the all-exact kernel and within the fp32
    tolerance of the oracle; most window components are expanded."""
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    monkeypatch.setenv('TPE_TABLES', '0')          # the per-candidate pruned kernel
    rs = np.random.RandomState(13)
    for dist, args, obs in (('uniform', dict(low=-5.0, high=5.0), rs.uniform(-5, 5, 6000)),
                            ('loguniform', dict(low=-5.0, high=5.0), np.exp(rs.uniform(-5, 5, 6000)))):
        post = parzen.fit_posterior(dist, args, obs[:25], obs[25:], 1.0)
        C = 1 << 20
        engine.profile = {}
        res, cand, l, g = engine.run([LevelProblem(post, 0, [0])], C, seed=17, want_lg=True, return_cand=True)
        rec = engine.profile['k_above_f32'][0]
        engine.profile = None
        executed, expanded = rec[2], rec[3]
        engine.expand = False
        try:
            res_x, g_x = engine.run([LevelProblem(post, 0, [0])], C, seed=17, want_lg=True)[::2]
        finally:
            engine.expand = True
        np.testing.assert_allclose(g[0], g_x[0], rtol=1e-5, atol=1e-5)     # both fp32 (parity tolerance)
        assert expanded > 0 and executed < 0.2 * rec[1], (dist, executed, expanded, rec[1])
        sub = rs.choice(C, 3000, replace=False)
        lpdf = O.lgmm1_lpdf if dist == 'loguniform' else O.gmm1_lpdf
        _check_lpdf(g[0][sub], lpdf(cand[0][sub], *post.above, low=post.low, high=post.high), 1e-5, dist)
        score = l[0] - g[0]
        assert int(res[0]['idx']) == int(np.argmax(score))


@pytest.mark.parametrize('dist,args', [('uniform', dict(low=-5.0, high=5.0)),
                                       ('loguniform', dict(low=-4.0, high=3.0)),
                                       ('normal', dict(mu=1.0, sigma=3.0)),
                                       ('lognormal', dict(mu=0.0, sigma=1.0)),
                                       ('quniform', dict(low=0.0, high=20.0, q=1.0)),
                                       ('qloguniform', dict(low=0.0, high=5.0, q=2.0)),
                                       ('qnormal', dict(mu=2.0, sigma=4.0, q=0.5)),
                                       ('qlognormal', dict(mu=1.0, sigma=0.7, q=0.25))])
@pytest.mark.parametrize('logpoly', ['1', '0'])
def test_tabulated_scoring_matches_oracle(engine, dist, args, logpoly, monkeypatch):
    """Tabulated scoring (cells: Taylor moments per value cell — or, the
    default where both sides fit one grid, the log-polynomial rows built from
    them (TPE_F_LOGPOLY; TPE_LOGPOLY=0: moment rows) — fp32; lattice: exact
    {l, g} per quantized value, fp64) on device draws against the oracle's
    lpdf, the argmax inside the oracle's eps-tie set, the table mode actually
    taken, and the result equal to the per-candidate path's up to the
    tolerance."""
    import os
    from hyperopt_amd import _native as N
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    rs = np.random.RandomState(61)
    q = args.get('q')
    if q and logpoly == '0':
        pytest.skip('lattice tables have no log-polynomial variant')
    monkeypatch.setenv('TPE_LOGPOLY', logpoly)
    log = dist.startswith('log') or dist.startswith('qlog')
    lo, hi = (args['low'], args['high']) if 'low' in args else (args['mu'] - 3 * args['sigma'],
                                                               args['mu'] + 3 * args['sigma'])
    obs = rs.uniform(lo, hi, 4000)
    obs = np.exp(obs) if log else obs
    if q:
        obs = np.round(obs / q) * q
    post = parzen.fit_posterior(dist, args, obs[:30], obs[30:], 1.0)
    C = 1 << 18                                        # >= 8 candidates per table row
    res, cand, l, g = engine.run([LevelProblem(post, 5, [11])], C, seed=13, want_lg=True, return_cand=True)
    prob, _ = engine.device_tables()
    assert prob[0]['tab_mode'] == (N.TAB_LATTICE if q else N.TAB_CELLS), dist
    if not q:                                          # (log-polynomial rows: both sides on one grid <= 2048 cells)
        lpf = bool(prob[0]['flags'] & N.F_LOGPOLY)
        assert lpf == (logpoly == '1' and max(prob[0]['tab_n']) <= 2048) or (lpf and logpoly == '1'), \
            (dist, prob[0]['tab_n'])
        if lpf:
            assert prob[0]['tab_n'][0] == prob[0]['tab_n'][1] <= 2048, (dist, prob[0]['tab_n'])
    tol = 1e-9 if q else 1e-5
    lpdf = O.lgmm1_lpdf if log else O.gmm1_lpdf
    kw = dict(low=post.low, high=post.high, q=q)
    u, inv = np.unique(cand[0], return_inverse=True)
    sub = np.arange(len(u)) if len(u) < 4000 else rs.choice(len(u), 3000, replace=False)
    lb = lpdf(u[sub], *post.below, **kw)
    la = lpdf(u[sub], *post.above, **kw)
    first = np.zeros(len(u), dtype=np.int64)
    first[inv[::-1]] = np.arange(C)[::-1]              # first candidate of each distinct value
    _check_lpdf(l[0][first[sub]], lb, tol, (dist, 'l'))
    _check_lpdf(g[0][first[sub]], la, tol, (dist, 'g'))
    if len(u) < 4000:                                  # lattice: every candidate scored by the oracle
        _check_argmax(int(res[0]['idx']), lb[inv], la[inv], tol, dist)
    k = int(res[0]['idx'])
    assert res[0]['value'] == cand[0][k] and int(np.argmax(l[0] - g[0])) == k
    os.environ['TPE_TABLES'] = '0'
    try:
        ref = engine.run([LevelProblem(post, 5, [11])], C, seed=13)
    finally:
        os.environ.pop('TPE_TABLES', None)
    assert abs(ref[0]['score'] - res[0]['score']) <= 4 * tol * max(1.0, abs(res[0]['score'])), dist


@pytest.mark.parametrize('dist,args', [('uniform', dict(low=-5.0, high=5.0)),
                                       ('loguniform', dict(low=-4.0, high=3.0)),
                                       ('normal', dict(mu=1.0, sigma=3.0))])
def test_tabulated_exact_fallback_matches_oracle(engine, dist, args, monkeypatch):
    """The cells' exact fallback (a wave sums the whole mixture for one
    candidate at a time): TPE_BATCH_TAB_EXACT flags every cell, so every
    candidate takes it; l, g against the oracle and the winner against the
    table path's."""
    from hyperopt_amd import _native as N
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    rs = np.random.RandomState(67)
    log = dist.startswith('log')
    lo, hi = (args['low'], args['high']) if 'low' in args else (args['mu'] - 3 * args['sigma'],
                                                               args['mu'] + 3 * args['sigma'])
    obs = rs.uniform(lo, hi, 3000)
    obs = np.exp(obs) if log else obs
    post = parzen.fit_posterior(dist, args, obs[:30], obs[30:], 1.0)
    C = 1 << 18
    base = engine.run([LevelProblem(post, 5, [11])], C, seed=19)
    monkeypatch.setenv('TPE_DEBUG_FLAGS', str(N.BATCH_TAB_EXACT))
    res, cand, l, g = engine.run([LevelProblem(post, 5, [11])], C, seed=19, want_lg=True, return_cand=True)
    prob, _ = engine.device_tables()
    assert prob[0]['tab_mode'] == N.TAB_CELLS, dist
    lpdf = O.lgmm1_lpdf if log else O.gmm1_lpdf
    kw = dict(low=post.low, high=post.high, q=None)
    sub = rs.choice(C, 2000, replace=False)
    _check_lpdf(l[0][sub], lpdf(cand[0][sub], *post.below, **kw), 1e-5, (dist, 'l'))
    _check_lpdf(g[0][sub], lpdf(cand[0][sub], *post.above, **kw), 1e-5, (dist, 'g'))
    k = int(res[0]['idx'])
    assert res[0]['value'] == cand[0][k] and int(np.argmax(l[0] - g[0])) == k
    assert abs(base[0]['score'] - res[0]['score']) <= 4e-5 * max(1.0, abs(res[0]['score'])), dist


# ---------------------------------------------------------------- dense table checks
def _f32_bounds(post):
    """f32_bounds (tpe_kernels.hip): the f32 clip range of a problem's coordinate."""
    lo, hi = -np.inf, np.inf
    if post.low is not None:
        lo = np.float32(post.low)
        if float(lo) < post.low:
            lo = np.nextafter(lo, np.float32(np.inf))
    if post.high is not None:
        hi = np.float32(post.high)
        while float(hi) >= post.high:
            hi = np.nextafter(hi, np.float32(-np.inf))
    return float(lo), float(hi)


def _lpdf_chunked(lpdf, x, mix, kw, chunk=2048):
    """The oracle's lpdf of many points, in chunks (it forms points x components)."""
    return np.concatenate([lpdf(x[i:i + chunk], *mix, **kw) for i in range(0, len(x), chunk)] or [np.zeros(0)])


def _dense_cells(row, tab4, post, log, what, n_u=33, tol=1e-5):
    """Every cell row of a label evaluated at ``n_u`` points of its cell (the
    kernel's f32 cell geometry: lp_log2 / cell_log2_lds) in f64 on the host,
    against the oracle's lpdf at the same f32 coordinates — log-polynomial rows
    (TPE_F_LOGPOLY: both sides' degree-5 polynomials of log2 s interleaved in
    one row) or moment rows (11 Taylor moments and the shift per side);
    flagged sides (NaN: exact fallback) skipped and counted."""
    from hyperopt_amd import _native as N
    assert row['tab_mode'] == N.TAB_CELLS, what
    lp = bool(row['flags'] & N.F_LOGPOLY)
    lo_f, hi_f = _f32_bounds(post)
    lpdf = O.lgmm1_lpdf if log else O.gmm1_lpdf
    kw = dict(low=post.low, high=post.high, q=None)
    checked = flagged = 0
    for sd, mix, base in ((0, post.below, float(row['below_base'])), (1, post.above, float(row['above_base']))):
        g = 0 if lp else sd                                     # (log-polynomial: one table for both)
        n, off = int(row['tab_n'][g]), int(row['tab_off'][g])
        rows = tab4[off:off + 3 * n].reshape(n, 12).astype(np.float64)
        lo, inv = np.float32(row['tab_lo'][g]), np.float32(row['tab_inv'][g])
        w = np.float32(1) / inv
        ih = np.float32(1) / (np.float32(0.5) * w)
        j = np.arange(n)
        c = ((j + 0.5) * np.float64(w) + np.float64(lo)).astype(np.float32)      # fmaf(j + 0.5, w, lo)
        uk = np.linspace(-1, 1, n_u).astype(np.float32)
        t = (c[:, None] + (np.float32(0.5) * w) * uk[None, :]).astype(np.float32)   # f32 points of each cell
        u = ((t - c[:, None]) * ih).astype(np.float64)
        ok = (np.floor((t - lo) * inv) == j[:, None]) & (t >= lo_f) & (t <= hi_f)
        if lp:
            cf = rows[:, sd::2]                                  # {b_k, a_k} at 2k
            good = np.isfinite(cf[:, 0])
            s2 = cf[:, 5:6]
            for k in range(4, -1, -1):
                s2 = s2 * u + cf[:, k:k + 1]
        else:
            M, m = rows[:, :11], rows[:, 11]
            good = np.isfinite(m)
            sm = M[:, 10:11]
            for k in range(9, -1, -1):
                sm = sm * u + M[:, k:k + 1]
            ok &= sm > 0
            s2 = m[:, None] + np.log2(np.where(sm > 0, sm, 1.0))
        ok &= good[:, None]
        flagged += int((~good).sum())
        lnx = t.astype(np.float64) if log else 0.0
        got = s2 * np.log(2.0) + base - lnx
        x = np.exp(t.astype(np.float64)) if log else t.astype(np.float64)
        _check_lpdf(got[ok], _lpdf_chunked(lpdf, x[ok], mix, kw), tol, (what, 'lg'[sd], n, int(ok.sum()), lp))
        checked += int(ok.sum())
    n_all = int(row['tab_n'][0]) + (0 if lp else int(row['tab_n'][1]))
    assert flagged <= max(4, n_all // 10), (what, 'flagged sides', flagged, n_all)   # (exact fallback: tested apart)
    return checked


def _dense_lattice(row, tab4, post, log, what, tol=1e-9):
    """Every lattice row {l, g} of a quantized label against the oracle's lpdf
    at its value, and every entry threshold (ABI 20) against the host's
    quantisation of the f32 coordinates either side of it."""
    from hyperopt_amd import _native as N
    assert row['tab_mode'] == N.TAB_LATTICE, what
    n, off = int(row['tab_n'][0]), int(row['tab_off'][0])
    lg = tab4[off:off + n].view(np.float64).reshape(n, 2)
    q = float(row['q'])
    x = (int(row['lat_lo']) + np.arange(n)).astype(np.float64) * q
    lpdf = O.lgmm1_lpdf if log else O.gmm1_lpdf
    kw = dict(low=post.low, high=post.high, q=q)
    lo_f, hi_f = _f32_bounds(post)
    thr = tab4[off + n:off + n + (n + 4) // 4].reshape(-1)[:n + 1]
    reach = thr[:-1] < thr[1:]                     # rows some f32 draw in the clip range takes
    assert reach.sum() >= 2, what
    with np.errstate(divide='ignore', invalid='ignore'):
        _check_lpdf(lg[reach, 0], lpdf(x[reach], *post.below, **kw), tol, (what, 'l', n))
        _check_lpdf(lg[reach, 1], lpdf(x[reach], *post.above, **kw), tol, (what, 'g', n))

    def qidx(t):
        t = np.float64(t)
        return np.round((np.exp(t) if log else t) / q)
    for m in range(n + 1):
        T = thr[m]
        target = int(row['lat_lo']) + m
        if T == np.inf:
            assert qidx(np.float32(hi_f)) < target, (what, m)
        else:
            assert qidx(T) >= target, (what, m, T)
            if T > lo_f:
                assert qidx(np.nextafter(np.float32(T), np.float32(-np.inf))) < target, (what, m, T)
    assert np.all(thr[1:] >= thr[:-1]), what
    return n


@pytest.mark.parametrize('dist,args', [('uniform', dict(low=-5.0, high=5.0)),
                                       ('loguniform', dict(low=-4.0, high=3.0)),
                                       ('normal', dict(mu=1.0, sigma=3.0)),
                                       ('lognormal', dict(mu=0.0, sigma=1.0)),
                                       ('quniform', dict(low=0.0, high=20.0, q=1.0)),
                                       ('qloguniform', dict(low=0.0, high=5.0, q=2.0)),
                                       ('qnormal', dict(mu=2.0, sigma=4.0, q=0.5)),
                                       ('qlognormal', dict(mu=1.0, sigma=0.7, q=0.25))])
def test_table_rows_dense_against_oracle(engine, dist, args):
    """Every table row the table stage builds for the 8 families, read back:
    each log-polynomial cell evaluated at 33 points of the cell in f64 against
    the oracle's gmm1_lpdf / lgmm1_lpdf (1e-5 max(|ref|, 1)); each lattice row
    exactly against the oracle (1e-9) and its entry thresholds against the
    host's quantisation (tpe.py:104-166, 259-301)."""
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import LevelProblem
    rs = np.random.RandomState(61)
    q = args.get('q')
    log = dist.startswith('log') or dist.startswith('qlog')
    lo, hi = (args['low'], args['high']) if 'low' in args else (args['mu'] - 3 * args['sigma'],
                                                               args['mu'] + 3 * args['sigma'])
    obs = rs.uniform(lo, hi, 1500)                     # (~1500 cells x 33 points x 1500 components: seconds)
    obs = np.exp(obs) if log else obs
    if q:
        obs = np.round(obs / q) * q
    post = parzen.fit_posterior(dist, args, obs[:30], obs[30:], 1.0)
    engine.run([LevelProblem(post, 5, [11])], 1 << 18, seed=13)
    prob, _ = engine.device_tables()
    tab4 = engine._bufs['tab'][:4 * int(engine._last_info.tab_units)].cpu().numpy().reshape(-1, 4)
    if q:
        assert _dense_lattice(prob[0], tab4, post, log, dist) > 0
    else:
        assert _dense_cells(prob[0], tab4, post, log, dist) > 1000


@pytest.mark.parametrize('branch', ['svm', 'rf'])
def test_headline_table_rows_dense_against_oracle(engine, branch):
    """The headline's labels (config 3 at 10k trials and 2^20 candidates): the
    svm branch's log-polynomial tables (svm_C, svm_rbf_gamma) and the rf
    branch's lattices (rf_n_est, rf_depth_n), fitted as tpe.suggest fits them,
    every row checked densely against the oracle as above."""
    import bench
    from hyperopt_amd import history as H, tpe
    from hyperopt_amd.engine import LevelProblem
    domain, trials = bench.make_history(10000, bench.SEED, loss=None if branch == 'svm' else bench.rf_loss)
    T = domain.table
    hist = H.extract(domain, trials)
    below = H.split_below(hist, 0.25)
    fits = tpe._Fits(T, hist, below, 1.0, None)
    labels = ('svm_C', 'svm_rbf_gamma') if branch == 'svm' else ('rf_n_est', 'rf_depth_n')
    rows = [T.by_label[k] for k in labels]
    posts = [fits.get(r) for r in rows]
    engine.run([LevelProblem(p, r.index, [10000]) for p, r in zip(posts, rows)], 1 << 20, seed=3)
    prob, _ = engine.device_tables()
    tab4 = engine._bufs['tab'][:4 * int(engine._last_info.tab_units)].cpu().numpy().reshape(-1, 4)
    by_ix = {int(p['ctr2']): p for p in prob}
    for r, post in zip(rows, posts):
        log = r.dist.startswith('log') or r.dist.startswith('qlog')
        row = by_ix[r.index]
        if branch == 'svm':
            assert _dense_cells(row, tab4, post, log, r.label) > 10000
        else:
            assert _dense_lattice(row, tab4, post, log, r.label) > 10
