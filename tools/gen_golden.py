#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE itself (build container only).

Usage:  oracle/make_refpy3.sh && python tools/gen_golden.py

Imports the 2to3 scratch copy of gsmafra/hyperopt at /tmp/refpy3 (never part
of this repository) and writes plain-data fixtures to tests/golden/:

* unit_vectors.json    — adaptive_parzen_normal, linear_forgetting_weights,
                         ap_filter_trials, *_lpdf, samplers, broadcast_best
* suggest_vectors.json — whole tpe.suggest / rand.suggest outputs on generated
                         histories over several search spaces
* fmin_traj.json       — full fmin(tpe.suggest) trajectories (config 1 + more)
* kernel_vectors.json  — larger mixtures + candidates + l/g (kernel parity)

Floats are stored with repr() precision, so JSON round-trips them exactly.
"""
import json
import os
import platform
import sys

import numpy as np
import scipy

REF = os.environ.get('REFPY3', '/tmp/refpy3')
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import hyperopt  # noqa: E402  (the reference, from the scratch copy)
from hyperopt import hp, tpe, rand, base, Trials  # noqa: E402
from hyperopt.fmin import fmin  # noqa: E402

from oracle.spacedesc import build_with_hp, params_from_desc, synthetic_loss  # noqa: E402

assert hyperopt.__file__.startswith(REF), hyperopt.__file__
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests', 'golden')


def tolist(a):
    a = np.asarray(a)
    if a.dtype.kind in 'iu':
        return [int(v) for v in a.ravel()]
    return [float(v) for v in a.ravel()]


def meta():
    return dict(numpy=np.__version__, scipy=scipy.__version__, python=platform.python_version(),
                machine=platform.machine(), reference='gsmafra/hyperopt ' + hyperopt.__version__,
                generator='tools/gen_golden.py')


# --------------------------------------------------------------------------
SPACES = {
    'u1': {'type': 'hp', 'dist': 'uniform', 'label': 'x', 'args': {'low': -10, 'high': 10}},
    'mixed10': {'type': 'dict', 'items': {
        'u0': {'type': 'hp', 'dist': 'uniform', 'label': 'u0', 'args': {'low': -5, 'high': 5}},
        'u1': {'type': 'hp', 'dist': 'uniform', 'label': 'u1', 'args': {'low': 0, 'high': 1}},
        'u2': {'type': 'hp', 'dist': 'uniform', 'label': 'u2', 'args': {'low': -1, 'high': 3}},
        'l0': {'type': 'hp', 'dist': 'loguniform', 'label': 'l0', 'args': {'low': -5, 'high': 0}},
        'l1': {'type': 'hp', 'dist': 'loguniform', 'label': 'l1', 'args': {'low': -2, 'high': 2}},
        'l2': {'type': 'hp', 'dist': 'loguniform', 'label': 'l2', 'args': {'low': 0, 'high': 3}},
        'q0': {'type': 'hp', 'dist': 'quniform', 'label': 'q0', 'args': {'low': 0, 'high': 20, 'q': 1}},
        'q1': {'type': 'hp', 'dist': 'quniform', 'label': 'q1', 'args': {'low': -4, 'high': 4, 'q': 0.5}},
        'c0': {'type': 'choice', 'label': 'c0', 'options': [{'type': 'literal', 'value': i} for i in range(5)]},
        'c1': {'type': 'choice', 'label': 'c1', 'options': [{'type': 'literal', 'value': i} for i in range(3)]},
    }},
    'allkinds': {'type': 'dict', 'items': {
        'a': {'type': 'hp', 'dist': 'uniform', 'label': 'a', 'args': {'low': -2, 'high': 2}},
        'b': {'type': 'hp', 'dist': 'quniform', 'label': 'b', 'args': {'low': 0, 'high': 10, 'q': 2}},
        'c': {'type': 'hp', 'dist': 'loguniform', 'label': 'c', 'args': {'low': -3, 'high': 1}},
        'd': {'type': 'hp', 'dist': 'qloguniform', 'label': 'd', 'args': {'low': 0, 'high': 4, 'q': 1}},
        'e': {'type': 'hp', 'dist': 'normal', 'label': 'e', 'args': {'mu': 1, 'sigma': 2}},
        'f': {'type': 'hp', 'dist': 'qnormal', 'label': 'f', 'args': {'mu': 0, 'sigma': 3, 'q': 0.5}},
        'g': {'type': 'hp', 'dist': 'lognormal', 'label': 'g', 'args': {'mu': 0, 'sigma': 1}},
        'h': {'type': 'hp', 'dist': 'qlognormal', 'label': 'h', 'args': {'mu': 1, 'sigma': 0.5, 'q': 0.25}},
        'i': {'type': 'hp', 'dist': 'randint', 'label': 'i', 'args': {'upper': 6}},
        'j': {'type': 'choice', 'label': 'j', 'options': [{'type': 'literal', 'value': 'p'},
                                                          {'type': 'literal', 'value': 'q'}]},
        'k': {'type': 'pchoice', 'label': 'k', 'p': [0.1, 0.6, 0.3],
              'options': [{'type': 'literal', 'value': i} for i in range(3)]},
    }},
    'tree': {'type': 'dict', 'items': {'model': {'type': 'choice', 'label': 'model', 'options': [
        {'type': 'dict', 'items': {
            'name': {'type': 'literal', 'value': 'svm'},
            'C': {'type': 'hp', 'dist': 'loguniform', 'label': 'svm_C', 'args': {'low': -5, 'high': 5}},
            'kernel': {'type': 'choice', 'label': 'svm_kernel', 'options': [
                {'type': 'dict', 'items': {'gamma': {'type': 'hp', 'dist': 'loguniform', 'label': 'svm_rbf_gamma',
                                                     'args': {'low': -5, 'high': 2}}}},
                {'type': 'dict', 'items': {'degree': {'type': 'hp', 'dist': 'quniform', 'label': 'svm_poly_degree',
                                                      'args': {'low': 2, 'high': 5, 'q': 1}}}}]}}},
        {'type': 'dict', 'items': {
            'name': {'type': 'literal', 'value': 'rf'},
            'n_est': {'type': 'hp', 'dist': 'quniform', 'label': 'rf_n_est', 'args': {'low': 10, 'high': 500, 'q': 10}},
            'depth': {'type': 'choice', 'label': 'rf_depth', 'options': [
                {'type': 'literal', 'value': None},
                {'type': 'hp', 'dist': 'quniform', 'label': 'rf_depth_n', 'args': {'low': 2, 'high': 30, 'q': 1}}]},
            'crit': {'type': 'choice', 'label': 'rf_crit', 'options': [{'type': 'literal', 'value': 'gini'},
                                                                       {'type': 'literal', 'value': 'entropy'}]}}},
        {'type': 'dict', 'items': {
            'name': {'type': 'literal', 'value': 'knn'},
            'k': {'type': 'hp', 'dist': 'quniform', 'label': 'knn_k', 'args': {'low': 1, 'high': 50, 'q': 1}},
            'p': {'type': 'hp', 'dist': 'uniform', 'label': 'knn_p', 'args': {'low': 1, 'high': 3}}}},
    ]}}},
    # label order deliberately puts a child ('zz') after its parent ('aa'), and a
    # flat label between them, to pin the ancestors-first RandomState order
    'order': {'type': 'dict', 'items': {
        'aa': {'type': 'choice', 'label': 'aa', 'options': [
            {'type': 'hp', 'dist': 'uniform', 'label': 'zz', 'args': {'low': 0, 'high': 1}},
            {'type': 'hp', 'dist': 'normal', 'label': 'bb', 'args': {'mu': 0, 'sigma': 1}}]},
        'mm': {'type': 'hp', 'dist': 'uniform', 'label': 'mm', 'args': {'low': -1, 'high': 1}},
    }},
}


def make_history(desc, n, seed):
    """n trials drawn by the reference rand.suggest, losses from synthetic_loss."""
    space = build_with_hp(desc, hp)
    domain = base.Domain(lambda x: 0.0, space)
    trials = Trials()
    rs = np.random.RandomState(seed)
    for tid in range(n):
        docs = rand.suggest([tid], domain, trials, rs.randint(2 ** 31 - 1))
        vals = {k: (v[0] if v else None) for k, v in docs[0]['misc']['vals'].items()}
        docs[0]['state'] = base.JOB_STATE_DONE
        docs[0]['result'] = {'status': 'ok', 'loss': synthetic_loss(vals, tid)}
        trials.insert_trial_docs(docs)
    trials.refresh()
    return domain, trials


def history_to_json(trials):
    out = []
    for d in trials.trials:
        out.append(dict(tid=int(d['tid']), loss=float(d['result']['loss']),
                        vals={k: [float(x) if isinstance(x, (float, np.floating)) else int(x) for x in v]
                              for k, v in d['misc']['vals'].items()}))
    return out


def doc_vals(docs):
    v = docs[0]['misc']['vals']
    return {k: (float(x[0]) if isinstance(x[0], (float, np.floating)) else int(x[0]))
            for k, x in v.items() if len(x)}


def gen_suggest_vectors():
    cases = []
    plan = [('u1', 30, [1, 2, 3], 24), ('u1', 120, [4], 100),
            ('mixed10', 40, [5, 6], 24), ('mixed10', 150, [7], 200),
            ('allkinds', 60, [8, 9, 10], 40), ('allkinds', 30, [11], 24),
            ('tree', 80, [12, 13, 14, 15], 64), ('tree', 200, [16], 128),
            ('order', 50, [17, 18, 19, 20], 16), ('mixed10', 10, [21], 24)]
    for name, n, seeds, C in plan:
        domain, trials = make_history(SPACES[name], n, seed=sum(map(ord, name)) + n)
        hist = history_to_json(trials)
        for s in seeds:
            docs = tpe.suggest([n], domain, trials, s, n_EI_candidates=C)
            cases.append(dict(space=name, n=n, seed=s, n_EI_candidates=C, history=hist,
                              result=doc_vals(docs)))
        # the start-up path on the same space
        docs = rand.suggest([n], domain, trials, seeds[0])
        cases.append(dict(space=name, n=n, seed=seeds[0], kind='rand', history=[],
                          result=doc_vals(docs)))
    return cases


def gen_fmin_traj():
    out = []
    for s in range(10):
        t = Trials()
        fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -10, 10), algo=tpe.suggest, max_evals=100,
             trials=t, rstate=np.random.RandomState(s))
        out.append(dict(space='u1', objective='(x-3)^2', seed=s, max_evals=100,
                        x=[float(d['misc']['vals']['x'][0]) for d in t.trials],
                        loss=[float(d['result']['loss']) for d in t.trials]))
    for name, evals, s in [('mixed10', 60, 3), ('tree', 70, 4), ('allkinds', 50, 5)]:
        t = Trials()
        params = params_from_desc(SPACES[name])

        def objective(_cfg, _t=t):
            # loss from the flat vals of the trial being evaluated (last doc)
            d = _t._dynamic_trials[-1]
            vals = {k: (v[0] if v else None) for k, v in d['misc']['vals'].items()}
            return synthetic_loss(vals, d['tid'])
        fmin(objective, build_with_hp(SPACES[name], hp), algo=tpe.suggest, max_evals=evals,
             trials=t, rstate=np.random.RandomState(s))
        out.append(dict(space=name, objective='synthetic_loss', seed=s, max_evals=evals,
                        vals=[{k: (float(v[0]) if isinstance(v[0], (float, np.floating)) else int(v[0]))
                               for k, v in d['misc']['vals'].items() if v} for d in t.trials],
                        loss=[float(d['result']['loss']) for d in t.trials],
                        labels=sorted(p['label'] for p in params)))
    return out


def gen_unit_vectors():
    rs = np.random.RandomState(123)
    U = {}
    # adaptive_parzen_normal
    apn = []
    inputs = [([], 1.0, 0.5, 1.0), ([0.7], 1.0, 0.5, 1.0), ([0.2], 1.0, 0.5, 1.0), ([0.5], 1.0, 0.5, 1.0),
              ([0.2, 0.9, 0.5, 0.7], 1.0, 0.5, 1.0), ([0.1, 0.1], 2.0, 0.1, 3.0),
              (list(rs.uniform(-5, 5, 30)), 1.0, 0.0, 10.0),
              (list(np.round(rs.uniform(0, 20, 300))), 1.0, 10.0, 20.0),        # ties + LF
              (list(rs.uniform(0, 1, 1000)), 1.0, 0.5, 1.0),
              (list(rs.normal(0, 1, 77)), 0.5, 1.0, 2.0)]
    for mus, pw, pmu, psig in inputs:
        w, m, s = tpe.adaptive_parzen_normal(mus, pw, pmu, psig)
        apn.append(dict(mus=tolist(mus), prior_weight=pw, prior_mu=pmu, prior_sigma=psig,
                        w=tolist(w), mu=tolist(m), sigma=tolist(s)))
    U['adaptive_parzen_normal'] = apn
    U['linear_forgetting_weights'] = [dict(N=N, LF=25, w=tolist(tpe.linear_forgetting_weights(N, 25)))
                                      for N in (0, 1, 24, 25, 26, 30, 100)]
    # ap_filter_trials
    aft = []
    for n, ratio in ((8, 1.0), (100, 0.7), (1000, 0.5)):
        l_idxs = np.arange(n)
        l_vals = rs.permutation(n).astype(float) + 0.5
        o_mask = rs.uniform(size=n) < ratio
        o_idxs = l_idxs[o_mask]
        o_vals = rs.uniform(0, 1, o_mask.sum())
        b, a = tpe.ap_filter_trials(o_idxs, o_vals, l_idxs, l_vals, 0.25)
        aft.append(dict(o_idxs=tolist(o_idxs), o_vals=tolist(o_vals), l_idxs=tolist(l_idxs),
                        l_vals=tolist(l_vals), gamma=0.25, below=tolist(b), above=tolist(a)))
    U['ap_filter_trials'] = aft
    # lpdfs
    lp = []
    for K, C in ((5, 50), (120, 300), (1001, 200)):
        w = rs.uniform(0.1, 1, K); w /= w.sum()
        mu = np.sort(rs.uniform(-3, 3, K))
        sig = rs.uniform(0.05, 2, K)
        x = rs.uniform(-3, 3, C)
        xq = np.round(x / 0.5) * 0.5
        for low, high in ((None, None), (-3.0, 3.0)):
            lp.append(dict(fn='GMM1_lpdf', w=tolist(w), mu=tolist(mu), sigma=tolist(sig), low=low, high=high,
                           q=None, x=tolist(x), out=tolist(tpe.GMM1_lpdf(x, w, mu, sig, low, high, None))))
            lp.append(dict(fn='GMM1_lpdf', w=tolist(w), mu=tolist(mu), sigma=tolist(sig), low=low, high=high,
                           q=0.5, x=tolist(xq), out=tolist(tpe.GMM1_lpdf(xq, w, mu, sig, low, high, 0.5))))
            ex = np.exp(x)
            exq = np.round(ex / 0.25) * 0.25
            lp.append(dict(fn='LGMM1_lpdf', w=tolist(w), mu=tolist(mu), sigma=tolist(sig), low=low, high=high,
                           q=None, x=tolist(ex), out=tolist(tpe.LGMM1_lpdf(ex, w, mu, sig, low, high, None))))
            lp.append(dict(fn='LGMM1_lpdf', w=tolist(w), mu=tolist(mu), sigma=tolist(sig), low=low, high=high,
                           q=0.25, x=tolist(exq), out=tolist(tpe.LGMM1_lpdf(exq, w, mu, sig, low, high, 0.25))))
    p = rs.uniform(0.1, 1, 7); p /= p.sum()
    xs = rs.randint(0, 7, 40)
    lp.append(dict(fn='categorical_lpdf', p=tolist(p), x=tolist(xs), out=tolist(tpe.categorical_lpdf(xs, p, 7))))
    U['lpdf'] = lp
    U['known_answers'] = dict(
        gmm1_trunc=tolist(tpe.GMM1_lpdf(np.array([0.1, 0.5, 0.95]), *tpe.adaptive_parzen_normal(
            [0.2, 0.9, 0.5, 0.7], 1.0, 0.5, 1.0), low=0, high=1)))
    # samplers
    sm = []
    for seed in (0, 1, 2):
        w = rs.uniform(0.1, 1, 6); w /= w.sum()
        mu = rs.uniform(-1, 1, 6); sig = rs.uniform(0.1, 1, 6)
        for fn, low, high, q in (('GMM1', None, None, None), ('GMM1', -1.0, 1.0, None), ('GMM1', -1.0, 1.0, 0.25),
                                 ('GMM1', None, None, 0.5), ('LGMM1', None, None, None), ('LGMM1', -1.0, 1.0, None),
                                 ('LGMM1', -1.0, 1.0, 0.5), ('LGMM1', None, None, 0.1)):
            f = getattr(tpe, fn)
            out = f(w, mu, sig, low=low, high=high, q=q, rng=np.random.RandomState(seed), size=(37,))
            sm.append(dict(fn=fn, seed=seed, w=tolist(w), mu=tolist(mu), sigma=tolist(sig), low=low, high=high,
                           q=q, size=37, out=tolist(out)))
        from hyperopt.pyll.stochastic import categorical
        p = rs.uniform(0.1, 1, 5); p /= p.sum()
        sm.append(dict(fn='categorical', seed=seed, p=tolist(p), size=29,
                       out=tolist(categorical(p, upper=5, rng=np.random.RandomState(seed), size=29))))
    U['samplers'] = sm
    U['broadcast_best'] = [dict(samples=[1, 2, 3], l=[0, 1, 1], g=[0, 0, 0],
                                out=tpe.broadcast_best([1, 2, 3], np.array([0., 1, 1]), np.array([0., 0, 0])))]
    return U


def gen_kernel_vectors():
    """Config-2/3-shaped mixtures fitted by the reference, with reference-drawn
    candidates and the reference's l / g, for GPU kernel parity."""
    rs = np.random.RandomState(7)
    out = []
    N = 2000
    gamma = 0.25
    n_below = min(int(np.ceil(gamma * np.sqrt(N))), 25)
    cases = [('uniform', dict(low=-5.0, high=5.0), lambda n: rs.uniform(-5, 5, n)),
             ('quniform', dict(low=-4.0, high=4.0, q=0.5), lambda n: np.round(rs.uniform(-4, 4, n) / 0.5) * 0.5),
             ('loguniform', dict(low=-5.0, high=2.0), lambda n: np.exp(rs.uniform(-5, 2, n))),
             ('qloguniform', dict(low=0.0, high=4.0, q=1.0), lambda n: np.round(np.exp(rs.uniform(0, 4, n)))),
             ('normal', dict(mu=1.0, sigma=2.0), lambda n: rs.normal(1, 2, n)),
             ('qnormal', dict(mu=0.0, sigma=3.0, q=0.5), lambda n: np.round(rs.normal(0, 3, n) / 0.5) * 0.5),
             ('lognormal', dict(mu=0.0, sigma=1.0), lambda n: np.exp(rs.normal(0, 1, n))),
             ('qlognormal', dict(mu=1.0, sigma=0.5, q=0.25), lambda n: np.round(np.exp(rs.normal(1, .5, n)) / .25) * .25),
             ('randint', dict(upper=7), lambda n: rs.randint(0, 7, n)),
             ('categorical', dict(p=[0.1, 0.2, 0.3, 0.4], upper=4), lambda n: rs.randint(0, 4, n))]
    for dist, args, gen in cases:
        vals = gen(N)
        losses = rs.uniform(0, 1, N) + 1e-9 * np.arange(N)
        tids = np.arange(N)
        below, above = tpe.ap_filter_trials(tids, vals, tids, losses, gamma)
        fn = tpe.adaptive_parzen_samplers[dist]
        kw = {k: v for k, v in args.items()}
        if dist == 'categorical':
            kw['p'] = np.asarray(kw['p'])
        pos = [kw[k] for k in ({'uniform': ('low', 'high'), 'quniform': ('low', 'high', 'q'),
                                'loguniform': ('low', 'high'), 'qloguniform': ('low', 'high', 'q'),
                                'normal': ('mu', 'sigma'), 'qnormal': ('mu', 'sigma', 'q'),
                                'lognormal': ('mu', 'sigma'), 'qlognormal': ('mu', 'sigma', 'q'),
                                'randint': ('upper',), 'categorical': ('p', 'upper')}[dist])]
        from hyperopt import pyll
        C = 4096
        b_post = fn(below, 1.0, *pos, size=C, rng=np.random.RandomState(11))
        a_post = fn(above, 1.0, *pos, size=C, rng=np.random.RandomState(11))
        cand = pyll.rec_eval(b_post)
        lpdf = getattr(tpe, b_post.name + '_lpdf')
        b_kw = {n: pyll.rec_eval(a) for n, a in b_post.named_args if n not in ('rng', 'size')}
        a_kw = {n: pyll.rec_eval(a) for n, a in a_post.named_args if n not in ('rng', 'size')}
        b_pos = [pyll.rec_eval(a) for a in b_post.pos_args]
        a_pos = [pyll.rec_eval(a) for a in a_post.pos_args]
        l = lpdf(cand, *b_pos, **b_kw)
        g = lpdf(cand, *a_pos, **a_kw)
        out.append(dict(dist=dist, args=args, N=N, n_below=n_below, vals=tolist(vals), losses=tolist(losses),
                        below=tolist(below), above=tolist(above), cand=tolist(cand), l=tolist(l), g=tolist(g),
                        best=int(np.argmax(l - g)), post=b_post.name,
                        b_params=[tolist(v) for v in b_pos[:3]] if b_post.name != 'categorical' else [tolist(b_pos[0])],
                        a_params=[tolist(v) for v in a_pos[:3]] if a_post.name != 'categorical' else [tolist(a_pos[0])]))
    return out


def dump(name, obj):
    path = os.path.join(OUT, name)
    with open(path, 'w') as f:
        json.dump(dict(meta=meta(), data=obj), f, separators=(',', ':'))
    print('wrote', path, os.path.getsize(path), 'bytes')


if __name__ == '__main__':
    os.makedirs(OUT, exist_ok=True)
    dump('unit_vectors.json', gen_unit_vectors())
    dump('kernel_vectors.json', gen_kernel_vectors())
    dump('suggest_vectors.json', dict(spaces=SPACES, cases=gen_suggest_vectors()))
    dump('fmin_traj.json', dict(spaces=SPACES, runs=gen_fmin_traj()))
