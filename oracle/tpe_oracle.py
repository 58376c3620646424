"""CPU ORACLE for the TPE suggest path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  ``hyperopt_amd`` never imports anything under ``oracle/``; its suggest
path fails loudly when the HIP library is missing.

It restates, in plain numpy/scipy float64 on one thread, the reference
algorithm of gsmafra/hyperopt 0.0.3 (``/root/reference``) for the
``tpe.suggest`` hot path and the ``rand.suggest`` start-up path.  Every
function cites the reference ``file:line`` it follows.  The numeric operation
order is kept where it decides the last bit (e.g. ``normal_cdf`` uses
``0.5 * (1 + erf(z))`` but ``lognormal_cdf`` uses ``.5 + .5 * erf(z)``), so the
restatement is bit-exact with the reference on the same numpy build.

Pinning: ``tests/golden/*.json`` were produced by running the reference itself
in the build container (``tools/gen_golden.py``, recipe in
``oracle/make_refpy3.sh``); ``tests/test_oracle_golden.py`` checks this module
against every vector.  The reference's own repository holds no tests or
fixtures, so those generated vectors are the pin.

Search spaces are described here by a flat *param table* (a list of dicts,
one per ``hp.*`` label) rather than a pyll graph::

    {"label": "x", "dist": "uniform", "args": {"low": -10, "high": 10},
     "parent": None}                       # or ("model", 1): active iff model == 1

which is what ``pyll_utils.expr_to_config`` (pyll_utils.py:144-225) extracts.
"""
import math

import numpy as np
from scipy.special import erf

EPS = 1e-12                      # tpe.py:25
DEFAULT_LF = 25                  # tpe.py:29

# ---------------------------------------------------------------------------
# elementwise densities / cdfs
# ---------------------------------------------------------------------------


def normal_cdf(x, mu, sigma):
    """tpe.py:96-101"""
    top = x - mu
    bottom = np.maximum(np.sqrt(2) * sigma, EPS)
    z = top / bottom
    return 0.5 * (1 + erf(z))


def lognormal_cdf(x, mu, sigma):
    """tpe.py:171-190 (note the different constant folding vs normal_cdf)"""
    if len(x) == 0:
        return np.asarray([])
    if x.min() < 0:
        raise ValueError('negative arg to lognormal_cdf', x)
    with np.errstate(divide='ignore'):
        top = np.log(np.maximum(x, EPS)) - mu
        bottom = np.maximum(np.sqrt(2) * sigma, EPS)
        z = top / bottom
        return .5 + .5 * erf(z)


def lognormal_lpdf(x, mu, sigma):
    """tpe.py:193-202"""
    sigma = np.maximum(sigma, EPS)
    Z = sigma * x * np.sqrt(2 * np.pi)
    E = 0.5 * ((np.log(x) - mu) / sigma) ** 2
    return -E - np.log(Z)


def logsum_rows(x):
    """tpe.py:253-256: two-pass max-shifted log-sum-exp over axis 1."""
    m = x.max(axis=1)
    return np.log(np.exp(x - m[:, None]).sum(axis=1)) + m


def _p_accept(weights, mus, sigmas, low, high):
    """tpe.py:130-136 and :270-276 (identical in GMM1_lpdf / LGMM1_lpdf)."""
    if low is None and high is None:
        return 1
    return np.sum(weights * (normal_cdf(high, mus, sigmas)
                             - normal_cdf(low, mus, sigmas)))


def gmm1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None):
    """tpe.py:104-166 — log-density of the (truncated, quantized) Gaussian
    mixture at every sample."""
    samples, weights, mus, sigmas = map(np.asarray, (samples, weights, mus, sigmas))
    if samples.size == 0:
        return np.asarray([])
    shape = samples.shape
    samples = samples.flatten()
    p_accept = _p_accept(weights, mus, sigmas, low, high)
    if q is None:
        dist = samples[:, None] - mus
        mahal = (dist / np.maximum(sigmas, EPS)) ** 2
        Z = np.sqrt(2 * np.pi * sigmas ** 2)
        coef = weights / Z / p_accept
        rval = logsum_rows(-0.5 * mahal + np.log(coef))
    else:
        prob = np.zeros(samples.shape, dtype='float64')
        ub = samples + q / 2.0
        lb = samples - q / 2.0
        if high is not None:
            ub = np.minimum(ub, high)
        if low is not None:
            lb = np.maximum(lb, low)
        for w, mu, sigma in zip(weights, mus, sigmas):
            inc = w * normal_cdf(ub, mu, sigma)
            inc -= w * normal_cdf(lb, mu, sigma)
            prob += inc
        with np.errstate(divide='ignore'):
            rval = np.log(prob) - np.log(p_accept)
    return rval.reshape(shape)


def lgmm1_lpdf(samples, weights, mus, sigmas, low=None, high=None, q=None):
    """tpe.py:259-301 — log-normal mixture.  Quirk kept: the unquantized
    branch never subtracts log(p_accept) even when bounded (:278-281)."""
    samples, weights, mus, sigmas = map(np.asarray, (samples, weights, mus, sigmas))
    shape = samples.shape
    samples = samples.flatten()
    p_accept = _p_accept(weights, mus, sigmas, low, high)
    if q is None:
        lpdfs = lognormal_lpdf(samples[:, None], mus, sigmas)
        rval = logsum_rows(lpdfs + np.log(weights))
    else:
        prob = np.zeros(samples.shape, dtype='float64')
        ub = samples + q / 2.0
        lb = samples - q / 2.0
        if high is not None:
            ub = np.minimum(ub, np.exp(high))
        if low is not None:
            lb = np.maximum(lb, np.exp(low))
        lb = np.maximum(0, lb)
        for w, mu, sigma in zip(weights, mus, sigmas):
            inc = w * lognormal_cdf(ub, mu, sigma)
            inc -= w * lognormal_cdf(lb, mu, sigma)
            prob += inc
        with np.errstate(divide='ignore'):
            rval = np.log(prob) - np.log(p_accept)
    return rval.reshape(shape)


def categorical_lpdf(sample, p):
    """tpe.py:50-57"""
    sample = np.asarray(sample)
    if sample.size:
        return np.log(np.asarray(p)[sample])
    return np.asarray([])


# ---------------------------------------------------------------------------
# samplers (numpy RandomState, the reference's consumption pattern)
# ---------------------------------------------------------------------------


def gmm1_sample(rng, weights, mus, sigmas, low=None, high=None, q=None, size=0):
    """tpe.py:62-93.  Bounded mixtures use the per-draw rejection loop."""
    weights, mus, sigmas = map(np.asarray, (weights, mus, sigmas))
    n = int(np.prod(size))
    if low is None and high is None:
        active = np.argmax(rng.multinomial(1, weights, (n,)), axis=1)
        samples = rng.normal(loc=mus[active], scale=sigmas[active])
    else:
        low, high = float(low), float(high)
        if low >= high:
            raise ValueError('low >= high', (low, high))
        out = []
        while len(out) < n:
            k = np.argmax(rng.multinomial(1, weights))
            draw = rng.normal(loc=mus[k], scale=sigmas[k])
            if low <= draw < high:
                out.append(draw)
        samples = np.asarray(out)
    samples = np.reshape(np.asarray(samples), size)
    return samples if q is None else np.round(samples / q) * q


def lgmm1_sample(rng, weights, mus, sigmas, low=None, high=None, q=None, size=0):
    """tpe.py:216-250: sample in log space, exponentiate, then quantize."""
    weights, mus, sigmas = map(np.asarray, (weights, mus, sigmas))
    n = int(np.prod(size))
    if low is None and high is None:
        active = np.argmax(rng.multinomial(1, weights, (n,)), axis=1)
        samples = np.exp(rng.normal(loc=mus[active], scale=sigmas[active]))
    else:
        low, high = float(low), float(high)
        if low >= high:
            raise ValueError('low >= high', (low, high))
        out = []
        while len(out) < n:
            k = np.argmax(rng.multinomial(1, weights))
            draw = rng.normal(loc=mus[k], scale=sigmas[k])
            if low <= draw < high:
                out.append(np.exp(draw))
        samples = np.asarray(out)
    samples = np.reshape(np.asarray(samples), size)
    return samples if q is None else np.round(samples / q) * q


def categorical_sample(rng, p, size):
    """pyll/stochastic.py:104-142 (1-D p): one multinomial row per draw."""
    p = np.asarray(p)
    if size == 0:
        return np.asarray([])
    sample = rng.multinomial(n=1, pvals=p, size=int(size))
    return np.dot(sample, np.arange(len(p)))


# ---------------------------------------------------------------------------
# Parzen estimator
# ---------------------------------------------------------------------------


def linear_forgetting_weights(N, LF):
    """tpe.py:381-394"""
    if N == 0:
        return np.asarray([])
    if N < LF:
        return np.ones(N)
    return np.concatenate([np.linspace(1.0 / N, 1.0, num=N - LF), np.ones(LF)])


def adaptive_parzen_normal(mus, prior_weight, prior_mu, prior_sigma, LF=DEFAULT_LF):
    """tpe.py:398-475: sort the observations, insert the prior at
    ``searchsorted`` (side='left'), bandwidth = larger neighbour gap, clip to
    [prior_sigma / min(100, 1 + K), prior_sigma], linear-forgetting weights."""
    mus = np.array(mus)
    n = len(mus)
    order = None
    if n == 0:
        srtd = np.asarray([prior_mu])
        sigma = np.asarray([prior_sigma])
        pos = 0
    elif n == 1:
        if prior_mu < mus[0]:
            pos = 0
            srtd = np.asarray([prior_mu, mus[0]])
            sigma = np.asarray([prior_sigma, prior_sigma * .5])
        else:
            pos = 1
            srtd = np.asarray([mus[0], prior_mu])
            sigma = np.asarray([prior_sigma * .5, prior_sigma])
    else:
        order = np.argsort(mus)
        pos = np.searchsorted(mus[order], prior_mu)
        srtd = np.zeros(n + 1)
        srtd[:pos] = mus[order[:pos]]
        srtd[pos] = prior_mu
        srtd[pos + 1:] = mus[order[pos:]]
        sigma = np.zeros_like(srtd)
        sigma[1:-1] = np.maximum(srtd[1:-1] - srtd[0:-2], srtd[2:] - srtd[1:-1])
        sigma[0] = srtd[1] - srtd[0]
        sigma[-1] = srtd[-1] - srtd[-2]
    if LF and LF < n:
        lfw = linear_forgetting_weights(n, LF)
        weights = np.zeros_like(srtd)
        weights[:pos] = lfw[order[:pos]]
        weights[pos] = prior_weight
        weights[pos + 1:] = lfw[order[pos:]]
    else:
        weights = np.ones(len(srtd))
        weights[pos] = prior_weight
    maxsigma = prior_sigma / 1.0
    minsigma = prior_sigma / min(100.0, (1.0 + len(srtd)))
    sigma = np.clip(sigma, minsigma, maxsigma)
    sigma[pos] = prior_sigma
    assert np.all(sigma > 0)
    weights /= weights.sum()
    return weights, srtd, sigma


def ap_filter_trials(o_idxs, o_vals, l_idxs, l_vals, gamma, gamma_cap=DEFAULT_LF):
    """tpe.py:613-641: the n_below best losses over ALL trials, then split this
    parameter's observations (kept in tid order) by tid membership."""
    o_idxs, o_vals, l_idxs, l_vals = map(np.asarray, [o_idxs, o_vals, l_idxs, l_vals])
    n_below = min(int(np.ceil(gamma * np.sqrt(len(l_vals)))), gamma_cap)
    l_order = np.argsort(l_vals)
    keep = set(l_idxs[l_order[:n_below]])
    below = [v for i, v in zip(o_idxs, o_vals) if i in keep]
    keep = set(l_idxs[l_order[n_below:]])
    above = [v for i, v in zip(o_idxs, o_vals) if i in keep]
    return np.asarray(below), np.asarray(above)


def broadcast_best_index(below_llik, above_llik):
    """tpe.py:749-759: argmax of l - g, first index on ties (np.argmax)."""
    return int(np.argmax(np.asarray(below_llik) - np.asarray(above_llik)))


# ---------------------------------------------------------------------------
# posterior construction per prior family (tpe.py:485-607)
# ---------------------------------------------------------------------------


class Posterior(object):
    """One fitted posterior: how to sample it and how to evaluate it."""

    def __init__(self, kind, params, low=None, high=None, q=None):
        self.kind = kind          # 'gmm1' | 'lgmm1' | 'categorical'
        self.params = params      # (w, mu, sigma) or (p,)
        self.low, self.high, self.q = low, high, q

    def sample(self, rng, size):
        if self.kind == 'gmm1':
            return gmm1_sample(rng, *self.params, low=self.low, high=self.high, q=self.q, size=size)
        if self.kind == 'lgmm1':
            return lgmm1_sample(rng, *self.params, low=self.low, high=self.high, q=self.q, size=size)
        return categorical_sample(rng, self.params[0], size)

    def lpdf(self, samples):
        if self.kind == 'gmm1':
            return gmm1_lpdf(samples, *self.params, low=self.low, high=self.high, q=self.q)
        if self.kind == 'lgmm1':
            return lgmm1_lpdf(samples, *self.params, low=self.low, high=self.high, q=self.q)
        return categorical_lpdf(samples, self.params[0])


def fit_posterior(dist, args, obs, prior_weight, LF=DEFAULT_LF):
    """adaptive_parzen_samplers registry, tpe.py:485-607."""
    a = args
    obs = np.asarray(obs)
    if dist in ('uniform', 'quniform'):                         # :485-502
        pmu, psig = 0.5 * (a['high'] + a['low']), 1.0 * (a['high'] - a['low'])
        fit = adaptive_parzen_normal(obs, prior_weight, pmu, psig, LF)
        return Posterior('gmm1', fit, a['low'], a['high'], a.get('q'))
    if dist == 'loguniform':                                    # :505-514
        pmu, psig = 0.5 * (a['high'] + a['low']), 1.0 * (a['high'] - a['low'])
        fit = adaptive_parzen_normal(np.log(obs), prior_weight, pmu, psig, LF)
        return Posterior('lgmm1', fit, a['low'], a['high'], None)
    if dist == 'qloguniform':                                   # :517-535
        pmu, psig = 0.5 * (a['high'] + a['low']), 1.0 * (a['high'] - a['low'])
        tobs = np.log(np.maximum(obs, np.maximum(EPS, np.exp(a['low']))))
        fit = adaptive_parzen_normal(tobs, prior_weight, pmu, psig, LF)
        return Posterior('lgmm1', fit, a['low'], a['high'], a['q'])
    if dist in ('normal', 'qnormal'):                           # :540-551
        fit = adaptive_parzen_normal(obs, prior_weight, a['mu'], a['sigma'], LF)
        return Posterior('gmm1', fit, None, None, a.get('q'))
    if dist == 'lognormal':                                     # :554-559
        fit = adaptive_parzen_normal(np.log(obs), prior_weight, a['mu'], a['sigma'], LF)
        return Posterior('lgmm1', fit, None, None, None)
    if dist == 'qlognormal':                                    # :562-568
        fit = adaptive_parzen_normal(np.log(np.maximum(obs, EPS)), prior_weight,
                                     a['mu'], a['sigma'], LF)
        return Posterior('lgmm1', fit, None, None, a['q'])
    if dist == 'randint':                                       # :573-581
        upper = a['upper']
        lfw = linear_forgetting_weights(len(obs), LF)
        counts = (np.bincount(obs.astype(np.int64), lfw, upper) if obs.size
                  else np.zeros(upper, dtype='int'))
        pseudo = counts + prior_weight
        return Posterior('categorical', (pseudo / np.sum(pseudo),))
    if dist == 'categorical':                                   # :590-607
        upper = a['upper']
        p = np.asarray(a['p'], dtype=float)
        lfw = linear_forgetting_weights(len(obs), LF)
        counts = (np.bincount(obs.astype(np.int64), lfw, upper) if obs.size
                  else np.zeros(upper, dtype='int'))
        pseudo = counts + upper * (prior_weight * p)
        return Posterior('categorical', (pseudo / np.sum(pseudo),))
    raise ValueError('unknown distribution %r' % dist)


# ---------------------------------------------------------------------------
# prior draws (rand.suggest / pyll/stochastic.py:30-101)
# ---------------------------------------------------------------------------


def prior_sample(rng, dist, a, size):
    if dist == 'uniform':
        return rng.uniform(a['low'], a['high'], size=size)
    if dist == 'quniform':
        return np.round(rng.uniform(a['low'], a['high'], size=size) / a['q']) * a['q']
    if dist == 'loguniform':
        return np.exp(rng.uniform(a['low'], a['high'], size=size))
    if dist == 'qloguniform':
        return np.round(np.exp(rng.uniform(a['low'], a['high'], size=size)) / a['q']) * a['q']
    if dist == 'normal':
        return rng.normal(a['mu'], a['sigma'], size=size)
    if dist == 'qnormal':
        return np.round(rng.normal(a['mu'], a['sigma'], size=size) / a['q']) * a['q']
    if dist == 'lognormal':
        return np.exp(rng.normal(a['mu'], a['sigma'], size=size))
    if dist == 'qlognormal':
        return np.round(np.exp(rng.normal(a['mu'], a['sigma'], size=size)) / a['q']) * a['q']
    if dist == 'randint':
        return rng.randint(a['upper'], size=size)
    if dist == 'categorical':
        return categorical_sample(rng, a['p'], size)
    raise ValueError(dist)


# ---------------------------------------------------------------------------
# evaluation order (pyll/base.py:679-836 LIFO rec_eval over as_apply-sorted dicts)
# ---------------------------------------------------------------------------


def _resolve_order(params):
    """Labels in the order their random draws consume the shared RandomState.

    ``rec_eval`` pops the vals dict's inputs, pushed in sorted-label order
    (pyll/base.py:179-190 sorts dict items), so labels are visited in
    DESCENDING order; a conditional label's draw size depends on its parent's
    choice, so its ancestors are resolved first (depth-first)."""
    by_label = {p['label']: p for p in params}
    order, seen = [], set()

    def visit(label):
        if label in seen:
            return
        parent = by_label[label].get('parent')
        if parent is not None:
            visit(parent[0])
        seen.add(label)
        order.append(label)

    for label in sorted(by_label, reverse=True):
        visit(label)
    return order


def _is_active(param, chosen):
    parent = param.get('parent')
    if parent is None:
        return True
    plabel, pval = parent
    return plabel in chosen and chosen[plabel] is not None and int(chosen[plabel]) == pval


# ---------------------------------------------------------------------------
# suggest
# ---------------------------------------------------------------------------


def rand_suggest(params, seed):
    """rand.py:14-33 for one new id: each active label draws size=1 from its
    prior, inactive labels draw size=0 (no RandomState consumption)."""
    rng = np.random.RandomState(seed)
    by_label = {p['label']: p for p in params}
    chosen = {}
    for label in _resolve_order(params):
        p = by_label[label]
        if _is_active(p, chosen):
            chosen[label] = prior_sample(rng, p['dist'], p['args'], 1)[0]
        else:
            chosen[label] = None
    return {k: v for k, v in chosen.items() if v is not None}


def history_arrays(history):
    """tpe.py:820-842 + base.py:108-123.

    ``history`` is a list of dicts ``{tid, loss (None => +inf), vals: {label:
    [v] or []}, from_tid (optional)}``.  Keeps the lowest-loss doc per tid
    (``<=`` so the later of equal losses wins) and sorts by tid."""
    best_loss, best_doc = {}, {}
    for doc in history:
        tid = doc.get('from_tid', doc['tid'])
        loss = doc['loss']
        loss = float('inf') if loss is None else float(loss)
        best_loss.setdefault(tid, loss)
        if loss <= best_loss[tid]:
            best_loss[tid] = loss
            best_doc[tid] = doc
    tids = sorted(best_doc)
    losses = [best_loss[t] for t in tids]
    docs = [best_doc[t] for t in tids]
    return tids, losses, docs


def _lpdf_chunk(job):
    post, cand = job
    return post.lpdf(cand)


def _lpdf(post, cand, pool, chunks):
    """post.lpdf(cand), optionally split over a process pool by candidate
    chunks — bit-identical, because every lpdf is computed row by row
    (logsum_rows, tpe.py:253-256; the quantized per-component loop is
    elementwise)."""
    if pool is None or chunks < 2 or post.kind == 'categorical' or len(cand) < 2 * chunks:
        return post.lpdf(cand)
    return np.concatenate(pool.map(_lpdf_chunk, [(post, c) for c in np.array_split(cand, chunks)]))


def tpe_suggest(params, history, seed, prior_weight=1.0, n_startup_jobs=20,
                n_EI_candidates=24, gamma=0.25, LF=DEFAULT_LF, trace=None, pool=None, chunks=1):
    """tpe.py:804-897 for one new id.  Returns {label: value} of active labels.

    If ``trace`` is a dict it receives, per label, the fitted posteriors, the
    candidates, l, g and the chosen index (for kernel-level fixtures).  With a
    ``pool`` (multiprocessing) the candidate scoring is split into ``chunks``
    (the all-core CPU baseline); the result is identical."""
    tids, losses, docs = history_arrays(history)
    if len(docs) < n_startup_jobs:
        return rand_suggest(params, seed)
    rng = np.random.RandomState(seed)
    by_label = {p['label']: p for p in params}
    chosen = {}
    for label in _resolve_order(params):
        p = by_label[label]
        o_idxs = [d['tid'] for d in docs if len(d['vals'].get(label, [])) == 1]
        o_vals = [d['vals'][label][0] for d in docs if len(d['vals'].get(label, [])) == 1]
        below, above = ap_filter_trials(o_idxs, o_vals, tids, losses, gamma)
        if not _is_active(p, chosen):
            chosen[label] = None
            continue
        post_b = fit_posterior(p['dist'], p['args'], below, prior_weight, LF)
        post_a = fit_posterior(p['dist'], p['args'], above, prior_weight, LF)
        cand = post_b.sample(rng, n_EI_candidates)
        l = _lpdf(post_b, cand, pool, chunks)
        g = _lpdf(post_a, cand, pool, chunks)
        best = broadcast_best_index(l, g)
        chosen[label] = cand[best]
        if trace is not None:
            trace[label] = dict(below=below, above=above, post_b=post_b, post_a=post_a,
                                cand=cand, l=l, g=g, best=best)
    return {k: v for k, v in chosen.items() if v is not None}


def fmin(fn, params, max_evals, rstate, suggest=tpe_suggest, **suggest_kw):
    """fmin.py:68-140 serial loop: one new id per iteration, seed drawn as
    ``rstate.randint(2**31 - 1)``, evaluated immediately.  ``fn`` receives the
    {label: value} dict of active labels."""
    history = []
    for tid in range(max_evals):
        seed = rstate.randint(2 ** 31 - 1)
        vals = suggest(params, history, seed, **suggest_kw) if suggest is tpe_suggest \
            else suggest(params, seed)
        loss = fn(vals)
        history.append(dict(tid=tid, loss=loss,
                            vals={p['label']: ([vals[p['label']]] if p['label'] in vals else [])
                                  for p in params}))
    return history


def suggest_rate_sample(params, history, seed, n_EI_candidates, **kw):
    """Timed unit for bench.py's cpu_baseline: one tpe_suggest; returns the
    number of candidate-scores it produced (Σ over active labels of C)."""
    out = tpe_suggest(params, history, seed, n_EI_candidates=n_EI_candidates, **kw)
    return len(out) * n_EI_candidates
