"""Host-side Parzen estimator and posterior construction.

The fit stays on the host in float64 numpy because it must reproduce the
reference's ``np.argsort`` permutation exactly (tie order among duplicate
observations changes the mixture, SURVEY.md §7 "Tie semantics"); calling the
same numpy routine on the same array is the only way to get that permutation.
The O(C*K) work it feeds runs on the GPU (``engine``).

References (gsmafra/hyperopt, /root/reference):
  linear_forgetting_weights  tpe.py:381-394
  adaptive_parzen_normal     tpe.py:398-475
  adaptive_parzen_samplers   tpe.py:485-607
  normal_cdf                 tpe.py:96-101 (p_accept, tpe.py:130-136)
"""
import math

import numpy as np
from scipy.special import erf, erfc

from . import _native as N

EPS = 1e-12
DEFAULT_LF = 25


def linear_forgetting_weights(n, lf):
    """Oldest observations (tid order) get a linear ramp from 1/n, the newest
    ``lf`` weigh 1 (tpe.py:381-394)."""
    if n == 0:
        return np.zeros(0)
    if n < lf:
        return np.ones(n)
    return np.concatenate([np.linspace(1.0 / n, 1.0, num=n - lf), np.ones(lf)])


def fit_parzen(obs, prior_weight, prior_mu, prior_sigma, lf=DEFAULT_LF):
    """Adaptive Parzen mixture (w, mu, sigma), mu sorted ascending — native
    (tpe_host_fit_parzen) with numpy's own argsort permutation."""
    obs = np.ascontiguousarray(obs, dtype=np.float64)
    n = obs.shape[0]
    order = np.argsort(obs) if n >= 2 else None
    w = np.empty(n + 1)
    mu = np.empty(n + 1)
    sigma = np.empty(n + 1)
    lib = N.load()
    pos = lib.tpe_host_fit_parzen(obs.ctypes.data, n, order.ctypes.data if order is not None else None,
                                  float(prior_weight), float(prior_mu), float(prior_sigma), int(lf or 0),
                                  w.ctypes.data, mu.ctypes.data, sigma.ctypes.data)
    if pos < 0:
        raise AssertionError('non-positive Parzen bandwidth (prior_sigma=%r)' % prior_sigma)
    return w, mu, sigma


def fit_parzen_numpy(obs, prior_weight, prior_mu, prior_sigma, lf=DEFAULT_LF):
    """Adaptive Parzen mixture (w, mu, sigma), mu sorted ascending — numpy
    version (the specification the native fit is tested against).

    Same semantics and float64 operation order as tpe.py:398-475: the prior is
    inserted at ``searchsorted`` (left) among the sorted observations, each
    bandwidth is the larger neighbour gap (one-sided at the ends), bandwidths
    are clipped to [prior_sigma / min(100, 1 + K), prior_sigma], the prior keeps
    prior_sigma, and linear-forgetting weights follow the observations through
    the sort."""
    obs = np.array(obs, dtype=float)
    n = obs.shape[0]
    if n == 0:
        mu = np.array([prior_mu], dtype=float)
        sigma = np.array([prior_sigma], dtype=float)
        pos = 0
        order = None
    elif n == 1:
        order = None
        if prior_mu < obs[0]:
            pos, mu = 0, np.array([prior_mu, obs[0]])
            sigma = np.array([prior_sigma, prior_sigma * .5])
        else:
            pos, mu = 1, np.array([obs[0], prior_mu])
            sigma = np.array([prior_sigma * .5, prior_sigma])
    else:
        order = np.argsort(obs)
        srt = obs[order]
        pos = int(np.searchsorted(srt, prior_mu))
        mu = np.empty(n + 1)
        mu[:pos] = srt[:pos]
        mu[pos] = prior_mu
        mu[pos + 1:] = srt[pos:]
        sigma = np.empty(n + 1)
        sigma[1:-1] = np.maximum(mu[1:-1] - mu[:-2], mu[2:] - mu[1:-1])
        sigma[0] = mu[1] - mu[0]
        sigma[-1] = mu[-1] - mu[-2]
    if lf and lf < n:
        ramp = linear_forgetting_weights(n, lf)[order]
        w = np.empty(n + 1)
        w[:pos] = ramp[:pos]
        w[pos] = prior_weight
        w[pos + 1:] = ramp[pos:]
    else:
        w = np.ones(len(mu))
        w[pos] = prior_weight
    lo = prior_sigma / min(100.0, 1.0 + len(mu))
    sigma = np.clip(sigma, lo, prior_sigma / 1.0)
    sigma[pos] = prior_sigma
    if not np.all(sigma > 0):
        raise AssertionError('non-positive Parzen bandwidth (prior_sigma=%r)' % prior_sigma)
    w /= w.sum()
    return w, mu, sigma


def normal_cdf(x, mu, sigma):
    """0.5 * (1 + erf((x - mu) / max(sqrt2 sigma, EPS))) — tpe.py:96-101."""
    return 0.5 * (1 + erf((x - mu) / np.maximum(np.sqrt(2) * sigma, EPS)))


def p_accept(w, mu, sigma, low, high):
    """Mixture mass inside [low, high) (tpe.py:130-136); 1 when unbounded."""
    if low is None and high is None:
        return 1
    return np.sum(w * (normal_cdf(high, mu, sigma) - normal_cdf(low, mu, sigma)))


# --------------------------------------------------------------------------
# posterior families (adaptive_parzen_samplers, tpe.py:485-607)
# --------------------------------------------------------------------------

_FAMILY = {
    'uniform': N.FAM_GAUSS, 'normal': N.FAM_GAUSS,
    'quniform': N.FAM_QGAUSS, 'qnormal': N.FAM_QGAUSS,
    'loguniform': N.FAM_LOGGAUSS, 'lognormal': N.FAM_LOGGAUSS,
    'qloguniform': N.FAM_QLOGGAUSS, 'qlognormal': N.FAM_QLOGGAUSS,
    'randint': N.FAM_CATEGORICAL, 'categorical': N.FAM_CATEGORICAL,
}


class Posterior(object):
    """A fitted below/above pair for one hyperparameter.

    family      engine family (``_native.FAM_*``)
    low, high   truncation in sampling space (log space for LGMM1), or None
    q           quantum or None
    below/above (w, mu, sigma) float64 arrays, or (p,) for categorical
    upper       number of categories (categorical)
    above_dev   None, or (device column, n_obs, below_idx int32, devhist.ValueOrder) when the above
                mixture is fitted on the device (engine: tpe_fit_above); then
                ``above`` is None and ``prior`` = (mu, sigma, weight, lf)
    """
    __slots__ = ('dist', 'family', 'low', 'high', 'q', 'below', 'above', 'upper', 'above_dev', 'prior', 'ptrs')

    def __init__(self, dist, family, low, high, q, below, above, upper=0, above_dev=None, prior=None, ptrs=None):
        self.dist, self.family = dist, family
        self.low, self.high, self.q = low, high, q
        self.below, self.above, self.upper = below, above, upper
        self.above_dev, self.prior = above_dev, prior
        # optional (below w, mu, sigma, K_below, above w, mu, sigma, K_above) host
        # addresses of the arrays above (set by the native fits: spares the
        # packer one ctypes address lookup per array)
        self.ptrs = ptrs

    @property
    def bounded(self):
        return self.low is not None or self.high is not None


def _cat_probs(dist, args, obs, prior_weight, lf):
    upper = int(args['upper'])
    obs = np.ascontiguousarray(obs, dtype=np.int64)
    p = None if dist == 'randint' else np.ascontiguousarray(args['p'], dtype=np.float64)
    out = np.empty(upper)
    rc = N.load().tpe_host_cat_probs(obs.ctypes.data, len(obs), upper, p.ctypes.data if p is not None else None,
                                     float(prior_weight), int(lf or 0), out.ctypes.data)
    if rc != 0:
        raise IndexError('categorical observation out of range [0, %d)' % upper)
    return out


def _cat_probs_numpy(dist, args, obs, prior_weight, lf):
    upper = int(args['upper'])
    lfw = linear_forgetting_weights(len(obs), lf)
    if len(obs):
        counts = np.bincount(np.asarray(obs, dtype=np.int64), lfw, upper)
    else:
        counts = np.zeros(upper, dtype='int')
    if dist == 'randint':                                   # tpe.py:573-581
        pseudo = counts + prior_weight
    else:                                                   # tpe.py:590-607
        pseudo = counts + upper * (prior_weight * np.asarray(args['p'], dtype=float))
    return pseudo / np.sum(pseudo)


DEVICE_FIT_FAMILIES = (N.FAM_GAUSS, N.FAM_LOGGAUSS)


def fit_coord(dist, args, obs):
    """The coordinate adaptive_parzen_normal fits a continuous label's
    observations in (tpe.py:485-568): the values, their log for the log
    families, clipped below first for the quantized log families.  Elementwise
    (so a column may be transformed in pieces)."""
    obs = np.asarray(obs, dtype=float)
    if dist in ('loguniform', 'lognormal'):
        return np.log(obs)
    if dist == 'qloguniform':                          # tpe.py:523-532
        return np.log(np.maximum(obs, np.maximum(EPS, np.exp(args['low']))))
    if dist == 'qlognormal':                           # tpe.py:564
        return np.log(np.maximum(obs, EPS))
    return obs


def fit_posterior(dist, args, below_obs, above_obs, prior_weight=1.0, lf=DEFAULT_LF, above_dev=None):
    """Fit the below and above posteriors of one hyperparameter.  With
    ``above_dev`` = (device column, n_obs, below_idx, value order) the above mixture is left
    to the device fit (continuous families only; ``above_obs`` is ignored)."""
    family = _FAMILY[dist]
    a = args
    if family == N.FAM_CATEGORICAL:
        return Posterior(dist, family, None, None, None,
                         (_cat_probs(dist, a, below_obs, prior_weight, lf),),
                         (_cat_probs(dist, a, above_obs, prior_weight, lf),), int(a['upper']))
    low = high = None
    if dist in ('uniform', 'quniform', 'loguniform', 'qloguniform'):
        low, high = float(a['low']), float(a['high'])
        pmu, psig = 0.5 * (a['high'] + a['low']), 1.0 * (a['high'] - a['low'])
    else:
        pmu, psig = a['mu'], a['sigma']
    q = a.get('q')
    q = None if q is None else float(q)

    def tr(obs):
        return fit_coord(dist, a, obs)

    below = fit_parzen(tr(below_obs), prior_weight, pmu, psig, lf)
    if above_dev is not None:
        if family not in DEVICE_FIT_FAMILIES:
            raise ValueError('device fit supports continuous families only, not %r' % dist)
        return Posterior(dist, family, low, high, q, below, None, above_dev=above_dev,
                         prior=(float(pmu), float(psig), float(prior_weight), int(lf or 0)))
    above = fit_parzen(tr(above_obs), prior_weight, pmu, psig, lf)
    return Posterior(dist, family, low, high, q, below, above)


def fit_split(dist, args, obs_tids, obs_vals, below_tids, order, prior_weight=1.0, lf=DEFAULT_LF, coord=None,
              addrs=None):
    """Continuous (non-quantized) label: the below/above split
    (ap_filter_trials, tpe.py:613-641) and both Parzen fits in one native call
    (tpe_host_fit_split), each side sorted by filtering ``order`` (a sorting
    permutation of all the label's values, History.value_order).  A side whose
    values repeat is refitted here with numpy's argsort permutation (the
    reference's tie order), so the result equals fit_posterior's bit for bit.
    ``below_tids`` ascending, ``obs_tids`` strictly ascending; ``coord``:
    optionally the values' kernel coordinate already computed (np.log of
    them for the log families, History.log_values); ``addrs``: optionally the
    host addresses (tids, coordinate, order, below_tids) of those same arrays
    (History.native_columns), sparing the per-call pointer lookups."""
    family = _FAMILY[dist]
    if family not in (N.FAM_GAUSS, N.FAM_LOGGAUSS):
        raise ValueError('fit_split fits continuous families only, not %r' % dist)
    a = args
    low = high = None
    if dist in ('uniform', 'loguniform'):
        low, high = float(a['low']), float(a['high'])
        pmu, psig = 0.5 * (a['high'] + a['low']), 1.0 * (a['high'] - a['low'])
    else:
        pmu, psig = a['mu'], a['sigma']
    if coord is not None:
        x = np.ascontiguousarray(coord, dtype=np.float64)
    else:
        x = np.ascontiguousarray(obs_vals, dtype=np.float64)
        if family == N.FAM_LOGGAUSS:
            x = np.log(x)                                 # monotone: `order` still sorts x
    tids = np.ascontiguousarray(obs_tids, dtype=np.int64)
    order = np.ascontiguousarray(order, dtype=np.int64)
    bt = np.ascontiguousarray(below_tids, dtype=np.int64)
    n = len(x)
    if len(order) != n:
        raise ValueError('order has %d entries for %d observations' % (len(order), n))
    cap = n + 1
    out = np.empty(6 * cap + 2)                       # (+ the two component counts, as int64)
    base = out.ctypes.data
    if addrs is None:
        addrs = (tids.ctypes.data, x.ctypes.data, order.ctypes.data, bt.ctypes.data)
    rc = N.load().tpe_host_fit_split(addrs[1], addrs[0], addrs[2], n, addrs[3], len(bt), float(prior_weight),
                                     float(pmu), float(psig), int(lf or 0), base, base + 8 * 6 * cap)
    k = out[6 * cap:].view(np.int64)
    if rc != 0:
        raise AssertionError('tpe_host_fit_split failed (%d): tids not strictly ascending, a bad order, or a '
                             'non-positive Parzen bandwidth (prior_sigma=%r)' % (rc, psig))
    sides = []
    mask = None
    ptrs = []
    for sd in range(2):
        m = int(k[sd])
        if m:
            r = out[3 * sd * cap:]
            sides.append((r[:m], r[cap:cap + m], r[2 * cap:2 * cap + m]))
            a0 = base + 3 * sd * cap * 8
            ptrs += [a0, a0 + cap * 8, a0 + 2 * cap * 8, m]
            continue
        if mask is None:
            mask = np.isin(tids, bt)
        sides.append(fit_parzen(x[mask] if sd == 0 else x[~mask], prior_weight, pmu, psig, lf))
    return Posterior(dist, family, low, high, None, sides[0], sides[1],
                     ptrs=tuple(ptrs) if len(ptrs) == 8 else None)      # both sides native


def cat_split(dist, args, obs_tids, obs_vals, below_tids, prior_weight=1.0, lf=DEFAULT_LF, addrs=None):
    """Categorical label: the below/above split and both pseudo-count
    posteriors in one native call (tpe_host_cat_split); equal to
    fit_posterior's.  ``below_tids`` ascending, ``obs_tids`` strictly
    ascending; ``addrs``: optionally (tids, values, below_tids) host addresses
    of those arrays (History.cat_columns)."""
    upper = int(args['upper'])
    obs = np.ascontiguousarray(obs_vals, dtype=np.int64)
    tids = np.ascontiguousarray(obs_tids, dtype=np.int64)
    bt = np.ascontiguousarray(below_tids, dtype=np.int64)
    p = None if dist == 'randint' else np.ascontiguousarray(args['p'], dtype=np.float64)
    out = np.empty(2 * upper)
    base = out.ctypes.data
    if addrs is None:
        addrs = (tids.ctypes.data, obs.ctypes.data, bt.ctypes.data)
    rc = N.load().tpe_host_cat_split(addrs[1], addrs[0], len(obs), addrs[2], len(bt), upper,
                                     p.ctypes.data if p is not None else None, float(prior_weight), int(lf or 0),
                                     base, base + 8 * upper)
    if rc != 0:
        raise IndexError('categorical observation out of range [0, %d) or tids not ascending' % upper)
    return Posterior(dist, N.FAM_CATEGORICAL, None, None, None, (out[:upper],), (out[upper:],), upper,
                     ptrs=(base, 0, 0, upper, base + 8 * upper, 0, 0, upper))


# --------------------------------------------------------------------------
# device tables (layout documented in include/tpe_hip.h)
# --------------------------------------------------------------------------

LOG2E = 1.0 / math.log(2.0)
A_SCALE = math.sqrt(0.5 * LOG2E)


def gauss_table(w, mu, sigma, post, log_family):
    """Rows {mu, a, c} and the additive base of one continuous mixture.

    GMM1_lpdf  (tpe.py:138-144): log coef = log(w / sqrt(2 pi sigma^2) / p_accept)
    LGMM1_lpdf (tpe.py:278-281): log coef = log w - log(max(sigma,EPS) sqrt(2 pi))
                                 (ln x subtracted per candidate; no p_accept)
    In log2 units: term_k(t) = c_k - (a_k (t - mu_k))^2 with
    a_k = sqrt(log2(e)/2) / max(sigma_k, EPS); c is shifted so max_k c_k = 0
    and lpdf = ln2 * log2(sum_k 2^term_k) + base."""
    se = np.maximum(sigma, EPS)
    with np.errstate(divide='ignore'):
        if log_family:
            logcoef = np.log(w) - np.log(se * np.sqrt(2 * np.pi))
        else:
            pa = p_accept(w, mu, sigma, post.low, post.high)
            logcoef = np.log(w / np.sqrt(2 * np.pi * sigma ** 2) / pa)
    c = logcoef * LOG2E
    finite = np.isfinite(c)
    shift = float(np.max(c[finite])) if finite.any() else 0.0
    return mu, A_SCALE / se, c - shift, shift * math.log(2.0)


def quant_table(w, mu, sigma, post):
    """Rows {mu, b = max(sqrt2 sigma, EPS), w} and base = -log(p_accept)
    (tpe.py:145-160, :282-299)."""
    pa = p_accept(w, mu, sigma, post.low, post.high)
    with np.errstate(divide='ignore'):
        base = -float(np.log(pa))
    return mu, np.maximum(np.sqrt(2) * sigma, EPS), w, base


def sampler_table(post):
    """Below-mixture sampler rows {cum, mu, sigma, fa, fb, flip}.

    Bounded GMM1/LGMM1 draw by rejection (tpe.py:82-87): a component with
    probability w_k, a normal draw, accepted if low <= x < high.  Accepted
    draws are exactly: component k with probability ∝ w_k * mass_k, then a
    normal truncated to [low, high) — which the device samples by inversion,
    p = fa + u (fb - fa), z = Phi^-1(p).  When the standardised interval lies
    right of 0 it is mirrored (flip) so fa, fb keep relative precision."""
    if post.family == N.FAM_CATEGORICAL:
        p = np.asarray(post.below[0], dtype=float)
        rows = np.zeros((len(p), 8))
        cum = np.cumsum(p) / np.sum(p)
        cum[-1] = 1.0
        rows[:, 0] = cum
        return rows
    w, mu, sigma = post.below
    rows = np.zeros((len(w), 8))
    rows[:, 1] = mu
    rows[:, 2] = sigma
    if post.low is None and post.high is None:
        za = np.full(len(w), -np.inf)
        zb = np.full(len(w), np.inf)
    else:
        za = (post.low - mu) / sigma
        zb = (post.high - mu) / sigma
    flip = za > 0
    a = np.where(flip, -zb, za)
    b = np.where(flip, -za, zb)
    fa = 0.5 * erfc(-a / np.sqrt(2))
    fb = 0.5 * erfc(-b / np.sqrt(2))
    mass = np.maximum(fb - fa, 0.0)
    sel = np.asarray(w, dtype=float) * (mass if (post.low is not None or post.high is not None) else 1.0)
    if not np.any(sel > 0):          # every component outside the bounds
        sel = np.asarray(w, dtype=float)
    cum = np.cumsum(sel) / np.sum(sel)
    cum[-1] = 1.0
    rows[:, 0] = cum
    rows[:, 3] = fa
    rows[:, 4] = fb
    rows[:, 5] = flip
    return rows


PRUNE_MIN_K = 64      # smaller above mixtures are evaluated whole
PRUNE_WIDE = 16       # widest components evaluated for every candidate


def prune_tables(mu, a, c):
    """Split a sorted continuous above mixture for the pruned f32 kernel.

    Returns (narrow_c, wide_idx, meta): ``narrow_c`` is ``c`` with the wide
    components set to -inf (they are evaluated from the separate wide list),
    meta = dict(prior_mu, prior_a, prior_c, narrow_cmax, narrow_amin, grid_lo,
    grid_inv, grid) — see include/tpe_hip.h (pruned above mixture)."""
    K = len(mu)
    if K <= PRUNE_MIN_K:
        return c, np.zeros(0, dtype=np.int64), None
    wide = np.argsort(a, kind='stable')[:PRUNE_WIDE]        # smallest a = widest sigma
    anchor = wide[0]
    narrow = np.ones(K, dtype=bool)
    narrow[wide] = False
    nc = np.array(c, dtype=np.float64)
    nc[wide] = -np.inf
    mu32 = np.asarray(mu, dtype=np.float32).astype(np.float64)
    lo, hi = float(mu32[0]), float(mu32[-1])
    G = int(min(4096, 4 * K))
    inv = np.float32(G / (hi - lo)) if hi > lo else np.float32(0.0)
    edges = lo + np.arange(G, dtype=np.float64) * (1.0 / float(inv) if inv > 0 else 0.0)
    grid = np.empty(G + 1, dtype=np.int32)
    grid[:G] = np.searchsorted(mu32, edges, side='left') if inv > 0 else 0
    grid[G] = K
    meta = dict(prior_mu=float(mu[anchor]), prior_a=float(a[anchor]), prior_c=float(c[anchor]),
                narrow_cmax=float(np.max(np.asarray(c)[narrow])), narrow_amin=float(np.min(np.asarray(a)[narrow])),
                grid_lo=lo, grid_inv=float(inv), grid=grid)
    return nc, wide, meta
