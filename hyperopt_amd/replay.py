"""Exact-replay candidate draws with the reference's RandomState stream.

Parity mode only (``tpe.suggest(..., sampler='replay')``).  The reference draws
candidates with one shared ``np.random.RandomState(seed)``: bounded mixtures by
a per-draw rejection loop (tpe.py:82-87, :240-244), unbounded ones with one
vectorised multinomial + normal (tpe.py:73-74, :224-231), categoricals with
one multinomial row per draw (pyll/stochastic.py:126-131).  MT19937 plus the
rejection loop is inherently sequential, so these draws stay on the host; the
scoring and argmax of the drawn candidates still run on the GPU.  The
performance path is ``sampler='philox'`` (device-side sampling).
"""
import numpy as np


def draw_mixture(rng, w, mu, sigma, low, high, q, log_space, size):
    n = int(size)
    w, mu, sigma = np.asarray(w), np.asarray(mu), np.asarray(sigma)
    if low is None and high is None:
        k = np.argmax(rng.multinomial(1, w, (n,)), axis=1)
        x = rng.normal(loc=mu[k], scale=sigma[k])
        if log_space:
            x = np.exp(x)
    else:
        low, high = float(low), float(high)
        if low >= high:
            raise ValueError('low >= high', (low, high))
        out = []
        while len(out) < n:
            k = np.argmax(rng.multinomial(1, w))
            d = rng.normal(loc=mu[k], scale=sigma[k])
            if low <= d < high:
                out.append(np.exp(d) if log_space else d)
        x = np.asarray(out)
    x = np.reshape(np.asarray(x), (n,))
    return x if q is None else np.round(x / q) * q


def draw_categorical(rng, p, size):
    if size == 0:
        return np.asarray([], dtype=np.int64)
    p = np.asarray(p)
    return np.dot(rng.multinomial(n=1, pvals=p, size=int(size)), np.arange(len(p)))


def draw(rng, post, size):
    """``size`` candidates from ``post``'s below mixture."""
    from . import _native as N
    if post.family == N.FAM_CATEGORICAL:
        return draw_categorical(rng, post.below[0], size)
    log_space = post.family in (N.FAM_LOGGAUSS, N.FAM_QLOGGAUSS)
    w, mu, sigma = post.below
    return draw_mixture(rng, w, mu, sigma, post.low, post.high, post.q, log_space, size)
