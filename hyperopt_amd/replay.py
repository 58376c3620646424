"""Exact-replay candidate draws with the reference's RandomState stream.

Parity mode only (``tpe.suggest(..., sampler='replay')``).  The reference draws
candidates with one shared ``np.random.RandomState(seed)``: bounded mixtures by
a per-draw rejection loop (tpe.py:82-87, :240-244), unbounded ones with one
vectorised multinomial + normal (tpe.py:73-74, :224-231), categoricals with
one multinomial row per draw (pyll/stochastic.py:126-131).  MT19937 plus the
rejection loop is sequential, so these draws stay on the host — in native code
(tpe_replay_mixture / tpe_replay_categorical: MT19937, the legacy polar gauss,
multinomial(1, p) by binomial inversion), continuing the RandomState's own
state, which is written back after every call.  exp and rounding are applied
here with numpy, vectorised, exactly as the reference applies them.  The
scoring and argmax of the drawn candidates run on the GPU.  The performance
path is ``sampler='philox'`` (device-side sampling).
"""
import numpy as np


def _state(rng):
    """RandomState -> MTState (legacy get_state tuple)."""
    from . import _native as N
    name, key, pos, has_gauss, gauss = rng.get_state(legacy=True)
    st = N.MTState()
    np.frombuffer(st.key, dtype=np.uint32)[:] = key
    st.pos, st.has_gauss, st.gauss = int(pos), int(has_gauss), float(gauss)
    return st


def _restore(rng, st):
    rng.set_state(('MT19937', np.frombuffer(st.key, dtype=np.uint32).copy(), int(st.pos), int(st.has_gauss),
                   float(st.gauss)))


def draw_mixture(rng, w, mu, sigma, low, high, q, log_space, size):
    """``size`` draws from the mixture (native MT19937 stream, numpy's exp and
    rounding); equal to draw_mixture_numpy's, RandomState left in the same
    state."""
    import ctypes
    from . import _native as N
    n = int(size)
    w = np.ascontiguousarray(w, dtype=np.float64)
    mu = np.ascontiguousarray(mu, dtype=np.float64)
    sigma = np.ascontiguousarray(sigma, dtype=np.float64)
    bounded = not (low is None and high is None)
    if bounded:
        low, high = float(low), float(high)
        if low >= high:
            raise ValueError('low >= high', (low, high))
    st = _state(rng)
    d = np.empty(n, dtype=np.float64)
    rc = N.load().tpe_replay_mixture(ctypes.addressof(st), w.ctypes.data, mu.ctypes.data, sigma.ctypes.data, len(w),
                                     int(bounded), low if bounded else 0.0, high if bounded else 0.0, n,
                                     d.ctypes.data)
    if rc != 0:
        # numpy's own error for the same arguments (bad pvals, negative scale)
        return draw_mixture_numpy(rng, w, mu, sigma, low if bounded else None, high if bounded else None, q,
                                  log_space, size)
    _restore(rng, st)
    x = np.exp(d) if log_space else d
    return x if q is None else np.round(x / q) * q


def draw_categorical(rng, p, size):
    """``size`` categorical draws (native multinomial rows), as
    draw_categorical_numpy."""
    import ctypes
    from . import _native as N
    if size == 0:
        return np.asarray([], dtype=np.int64)
    p = np.ascontiguousarray(p, dtype=np.float64)
    st = _state(rng)
    out = np.empty(int(size), dtype=np.int64)
    rc = N.load().tpe_replay_categorical(ctypes.addressof(st), p.ctypes.data, len(p), int(size), out.ctypes.data)
    if rc != 0:
        return draw_categorical_numpy(rng, p, size)
    _restore(rng, st)
    return out


def draw_mixture_numpy(rng, w, mu, sigma, low, high, q, log_space, size):
    """The reference's draw sequence in numpy (tpe.py:71-93, :223-250): the
    specification draw_mixture is tested against."""
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


def draw_categorical_numpy(rng, p, size):
    """pyll/stochastic.py:126-131 in numpy (draw_categorical's specification)."""
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
