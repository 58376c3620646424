"""k_sample_tab's CDF guide (tpe_kernels.hip, GuideEnt / guided_comp): a step
of the selection CDF is tested on the uniform's 32-bit word w as w >= T(c),
T(c) = ceil(c 2^32 - 1/2), instead of as !(u < c) on u = (w + 1/2) 2^-32
(draw_uniforms' u01w).  The two must agree for every w and every CDF value
c, T(c) >= 2^32 meaning "never passed"; checked here in f64 exactly as the
kernel computes both (no GPU).  Likewise the run keys (key32) that the
sample stage reduces by a wave max must order candidates exactly as
better32 (np.argmax: NaN first, then value, first index on ties)."""
import numpy as np


def _thresh(c):
    t = np.ceil(c * 4294967296.0 - 0.5)
    never = ~(t < 4294967296.0)
    return np.where(never, 0, np.maximum(t, 0)).astype(np.uint64), never


def _u01w(w):
    return (w.astype(np.float64) + 0.5) * 2.3283064365386963e-10


def test_integer_thresholds_match_the_f64_compare():
    rs = np.random.RandomState(7)
    cs = np.concatenate([
        rs.uniform(0, 1, 2000),
        np.array([0.0, 1e-300, 2.0 ** -33, 2.0 ** -32, 1.5 * 2.0 ** -32, 0.5, 1.0 - 2.0 ** -33,
                  1.0 - 2.0 ** -32, 1.0 - 1.5 * 2.0 ** -32, 1.0, np.inf]),
        (np.arange(1, 200) + 0.5) * 2.0 ** -32,          # exactly on a uniform: u < c is false there
        (np.arange(1, 200)) * 2.0 ** -32,
        np.nextafter((np.arange(1, 50) + 0.5) * 2.0 ** -32, 0.0),
    ])
    T, never = _thresh(cs)
    for c, t, nv in zip(cs, T, never):
        # every w near the threshold and a random sample elsewhere
        base = int(min(max(c, 0.0), 1.0) * 4294967296.0) if np.isfinite(c) else 4294967295
        near = np.arange(base - 3, base + 4, dtype=np.int64)
        ws = np.concatenate([near[(near >= 0) & (near < 2 ** 32)],
                             rs.randint(0, 2 ** 32, 64, dtype=np.uint64).astype(np.int64),
                             np.array([0, 2 ** 32 - 1])]).astype(np.uint64)
        passed_f64 = ~(_u01w(ws) < c)
        passed_int = np.zeros(len(ws), dtype=bool) if nv else ws >= t
        assert np.array_equal(passed_f64, passed_int), (c, t, nv)


def test_guide_bucket_is_the_top_byte():
    # floor(u * 256) of u01w(w) is w's top 8 bits for every w (no clamp needed)
    rs = np.random.RandomState(3)
    ws = np.concatenate([rs.randint(0, 2 ** 32, 100000, dtype=np.uint64),
                         np.array([0, 2 ** 24 - 1, 2 ** 24, 2 ** 32 - 1], dtype=np.uint64)])
    b = np.minimum(np.floor(_u01w(ws) * 256.0), 255).astype(np.uint64)
    assert np.array_equal(b, ws >> np.uint64(24))


def _better32(d, i, bd, bi):
    # tpe_kernels.hip better32: np.argmax order (NaN first, then value, first index)
    if bi < 0:
        return i >= 0
    if i < 0:
        return False
    n, bn = d != d, bd != bd
    if n or bn:
        return n and (not bn or i < bi)
    return d > bd or (d == bd and i < bi)


def _key32(d, i):
    # tpe_kernels.hip key32: the same order as one unsigned 64-bit key
    if i < 0:
        return 0
    if d != d:
        hi = 0xFFFFFFFF
    else:
        b = int(np.float32(d + np.float32(0.0)).view(np.uint32))
        hi = (~b & 0xFFFFFFFF) if b & 0x80000000 else (b | 0x80000000)
    return (hi << 32) | (~i & 0xFFFFFFFF)


def test_run_keys_order_candidates_as_better32():
    rs = np.random.RandomState(11)
    vals = [np.float32(v) for v in (0.0, -0.0, 1.0, -1.0, 3.5, -3.5, np.inf, -np.inf, np.nan, 1e-38, -1e-38)]
    vals += [np.float32(v) for v in rs.normal(0, 4, 40)]
    pairs = [(d, i) for d in vals for i in (-1, 0, 1, 7, 1000, 2 ** 31 - 1)]
    for _ in range(20000):
        (d1, i1), (d2, i2) = pairs[rs.randint(len(pairs))], pairs[rs.randint(len(pairs))]
        if i1 == i2 and i1 >= 0:
            continue                                   # candidate indices are unique within a run
        assert _better32(d1, i1, d2, i2) == (_key32(d1, i1) > _key32(d2, i2)), (d1, i1, d2, i2)
