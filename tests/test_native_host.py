"""The native host runtime (tpe_host.cpp) against its numpy specification:
bit-exact Parzen fits and categorical posteriors, and the packed level tables
equal to the numpy packer (no GPU needed)."""
import ctypes

import numpy as np
import pytest

from hyperopt_amd import _native as N
from hyperopt_amd import parzen
from hyperopt_amd.engine import Engine, LevelProblem


def _cases():
    rs = np.random.RandomState(0)
    yield np.zeros(0), 1.0, 0.5, 1.0
    yield np.array([0.3]), 1.0, 0.5, 1.0
    yield np.array([0.7]), 1.0, 0.5, 1.0
    yield np.array([0.5, 0.5]), 2.0, 0.5, 1.0
    for n in (2, 3, 24, 25, 26, 27, 100, 1000, 8191, 8192, 8193, 20000):
        yield rs.uniform(-3, 3, n), 1.0, 0.0, 6.0
        yield np.round(rs.uniform(0, 20, n)), 1.0, 10.0, 20.0        # ties everywhere
        yield rs.normal(0, 1, n) * 1e-3, 0.5, 1.0, 2.0                  # prior far right


def test_native_fit_matches_numpy_bit_exact():
    for obs, pw, pmu, psig in _cases():
        a = parzen.fit_parzen(obs, pw, pmu, psig)
        b = parzen.fit_parzen_numpy(obs, pw, pmu, psig)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)


def test_native_cat_probs_match_numpy_bit_exact():
    rs = np.random.RandomState(1)
    for n in (0, 1, 24, 25, 26, 300, 9000):
        for upper in (2, 5, 17):
            obs = rs.randint(0, upper, n)
            for dist, args in (('randint', dict(upper=upper)),
                               ('categorical', dict(upper=upper, p=list(rs.dirichlet(np.ones(upper)))))):
                a = parzen._cat_probs(dist, args, obs, 1.0, 25)
                b = parzen._cat_probs_numpy(dist, args, obs, 1.0, 25)
                np.testing.assert_array_equal(a, b)
    with pytest.raises(IndexError):
        parzen._cat_probs('randint', dict(upper=3), np.array([0, 3]), 1.0, 25)


@pytest.mark.parametrize('dist,args', [
    ('uniform', dict(low=-3.0, high=3.0)),
    ('normal', dict(mu=0.5, sigma=2.0)),
    ('loguniform', dict(low=-4.0, high=2.0)),
    ('lognormal', dict(mu=0.0, sigma=1.0)),
])
def test_fit_split_matches_fit_posterior(dist, args):
    """tpe_host_fit_split (merge split + the label's sorting permutation
    filtered per side + fit) against the masked fit_posterior path, bit-exact;
    sides with repeated values take numpy's permutation."""
    rs = np.random.RandomState(3)
    for n in (0, 1, 2, 25, 26, 300, 3000):
        tids = np.sort(rs.choice(4 * n + 10, n, replace=False)).astype(np.int64)
        for ties in (False, True):
            v = rs.uniform(-3, 3, n)
            if ties:
                v = np.round(v * 2) / 2
            vals = np.exp(v) if dist in ('loguniform', 'lognormal') else v
            order = np.argsort(vals, kind='stable')
            for nb in (0, 1, min(n, 25)):
                below = rs.permutation(tids)[:nb]
                a = parzen.fit_split(dist, args, tids, vals, np.sort(below), order, 1.0, 25)
                m = np.isin(tids, below)
                b = parzen.fit_posterior(dist, args, vals[m], vals[~m], 1.0, 25)
                assert (a.family, a.low, a.high, a.q) == (b.family, b.low, b.high, b.q)
                for sa, sb in ((a.below, b.below), (a.above, b.above)):
                    for x, y in zip(sa, sb):
                        np.testing.assert_array_equal(x, y)
    with pytest.raises(AssertionError):
        parzen.fit_split(dist, args, np.array([2, 1]), np.array([0.5, 0.7]), np.zeros(0, np.int64), np.array([0, 1]))
    with pytest.raises(AssertionError):
        parzen.fit_split(dist, args, np.array([1, 2]), np.array([0.5, 0.7]), np.zeros(0, np.int64), np.array([0, 2]))


def test_value_order_incremental():
    """The Trials cache's per-label sorting permutation, extended by merges as
    documents arrive, always sorts the column (and is None with a NaN)."""
    from hyperopt_amd import history as H
    c = H._Cache(['x'], {'x': False})
    rs = np.random.RandomState(5)
    col = c.obs_val['x']
    for step in range(40):
        for _ in range(rs.randint(0, 7)):
            col.append(rs.uniform() if rs.rand() > 0.2 else 0.5)
        vals = col.view()
        perm = c.value_order('x')
        assert sorted(perm.tolist()) == list(range(len(vals)))
        assert np.all(np.diff(vals[perm]) >= 0)
    col.append(np.nan)
    assert c.value_order('x') is None


def test_log_values_incremental():
    """The cache's np.log column (fit_split's kernel coordinate for the log
    families), extended as documents arrive, equals one np.log of the column."""
    from hyperopt_amd import history as H
    c = H._Cache(['x'], {'x': False})
    rs = np.random.RandomState(6)
    col = c.obs_val['x']
    for step in range(30):
        for _ in range(rs.randint(0, 90)):
            col.append(rs.uniform(1e-3, 1e3))
        np.testing.assert_array_equal(c.log_values('x'), np.log(col.view()))


def _engine(precision):
    e = Engine.__new__(Engine)
    e.lib, e.tile, e.precision, e._pinned, e._bufs, e.profile = N.load(), 2048, precision, None, {}, None
    return e


def _blob(e, info, off, dtype, count):
    return np.frombuffer(e._pinned.numpy(), dtype=dtype, count=count, offset=int(off))


@pytest.mark.parametrize('precision', ['fp32', 'fp64'])
def test_native_pack_matches_numpy_packer(precision):
    rs = np.random.RandomState(2)
    posts = [parzen.fit_posterior('loguniform', dict(low=-5.0, high=5.0), np.exp(rs.uniform(-5, 5, 20)),
                                  np.exp(rs.uniform(-5, 5, 3000)), 1.0),
             parzen.fit_posterior('uniform', dict(low=-1.0, high=2.0), rs.uniform(-1, 2, 5), rs.uniform(-1, 2, 40), 1.0),
             parzen.fit_posterior('normal', dict(mu=0.0, sigma=2.0), rs.normal(0, 2, 9), rs.normal(0, 2, 500), 1.0),
             parzen.fit_posterior('quniform', dict(low=0.0, high=10.0, q=1.0), np.round(rs.uniform(0, 10, 9)),
                                  np.round(rs.uniform(0, 10, 300)), 1.0),
             parzen.fit_posterior('qlognormal', dict(mu=1.0, sigma=0.5, q=0.25),
                                  np.round(np.exp(rs.normal(1, .5, 9)) / .25) * .25,
                                  np.round(np.exp(rs.normal(1, .5, 90)) / .25) * .25, 1.0),
             parzen.fit_posterior('categorical', dict(p=[.2, .3, .5], upper=3), rs.randint(0, 3, 9),
                                  rs.randint(0, 3, 90), 1.0),
             # (a bounded side of >= 2048 components: its acceptance terms come from
             # the packer's parallel pass, summed in numpy's order)
             parzen.fit_posterior('quniform', dict(low=-3.0, high=3.0, q=0.01), np.round(rs.uniform(-3, 3, 9), 2),
                                  np.round(np.clip(rs.normal(2.5, 0.4, 3000), -3, 3), 2), 1.0)]
    lps = [LevelProblem(p, i + 3, np.arange(i + 1) + 100) for i, p in enumerate(posts)]
    e = _engine(precision)
    for C in (24, 5000, 1 << 17):      # 2^17: fine sort keys and per-tile tail splits
        ref = e._build_numpy(lps, C, 77, 10, None)
        info = e._pack(lps, C, 77, 10, None)
        P = ref['P']
        assert info.n_problems == P and info.n_tiles == len(ref['tiles'])
        assert [info.n_work_cont, info.n_work_qgauss, info.n_work_qlog] == ref['counts_w']
        assert info.part_total == ref['part_total']
        prob = _blob(e, info, info.off_problems, N.PROBLEM_DTYPE, P)
        for f in N.PROBLEM_DTYPE.names:
            np.testing.assert_allclose(prob[f].astype(float), ref['prob'][f].astype(float), rtol=1e-6, atol=0,
                                       err_msg=f)
        # the large bounded quantized side's -log(acceptance mass): the same bits as numpy's
        assert prob['above_base'][-1] == ref['prob']['above_base'][-1]
        np.testing.assert_array_equal(_blob(e, info, info.off_tiles, N.TILE_DTYPE, info.n_tiles), ref['tiles'])
        nw = sum(ref['counts_w'])
        np.testing.assert_array_equal(_blob(e, info, info.off_work, N.WORK_DTYPE, nw), ref['work'])
        c32 = _blob(e, info, info.off_comp32, np.float32, ref['comp32'].size)
        np.testing.assert_allclose(c32, ref['comp32'].reshape(-1), rtol=1e-6, atol=1e-6)
        c64 = _blob(e, info, info.off_comp64, np.float64, ref['comp64'].size)
        np.testing.assert_allclose(c64, ref['comp64'].reshape(-1), rtol=1e-12, atol=0)
        smp = _blob(e, info, info.off_samp, np.float64, ref['samp'].size)
        np.testing.assert_allclose(smp, ref['samp'].reshape(-1), rtol=1e-12, atol=1e-300)
        if precision == 'fp32':
            g = _blob(e, info, info.off_grid, np.int32, ref['grid'].size)
            np.testing.assert_array_equal(g, ref['grid'])
        # score tables (include/tpe_hip.h "Tabulated scoring"): the same jobs and storage
        assert (info.n_tab_jobs, info.tab_units, info.tab_blocks) == (len(ref['tab_jobs']), ref['tab_units'],
                                                                     ref['tab_blocks'])
        np.testing.assert_array_equal(_blob(e, info, info.off_tab_jobs, N.TAB_JOB_DTYPE, info.n_tab_jobs),
                                      ref['tab_jobs'])
        modes = set(prob['tab_mode'].tolist())
        if C == 1 << 17:      # every continuous f32 label and the lattice labels tabulate at this size
            assert N.TAB_LATTICE in modes and (N.TAB_CELLS in modes) == (precision == 'fp32'), modes
        if C == 24:           # fewer candidates than cells: per-candidate scoring
            assert N.TAB_CELLS not in modes


def test_native_pack_chunked_sides_match_numpy_packer():
    """A level with >= 16384 components of large tabulated f32 sides: their
    rows and acceptance terms come from the chunk tasks (the mass folded into
    the side's base after the terms pass) and match the numpy packer's rows
    and bases."""
    rs = np.random.RandomState(4)
    posts = [parzen.fit_posterior('uniform', dict(low=-5.0, high=5.0), rs.uniform(-5, 5, 25), rs.uniform(-5, 5, 9000),
                                  1.0),
             parzen.fit_posterior('normal', dict(mu=0.0, sigma=2.0), rs.normal(0, 2, 20), rs.normal(0, 2, 6000), 1.0),
             parzen.fit_posterior('uniform', dict(low=0.0, high=1.0), rs.uniform(0, 1, 9), rs.uniform(0, 1, 4000),
                                  1.0)]
    lps = [LevelProblem(p, i + 3, np.arange(i + 1) + 100) for i, p in enumerate(posts)]
    e = _engine('fp32')
    C = 1 << 17
    ref = e._build_numpy(lps, C, 77, 10, None)
    info = e._pack(lps, C, 77, 10, None)
    P = ref['P']
    prob = _blob(e, info, info.off_problems, N.PROBLEM_DTYPE, P)
    assert set(prob['tab_mode'].tolist()) == {N.TAB_CELLS}
    for f in ('below_base', 'above_base', 'above_len', 'below_len'):
        np.testing.assert_allclose(prob[f].astype(float), ref['prob'][f].astype(float), rtol=1e-6, atol=0, err_msg=f)
    c32 = _blob(e, info, info.off_comp32, np.float32, ref['comp32'].size)
    np.testing.assert_allclose(c32, ref['comp32'].reshape(-1), rtol=1e-6, atol=1e-6)


def test_host_pool_swaps_under_concurrent_dispatch():
    """tpe_host_threads replaces the worker pool while other threads dispatch
    to it (the packer's parallel label fills): every pack stays identical to
    a serial one, and retired pools are freed by their last holder (no
    use-after-free: the dispatchers still holding one run serially)."""
    import threading
    rs = np.random.RandomState(9)
    posts = [parzen.fit_posterior('uniform', dict(low=-1.0, high=2.0), rs.uniform(-1, 2, 5), rs.uniform(-1, 2, 400),
                                  1.0) for _ in range(12)]
    lps = [LevelProblem(p, i, [100 + i]) for i, p in enumerate(posts)]
    lib = N.load()
    prev = ctypes.c_int32(0)
    assert lib.tpe_host_threads(-1, ctypes.byref(prev)) == 0
    def pack(e):
        if e._pinned is not None:
            e._pinned.zero_()                # (section padding is not written by the packer)
        inf = e._pack(lps, 4096, 5, 0, None)
        if inf.blob_bytes > 0 and e._pinned is not None:
            e._pinned.zero_()
            inf = e._pack(lps, 4096, 5, 0, None)
        return bytes(e._pinned.numpy()[:int(inf.blob_bytes)])
    ref = pack(_engine('fp32'))
    errors = []
    stop = threading.Event()

    def dispatcher():
        e = _engine('fp32')
        try:
            while not stop.is_set():
                if pack(e) != ref:
                    errors.append('pack differs')
        except Exception as ex:          # pragma: no cover
            errors.append(repr(ex))
    ts = [threading.Thread(target=dispatcher) for _ in range(3)]
    for t in ts:
        t.start()
    try:
        for k in range(60):
            assert lib.tpe_host_threads((2, 5, 3, 8)[k % 4], None) == 0
    finally:
        stop.set()
        for t in ts:
            t.join()
        lib.tpe_host_threads(prev.value, None)
    assert not errors, errors[:3]


class _FakeColumn(object):
    """Stand-in for a device column: the packer only records its address."""

    def data_ptr(self):
        return 0xD0000000


class _FakeOrder(object):
    """Stand-in for a devhist.ValueOrder with ``n`` observations already sorted."""

    class _Group(object):
        def ensure(self, slots, n_obs):
            pass

    def __init__(self, n):
        self.n = n
        self.group, self.slot = self._Group(), 0

    def ptrs(self, n_obs):
        return (0xE0000000 if self.n else 0, 0xE1000000 if self.n else 0, self.n,
                0xE2000000 if self.n < n_obs else 0, 0xE3000000 if self.n < n_obs else 0)


def test_pack_reserves_device_fit_rows():
    """A device-fitted above mixture (tpe_fit_job) gets its comp32 rows, wide
    rows and grid at the END of those sections (the grid's from a 256-B
    boundary), outside the host-written upload ranges, and a patch area for the
    problem fields the fit writes (the early fit: tpe_level_run)."""
    rs = np.random.RandomState(5)
    n_obs, bidx = 500, np.array([3, 10, 77], dtype=np.int32)
    host = parzen.fit_posterior('normal', dict(mu=0.0, sigma=2.0), rs.normal(0, 2, 9), rs.normal(0, 2, 300), 1.0)
    dev = parzen.fit_posterior('uniform', dict(low=-1.0, high=2.0), rs.uniform(-1, 2, 3), None, 1.0,
                               above_dev=(_FakeColumn(), n_obs, bidx, _FakeOrder(0)))
    assert dev.above is None and dev.prior == (0.5, 3.0, 1.0, 25)
    lps = [LevelProblem(host, 1, [5, 6]), LevelProblem(dev, 2, [5, 6, 7])]
    e = _engine('fp32')
    info = e._pack(lps, 4096, 1, 0, None)
    K = n_obs - len(bidx) + 1
    # a fresh order: every observation is new, the scratch segment holds them all
    assert info.n_fit == 1 and info.fit_total == n_obs and info.sort_end_bit > 0
    assert info.fit_max_new == n_obs and info.fit_max_obs == n_obs
    j = _blob(e, info, info.off_fit, N.FIT_JOB_DTYPE, 1)[0]
    assert j['obs'] == 0xD0000000 and j['n_obs'] == n_obs and j['seg_off'] == 0 and j['n_below'] == 3
    assert (j['ord_key_in'], j['ord_idx_in'], j['n_ord_in']) == (0, 0, 0)
    assert (j['ord_key_out'], j['ord_idx_out']) == (0xE2000000, 0xE3000000)
    assert j['problem_first'] == 2 and j['n_problems'] == 3 and j['family'] == N.FAM_GAUSS
    assert (j['prior_mu'], j['prior_sigma'], j['prior_weight'], j['lf']) == (0.5, 3.0, 1.0, 25)
    assert (j['low'], j['high']) == (-1.0, 2.0)
    np.testing.assert_array_equal(_blob(e, info, info.off_below_idx, np.int32, 3), bidx)
    np.testing.assert_array_equal(_blob(e, info, info.off_fit_seg, np.int64, 2), [0, n_obs])
    prob = _blob(e, info, info.off_problems, N.PROBLEM_DTYPE, 5)
    ups = [(int(info.up_off[i]), int(info.up_len[i])) for i in range(info.n_up)]
    host_rows = dict(ups)[info.off_comp32] // 16
    for p in prob[2:]:
        assert p['above_len'] == K and p['above_off'] == host_rows == j['above_off']
        assert p['wide_off'] == host_rows + K == j['wide_off']
        assert p['grid_off'] == j['grid_off'] and p['grid_n'] == j['grid_n'] == min(4096, 4 * K)
        assert p['narrow_amin'] > 0
    # host rows of the other label lie before the device region, its grid too
    assert prob[0]['above_off'] + prob[0]['above_len'] <= host_rows
    assert prob[0]['grid_off'] + prob[0]['grid_n'] + 1 <= j['grid_off']
    assert j['grid_off'] % 64 == 0 and ups[0] == (0, info.off_grid + 4 * (prob[0]['grid_off'] + prob[0]['grid_n'] + 1))
    dev_ranges = [(info.off_grid + 4 * j['grid_off'], 4 * (j['grid_n'] + 1)),
                  (info.off_comp32 + 16 * host_rows, 16 * (K + 16)), (info.off_patch, 5 * N.PROBLEM_DTYPE.itemsize)]
    for o, n in dev_ranges:                                  # (device-only bytes: in no upload range)
        assert all(o + n <= uo or o >= uo + un for uo, un in ups), (o, n, ups)
    assert info.off_patch >= info.off_comp32 + 16 * (host_rows + K + 16)
    assert ups[-1][0] == info.off_problems and ups[-1][0] + ups[-1][1] == info.blob_bytes
    with pytest.raises(RuntimeError):
        _engine('fp64')._pack(lps, 4096, 1, 0, None)


def test_pack_device_fit_resident_order():
    """A label whose value order already holds some observations merges only
    the rest: its scratch segment is sized by the compacted above order, and a
    fully sorted order passes no output buffers."""
    rs = np.random.RandomState(6)
    n_obs, bidx = 600, np.array([1, 50], dtype=np.int32)
    K = n_obs - len(bidx) + 1
    for n_sorted, out in ((n_obs - 7, True), (n_obs, False)):
        dev = parzen.fit_posterior('uniform', dict(low=-1.0, high=2.0), rs.uniform(-1, 2, 2), None, 1.0,
                                   above_dev=(_FakeColumn(), n_obs, bidx, _FakeOrder(n_sorted)))
        e = _engine('fp32')
        info = e._pack([LevelProblem(dev, 0, [9])], 4096, 1, 0, None)
        assert info.fit_total == K - 1 and info.fit_max_new == n_obs - n_sorted and info.fit_max_obs == n_obs
        assert info.fit_max_merge == n_obs - n_sorted and info.fit_n_delta == 0
        j = _blob(e, info, info.off_fit, N.FIT_JOB_DTYPE, 1)[0]
        assert (j['ord_key_in'], j['ord_idx_in'], j['n_ord_in']) == (0xE0000000, 0xE1000000, n_sorted)
        assert (j['ord_key_out'] != 0) == out and (j['ord_idx_out'] != 0) == out
    # delta mode: at most TPE_FIT_DELTA_MAX new observations and no output
    # buffers — the job reads them beside the order (no merge)
    for n_new in (1, N.FIT_DELTA_MAX):
        dl = parzen.fit_posterior('uniform', dict(low=-1.0, high=2.0), rs.uniform(-1, 2, 2), None, 1.0,
                                  above_dev=(_FakeColumn(), n_obs, bidx, _NoOut(n_obs - n_new)))
        e = _engine('fp32')
        info = e._pack([LevelProblem(dl, 0, [9])], 4096, 1, 0, None)
        j = _blob(e, info, info.off_fit, N.FIT_JOB_DTYPE, 1)[0]
        assert j['n_ord_in'] == n_obs - n_new and j['ord_key_out'] == 0 and j['ord_idx_out'] == 0
        assert info.fit_max_new == n_new and info.fit_max_merge == 0 and info.fit_n_delta == 1
    # more new observations than that (or no order at all) without output buffers: refused
    for n_in in (n_obs - N.FIT_DELTA_MAX - 1, 0):
        bad = parzen.fit_posterior('uniform', dict(low=-1.0, high=2.0), rs.uniform(-1, 2, 2), None, 1.0,
                                   above_dev=(_FakeColumn(), n_obs, bidx, _NoOut(n_in)))
        with pytest.raises(RuntimeError):
            _engine('fp32')._pack([LevelProblem(bad, 0, [9])], 4096, 1, 0, None)


class _NoOut(_FakeOrder):
    def ptrs(self, n_obs):
        return (0xE0000000, 0xE1000000, self.n, 0, 0)


def test_cat_split_matches_fit_posterior():
    """tpe_host_cat_split (merge split + both pseudo-count posteriors) equals
    the masked fit_posterior path bit for bit."""
    rs = np.random.RandomState(4)
    for n in (0, 1, 24, 25, 26, 300):
        tids = np.sort(rs.choice(4 * n + 10, n, replace=False)).astype(np.int64)
        for upper in (2, 7):
            obs = rs.randint(0, upper, n)
            for dist, args in (('randint', dict(upper=upper)),
                               ('categorical', dict(upper=upper, p=list(rs.dirichlet(np.ones(upper)))))):
                below = np.sort(rs.permutation(tids)[:min(n, 25)])
                a = parzen.cat_split(dist, args, tids, obs, below, 1.0, 25)
                m = np.isin(tids, below)
                b = parzen.fit_posterior(dist, args, obs[m], obs[~m], 1.0, 25)
                np.testing.assert_array_equal(a.below[0], b.below[0])
                np.testing.assert_array_equal(a.above[0], b.above[0])
                assert a.upper == b.upper and a.family == b.family


def test_split_below_incremental_matches_full():
    """The Trials cache's incremental smallest-loss ranking gives split_below
    the same below set as the full argpartition/argsort path, as documents
    arrive (ties at the boundary fall back to the reference's argsort)."""
    from hyperopt_amd import history as H
    rs = np.random.RandomState(9)
    c = H._Cache(['x'], {'x': False})
    for step in range(60):
        for _ in range(rs.randint(1, 40)):
            c.tids.append(c.tids.n)
            c.losses.append(float(rs.randint(0, 50)) if rs.rand() < 0.3 else rs.uniform())
        hist = H.History(c.tids.view(), c.losses.view(), {}, cache=c)
        plain = H.History(c.tids.view(), c.losses.view(), {})
        for gamma in (0.25, 1.0):
            a = H.split_below(hist, gamma)
            b = H.split_below(plain, gamma)
            assert sorted(a.tolist()) == sorted(b.tolist()), (step, gamma)


def test_lazy_categorical_flag_native_matches_numpy():
    """TPE_F_CAT_LAZY is set by both packers alike: on when the best-scoring
    drawable category has selection probability >= 2^-16, off when it is rarer,
    and ignored by every non-categorical problem."""
    cases = [([0.2, 0.5, 0.3], [0.4, 0.3, 0.3], True),
             ([0.9997, 0.0003], [0.9999999, 1e-7], True),
             ([0.99999, 0.00001], [0.99999999, 1e-8], False),
             ([0.5, 0.0, 0.5], [0.3, 0.4, 0.3], True),
             ([0.25, 0.25, 0.5], [0.25, 0.25, 0.5], True)]
    e = _engine('fp32')
    for pb, pa, lazy in cases:
        post = parzen.Posterior('categorical', N.FAM_CATEGORICAL, None, None, None, (np.array(pb),),
                                (np.array(pa),), len(pb))
        lps = [LevelProblem(post, 4, [0, 1])]
        ref = e._build_numpy(lps, 4096, 3, 10, None)
        info = e._pack(lps, 4096, 3, 10, None)
        prob = _blob(e, info, info.off_problems, N.PROBLEM_DTYPE, info.n_problems)
        np.testing.assert_array_equal(prob['flags'], ref['prob']['flags'])
        assert all(bool(f & N.F_CAT_LAZY) == lazy for f in prob['flags']), (pb, pa)


def test_native_replay_matches_golden_samplers(golden):
    """tpe_replay_mixture / tpe_replay_categorical (native MT19937, legacy
    polar gauss, multinomial by binomial inversion) reproduce the reference's
    own sampler outputs (tests/golden/unit_vectors.json, generated by the
    reference's GMM1/LGMM1/categorical) bit for bit."""
    from hyperopt_amd import replay as R
    for case in golden('unit_vectors.json')['samplers']:
        rng = np.random.RandomState(case['seed'])
        if case['fn'] == 'categorical':
            out = R.draw_categorical(rng, case['p'], case['size'])
        else:
            out = R.draw_mixture(rng, case['w'], case['mu'], case['sigma'], case['low'], case['high'], case['q'],
                                 case['fn'] == 'LGMM1', case['size'])
        np.testing.assert_array_equal(np.ravel(out), np.ravel(np.asarray(case['out'])))


def test_native_replay_continues_randomstate():
    """Native draws equal numpy's RandomState draws on random mixtures
    (bounded/unbounded, log, quantized, zero weights, a pending cached gauss)
    and leave the RandomState exactly where numpy would."""
    from hyperopt_amd import replay as R
    rs = np.random.RandomState(0)
    for t in range(150):
        k = rs.randint(1, 30)
        w = rs.dirichlet(np.ones(k) * rs.choice([0.1, 1.0, 5.0]))
        if k > 1 and rs.rand() < 0.2:
            w[rs.randint(k)] = 0.0
            w /= w.sum()
        mu, sg = rs.uniform(-3, 3, k), rs.uniform(0.05, 2, k)
        low, high = (-2.0, 2.5) if rs.rand() < 0.5 else (None, None)
        q, lg, n = [None, 0.5][rs.randint(2)], rs.rand() < 0.3, rs.randint(0, 300)
        seed = rs.randint(1 << 30)
        a, b = np.random.RandomState(seed), np.random.RandomState(seed)
        a.normal(), b.normal()
        np.testing.assert_array_equal(R.draw_mixture(a, w, mu, sg, low, high, q, lg, n),
                                      R.draw_mixture_numpy(b, w, mu, sg, low, high, q, lg, n))
        assert a.uniform() == b.uniform() and a.normal() == b.normal(), t
        p = rs.dirichlet(np.ones(k))
        np.testing.assert_array_equal(R.draw_categorical(a, p, n), R.draw_categorical_numpy(b, p, n))
        assert a.randint(1 << 30) == b.randint(1 << 30), t
    with pytest.raises(ValueError):                   # numpy's own error for bad weights
        R.draw_mixture(np.random.RandomState(1), [1.5, -0.5], [0.0, 1.0], [1.0, 1.0], None, None, None, False, 3)
