"""The one-call native suggest (tpe_suggest_tree) against the general path.

Both paths fit with the same native routines (tpe_host_fit_split /
tpe_host_cat_split) and run the same level batches, so every suggestion must
be identical: fused (speculative) batches, level-by-level evaluation, the
no-prediction case, batched new_ids, columnar histories without a Trials
cache, and the hand-over to the general path (quantized labels).
"""
import numpy as np
import pytest

from tests.helpers import doc_values

from hyperopt_amd import _native as N

pytestmark = pytest.mark.gpu


def _both(fn):
    from hyperopt_amd import tpe
    from hyperopt_amd.engine import get_engine
    eng = get_engine()
    eng.last_tree_path = None
    nat = fn()
    path = eng.last_tree_path
    tpe.NATIVE_TREE = False
    try:
        gen = fn()
    finally:
        tpe.NATIVE_TREE = True
    return nat, gen, path


def test_native_tree_fused_matches_general_path():
    import bench
    from hyperopt_amd import tpe
    domain, trials = bench.make_history(3000, 0)
    for seed in (1, 2, 3):
        for C in (1 << 16, 1 << 20):
            nat, gen, path = _both(lambda: doc_values(tpe.suggest([3000], domain, trials, seed, n_EI_candidates=C)))
            assert path is not None and path[0] == 1 and path[1] == 1, path     # one fused batch
            assert nat == gen, (seed, C, nat, gen)
            assert set(nat) == {'model', 'svm_C', 'svm_kernel', 'svm_rbf_gamma'}


def test_native_tree_level_by_level_and_no_prediction():
    """SPECULATE off (level by level) and a candidate count too small for a
    gate prediction (C * p < 64 draws): the native level runs equal the
    general path's."""
    import bench
    from hyperopt_amd import tpe
    domain, trials = bench.make_history(3000, 0)
    tpe.SPECULATE = False
    try:
        nat, gen, path = _both(lambda: doc_values(tpe.suggest([3000], domain, trials, 9, n_EI_candidates=1 << 14)))
    finally:
        tpe.SPECULATE = True
    assert path[0] == 0 and path[1] >= 2 and nat == gen, (path, nat, gen)
    nat, gen, path = _both(lambda: doc_values(tpe.suggest([3000], domain, trials, 9, n_EI_candidates=64)))
    assert path[0] == 0 and path[1] >= 2 and nat == gen, (path, nat, gen)


def test_native_tree_batched_ids():
    import bench
    from hyperopt_amd import tpe
    domain, trials = bench.make_history(2000, 1)
    ids = list(range(2000, 2006))
    for spec in (True, False):
        tpe.SPECULATE = spec
        try:
            nat, gen, path = _both(lambda: [doc_values([d]) for d in
                                            tpe.suggest(ids, domain, trials, 4, n_EI_candidates=4096)])
        finally:
            tpe.SPECULATE = True
        assert nat == gen and path is not None, (spec, path)


def test_native_tree_columnar_history():
    """suggest_choices on a structure-of-arrays history (no Trials cache):
    flat 5-dim space, 64 ids."""
    import bench
    from hyperopt_amd import tpe
    labels = ['x%d' % i for i in range(5)]
    hist = bench.soa_history(labels, 4000, 3, lambda v: sum((x - 0.3) ** 2 for x in v.values()))
    table = bench.flat_uniform_table(labels)
    ids = np.arange(4000, 4064)
    nat, gen, path = _both(lambda: tpe.suggest_choices(table, hist, ids, 11, n_EI_candidates=2048))
    assert path == (0, 1) and nat == gen
    # the columnar result (SoA out) holds the same choices, native and general
    for native in (True, False):
        tpe.NATIVE_TREE = native
        try:
            cc = tpe.suggest_choices(table, hist, ids, 11, n_EI_candidates=2048, columns=True)
        finally:
            tpe.NATIVE_TREE = True
        assert cc.labels == table.labels and cc.values.shape == (len(ids), 5) and cc.active.all()
        assert cc.dicts(table) == nat
        assert all(type(v) is np.float64 for v in cc.dicts(table)[0].values())   # (the reference's types)


def test_native_tree_batched_result_types():
    """A batch's per-id dicts and a single id's hold the same value types, the
    reference's np.int64 categories and np.float64 values (None when
    inactive), in level order (tpe.py:812 suggests one id at a time)."""
    import bench
    from hyperopt_amd import tpe
    domain, trials = bench.make_history(2000, 1)
    ids = list(range(2000, 2012))
    nat, gen, path = _both(lambda: tpe.suggest_choices(domain.table, __import__('hyperopt_amd').history.extract(
        domain, trials), ids, 4, n_EI_candidates=4096))
    assert nat == gen and path is not None
    order = domain.table.level_order()
    for d in nat:
        assert list(d) == order
        for r in domain.table.rows:
            v = d[r.label]
            assert v is None or type(v) is (np.int64 if r.categorical else np.float64), (r.label, type(v))
    one = tpe.suggest_choices(domain.table, __import__('hyperopt_amd').history.extract(domain, trials), ids[:1], 4,
                              n_EI_candidates=4096)[0]
    for r in domain.table.rows:
        v = one[r.label]
        assert v is None or type(v) is (np.int64 if r.categorical else np.float64), (r.label, type(v))


def test_native_tree_device_fit_labels():
    """Labels large enough for the device Parzen fit run natively too (below
    sides fitted in C, above sides by tpe_fit_above from the resident value
    orders): a flat 40-dim space over a 20k-trial history and a tree space
    with a log-family label, identical to the general path, twice (the second
    call on the merged orders, then one more observation appended)."""
    import bench
    from hyperopt_amd import base, hp, history as H, tpe
    from hyperopt_amd.engine import get_engine
    eng = get_engine()
    assert eng.device_fit_min <= 20000
    labels = ['x%02d' % i for i in range(40)]
    hist = bench.soa_history(labels, 20000, 5, lambda v: sum((x - 0.3) ** 2 for x in v.values()))
    table = bench.flat_uniform_table(labels)
    for seed in (3, 4):
        nat, gen, path = _both(lambda: tpe.suggest_choices(table, hist, [20000], seed, n_EI_candidates=4096))
        assert path == (0, 1) and nat == gen, seed
    # conditional tree, log-family device label, appended documents (Trials cache)
    space = {'m': hp.choice('m', [{'a': hp.loguniform('a', -3, 2)}, {'b': hp.uniform('b', 0, 1)}]),
             'u': hp.uniform('u', -2, 2)}
    domain = base.Domain(lambda d: 0.0, space)
    trials = base.Trials()
    rs = np.random.RandomState(8)
    docs = []
    for tid in range(36000):
        m = int(rs.uniform() < 0.3)
        vals = {'m': [m], 'a': [] if m else [float(np.exp(rs.uniform(-3, 2)))], 'b': [float(rs.uniform())] if m else [],
                'u': [float(rs.uniform(-2, 2))]}
        idxs = {k: ([tid] if v else []) for k, v in vals.items()}
        d = trials.new_trial_docs([tid], [None], [{'status': 'ok', 'loss': float(rs.uniform()) + 1e-9 * tid}],
                                  [dict(tid=tid, cmd=None, workdir=None, idxs=idxs, vals=vals)])[0]
        d['state'] = base.JOB_STATE_DONE
        docs.append(d)
    trials.insert_trial_docs(docs)
    trials.refresh()
    for step in range(2):
        nid = 36000 + step
        nat, gen, path = _both(lambda: doc_values(tpe.suggest([nid], domain, trials, 40 + step,
                                                              n_EI_candidates=1 << 16)))
        assert path is not None and nat == gen, (step, nat, gen)
        hist = H.extract(domain, trials)
        assert len(hist.obs['a'][0]) >= eng.device_fit_min
        d = tpe.suggest([nid], domain, trials, 50 + step, n_EI_candidates=1024)[0]
        d['state'] = base.JOB_STATE_DONE
        d['result'] = {'status': 'ok', 'loss': 0.01}
        trials.insert_trial_docs([d])
        trials.refresh()


def test_native_tree_takes_caller_fits_of_quantized_labels():
    """The rf branch (quantized rf_n_est / rf_depth_n): tpe_suggest_tree flags
    the quantized labels, the host fits them exactly as the general path does
    (numpy's tie order) and the second call runs the tree natively — same
    suggestion as the general path.  Also the mixed 10-dim space of config 2."""
    import bench
    from hyperopt_amd import base, hp, tpe
    domain, trials = bench.make_history(3000, 0, loss=bench.rf_loss)
    for seed in (5, 6):
        nat, gen, path = _both(lambda: doc_values(tpe.suggest([3000], domain, trials, seed, n_EI_candidates=1 << 16)))
        assert path is not None and nat == gen, (seed, path, nat, gen)
        assert int(nat['model']) == 1
    d2 = base.Domain(lambda d: 0.0, bench.mixed10_space(hp))
    from hyperopt_amd import rand
    t2 = base.Trials()
    rs = np.random.RandomState(0)
    docs = []
    for tid in range(300):
        d = rand.suggest([tid], d2, t2, rs.randint(2 ** 31 - 1))[0]
        v = {k: x[0] for k, x in d['misc']['vals'].items() if x}
        d['state'] = base.JOB_STATE_DONE
        d['result'] = {'status': 'ok', 'loss': sum((float(x) - 0.3) ** 2 for x in v.values()) + 1e-9 * tid}
        docs.append(d)
    t2.insert_trial_docs(docs)
    t2.refresh()
    nat, gen, path = _both(lambda: doc_values(tpe.suggest([300], d2, t2, 3, n_EI_candidates=10000)))
    assert path is not None and nat == gen, (nat, gen)


def test_native_tree_stale_fit_hint():
    """The labels a call had to fit on the host are fitted up front by the next
    call on the same space (ParamTable.native_fit_hint).  A branch switch leaves
    the hint naming labels the new branch does not use: still the general path's
    suggestion, both ways, and the hint follows the branch."""
    import bench
    from hyperopt_amd import tpe
    domain, rf_trials = bench.make_history(3000, 0, loss=bench.rf_loss)
    _, svm_trials = bench.make_history(3000, 0)
    table = domain.table
    for trials, model, seed in ((rf_trials, 1, 11), (svm_trials, 0, 12), (rf_trials, 1, 13), (rf_trials, 1, 14)):
        nat, gen, path = _both(lambda: doc_values(tpe.suggest([3000], domain, trials, seed, n_EI_candidates=1 << 16)))
        assert path is not None and nat == gen, (seed, path, nat, gen)
        assert int(nat['model']) == model
        named = {table.rows[ix].label for ix in getattr(table, 'native_fit_hint', ())}
        assert named <= {'rf_n_est', 'rf_depth_n', 'svm_poly_degree', 'knn_k'}, named
        if model == 1:
            assert 'rf_n_est' in named, named
        else:
            assert not named & {'rf_n_est', 'rf_depth_n'}, named


def test_engine_stream_follows_torch():
    """Engine._stream (the raw current-stream accessor) is torch's current
    stream, also inside a torch.cuda.stream context."""
    import torch
    from hyperopt_amd.engine import get_engine
    eng = get_engine()
    assert eng._stream() == torch.cuda.current_stream(eng.device).cuda_stream
    s = torch.cuda.Stream(device=eng.device)
    with torch.cuda.stream(s):
        assert eng._stream() == s.cuda_stream
    assert eng._stream() == torch.cuda.current_stream(eng.device).cuda_stream


def test_expanded_level_matches_host_written_level(monkeypatch):
    """An expanded level (>= 256 problems, every label tabulated: the device
    writes the problems and tiles from one template per label, k_expand) gives
    exactly the suggestions of the same level with every problem and tile
    written by the host (TPE_EXPAND=0), for ids that do not start at 0 and a
    candidate count that leaves the last tile partial."""
    import bench
    from hyperopt_amd import tpe
    labels = ['x%02d' % i for i in range(6)]
    hist = bench.soa_history(labels, 3000, bench.SEED, lambda v: sum((x - 0.3) ** 2 for x in v.values()))
    table = bench.flat_uniform_table(labels)
    ids = np.arange(7000, 7000 + 300)
    C = 3000
    outs = []
    for env in ('1', '0'):
        monkeypatch.setenv('TPE_EXPAND', env)
        cc = tpe.suggest_choices(table, hist, ids, 21, n_EI_candidates=C, columns=True)
        outs.append(np.asarray(cc.values))
    assert outs[0].shape == (len(ids), len(labels))
    assert np.array_equal(outs[0], outs[1])
    assert np.all(np.isfinite(outs[0])) and np.all(outs[0] >= -5) and np.all(outs[0] < 5)


def test_repeated_values_label_crossing_device_fit_min():
    """A continuous label with repeated values (its host fits need numpy's tie
    order: the native call flags it, the next call gets the caller's fit up
    front) whose history grows across device_fit_min, through the window
    n_obs in [device_fit_min, device_fit_min + n_below) where both paths must
    agree on the device fit: every suggest equals the general path's, and the
    label's resident value order is np.argsort(kind='stable') of its values
    after every suggest that used it."""
    from hyperopt_amd import base, devhist, hp, history as H, tpe
    from hyperopt_amd.engine import get_engine
    eng = get_engine()
    old = eng.device_fit_min
    dmin = 2000
    table = base.Domain(lambda d: 0.0, {'u': hp.uniform('u', -5, 5), 'v': hp.uniform('v', 0, 1)}).table
    rs = np.random.RandomState(21)
    Nt = dmin + 60
    vals = {'u': np.round(rs.uniform(-5, 5, Nt), 2), 'v': rs.uniform(0, 1, Nt)}
    tids = np.arange(Nt, dtype=np.int64)
    losses = rs.uniform(size=Nt) + 1e-9 * tids
    dev = {}
    try:
        eng.device_fit_min = dmin
        for n in (dmin - 20, dmin - 10, dmin + 2, dmin + 6, dmin + 30, dmin + 60):
            hist = H.History(tids[:n], losses[:n].copy(), {k: (tids[:n], v[:n]) for k, v in vals.items()}, dev=dev)
            nb = len(H.split_below(hist, 0.25))
            got = tpe.suggest_choices(table, hist, [n], 100 + n, n_EI_candidates=4096)[0]
            fresh = H.History(tids[:n], losses[:n].copy(), {k: (tids[:n], v[:n]) for k, v in vals.items()}, dev={})
            tpe.NATIVE_TREE = False
            try:
                want = tpe.suggest_choices(table, fresh, [n], 100 + n, n_EI_candidates=4096)[0]
            finally:
                tpe.NATIVE_TREE = True
            assert got == want, (n, got, want)
            if tpe.device_fits(n, nb, dmin):
                dc = devhist.columns(hist, eng.device)
                for label in ('u', 'v'):
                    o = dc.order(label)        # (delta mode: the last merged prefix)
                    assert 0 < o.n <= n and n - o.n <= N.FIT_DELTA_MAX, (label, n, o.n)
                    keys, idx = o.host()
                    w = np.argsort(vals[label][:o.n], kind='stable')
                    np.testing.assert_array_equal(idx, w, err_msg='%s n=%d' % (label, n))
                    np.testing.assert_array_equal(keys, vals[label][:o.n][w], err_msg='%s n=%d' % (label, n))
    finally:
        eng.device_fit_min = old


def test_quantized_labels_one_native_call():
    """Quantized labels (the rf branch, and config 2's mixed space) are fitted
    inside tpe_suggest_tree from numpy's argsort of each side (the reference's
    tie order, tpe.py:427-428) that the host passes in: after the first
    suggest on a space, every suggest is ONE native call, and equal to the
    general path's suggestion."""
    import bench
    from hyperopt_amd import tpe
    from hyperopt_amd.engine import get_engine
    eng = get_engine()
    domain, trials = bench.make_history(3000, 0, loss=bench.rf_loss)
    tpe.suggest([3000], domain, trials, 1, n_EI_candidates=1 << 16)
    for seed in (7, 8, 9):
        c0 = eng.tree_calls
        nat = doc_values(tpe.suggest([3000], domain, trials, seed, n_EI_candidates=1 << 16))
        assert eng.tree_calls - c0 == 1, seed
        tpe.NATIVE_TREE = False
        try:
            gen = doc_values(tpe.suggest([3000], domain, trials, seed, n_EI_candidates=1 << 16))
        finally:
            tpe.NATIVE_TREE = True
        assert nat == gen and int(nat['model']) == 1, (seed, nat, gen)
    domain, trials = bench.mixed10_history(1000, 3)
    tpe.suggest([1000], domain, trials, 1, n_EI_candidates=10000)
    for seed in (4, 5):
        c0 = eng.tree_calls
        nat = doc_values(tpe.suggest([1000], domain, trials, seed, n_EI_candidates=10000))
        assert eng.tree_calls - c0 == 1, seed
        tpe.NATIVE_TREE = False
        try:
            gen = doc_values(tpe.suggest([1000], domain, trials, seed, n_EI_candidates=10000))
        finally:
            tpe.NATIVE_TREE = True
        assert nat == gen, (seed, nat, gen)


@pytest.mark.parametrize('extra', [0, 16])
def test_fast_sample_kernel_matches_general(monkeypatch, extra):
    """The sample stage's specialised kernel (tpe_batch.tab_fast: cells tables
    in LDS, staging overlapped with the first draws) chooses exactly what the
    general kernel chooses — the same draws, look-ups and run reduction — on
    the config-3 tree (one id, 2^20 candidates: dynamic pair hand-out), a
    batched 20-dim level (expanded, one pair per problem) and a tiny C (single
    tiles); ``extra`` = TPE_BATCH_TAB_EXACT: every candidate through the exact
    fallback."""
    import bench
    from hyperopt_amd import tpe
    domain, trials = bench.make_history(3000, 0)
    labels = ['x%02d' % i for i in range(20)]
    hist = bench.soa_history(labels, 3000, 5, lambda v: sum((x - 0.3) ** 2 for x in v.values()))
    table = bench.flat_uniform_table(labels)

    def run():
        out = [doc_values(tpe.suggest([3000], domain, trials, s, n_EI_candidates=1 << 20)) for s in (3, 4)]
        cc = tpe.suggest_choices(table, hist, np.arange(3000, 3300), 6, n_EI_candidates=4096, columns=True)
        out.append(cc.values.tolist())
        out.append(doc_values(tpe.suggest([3000], domain, trials, 7, n_EI_candidates=2048)))
        return out
    monkeypatch.setenv('TPE_DEBUG_FLAGS', str(extra))
    fast = run()
    monkeypatch.setenv('TPE_DEBUG_FLAGS', str(extra | N.BATCH_NO_FAST2))     # k_sample_tab's 1024-thread FAST pass
    fast1024 = run()
    monkeypatch.setenv('TPE_DEBUG_FLAGS', str(extra | N.BATCH_NO_TAB_FAST))
    gen = run()
    assert fast == gen
    assert fast1024 == gen


def test_fast_sample_kernel_single_label_partial_staging_round(monkeypatch):
    """A level of ONE tabulated label — its table is the level's largest, so the
    dynamic LDS holds exactly its 3 * n0 row units, and 3 * n0 is (for these
    histories) not a multiple of the 512-lane staging round: the LDS-DMA lanes
    past the rows must issue nothing.  Several history sizes
    (different cell counts); k_sample_fast chooses exactly what the general
    kernel chooses, so neither the staged rows nor the static LDS after them
    (guide, run records) were overwritten."""
    import bench
    from hyperopt_amd import tpe
    table = bench.flat_uniform_table(['x'])
    hists = [bench.soa_history(['x'], n, 11 + n, lambda v: (v['x'] - 0.3) ** 2) for n in (40, 160, 700, 2500)]

    def run():
        return [tpe.suggest_choices(table, h, np.arange(len(h.losses), len(h.losses) + 3), 9,
                                    n_EI_candidates=1 << 18, columns=True).values.tolist() for h in hists]
    monkeypatch.setenv('TPE_DEBUG_FLAGS', '0')
    fast = run()
    monkeypatch.setenv('TPE_DEBUG_FLAGS', str(N.BATCH_NO_TAB_FAST))
    gen = run()
    assert fast == gen


@pytest.fixture(scope='module')
def quantized_workloads():
    """The rf-steered config-3 history (quantized rf_n_est / rf_depth_n labels,
    lattices) and config 2's 10-dim mixed space (cells and lattices in one
    level), smaller histories."""
    import bench
    qdom, qtr = bench.make_history(3000, 1, loss=bench.rf_loss)
    mdom, mtr = bench.mixed10_history(1000, 2)
    return qdom, qtr, mdom, mtr


def test_fast_sample_kernel_lattices_match_general(monkeypatch, quantized_workloads):
    """k_sample_fast's lattice path (ABI 20: quantised by the table's entry
    thresholds, argmax by score rank) chooses exactly what the general kernel
    chooses (np.round(x / q) per candidate, f64 score order) on the rf branch
    at 2^20 candidates and on config 2's mixed level (10^4 candidates) —
    several seeds, the fast path confirmed by the profiler's kernel timing."""
    from hyperopt_amd import tpe
    from hyperopt_amd.engine import get_engine
    qdom, qtr, mdom, mtr = quantized_workloads

    def run():
        out = [doc_values(tpe.suggest([3000], qdom, qtr, s, n_EI_candidates=1 << 20)) for s in (3, 4, 5)]
        out += [doc_values(tpe.suggest([1000], mdom, mtr, s, n_EI_candidates=10000)) for s in (6, 7, 8)]
        return [{k: float(v) for k, v in d.items()} for d in out]
    monkeypatch.setenv('TPE_DEBUG_FLAGS', '0')
    fast = run()
    eng = get_engine()
    eng.lib.tpe_level_profile(1)
    try:
        tpe.suggest([3000], qdom, qtr, 3, n_EI_candidates=1 << 20)
        prof = (N.StageProf * len(N.STAGES))()
        N.check(eng.lib.tpe_level_profile_read(prof, len(N.STAGES)), eng.lib, 'profile')
        assert prof[N.STAGES.index('k_sample')].kernel_ns > 0      # (the specialised pass ran)
    finally:
        eng.lib.tpe_level_profile(0)
    monkeypatch.setenv('TPE_DEBUG_FLAGS', '32')                    # TPE_BATCH_NO_TAB_FAST: the general kernel
    gen = run()
    assert fast == gen
    assert any(int(d.get('model', -1)) == 1 for d in fast[:3])     # (the rf branch was suggested)


@pytest.mark.parametrize('branch', ['svm', 'rf'])
def test_fast_sample_kernel_lg_against_oracle(branch):
    """tpe_debug_fast_lg: k_sample_fast itself writes every candidate's value,
    l and g; on the headline (config 3, 10k trials, 2^20 candidates; svm
    branch: log-polynomial cells, rf branch: lattices) 3000 of each label's
    are checked against the oracle's lpdf of the oracle's own fits of the
    history (ap_filter_trials + adaptive_parzen_normal: nothing of this
    build's fits; 1e-5 relative, lattices 1e-9), and the suggested value is the
    argmax of l - g over the label's candidates (within the eps-tie set)."""
    import torch
    import bench
    from hyperopt_amd import history as H, tpe
    from hyperopt_amd.engine import get_engine
    from oracle import tpe_oracle as O
    eng = get_engine()
    domain, trials = bench.make_history(10000, bench.SEED, loss=None if branch == 'svm' else bench.rf_loss)
    T = domain.table
    C = 1 << 20
    buf = torch.full((4 * 8 * C,), float('nan'), dtype=torch.float64, device=eng.device)
    N.check(eng.lib.tpe_debug_fast_lg(buf.data_ptr(), 8 * C), eng.lib, 'tpe_debug_fast_lg')
    try:
        doc = tpe.suggest([10000], domain, trials, 77, n_EI_candidates=C)[0]
        torch.cuda.synchronize()
    finally:
        N.check(eng.lib.tpe_debug_fast_lg(None, 0), eng.lib, 'tpe_debug_fast_lg')
    rec = buf.cpu().numpy().reshape(-1, 4)
    rec = rec[np.isfinite(rec[:, 3])]
    hist = H.extract(domain, trials)
    chosen = {k: v[0] for k, v in doc['misc']['vals'].items() if v}
    rs = np.random.RandomState(5)
    seen = 0
    for r in T.rows:
        mine = rec[rec[:, 3] == r.index]
        if not len(mine) or r.categorical or r.label not in chosen:
            continue
        assert len(mine) == C, r.label
        q = r.args.get('q')
        otids, ovals = hist.obs[r.label]
        below, above = O.ap_filter_trials(otids, ovals, hist.tids, hist.losses, 0.25)
        pb, pa = (O.fit_posterior(r.dist, dict(r.args), o, 1.0) for o in (below, above))
        tol = 1e-9 if q else 1e-5
        sub = rs.choice(len(mine), 3000, replace=False)
        x = mine[sub, 0]
        for col, post in ((1, pb), (2, pa)):
            ref = post.lpdf(x)
            got = mine[sub, col]
            fin = np.isfinite(ref)
            err = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1.0)
            assert err.max() <= tol, (r.label, col, float(err.max()))
        score = mine[:, 1] - mine[:, 2]
        m = np.nanmax(score)
        eps = 4 * tol * max(1.0, float(np.nanmax(np.abs(mine[:, 1:3]))))
        ties = np.nonzero(score >= m - eps)[0]
        assert float(chosen[r.label]) in set(mine[ties, 0].tolist()), r.label
        seen += 1
    assert seen >= (2 if branch == 'svm' else 1), seen
