"""C-ABI checks that need no GPU: the library loads, exports every function
include/tpe_hip.h declares, and the Python mirrors of the C structs have the
C compiler's layout (sizes and field offsets)."""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from hyperopt_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'tpe_hip.h')


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return re.findall(r'^\s*(?:const\s+)?\w+\s*\*?\s*(tpe_\w+)\s*\(', src, flags=re.M)


def test_header_declares_bindings():
    assert set(declared_functions()) == set(N.EXPORTS)


def test_library_exports_every_symbol():
    lib = N.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.tpe_abi_version() == N.ABI_VERSION
    assert lib.tpe_tile_size() == 2048
    n = ctypes.c_int(-1)
    rc = lib.tpe_device_count(ctypes.byref(n))
    assert rc in (0, -3) and n.value >= 0


def test_null_batch_is_rejected_without_gpu():
    lib = N.load()
    assert lib.tpe_run_batch(None, None) == -1
    assert b'null batch' in lib.tpe_last_error()
    b = N.Batch()
    b.n_problems = -1
    assert lib.tpe_run_batch(ctypes.byref(b), None) == -1


def _c_layout():
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "tpe_hip.h"
#define F(T, f) printf("%s.%s %zu\n", #T, #f, offsetof(T, f));
int main(void) {
  printf("tpe_problem %zu\ntpe_tile %zu\ntpe_work %zu\ntpe_best %zu\ntpe_result %zu\ntpe_batch %zu\n",
         sizeof(tpe_problem), sizeof(tpe_tile), sizeof(tpe_work), sizeof(tpe_best), sizeof(tpe_result),
         sizeof(tpe_batch));
  F(tpe_problem, cand_off) F(tpe_problem, sort_slot) F(tpe_problem, n_splits) F(tpe_problem, above_len)
  F(tpe_problem, low) F(tpe_problem, above_base) F(tpe_problem, key0) F(tpe_problem, ctr3)
  F(tpe_batch, comp32) F(tpe_batch, tiles) F(tpe_batch, n_tiles) F(tpe_batch, work) F(tpe_batch, n_work_qlog)
  F(tpe_batch, part) F(tpe_batch, result)
  F(tpe_result, value) F(tpe_result, global_idx)
  return 0;
}
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, 'l.c')
        open(c, 'w').write(prog)
        exe = os.path.join(d, 'l')
        subprocess.check_call(['gcc', '-I', os.path.dirname(HEADER), c, '-o', exe])
        out = subprocess.check_output([exe]).decode()
    return dict((line.split()[0], int(line.split()[1])) for line in out.strip().splitlines())


def test_struct_layout_matches_c():
    lay = _c_layout()
    assert lay['tpe_problem'] == N.PROBLEM_DTYPE.itemsize
    assert lay['tpe_tile'] == N.TILE_DTYPE.itemsize
    assert lay['tpe_work'] == N.WORK_DTYPE.itemsize
    assert lay['tpe_best'] == N.BEST_DTYPE.itemsize
    assert lay['tpe_result'] == N.RESULT_DTYPE.itemsize
    assert lay['tpe_batch'] == ctypes.sizeof(N.Batch)
    for key, off in lay.items():
        if '.' not in key:
            continue
        st, f = key.split('.')
        if st == 'tpe_problem':
            assert N.PROBLEM_DTYPE.fields[f][1] == off, key
        elif st == 'tpe_result':
            assert N.RESULT_DTYPE.fields[f][1] == off, key
        elif st == 'tpe_batch':
            assert getattr(N.Batch, f).offset == off, key


def test_engine_refuses_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip('a GPU is visible')
    from hyperopt_amd.engine import Engine
    with pytest.raises(N.NativeUnavailable):
        Engine()


CTYPES_MIRRORS = (('tpe_batch', N.Batch), ('tpe_label_in', N.LabelIn), ('tpe_pack_info', N.PackInfo),
                  ('tpe_level_ws', N.LevelWS), ('tpe_level_need', N.LevelNeed), ('tpe_mt_state', N.MTState),
                  ('tpe_stage_prof', N.StageProf), ('tpe_tree_label', N.TreeLabel), ('tpe_exchange', N.Exchange))


def test_ctypes_mirrors_match_c():
    """Every field offset and the size of each ctypes mirror equal gcc's."""
    lines = []
    for cname, cls in CTYPES_MIRRORS:
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in cls._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    prog = '#include <stdio.h>\n#include <stddef.h>\n#include "tpe_hip.h"\nint main(void) {\n%s\nreturn 0; }\n' % (
        '\n'.join(lines))
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, 'm.c')
        open(c, 'w').write(prog)
        exe = os.path.join(d, 'm')
        subprocess.check_call(['gcc', '-I', os.path.dirname(HEADER), c, '-o', exe])
        out = subprocess.check_output([exe]).decode()
    lay = dict((line.split()[0], int(line.split()[1])) for line in out.strip().splitlines())
    for cname, cls in CTYPES_MIRRORS:
        assert lay[cname] == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert getattr(cls, f).offset == lay[cname + '.' + f], (cname, f)


def test_level_run_reports_space_without_gpu(monkeypatch):
    """tpe_level_run sizes a level before touching the device: with empty
    workspaces it returns TPE_E_SPACE and the needs of a 2^20-candidate level
    (an unpruned one: the sort workspace query needs a device) — tabulated
    (score tables, no above-mixture partial sums) and, with TPE_TABLES=0,
    per candidate."""
    from hyperopt_amd import parzen
    from hyperopt_amd.engine import Engine, LevelProblem
    rs = np.random.RandomState(0)
    post = parzen.fit_posterior('uniform', dict(low=-5.0, high=5.0), rs.uniform(-5, 5, 10),
                                rs.uniform(-5, 5, 50), 1.0)
    labels, keep = Engine._labels([LevelProblem(post, 0, [7, 8])])
    ws, need = N.LevelWS(), N.LevelNeed()
    lib = N.load()
    out = np.empty(2, dtype=N.RESULT_DTYPE)
    rc = lib.tpe_level_run(labels, 1, 1 << 20, 5, 0, 0, N.PREC_F32, 0, ctypes.byref(ws), ctypes.byref(need), None,
                           out.ctypes.data)
    assert rc == N.E_SPACE
    assert need.cand == 2 << 20 and need.result == 2 and need.best == 2 * 512 * N.BEST_PER_TILE
    assert need.blob_bytes > 0 and need.pinned_bytes >= need.blob_bytes + 2 * 48
    # 50 above components over [-5, 5): cells of the narrowest bandwidth's scale, both sides
    assert need.part == 0 and need.tab > 0 and need.tab % N.TAB_ROW_UNITS == 0
    monkeypatch.setenv('TPE_TABLES', '0')
    rc = lib.tpe_level_run(labels, 1, 1 << 20, 5, 0, 0, N.PREC_F32, 0, ctypes.byref(ws), ctypes.byref(need), None,
                           out.ctypes.data)
    assert rc == N.E_SPACE and need.tab == 0 and need.part >= 2 << 20


def test_tree_labels_dtype_matches_ctypes():
    assert N.TREE_LABEL_DTYPE.itemsize == ctypes.sizeof(N.TreeLabel)
    for f, _ in N.TreeLabel._fields_:
        assert N.TREE_LABEL_DTYPE.fields[f][1] == getattr(N.TreeLabel, f).offset, f


def _tree_call(table, hist, C, min_draws=64.0, flags=0, shard=None, ex=None, fit_min=16384, engine=None):
    from hyperopt_amd import history as H, tpe
    arr, keep = tpe._tree_labels(table, hist, engine)[:2]
    below = np.sort(H.split_below(hist, 0.25)).astype(np.int64)
    ws, need = N.LevelWS(), N.LevelNeed()
    vals = np.empty((1, len(arr)))
    act = np.empty((1, len(arr)), dtype=np.int8)
    path = (ctypes.c_int32 * 2)()
    need_fit = np.zeros(len(arr), dtype=np.int8)
    ids = np.array([len(hist)], dtype=np.int64)
    c_loc, base, c_glob = C, 0, 0
    if shard is not None:
        from hyperopt_amd.dist import shard_range
        base, hi = shard_range(C, *shard)
        c_loc, c_glob = hi - base, C
    rc = N.load().tpe_suggest_tree(arr.ctypes.data, len(arr), below.ctypes.data, len(below), 1.0, 25, ids.ctypes.data,
                                   1, c_loc, base, c_glob, ex, 5, min_draws, fit_min, flags, ctypes.byref(ws),
                                   ctypes.byref(need), None, vals.ctypes.data, act.ctypes.data, path,
                                   need_fit.ctypes.data)
    return rc, need, path, need_fit


def test_suggest_tree_fits_and_predicts_without_gpu():
    """tpe_suggest_tree on the config-3 tree: native fits and the gate
    prediction run on the host and size the fused batch before any device
    call (empty workspaces -> TPE_E_SPACE): one problem per label the Python
    prediction (tpe._predict_activity) keeps active; level by level, the
    first level's single problem."""
    import bench
    from hyperopt_amd import history as H, tpe
    domain, trials = bench.make_history(3000, 0)
    hist = H.extract(domain, trials)
    C = 1 << 16
    rc, need, path, _ = _tree_call(domain.table, hist, C)
    assert rc == N.E_SPACE and path[1] == 1, rc
    fits = tpe._Fits(domain.table, hist, H.split_below(hist, 0.25), 1.0, None)
    pred = tpe._predict_activity(domain.table, fits, C)
    n_act = sum(v is not None for v in pred.values())
    assert need.result == n_act == 4 and need.cand == n_act * C
    rc, need, path, _ = _tree_call(domain.table, hist, C, flags=N.TREE_NO_SPECULATE)
    assert rc == N.E_SPACE and need.result == 1 and need.cand == C


def test_suggest_tree_hands_quantized_labels_back():
    """A root quantized label needs numpy's tie order: TPE_E_FALLBACK before
    anything is sized or launched, the label flagged for the caller's fit; with
    that fit in its record the call proceeds to sizing the level."""
    from hyperopt_amd import base, hp, history as H, rand
    domain = base.Domain(lambda d: 0.0, {'q': hp.quniform('q', 0, 10, 1), 'x': hp.uniform('x', -1, 1)})
    trials = base.Trials()
    rs = np.random.RandomState(0)
    for tid in range(40):
        d = rand.suggest([tid], domain, trials, rs.randint(2 ** 31 - 1))[0]
        d['state'] = base.JOB_STATE_DONE
        d['result'] = {'status': 'ok', 'loss': float(rs.uniform())}
        trials.insert_trial_docs([d])
    trials.refresh()
    hist = H.extract(domain, trials)
    rc, need, path, need_fit = _tree_call(domain.table, hist, 1024)
    assert rc == N.E_FALLBACK and path[1] == 0
    q = domain.table.by_label['q'].index
    assert need_fit.tolist() == [1 if i == q else 0 for i in range(len(need_fit))]
    from hyperopt_amd import tpe
    fits = tpe._Fits(domain.table, hist, H.split_below(hist, 0.25), 1.0, None)
    post = fits.get(domain.table.by_label['q'])
    arr, keep = tpe._tree_labels(domain.table, hist)[:2]
    arr = arr.copy()
    cols = [[np.ascontiguousarray(c) for c in side] for side in (post.below, post.above)]
    for sd in range(2):
        arr[q]['host_k'][sd] = len(cols[sd][0])
        arr[q]['host_w'][sd], arr[q]['host_mu'][sd], arr[q]['host_sigma'][sd] = [c.ctypes.data for c in cols[sd]]
    orig = tpe._tree_labels
    tpe._tree_labels = lambda t, h, e=None: (arr, keep, None)
    try:
        rc, need, path, need_fit = _tree_call(domain.table, hist, 1024)
    finally:
        tpe._tree_labels = orig
    assert rc == N.E_SPACE and not need_fit.any() and need.result == 2


def test_suggest_tree_refuses_device_fit_sizes_up_front():
    """A continuous label large enough for the device Parzen fit sends the
    space to the general path before any fit or level run (no level issued,
    no label flagged for the caller)."""
    import bench
    from hyperopt_amd import history as H
    domain, trials = bench.make_history(3000, 0)
    hist = H.extract(domain, trials)
    n_max = max(len(hist.obs[r.label][0]) for r in domain.table.rows
                if r.dist in ('uniform', 'loguniform', 'normal', 'lognormal'))
    rc, need, path, need_fit = _tree_call(domain.table, hist, 1 << 16, fit_min=n_max)
    assert rc == N.E_FALLBACK and path[1] == 0 and not need_fit.any()


def test_combine_results_native_matches_numpy():
    """tpe_combine_results (the native exchange's reduction) == dist.combine_results
    (np.argmax over (score, global index), empty records skipped)."""
    from hyperopt_amd.dist import combine_results
    lib = N.load()
    rs = np.random.RandomState(4)
    for trial in range(300):
        world, P = rs.randint(1, 6), rs.randint(1, 7)
        st = np.zeros((world, P), dtype=N.RESULT_DTYPE)
        st['score'] = rs.choice([0.0, 1.0, 2.0, np.nan, -np.inf, np.inf], size=(world, P))
        st['global_idx'] = rs.permutation(world * P * 3)[:world * P].reshape(world, P)
        st['idx'] = np.where(rs.uniform(size=(world, P)) < 0.15, -1, st['global_idx'])
        st['value'] = rs.uniform(size=(world, P))
        out = np.empty(P, dtype=N.RESULT_DTYPE)
        assert lib.tpe_combine_results(st.ctypes.data, world, P, out.ctypes.data) == 0
        ref = combine_results(st)
        np.testing.assert_array_equal(out['global_idx'], ref['global_idx'])
        np.testing.assert_array_equal(out['value'], ref['value'])


def _exchange_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import bench
        from hyperopt_amd import dist as D, history as H

        class _Eng(object):                 # what _Exchange needs of an Engine (host gather: no device)
            lib = N.load()
            _dev_index = 0
        ex = D._Exchange(_Eng(), None)
        domain, trials = bench.make_history(600, 0)
        hist = H.extract(domain, trials)
        # empty workspaces: every rank's first level run needs more room; the
        # ranks still exchange (statuses, empty records) and all return E_SPACE
        rc, need, path, _ = _tree_call(domain.table, hist, 1 << 16, shard=(rank, world), ex=ex.ptr(32))
        q.put((rank, rc, int(path[1]), int(need.cand), None))
    except Exception as e:
        q.put((rank, None, None, None, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_tree_exchanges_status_without_gpu():
    """Two gloo ranks run tpe_suggest_tree sharded (each half of the 2^16
    candidates): the native call issues the exchange through the host gather
    callback after its first level run and both ranks return TPE_E_SPACE in
    lock-step, each sized for its own half."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, rc, levels, cand, err in got:
        assert err is None, err
        assert rc == N.E_SPACE and levels == 1 and cand == 4 * (1 << 15), (rank, rc, levels, cand)


def test_suggest_tree_sizes_device_fits_without_gpu():
    """A flat continuous space whose labels are large enough for the device
    Parzen fit runs natively: tpe_suggest_tree fits every below side on the
    host (<= 25 observations) and sizes the device fits (columns and resident
    value orders in the records; host tensors stand in for device ones — the
    call stops before touching them)."""
    import bench
    import torch
    from hyperopt_amd import devhist, tpe

    class _Eng(object):
        precision, device_fit_min, device = 'fp32', 100, torch.device('cpu')
    labels = ['x%d' % i for i in range(3)]
    hist = bench.soa_history(labels, 400, 1, lambda v: sum((x - 0.3) ** 2 for x in v.values()))
    table = bench.flat_uniform_table(labels)
    arr, keep, devs = tpe._tree_labels(table, hist, _Eng())[:3]
    ixs, slots, ns, group = devs
    assert sorted(ixs.tolist()) == [0, 1, 2] and ns.tolist() == [400] * 3
    assert np.all(arr['dev_obs'] != 0) and np.all(arr['n_ord_in'] == 0) and np.all(arr['ord_key_out'] != 0)
    # one flat column store: the labels' columns are its segments, holding the values
    dc = devhist.columns(hist, torch.device('cpu'))
    for k, label in enumerate(labels):
        seg = dc.view(label)
        assert int(arr[table.by_label[label].index]['dev_obs']) == seg.data_ptr()
        np.testing.assert_array_equal(seg[:400].numpy(), hist.obs[label][1])
    rc, need, path, need_fit = _tree_call(table, hist, 4096, fit_min=100, engine=_Eng())
    # (pruned above mixtures: without a device the sort-workspace query that
    # follows the sizing fails instead of returning TPE_E_SPACE)
    assert rc in (N.E_SPACE, N.E_HIP) and path[1] == 1 and not need_fit.any(), rc
    assert need.result == 3 and need.fit >= 3 * 400          # every label's fit scratch (all observations new)
    # the memo: the same records while nothing moved; a committed order moves them
    assert tpe._tree_labels(table, hist, _Eng())[0] is arr
    group.commit_many(slots[ixs == 0], ns[ixs == 0])
    arr2 = tpe._tree_labels(table, hist, _Eng())[0]
    assert arr2 is not arr and arr2[0]['n_ord_in'] == 400 and arr2[0]['ord_key_out'] == 0
    assert devhist.columns(hist, torch.device('cpu')).order('x0').n == 400


def test_tree_labels_dense_history_matches_dict_history():
    """A dense history (history.DenseObs: every label a row of one matrix) gives
    the same tree records as the same columns passed as a dict — device
    columns, resident-order pointers and host addresses alike — appended to
    step by step (FMinIter's one observation per label)."""
    import bench
    import torch
    from hyperopt_amd import tpe
    from hyperopt_amd.history import DenseLayout, DenseObs, History

    class _Eng(object):
        precision, device_fit_min, device = 'fp32', 100, torch.device('cpu')
    labels = ['x%d' % i for i in range(5)]
    table = bench.flat_uniform_table(labels)
    rs = np.random.RandomState(2)
    cap, N0 = 500, 300
    m = np.ascontiguousarray(rs.uniform(-5, 5, (len(labels), cap)))
    tids = np.arange(cap, dtype=np.int64)
    losses = rs.uniform(size=cap)
    layout = DenseLayout(labels)
    dev_a, dev_b = {}, {}
    prev = None
    for n in (N0, N0 + 1, N0 + 2, N0 + 40):
        ha = History(tids[:n], losses[:n], DenseObs(layout, m, tids[:n]), dev=dev_a)
        hb = History(tids[:n], losses[:n], {k: (tids[:n], m[i, :n]) for i, k in enumerate(labels)}, dev=dev_b)
        ta, tb = tpe._tree_labels(table, ha, _Eng()), tpe._tree_labels(table, hb, _Eng())
        ra, rb = ta[0], tb[0]
        # (the dense views share one device state: their records are reused, rewritten)
        assert prev is None or ra is prev
        prev = ra
        for f in ('n_obs', 'tids', 'values', 'order', 'n_ord_in'):
            np.testing.assert_array_equal(ra[f], rb[f], err_msg='%s n=%d' % (f, n))
        for f in ('dev_obs', 'ord_key_in', 'ord_key_out'):
            np.testing.assert_array_equal(ra[f] != 0, rb[f] != 0, err_msg=f)
        ca, cb = dev_a['cpu'], dev_b['cpu']
        for k in labels:
            np.testing.assert_array_equal(ca.view(k)[:n].numpy(), cb.view(k)[:n].numpy())
            assert ca.count(k) == cb.count(k) == n
        for t in (ta, tb):
            ixs, slots, ns, g = t[2]
            g.commit_many(slots, ns)
