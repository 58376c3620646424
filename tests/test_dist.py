"""Multi-rank combine step on CPU: np.argmax semantics of the cross-shard
winner, and a world_size-2 gloo all-gather (the RCCL path is the same call)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from hyperopt_amd import _native as N
from hyperopt_amd.dist import combine_results, shard_range


def _res(rows):
    out = np.zeros(len(rows), dtype=N.RESULT_DTYPE)
    for i, (score, gidx, value) in enumerate(rows):
        out[i]['score'], out[i]['global_idx'], out[i]['value'] = score, gidx, value
        out[i]['idx'] = -1 if gidx < 0 else gidx
    return out


def test_shard_range_partitions():
    for n in (0, 1, 7, 1 << 20):
        for w in (1, 2, 3, 8):
            r = [shard_range(n, k, w) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))


def test_combine_matches_np_argmax():
    rs = np.random.RandomState(0)
    for trial in range(200):
        world, per = rs.randint(1, 6), rs.randint(1, 9)
        scores = rs.choice([0.0, 1.0, 2.0, np.nan, -np.inf], size=world * per,
                           p=[.3, .3, .3, .05, .05]) if trial % 2 else rs.uniform(size=world * per)
        ref = int(np.argmax(scores))
        parts = []
        for r in range(world):
            seg = scores[r * per:(r + 1) * per]
            i = int(np.argmax(seg))
            parts.append(_res([(seg[i], r * per + i, float(r * per + i))]))
        got = combine_results(np.stack(parts))[0]
        assert got['global_idx'] == ref, (scores, got)


def test_combine_skips_empty_shards():
    parts = np.stack([_res([(0.0, -1, 0.0)]), _res([(-5.0, 3, 3.0)]), _res([(0.0, -1, 0.0)])])
    assert combine_results(parts)[0]['global_idx'] == 3


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from hyperopt_amd.dist import allgather_results
    # problem 0: rank 1 holds the max; problem 1: tie -> lower global index (rank 0)
    local = _res([(1.0 + rank, 10 * rank + 1, float(rank)), (5.0, 100 + rank, float(rank))])
    out = allgather_results(local)
    q.put((rank, out['global_idx'].tolist(), out['value'].tolist()))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_allgather():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, gidx, val in out:
        assert gidx == [11, 100] and val == [1.0, 0.0]


def _from_rec(r):
    out = np.zeros(len(r['score']), dtype=N.RESULT_DTYPE)
    for f, v in r.items():
        out[f] = v
    return out


def _engine_worker(rank, world, port, cases, q):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from hyperopt_amd.dist import allgather_results
    out = []
    for case in cases:
        res = allgather_results(_from_rec(case['shards'][rank]))
        out.append({f: res[f].tolist() for f in ('score', 'value', 'global_idx')})
    q.put((rank, out))
    dist.destroy_process_group()


def test_gloo_world2_combines_recorded_engine_shards():
    """Real device outputs (tests/golden/shard_results.json, recorded on an
    MI355X by tools/gen_shard_fixture.py: the config-3 tree's fused level run
    unsharded and as two candidate shards) combined over a world-2 gloo group
    equal the unsharded run on every problem."""
    from tests.conftest import load_golden
    cases = load_golden('shard_results.json')
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, 2, port, cases, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got in out:
        for case, g in zip(cases, got):
            full = case['full']
            assert g['global_idx'] == full['global_idx'], (rank, case['C'], case['seed'])
            assert g['value'] == full['value'] and g['score'] == full['score']


# ------------------------------------------------------------ id / label axes
def _axes_worker(rank, world, port, q):
    """The new-id and hyperparameter gathers (dist.gather_id_blocks /
    gather_label_columns) through the C exchange (tpe_exchange_allgather, host
    gather over gloo — the RCCL path runs the same call on a device buffer)."""
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hyperopt_amd import dist as D
        ex = D._Exchange(None, None)
        out = {}
        # new-id axis: 11 ids x 3 labels, the full matrix is a known function
        n, L = 11, 3
        full_v = np.arange(n * L, dtype=np.float64).reshape(n, L) * 0.5
        full_a = (np.arange(n * L).reshape(n, L) % 3) != 0
        full_v[~full_a] = np.nan
        lo, hi = D.shard_range(n, rank, world)
        v, a = D.gather_id_blocks(ex, full_v[lo:hi], full_a[lo:hi], n, L)
        out['ids'] = (np.array_equal(v, full_v, equal_nan=True), bool((a == full_a).all()))
        # hyperparameter axis: each rank knows only its own columns (and the gates)
        owner = [-1, 0, 1, 2, 0, 1, 2, 0][:8]
        owner = [o if o < world else o % world for o in owner]
        full = np.random.RandomState(5).uniform(size=(4, 8))
        mine = np.where([o in (-1, rank) for o in owner], full, np.nan)
        got = D.gather_label_columns(ex, mine, owner)
        out['labels'] = bool(np.array_equal(got, full))
        # 2-D axis: 9 ids x 8 labels (one gate) over (G, B) = grid_shape, and a
        # forced (G, B) = (world, 1) and (1, world): each rank its labels of its ids
        n2, own1 = 9, [-1] + list(range(7))
        full2 = np.random.RandomState(6).uniform(size=(n2, 8))
        act2 = np.random.RandomState(7).uniform(size=(n2, 8)) > 0.3
        ok = []
        for shape in (D.grid_shape(7, n2, world), (world, 1), (1, world)):
            g, b = D.grid_cell(rank, shape)
            owner = [o if o < 0 else o % shape[0] for o in own1]
            lo2, hi2 = D.shard_range(n2, b, shape[1])
            mine = np.where([o in (-1, g) for o in owner], full2[lo2:hi2], np.nan)
            v, a = D.gather_grid_blocks(ex, shape, mine, act2[lo2:hi2], n2, owner)
            ok.append(bool(np.array_equal(v, full2) and np.array_equal(a, act2)))
        out['grid'] = ok
        # a failed rank: every rank raises, none waits
        try:
            D.gather_id_blocks(ex, full_v[lo:hi], full_a[lo:hi], n, L, failed=(rank == world - 1))
            out['failure'] = 'no error'
        except RuntimeError as e:
            out['failure'] = str(e)
        q.put((rank, out, None))
    except Exception as e:
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3, 4])
def test_gloo_id_and_label_axis_gathers(world):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_axes_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got, err in out:
        assert err is None, (rank, err)
        assert got['ids'] == (True, True), (rank, got)
        assert got['labels'], rank
        assert got['grid'] == [True, True, True], (rank, got['grid'])
        assert 'failed on rank(s) [%d]' % (world - 1) in got['failure'], (rank, got['failure'])


def test_label_owners_round_robin_non_gates():
    """Hyperparameter axis: the gates on every rank, the other labels
    round-robin in table order."""
    import bench
    from hyperopt_amd import hp
    from hyperopt_amd.space import ParamTable
    from hyperopt_amd.dist import label_owners
    T = ParamTable(bench.tree_space(hp))
    for world in (1, 2, 3, 8):
        own = label_owners(T, world)
        gates = set(T.parent_labels)
        assert [o == -1 for o in own] == [r.label in gates for r in T.rows]
        ng = [o for o in own if o >= 0]
        assert ng == [k % world for k in range(len(ng))]


def test_grid_shape_balances_problems():
    """2-D shard shape: the smallest largest per-rank problem share, the most
    label groups among equal shares (config 4 at 8 ranks: 4 groups of 5
    labels x 2 blocks of 2048 ids — 10240 problems a rank, where the label
    axis alone gives 3 labels x 4096 ids = 12288 to the fullest rank)."""
    from hyperopt_amd.dist import grid_shape, label_cost
    # a label's own part (fits, rows, table) repeated by each id block of its
    # group: config 4's (10^4 observations, 4096 candidates) keeps whole labels
    assert grid_shape(20, 4096, 8, label_cost(10000, 4096)) == (8, 1)
    assert grid_shape(3, 4096, 8, label_cost(10000, 4096)) == (2, 4)
    assert grid_shape(20, 4096, 8, label_cost(100, 2 ** 20)) == (4, 2)
    assert grid_shape(20, 4096, 8) == (4, 2)
    assert grid_shape(20, 4096, 4) == (4, 1)
    assert grid_shape(20, 4096, 2) == (2, 1)
    assert grid_shape(20, 4096, 1) == (1, 1)
    assert grid_shape(1000, 1, 8) == (8, 1)
    assert grid_shape(3, 4096, 8) == (1, 8)
    assert grid_shape(6, 512, 4) == (2, 2)
    for L, n, w in ((20, 4096, 8), (7, 100, 6), (1000, 2, 4), (5, 5, 8)):
        G, B = grid_shape(L, n, w)
        assert G * B == w and G <= max(L, 1)
        share = -(-L // G) * -(-n // B)
        assert all(share <= -(-L // g) * -(-n // (w // g)) for g in range(1, w + 1) if w % g == 0 and g <= L)
