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
