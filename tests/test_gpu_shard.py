"""End-to-end candidate sharding on the device: two processes (gloo, both on
the one GPU) each run tpe.suggest(..., shard=(rank, 2)) — half of the
candidate index range, the same Philox counters a single device would use —
and combine through dist.allgather_results; the result must be the unsharded
suggest's (reference tpe.py:749-759: the per-parameter argmax over every
candidate).  Categorical choices (the tree's gates among them) must match
exactly; a continuous value either matches or scores within the fp32 eps-tie
tolerance of the unsharded winner (fp32 above sums of pruned labels follow
the batch layout)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.helpers import doc_values

pytestmark = pytest.mark.gpu

N_HIST = 3000
CASES = [('fp32', 1 << 18, 11), ('fp32', 1 << 16, 12), ('fp64', 1 << 16, 13)]


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import bench
        from hyperopt_amd import tpe
        from hyperopt_amd.engine import get_engine
        domain, trials = bench.make_history(N_HIST, 0)
        out, paths = [], []
        for precision, C, seed in CASES:
            eng = get_engine(precision=precision)
            eng.last_tree_path = None
            docs = tpe.suggest([N_HIST], domain, trials, seed, n_EI_candidates=C, precision=precision,
                               shard=(rank, world))
            out.append({k: float(v) for k, v in doc_values(docs).items()})
            paths.append(eng.last_tree_path)
        q.put((rank, (out, paths), None))
    except Exception as e:          # report, do not hang the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _score(post, x):
    """l - g of value x under a posterior (oracle lpdf, float64)."""
    from oracle import tpe_oracle as O
    lpdf = O.lgmm1_lpdf if post.family == 1 else O.gmm1_lpdf
    kw = dict(low=post.low, high=post.high, q=post.q)
    xs = np.array([x])
    return float(lpdf(xs, *post.below, **kw)[0] - lpdf(xs, *post.above, **kw)[0])


def test_two_process_shard_matches_unsharded():
    import bench
    from hyperopt_amd import history as H, tpe
    from hyperopt_amd.engine import get_engine
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        rank, out, err = q.get(timeout=240)
        assert err is None, (rank, err)
        got[rank], paths = out
        # fp32: the native tree path, its level results exchanged inside the native
        # call (gloo: the host gather); fp64 takes the general path
        for (precision, C, seed), path in zip(CASES, paths):
            assert (path is not None) == (precision == 'fp32'), (rank, precision, path)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1]                       # every rank holds the combined winner
    domain, trials = bench.make_history(N_HIST, 0)
    T = domain.table
    for (precision, C, seed), sharded in zip(CASES, got[0]):
        ref = {k: float(v) for k, v in doc_values(tpe.suggest([N_HIST], domain, trials, seed, n_EI_candidates=C,
                                                               precision=precision)).items()}
        assert set(ref) == set(sharded), (precision, C, seed)
        hist = H.extract(domain, trials)
        fits = tpe._Fits(T, hist, H.split_below(hist, 0.25), 1.0, get_engine(precision=precision))
        for k, v in ref.items():
            row = T.by_label[k]
            if row.categorical or v == sharded[k]:
                assert v == sharded[k], (precision, C, seed, k, v, sharded[k])
                continue
            post = fits.get(row)
            s_ref, s_got = _score(post, v), _score(post, sharded[k])
            assert abs(s_ref - s_got) <= 1e-5 * max(1.0, abs(s_ref)), (precision, C, seed, k, v, sharded[k])


def _rccl_worker(port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1)
    try:
        import bench
        from hyperopt_amd import dist as D, tpe
        from hyperopt_amd.engine import get_engine
        domain, trials = bench.make_history(N_HIST, 0)
        ref = [doc_values(tpe.suggest([N_HIST], domain, trials, s, n_EI_candidates=1 << 18)) for s in (21, 22)]
        D.EXCHANGE_ALWAYS = True
        eng = get_engine()
        got = []
        for s in (21, 22):
            eng.last_tree_path = None
            got.append(doc_values(tpe.suggest([N_HIST], domain, trials, s, n_EI_candidates=1 << 18, shard=(0, 1))))
            assert eng.last_tree_path is not None
        ex = D.exchange_for(eng)
        q.put(([{k: float(v) for k, v in r.items()} for r in ref], [{k: float(v) for k, v in g.items()} for g in got],
               ex.comm is not None, None))
        ex.close()
    except Exception as e:
        q.put((None, None, None, repr(e)))
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_one_rank():
    """The RCCL exchange path of the native tree (tpe_comm_init from C, an
    in-place ncclAllGather of the level results on the suggest's stream, the
    host reduction) on a one-rank nccl group — the one GPU of the box — with
    the exchange forced on: the suggestions equal the unsharded ones."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    ref, got, rccl, err = q.get(timeout=240)
    p.join(timeout=60)
    assert err is None, err
    assert rccl, 'the exchange did not take the RCCL path'
    assert ref == got
