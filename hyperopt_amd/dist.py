"""Multi-GPU combine step: the only collective of the suggest path.

Candidates of one suggest shard along the candidate axis (each rank owns a
contiguous global index range and draws exactly the candidates a single GPU
would draw at those indices — Philox counters are global indices).  Each rank
selects its local best per problem; one all-gather of the per-problem results
(48 B each) and a host argmax with ``np.argmax`` semantics — NaN first, then
the largest score, then the lowest global index — give every rank the same
winner, so tree levels stay in lock-step.  New-id and hyperparameter sharding
need no collective at all.

The native tree path (tpe_suggest_tree) does this exchange itself after every
level (include/tpe_hip.h, "Candidate-shard exchange"): ``exchange_for`` gives
it an RCCL communicator (nccl process groups: an all-gather over xGMI on a
device buffer, issued from C on the suggest's stream) or a host all-gather
through ``torch.distributed`` (gloo groups).  ``allgather_results`` is the
same combine for the Python general path.
"""
import ctypes
import os

import numpy as np

from . import _native as N


def shard_range(n_total, rank, world):
    """Contiguous [start, stop) of the candidate index range owned by ``rank``."""
    return (n_total * rank) // world, (n_total * (rank + 1)) // world


def combine_results(stacked):
    """[world, P] RESULT_DTYPE -> [P]: the global winner of every problem."""
    stacked = np.asarray(stacked)
    if stacked.ndim == 1:
        return stacked
    world, P = stacked.shape
    out = stacked[0].copy()
    for r in range(1, world):
        cand = stacked[r]
        cur_nan, new_nan = np.isnan(out['score']), np.isnan(cand['score'])
        cur_empty, new_empty = out['idx'] < 0, cand['idx'] < 0
        with np.errstate(invalid='ignore'):
            better = (new_nan & (~cur_nan | (cand['global_idx'] < out['global_idx']))) | \
                     (~new_nan & ~cur_nan & ((cand['score'] > out['score'])
                                             | ((cand['score'] == out['score'])
                                                & (cand['global_idx'] < out['global_idx']))))
        better = (better & ~new_empty) | (cur_empty & ~new_empty)
        out[better] = cand[better]
    return out


def allgather_results(res, group=None, device=None):
    """All-gather per-problem results over ``torch.distributed`` and combine."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return res
    flat = torch.from_numpy(np.ascontiguousarray(res).view(np.float64).reshape(-1).copy())
    backend = dist.get_backend(group)
    if backend == 'nccl':
        flat = flat.to(device if device is not None else torch.device('cuda', torch.cuda.current_device()))
    outs = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(outs, flat, group=group)
    stacked = np.stack([o.cpu().numpy() for o in outs]).view(N.RESULT_DTYPE).reshape(world, -1)
    return combine_results(stacked)


class _Exchange(object):
    """A tpe_exchange for one (engine, process group): the struct, the
    objects it points at, and the device scratch of the RCCL path."""

    def __init__(self, engine, group, always=False):
        import torch
        import torch.distributed as dist
        self.engine, self.group = engine, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.lib = engine.lib
        self.comm = None
        self.scratch = None
        self.ex = N.Exchange()
        self.ex.rank, self.ex.world, self.ex.always = self.rank, self.world, 1 if always else 0
        mode = os.environ.get('TPE_EXCHANGE', 'auto')
        if dist.get_backend(group) == 'nccl' and mode != 'host':
            # RCCL communicator of this process group: rank 0's id, broadcast
            idb = ctypes.create_string_buffer(N.COMM_ID_BYTES)
            if self.rank == 0:
                N.check(self.lib.tpe_comm_unique_id(idb), self.lib, 'tpe_comm_unique_id')
            obj = [bytes(idb.raw)]
            dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
            idb = ctypes.create_string_buffer(obj[0], N.COMM_ID_BYTES)
            comm = ctypes.c_void_p()
            N.check(self.lib.tpe_comm_init(self.rank, self.world, idb, engine._dev_index, ctypes.byref(comm)),
                    self.lib, 'tpe_comm_init')
            self.comm = comm
            self.ex.comm = comm.value
            self.ex.gather = N.GATHER_FN()
        else:
            torch_dev = torch.device('cuda', engine._dev_index) if dist.get_backend(group) == 'nccl' else None

            def gather(ctx, mine, nbytes, out):
                try:
                    buf = (ctypes.c_ubyte * nbytes).from_address(mine)
                    t = torch.frombuffer(bytearray(buf), dtype=torch.uint8)
                    if torch_dev is not None:
                        t = t.to(torch_dev)
                    parts = [torch.empty_like(t) for _ in range(self.world)]
                    dist.all_gather(parts, t, group=group)
                    allb = torch.cat(parts).cpu().numpy()
                    ctypes.memmove(out, allb.ctypes.data, allb.nbytes)
                    return 0
                except Exception:            # reported as a failed exchange by the native call
                    return -1
            self._gather = N.GATHER_FN(gather)   # (kept alive with the struct)
            self.ex.gather = self._gather

    def ptr(self, max_problems):
        """The struct for a suggest of at most ``max_problems`` problems per level."""
        if self.comm is not None:
            import torch
            need = self.world * (N.EXCHANGE_HEADER + max(int(max_problems), 1) * N.RESULT_DTYPE.itemsize)
            if self.scratch is None or self.scratch.numel() < need:
                self.scratch = torch.empty(max(need, 2 * (self.scratch.numel() if self.scratch is not None else 0)),
                                           dtype=torch.uint8, device=self.engine.device)
                self.ex.dev, self.ex.dev_bytes = self.scratch.data_ptr(), self.scratch.numel()
        return ctypes.byref(self.ex)

    def close(self):
        if self.comm is not None:
            self.lib.tpe_comm_destroy(self.comm)
            self.comm = None
            self.ex.comm = None


_EXCHANGES = {}
# exchange even in a world of one rank (tests of the exchange on one GPU)
EXCHANGE_ALWAYS = False


def exchange_for(engine, group=None, always=None):
    """The engine's exchange over ``group`` (default: the default process
    group), created on first use — collectively: every rank of the group must
    call it (tpe.suggest does, on its first sharded call)."""
    always = EXCHANGE_ALWAYS if always is None else always
    key = (id(engine), id(group), bool(always))
    ex = _EXCHANGES.get(key)
    if ex is None:
        ex = _EXCHANGES[key] = _Exchange(engine, group, always)
    return ex
