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

The other two axes (include/tpe_hip.h, "Shard axes") exchange once, after the
whole suggest: ``gather_id_blocks`` (new-id axis: every rank's block of ids)
and ``gather_label_columns`` (hyperparameter axis: every rank's labels), both
through ``tpe_exchange_allgather`` on the same exchange.  A rank whose own
part failed still takes part (status word), so no rank waits forever and every
rank raises.
"""
import ctypes
import os

import numpy as np

from . import _native as N


def shard_range(n_total, rank, world):
    """Contiguous [start, stop) of the candidate index range owned by ``rank``."""
    return (n_total * rank) // world, (n_total * (rank + 1)) // world


def label_owners(table, world):
    """Hyperparameter-axis shard of a ParamTable over ``world`` ranks: per label
    (table order) the rank that evaluates it, -1 for the gates — every rank
    evaluates those, so every rank knows which labels are active.  The other
    labels go round-robin in table order (config 5: 1000 labels, 125 a rank)."""
    gates = set(table.parent_labels)
    owner, k = [], 0
    for r in table.rows:
        if r.label in gates:
            owner.append(-1)
        else:
            owner.append(k % world)
            k += 1
    return owner


def grid_shape(n_labels, n_ids, world, label_cost=0.0):
    """(G, B) of the 2-D shard of a batched suggest's (label x new id) problem
    grid over ``world`` ranks: G label groups (dist.label_owners over G) times
    B id blocks (shard_range over B), G * B = world.  A rank's work is its
    labels' own part (fits, component rows, tables: made again by each of a
    group's B ranks) plus its problems' (the candidates of every id of its
    block): ceil(n_labels / G) * (label_cost + ceil(n_ids / B)), with
    ``label_cost`` a label's own part in problems; the smallest wins, among
    equals the most label groups.  label_cost 0: the most even problem
    count.  ``n_labels``: the labels that shard (the non-gates)."""
    best = None
    for g in range(1, world + 1):
        if world % g or (g > max(1, n_labels)):
            continue
        b = world // g
        cost = -(-max(n_labels, 1) // g) * (float(label_cost) + -(-max(n_ids, 1) // b))
        key = (cost, -g)
        if best is None or key < best[0]:
            best = (key, g, b)
    return best[1], best[2]


def label_cost(n_obs, n_cand):
    """A label's own part of a batched suggest (its Parzen fits, component
    rows and table) in units of one problem's candidates (draw + score of
    n_cand): ~3.5 ns per observation against ~5 ps per candidate on MI355X
    (config 4: 20 labels' fits, rows and tables 0.70 ms for 10^4
    observations each; 4096 x 20 problems' sample pass 1.68 ms at 4096
    candidates)."""
    return 700.0 * float(n_obs) / max(float(n_cand), 1.0)


def grid_cell(rank, shape):
    """(label group, id block) of ``rank`` in a (G, B) grid: the B ranks of a
    label group are consecutive."""
    return rank // shape[1], rank % shape[1]


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
        # (no engine: a host-gather exchange, e.g. the CPU tests of the gathers)
        self.lib = engine.lib if engine is not None else N.load()
        self.comm = None
        self.scratch = None
        self.ex = N.Exchange()
        self.ex.rank, self.ex.world, self.ex.always = self.rank, self.world, 1 if always else 0
        mode = os.environ.get('TPE_EXCHANGE', 'auto')
        if dist.get_backend(group) == 'nccl' and mode != 'host' and engine is not None:
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
            torch_dev = torch.device('cuda', engine._dev_index) if dist.get_backend(group) == 'nccl' and \
                engine is not None else None

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

    def allgather(self, buf, stream=None):
        """All-gather of a host byte buffer (one per rank, equal sizes) through
        tpe_exchange_allgather: uint8 [world, nbytes] in rank order."""
        buf = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
        n = buf.nbytes
        out = np.empty((self.world, n), dtype=np.uint8)
        if self.comm is not None:
            self._scratch(self.world * n)
        N.check(self.lib.tpe_exchange_allgather(ctypes.byref(self.ex), buf.ctypes.data, n, out.ctypes.data,
                                                stream if stream is not None or self.engine is None
                                                else self.engine._stream()),
                self.lib, 'tpe_exchange_allgather')
        return out

    def _scratch(self, need):
        import torch
        if self.scratch is None or self.scratch.numel() < need:
            self.scratch = torch.empty(max(need, 2 * (self.scratch.numel() if self.scratch is not None else 0)),
                                       dtype=torch.uint8, device=self.engine.device)
            self.ex.dev, self.ex.dev_bytes = self.scratch.data_ptr(), self.scratch.numel()

    def ptr(self, max_problems, n_cand=0):
        """The struct for a suggest of at most ``max_problems`` problems per
        level and ``n_cand`` candidates per problem on this rank (RCCL: device
        scratch for the exchange slots, and for the level's run records and
        results that the device combine reduces: tpe_internal_level_run_ex)."""
        if self.comm is not None:
            P = max(int(max_problems), 1)
            rec = N.RESULT_DTYPE.itemsize
            slots = (self.world * (N.EXCHANGE_HEADER + P * rec) + 255) // 256 * 256
            tiles = P * (-(-max(int(n_cand), 1) // N.tile_size()))
            self._scratch(slots + (tiles + P) * rec)
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


# ------------------------------------------------------------ id / label axes
_HDR = 8        # per-rank payload header: int64 status (0 ok, 1 failed)


def _exchange_status(ex, payload, failed):
    """All-gather ``payload`` (bytes, equal size on every rank) after an int64
    status word; raises on every rank when some rank failed."""
    buf = np.zeros(_HDR + payload.nbytes, dtype=np.uint8)
    buf[:_HDR].view(np.int64)[0] = 1 if failed else 0
    buf[_HDR:] = payload.view(np.uint8).reshape(-1)
    allb = ex.allgather(buf)
    bad = [r for r in range(ex.world) if allb[r, :_HDR].view(np.int64)[0] != 0]
    if bad:
        raise RuntimeError('sharded suggest failed on rank(s) %s' % bad)
    return allb[:, _HDR:]


def gather_id_blocks(ex, values, active, n_ids, n_labels, failed=False):
    """New-id axis: rank r computed ids [shard_range(n_ids, r, world)) —
    ``values`` float64 / ``active`` bool [block x n_labels] — and every rank
    gets the whole [n_ids x n_labels] pair (one all-gather, blocks padded to
    the largest)."""
    world = ex.world
    blocks = [shard_range(n_ids, r, world) for r in range(world)]
    m = max(hi - lo for lo, hi in blocks)
    per = m * n_labels
    pay = np.zeros(per * 9, dtype=np.uint8)
    if not failed:
        lo, hi = blocks[ex.rank]
        k = (hi - lo) * n_labels
        pay[:8 * per].view(np.float64)[:k] = np.asarray(values, dtype=np.float64).reshape(-1)
        pay[8 * per:8 * per + k] = np.asarray(active, dtype=bool).reshape(-1)
    allb = _exchange_status(ex, pay, failed)
    out_v = np.empty((n_ids, n_labels))
    out_a = np.empty((n_ids, n_labels), dtype=bool)
    for r, (lo, hi) in enumerate(blocks):
        k = (hi - lo) * n_labels
        out_v[lo:hi] = allb[r, :8 * per].view(np.float64)[:k].reshape(hi - lo, n_labels)
        out_a[lo:hi] = allb[r, 8 * per:8 * per + k].view(bool).reshape(hi - lo, n_labels)
    return out_v, out_a


def gather_grid_blocks(ex, shape, values, active, n_ids, owner, failed=False):
    """2-D axis: rank r = (g, b) computed the ids of block b (shard_range over
    B) for the labels of group g (``owner[ix] == g``; the gates, owner -1, on
    every rank) — ``values`` float64 / ``active`` bool [block x n_labels] —
    and every rank gets the whole [n_ids x n_labels] pair: one all-gather of
    every rank's block (padded to the largest), each label's column from its
    group's rank of that block, the activity from the block's group-0 rank
    (every rank of a block evaluated the same gates)."""
    G, B = shape
    world = ex.world
    L = len(owner)
    blocks = [shard_range(n_ids, b, B) for b in range(B)]
    m = max(hi - lo for lo, hi in blocks)
    per = m * L
    pay = np.zeros(per * 9, dtype=np.uint8)
    if not failed:
        g, b = grid_cell(ex.rank, shape)
        lo, hi = blocks[b]
        k = (hi - lo) * L
        pay[:8 * per].view(np.float64)[:k] = np.asarray(values, dtype=np.float64).reshape(-1)
        pay[8 * per:8 * per + k] = np.asarray(active, dtype=bool).reshape(-1)
    allb = _exchange_status(ex, pay, failed)
    out_v = np.empty((n_ids, L))
    out_a = np.empty((n_ids, L), dtype=bool)
    own = np.asarray(owner)
    cols = [np.flatnonzero((own == g) | ((own < 0) & (g == 0))) for g in range(G)]
    for r in range(world):
        g, b = grid_cell(r, shape)
        lo, hi = blocks[b]
        k = (hi - lo) * L
        v = allb[r, :8 * per].view(np.float64)[:k].reshape(hi - lo, L)
        out_v[lo:hi, cols[g]] = v[:, cols[g]]
        if g == 0:
            out_a[lo:hi] = allb[r, 8 * per:8 * per + k].view(bool).reshape(hi - lo, L)
    return out_v, out_a


def gather_label_columns(ex, values, owner, failed=False):
    """Hyperparameter axis: ``values`` float64 [n_ids x n_labels] holds this
    rank's labels (``owner[ix] == rank``; the gates, owner -1, everywhere);
    the other columns are filled from their owners (one all-gather of each
    rank's columns, padded to the largest share).  Activity needs no exchange:
    every rank evaluated the gates.  (A failed rank passes NaN values of the
    right shape.)"""
    world, rank = ex.world, ex.rank
    values = np.asarray(values, dtype=np.float64)
    n = values.shape[0]
    cols = [[ix for ix, o in enumerate(owner) if o == r] for r in range(world)]
    m = max(len(c) for c in cols)
    pay = np.zeros((n, m))
    if not failed and cols[rank]:
        pay[:, :len(cols[rank])] = values[:, cols[rank]]
    allb = _exchange_status(ex, pay, failed)
    out = values.copy()
    for r in range(world):
        if r != rank and cols[r]:
            out[:, cols[r]] = allb[r].view(np.float64).reshape(n, m)[:, :len(cols[r])]
    return out
