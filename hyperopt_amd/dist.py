"""Multi-GPU combine step: the only collective of the suggest path.

Candidates of one suggest shard along the candidate axis (each rank owns a
contiguous global index range and draws exactly the candidates a single GPU
would draw at those indices — Philox counters are global indices).  Each rank
selects its local best per problem; one all-gather of the per-problem results
(48 B each) and a host argmax with ``np.argmax`` semantics — NaN first, then
the largest score, then the lowest global index — give every rank the same
winner, so tree levels stay in lock-step.  New-id and hyperparameter sharding
need no collective at all.
"""
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
