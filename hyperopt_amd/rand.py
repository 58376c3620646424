"""Random search — the start-up path of TPE (reference rand.py:14-33).

Host code by design: it draws one value per active label from the prior with
the reference's shared ``np.random.RandomState(seed)``, in the reference's
consumption order (descending labels, ancestors first — the order its
``rec_eval`` interpreter visits them), so start-up trajectories are identical
to the reference's.  Prior draws follow pyll/stochastic.py:30-142.
"""
import numpy as np

from . import base


def prior_draw(rng, dist, a, size):
    """One vectorised prior draw (pyll/stochastic.py:30-142)."""
    if dist == 'uniform':
        return rng.uniform(a['low'], a['high'], size=size)
    if dist == 'quniform':
        return np.round(rng.uniform(a['low'], a['high'], size=size) / a['q']) * a['q']
    if dist == 'loguniform':
        return np.exp(rng.uniform(a['low'], a['high'], size=size))
    if dist == 'qloguniform':
        return np.round(np.exp(rng.uniform(a['low'], a['high'], size=size)) / a['q']) * a['q']
    if dist == 'normal':
        return rng.normal(a['mu'], a['sigma'], size=size)
    if dist == 'qnormal':
        return np.round(rng.normal(a['mu'], a['sigma'], size=size) / a['q']) * a['q']
    if dist == 'lognormal':
        return np.exp(rng.normal(a['mu'], a['sigma'], size=size))
    if dist == 'qlognormal':
        return np.round(np.exp(rng.normal(a['mu'], a['sigma'], size=size)) / a['q']) * a['q']
    if dist == 'randint':
        return rng.randint(a['upper'], size=size)
    if dist == 'categorical':
        if size == 0:
            return np.asarray([])
        p = np.asarray(a['p'])
        return np.dot(rng.multinomial(n=1, pvals=p, size=size), np.arange(len(p)))
    raise ValueError('unknown distribution %r' % dist)


def sample_config(table, rng):
    """{label: value} of the active labels of one random configuration."""
    chosen = {}
    for row in table.rng_order():
        if table.active(row, chosen):
            chosen[row.label] = prior_draw(rng, row.dist, row.args, 1)[0]
        else:
            chosen[row.label] = None
    return chosen


def docs_from_choices(new_ids, domain, trials, choices):
    """Trial documents for ``new_ids`` from per-id {label: value or None}."""
    rval = []
    for new_id, chosen in zip(new_ids, choices):
        # the misc miscs_update_idxs_vals builds for one id (base.py:77-105), directly
        # (tracked: edits of the returned documents reach the Trials' history cache)
        misc = base.tracked_misc(new_id, domain.cmd, domain.workdir, chosen)
        rval.extend(trials.new_trial_docs([new_id], [None], [domain.new_result()], [misc]))
    return rval


def suggest(new_ids, domain, trials, seed):
    """Random configurations for ``new_ids`` (one shared RandomState, rand.py:14-33)."""
    rng = np.random.RandomState(seed)
    choices = [sample_config(domain.table, rng) for _ in new_ids]
    return docs_from_choices(new_ids, domain, trials, choices)


def suggest_batch(new_ids, domain, trials, seed):
    """idxs/vals of random configurations for ``new_ids`` drawn vectorised
    (one draw of size = number of active ids per label), as rand.py:36-46."""
    rng = np.random.RandomState(seed)
    table = domain.table
    chosen = [dict() for _ in new_ids]
    idxs = dict((r.label, []) for r in table.rows)
    vals = dict((r.label, []) for r in table.rows)
    for row in table.rng_order():
        act = [i for i, c in enumerate(chosen) if table.active(row, c)]
        draw = prior_draw(rng, row.dist, row.args, len(act))
        for c in chosen:
            c[row.label] = None
        for i, v in zip(act, draw):
            chosen[i][row.label] = v
            idxs[row.label].append(new_ids[i])
            vals[row.label].append(v)
    return idxs, vals
