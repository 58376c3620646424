"""Shared test helpers: build hyperopt_amd spaces / Trials from golden data."""
import numpy as np

from oracle.spacedesc import build_with_hp


def amd_space(desc):
    from hyperopt_amd import hp
    return build_with_hp(desc, hp)


def trials_from_history(hist, domain):
    """A hyperopt_amd Trials holding the golden history documents (DONE)."""
    from hyperopt_amd import base
    trials = base.Trials()
    labels = domain.table.labels
    docs = []
    for d in hist:
        vals = {k: list(d['vals'].get(k, [])) for k in labels}
        cat = {r.label: r.categorical for r in domain.table.rows}
        vals = {k: [np.int64(v[0]) if cat[k] else np.float64(v[0])] if v else [] for k, v in vals.items()}
        idxs = {k: ([d['tid']] if v else []) for k, v in vals.items()}
        misc = dict(tid=d['tid'], cmd=domain.cmd, workdir=None, idxs=idxs, vals=vals)
        doc = trials.new_trial_docs([d['tid']], [None], [{'status': 'ok', 'loss': d['loss']}], [misc])[0]
        doc['state'] = base.JOB_STATE_DONE
        docs.append(doc)
    trials.insert_trial_docs(docs)
    trials.refresh()
    return trials


def doc_values(docs):
    v = docs[0]['misc']['vals']
    return {k: x[0] for k, x in v.items() if len(x)}
