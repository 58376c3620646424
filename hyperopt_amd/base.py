"""Trials / Domain data model — the idxs/vals document layout of the reference.

Kept compatible with base.py of gsmafra/hyperopt 0.0.3 (cited per symbol):
trial documents, ``misc['idxs']/misc['vals']`` one-element lists, the STATUS
and JOB_STATE constants, ``Trials`` accessors and ``Domain.evaluate``.  What
changes is underneath: ``Domain`` flattens the space once into a
``ParamTable`` (no pyll graph, no VectorizeHelper), and ``Trials`` carries a
derivable SoA cache of the history for the suggest hot path (``history``).
"""
import datetime
import logging
import operator

import numpy as np

from .exceptions import DuplicateLabel, InvalidLoss, InvalidResultStatus, InvalidTrial  # noqa: F401
from . import space as _space

logger = logging.getLogger(__name__)

# base.py:26-52
STATUS_NEW = 'new'
STATUS_RUNNING = 'running'
STATUS_SUSPENDED = 'suspended'
STATUS_OK = 'ok'
STATUS_FAIL = 'fail'
STATUS_STRINGS = ('new', 'running', 'suspended', 'ok', 'fail')

JOB_STATE_NEW = 0
JOB_STATE_RUNNING = 1
JOB_STATE_DONE = 2
JOB_STATE_ERROR = 3
JOB_STATES = [JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR]

TRIAL_KEYS = ['tid', 'spec', 'result', 'misc', 'state', 'owner', 'book_time', 'refresh_time', 'exp_key']
TRIAL_MISC_KEYS = ['tid', 'cmd', 'idxs', 'vals']


def SONify(arg, memo=None):
    return arg


def miscs_update_idxs_vals(miscs, idxs, vals, assert_all_vals_used=True, idxs_map=None):
    """Unpack idxs/vals into misc dicts (base.py:77-105)."""
    if idxs_map is None:
        idxs_map = {}
    assert set(idxs.keys()) == set(vals.keys())
    misc_by_id = dict((m['tid'], m) for m in miscs)
    for m in miscs:
        m['idxs'] = dict((key, []) for key in idxs)
        m['vals'] = dict((key, []) for key in idxs)
    for key in idxs:
        assert len(idxs[key]) == len(vals[key])
        for tid, val in zip(idxs[key], vals[key]):
            tid = idxs_map.get(tid, tid)
            if assert_all_vals_used or tid in misc_by_id:
                misc_by_id[tid]['idxs'][key] = [tid]
                misc_by_id[tid]['vals'][key] = [val]
    return miscs


def miscs_to_idxs_vals(miscs, keys=None):
    """Pack misc dicts into per-label idxs/vals lists (base.py:108-123)."""
    if keys is None:
        if len(miscs) == 0:
            raise ValueError('cannot infer keys from empty miscs')
        keys = miscs[0]['idxs'].keys()
    idxs = dict((k, []) for k in keys)
    vals = dict((k, []) for k in keys)
    for misc in miscs:
        for node_id in idxs:
            t_idxs = misc['idxs'][node_id]
            t_vals = misc['vals'][node_id]
            assert len(t_idxs) == len(t_vals)
            assert t_idxs == [] or t_idxs == [misc['tid']]
            idxs[node_id].extend(t_idxs)
            vals[node_id].extend(t_vals)
    return idxs, vals


def spec_from_misc(misc):
    """base.py:126-135"""
    spec = {}
    for k, v in misc['vals'].items():
        if len(v) == 0:
            pass
        elif len(v) == 1:
            spec[k] = v[0]
        else:
            raise NotImplementedError('multiple values', (k, v))
    return spec


def coarse_utcnow():
    """utils.py:127-136: UTC now rounded down to milliseconds."""
    now = datetime.datetime.utcnow()
    return now.replace(microsecond=(now.microsecond // 1000) * 1000)


class Trials(object):
    """History of evaluated and scheduled trials (base.py:138-438)."""

    def __init__(self, exp_key=None, refresh=True):
        self._ids = set()
        self._dynamic_trials = []
        self._exp_key = exp_key
        self.attachments = {}
        if refresh:
            self.refresh()

    # the SoA history cache is derivable state: never pickled
    def __getstate__(self):
        d = dict(self.__dict__)
        d.pop('_tpe_history', None)
        return d

    def aname(self, trial, name):
        return 'ATTACH::%s::%s' % (trial['tid'], name)

    def trial_attachments(self, trial):
        outer = self

        class Attachments(object):
            def __contains__(_self, name):
                return outer.aname(trial, name) in outer.attachments

            def __getitem__(_self, name):
                return outer.attachments[outer.aname(trial, name)]

            def __setitem__(_self, name, value):
                outer.attachments[outer.aname(trial, name)] = value

            def __delitem__(_self, name):
                del outer.attachments[outer.aname(trial, name)]
        return Attachments()

    def __iter__(self):
        return iter(self._trials)

    def __len__(self):
        return len(self._trials)

    def __getitem__(self, item):
        raise NotImplementedError('')

    def refresh(self):
        """Drop ERROR trials (and other experiments' trials) from the view.

        ``_view_gen`` counts the refreshes whose view is NOT the previous view
        plus appended documents (a document dropped, replaced or reordered):
        derived caches of the view (history.py) rebuild when it moves."""
        old = getattr(self, '_trials', None)
        if self._exp_key is None:
            self._trials = [tt for tt in self._dynamic_trials if tt['state'] != JOB_STATE_ERROR]
        else:
            self._trials = [tt for tt in self._dynamic_trials
                            if tt['state'] != JOB_STATE_ERROR and tt['exp_key'] == self._exp_key]
        new = self._trials
        if old is not None and not (len(new) >= len(old) and all(map(operator.is_, old, new))):
            self._view_gen = getattr(self, '_view_gen', 0) + 1
        self._ids.update([tt['tid'] for tt in self._trials])

    @property
    def trials(self):
        return self._trials

    @property
    def tids(self):
        return [tt['tid'] for tt in self._trials]

    @property
    def specs(self):
        return [tt['spec'] for tt in self._trials]

    @property
    def results(self):
        return [tt['result'] for tt in self._trials]

    @property
    def miscs(self):
        return [tt['misc'] for tt in self._trials]

    @property
    def idxs_vals(self):
        return miscs_to_idxs_vals(self.miscs)

    @property
    def idxs(self):
        return self.idxs_vals[0]

    @property
    def vals(self):
        return self.idxs_vals[1]

    def assert_valid_trial(self, trial):
        if not (hasattr(trial, 'keys') and hasattr(trial, 'values')):
            raise InvalidTrial('trial should be dict-like', trial)
        for key in TRIAL_KEYS:
            if key not in trial:
                raise InvalidTrial('trial missing key %s', key)
        for key in TRIAL_MISC_KEYS:
            if key not in trial['misc']:
                raise InvalidTrial('trial["misc"] missing key', key)
        if trial['tid'] != trial['misc']['tid']:
            raise InvalidTrial('tid mismatch between root and misc', trial)
        if trial['exp_key'] != self._exp_key:
            raise InvalidTrial('wrong exp_key', (trial['exp_key'], self._exp_key))
        return trial

    def _insert_trial_docs(self, docs):
        rval = [doc['tid'] for doc in docs]
        self._dynamic_trials.extend(docs)
        return rval

    def insert_trial_docs(self, docs):
        docs = [self.assert_valid_trial(SONify(doc)) for doc in docs]
        return self._insert_trial_docs(docs)

    def new_trial_ids(self, N):
        aa = len(self._ids)
        rval = list(range(aa, aa + N))
        self._ids.update(rval)
        return rval

    def new_trial_docs(self, tids, specs, results, miscs):
        assert len(tids) == len(specs) == len(results) == len(miscs)
        rval = []
        for tid, spec, result, misc in zip(tids, specs, results, miscs):
            doc = dict(state=JOB_STATE_NEW, tid=tid, spec=spec, result=result, misc=misc)
            doc['exp_key'] = self._exp_key
            doc['owner'] = None
            doc['version'] = 0
            doc['book_time'] = None
            doc['refresh_time'] = None
            rval.append(doc)
        return rval

    def count_by_state_synced(self, arg, trials=None):
        if trials is None:
            trials = self._trials
        if arg in JOB_STATES:
            queue = [doc for doc in trials if doc['state'] == arg]
        elif hasattr(arg, '__iter__'):
            states = set(arg)
            assert all(x in JOB_STATES for x in states)
            queue = [doc for doc in trials if doc['state'] in states]
        else:
            raise TypeError(arg)
        return len(queue)

    def count_by_state_unsynced(self, arg):
        if self._exp_key is not None:
            exp_trials = [tt for tt in self._dynamic_trials if tt['exp_key'] == self._exp_key]
        else:
            exp_trials = self._dynamic_trials
        return self.count_by_state_synced(arg, trials=exp_trials)

    def losses(self, bandit=None):
        if bandit is None:
            return [r.get('loss') for r in self.results]
        return list(map(bandit.loss, self.results, self.specs))

    def statuses(self, bandit=None):
        if bandit is None:
            return [r.get('status') for r in self.results]
        return list(map(bandit.status, self.results, self.specs))

    @property
    def best_trial(self):
        """Trial with lowest loss and status=STATUS_OK (base.py:417-426)."""
        candidates = [t for t in self.trials if t['result']['status'] == STATUS_OK]
        losses = [float(t['result']['loss']) for t in candidates]
        assert not np.any(np.isnan(losses))
        return candidates[int(np.argmin(losses))]

    @property
    def argmin(self):
        vals = self.best_trial['misc']['vals']
        return dict((k, v[0]) for k, v in vals.items() if v)


class Ctrl(object):
    """Control object for interruptible, checkpoint-able evaluation (base.py:441-472)."""
    info = logger.info
    warn = logger.warning
    error = logger.error
    debug = logger.debug

    def __init__(self, trials, current_trial=None):
        self.trials = Trials() if trials is None else trials
        self.current_trial = current_trial

    def checkpoint(self, r=None):
        assert self.current_trial in self.trials._trials
        if r is not None:
            self.current_trial['result'] = r

    @property
    def attachments(self):
        return self.trials.trial_attachments(trial=self.current_trial)


class Domain(object):
    """Picklable search space + objective (base.py:474-641)."""
    rec_eval_print_node_on_error = False

    def __init__(self, fn, expr, workdir=None, pass_expr_memo_ctrl=None, name=None):
        self.fn = fn
        if pass_expr_memo_ctrl is None:
            self.pass_expr_memo_ctrl = getattr(fn, 'fmin_pass_expr_memo_ctrl', False)
        else:
            self.pass_expr_memo_ctrl = pass_expr_memo_ctrl
        self.expr = expr
        self.table = _space.ParamTable(expr)
        self.params = dict((r.label, r.node) for r in self.table.rows)
        self.name = name
        self.workdir = workdir
        self.cmd = ('domain_attachment', 'FMinIter_Domain')

    def memo_from_config(self, config):
        return dict(config)

    def evaluate(self, config, ctrl, attach_attachments=True):
        if self.pass_expr_memo_ctrl:
            rval = self.fn(expr=self.expr, memo=self.memo_from_config(config), ctrl=ctrl)
        else:
            rval = self.fn(_space.evaluate(self.expr, config))
        if isinstance(rval, (float, int, np.number)):
            dict_rval = {'loss': float(rval), 'status': STATUS_OK}
        else:
            dict_rval = dict(rval)
            status = dict_rval['status']
            if status not in STATUS_STRINGS:
                raise InvalidResultStatus(dict_rval)
            if status == STATUS_OK:
                try:
                    dict_rval['loss'] = float(dict_rval['loss'])
                except (TypeError, KeyError):
                    raise InvalidLoss(dict_rval)
        if attach_attachments:
            attachments = dict_rval.pop('attachments', {})
            for key, val in attachments.items():
                ctrl.attachments[key] = val
        return dict_rval

    def loss(self, result, config=None):
        return result.get('loss', None)

    def loss_variance(self, result, config=None):
        return result.get('loss_variance', 0.0)

    def true_loss(self, result, config=None):
        try:
            return result['true_loss']
        except KeyError:
            return self.loss(result, config=config)

    def status(self, result, config=None):
        return result['status']

    def new_result(self):
        return {'status': STATUS_NEW}
