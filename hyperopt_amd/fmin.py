"""Serial optimisation driver (reference fmin.py:20-175).

Same loop as ``FMinIter.run``: one new id at a time (``max_queue_len=1``),
``algo(new_ids, domain, trials, rstate.randint(2**31 - 1))``, then serial
evaluation.  Differences kept deliberately small: ``trials=None`` creates a
``Trials`` (the reference crashes), ``fmin`` returns ``trials.argmin`` when
``return_argmin`` (the reference returns None), and the RUNNING state is
actually assigned (fmin.py:43 compares instead of assigning).
"""
import logging
import os
import pickle
import sys

import numpy as np

from . import base
from .base import coarse_utcnow

logger = logging.getLogger(__name__)


class FMinIter(object):
    catch_eval_exceptions = False
    pickle_protocol = -1

    def __init__(self, algo, domain, trials, rstate, max_queue_len=1, poll_interval_secs=1.0,
                 max_evals=sys.maxsize):
        self.algo = algo
        self.domain = domain
        self.trials = trials
        self.poll_interval_secs = poll_interval_secs
        self.max_queue_len = max_queue_len
        self.max_evals = max_evals
        self.rstate = rstate

    def serial_evaluate(self, N=-1):
        for trial in self.trials._dynamic_trials:
            if trial['state'] == base.JOB_STATE_NEW:
                trial['state'] = base.JOB_STATE_RUNNING
                now = coarse_utcnow()
                trial['book_time'] = now
                trial['refresh_time'] = now
                spec = base.spec_from_misc(trial['misc'])
                ctrl = base.Ctrl(self.trials, current_trial=trial)
                try:
                    result = self.domain.evaluate(spec, ctrl)
                except Exception as e:
                    logger.info('job exception: %s' % str(e))
                    trial['state'] = base.JOB_STATE_ERROR
                    trial['misc']['error'] = (str(type(e)), str(e))
                    trial['refresh_time'] = coarse_utcnow()
                    if not self.catch_eval_exceptions:
                        self.trials.refresh()
                        raise
                else:
                    trial['state'] = base.JOB_STATE_DONE
                    trial['result'] = result
                    trial['refresh_time'] = coarse_utcnow()
                N -= 1
                if N == 0:
                    break
        self.trials.refresh()

    def run(self, N):
        trials = self.trials
        algo = self.algo
        n_queued = 0

        def get_queue_len():
            return self.trials.count_by_state_unsynced(base.JOB_STATE_NEW)

        stopped = False
        while n_queued < N:
            qlen = get_queue_len()
            while qlen < self.max_queue_len and n_queued < N:
                n_to_enqueue = min(self.max_queue_len - qlen, N - n_queued)
                new_ids = trials.new_trial_ids(n_to_enqueue)
                self.trials.refresh()
                new_trials = algo(new_ids, self.domain, trials, self.rstate.randint(2 ** 31 - 1))
                assert len(new_ids) >= len(new_trials)
                if len(new_trials):
                    self.trials.insert_trial_docs(new_trials)
                    self.trials.refresh()
                    n_queued += len(new_trials)
                    qlen = get_queue_len()
                else:
                    stopped = True
                    break
            self.serial_evaluate()
            if stopped:
                break
        qlen = get_queue_len()
        if qlen:
            logger.info('Exiting run, not waiting for %d jobs.' % qlen)

    def __iter__(self):
        return self

    def exhaust(self):
        n_done = len(self.trials)
        self.run(self.max_evals - n_done)
        self.trials.refresh()
        return self


def fmin(fn, space, algo, max_evals, trials=None, rstate=None, pass_expr_memo_ctrl=None,
         catch_eval_exceptions=False, return_argmin=True, max_queue_len=1):
    """Minimise ``fn`` over ``space`` (fmin.py:121-140)."""
    if rstate is None:
        env_rseed = os.environ.get('HYPEROPT_FMIN_SEED', '')
        rstate = np.random.RandomState(int(env_rseed)) if env_rseed else np.random.RandomState()
    if trials is None:
        trials = base.Trials()
    domain = base.Domain(fn, space, pass_expr_memo_ctrl=pass_expr_memo_ctrl)
    rval = FMinIter(algo, domain, trials, max_evals=max_evals, rstate=rstate, max_queue_len=max_queue_len)
    rval.catch_eval_exceptions = catch_eval_exceptions
    rval.exhaust()
    if return_argmin and len(trials):
        try:
            return trials.argmin
        except (AssertionError, ValueError, IndexError):
            return None
    return None


def dump_trials(trials, path):
    with open(path, 'wb') as f:
        pickle.dump(trials, f, protocol=FMinIter.pickle_protocol)


def fmin_path(objective, space, max_evals, path):
    """Resumable fmin: load pickled Trials from ``path`` if present, run
    ``max_evals`` more evaluations with TPE, dump (also on error) — fmin.py:147-175.
    Only load files you wrote yourself: unpickling executes code."""
    from . import tpe
    try:
        with open(path, 'rb') as f:
            trials = pickle.load(f)
    except Exception:                 # any unreadable file starts fresh, as the reference's bare except
        logger.info('No trial file at %s, creating a new one', path)
        trials = base.Trials()
    try:
        fmin(objective, space=space, algo=tpe.suggest, max_evals=len(trials) + max_evals, trials=trials)
        dump_trials(trials, path)
    except BaseException:
        dump_trials(trials, path)
        raise
    return trials
