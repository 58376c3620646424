"""``hp.*`` search-space constructors (reference hp.py:6-18, pyll_utils.py:35-116).

Same names, positional arguments and label validation as the reference.
Continuous parameters are seen by the objective as Python floats (the
reference wraps them in ``scope.float``); ``randint`` values stay integers;
``choice``/``pchoice`` select one of their options.
"""
from .space import Param, Switch


def _label(label):
    if not isinstance(label, str):
        raise TypeError('require string label')
    return label


def _mk(dist, as_float):
    names = {'uniform': ('low', 'high'), 'quniform': ('low', 'high', 'q'),
             'loguniform': ('low', 'high'), 'qloguniform': ('low', 'high', 'q'),
             'normal': ('mu', 'sigma'), 'qnormal': ('mu', 'sigma', 'q'),
             'lognormal': ('mu', 'sigma'), 'qlognormal': ('mu', 'sigma', 'q'),
             'randint': ('upper',)}[dist]

    def ctor(label, *args, **kwargs):
        _label(label)
        vals = dict(zip(names, args))
        for k, v in kwargs.items():
            if k not in names or k in vals:
                raise TypeError('%s() got an unexpected argument %r' % (dist, k))
            vals[k] = v
        missing = [n for n in names if n not in vals]
        if missing:
            raise TypeError('%s() missing argument(s) %s' % (dist, ', '.join(missing)))
        return Param(label, dist, vals, as_float)
    ctor.__name__ = dist
    return ctor


uniform = _mk('uniform', True)
quniform = _mk('quniform', True)
loguniform = _mk('loguniform', True)
qloguniform = _mk('qloguniform', True)
normal = _mk('normal', True)
qnormal = _mk('qnormal', True)
lognormal = _mk('lognormal', True)
qlognormal = _mk('qlognormal', True)
randint = _mk('randint', False)


def choice(label, options):
    """One of ``options`` (pyll_utils.py:50-54: switch over randint(len))."""
    _label(label)
    options = list(options)
    return Switch(Param(label, 'randint', {'upper': len(options)}, False), options)


def pchoice(label, p_options):
    """One of the options with given probabilities (pyll_utils.py:35-47)."""
    _label(label)
    p, options = zip(*p_options)
    return Switch(Param(label, 'categorical', {'p': list(p), 'upper': len(options)}, False), options)
