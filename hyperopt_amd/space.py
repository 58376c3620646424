"""Search-space IR: what ``hp.*`` builds instead of a pyll graph.

The reference builds a pyll expression graph (pyll_utils.py:35-116), then a
vectorised idxs/vals graph per fmin (vectorize.py:152-378) that its TPE
rewrites and interprets on every suggest (tpe.py:644-716, pyll/base.py:679-836).
Here a space is a small tree of ``Param`` / ``Switch`` / ``Apply`` nodes plus
plain dict/list/tuple containers, flattened once into a ``ParamTable``: one row
per label with its distribution and its parent condition (the information
``pyll_utils.expr_to_config`` extracts, pyll_utils.py:144-225).
"""
import operator

import numpy as np

from .exceptions import DuplicateLabel

# prior distributions and their positional arguments (pyll/stochastic.py:30-142)
POSITIONAL = {
    'uniform': ('low', 'high'),
    'quniform': ('low', 'high', 'q'),
    'loguniform': ('low', 'high'),
    'qloguniform': ('low', 'high', 'q'),
    'normal': ('mu', 'sigma'),
    'qnormal': ('mu', 'sigma', 'q'),
    'lognormal': ('mu', 'sigma'),
    'qlognormal': ('mu', 'sigma', 'q'),
    'randint': ('upper',),
    'categorical': ('p', 'upper'),
}
CATEGORICAL = ('randint', 'categorical')


class Node(object):
    """Base of every deferred search-space expression."""

    def _ap(self, fn, *args):
        return Apply(fn, (self,) + args)

    def __add__(self, o): return Apply(operator.add, (self, o))
    def __radd__(self, o): return Apply(operator.add, (o, self))
    def __sub__(self, o): return Apply(operator.sub, (self, o))
    def __rsub__(self, o): return Apply(operator.sub, (o, self))
    def __mul__(self, o): return Apply(operator.mul, (self, o))
    def __rmul__(self, o): return Apply(operator.mul, (o, self))
    def __truediv__(self, o): return Apply(operator.truediv, (self, o))
    def __rtruediv__(self, o): return Apply(operator.truediv, (o, self))
    def __floordiv__(self, o): return Apply(operator.floordiv, (self, o))
    def __pow__(self, o): return Apply(operator.pow, (self, o))
    def __rpow__(self, o): return Apply(operator.pow, (o, self))
    def __neg__(self): return Apply(operator.neg, (self,))
    def __getitem__(self, i): return Apply(operator.getitem, (self, i))


class Param(Node):
    """A labelled random variable (``hyperopt_param(label, dist(...))``)."""

    def __init__(self, label, dist, args, as_float):
        if not isinstance(label, str):
            raise TypeError('require string label')
        self.label, self.dist, self.args, self.as_float = label, dist, dict(args), as_float

    def __repr__(self):
        return 'Param(%r, %s, %r)' % (self.label, self.dist, self.args)


class Switch(Node):
    """``switch(index_param, *options)`` — only the chosen option is evaluated."""

    def __init__(self, param, options):
        self.param, self.options = param, list(options)


class Apply(Node):
    """A deterministic function of sub-expressions, evaluated with the config."""

    def __init__(self, fn, args, kwargs=None):
        self.fn, self.args, self.kwargs = fn, tuple(args), dict(kwargs or {})


class Literal(Node):
    def __init__(self, value):
        self.value = value


class _Scope(object):
    """Minimal ``pyll.scope`` for deferred expressions in a space."""

    def __getattr__(self, name):
        import builtins
        import math
        fn = {'int': int, 'float': float, 'exp': np.exp, 'log': np.log, 'sqrt': np.sqrt,
              'minimum': np.minimum, 'maximum': np.maximum, 'max': max, 'min': min,
              'len': len, 'abs': abs, 'sin': math.sin, 'cos': math.cos, 'round': round,
              'str': str, 'dict': dict, 'list': list, 'tuple': tuple}.get(name)
        if fn is None:
            fn = getattr(builtins, name, None)
        if fn is None:
            raise AttributeError(name)
        return lambda *a, **k: Apply(fn, a, k)

    def switch(self, index, *options):
        if not isinstance(index, Param):
            raise TypeError('switch index must be a hp parameter')
        return Switch(index, options)


scope = _Scope()


# ---------------------------------------------------------------- flatten
class ParamRow(object):
    """One hyperparameter of a flattened space.

    parents: list of (parent_label, option_index); None entry = unconditional."""
    __slots__ = ('label', 'dist', 'args', 'parents', 'index', 'depth', 'node')

    def __init__(self, node, parent):
        self.label, self.dist, self.args = node.label, node.dist, node.args
        self.parents = [parent]
        self.node = node
        self.index = -1
        self.depth = 0

    @property
    def categorical(self):
        return self.dist in CATEGORICAL


class ParamTable(object):
    """Flat table of a space's hyperparameters.

    rows are sorted by label; ``index`` is the position in that order (the
    Philox counter word of the label); ``depth`` = tree level (roots 0)."""

    def __init__(self, space):
        self.space = space
        rows = {}

        def walk(node, parent):
            if isinstance(node, Param):
                add(node, parent)
            elif isinstance(node, Switch):
                add(node.param, parent)
                for i, opt in enumerate(node.options):
                    walk(opt, (node.param.label, i))
            elif isinstance(node, Apply):
                for a in node.args:
                    walk(a, parent)
                for a in node.kwargs.values():
                    walk(a, parent)
            elif isinstance(node, dict):
                for k in sorted(node, key=str):
                    walk(node[k], parent)
            elif isinstance(node, (list, tuple)):
                for v in node:
                    walk(v, parent)

        def add(node, parent):
            row = rows.get(node.label)
            if row is None:
                rows[node.label] = ParamRow(node, parent)
            elif row.node is not node:
                raise DuplicateLabel(node.label)
            elif parent not in row.parents:
                row.parents.append(parent)

        walk(space, None)
        for row in rows.values():
            if None in row.parents:
                row.parents = [None]
        self.labels = sorted(rows)
        self.rows = [rows[k] for k in self.labels]
        self.by_label = rows
        for i, r in enumerate(self.rows):
            r.index = i

        def depth(r, seen=()):
            if r.parents == [None]:
                return 0
            if r.label in seen:
                raise ValueError('cyclic conditional structure at %r' % r.label)
            return 1 + max(depth(rows[p[0]], seen + (r.label,)) for p in r.parents)
        for r in self.rows:
            r.depth = depth(r)
        self.n_levels = 1 + max((r.depth for r in self.rows), default=-1)
        # labels that gate other labels (switch index parameters)
        self.parent_labels = frozenset(p[0] for r in self.rows for p in r.parents if p is not None)

    def __len__(self):
        return len(self.rows)

    def levels(self):
        """Rows grouped by tree depth (computed once; the table is immutable)."""
        out = self.__dict__.get('_levels')
        if out is None:
            out = [[] for _ in range(self.n_levels)]
            for r in self.rows:
                out[r.depth].append(r)
            self._levels = out
        return [list(level) for level in out]

    def level_order(self):
        """Labels level by level (the key order of a choices dict)."""
        order = self.__dict__.get('_level_order')
        if order is None:
            order = self._level_order = [r.label for level in self.levels() for r in level]
        return order

    def rng_order(self):
        """Order in which the reference's shared RandomState is consumed:
        labels visited in descending order (rec_eval pops the sorted vals-dict
        inputs LIFO, pyll/base.py:179-190, 794-797), ancestors first.  Static
        per table: computed once (an iterative walk — a recursive closure is a
        reference cycle, garbage for the collector on every call)."""
        order = self.__dict__.get('_rng_order')
        if order is not None:
            return order
        order, seen = [], set()
        for r0 in reversed(self.rows):
            stack = [(r0, False)]
            while stack:
                r, expanded = stack.pop()
                if r.label in seen:
                    continue
                if expanded:
                    seen.add(r.label)
                    order.append(r)
                    continue
                stack.append((r, True))
                # (the parents visited first, in their listed order)
                for p in reversed(r.parents):
                    if p is not None and p[0] not in seen:
                        stack.append((self.by_label[p[0]], False))
        self._rng_order = order
        return order

    def active(self, row, chosen):
        """Is ``row`` active given chosen values {label: value or None}?"""
        for p in row.parents:
            if p is None:
                return True
            v = chosen.get(p[0])
            if v is not None and int(v) == p[1]:
                return True
        return False


# --------------------------------------------------------------- evaluate
class _Missing(object):
    pass


def evaluate(node, config):
    """Evaluate a space with ``config`` {label: value} (base.py:566-613 with
    rec_eval's lazy switch, pyll/base.py:762-781)."""
    if isinstance(node, Param):
        v = config.get(node.label, _Missing)
        if v is _Missing:
            raise KeyError('config has no value for active parameter %r' % node.label)
        return float(v) if node.as_float else v
    if isinstance(node, Switch):
        i = evaluate(node.param, config)
        try:
            ii = int(i)
        except Exception:
            raise TypeError('switch argument was', i)
        if ii != i or ii < 0:
            raise ValueError('switch pos must be positive int', i)
        return evaluate(node.options[ii], config)
    if isinstance(node, Apply):
        return node.fn(*[evaluate(a, config) for a in node.args],
                       **{k: evaluate(v, config) for k, v in node.kwargs.items()})
    if isinstance(node, Literal):
        return node.value
    if isinstance(node, dict):
        return {k: evaluate(v, config) for k, v in node.items()}
    if isinstance(node, list):
        return [evaluate(v, config) for v in node]
    if isinstance(node, tuple):
        return tuple(evaluate(v, config) for v in node)
    return node
