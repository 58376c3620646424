"""Structure-of-arrays view of a Trials history, cached incrementally.

Replaces the per-call document walk of the reference — the best-doc-per-tid
loop of tpe.py:820-842 and ``miscs_to_idxs_vals`` (base.py:108-123) — with a
cache attached to the ``Trials`` object.  The cache is
derivable state: it is rebuilt whenever the document list stops being an
extension of what it saw, it is never pickled, and losses of documents that
were not yet final are re-read on every call, so ``Trials`` stays the only
source of truth (resume via pickled Trials keeps working).

Fast path requirements (else the generic reference-order walk is used):
documents in increasing tid order, unique tids, no ``misc['from_tid']``,
and ``Domain.loss`` not overridden.

Staleness: a ``Trials`` stores the caller's documents as they are; the ones
built by this package (suggestions, Domain results) are tracked dicts
(base._Doc) whose in-place edits, at any depth, land in ``Trials._mutated``.
A view edit, or a refresh that changes the view other than by appends, moves
``Trials._view_gen``.  The cache rebuilds when a completed document it has
consumed appears in the mutation log or the view generation moved.  Pending
documents (values and loss) and *watched* documents — plain dicts, or tracked
ones holding a container of the caller's (base.watched) — are re-read on every
call and compared with what the cache consumed.  So every edit the
reference's per-call walk would see (tpe.py:820-842) is seen here, with a
pass over the watched documents only.
"""
import bisect
import ctypes
import itertools
import math
import weakref

import numpy as np

from . import base

try:                                   # (optional until built: python -m hyperopt_amd.build)
    from ._hostaddr import insert_sorted as _insert_sorted, obs_append as _obs_append
except ImportError:                    # pragma: no cover
    _insert_sorted = _obs_append = None
_I64, _F64 = np.dtype(np.int64), np.dtype(np.float64)

_CACHES = weakref.WeakKeyDictionary()


class DenseLayout(object):
    """The labels of a dense history (DenseObs) and their matrix rows, kept
    across the histories of one growing matrix (memos of row indices live here)."""
    __slots__ = ('labels', 'rows', 'memo')

    def __init__(self, labels):
        self.labels = list(labels)
        self.rows = {k: i for i, k in enumerate(self.labels)}
        self.memo = {}

    def row_index(self, labels):
        """Row indices (int64) of ``labels`` (memoised by the list object: pass
        the same list to hit)."""
        m = self.memo.get(id(labels))
        if m is None or m[0] is not labels:
            m = self.memo[id(labels)] = (labels, np.array([self.rows[k] for k in labels], dtype=np.int64))
        return m[1]


class DenseObs(object):
    """Observations of a flat space whose labels are all observed in every
    trial (a columnar caller's history, config 5): one float64 row per label of
    a C-contiguous matrix [labels x capacity], the first n values in tid order,
    and the trials' tids shared by every label.  A mapping label -> (tids,
    values) like History.obs (views made on access), which tpe._tree_labels
    reads as the matrix itself — no per-label Python for a thousand labels."""
    __slots__ = ('layout', 'matrix', 'tids', 'n')

    def __init__(self, layout, matrix, tids):
        assert matrix.dtype == np.float64 and matrix.flags.c_contiguous and matrix.shape[0] == len(layout.labels)
        assert matrix.shape[1] >= len(tids)
        self.layout, self.matrix, self.tids, self.n = layout, matrix, tids, len(tids)

    def __getitem__(self, label):
        return self.tids, self.matrix[self.layout.rows[label], :self.n]

    def get(self, label, default=None):
        i = self.layout.rows.get(label)
        return default if i is None else (self.tids, self.matrix[i, :self.n])

    def __contains__(self, label):
        return label in self.layout.rows

    def __iter__(self):
        return iter(self.layout.labels)

    def __len__(self):
        return len(self.layout.labels)

    def keys(self):
        return list(self.layout.labels)

    def items(self):
        return [(k, self[k]) for k in self.layout.labels]

    def values(self):
        return [self[k] for k in self.layout.labels]


class History(object):
    """tids (int64, ascending), losses (float64, +inf for missing), and per
    label the (tid, value) observations in tid order.  ``dev`` holds the
    device copies of the observation columns (devhist.DeviceColumns per
    device); it lives as long as the append-only source it mirrors."""
    __slots__ = ('tids', 'losses', 'obs', 'dev', 'sorted_obs', '_cache', '_orders', '_logs', 'tree_memo')

    def __init__(self, tids, losses, obs, dev=None, sorted_obs=True, cache=None):
        self.tids, self.losses, self.obs = tids, losses, obs
        self.dev = {} if dev is None else dev
        self.sorted_obs = sorted_obs     # every label's observation tids ascending
        self._cache = cache
        self._orders = None
        self._logs = None
        self.tree_memo = None          # tpe._tree_labels of this (immutable) view without a Trials cache

    def smallest(self, m):
        if self._cache is not None:
            return self._cache.smallest(m)
        return self._top_state().smallest(self.losses, m)

    def _top_state(self):
        """The incremental loss ranking of this History's append-only source
        (_TopState), kept in ``dev`` — the dict Histories over one append-only
        source share (a columnar FMinIter loop makes a History per suggest over
        growing views of the same buffers, bench.py config 5 --appending)."""
        st = self.dev.get('_top')
        if st is None:
            st = self.dev['_top'] = _TopState()
        return st

    def native_columns(self, label, log=False):
        """(tids, coordinate, value order) host addresses of a label's columns
        for the native fits — the cache's buffers, no per-call lookups — or
        None without a Trials cache.  Call after value_order(label)."""
        c = self._cache
        if c is None:
            return None
        if log:
            self.log_values(label)
            xa = c.logs[label].addr
        else:
            xa = c.obs_val[label].addr
        return c.obs_tid[label].addr, xa, c.order_addr(label)

    def coord_addr(self, label, key):
        """Address of coord_values(label, key, ...)'s array (valid right after
        that call; None without a Trials cache)."""
        c = self._cache
        if c is None:
            return None
        return c.logs[(key, label)].addr

    def cat_columns(self, label):
        """(tids, values) addresses of a categorical label (see native_columns)."""
        c = self._cache
        if c is None:
            return None
        return c.obs_tid[label].addr, c.obs_val[label].addr

    def log_values(self, label):
        """np.log of the label's observation values (the kernel coordinate of
        the log families) — extended incrementally by the Trials cache, else
        computed once per History."""
        if self._cache is not None:
            return self._cache.log_values(label)
        if self._logs is None:
            self._logs = {}
        v = self._logs.get(label)
        if v is None:
            v = self._logs[label] = np.log(np.asarray(self.obs[label][1], dtype=np.float64))
        return v

    def coord_values(self, label, key, fn):
        """fn(values) of a label's observations for an elementwise ``fn`` (a
        fit coordinate, parzen.fit_coord), memoised under ``key`` — extended
        incrementally by the Trials cache, else computed once per History."""
        if self._cache is not None:
            return self._cache.coord_values(label, key, fn)
        if self._logs is None:
            self._logs = {}
        v = self._logs.get((key, label))
        if v is None:
            v = self._logs[(key, label)] = np.ascontiguousarray(fn(self.obs[label][1]), dtype=np.float64)
        return v

    def value_order(self, label):
        """A permutation sorting the label's (float) observation values
        ascending — kept incrementally by the Trials cache, else computed once
        per History; None when a value is NaN."""
        if self._cache is not None:
            return self._cache.value_order(label)
        # no Trials cache (columnar callers): one stable argsort per label and History
        if self._orders is None:
            self._orders = {}
        perm = self._orders.get(label)
        if perm is None:
            vals = self.obs[label][1]
            if vals.dtype.kind != 'f':
                return None
            perm = np.argsort(vals)          # any sorting permutation (ties: see fit_split)
            if len(perm) and np.isnan(vals[perm[-1]]):
                perm = False
            self._orders[label] = perm
        return None if perm is False else perm

    def __len__(self):
        return len(self.tids)


class _Grow(object):
    """Append-only column; ``addr`` = host address of its buffer (kept with
    the buffer, so native calls need no per-call pointer lookup)."""
    __slots__ = ('a', 'n', 'addr')

    def __init__(self, dtype):
        self.a = np.empty(64, dtype=dtype)
        self.n = 0
        self.addr = self.a.ctypes.data

    def append(self, v):
        if self.n == self.a.shape[0]:
            self.a = np.concatenate([self.a, np.empty_like(self.a)])
            self.addr = self.a.ctypes.data
        self.a[self.n] = v
        self.n += 1

    def view(self):
        return self.a[:self.n]

    def reserve(self, cap):
        if cap > self.a.shape[0]:
            a = np.empty(cap, dtype=self.a.dtype)
            a[:self.n] = self.a[:self.n]
            self.a, self.addr = a, a.ctypes.data

    @classmethod
    def of(cls, arr):
        """A column holding ``arr`` (with room to grow)."""
        g = cls(arr.dtype)
        g.reserve(max(64, 2 * len(arr)))
        g.a[:len(arr)] = arr
        g.n = len(arr)
        return g


class _Cache(object):
    def __init__(self, labels, categorical, gen=0):
        self.gen = gen                 # Trials._view_gen the cache was built against
        self.docs = []                 # document objects in list order
        self.pos = {}                  # id(document) -> its position in docs
        self.tids = _Grow(np.int64)
        self.losses = _Grow(np.float64)
        self.pending = []              # positions whose loss may still change
        self.pending_vals = {}         # position -> (misc['vals'] object, its values) of a pending document
        self.watch = []                # (document, snapshot) of the completed watched documents
        self.watch_res = []            # result dicts of the completed loss-watched documents ...
        self.watch_loss = []           # ... and the losses read from them
        self.obs_tid = {k: _Grow(np.int64) for k in labels}     # tid of each observation (append-only)
        self.obs_val = {k: _Grow(np.int64 if categorical[k] else np.float64) for k in labels}
        self.labels = labels
        self._cols = ([self.obs_tid[k] for k in labels], [self.obs_val[k] for k in labels])     # (label order)
        self.ok = True                 # fast path still valid
        self.dev = {}                  # device mirrors of the (append-only) columns
        self.orders = {}               # label -> _Grow: value-sorting permutation of its observations
        self.sorted_vals = {}          # label -> its values in that order
        self.order_ok = {}             # label -> the permutation, or None when a value is NaN
        self.logs = {}                 # label -> _Grow of np.log of its observation values
        self.top = None                # positions of the smallest losses, sorted by (loss, position)
        self.top_n = 0                 # documents merged into `top`
        self.top_pos = []              # the same as lists (top is True: only the lists are current)
        self.top_keys = []             # ... and their losses
        self.hist = None               # History view of the current documents (no pending losses)
        self.below_memo = None         # (top_n, n_below, below tids) of split_below
        self.changed = set(labels)     # labels whose column views are stale (obs_views)
        self._views = dict.fromkeys(labels)     # (label order)

    def extend(self, docs, start, log):
        tids, losses, obs_tid, obs_val, changed = self.tids, self.losses, self.obs_tid, self.obs_val, self.changed
        last = int(tids.a[tids.n - 1]) if tids.n else None
        for i in range(start, len(docs)):
            d = docs[i]
            misc = d['misc']
            if 'from_tid' in misc:
                self.ok = False
                return
            tid = d['tid']
            if last is not None and tid <= last:
                self.ok = False
                return
            last = int(tid)
            self.pos[id(d)] = len(self.docs)
            self.docs.append(d)
            tids.append(tid)
            loss = d['result'].get('loss')
            final = d['state'] == base.JOB_STATE_DONE and loss is not None
            losses.append(np.inf if loss is None else float(loss))
            vals = misc['vals']
            if not final:
                self.pending.append(tids.n - 1)
                self.pending_vals[tids.n - 1] = (vals, self._snap(vals))
            else:
                self._watch(d, log)
            # (the loop below in C for the dicts it reads as they read: from the
            # label it hands back, a column to grow, on in Python)
            j = _obs_append(self.labels, vals, tid, *self._cols, changed) \
                if _obs_append is not None and (type(vals) is dict or type(vals) is base._Part) else 0
            if j < 0:
                continue
            for k in self.labels[j:]:
                v = vals.get(k)
                if v:
                    obs_tid[k].append(tid)
                    obs_val[k].append(v[0])
                    changed.add(k)

    def obs_views(self):
        """{label: (tids, values)} views of the columns; only the labels that
        gained observations since the last call get new views (a new dict per
        call: a History keeps the one it was given)."""
        ov = self._views
        for k in self.changed:
            ov[k] = (self.obs_tid[k].view(), self.obs_val[k].view())
        self.changed.clear()
        return dict(ov)

    def _snap(self, vals):
        return tuple(tuple(vals.get(k) or ()) for k in self.labels)

    def doc_snap(self, d):
        """What the cache reads of a document (tid, state, loss, from_tid,
        values; tuple equality: identical objects compare equal, NaN too)."""
        misc = d['misc']
        return (d['tid'], d['state'], d['result'].get('loss'), 'from_tid' in misc, self._snap(misc['vals']))

    def _watch(self, d, log):
        w = base.watched(d, log)
        if w == 1:
            r = d['result']
            self.watch_res.append(r)
            self.watch_loss.append(r.get('loss'))
        elif w:
            self.watch.append((d, self.doc_snap(d)))

    def watch_changed(self):
        """A watched document no longer reads as it did when consumed."""
        if self.watch_res and list(map(dict.get, self.watch_res, itertools.repeat('loss'))) != self.watch_loss:
            return True
        snap = self.doc_snap
        for d, s in self.watch:
            if snap(d) != s:
                return True
        return False

    def pending_vals_changed(self):
        """A pending document's values were edited or replaced (a running
        trial's document is still written to; the reference re-reads every
        document, tpe.py:820-842)."""
        for i in self.pending:
            vals, snap = self.pending_vals[i]
            cur = self.docs[i]['misc']['vals']
            if cur is not vals or self._snap(cur) != snap:
                return True
        return False

    def log_values(self, k):
        """np.log(obs_val[k]), the values appended since the last call logged
        and appended (elementwise, so equal to one np.log of the column)."""
        vals = self.obs_val[k].view()
        n = len(vals)
        g = self.logs.get(k)
        if g is None or g.n > n:
            g = self.logs[k] = _Grow(np.float64)
        if g.n < n:
            if g.a.shape[0] < n:
                a = np.empty(max(n, 2 * g.a.shape[0]), dtype=np.float64)
                a[:g.n] = g.a[:g.n]
                g.a = a
                g.addr = a.ctypes.data
            g.a[g.n:n] = np.log(vals[g.n:n])
            g.n = n
        return g.view()

    def coord_values(self, k, key, fn):
        """fn(obs_val[k]) for an elementwise fn, the values appended since the
        last call transformed and appended (equal to fn of the column)."""
        vals = self.obs_val[k].view()
        n = len(vals)
        g = self.logs.get((key, k))
        if g is None or g.n > n:
            g = self.logs[(key, k)] = _Grow(np.float64)
        if g.n < n:
            if g.a.shape[0] < n:
                a = np.empty(max(n, 2 * g.a.shape[0]), dtype=np.float64)
                a[:g.n] = g.a[:g.n]
                g.a = a
                g.addr = a.ctypes.data
            g.a[g.n:n] = fn(vals[g.n:n])
            g.n = n
        return g.view()

    def order_addr(self, k):
        """Address of value_order(k)'s array (valid right after that call)."""
        return self.orders[k].addr

    def value_order(self, k):
        """Sorting permutation of obs_val[k], extended by a merge of the
        observations appended since the last call (O(n) per suggest instead of
        a sort).  Any sort of a column without repeated values is the one
        np.argsort gives; the fit checks each side for repeats itself.
        (One appended value — FMinIter's case — is inserted in place: the tail
        of the permutation and of the sorted values moves up one slot.)"""
        g = self.obs_val[k]
        n = g.n
        pg = self.orders.get(k)
        if pg is not None and pg.n == n:
            return self.order_ok[k]
        vals = g.view()
        sg = self.sorted_vals.get(k)
        if pg is not None and n - pg.n == 1 and pg.n > 0:
            m = pg.n
            v = vals[m]
            for q in (pg, sg):
                if q.n == q.a.shape[0]:
                    q.reserve(2 * q.n)
            if _insert_sorted is not None and pg.a.dtype == _I64 and sg.a.dtype == _F64:
                _insert_sorted(pg.a, sg.a, m, float(v), m)    # (_hostaddr: the same search and moves)
            else:
                at = int(sg.view().searchsorted(v, side='right'))
                for q, x in ((pg, m), (sg, v)):
                    w = q.a.itemsize
                    ctypes.memmove(q.addr + (at + 1) * w, q.addr + at * w, (m - at) * w)
                    q.a[at] = x
            pg.n = sg.n = m + 1
        else:
            if pg is None:
                perm = np.argsort(vals)
                sv = vals[perm]
            else:
                # (the sorted values are kept beside the permutation: the insertion
                # points are a binary search, not a gather of the whole column)
                m = pg.n
                nv = vals[m:]
                o = np.argsort(nv, kind='stable')
                at = np.searchsorted(sg.view(), nv[o], side='right')
                perm = np.insert(pg.view(), at, o + m)
                sv = np.insert(sg.view(), at, nv[o])
            pg = self.orders[k] = _Grow.of(perm)
            sg = self.sorted_vals[k] = _Grow.of(sv)
        perm = pg.view()
        ok = self.order_ok[k] = None if n and sg.a[n - 1] != sg.a[n - 1] else perm     # NaN sorts last
        return ok

    TOP = 64

    def smallest(self, m):
        """Positions of the m smallest losses ordered by (loss, position), kept
        by merging the documents appended since the last call; None when a
        loss may still change (pending documents) or is NaN, or m is too large."""
        n = self.losses.n
        if self.pending or m > self.TOP:
            return None
        L = self.losses.view()
        if self.top is None or self.top_n > n:
            self.top, self.top_n = np.zeros(0, dtype=np.int64), 0
        if 0 < n - self.top_n <= 8 and self.top_n:
            # a few appended documents (FMinIter: one per suggest): merged into the
            # (loss, position) order one at a time — a new position follows every
            # kept one, so it goes after equal losses (bisect_right)
            keys, pos = self.top_keys, self.top_pos
            for p in range(self.top_n, n):
                v = float(L[p])
                if v != v:
                    self.top = self.below_memo = None
                    return None
                if len(pos) == self.TOP and v >= keys[-1]:
                    continue
                j = bisect.bisect_right(keys, v)
                keys.insert(j, v)
                pos.insert(j, p)
                if len(pos) > self.TOP:
                    keys.pop()
                    pos.pop()
            self.top_n = n
            self.top = True
            return pos[:m]
        if self.top_n < n:
            if self.top is True:
                self.top = np.asarray(self.top_pos, dtype=np.int64)
            new = np.arange(self.top_n, n, dtype=np.int64)
            if np.isnan(L[new]).any():
                self.top = self.below_memo = None
                return None
            if len(new) > 4 * self.TOP:      # (re)build: every loss <= the TOP-th smallest
                kth = np.partition(L[new], self.TOP - 1)[self.TOP - 1]
                new = new[L[new] <= kth]
            cand = np.concatenate([self.top, new])
            o = np.lexsort((cand, L[cand]))[:self.TOP]
            self.top, self.top_n = cand[o], n
            self.top_pos = self.top.tolist()
            self.top_keys = L[self.top].tolist()
        return self.top_pos[:m] if self.top is True else self.top[:m]

    def refresh_pending(self, log):
        if not self.pending:
            return
        self.top = self.below_memo = None     # pending losses may change: rebuild the ranking
        keep = []
        L = self.losses.a
        for i in self.pending:
            d = self.docs[i]
            loss = d['result'].get('loss')
            L[i] = np.inf if loss is None else float(loss)
            if not (d['state'] == base.JOB_STATE_DONE and loss is not None):
                keep.append(i)
            else:
                self.pending_vals.pop(i, None)
                self._watch(d, log)
        self.pending = keep


def _generic(domain, docs, table):
    """Reference-order walk (tpe.py:820-842 + base.py:108-123)."""
    best_loss, best_doc = {}, {}
    for doc in docs:
        tid = doc['misc'].get('from_tid', doc['tid'])
        loss = domain.loss(doc['result'], doc['spec'])
        loss = float('inf') if loss is None else float(loss)
        best_loss.setdefault(tid, loss)
        if loss <= best_loss[tid]:
            best_loss[tid] = loss
            best_doc[tid] = doc
    tids = sorted(best_doc)
    losses = np.array([best_loss[t] for t in tids], dtype=np.float64)
    obs = {}
    for r in table.rows:
        ot, ov = [], []
        for t in tids:
            misc = best_doc[t]['misc']
            v = misc['vals'][r.label]
            i = misc['idxs'][r.label]
            assert len(i) == len(v) and (i == [] or i == [misc['tid']])
            if v:
                ot.append(i[0])
                ov.append(v[0])
        obs[r.label] = (np.array(ot, dtype=np.int64),
                        np.array(ov, dtype=np.int64 if r.categorical else np.float64))
    srt = all(len(o[0]) < 2 or bool(np.all(np.diff(o[0]) > 0)) for o in obs.values())
    return History(np.array(tids, dtype=np.int64), losses, obs, sorted_obs=srt)


def extract(domain, trials):
    """History of ``trials`` for ``domain``'s parameters."""
    docs = trials.trials
    table = domain.table
    if type(domain).loss is not base.Domain.loss:
        return _generic(domain, docs, table)
    cache = _CACHES.get(trials)
    labels = table.labels
    gen = getattr(trials, '_view_gen', 0)
    if cache is not None and (cache.labels != labels or not cache.ok or cache.gen != gen):
        cache = None
    log = getattr(trials, '_mutated', None)
    if cache is not None:
        # the cache follows an append-only view (FMinIter's use).  A refresh or
        # view edit that drops, replaces or reorders documents moves
        # Trials._view_gen (above); an in-place edit of a completed tracked
        # document the cache has consumed is in the Trials' mutation log; a
        # pending document is re-read in full (its values and, below, its
        # loss), a watched one compared with what was consumed.
        if len(cache.docs) > len(docs) or cache.pending_vals_changed() or cache.watch_changed():
            cache = None
        elif log:
            pos, pend = cache.pos, set(cache.pending)
            for k, doc in log.items():
                p = pos.get(k)
                if p is not None and p not in pend and cache.docs[p] is doc:
                    cache = None
                    break
    if log:
        log.clear()
    if cache is None:
        cache = _Cache(labels, {r.label: r.categorical for r in table.rows}, gen)
        start = 0
    else:
        start = len(cache.docs)
        if start == len(docs) and not cache.pending and cache.hist is not None:
            return cache.hist             # nothing appended, no loss can change: the same view
    cache.extend(docs, start, log)
    if not cache.ok:
        _CACHES.pop(trials, None)
        return _generic(domain, docs, table)
    _CACHES[trials] = cache
    cache.refresh_pending(log)
    tids = cache.tids.view()
    hist = History(tids, cache.losses.view(), cache.obs_views(), dev=cache.dev, cache=cache)
    cache.hist = hist if not cache.pending else None
    return hist


def _smallest_plain(losses, m, stride=64):
    """Positions of the m smallest losses ordered by (loss, position) — NaN
    never among them, as np.argsort puts it last — without an O(N) selection:
    the m-th smallest of a strided sample is at least the m-th smallest of all,
    so every loss up to it (about m * stride of them, ties included) holds the
    m smallest, and a stable sort of those orders them.  None for short
    histories or when the sample cannot bound them (NaN)."""
    n = len(losses)
    if m <= 0 or n < 2 * stride * m:
        return None
    t = np.partition(losses[::stride], m - 1)[m - 1]
    if not t == t:
        return None
    cand = np.flatnonzero(losses <= t)
    lc = losses[cand]
    if len(cand) > 4 * m:                  # (ties at the m-th value all kept, then the stable sort)
        keep = lc <= lc[np.argpartition(lc, m - 1)[m - 1]]
        cand, lc = cand[keep], lc[keep]
    return cand[np.argsort(lc, kind='stable')[:m]]


class _TopState(object):
    """The m smallest losses of an append-only loss buffer, ordered by (loss,
    position), kept across suggests: one appended loss (FMinIter: a suggest
    follows every evaluation) is merged in by one bisection instead of a pass
    over all N (the reference's argsort over every loss, tpe.py:625-629 — the
    same positions).  Rebuilt when the buffer (its data address) changes, when
    it is shorter than before, or when more than 8 losses were appended; a
    History is an immutable view of its source (its value orders and tree
    records are memoised on it too), so the prefix seen so far is not re-read.
    ``below``: the split_below result for (n, n_below) of the current ranking."""
    __slots__ = ('addr', 'n', 'pos', 'keys', 'below')
    TOP = 64

    def __init__(self):
        self.addr, self.n, self.pos, self.keys, self.below = None, 0, None, None, None

    def smallest(self, L, m):
        n = len(L)
        if m > self.TOP:
            return _smallest_plain(L, m)
        addr = L.__array_interface__['data'][0] if n else None
        if self.addr is None or self.addr != addr or n < self.n or n - self.n > 8:
            top = _smallest_plain(L, self.TOP)
            if top is None:
                top = np.argsort(L, kind='stable')[:self.TOP]
            self.pos, self.keys, self.n, self.below = top.tolist(), L[top].tolist(), n, None
            # (a NaN ranks last, as in np.argsort: kept out of the incremental order)
            self.addr = addr if all(k == k for k in self.keys) else None
            return self.pos[:m]
        if n > self.n:
            keys, pos = self.keys, self.pos
            for p in range(self.n, n):
                v = float(L[p])
                if v != v:
                    self.addr = None              # (rebuilt next time)
                    return _smallest_plain(L, m) if n >= 2 * 64 * m else np.argsort(L, kind='stable')[:m]
                if len(pos) == self.TOP and v >= keys[-1]:
                    continue
                j = bisect.bisect_right(keys, v)  # (a new position follows every kept one)
                keys.insert(j, v)
                pos.insert(j, p)
                if len(pos) > self.TOP:
                    keys.pop()
                    pos.pop()
            self.n, self.below = n, None
        return self.pos[:m]


class BelowTids(np.ndarray):
    """Below-set tids in the reference's order with their ascending copy
    (``sorted_view``) made once — the native tree call takes them sorted."""

    @classmethod
    def of(cls, tids):
        b = tids.view(cls)
        b.sorted_view = np.sort(tids)
        b.positions = {}               # label -> (column length, History, below positions): tpe._below_positions
        return b

    def __array_finalize__(self, obj):
        self.sorted_view = None
        self.positions = None


def split_below(history, gamma, gamma_cap=25):
    """Tids of the ``n_below`` best losses (ap_filter_trials, tpe.py:625-629).

    The below set only depends on WHICH losses are smallest, so an O(N)
    ``np.argpartition`` gives it exactly unless the loss at the boundary is
    tied with one outside it; then the reference's ``np.argsort`` order (same
    numpy call on the same float64 array) decides, as in the reference."""
    losses = history.losses
    n = len(losses)
    n_below = min(int(math.ceil(gamma * math.sqrt(n))), gamma_cap)
    if n_below <= 0:
        return history.tids[:0]
    if n_below >= n:
        return history.tids.copy()
    c = history._cache
    if c is not None:
        memo = c.below_memo
        if memo is not None and memo[0] == c.top_n and memo[1] == n_below and c.top is not None and n == c.top_n:
            return memo[2]
    top = history.smallest(n_below + 1)
    st = history.dev.get('_top') if c is None else None
    if st is not None and st.below is not None and st.below[0] == (n, n_below) and st.addr is not None \
            and st.below[1] is history.tids:
        return st.below[2]
    if top is not None and len(top) == n_below + 1:
        keys = c.top_keys if c is not None and c.top is True else None
        if (keys[n_below - 1] != keys[n_below]) if keys is not None else \
                (losses[top[n_below - 1]] != losses[top[n_below]]):
            # the same set as below, without a pass over N (ascending: the
            # native call takes it sorted, BelowTids.sorted_view)
            b = BelowTids.of(history.tids[np.asarray(top[:n_below], dtype=np.int64)])
            if c is not None and c.top is not None:
                c.below_memo = (c.top_n, n_below, b)
            elif st is not None and st.addr is not None:
                st.below = ((n, n_below), history.tids, b)
            return b
    part = np.argpartition(losses, n_below - 1)
    kth = losses[part[n_below - 1]]
    rest = losses[part[n_below:]]
    if np.isnan(kth) or np.any(rest == kth) or np.isnan(losses).any():
        order = np.argsort(losses)
        return history.tids[order[:n_below]]
    return history.tids[part[:n_below]]


def below_index(obs_tids, below_tids, sorted_obs=True):
    """Ascending positions (int32) of the below observations among a label's
    observations (tpe.py:629-636: membership of the tid in the below set).
    With ascending ``obs_tids`` (History.sorted_obs) this is O(n_below log n)."""
    n = len(obs_tids)
    if len(below_tids) == 0 or n == 0:
        return np.zeros(0, dtype=np.int32)
    if not sorted_obs:
        return np.nonzero(np.isin(obs_tids, below_tids))[0].astype(np.int32)
    b = np.asarray(below_tids, dtype=np.int64)
    idx = np.searchsorted(obs_tids, b)
    ok = idx < n
    ok[ok] = obs_tids[idx[ok]] == b[ok]
    return np.sort(idx[ok]).astype(np.int32)


def below_mask(obs_tids, below_tids, sorted_obs=True):
    """Membership of each observation in the below set, in tid order
    (tpe.py:629-636)."""
    m = np.zeros(len(obs_tids), dtype=bool)
    m[below_index(obs_tids, below_tids, sorted_obs)] = True
    return m
