"""Device-resident observation columns (GPU Parzen fit).

The reference re-reads every observation of every hyperparameter from the
Trials documents on each suggest (tpe.py:820-842) and fits the above mixture
in numpy (tpe.py:398-475).  For large histories the engine instead keeps one
float64 column per hyperparameter in HBM, in tid order, and fits the above
mixture on the device (tpe_fit_above).  A column is append-only: each call
uploads only the observations it has not seen yet, so a 100k-trial history
costs its upload once, not per suggest — and so is the label's value order
(ValueOrder): each observation is sorted into it once.

Every label's column is a segment of ONE flat device tensor per History (and
every label's value order a segment of two more), so a suggest that appends
an observation to a thousand labels uploads them with one scatter, and the
columns' and orders' addresses come out of numpy arrays (a thousand labels'
records are filled without a per-label device call).  Segments keep spare
room; one that outgrows it re-lays out the tensor (every segment doubles).
"""
import numpy as np

from . import _native as N

try:
    from . import _hostaddr               # (csrc/hostaddr.c, built with the library)
except ImportError:                       # pragma: no cover - before the build
    _hostaddr = None

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None


def _stream(device):
    """The device's current stream as a raw hipStream_t (the engine's stream:
    engine.Engine._stream)."""
    raw = getattr(torch._C, '_cuda_getCurrentRawStream', None)
    return raw(device.index or 0) if raw is not None else torch.cuda.current_stream(device).cuda_stream


class _Staging(object):
    """Pinned host memory the column kernels read in place (tpe_scatter_f64,
    tpe_move_ranges: system-scope loads through its device address), reused
    once the stream has passed the last launch that read it (its event)."""

    def __init__(self):
        self.pin = self.dev = self.ev = None

    def get(self, n_words):
        """(int64 host view of >= n_words words, its device address)."""
        if self.pin is None or self.pin.numel() < n_words:
            if self.ev is not None:
                self.ev.synchronize()               # (the old buffer goes back to torch's pinned pool)
            self.pin = torch.empty(max(int(n_words), 8192), dtype=torch.int64, pin_memory=True)
            import ctypes
            dp = ctypes.c_void_p()
            lib = N.load()
            N.check(lib.tpe_pinned_device_address(self.pin.data_ptr(), ctypes.byref(dp)), lib,
                    'tpe_pinned_device_address')
            if not dp.value:
                raise N.NativeUnavailable('pinned staging is not device-addressable')
            self.dev, self.ev = dp.value, None
        elif self.ev is not None:
            self.ev.synchronize()                   # (the last kernel reading it has run)
        return self.pin.numpy(), self.dev

    def used(self):
        # (one event, re-recorded after each launch that reads the buffer: an
        # Event object a launch cost ~10 us of Python)
        if self.ev is None:
            self.ev = torch.cuda.Event()
        self.ev.record()


def _move(device, staging, src, dst, src_off, dst_off, n, elem_bytes):
    """dst[dst_off[i] + j] = src[src_off[i] + j], j < n[i], on the device
    (tpe_move_ranges; src / dst distinct device tensors)."""
    keep = n > 0
    src_off, dst_off, n = src_off[keep], dst_off[keep], n[keep]
    if not len(n):
        return
    if device.type != 'cuda':                      # (CPU tensors: the tests of the bookkeeping)
        dst[torch.from_numpy(_positions(dst_off, n))] = src[torch.from_numpy(_positions(src_off, n))]
        return
    h, dev = staging.get(3 * len(n))
    h[0:3 * len(n):3], h[1:3 * len(n):3], h[2:3 * len(n):3] = src_off, dst_off, n
    lib = N.load()
    N.check(lib.tpe_move_ranges(dev, len(n), elem_bytes, src.data_ptr(), dst.data_ptr(), _stream(device)), lib,
            'tpe_move_ranges')
    staging.used()


def _room(n):
    """Segment capacity for n entries (room to append)."""
    return int(n + max(1024, n // 8))


def _positions(off, n):
    """Concatenated ranges [off[i], off[i] + n[i]) (int64)."""
    off = np.asarray(off, dtype=np.int64)
    n = np.asarray(n, dtype=np.int64)
    tot = int(n.sum())
    if tot == 0:
        return np.zeros(0, dtype=np.int64)
    start = np.repeat(off - np.concatenate([[0], np.cumsum(n)[:-1]]), n)
    return start + np.arange(tot, dtype=np.int64)


class _Orders(object):
    """The resident value orders of a DeviceColumns' labels: per slot a
    segment of two (t: float64, position: int32) buffer pairs — the current
    pair holds the order of the first ``n`` observations; a level run that sees
    more merges the new ones into the other pair (tpe_fit_above) and
    ``commit`` makes it current."""

    def __init__(self, device, owner):
        self.device, self.owner = device, owner
        self.keys = self.idx = None            # [2 x TC] float64 / int32
        self.tc = 0
        self.off = np.zeros(0, dtype=np.int64)
        self.cap = np.zeros(0, dtype=np.int64)
        self.cur = np.zeros(0, dtype=np.int64)
        self.n = np.zeros(0, dtype=np.int64)
        self.kbase = self.ibase = 0

    def add(self):
        self.off = np.append(self.off, 0)
        self.cap = np.append(self.cap, 0)
        self.cur = np.append(self.cur, 0)
        self.n = np.append(self.n, 0)
        return len(self.n) - 1

    def ensure(self, slots, n_obs):
        """Room for n_obs[i] entries in slot slots[i] (a re-layout moves every
        slot's current order; the owner's version moves)."""
        slots = np.asarray(slots, dtype=np.int64)
        n_obs = np.asarray(n_obs, dtype=np.int64)
        if self.keys is not None and not np.any(n_obs > self.cap[slots]):
            return
        cap = self.cap.copy()
        grow = np.zeros(len(cap), dtype=bool)
        grow[slots[n_obs > cap[slots]]] = True
        want = np.zeros(len(cap), dtype=np.int64)
        np.maximum.at(want, slots, n_obs)
        cap[grow] = np.maximum(np.array([_room(int(w)) for w in want[grow]], dtype=np.int64), 2 * cap[grow])
        off = np.concatenate([[0], np.cumsum(cap)[:-1]]).astype(np.int64)
        tc = int(cap.sum())
        keys = torch.empty(2 * max(tc, 1), dtype=torch.float64, device=self.device)
        idx = torch.empty(2 * max(tc, 1), dtype=torch.int32, device=self.device)
        if self.keys is not None and int(self.n.sum()):
            # every slot's current order into its new place (one range each)
            so, do = self.cur * self.tc + self.off, self.cur * tc + off
            _move(self.device, self.owner._staging, self.keys, keys, so, do, self.n, 8)
            _move(self.device, self.owner._staging, self.idx, idx, so, do, self.n, 4)
        self.keys, self.idx, self.tc, self.off, self.cap = keys, idx, tc, off, cap
        self.kbase, self.ibase = keys.data_ptr(), idx.data_ptr()
        self.owner.version += 1

    @staticmethod
    def _runs(on, n_obs):
        """(n_in, merged) of runs over n_obs observations given orders of on:
        the order's length when it is a prefix (a longer one is another
        column's: none), and whether the run merges into the other buffer pair
        — not when it is in delta mode (a few new observations read beside the
        order, include/tpe_hip.h TPE_FIT_DELTA_MAX)."""
        n_in = np.where(on <= n_obs, on, 0)
        new = n_obs - n_in
        return n_in, (new > 0) & ((n_in == 0) | (new > N.FIT_DELTA_MAX))

    def ptrs_many(self, slots, n_obs):
        """(key_in, idx_in, n_in, key_out, idx_out) device addresses, as int64
        arrays, for runs that fit slot slots[i]'s first n_obs[i] observations
        (key_out = 0: no merge)."""
        slots = np.asarray(slots, dtype=np.int64)
        n_obs = np.asarray(n_obs, dtype=np.int64)
        on = self.n[slots]
        n_in, out = self._runs(on, n_obs)
        if out.any():
            self.ensure(slots[out], n_obs[out])
        on, cur, off = self.n[slots], self.cur[slots], self.off[slots]
        has = n_in > 0
        kin = np.where(has, self.kbase + 8 * (cur * self.tc + off), 0)
        iin = np.where(has, self.ibase + 4 * (cur * self.tc + off), 0)
        kout = np.where(out, self.kbase + 8 * ((1 - cur) * self.tc + off), 0)
        iout = np.where(out, self.ibase + 4 * ((1 - cur) * self.tc + off), 0)
        return kin, iin, n_in, kout, iout

    def commit_many(self, slots, n_obs):
        """Runs with ``ptrs_many(slots, n_obs)`` were enqueued: the merged
        orders are now current (delta-mode runs left theirs as they were)."""
        slots = np.asarray(slots, dtype=np.int64)
        n_obs = np.asarray(n_obs, dtype=np.int64)
        mv = self._runs(self.n[slots], n_obs)[1]
        if mv.any():
            s = slots[mv]
            self.cur[s] = 1 - self.cur[s]
            self.n[s] = n_obs[mv]
            self.owner.version += 1


class ValueOrder(object):
    """Resident value order of one device-fitted label (include/tpe_hip.h,
    "Device value order"): the label's observations as (t, position) pairs
    sorted by t, where t is the kernel coordinate (x, or ln x for the log
    families) — a slot of its DeviceColumns' order buffers.  The reference
    re-sorts every suggest (tpe.py:427); this sorts each observation once."""
    __slots__ = ('group', 'slot')

    def __init__(self, group, slot):
        self.group, self.slot = group, slot

    @property
    def n(self):
        return int(self.group.n[self.slot])

    def ptrs(self, n_obs):
        """(key_in, idx_in, n_in, key_out, idx_out) device addresses for a run
        that fits the label's first ``n_obs`` observations."""
        return tuple(int(a[0]) for a in self.group.ptrs_many([self.slot], [n_obs]))

    def commit(self, n_obs):
        """A run with ``ptrs(n_obs)`` was enqueued: its output is the order."""
        self.group.commit_many([self.slot], [n_obs])

    def host(self):
        """(t, position) of the current order, copied to the host (tests)."""
        g, s = self.group, self.slot
        n = int(g.n[s])
        if n == 0:
            return np.zeros(0), np.zeros(0, dtype=np.int64)
        o = int(g.cur[s]) * g.tc + int(g.off[s])
        return g.keys[o:o + n].cpu().numpy(), g.idx[o:o + n].cpu().numpy().astype(np.int64) & 0xFFFFFFFF


class DeviceColumns(object):
    """float64 device copies of a History's observation columns (one device),
    in the kernel coordinate (x, or np.log(x) for the log families), and the
    labels' resident value orders: segments of flat device tensors, slot s of
    the column store and slot s of the order group belonging to one label."""

    def __init__(self, device):
        self.device = device
        self.version = 0              # bumped whenever a column or an order moves (memos of their addresses)
        self.store = None
        self.base = 0
        self.slot = {}                # label -> slot
        self.views = []               # slot -> the store's segment (a tensor view)
        self.off = np.zeros(0, dtype=np.int64)
        self.cap = np.zeros(0, dtype=np.int64)
        self.n = np.zeros(0, dtype=np.int64)        # values uploaded per slot
        self.orders = _Orders(device, self)
        self._last_labels, self._last_slots = None, None
        self._staging = _Staging()                    # (_scatter's and the re-layouts' pinned ranges)

    def _add(self, label):
        s = self.slot[label] = len(self.views)
        self.views.append(None)
        self.off = np.append(self.off, 0)
        self.cap = np.append(self.cap, 0)
        self.n = np.append(self.n, 0)
        assert self.orders.add() == s
        return s

    def _relayout(self, want):
        """Every slot to a segment of at least want[s] (doubling the grown ones),
        the uploaded values kept (one gather)."""
        cap = self.cap.copy()
        grow = want > cap
        cap[grow] = np.maximum(np.array([_room(int(w)) for w in want[grow]], dtype=np.int64), 2 * cap[grow])
        off = np.concatenate([[0], np.cumsum(cap)[:-1]]).astype(np.int64)
        store = torch.empty(max(int(cap.sum()), 1), dtype=torch.float64, device=self.device)
        if self.store is not None and int(self.n.sum()):
            _move(self.device, self._staging, self.store, store, self.off, off, self.n, 8)
        self.store, self.off, self.cap = store, off, cap
        self.base = store.data_ptr()
        self.views = [store[o:o + c] for o, c in zip(off.tolist(), cap.tolist())]
        self.version += 1

    def upload(self, labels, values, lengths=None, dense=None):
        """Make the column of labels[i] hold values[i] (a float64 array that
        extends what earlier calls for the label passed; a shorter one — another
        History's — starts the label over, its order too); the values not
        uploaded yet go up in one scatter (``lengths``: len(values[i]) when the
        caller has them).  Returns the labels' slots (int64)."""
        get = self.slot.get
        if labels is self._last_labels:          # (the caller's same list: its slots are known)
            slots = self._last_slots
        else:
            slots = np.fromiter((get(k, -1) for k in labels), dtype=np.int64, count=len(labels))
            if len(slots) and slots.min() < 0:
                for i in np.flatnonzero(slots < 0).tolist():
                    s = get(labels[i])
                    slots[i] = s if s is not None else self._add(labels[i])
            self._last_labels, self._last_slots = labels, slots
        if dense is not None:
            matrix, rows, n_dense = dense
            nv = np.full(len(labels), n_dense, dtype=np.int64)
        else:
            nv = np.fromiter(map(len, values), dtype=np.int64, count=len(values)) if lengths is None else lengths
        m = self.n[slots]
        short = m > nv
        if short.any():
            s = slots[short]
            self.n[s] = 0
            self.orders.n[s] = 0
            self.orders.cur[s] = 0
            m = self.n[slots]
        if self.store is None or np.any(nv > self.cap[slots]):
            want = np.zeros(len(self.cap), dtype=np.int64)
            np.maximum.at(want, slots, nv)
            self._relayout(want)
        up = np.flatnonzero(nv > m)
        if len(up) and dense is not None:
            m0 = int(m[up[0]])
            if len(up) == len(m) and bool((m == m0).all()):
                vals = matrix[rows, m0:n_dense].ravel()          # (row by row: _positions' order)
            else:
                vals = np.concatenate([matrix[rows[i], int(m[i]):n_dense] for i in up.tolist()])
        elif len(up):
            try:                                 # (float64 columns: their new values gathered natively)
                vals = _hostaddr.tails(values, m, nv)
            except (ValueError, AttributeError):
                ml, nl = m.tolist(), nv.tolist()
                vals = np.concatenate([values[i][ml[i]:nl[i]] for i in up.tolist()]).astype(np.float64, copy=False)
        if len(up):
            su = slots[up]
            pos = _positions(self.off[su] + m[up], nv[up] - m[up])
            self._scatter(pos, vals)
            self.n[su] = nv[up]
            self.version += 1
        return slots

    def upload_rows(self, labels, matrix, rows, n):
        """``upload`` for a dense history: the column of labels[i] holds
        matrix[rows[i], :n] (history.DenseObs) — the new values of every label
        gathered as one 2-D slice when they start at the same index (FMinIter's
        appends), else per label."""
        return self.upload(labels, (), dense=(matrix, rows, n))

    def _scatter(self, pos, vals):
        """store[pos] = vals: on a GPU one kernel (tpe_scatter_f64) reads the
        values and positions from a pinned staging buffer in place — no copy,
        no framework op; the buffer's reuse waits for that launch's event."""
        k = len(vals)
        if self.device.type != 'cuda':             # (CPU tensors: the tests of the bookkeeping)
            self.store[torch.from_numpy(pos)] = torch.from_numpy(vals)
            return
        h, dev = self._staging.get(2 * k)
        h[:k].view(np.float64)[:] = vals
        h[k:2 * k] = pos
        lib = N.load()
        N.check(lib.tpe_scatter_f64(dev, k, self.base, _stream(self.device)), lib, 'tpe_scatter_f64')
        self._staging.used()

    def columns(self, items):
        """Device tensors (store segments) whose first ``len(values)`` entries
        are ``values``, for every (label, values) of ``items`` (``upload``)."""
        slots = self.upload([k for k, _ in items], [v for _, v in items])
        return [self.views[s] for s in slots.tolist()]

    def column(self, label, values):
        """Device tensor whose first ``len(values)`` entries are ``values``
        (values must extend what earlier calls for this label passed)."""
        return self.columns([(label, values)])[0]

    def order(self, label):
        """The label's ValueOrder (after ``column`` for that label)."""
        return ValueOrder(self.orders, self.slot[label])

    def count(self, label):
        """Values of the label uploaded so far."""
        return int(self.n[self.slot[label]])

    def view(self, label):
        """The label's segment of the store."""
        return self.views[self.slot[label]]

    def addresses(self, slots):
        """Device addresses of the slots' columns (int64 array)."""
        return self.base + 8 * self.off[slots]


def columns(hist, device):
    """The DeviceColumns of ``hist`` (a history.History) on ``device``."""
    key = str(device)
    dc = hist.dev.get(key)
    if dc is None:
        dc = hist.dev[key] = DeviceColumns(device)
    return dc
