"""Device-resident observation columns (GPU Parzen fit).

The reference re-reads every observation of every hyperparameter from the
Trials documents on each suggest (tpe.py:820-842) and fits the above mixture
in numpy (tpe.py:398-475).  For large histories the engine instead keeps one
float64 column per hyperparameter in HBM, in tid order, and fits the above
mixture on the device (tpe_fit_above).  A column is append-only: each call
uploads only the observations it has not seen yet, so a 100k-trial history
costs its upload once, not per suggest — and so is the label's value order
(ValueOrder): each observation is sorted into it once.
"""
import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None


class ValueOrder(object):
    """Resident value order of one device-fitted label (include/tpe_hip.h,
    "Device value order"): the label's observations as (t, position) pairs
    sorted by t, where t is the kernel coordinate (x, or ln x for the log
    families).  Two float64/int32 buffer pairs: the current pair holds the
    order of the first ``n`` observations; a level run that sees more
    observations merges the new ones into the other pair (tpe_fit_above), and
    ``commit`` makes that pair current.  The reference re-sorts every
    suggest (tpe.py:427); this sorts each observation once."""
    __slots__ = ('device', 'keys', 'idx', 'cur', 'n', 'owner')

    def __init__(self, device, owner=None):
        self.device = device
        self.owner = owner            # the DeviceColumns whose version a change bumps
        self.keys = [None, None]
        self.idx = [None, None]
        self.cur = 0
        self.n = 0

    def _room(self, side, n):
        t = self.keys[side]
        if t is None or t.numel() < n:
            cap = max(n, 1024, 2 * (t.numel() if t is not None else 0))
            self.keys[side] = torch.empty(cap, dtype=torch.float64, device=self.device)
            self.idx[side] = torch.empty(cap, dtype=torch.int32, device=self.device)
            self._bump()

    def ptrs(self, n_obs):
        """(key_in, idx_in, n_in, key_out, idx_out) device addresses for a run
        that fits the label's first ``n_obs`` observations."""
        n_in = self.n if self.n <= n_obs else 0          # (a longer order is of another column)
        cur, nxt = self.cur, 1 - self.cur
        kin = self.keys[cur].data_ptr() if n_in else 0
        iin = self.idx[cur].data_ptr() if n_in else 0
        if n_in == n_obs:
            return kin, iin, n_in, 0, 0
        self._room(nxt, n_obs)
        return kin, iin, n_in, self.keys[nxt].data_ptr(), self.idx[nxt].data_ptr()

    def commit(self, n_obs):
        """A run with ``ptrs(n_obs)`` was enqueued: its output is the order."""
        if self.n != n_obs:
            self.cur, self.n = 1 - self.cur, n_obs
            self._bump()

    def _bump(self):
        if self.owner is not None:
            self.owner.version += 1

    def host(self):
        """(t, position) of the current order, copied to the host (tests)."""
        n = self.n
        if n == 0:
            return np.zeros(0), np.zeros(0, dtype=np.int64)
        return (self.keys[self.cur][:n].cpu().numpy(),
                self.idx[self.cur][:n].cpu().numpy().astype(np.int64) & 0xFFFFFFFF)


class DeviceColumns(object):
    """float64 device copies of a History's observation columns (one device),
    in the kernel coordinate (x, or np.log(x) for the log families), and the
    labels' resident value orders."""

    def __init__(self, device):
        self.device = device
        self.cols = {}                # label -> [tensor, n uploaded, ValueOrder]
        self.version = 0              # bumped whenever a column or an order moves (memos of their addresses)

    def column(self, label, values):
        """Device tensor whose first ``len(values)`` entries are ``values``
        (values must extend what earlier calls for this label passed)."""
        n = len(values)
        ent = self.cols.get(label)
        if ent is None or ent[1] > n:
            ent = self.cols[label] = [torch.empty(max(n, 1024), dtype=torch.float64, device=self.device), 0,
                                      ValueOrder(self.device, self)]
            self.version += 1
        t, m = ent[0], ent[1]
        if n > m:
            if n > t.numel():
                grown = torch.empty(max(n, 2 * t.numel()), dtype=torch.float64, device=self.device)
                grown[:m].copy_(t[:m])
                t = ent[0] = grown
            src = torch.from_numpy(np.ascontiguousarray(values[m:n], dtype=np.float64))
            t[m:n].copy_(src)
            ent[1] = n
            self.version += 1
        return t

    def order(self, label):
        """The label's ValueOrder (after ``column`` for that label)."""
        return self.cols[label][2]


def columns(hist, device):
    """The DeviceColumns of ``hist`` (a history.History) on ``device``."""
    key = str(device)
    dc = hist.dev.get(key)
    if dc is None:
        dc = hist.dev[key] = DeviceColumns(device)
    return dc
