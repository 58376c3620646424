"""Device-resident observation columns (GPU Parzen fit).

The reference re-reads every observation of every hyperparameter from the
Trials documents on each suggest (tpe.py:820-842) and fits the above mixture
in numpy (tpe.py:398-475).  For large histories the engine instead keeps one
float64 column per hyperparameter in HBM, in tid order, and fits the above
mixture on the device (tpe_fit_above).  A column is append-only: each call
uploads only the observations it has not seen yet, so a 100k-trial history
costs its upload once, not per suggest.
"""
import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None


class DeviceColumns(object):
    """float64 device copies of a History's observation columns (one device)."""

    def __init__(self, device):
        self.device = device
        self.cols = {}                # label -> [tensor, n uploaded]

    def column(self, label, values):
        """Device tensor whose first ``len(values)`` entries are ``values``
        (values must extend what earlier calls for this label passed)."""
        n = len(values)
        ent = self.cols.get(label)
        if ent is None or ent[1] > n:
            ent = self.cols[label] = [torch.empty(max(n, 1024), dtype=torch.float64, device=self.device), 0]
        t, m = ent
        if n > m:
            if n > t.numel():
                grown = torch.empty(max(n, 2 * t.numel()), dtype=torch.float64, device=self.device)
                grown[:m].copy_(t[:m])
                t = ent[0] = grown
            src = torch.from_numpy(np.ascontiguousarray(values[m:n], dtype=np.float64))
            t[m:n].copy_(src)
            ent[1] = n
        return t


def columns(hist, device):
    """The DeviceColumns of ``hist`` (a history.History) on ``device``."""
    key = str(device)
    dc = hist.dev.get(key)
    if dc is None:
        dc = hist.dev[key] = DeviceColumns(device)
    return dc
