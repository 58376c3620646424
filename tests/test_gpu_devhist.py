"""devhist's flat stores on the device: the appended observations go up by
tpe_scatter_f64 (one kernel reading pinned memory in place) and re-layouts
move every segment by tpe_move_ranges — no framework op on the data (VERDICT
round 5, next 6).  The same cases as tests/test_devhist.py's CPU ones."""
import numpy as np
import pytest
import torch

from tests.test_devhist import columns_case, orders_case

pytestmark = pytest.mark.gpu


def test_device_columns_scatter_and_relayout():
    columns_case(torch.device('cuda', 0))
    torch.cuda.synchronize()


def test_device_orders_relayout():
    orders_case(torch.device('cuda', 0))
    torch.cuda.synchronize()


def test_scatter_many_labels_one_launch():
    """A thousand labels' appended observation each (config 5's FMinIter step):
    every column equals the host values after each of 40 appends, across the
    re-layouts the growth forces."""
    from hyperopt_amd import devhist
    dc = devhist.DeviceColumns(torch.device('cuda', 0))
    rs = np.random.RandomState(3)
    L, N0 = 1000, 900
    m = rs.uniform(size=(L, N0 + 2000))
    labels = ['x%04d' % i for i in range(L)]
    rows = np.arange(L)
    for n in [N0] + list(range(N0 + 1, N0 + 41)) + [N0 + 2000]:     # (the last outgrows the room)
        dc.upload_rows(labels, m, rows, n)
    store = dc.store.cpu().numpy()
    for i in (0, 1, 499, 999):
        s = dc.slot[labels[i]]
        np.testing.assert_array_equal(store[dc.off[s]:dc.off[s] + N0 + 2000], m[i])
