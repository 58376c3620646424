"""devhist's flat device stores, on CPU tensors (the layout logic only: the
device fit that reads and merges them is tests/test_gpu_configs.py's)."""
import numpy as np
import torch

from hyperopt_amd import devhist


def test_columns_append_grow_and_restart():
    columns_case(torch.device('cpu'))


def columns_case(device):
    """Labels appended to in one batch keep every uploaded value across
    re-layouts; a shorter column (another History's) starts its label over;
    the segment addresses are the views' addresses.  (tests/test_gpu_devhist.py
    runs it on the device: the scatter and re-layout kernels.)"""
    dc = devhist.DeviceColumns(device)
    rs = np.random.RandomState(0)
    full = {('l%d' % i): rs.uniform(size=6000) for i in range(5)}
    n = {k: 0 for k in full}
    for step in range(40):
        labels = [k for k in full if rs.uniform() < 0.7]
        for k in labels:
            n[k] = min(len(full[k]), n[k] + int(rs.randint(1, 400)))
        views = dc.columns([(k, full[k][:n[k]]) for k in labels])
        for k, v in zip(labels, views):
            np.testing.assert_array_equal(v[:n[k]].cpu().numpy(), full[k][:n[k]])
            assert dc.count(k) == n[k]
        if labels:
            assert dc.addresses([dc.slot[k] for k in labels]).tolist() == [v.data_ptr() for v in views]
        for k in full:                      # untouched labels survive re-layouts
            if k in dc.slot:
                np.testing.assert_array_equal(dc.view(k)[:dc.count(k)].cpu().numpy(), full[k][:dc.count(k)])
    short = rs.uniform(size=10)
    v = dc.column('l0', short)
    np.testing.assert_array_equal(v[:10].cpu().numpy(), short)
    assert dc.order('l0').n == 0


def test_orders_ensure_keeps_current_side():
    orders_case(torch.device('cpu'))


def orders_case(device):
    """Value orders: ptrs of a longer run point at the other side, commit
    flips it, and making room for one label moves every label's current order
    with its contents (what a level run reads next)."""
    dc = devhist.DeviceColumns(device)
    dc.columns([('a', np.zeros(100)), ('b', np.zeros(50))])
    g = dc.orders
    sa, sb = dc.order('a').slot, dc.order('b').slot
    kin, iin, n_in, kout, iout = g.ptrs_many([sa, sb], [100, 50])
    assert n_in.tolist() == [0, 0] and kin.tolist() == [0, 0] and np.all(kout != 0)

    def fill(slot, n, salt):
        # what the merge kernel would write to the out side
        o = (1 - int(g.cur[slot])) * g.tc + int(g.off[slot])
        g.keys[o:o + n] = torch.arange(n, dtype=torch.float64) + salt
        g.idx[o:o + n] = torch.arange(n, dtype=torch.int32)
    fill(sa, 100, 0.5)
    fill(sb, 50, 0.25)
    g.commit_many([sa, sb], [100, 50])
    assert dc.order('a').n == 100 and dc.order('b').n == 50
    v0 = dc.version
    kin, iin, n_in, kout, iout = g.ptrs_many([sa], [100])
    assert n_in.tolist() == [100] and kout.tolist() == [0]     # nothing new: no merge output
    assert dc.version == v0
    g.ensure([sb], [50000])                                   # b outgrows its room: everything moves
    assert dc.version > v0
    ka, ia = dc.order('a').host()
    kb, ib = dc.order('b').host()
    np.testing.assert_array_equal(ka, np.arange(100) + 0.5)
    np.testing.assert_array_equal(kb, np.arange(50) + 0.25)
    np.testing.assert_array_equal(ia, np.arange(100))
    kin, iin, n_in, kout, iout = g.ptrs_many([sa, sb], [100, 50000])
    assert n_in.tolist() == [100, 50] and kout[0] == 0 and kout[1] != 0
    assert g.keys[(kin[1] - g.kbase) // 8].item() == 0.25


def test_delta_mode_runs_leave_the_order():
    """A run with at most FIT_DELTA_MAX new observations over a resident order
    gets no merge buffers and its commit leaves the order as it was (the
    kernels read the new ones beside it); more new ones, or no order, merge."""
    from hyperopt_amd import _native as N
    dc = devhist.DeviceColumns(torch.device('cpu'))
    dc.columns([('a', np.zeros(1000))])
    g, sa = dc.orders, dc.order('a').slot
    kin, iin, n_in, kout, iout = g.ptrs_many([sa], [1000])
    assert n_in[0] == 0 and kout[0] != 0                # no order yet: a merge of everything
    g.commit_many([sa], [1000])
    for n in (1001, 1000 + N.FIT_DELTA_MAX):
        kin, iin, n_in, kout, iout = g.ptrs_many([sa], [n])
        assert n_in[0] == 1000 and kin[0] != 0 and kout[0] == 0 and iout[0] == 0
        g.commit_many([sa], [n])
        assert dc.order('a').n == 1000
    kin, iin, n_in, kout, iout = g.ptrs_many([sa], [1001 + N.FIT_DELTA_MAX])
    assert n_in[0] == 1000 and kout[0] != 0
    g.commit_many([sa], [1001 + N.FIT_DELTA_MAX])
    assert dc.order('a').n == 1001 + N.FIT_DELTA_MAX
