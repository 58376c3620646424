"""The below-side sorting network of a device-fitted label (csrc/sort_net.h,
used by tpe_suggest.cpp's fit_label): compiled on its own into a small
library and checked against numpy on random arrays — ties, repeated values,
signed zeros, infinities and NaN (NaN last, as np.argsort puts it).  Tied
values may come out in any order (the fit's below side has every weight 1)."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HDR = os.path.join(HERE, '..', 'hyperopt_amd', 'csrc', 'sort_net.h')

WRAPPER = r'''
#include "sort_net.h"
extern "C" void sort_small_c(const double* x, long long n, long long* ord) {
  int64_t o[tpe_sort_net::kSortNet];
  tpe_sort_net::sort_small(x, n, o);
  for (long long i = 0; i < n; ++i) ord[i] = o[i];
}
extern "C" int sort_net_cap(void) { return tpe_sort_net::kSortNet; }
'''


@pytest.fixture(scope='module')
def net(tmp_path_factory):
    gxx = shutil.which(os.environ.get('CXX', 'g++'))
    if gxx is None:
        pytest.skip('no C++ compiler')
    d = tmp_path_factory.mktemp('sortnet')
    src, lib = d / 'w.cpp', d / 'libsortnet.so'
    src.write_text(WRAPPER)
    subprocess.run([gxx, '-O2', '-std=c++17', '-fPIC', '-shared', '-I', os.path.dirname(HDR), str(src), '-o', str(lib)],
                   check=True)
    so = ctypes.CDLL(str(lib))
    so.sort_small_c.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
    so.sort_small_c.restype = None
    return so


def test_network_sorts_like_numpy(net):
    assert net.sort_net_cap() == 32
    rs = np.random.RandomState(11)
    pool = np.array([0.0, -0.0, 1.5, -2.25, np.inf, -np.inf, np.nan, 3.0, 3.0])
    for trial in range(4000):
        n = rs.randint(0, 33)
        kind = trial % 4
        if kind == 0:
            x = rs.uniform(-5, 5, n)
        elif kind == 1:
            x = rs.choice(pool, n)
        elif kind == 2:
            x = np.round(rs.normal(0, 2, n), 1)               # many ties
        else:
            x = rs.uniform(-5, 5, n)
            x[rs.rand(n) < 0.2] = np.nan
        ord_ = np.zeros(max(n, 1), dtype=np.int64)
        net.sort_small_c(x.ctypes.data, n, ord_.ctypes.data)
        o = ord_[:n]
        assert sorted(o.tolist()) == list(range(n))           # a permutation
        got, ref = x[o], x[np.argsort(x, kind='stable')]
        np.testing.assert_array_equal(got, ref)               # NaN last; ties interchangeable
