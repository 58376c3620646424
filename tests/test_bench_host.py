"""bench.py's host-side records (no GPU): the tail record's cgroup counters and
the contention counters it carries beside them."""
import time

import bench


def test_cgroup_cpu_stat_is_a_dict_of_counters():
    st = bench.cgroup_cpu_stat()
    assert isinstance(st, dict)
    assert all(isinstance(v, int) for v in st.values())


def test_host_contention_counts_grow_and_are_non_negative():
    a = bench.host_contention()
    time.sleep(0.01)                               # (a voluntary switch at least)
    b = bench.host_contention()
    assert {'nivcsw', 'nvcsw'} <= set(a)
    for k in ('nivcsw', 'nvcsw') + tuple(k for k in a if k.startswith('psi_') and k != 'psi_source'):
        assert b[k] >= a[k] >= 0, k
    assert b['nvcsw'] > a['nvcsw']
    if 'psi_source' in a:
        assert a['psi_source'] in ('/sys/fs/cgroup/cpu.pressure', '/proc/pressure/cpu')
