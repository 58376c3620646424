"""Per-workgroup phase times of k_fit_main on config 5.  The trace points are not
in the production kernel file: apply tools/fit_trace.patch, build the variant
(hyperopt_amd.build.build(out='hyperopt_amd/libtpe_hip_fittrace.so',
defines=('TPE_FIT_TRACE',))), revert the patch, then on the GPU box:
TPE_HIP_LIB=$PWD/hyperopt_amd/libtpe_hip_fittrace.so python tools/fit_trace.py
(s_memrealtime stamps, 10-ns ticks, by lane 0 of each workgroup after its phase)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import _native as N  # noqa: E402


class _A:
    axis4 = 'labels'
    appending = False
    dims = 1000
    history5 = 100000


def main():
    step = bench.config_workload(5, 0, 1, _A())[1]
    from hyperopt_amd.engine import get_engine
    get_engine(torch.device('cuda', 0))
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    lib = N.load()
    fn = lib.tpe_debug_fit_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(65536 * 6, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(65536, 6)[:49000, :5].astype(np.int64)
    ok = (t > 0).all(axis=1) & (np.diff(t, axis=1) >= 0).all(axis=1)
    t = t[ok]
    print('workgroups traced', len(t))
    span = (t[:, 4].max() - t[:, 0].min()) * 10e-3
    print('kernel span from the first start to the last end: %.1f us' % span)
    names = ['prologue+below', 'stretch+stage', 'rows loop', 'reduce+grid']
    d = np.diff(t, axis=1) * 10e-3
    for k, nm in enumerate(names):
        print('  %-16s median %6.2f us  mean %6.2f  p90 %6.2f' % (nm, np.median(d[:, k]), d[:, k].mean(),
                                                               np.percentile(d[:, k], 90)))
    tot = d.sum(axis=1)
    print('  %-16s median %6.2f us  mean %6.2f' % ('workgroup', np.median(tot), tot.mean()))
    # concurrency: workgroup-time / span
    print('  mean workgroups in flight: %.0f' % (tot.sum() / span))


if __name__ == '__main__':
    main()
