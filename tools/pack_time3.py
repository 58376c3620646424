"""CPU timing of tpe_host_pack_level on the headline level (config 3's svm/rbf
branch: model, svm_kernel, svm_C, svm_rbf_gamma fitted on the host from the
10k-trial history, one new id, 2^20 candidates).  No GPU.  Usage:
python tools/pack_time3.py [REPS]; TPE_PACK_LIB = a host-only build with
-DTPE_PACK_TRACE (the packer's sections timed on stderr:
tools/build_pack_trace.sh)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402

import bench  # noqa: E402
from hyperopt_amd import _native as N, history as H, tpe  # noqa: E402
from hyperopt_amd.engine import Engine, LevelProblem  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    if os.environ.get('TPE_PACK_LIB'):
        lib = ctypes.CDLL(os.environ['TPE_PACK_LIB'])
        lib.tpe_host_pack_level.restype = ctypes.c_int
        lib.tpe_host_pack_level.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64,
                                            ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                            ctypes.c_int64, ctypes.c_void_p]
    else:
        lib = N.load()
    domain, trials = bench.make_history(10000, bench.SEED)
    T = domain.table
    hist = H.extract(domain, trials)
    below = H.split_below(hist, 0.25)
    fits = tpe._Fits(T, hist, below, 1.0, None)
    rows = [T.by_label[k] for k in ('model', 'svm_kernel', 'svm_C', 'svm_rbf_gamma')]
    ids = np.array([len(hist)], dtype=np.int64)
    problems = [LevelProblem(fits.get(r), r.index, ids) for r in rows]
    recs, keep = Engine._labels(problems)
    info = N.PackInfo()
    cap = 64 << 20
    blob = np.zeros(cap, dtype=np.uint8)
    ts = []
    for _ in range(reps):
        s = time.perf_counter()
        rc = lib.tpe_host_pack_level(recs, len(problems), 1 << 20, 7, 0, 0, N.PREC_F32, blob.ctypes.data, cap,
                                     ctypes.byref(info))
        ts.append(time.perf_counter() - s)
        assert rc == 0, rc
    print('headline level: tpe_host_pack_level p50 %.1f us, min %.1f (blob %d B, %d tab jobs, %d tab units, '
          'upload %s)' % (1e6 * np.median(ts), 1e6 * min(ts), info.blob_bytes, info.n_tab_jobs, info.tab_units,
                          [(int(info.up_off[i]), int(info.up_len[i])) for i in range(info.n_up)]))
    print('  labels: ' + ', '.join('%s below %d above %d' % (r.label, len(p.post.below[0]),
                                                            len(p.post.above[0]) if p.post.above is not None else -1)
                                   for r, p in zip(rows, problems)))


if __name__ == '__main__':
    main()
