"""CPU timing of tpe_host_pack_level on a config-4-shaped level (no GPU): D
uniform(-5, 5) labels fitted on the host from a 10k-trial history (25 below,
the rest above), each active for every one of n_ids new ids, C = 4096 — an
expanded level (include/tpe_hip.h).  Usage: python tools/pack_time4.py [D]
[N_IDS] [REPS]; TPE_PACK_LIB = a host-only build with -DTPE_PACK_TRACE (the
packer's sections timed on stderr: tools/build_pack_trace.sh)"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402

from hyperopt_amd import _native as N, parzen  # noqa: E402


def main():
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n_ids = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    if os.environ.get('TPE_PACK_LIB'):
        lib = ctypes.CDLL(os.environ['TPE_PACK_LIB'])
        lib.tpe_host_pack_level.restype = ctypes.c_int
        lib.tpe_host_pack_level.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64,
                                            ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                            ctypes.c_int64, ctypes.c_void_p]
    else:
        lib = N.load()
    rs = np.random.RandomState(0)
    recs = np.zeros(D, dtype=N.LABEL_DTYPE)
    keep = [recs]
    ids = np.arange(10000, 10000 + n_ids, dtype=np.int64)
    keep.append(ids)
    for i in range(D):
        fits = []
        for n in (25, 9975):
            w, mu, sg = parzen.fit_parzen(rs.uniform(-5, 5, n), 1.0, 0.0, 10.0)
            fits.append((np.ascontiguousarray(w), np.ascontiguousarray(mu), np.ascontiguousarray(sg)))
        keep.append(fits)
        r = recs[i]
        r['family'], r['flags'], r['label_ix'] = N.FAM_GAUSS, N.F_HAS_LOW | N.F_HAS_HIGH, i
        r['low'], r['high'] = -5.0, 5.0
        (bw, bm, bs), (aw, am, as_) = fits
        r['below_w'], r['below_mu'], r['below_sigma'], r['below_k'] = bw.ctypes.data, bm.ctypes.data, bs.ctypes.data, len(bw)
        r['above_w'], r['above_mu'], r['above_sigma'], r['above_k'] = aw.ctypes.data, am.ctypes.data, as_.ctypes.data, len(aw)
        r['ids'], r['n_ids'] = ids.ctypes.data, n_ids
        r['lf'] = 25
        r['prior_mu'], r['prior_sigma'], r['prior_weight'] = 0.0, 10.0, 1.0
    info = N.PackInfo()
    cap = 256 << 20
    blob = np.zeros(cap, dtype=np.uint8)
    ts = []
    for _ in range(reps):
        s = time.perf_counter()
        rc = lib.tpe_host_pack_level(recs.ctypes.data, D, 4096, 7, 0, 0, N.PREC_F32, blob.ctypes.data, cap,
                                     ctypes.byref(info))
        ts.append(time.perf_counter() - s)
        assert rc == 0, rc
    print('D %d ids %d: tpe_host_pack_level p50 %.1f us, min %.1f (blob %d B, expanded %d, %d tab jobs, %d tab units)'
          % (D, n_ids, 1e6 * np.median(ts), 1e6 * min(ts), info.blob_bytes, info.n_expand, info.n_tab_jobs,
             info.tab_units))


if __name__ == '__main__':
    main()
