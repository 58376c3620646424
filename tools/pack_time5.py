"""CPU timing of tpe_host_pack_level on a config-5-shaped level (no GPU): D
device-fitted uniform labels (the below side fitted on the host, the above side
a device fit of N observations — fake device addresses: the packer only
records them) at C = 4096.  Usage: python tools/pack_time5.py [D] [N] [REPS]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402

from hyperopt_amd import _native as N, parzen  # noqa: E402


def main():
    D = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    n_obs = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    if os.environ.get('TPE_PACK_LIB'):       # host-only build with the section clock (tools/build_pack_trace.sh)
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
    ids = np.array([n_obs], dtype=np.int64)
    bidx = np.sort(rs.choice(n_obs, 25, replace=False)).astype(np.int32)
    keep += [ids, bidx]
    for i in range(D):
        w, mu, sg = parzen.fit_parzen(rs.uniform(-5, 5, 25), 1.0, 0.0, 10.0)
        keep.append((w, mu, sg))
        r = recs[i]
        r['family'], r['flags'], r['label_ix'] = N.FAM_GAUSS, N.F_HAS_LOW | N.F_HAS_HIGH, i
        r['low'], r['high'] = -5.0, 5.0
        r['below_w'], r['below_mu'], r['below_sigma'], r['below_k'] = w.ctypes.data, mu.ctypes.data, sg.ctypes.data, 26
        r['above_k'] = n_obs - 25 + 1
        r['ids'], r['n_ids'] = ids.ctypes.data, 1
        r['dev_obs'], r['n_obs'] = 0x1000, n_obs            # (a device address the packer only copies)
        r['below_idx'], r['n_below'], r['lf'] = bidx.ctypes.data, 25, 25
        r['prior_mu'], r['prior_sigma'], r['prior_weight'] = 0.0, 10.0, 1.0
        r['ord_key_in'], r['ord_idx_in'], r['n_ord_in'] = 0x2000, 0x3000, n_obs
    info = N.PackInfo()
    cap = 4 << 30                                  # (the device-fit reserve counts: untouched pages)
    blob = np.empty(cap, dtype=np.uint8)
    ts = []
    for _ in range(reps):
        s = time.perf_counter()
        rc = lib.tpe_host_pack_level(recs.ctypes.data, D, 4096, 7, 0, 0, N.PREC_F32, blob.ctypes.data, cap,
                                     ctypes.byref(info))
        ts.append(time.perf_counter() - s)
        assert rc == 0, rc
    print('D %d n_obs %d: tpe_host_pack_level p50 %.1f us (blob %d B, %d tab jobs, fgt boxes %d)'
          % (D, n_obs, 1e6 * np.median(ts), info.blob_bytes, info.n_tab_jobs, info.fgt_max_boxes))


if __name__ == '__main__':
    main()
