"""Summarise rocprofv3 --pmc CSVs per kernel (average per dispatch)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    for k in ('k_above_f32', 'k_above_f64', 'k_above_q', 'k_sample_fast', 'k_sample_tab', 'k_sample', 'k_tables',
              'k_finalize', 'k_select',
              'k_fit_stats', 'k_fit_emit', 'k_fit_combine', 'k_fit_wide', 'k_ord_chunks', 'k_ord_merge', 'k_ord_below',
              'k_ord_compact', 'k_upload'):
        if k in name:
            return k
    return 'rocprim' if 'rocprim' in name else name[:40]


def main(root):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, '*', '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r.get('Kernel_Name', ''))
            acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
    out = {}
    for k, d in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in d.items()}
        out[k]['dispatches'] = max(len(v) for v in d.values())
    # HBM traffic per launch of the bench's kernels (guide: FETCH_SIZE is KB and
    # reads half of a wide coalesced stream on gfx950 -> double it; WRITE_SIZE
    # exact for 16-B stores).  'sort' = every rocPRIM dispatch of one tpe_sort
    # call; the bench makes one sort per suggest, i.e. per k_select dispatch.
    traffic = {}
    for k in ('k_above_f32', 'k_sample', 'k_sample_fast', 'k_sample_tab', 'k_tables', 'k_finalize', 'k_select'):
        a = out.get(k, {})
        if 'FETCH_SIZE' in a and 'WRITE_SIZE' in a:
            traffic[k] = dict(kernel=k, fetch_kb=a['FETCH_SIZE'], write_kb=a['WRITE_SIZE'],
                              bytes_per_launch=(2 * a['FETCH_SIZE'] + a['WRITE_SIZE']) * 1024)
    r, sel = out.get('rocprim', {}), out.get('k_select', {})
    if 'FETCH_SIZE' in r and 'WRITE_SIZE' in r and sel.get('dispatches'):
        per = r['dispatches'] / sel['dispatches']
        traffic['sort'] = dict(kernel='sort', rocprim_dispatches_per_sort=per,
                               fetch_kb=r['FETCH_SIZE'] * per, write_kb=r['WRITE_SIZE'] * per,
                               bytes_per_launch=(2 * r['FETCH_SIZE'] + r['WRITE_SIZE']) * 1024 * per)
    for t in traffic.values():
        t['correction'] = 'FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM)'
    out['traffic'] = traffic
    # the build these counters belong to (bench.py flags a summary of another build as stale)
    import hashlib
    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'hyperopt_amd', 'libtpe_hip.so')
    if os.path.exists(lib):
        out['lib_sha256'] = hashlib.sha256(open(lib, 'rb').read()).hexdigest()
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == '__main__':
    main(sys.argv[1])
