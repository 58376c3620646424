"""Summarise rocprofv3 --pmc CSVs per kernel (average per dispatch)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    for k in ('k_above_f32', 'k_above_f64', 'k_above_q', 'k_sample', 'k_finalize', 'k_select'):
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
    # traffic of the dominant kernel (guide: FETCH_SIZE is KB and reads half of a wide
    # coalesced stream on gfx950 -> double it; WRITE_SIZE exact for 16-B stores)
    a = out.get('k_above_f32', {})
    if 'FETCH_SIZE' in a and 'WRITE_SIZE' in a:
        out['traffic_k_above_f32'] = dict(fetch_kb=a['FETCH_SIZE'], write_kb=a['WRITE_SIZE'],
                                          bytes_per_launch=(2 * a['FETCH_SIZE'] + a['WRITE_SIZE']) * 1024,
                                          correction='FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM)')
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == '__main__':
    main(sys.argv[1])
