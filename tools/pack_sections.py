"""Median per-section times from a TPE_PACK_TRACE run's stderr ("pack NAME us"
and "fill_label LI us" lines; the first 50 calls skipped as warm-up).
Usage: python tools/pack_sections.py LOG"""
import collections
import sys

import numpy as np


def main():
    d = collections.OrderedDict()
    for line in open(sys.argv[1]):
        p = line.split()
        if len(p) >= 3 and p[0] in ('pack', 'fill_label'):
            d.setdefault(p[0] + ' ' + p[1], []).append(float(p[2]))
    for k, v in d.items():
        v = v[50:] if len(v) > 100 else v
        print('%-24s %8.2f us' % (k, float(np.median(v))))


if __name__ == '__main__':
    main()
