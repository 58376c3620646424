"""Per-kernel median durations from a rocprofv3 kernel-trace CSV."""
import collections
import csv
import sys


def short(name):
    if 'rocprim' in name:
        for k in ('segmented_sort', 'segmented_radix', 'onesweep_iteration', 'global_offsets', 'histogram',
                  'block_sort', 'warp_sort', 'merge', 'scan', 'lookback'):
            if k in name:
                return 'rocprim:' + k
        return 'rocprim:' + name[:60]
    if name.startswith('void '):
        name = name[5:]
    name = name.replace('(anonymous namespace)::', '')
    if '::' in name:
        name = name.split('(')[1] if name.startswith('(') else name
    return name.split('(')[0].split('::')[-1][:48]


def main(path):
    rows = list(csv.DictReader(open(path)))
    d = collections.defaultdict(list)
    for r in rows:
        nm = r['Kernel_Name']
        key = (short(nm if not nm.startswith('(anonymous') else nm.split('::', 1)[1]), r['Grid_Size_X'],
               r['Workgroup_Size_X'])
        d[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print('%-48s grid %-9s wg %-5s n=%4d med %8.1f us  sum %9.1f us' % (k[0], k[1], k[2], len(v), v[len(v) // 2],
                                                                           sum(v)))


if __name__ == '__main__':
    main(sys.argv[1])
