"""Timeline of the last suggests in a rocprofv3 --hip-trace --kernel-trace
--memory-copy-trace capture (csv): every HIP API call, kernel and copy between
the ends of consecutive k_sample_tab kernels (the last stage of a config-3
suggest), relative to the window start (us); hipStreamQuery polls are counted,
not listed."""
import csv
import glob
import os
import sys


def rows(root, pat):
    out = []
    for f in glob.glob(os.path.join(root, '**', pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main(root, n_show=2):
    api = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function']) for r in rows(root, '*hip_api_trace.csv')]
    ker = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K ' + r['Kernel_Name'].replace(
        '(anonymous namespace)::', '').replace('void ', '').split('(')[0][:40]) for r in rows(root, '*kernel_trace.csv')]
    cpy = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), 'C ' + r.get('Direction', 'copy') + ' ' +
            r.get('Size', '')) for r in rows(root, '*memory_copy_trace.csv')]
    sel = sorted(k for k in ker if 'k_sample_tab' in k[2])
    if len(sel) < n_show + 1:
        print('not enough suggests traced')
        return
    for j in range(len(sel) - n_show, len(sel)):
        t0, t1 = sel[j - 1][1], sel[j][1]
        ev = sorted(e for e in api + ker + cpy if t0 <= e[0] < t1)
        polls = [e for e in ev if e[2] == 'hipStreamQuery']
        print('--- suggest window %.1f us (%d hipStreamQuery polls, last ends at %.1f)' % (
            (t1 - t0) / 1e3, len(polls), (polls[-1][1] - t0) / 1e3 if polls else 0.0))
        for s, e, nm in ev:
            if nm != 'hipStreamQuery':
                print('%9.1f %8.1f  %s' % ((s - t0) / 1e3, (e - s) / 1e3, nm))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
