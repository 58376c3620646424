"""Projected N-rank step times of the three sharded axes from one-GPU
measurements (cost the multi-GPU host share before
any 8-GPU run).  Model, per config, from the bench line's host phases
(tpe_host_phases, us since the native call's entry) and device stages:

  config 3 (candidate axis, weak: 2^20 candidates per rank)
      T(N) = T1 + L * (x1 + a * (N - 1))
      L exchanged levels per suggest (1: the speculative fused batch; 2 when the
      prediction fails: the gate level, then the branch level), x1 the forced
      one-rank exchange's cost per level (k_runs_reduce, measured), a the
      per-hop latency of a small RCCL all-gather ring over xGMI (assumed).
  config 4 (new-id axis, strong: 4096 ids over the ranks; --axis4 ids)
      T(N) = F + V / N + X(N)
      F (every rank, unsharded): the label fits (prefit), the pack of the
      labels' component rows (pack - prefit) and the label tables (k_tables);
      V (sharded): the rest of the step (the id-block's sample pass, records,
      result assembly); X(N) the all-gather of the id blocks' values and
      activity (ids * labels * 9 B) at bandwidth bw after one latency.
  config 4 (hyperparameter axis, strong: the 20 labels over the ranks; the
      default --axis4 labels): F the Python around the native call, V the
      native call times ceil(20 / N) / 20, X(N) as above.
  config 4 (2-D axis, strong, the default --axis4 grid: G label groups x B id
      blocks, dist.grid_shape): T(N) = F + Fl * ceil(20 / G) / 20 + Vp * share
      + X(N); F the Python around the native call, Fl the per-label native
      work (prefit + pack + k_tables: made by each of a group's B ranks), Vp
      the rest of the native call (the sample pass, records and results of
      the problems), share = ceil(20 / G) * ceil(4096 / B) / (20 * 4096).
  config 5 (hyperparameter axis, strong: 1000 labels over the ranks)
      T(N) = F + V / N + X(N)
      F: the Python around the native call (history view, below split over
      all 10^5 losses — per rank, unsharded); V: the native call (fits, pack,
      device fit and tables of the rank's labels); X(N) the columns' gather.

Usage: python tools/project_scaling.py CFG3_BENCH.json CFG4.json CFG5.json
[--x1-us 2.95] [--hop-us 3] [--bw-gbs 50]; prints the table in DESIGN.md §6."""
import argparse
import json


def last_json(path):
    lines = [ln for ln in open(path).read().splitlines() if ln.startswith('{')]
    return json.loads(lines[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('cfg3')
    ap.add_argument('cfg4')
    ap.add_argument('cfg5')
    ap.add_argument('--x1-us', type=float, default=2.95, help='forced one-rank exchange per level (us)')
    ap.add_argument('--hop-us', type=float, default=3.0, help='RCCL small all-gather latency per ring hop (us)')
    ap.add_argument('--bw-gbs', type=float, default=50.0, help='all-gather bandwidth per rank (GB/s)')
    ap.add_argument('--levels', type=int, default=1, help='exchanges per suggest (1: the speculative fused level)')
    a = ap.parse_args()
    Ns = (1, 2, 4, 8)
    rows = []
    c3 = last_json(a.cfg3)
    t1 = c3['p50_suggest_ms'] * 1e3
    for n in Ns:
        t = t1 + (0 if n == 1 else a.levels * (a.x1_us + a.hop_us * (n - 1)))
        rows.append(('3 weak', n, t, t1 / t))
    c4 = last_json(a.cfg4)
    h4 = c4['host_phases_us']
    F4 = h4['pack'] + 1e3 * c4['stage_ms_per_step']['k_tables']
    T4 = c4['p50_step_ms'] * 1e3
    V4 = T4 - F4
    nbytes4 = 4096 * 20 * 9
    for n in Ns:
        x = 0 if n == 1 else a.hop_us * (n - 1) + nbytes4 * (n - 1) / n / (a.bw_gbs * 1e3)
        t = F4 + V4 / n + x
        rows.append(('4 ids', n, t, T4 / (n * t)))
    # config 4 over the hyperparameter axis (bench.py --axis4 labels): every
    # native part shards with the labels (ceil(20 / N) a rank), the Python
    # around the call does not
    F4l, V4l = T4 - h4['return'], h4['return']
    for n in Ns:
        x = 0 if n == 1 else a.hop_us * (n - 1) + nbytes4 * (n - 1) / n / (a.bw_gbs * 1e3)
        t = F4l + V4l * (-(-20 // n)) / 20 + x
        rows.append(('4 labels', n, t, T4 / (n * t)))
    # the 2-D grid: the label part made by every rank of a group, the problem
    # part divided by the whole grid
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
    from hyperopt_amd.dist import grid_shape
    Fl = h4['pack'] + 1e3 * c4['stage_ms_per_step']['k_tables']
    Vp = h4['return'] - Fl
    for n in Ns:
        G, B = grid_shape(20, 4096, n)
        share = (-(-20 // G)) * (-(-4096 // B)) / (20.0 * 4096)
        x = 0 if n == 1 else a.hop_us * (n - 1) + nbytes4 * (n - 1) / n / (a.bw_gbs * 1e3)
        t = F4l + Fl * (-(-20 // G)) / 20.0 + Vp * share + x
        rows.append(('4 grid %dx%d' % (G, B), n, t, T4 / (n * t)))
    c5 = last_json(a.cfg5)
    h5 = c5['host_phases_us']
    T5 = c5['p50_step_ms'] * 1e3
    V5 = h5['return']
    F5 = T5 - V5
    nbytes5 = 1000 * 9
    for n in Ns:
        x = 0 if n == 1 else a.hop_us * (n - 1) + nbytes5 * (n - 1) / n / (a.bw_gbs * 1e3)
        t = F5 + V5 / n + x
        rows.append(('5 strong', n, t, T5 / (n * t)))
    print('inputs: cfg3 p50 %.1f us; cfg4 ids F %.0f V %.0f us, labels F %.0f V %.0f us, grid label part %.0f '
          'problem part %.0f us; cfg5 F %.0f V %.0f us; x1 %.2f us/level, hop %.1f us, bw %.0f GB/s'
          % (t1, F4, V4, F4l, V4l, Fl, Vp, F5, V5, a.x1_us, a.hop_us, a.bw_gbs))
    print('%-14s %3s %10s %10s' % ('config', 'N', 'T(N) us', 'eff'))
    for name, n, t, e in rows:
        print('%-14s %3d %10.1f %10.2f' % (name, n, t, e))


if __name__ == '__main__':
    main()
