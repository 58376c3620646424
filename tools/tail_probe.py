"""Where the headline suggest's slow steps go.

Runs bench.py's config-3 step (tpe.suggest, 2^20 candidates, 10k-trial
history) for STEPS steps after WARMUP and records per step:
  wall_us         the step's wall time (perf_counter)
  ph              the native call's host phases (tpe_host_phases: us since its entry)
  gc              collections that ran inside the step: (generation, us)
  run_us/wait_us  the main thread's CPU time and run-queue wait in the step
                  (/proc/thread-self/schedstat)
  nivcsw/nvcsw    the main thread's involuntary / voluntary context switches
  proc_cpu_us     the whole process's CPU time in the step (all threads)
and, around the whole loop, the cgroup's cpu.stat (nr_throttled, throttled_usec).
The reads happen between steps, outside each step's wall time.

  python tools/tail_probe.py [--steps 2000] [--warmup 5] [--nogc] [--tag NAME]
writes gpurun_out/tail_<tag>.json and prints a summary."""
import argparse
import ctypes
import gc
import json
import os
import resource
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def cpu_stat():
    out = {}
    try:
        with open('/sys/fs/cgroup/cpu.stat') as f:
            for line in f:
                k, v = line.split()
                out[k] = int(v)
    except OSError:
        pass
    return out


def schedstat():
    try:
        with open('/proc/thread-self/schedstat') as f:
            a = f.read().split()
        return int(a[0]), int(a[1])
    except OSError:
        return 0, 0


def proc_cpu_ns():
    return time.clock_gettime_ns(time.CLOCK_PROCESS_CPUTIME_ID)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--nogc', action='store_true')
    ap.add_argument('--tag', default='default')
    ap.add_argument('--cands', type=int, default=1 << 20)
    args = ap.parse_args()
    import bench
    import torch
    domain, trials = bench.make_history(bench.N_HISTORY, bench.SEED)
    device = torch.device('cuda', 0)
    torch.cuda.set_device(device)
    from hyperopt_amd import _native as N, tpe
    from hyperopt_amd.engine import get_engine
    eng = get_engine(device)
    new_id = bench.N_HISTORY

    def step(i):
        return tpe.suggest([new_id], domain, trials, bench.SEED + i, n_EI_candidates=args.cands)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    gc_ev = []
    cur = {'t': 0.0}

    def on_gc(phase, info):
        if phase == 'start':
            cur['t'] = time.perf_counter()
        else:
            gc_ev.append((info['generation'], 1e6 * (time.perf_counter() - cur['t'])))
    if args.nogc:
        gc.disable()
    gc.callbacks.append(on_gc)
    buf = (ctypes.c_double * len(N.PHASES))()
    eng.lib.tpe_host_phases(1, None, 0)
    rows = []
    cs0 = cpu_stat()
    t_all = time.perf_counter()
    for i in range(args.steps):
        g0 = len(gc_ev)
        r0, w0 = schedstat()
        ru0 = resource.getrusage(resource.RUSAGE_THREAD)
        p0 = proc_cpu_ns()
        s0 = time.perf_counter()
        step(1000 + i)
        s1 = time.perf_counter()
        p1 = proc_cpu_ns()
        ru1 = resource.getrusage(resource.RUSAGE_THREAD)
        r1, w1 = schedstat()
        eng.lib.tpe_host_phases(1, buf, len(N.PHASES))
        rows.append(dict(i=i, wall_us=round(1e6 * (s1 - s0), 1),
                         ph=[round(float(v), 1) for v in buf],
                         gc=[(g, round(d, 1)) for g, d in gc_ev[g0:]],
                         run_us=round((r1 - r0) / 1e3, 1), wait_us=round((w1 - w0) / 1e3, 1),
                         nivcsw=ru1.ru_nivcsw - ru0.ru_nivcsw, nvcsw=ru1.ru_nvcsw - ru0.ru_nvcsw,
                         proc_cpu_us=round((p1 - p0) / 1e3, 1)))
    t_all = time.perf_counter() - t_all
    cs1 = cpu_stat()
    eng.lib.tpe_host_phases(0, None, 0)
    gc.callbacks.remove(on_gc)
    if args.nogc:
        gc.enable()
    # what a suggest leaves to the cyclic collector: 20 more steps with the
    # collector off, then one collection with DEBUG_SAVEALL
    gc.collect()
    gc.disable()
    gc.set_debug(gc.DEBUG_SAVEALL)
    c0 = gc.get_count()[0]
    for i in range(20):
        step(90000 + i)
    grown = gc.get_count()[0] - c0
    n_garbage = gc.collect()
    import collections
    census = collections.Counter(type(o).__name__ for o in gc.garbage).most_common(12)
    gc.set_debug(0)
    gc.garbage.clear()
    # what stays alive per suggest (tracked objects by type, 50 steps)
    live0 = collections.Counter(type(o).__name__ for o in gc.get_objects())
    for i in range(50):
        step(95000 + i)
    gc.collect()
    live1 = collections.Counter(type(o).__name__ for o in gc.get_objects())
    kept = {k: v - live0.get(k, 0) for k, v in live1.items() if v - live0.get(k, 0) != 0}
    gc.enable()
    th = ctypes.c_int32(0)
    eng.lib.tpe_host_threads(-1, ctypes.byref(th))
    wall = np.array([r['wall_us'] for r in rows])
    p50 = float(np.median(wall))
    slow = sorted(rows, key=lambda r: -r['wall_us'])[:12]
    # steps in 20-step windows, as the driver times them: the mean / p50 spread
    win = wall[:len(wall) // 20 * 20].reshape(-1, 20)
    summary = dict(tag=args.tag, steps=args.steps, host_threads=th.value, env={k: v for k, v in os.environ.items()
                                                                             if k.startswith(('TPE_', 'HIP_', 'AMD_', 'GPU_', 'HSA_'))},
                   p50_us=p50, mean_us=float(wall.mean()), p99_us=float(np.percentile(wall, 99)),
                   p999_us=float(np.percentile(wall, 99.9)), max_us=float(wall.max()),
                   over_1p5x=int(np.sum(wall > 1.5 * p50)), over_2x=int(np.sum(wall > 2 * p50)),
                   over_3x=int(np.sum(wall > 3 * p50)),
                   win20_mean_over_p50=dict(median=float(np.median(win.mean(1) / np.median(win, 1))),
                                            max=float(np.max(win.mean(1) / np.median(win, 1)))),
                   gc_by_gen={g: sum(1 for x in gc_ev if x[0] == g) for g in (0, 1, 2)},
                   gc_us_total=round(sum(d for _, d in gc_ev), 1),
                   cgroup={k: cs1.get(k, 0) - cs0.get(k, 0) for k in cs1}, loop_s=t_all,
                   proc_cpus_avg=float(sum(r['proc_cpu_us'] for r in rows) / max(1.0, wall.sum())),
                   nivcsw_total=int(sum(r['nivcsw'] for r in rows)), wait_us_total=float(sum(r['wait_us'] for r in rows)),
                   phase_names=list(N.PHASES), median_phases=[float(x) for x in np.median([r['ph'] for r in rows], 0)],
                   gc_count_growth_per_step=grown / 20.0, cyclic_garbage_per_step=n_garbage / 20.0,
                   garbage_census_20_steps=census, live_objects_kept_50_steps=kept,
                   slowest=slow)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(ROOT, 'gpurun_out', 'tail_%s.json' % args.tag), 'w') as f:
        json.dump(dict(summary=summary, rows=rows), f)
    s = dict(summary)
    s.pop('slowest')
    print(json.dumps(s))
    for r in slow:
        print('  slow', json.dumps(r))


if __name__ == '__main__':
    main()
