#!/usr/bin/env python3
"""Headline benchmark: EI candidates scored/sec + tpe.suggest p50 latency.

Workload (BASELINE.json configs[2], "config 3"): the conditional hp.choice
tree space (svm{C, kernel{rbf: gamma, poly: degree}} | rf{...} | knn{...}),
a 10,000-trial synthetic history, n_EI_candidates = 2^20 per GPU, one
``tpe.suggest`` per step (host history/fit + device sample/score/select,
entry to returned document).  N GPUs: weak scaling along the candidate axis —
each rank scores 2^20 candidates of every active hyperparameter, total
C = N * 2^20, per-level winner combined by one all-gather (dist.py).

value  = sum over steps of (active hyperparameters x total candidates) / time
roofline: the dominant stage by device time (k_sample_tab on config 3),
          timed per launch with HIP events the level runner records on its own
          stream (tpe_level_profile), priced by the ALGORITHMIC VALU work of its
          candidates (TAB_CAND_OPS, or TAB_CAND_OPS_LOGPOLY for the format the
          labels tabulate in, per candidate) against the issue peak; the
          executed-instruction fraction (SQ_INSTS_VALU of a separate PMC pass of
          the same build, pmc_stale flags a mismatch) beside it.
cpu_baseline: the CPU oracle (numpy restatement of the reference) on a bounded
          sample of the same workload, candidate-chunked over a measured process
          sweep (the best pool is the figure; 1 core beside it).
p50_suggest_ms_appending: the same suggest in an FMinIter loop (one finished
          document inserted before every suggest, fmin.py:88-92).
config4_strong: BASELINE config 4 (4096 new ids x 4096 candidates x 20 dims)
          with its (label x id) problem grid cut into label groups x id blocks
          (--axis4 grid, the default: dist.grid_shape, 4 x 2 at 8 ranks), or
          the hyperparameters (--axis4 labels) or the ids (--axis4 ids) alone,
          split over the N ranks and one all-gather of the chosen values
          (tpe.suggest_choices(shard_grid= / shard_labels= / shard_ids=...)):
          strong scaling of the axes that shard without a per-level exchange.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

C_PER_GPU = 1 << 20
N_HISTORY = 10000
SEED = 20241015


def tree_space(hp):
    return {'model': hp.choice('model', [
        {'name': 'svm', 'C': hp.loguniform('svm_C', -5, 5),
         'kernel': hp.choice('svm_kernel', [{'gamma': hp.loguniform('svm_rbf_gamma', -5, 2)},
                                            {'degree': hp.quniform('svm_poly_degree', 2, 5, 1)}])},
        {'name': 'rf', 'n_est': hp.quniform('rf_n_est', 10, 500, 10),
         'depth': hp.choice('rf_depth', [None, hp.quniform('rf_depth_n', 2, 30, 1)]),
         'crit': hp.choice('rf_crit', ['gini', 'entropy'])},
        {'name': 'knn', 'k': hp.quniform('knn_k', 1, 50, 1), 'p': hp.uniform('knn_p', 1, 3)}])}


def synthetic_loss(v, tid):
    """Smooth synthetic objective favouring the svm/rbf branch; 1e-9*tid breaks ties."""
    loss = 1.0
    if v.get('model') == 0:
        loss = 0.5 + 0.05 * (math.log(float(v['svm_C'])) - 1.0) ** 2
        if v.get('svm_kernel') == 0:
            loss -= 0.2 - 0.02 * (math.log(float(v['svm_rbf_gamma'])) + 2.0) ** 2
    elif v.get('model') == 1:
        loss = 0.8 + 1e-4 * abs(float(v['rf_n_est']) - 200)
    else:
        loss = 0.9 + 0.01 * abs(float(v['knn_k']) - 7)
    return loss + 1e-9 * tid


def rf_loss(v, tid):
    """A synthetic loss that steers the tree to its rf branch (quantized
    rf_n_est / rf_depth_n labels at the full candidate count)."""
    import math
    loss = 1.0
    if v.get('model') == 1:
        loss = 0.3 + 1e-3 * abs(float(v['rf_n_est']) - 180) + 0.05 * int(v['rf_crit'])
        if v.get('rf_depth') == 1:
            loss -= 0.1 - 0.005 * abs(float(v['rf_depth_n']) - 12)
    elif v.get('model') == 2:
        loss = 0.6 + 0.01 * abs(float(v['knn_k']) - 7) + 0.05 * (float(v['knn_p']) - 2) ** 2
    elif v.get('model') == 0:
        loss = 0.8 + 0.01 * (math.log(float(v['svm_C']))) ** 2
    return loss + 1e-9 * tid


def loss_domain(space, loss):
    """A Domain whose objective is ``loss(flat values, tid)``: called with the
    trial's {label: value} spec and its Ctrl (pass_expr_memo_ctrl)."""
    from hyperopt_amd import base

    def fn(expr, memo, ctrl):
        return loss(memo, ctrl.current_trial['tid'])
    return base.Domain(fn, space, pass_expr_memo_ctrl=True)


def evaluate(domain, trials, d):
    """Evaluate document ``d`` and store its result as FMinIter.serial_evaluate
    does (fmin.py:40-70): Domain.evaluate's result dict, state DONE."""
    from hyperopt_amd import base
    result = domain.evaluate(base.spec_from_misc(d['misc']), base.Ctrl(trials, current_trial=d))
    d['state'] = base.JOB_STATE_DONE
    d['result'] = result


def make_history(n, seed, loss=None):
    """``n`` prior draws of the config-3 tree space (rand.suggest) with losses
    from ``loss(vals, tid)`` (default synthetic_loss), evaluated as fmin
    evaluates them."""
    from hyperopt_amd import base, hp, rand
    domain = loss_domain(tree_space(hp), synthetic_loss if loss is None else loss)
    trials = base.Trials()
    rs = np.random.RandomState(seed)
    docs = []
    for tid in range(n):
        d = rand.suggest([tid], domain, trials, rs.randint(2 ** 31 - 1))[0]
        evaluate(domain, trials, d)
        docs.append(d)
    trials.insert_trial_docs(docs)
    trials.refresh()
    return domain, trials


def host_cpu():
    """Model and core counts of this host (the GPU box's host when run there)."""
    model = ''
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else os.cpu_count()
    quota = None                      # the cgroup's CPU share (cpu.max quota / period), if any
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, per = f.read().split()[:2]
        if q != 'max' and float(per) > 0:
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return dict(model=model, logical_cpus=os.cpu_count(), usable_cpus=aff, cgroup_cpu_quota=quota)


def cpu_baseline(domain, trials, budget_s=10.0, sweep=(16, 64, 128, 256), sweep_s=5.0):
    """The oracle (numpy restatement of the reference, tools/oracle_vs_reference.py
    times it against the reference itself) on a bounded sample of the same
    workload: whole suggests at C = 16384 on the same 10k-trial history,
    (1) on one core for ~budget_s and (2) candidate-chunked over process pools
    of each size in ``sweep`` (capped at the usable cores) for ~sweep_s each —
    chunking is exact, logsum_rows is row-wise (tpe.py:253-256); sampling stays
    serial, as in the reference.  The reported figure is the best pool of the
    sweep (the knee: more processes than the host's CPU share buy nothing).
    Called before the GPU is initialised (the pools fork)."""
    import multiprocessing as mp
    from oracle import tpe_oracle as O
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(1)
    except Exception:  # pragma: no cover
        limiter = None
    params = []
    for r in domain.table.rows:
        parent = None if r.parents == [None] else tuple(r.parents[0])
        params.append(dict(label=r.label, dist=r.dist, args=dict(r.args), parent=parent))
    hist = [dict(tid=d['tid'], loss=d['result']['loss'], vals=d['misc']['vals']) for d in trials.trials]
    C = 16384

    def run(pool, chunks, secs):
        n_scores, calls, t0 = 0, 0, time.time()
        while time.time() - t0 < secs:
            out = O.tpe_suggest(params, hist, 1000 + calls, n_EI_candidates=C, pool=pool, chunks=chunks)
            n_scores += len(out) * C
            calls += 1
        dt = time.time() - t0
        return n_scores / dt, calls, dt

    v1, c1, d1 = run(None, 1, budget_s)
    cpu = host_cpu()
    pts = []
    for P in sorted(set(max(1, min(p, cpu['usable_cpus'])) for p in sweep)):
        with mp.get_context('fork').Pool(P) as pool:
            run(pool, P, 0.5)                       # pool warm-up (imports, first tasks)
            vp, cp, dp = run(pool, P, sweep_s)
        pts.append(dict(processes=P, value=vp, calls=cp, secs=dp))
    if limiter is not None:
        limiter.unregister()
    best = max(pts, key=lambda p: p['value'])
    # the knee: the smallest pool within 5 % of the best (more processes than
    # the host's CPU share buy nothing)
    knee = min((p for p in pts if p['value'] >= 0.95 * best['value']), key=lambda p: p['processes'])
    # (cores: the CPU time the pool could use — a cgroup quota caps it below the
    # process count)
    quota = cpu.get('cgroup_cpu_quota')
    cores = min(best['processes'], int(math.ceil(quota))) if quota else best['processes']
    return dict(value=best['value'], unit='candidate-scores/s', cores=cores, processes=best['processes'], kind='port',
                knee_processes=knee['processes'],
                sample='%d oracle tpe_suggest calls, C=16384, same 10k-trial history, candidate scoring chunked '
                       'over %d processes on %d cores, %.1fs (best of the process sweep)'
                       % (best['calls'], best['processes'], cores, best['secs']),
                sweep=[dict(processes=p['processes'], value=p['value']) for p in pts],
                single_core=dict(value=v1, cores=1,
                                 sample='%d oracle tpe_suggest calls, C=16384, %.1fs, 1 core' % (c1, d1)),
                host=cpu)


class CpuBaselineChild:
    """cpu_baseline in a child process forked before anything initialises the
    GPU (its pools fork in turn), held on a pipe until the GPU measurements are
    done: the 10-30 s of host load (a 256-process sweep) then no longer runs
    just before the timed steps (the first timed suggest after it took 0.21 ms
    instead of 0.10).  result() starts it and waits; close() ends an unused
    child (the pipe's end: EOF)."""

    def __init__(self, pre):
        import multiprocessing as mp
        ctx = mp.get_context('fork')
        self.conn, child = ctx.Pipe()
        self.proc = ctx.Process(target=CpuBaselineChild._main, args=(child, self.conn, pre))
        self.proc.start()
        child.close()

    @staticmethod
    def _main(conn, parent_end, pre):
        parent_end.close()            # (the fork's copy: the parent's close must reach EOF here)
        try:
            conn.recv()
        except EOFError:
            return
        conn.send(cpu_baseline(*pre))

    def result(self):
        self.conn.send('go')
        out = self.conn.recv()
        self.close()
        return out

    def close(self):
        if self.proc is not None:
            self.conn.close()
            self.proc.join()
            self.proc = None


# ------------------------------------------------------------------ roofline
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
# VALU issue peak: a wave64 VALU instruction issues over 2 cycles on a SIMD32
# (MI355X_MICROARCH.md, Wave scheduling): 0.5 wave-instructions / cycle / SIMD
# x 4 SIMDs x 256 CUs x 2.4 GHz
PEAK_VALU_GINST = 0.5 * 4 * 256 * 2.4      # = 1228.8 G wave-instructions/s
# counter summary of the same bench command (tools/gpu.sh pmc -> tools/pmc_summary.py)
PMC_SUMMARY_REL = 'profiles/r06_pmc_summary.json'
PMC_SUMMARY = os.path.join(ROOT, PMC_SUMMARY_REL)
VALU_KERNELS = ('k_sample', 'k_tables', 'k_select', 'above', 'k_finalize')


LIB_PATH = os.path.join(ROOT, 'hyperopt_amd', 'libtpe_hip.so')

# Algorithmic work of one tabulated candidate (k_sample_tab), in VALU lane
# operations — the operations the method needs, whatever the code executes
# ("Roofline"); a wave-instruction does 64 of them.
TAB_CAND_OPS = {
    'philox': 40,        # half a Philox-4x32-10 block: 10 rounds x (2 mad_u64 + 4 xor + 2 key adds) / 2
    'uniforms': 5,       # 32-bit selection uniform, 23-bit inversion uniform
    'guide_scan': 6,     # guide-table bucket, one LDS read, ~1.5 compare steps of the CDF scan
    'ndtri_f32': 19,     # p from the truncation bounds, log(4p(1-p)), degree-8 polynomial, sign
    'affine': 1,         # t = mu + sigma * z
    'cells': 26,         # per side: cell index, bounds test, centre, u = (t - c) / h, row address
    'horner': 20,        # per side: degree-10 Horner sum of the moments
    'log2': 4,           # per side: log2 of the sum + shift m
    'compare': 6,        # l2 - g2, flag tests, running best (value, index)
}
TAB_CAND_OPS_TOTAL = sum(TAB_CAND_OPS.values())
# ... the same with TPE_F_LOGPOLY rows (include/tpe_hip.h "Tabulated scoring"),
# the format the headline's labels tabulate in: one cell look-up for both
# sides, two degree-5 polynomials that are the log2 sums themselves
TAB_CAND_OPS_LOGPOLY = dict(TAB_CAND_OPS, cells=13, horner=10, log2=0)


def tab_format(domain, trials, n_cand):
    """'logpoly' when every tabulated label of the headline suggest's level
    packs TPE_F_LOGPOLY rows (tpe_host_pack_level on the host, as the suggest
    packs it), else 'moments' — the format whose operations price the sample
    stage's algorithmic work."""
    import ctypes
    from hyperopt_amd import _native as N, history as H, tpe
    from hyperopt_amd.engine import Engine, LevelProblem
    lib = N.load()
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
    blob = np.empty(cap, dtype=np.uint8)
    rc = lib.tpe_host_pack_level(recs, len(problems), int(n_cand), 7, 0, 0, N.PREC_F32, blob.ctypes.data, cap,
                                 ctypes.byref(info))
    if rc != 0:
        return 'moments'
    prob = np.frombuffer(blob, dtype=N.PROBLEM_DTYPE, count=int(info.n_problems), offset=int(info.off_problems))
    tab = prob[prob['tab_mode'] == N.TAB_CELLS]
    return 'logpoly' if len(tab) and np.all(tab['flags'] & N.F_LOGPOLY) else 'moments'


def lib_hash(path=LIB_PATH):
    import hashlib
    if not os.path.exists(path):
        return None
    with open(path, 'rb') as f:
        return hashlib.sha256(f.read()).hexdigest()


def _pmc():
    if not os.path.exists(PMC_SUMMARY):
        return {}
    with open(PMC_SUMMARY) as f:
        return json.load(f)


# a profiled stage and the kernels it launches (counters are summed per dispatch)
STAGE_KERNELS = {'k_sample': ('k_sample', 'k_sample_tab', 'k_sample_fast'),
                 'above': ('k_above_f32', 'k_above_f64', 'k_above_q')}


def _stage_counters(pmc, stage):
    parts = [pmc[k] for k in STAGE_KERNELS.get(stage, (stage,)) if k in pmc]
    if len(parts) <= 1:
        return parts[0] if parts else {}
    return {c: sum(p.get(c, 0.0) for p in parts) for c in set().union(*parts) if c != 'dispatches'}


def roofline(prof, fmt='moments'):
    """Roofline of every measured stage and of the dominant one (largest total
    device time): work per launch / the launch's average duration, the
    duration timed live with HIP events on the engine stream.

    VALU-bound kernels are priced by EXECUTED work: the VALU wave-instructions
    one launch issues (SQ_INSTS_VALU per dispatch of the same bench command,
    profiles/r02_pmc_summary.json) against the issue peak; the sort (when a
    level still sorts) by its HBM bytes.  The algorithmic CE rate (C x K
    component evaluations the reference performs) is reported beside it: the
    tabulated kernels do not evaluate C x K terms, so that rate exceeds the
    direct-evaluation ceiling and is context, not a roofline fraction."""
    pmc = _pmc()
    kernels = {}
    stage_total = {}           # every stage's time on the stream, measured alike (the dominant one's pick)
    for name, recs in prof.items():
        ms = np.array([r[0] for r in recs])
        if not len(ms) or name == 'fit':
            continue
        stage_ms = ms
        # the sample stage's tabulated pass is timed by its own launch's start /
        # stop events (tpe_stage_prof.kernel_ns): the kernel as rocprofv3 sees it,
        # without the dispatch after the table stage the stage's events include
        kms = np.array([r[3] if len(r) > 3 else 0.0 for r in recs])
        if np.all(kms > 0):
            ms = kms
        secs = ms.sum() * 1e-3
        k = dict(avg_launch_ms=float(ms.mean()), launches=int(len(ms)), total_ms=float(ms.sum()))
        stage_total[name] = float(stage_ms.sum())
        if ms is not stage_ms:
            k.update(timing='kernel start/stop events (hipExtLaunchKernel)',
                     avg_stage_ms=float(stage_ms.mean()))
        c = _stage_counters(pmc, name)
        if name == 'sort':
            nbytes = np.array([r[1] for r in recs])
            ach = nbytes.sum() / secs / 1e9
            k.update(bound='hbm', achieved=ach, peak=PEAK_HBM_GBS, unit='GB/s', frac=ach / PEAK_HBM_GBS,
                     bytes_per_launch=float(nbytes.mean()),
                     note='rocPRIM onesweep radix sort of (u32 bucket key, u64 position|t) pairs')
        elif name == 'k_sample' and len(recs[0]) > 2 and recs[0][2] > 0:
            # tabulated scoring: the algorithmic VALU work of the candidates
            # (TAB_CAND_OPS per candidate) / the launch time / the issue peak
            cands = float(np.mean([r[1] for r in recs]))
            ops = TAB_CAND_OPS_LOGPOLY if fmt == 'logpoly' else TAB_CAND_OPS
            alg = cands * sum(ops.values()) / 64.0
            ach = alg / (ms.mean() * 1e-3) / 1e9
            k.update(bound='valu', achieved=ach, peak=PEAK_VALU_GINST, unit='G VALU wave-instructions/s',
                     frac=ach / PEAK_VALU_GINST, work='algorithmic', table_format=fmt,
                     algorithmic_valu_per_launch=alg, candidates_per_launch=cands,
                     ops_per_candidate=sum(ops.values()), ops_model=ops)
            if 'SQ_INSTS_VALU' in c:
                inst = float(c['SQ_INSTS_VALU'])
                exe = inst / (ms.mean() * 1e-3) / 1e9
                k.update(executed_valu_per_launch=inst, executed_achieved=exe,
                         frac_executed=exe / PEAK_VALU_GINST, executed_per_algorithmic=inst / alg,
                         executed_source=PMC_SUMMARY_REL + ' (SQ_INSTS_VALU per dispatch)')
        elif name in VALU_KERNELS and 'SQ_INSTS_VALU' in c:
            inst = float(c['SQ_INSTS_VALU'])
            ach = inst / (ms.mean() * 1e-3) / 1e9
            k.update(bound='valu', achieved=ach, peak=PEAK_VALU_GINST, unit='G VALU wave-instructions/s',
                     frac=ach / PEAK_VALU_GINST, work='executed', executed_valu_per_launch=inst,
                     executed_source=PMC_SUMMARY_REL + ' (SQ_INSTS_VALU per dispatch)')
        else:
            k.update(bound=None)
        if name == 'k_sample' and len(recs[0]) > 2:
            ce = np.array([r[2] for r in recs])
            k.update(algorithmic_ce_per_launch=float(ce.mean()), algorithmic_ce_per_s=float(ce.sum() / secs),
                     direct_ce_ceiling=7.97e12, direct_ce_ceiling_source='profiles/r01_ce_ubench.txt')
        if 'FETCH_SIZE' in c and 'WRITE_SIZE' in c:
            k['traffic'] = (2 * c['FETCH_SIZE'] + c['WRITE_SIZE']) * 1024.0
        kernels[name] = k
    # (by the stages' stream times: the sample stage's kernel-only time would
    # otherwise be compared with the table stage's time including its dispatch)
    dom = max((n for n in kernels if kernels[n].get('bound')), key=lambda n: stage_total[n], default=None)
    if dom is None:
        return None, kernels
    r = dict(kernels[dom])
    r['kernel'] = dom
    r['stage_kernels'] = [k for k in STAGE_KERNELS.get(dom, (dom,)) if k in _pmc()] or [dom]
    r.setdefault('traffic', None)
    if r['traffic'] is not None:
        r['traffic_source'] = PMC_SUMMARY_REL + ': (2 x FETCH_SIZE + WRITE_SIZE) per dispatch (gfx950 ' \
                              'FETCH_SIZE correction, MI355X_MICROARCH.md)'
    # the counters belong to the library that runs (its hash is in the summary)
    built = pmc.get('lib_sha256')
    r['pmc_stale'] = bool(pmc) and (built is None or built != lib_hash())
    return r, kernels


# ---------------------------------------------------------------- other configs
def soa_history(labels, n, seed, loss_fn):
    """Synthetic structure-of-arrays history (history.History): every label
    active in every trial, values ~ U(-5, 5), losses from ``loss_fn``."""
    from hyperopt_amd.history import History
    rs = np.random.RandomState(seed)
    tids = np.arange(n, dtype=np.int64)
    vals = {k: rs.uniform(-5, 5, n) for k in labels}
    losses = loss_fn(vals) + 1e-9 * tids
    return History(tids, losses, {k: (tids, v) for k, v in vals.items()})


def flat_uniform_table(labels):
    from hyperopt_amd import hp
    from hyperopt_amd.space import ParamTable
    return ParamTable({k: hp.uniform(k, -5, 5) for k in labels})


def mixed10_space(hp):
    return {'u0': hp.uniform('u0', -5, 5), 'u1': hp.uniform('u1', 0, 1), 'u2': hp.uniform('u2', -1, 3),
            'l0': hp.loguniform('l0', -5, 0), 'l1': hp.loguniform('l1', -2, 2), 'l2': hp.loguniform('l2', 0, 3),
            'q0': hp.quniform('q0', 0, 20, 1), 'q1': hp.quniform('q1', -4, 4, 0.5),
            'c0': hp.choice('c0', list(range(5))), 'c1': hp.choice('c1', list(range(3)))}


def mixed10_history(n, seed):
    """Config 2's history: ``n`` prior draws of the 10-dim mixed space with
    loss sum((v - 0.3)^2) + 1e-9 * tid."""
    from hyperopt_amd import base, hp, rand
    domain = loss_domain(mixed10_space(hp), lambda v, tid: sum((float(x) - 0.3) ** 2 for x in v.values()) + 1e-9 * tid)
    trials = base.Trials()
    rs = np.random.RandomState(seed)
    docs = []
    for tid in range(n):
        d = rand.suggest([tid], domain, trials, rs.randint(2 ** 31 - 1))[0]
        evaluate(domain, trials, d)
        docs.append(d)
    trials.insert_trial_docs(docs)
    trials.refresh()
    return domain, trials


def config_workload(config, rank, world, args):
    """(description, setup info, step(i) -> candidate-scores, cpu_baseline_fn or None)"""
    from hyperopt_amd import base, hp, rand, tpe
    if config == 1:
        from hyperopt_amd import Trials, fmin

        def step(i):
            t = Trials()
            fmin(lambda x: (x - 3) ** 2, hp.uniform('x', -10, 10), algo=tpe.suggest, max_evals=100, trials=t,
                 rstate=np.random.RandomState(i))
            return 80 * 24        # 80 TPE suggests (after 20 start-up) x 24 candidates
        return 'config1: fmin(tpe.suggest), hp.uniform 1-D quadratic, 100 trials, n_EI_candidates=24', step, None
    if config == 2:
        domain, trials = mixed10_history(1000, SEED)
        C = 10000

        def step(i):
            docs = tpe.suggest([1000], domain, trials, SEED + i, n_EI_candidates=C * world,
                               shard=(rank, world) if world > 1 else None)
            return sum(1 for v in docs[0]['misc']['vals'].values() if v) * C * world
        return 'config2: 10-dim mixed space, 1000-trial history, n_EI_candidates=10000', step, None
    if config == 4:
        labels = ['x%02d' % i for i in range(20)]
        hist = soa_history(labels, 10000, SEED, lambda v: sum((x - 0.3) ** 2 for x in v.values()))
        table = flat_uniform_table(labels)
        n_ids, C = 4096, 4096
        ids = np.arange(10000, 10000 + n_ids)
        sid = (rank, world) if world > 1 else None
        # N > 1: the 2-D grid (each rank a label group's fits, rows and tables and
        # its id block's sample pass: every rank the same problem count), the
        # hyperparameter axis (each rank its labels for every id) or the new-id
        # axis (each rank its block of ids, every label's fits and tables on
        # every rank); one all-gather of the chosen values either way — every
        # rank holds all 4096 x 20
        axis = getattr(args, 'axis4', 'grid')
        kw = {dict(grid='shard_grid', labels='shard_labels', ids='shard_ids')[axis]: sid}

        def step(i, columns=True):
            # SoA in, SoA out (tpe.ChoiceColumns); columns=False: per-id dicts
            tpe.suggest_choices(table, hist, ids, SEED + i, n_EI_candidates=C, columns=columns, **kw)
            return len(labels) * n_ids * C          # whole job
        what = dict(grid='(label group x id block) grid', labels='hyperparameters', ids='new_ids')[axis]
        return ('config4: batched suggest, 4096 new_ids x 4096 candidates, 20-dim U(-5,5), 10k-trial '
                'history, %s sharded over ranks + one all-gather of the chosen values, columnar results'
                % what), step, None
    if config == 5 and args.appending:
        # FMinIter's flow on the columnar history (fmin.py:88-92): every suggest
        # follows the evaluation of the previous one, appended as one observation
        # of every label — the history views grow by one and share the device
        # columns and resident value orders (History.dev), as a Trials cache's do
        from hyperopt_amd.history import DenseLayout, DenseObs, History
        D, N, C = args.dims, args.history5, 4096
        labels = ['x%04d' % i for i in range(D)]
        cap = N + args.steps + args.warmup + 64
        rs = np.random.RandomState(SEED)
        tids = np.arange(cap, dtype=np.int64)
        vals2d = np.empty((D, cap))                    # (one row per label: the evaluation writes a column)
        cols = {k: vals2d[i] for i, k in enumerate(labels)}
        row = {k: i for i, k in enumerate(labels)}
        layout = DenseLayout(labels)
        for k in labels:
            cols[k][:N] = rs.uniform(-5, 5, N)
        rl = np.random.RandomState(SEED + 1)
        losses = np.empty(cap)
        losses[:N] = rl.uniform(size=N) + 1e-9 * np.arange(N)
        table = flat_uniform_table(labels)
        sid = (rank, world) if world > 1 else None
        dev = {}
        state = dict(n=N)

        def step(i):
            n = state['n']
            # (the columnar history: every label a row of one matrix — history.DenseObs)
            hist = History(tids[:n], losses[:n], DenseObs(layout, vals2d, tids[:n]), dev=dev)
            cc = tpe.suggest_choices(table, hist, [n], SEED + i, n_EI_candidates=C, shard_labels=sid, columns=True)
            if state.get('lab') != cc.labels:        # (the suggestion's label order -> rows, once)
                state['lab'], state['ri'] = cc.labels, np.array([row[k] for k in cc.labels], dtype=np.int64)
            vals2d[state['ri'], n] = cc.values[0]    # the suggestion, evaluated (synthetic loss)
            losses[n] = rl.uniform() + 1e-9 * n
            state['n'] = n + 1
            return D * C
        return ('config5 appending: %d-dim U(-5,5), %d-trial history growing by one evaluated suggestion per '
                'step (FMinIter flow), n_EI_candidates=4096' % (D, N)), step, None
    if config == 5:
        D, N, C = args.dims, args.history5, 4096
        labels = ['x%04d' % i for i in range(D)]
        hist = soa_history(labels, N, SEED, lambda v: np.zeros(N))
        rs = np.random.RandomState(SEED + 1)
        hist.losses[:] = rs.uniform(size=N) + 1e-9 * np.arange(N)
        table = flat_uniform_table(labels)
        sid = (rank, world) if world > 1 else None

        def step(i):
            # N > 1: each rank fits and scores its labels (dist.label_owners), one
            # all-gather of the chosen values — every rank holds the whole suggestion
            tpe.suggest_choices(table, hist, [N], SEED + i, n_EI_candidates=C, shard_labels=sid)
            return D * C
        return ('config5: %d-dim U(-5,5), %d-trial history, n_EI_candidates=4096, hyperparameters sharded '
                'over ranks + one all-gather of the chosen values' % (D, N)), step, None
    raise ValueError(config)



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-quantized', action='store_true', help='skip the rf-branch (quantized) report')
    ap.add_argument('--no-appending', action='store_true', help='skip the FMinIter-style appending loop')
    ap.add_argument('--no-config4', action='store_true', help='skip the config-4 strong-scaling record')
    ap.add_argument('--history', type=int, default=N_HISTORY)
    ap.add_argument('--cands', type=int, default=C_PER_GPU)
    ap.add_argument('--config', type=int, default=3, help='BASELINE.json config (3 = headline)')
    ap.add_argument('--axis4', choices=('grid', 'labels', 'ids'), default='grid',
                    help='config 4 over N > 1 ranks: shard the (label x id) grid, the hyperparameters or the new ids')
    ap.add_argument('--dims', type=int, default=1000, help='config 5 dimensions')
    ap.add_argument('--history5', type=int, default=100000, help='config 5 history length')
    ap.add_argument('--appending', action='store_true',
                    help='config 5: one evaluated suggestion appended to the history before every suggest')
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    pre = None
    cpu = None
    cpu_child = None
    if args.config == 3:
        pre = make_history(args.history, SEED)
        # the CPU baseline's process, forked before anything initialises the GPU
        # (its process pools fork), run after the GPU measurements; rank 0 at N = 1 only
        if world == 1 and not args.no_cpu_baseline:
            cpu_child = CpuBaselineChild(pre)
    try:
        main_gpu(args, world, rank, local, pre, cpu_child)
    finally:
        if cpu_child is not None:
            cpu_child.close()


def main_gpu(args, world, rank, local, pre, cpu_child):
    import torch
    import torch.distributed as dist
    cpu = None
    if world > 1:
        if os.environ.get('TPE_BENCH_BACKEND', 'nccl') != 'nccl':
            local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        # TPE_BENCH_BACKEND=gloo: a rehearsal of the N > 1 flow with several ranks on
        # one GPU (RCCL takes one rank per device); the driver's runs use nccl (RCCL)
        backend = os.environ.get('TPE_BENCH_BACKEND', 'nccl')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    device = torch.device('cuda', local)
    torch.cuda.set_device(device)

    from hyperopt_amd import engine as engine_mod, tpe
    from hyperopt_amd.engine import get_engine
    get_engine(device)
    if args.config != 3:
        return run_other(args, rank, world, device)
    domain, trials = pre
    new_id = args.history
    shard = (rank, world) if world > 1 else None
    C_total = args.cands * world

    def step(i):
        return tpe.suggest([new_id], domain, trials, SEED + i, n_EI_candidates=C_total, shard=shard)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    import gc
    cg0 = cgroup_cpu_stat()      # (read before the warm-up: nothing between it and the timed steps)
    hc0 = host_contention()
    for i in range(args.warmup):
        step(i)
    barrier()
    lat = []
    n_active = 0
    _GC_COUNT.clear()
    gc.callbacks.append(_count_gc)
    t0 = time.perf_counter()
    for i in range(args.steps):
        s0 = time.perf_counter()
        docs = step(1000 + i)
        lat.append(time.perf_counter() - s0)
        n_active += sum(1 for v in docs[0]['misc']['vals'].values() if v)
    barrier()
    elapsed = time.perf_counter() - t0
    cg1 = cgroup_cpu_stat()
    hc1 = host_contention()
    gc.callbacks.remove(_count_gc)
    gc_timed = dict(_GC_COUNT)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = n_active * C_total / elapsed

    # strong scaling: the BASELINE 2^20 candidates in total, split over the ranks
    strong = None
    if world > 1:
        C_strong = args.cands

        def step_strong(i):
            return tpe.suggest([new_id], domain, trials, SEED + i, n_EI_candidates=C_strong, shard=shard)

        for i in range(args.warmup):
            step_strong(7000 + i)
        barrier()
        lat_s, act_s = [], 0
        t0 = time.perf_counter()
        for i in range(args.steps):
            s0 = time.perf_counter()
            d = step_strong(8000 + i)
            lat_s.append(time.perf_counter() - s0)
            act_s += sum(1 for v in d[0]['misc']['vals'].values() if v)
        barrier()
        el_s = time.perf_counter() - t0
        t = torch.tensor([el_s], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el_s = float(t.item())
        strong = dict(n_EI_candidates_total=C_strong, per_rank=C_strong // world, value=act_s * C_strong / el_s,
                      unit='candidate-scores/s', ms_per_step=1e3 * el_s / args.steps,
                      p50_suggest_ms=1e3 * float(np.median(lat_s)),
                      p99_suggest_ms=1e3 * float(np.percentile(lat_s, 99)))

    # dominant-kernel roofline, measured live: the level runner's own HIP events
    # between the stages it issues, on its stream (tpe_level_profile) — stages
    # the production flow skips (k_select under early selection) are absent
    eng = engine_mod._ENGINES[str(device)]
    eng.profile = {}
    for i in range(5):
        step(5000 + i)
    torch.cuda.synchronize()
    prof = eng.profile
    eng.profile = None
    roof, kernels = roofline(prof, tab_format(domain, trials, C_total))
    stages = {k: float(np.mean([a[0] for a in v])) for k, v in prof.items()}
    ranks = rank_report(world, rank, lat, host_phases(eng, step, k=10, base=6000) if world > 1 else None, stages)
    # the timed loop's own record (N = 1): every step's latency, the collections
    # and the cgroup's CPU throttling over it, and — from a separate untimed pass
    # of 200 more steps — the host phases of the slowest steps
    tail = None
    if world == 1:
        tail = dict(steps_ms=[round(1e3 * x, 4) for x in lat], gc_collections=gc_timed,
                    cgroup_cpu_stat_warmup_and_timed={k: cg1.get(k, 0) - cg0.get(k, 0) for k in cg1},
                    host_contention_warmup_and_timed={k: (v - hc0[k] if k in hc0 and not isinstance(v, str) else v)
                                                      for k, v in hc1.items()},
                    slowest_of_200=slow_steps(eng, step, 200, base=30000))


    # one quantized-branch workload beside the line: the same tree and sizes with
    # a history steered to the rf branch (quantized labels at 2^20 candidates)
    quant = None
    if world == 1 and not args.no_quantized:
        qdom, qtr = make_history(args.history, SEED, loss=rf_loss)
        for i in range(args.warmup):
            tpe.suggest([new_id], qdom, qtr, SEED + 9000 + i, n_EI_candidates=C_total)
        torch.cuda.synchronize()
        ql, qd = [], None
        for i in range(10):
            s0 = time.perf_counter()
            qd = tpe.suggest([new_id], qdom, qtr, SEED + 9100 + i, n_EI_candidates=C_total)
            ql.append(time.perf_counter() - s0)
        vals = {k: float(v[0]) for k, v in qd[0]['misc']['vals'].items() if v}
        quant = dict(workload='config3 tree, rf-steered %d-trial history (quantized rf_n_est/rf_depth_n), '
                              'n_EI_candidates=%d' % (args.history, C_total),
                     p50_suggest_ms=1e3 * float(np.median(ql)), active_labels=sorted(vals),
                     model=int(vals.get('model', -1)))

    # the suggest as FMinIter.run issues it (fmin.py:88-92): every suggest follows
    # the insertion of the previous suggestion, evaluated (synthetic loss) — the
    # history grows by one document per step, so each suggest extends the SoA
    # cache, its value orders and the tree records instead of reusing them
    appending = None
    if not args.no_appending:
        n_app = max(10, min(args.steps, 50))
        lat_a, tid = [], new_id
        for i in range(n_app + 2):
            s0 = time.perf_counter()
            docs = tpe.suggest([tid], domain, trials, SEED + 20000 + i, n_EI_candidates=C_total, shard=shard)
            dt = time.perf_counter() - s0
            if i >= 2:                      # (the first two: warm-up)
                lat_a.append(dt)
            trials.insert_trial_docs(docs)
            trials.refresh()
            evaluate(domain, trials, trials.trials[-1])
            tid += 1
        appending = dict(p50_suggest_ms=1e3 * float(np.median(lat_a)),
                         p99_suggest_ms=1e3 * float(np.percentile(lat_a, 99)), suggests=n_app,
                         history_from=new_id, history_to=tid,
                         note='one evaluated document inserted (and trials.refresh()) before every suggest, '
                              'as FMinIter.run does; the suggest alone is timed')

    # config 4 (BASELINE configs[3]: the batched suggest that shards naturally)
    # beside the line: 4096 new ids x 4096 candidates x 20 dims in total, the ids
    # split over the N ranks (strong scaling) and one all-gather of the results
    cfg4 = None
    if not args.no_config4:
        desc4, step4, _ = config_workload(4, rank, world, args)
        for i in range(2):
            step4(i)
        barrier()
        t0 = time.perf_counter()
        n4, units4 = 5, 0
        for i in range(n4):
            units4 = step4(100 + i)
        barrier()
        el4 = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el4], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el4 = float(t.item())
        cfg4 = dict(workload=desc4, value=units4 * n4 / el4, unit='candidate-scores/s', steps=n4,
                    ms_per_step=1e3 * el4 / n4, scaling='strong', n_gpus=world,
                    parallelism='%s shard x%d' % (dict(grid='label-group x id-block', labels='hyperparameter',
                                                       ids='new-id')[args.axis4], world))

    if cpu_child is not None:
        cpu = cpu_child.result()          # (after every GPU measurement of the line)
    if rank == 0:
        out = {
            'metric': 'EI candidates scored/sec (node) + tpe.suggest p50 latency, 1M cands x 10k trials',
            'value': value, 'unit': 'candidate-scores/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': 1e3 * elapsed / args.steps, 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
            'config': {'workload': 'config3: conditional hp.choice tree, %d-trial history, '
                                   'n_EI_candidates=%d per GPU (%d total), one tpe.suggest per step'
                                   % (args.history, args.cands, C_total),
                       'history': args.history, 'n_EI_candidates': C_total,
                       'parallelism': 'candidate-shard x%d' % world},
            'p50_suggest_ms': 1e3 * float(np.median(lat)), 'p99_suggest_ms': 1e3 * float(np.percentile(lat, 99)),
            'mean_suggest_ms': 1e3 * float(np.mean(lat)),
            'tail': tail,
            'ranks': ranks,
            'p50_suggest_ms_appending': appending['p50_suggest_ms'] if appending else None,
            'appending': appending,
            'active_hyperparameters_per_suggest': n_active / args.steps,
            'stage_ms': stages, 'roofline': roof, 'kernels': kernels, 'cpu_baseline': cpu,
            'quantized_branch': quant,
            'config4_strong': cfg4,
            # the same 2^20 candidates in total over N ranks (N = 1: the line itself)
            'strong_scaling': strong if strong is not None else dict(
                n_EI_candidates_total=C_total, per_rank=C_total, value=value, unit='candidate-scores/s',
                ms_per_step=1e3 * elapsed / args.steps, p50_suggest_ms=1e3 * float(np.median(lat)),
                p99_suggest_ms=1e3 * float(np.percentile(lat, 99))),
        }
        if cpu:
            out['speedup_vs_cpu_baseline'] = value / cpu['value']
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


_GC_COUNT = {}


def _count_gc(phase, info):
    """gc.callbacks hook: the collector's runs per generation (the multi-GPU
    rank report shows whether a step's tail is a collection)."""
    if phase == 'start':
        g = 'gen%d' % info['generation']
        _GC_COUNT[g] = _GC_COUNT.get(g, 0) + 1


def cgroup_cpu_stat():
    """The cgroup's cpu.stat counters (cgroup v2: nr_periods, nr_throttled,
    throttled_usec, usage_usec, ...), {} where absent."""
    out = {}
    try:
        with open('/sys/fs/cgroup/cpu.stat') as f:
            for line in f:
                k, v = line.split()
                out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


def host_contention():
    """Signs of other load on the host's CPUs: this process's involuntary and
    voluntary context switches (all its threads, getrusage) and the CPU
    pressure-stall totals (us some task waited for a CPU: the cgroup's
    cpu.pressure, else the host's /proc/pressure/cpu), {} where absent."""
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    out = {'nivcsw': ru.ru_nivcsw, 'nvcsw': ru.ru_nvcsw}
    for path in ('/sys/fs/cgroup/cpu.pressure', '/proc/pressure/cpu'):
        try:
            with open(path) as f:
                for line in f:
                    p = line.split()
                    out['psi_%s_total_us' % p[0]] = int(p[-1].split('=')[1])
            out['psi_source'] = path
            break
        except (OSError, ValueError, IndexError):
            continue
    return out


def slow_steps(eng, step, k=200, base=30000, n_show=5):
    """k more (untimed-loop) steps with the native host phase clock on: the
    p50 / mean / p99 of their walls and the phases of the n_show slowest —
    which part of a slow step grew (Python outside the native call, the fits,
    the pack, the device round trip)."""
    import ctypes
    import gc
    from hyperopt_amd import _native as N
    buf = (ctypes.c_double * len(N.PHASES))()
    ev = []
    cb = (lambda phase, info: ev.append((len(rows), info['generation'])) if phase == 'start' else None)
    rows = []
    gc.callbacks.append(cb)
    eng.lib.tpe_host_phases(1, None, 0)
    for i in range(k):
        s0 = time.perf_counter()
        step(base + i)
        w = 1e6 * (time.perf_counter() - s0)
        eng.lib.tpe_host_phases(1, buf, len(N.PHASES))
        rows.append((w, [round(float(v), 1) for v in buf]))
    eng.lib.tpe_host_phases(0, None, 0)
    gc.callbacks.remove(cb)
    w = np.array([r[0] for r in rows])
    order = np.argsort(-w)[:n_show]
    med = np.median(np.array([r[1] for r in rows]), axis=0)
    return dict(steps=k, p50_us=round(float(np.median(w)), 1), mean_us=round(float(w.mean()), 1),
                p99_us=round(float(np.percentile(w, 99)), 1), phase_names=list(N.PHASES),
                median_phases_us=[round(float(x), 1) for x in med],
                slowest=[dict(step=int(j), wall_us=round(float(w[j]), 1), phases_us=rows[j][1],
                              gc=[g for s, g in ev if s == j]) for j in order])


def host_phases(eng, step, k=3, base=300):
    """Median host phases of the native suggest (tpe_host_phases: us since its
    entry) over k more steps, and the steps' wall time ('step_wall'), or None."""
    import ctypes
    from hyperopt_amd import _native as N
    buf = (ctypes.c_double * len(N.PHASES))()
    eng.lib.tpe_host_phases(1, None, 0)
    ph, wall = [], []
    for i in range(k):
        s0 = time.perf_counter()
        step(base + i)
        wall.append(1e6 * (time.perf_counter() - s0))
        eng.lib.tpe_host_phases(1, buf, len(N.PHASES))
        ph.append(list(buf))
    eng.lib.tpe_host_phases(0, None, 0)
    med = np.median(np.array(ph), axis=0)
    if not med[-1] > 0:
        return None
    out = {k: round(float(v), 1) for k, v in zip(N.PHASES, med)}
    out['step_wall'] = round(float(np.median(wall)), 1)
    return out


def rank_report(world, rank, lat, phases, stages):
    """Every rank's step latencies (p50 / mean / p99 / max, ms), host phases and
    device stage times, gathered to all ranks (world > 1; None otherwise): the
    per-rank host share of a multi-GPU step."""
    if world <= 1:
        return None
    import torch.distributed as dist
    a = 1e3 * np.asarray(lat)
    info = dict(rank=rank, p50_ms=float(np.median(a)), mean_ms=float(np.mean(a)), p99_ms=float(np.percentile(a, 99)),
                max_ms=float(np.max(a)), steps_over_2x_p50=int(np.sum(a > 2 * np.median(a))),
                steps_ms=[round(float(x), 3) for x in a[:64]], gc_collections=dict(_GC_COUNT),
                host_phases_us=phases, stage_ms=stages)
    got = [None] * world
    dist.all_gather_object(got, info)
    return got


def run_other(args, rank, world, device):
    """Configs 1, 2, 4, 5: same timing discipline, own metric line."""
    import torch
    import torch.distributed as dist
    desc, step, _ = config_workload(args.config, rank, world, args)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for i in range(args.warmup):
        step(i)
    barrier()
    lat, units = [], 0
    import gc
    _GC_COUNT.clear()
    gc.callbacks.append(_count_gc)
    t0 = time.perf_counter()
    for i in range(args.steps):
        s0 = time.perf_counter()
        units = step(100 + i)
        lat.append(time.perf_counter() - s0)
    barrier()
    gc.callbacks.remove(_count_gc)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # per-stage device time of one more step (HIP events on the launch stream)
    from hyperopt_amd import engine as engine_mod
    eng = engine_mod._ENGINES[str(device)]
    eng.profile = {}
    step(10 ** 6)
    torch.cuda.synchronize()
    stages = {k: float(np.sum([a[0] for a in v])) for k, v in eng.profile.items()}
    eng.profile = None
    extra = {}
    # host phases of the native suggest over a few more steps, and the step's wall
    # time outside that call (Python)
    phases = host_phases(eng, step)
    if phases is not None:
        extra['host_phases_us'] = phases
    ranks = rank_report(world, rank, lat, phases, stages)
    if ranks is not None:
        extra['ranks'] = ranks
    if args.config == 4:
        # the same batched suggest returning per-id dicts (numpy int64 / float64
        # values, as the reference's: tpe._result_dicts)
        lat_d = []
        for i in range(3):
            s0 = time.perf_counter()
            step(200 + i, columns=False)
            lat_d.append(time.perf_counter() - s0)
        extra['p50_step_ms_dict_results'] = 1e3 * float(np.median(lat_d))
    if rank == 0:
        out = {'metric': 'EI candidates scored/sec (node)', 'value': units * args.steps / elapsed,
               'unit': 'candidate-scores/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
               'ms_per_step': 1e3 * elapsed / args.steps, 'higher_is_better': True,
               'scaling': 'strong' if args.config in (4, 5) else 'weak', 'vs_baseline': None, 'dtype': 'f32',
               'data': 'synthetic', 'config': {'workload': desc, 'config': args.config,
                                               'appending': bool(args.appending)},
               'p50_step_ms': 1e3 * float(np.median(lat)), 'stage_ms_per_step': stages}
        out.update(extra)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
