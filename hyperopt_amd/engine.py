"""Device engine: packs fitted posteriors into the C-ABI tables and runs them.

One ``Engine.run`` call = one batched launch sequence (sample -> score ->
select) over every (hyperparameter, new_id) *problem* of one tree level.  All
device memory is owned here through torch tensors (torch is only the
allocator / stream provider); the kernels are libtpe_hip.so.

Device layout (HBM, all caller-owned, grow-only pools):
  problems  tpe_problem[P]            136 B each
  comp32    float4[K_total]           continuous families, f32 precision
  comp64    double4[K_total]          quantized / categorical / f64 precision
  samp      double[8][Kb_total]       below-mixture sampler rows
  cand      double[C_total]           candidate values (returned to the user)
  coord     float[C_total]            kernel coordinate (x or ln x) in f32
  part      double[sum_p splits_p*C_p] above-mixture partial sums
  tile_best tpe_best[T * BEST_PER_TILE], result tpe_result[P]
Mixtures are shared by every problem of the same hyperparameter (the history
is common to all new_ids), so component tables scale with labels, not ids.
"""
import ctypes
import math
import os

import numpy as np

from . import _native as N
from . import parzen

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None
# raw current-stream accessor of the torch build (None: go through torch.cuda.current_stream)
_RAW_STREAM = getattr(torch._C, '_cuda_getCurrentRawStream', None) if torch is not None else None
try:                                    # (the native trampoline of tpe_suggest_tree; optional until built)
    from ._hostaddr import call_tree as _CALL_TREE
except ImportError:                     # pragma: no cover
    _CALL_TREE = None

# target number of above-mixture work items per launch (>= 8 per CU on 256 CUs)
TARGET_WORK = 2048
MIN_COMPONENTS_PER_SPLIT = 128
# continuous above mixtures with at least this many observations are fitted on
# the device (tpe_fit_above) in fp32 mode; TPE_DEVICE_FIT_MIN overrides
DEVICE_FIT_MIN = int(os.environ.get('TPE_DEVICE_FIT_MIN', '16384'))
PRUNE_MIN_K = 64
FINE_KEY_MIN_CAND = 65536          # tpe_host.cpp kFineKeyMinCand: 12-bit sort buckets from here
TAIL_MIN_TILES = 32                # tpe_host.cpp kTailMinTiles: per-tile tail splits from here


def _coord_range(post):
    """Value range of the kernel coordinate (x, or ln x for log families) the
    candidates of ``post`` fall in: the bounds, else the below mixture +-8 sigma."""
    if post.family == N.FAM_CATEGORICAL:
        return 0.0, float(max(post.upper, 1))
    if post.low is not None and post.high is not None:
        return float(post.low), float(post.high)
    w, mu, sg = post.below
    return float(np.min(mu - 8 * sg)), float(np.max(mu + 8 * sg))


TAB_ETA = 0.05                     # tpe_host.cpp kTabEta: a_max * h <= eta per cell
TAB_MAX_CELLS = 65536
TAB_MAX_LATTICE = 1 << 18
TAB_MIN_RATIO, TAB_MIN_RATIO_DEVFIT = 8.0, 64.0   # tpe_host.cpp kTabMinRatio*: candidates per cell row
LOGPOLY_MAX_CELLS = 2048           # tpe_host.cpp kLogpolyMaxCells (TPE_F_LOGPOLY: one grid for both sides)
LP_ROW_COST = 1.25                 # tpe_host.cpp kLpRowCost (a LOGPOLY row in cell rows)
LP_DIRECT_ROWS = 64                # tpe_host.cpp kLpDirectRows
MOM_DIRECT_ROWS = 64               # tpe_host.cpp kMomDirectRows
MOM_CELLS_PER_WAVE = 4             # tpe_host.cpp kMomCellsPerWave
LP_ROWS_PER_WAVE = 5               # tpe_host.cpp kLpRowsPerWave
A_SCALE_LIT = 0.84932180028801907  # tpe_host.cpp kAScale (the same double)


def _tab_plan(lp, n_cand, f64):
    """Tabulated scoring of one level label (tpe_host.cpp, "tabulated scoring"):
    dict(mode, n=(cells or lattice values per side), lo, hi, lat_lo)."""
    post = lp.post
    none = dict(mode=N.TAB_NONE, n=(0, 0), lo=0.0, hi=0.0, lat_lo=0)
    if os.environ.get('TPE_TABLES', '1').startswith('0') or n_cand <= 0 or len(lp.ids) == 0:
        return none
    fam = post.family
    if fam == N.FAM_CATEGORICAL or len(post.below[0]) == 0:
        return none
    klo, khi = _coord_range(post)
    if not (math.isfinite(klo) and math.isfinite(khi) and khi > klo):
        return none
    ct = float(len(lp.ids)) * float(n_cand)

    def cells(sig):
        n = math.ceil((khi - klo) * (A_SCALE_LIT / max(sig, parzen.EPS)) / (2.0 * TAB_ETA))
        return int(n) if 1.0 <= n < 1e15 else -1
    if fam in (N.FAM_GAUSS, N.FAM_LOGGAUSS) and not f64:
        s0 = float(np.min(post.below[2]))
        if post.above_dev is not None:
            n_obs, bidx = post.above_dev[1:3]
            s1 = post.prior[1] / min(100.0, 1.0 + float(n_obs - len(bidx) + 1))
        else:
            s1 = float(np.min(post.above[2]))
        n0, n1 = cells(s0), cells(s1)
        ratio = TAB_MIN_RATIO_DEVFIT if post.above_dev is not None else TAB_MIN_RATIO
        nl = max(n0, n1)
        # (a device-fitted label takes box-moment cells when TPE_FGT allows: tpe_host.cpp)
        boxes = post.above_dev is not None and not os.environ.get('TPE_FGT', '1').startswith('0')
        if (not os.environ.get('TPE_LOGPOLY', '1').startswith('0') and not boxes and n0 > 0 and n1 > 0
                and nl <= LOGPOLY_MAX_CELLS and ct >= ratio * LP_ROW_COST * nl):
            return dict(mode=N.TAB_CELLS, n=(nl, nl), lo=klo, hi=khi, lat_lo=0, logpoly=True)
        if 0 < n0 <= TAB_MAX_CELLS and 0 < n1 <= TAB_MAX_CELLS and ct >= ratio * (n0 + n1):
            return dict(mode=N.TAB_CELLS, n=(n0, n1), lo=klo, hi=khi, lat_lo=0)
    elif fam in (N.FAM_QGAUSS, N.FAM_QLOGGAUSS) and post.q and post.q > 0 and lp.inject is None:
        tlo, thi = klo, khi
        if post.low is None or post.high is None:
            w, mu, sg = post.below
            tlo, thi = float(np.min(mu - 9 * sg)), float(np.max(mu + 9 * sg))
        lg = fam == N.FAM_QLOGGAUSS
        xlo, xhi = (math.exp(tlo), math.exp(thi)) if lg else (tlo, thi)
        mlo, mhi = math.floor(xlo / post.q) - 1.0, math.ceil(xhi / post.q) + 1.0
        nl = mhi - mlo + 1.0
        if math.isfinite(nl) and 1.0 <= nl <= TAB_MAX_LATTICE and abs(mlo) < 9e15 and ct >= 2.0 * nl:
            return dict(mode=N.TAB_LATTICE, n=(int(nl), 0), lo=klo, hi=khi, lat_lo=int(mlo))
    return none


def _rows32(mu, a, c):
    """float4 {mu_hi, mu_lo, a, c} rows (mu split so t - mu keeps ~48 bits)."""
    r = np.empty((len(mu), 4), dtype=np.float32)
    hi = np.asarray(mu, dtype=np.float32)
    r[:, 0] = hi
    r[:, 1] = (np.asarray(mu, dtype=np.float64) - hi.astype(np.float64)).astype(np.float32)
    r[:, 2] = a
    r[:, 3] = c
    return r


class LevelProblem(object):
    """One hyperparameter of one tree level, active for ``ids``.

    post     parzen.Posterior
    label_ix stable label index (Philox counter word 2)
    ids      int64 array of new_ids for which this label is active
    inject   optional float64 [len(ids), n_cand] candidates (replay / tests)
    """
    __slots__ = ('post', 'label_ix', 'ids', 'inject')

    def __init__(self, post, label_ix, ids, inject=None):
        self.post, self.label_ix = post, int(label_ix)
        self.ids = np.ascontiguousarray(ids, dtype=np.int64)
        self.inject = inject


class _TreeIO(object):
    """Engine.suggest_tree's argument and result arrays (grown, never shrunk)
    with their addresses looked up once."""

    def __init__(self, n, nl, nb, old=None):
        if old is not None:
            n, nl, nb = max(n, old.n_cap), max(nl, old.l_cap), max(nb, old.b_cap)
        self.n_cap, self.l_cap, self.b_cap = n, nl, max(nb, 64)
        self.ids = np.zeros(n, dtype=np.int64)
        self.below = np.zeros(self.b_cap, dtype=np.int64)
        self.values = np.zeros(n * nl)
        self.active = np.ones(n * nl, dtype=np.int8)
        self.need_fit = np.zeros(nl, dtype=np.int8)
        self.ids_ptr, self.below_ptr = self.ids.ctypes.data, self.below.ctypes.data
        self.values_ptr, self.active_ptr = self.values.ctypes.data, self.active.ctypes.data
        self.need_fit_ptr = self.need_fit.ctypes.data


class Engine(object):
    """Per-device engine.  ``precision`` is 'fp32' (default, performance) or
    'fp64' (parity mode: float64 continuous families)."""

    def __init__(self, device=None, precision='fp32'):
        if torch is None:
            raise N.NativeUnavailable('torch is required for device memory')
        self.lib = N.load()
        n = ctypes.c_int(0)
        if self.lib.tpe_device_count(ctypes.byref(n)) != 0 or n.value == 0 or not torch.cuda.is_available():
            raise N.NativeUnavailable('no HIP device visible: the TPE engine has no CPU fallback')
        if device is None:
            device = torch.device('cuda', torch.cuda.current_device())
        self.device = torch.device(device)
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.tile = self.lib.tpe_tile_size()
        self.device_fit_min = DEVICE_FIT_MIN
        self.tree_calls = 0              # tpe_suggest_tree calls (tests: one per steady-state suggest)
        self.set_precision(precision)
        self._bufs = {}
        self._pinned = None
        self._ws = None                   # cached tpe_level_ws (run_level)
        self._tree_out = ((ctypes.c_int32 * 2)(), N.LevelNeed())   # suggest_tree's path / need records
        # (their addresses and tpe_suggest_tree's, for the native trampoline)
        self._tree_addr = (ctypes.addressof(self._tree_out[0]), ctypes.addressof(self._tree_out[1]),
                           ctypes.cast(self.lib.tpe_suggest_tree, ctypes.c_void_p).value)
        self._tree_io = None              # suggest_tree's argument / result buffers (_TreeIO)
        # when a dict: every run() times each stage with HIP events on the
        # launch stream and appends (ms, CE of the launch) under the kernel name;
        # profile_repeat > 1 re-issues each (idempotent) stage back to back and
        # reports the mean (steady-state stage cost, tools/stage_bench.py)
        self.profile = None
        self.profile_repeat = 1
        # pruned f32 above kernel: local (Taylor) expansion of components whose
        # series converges over a wave's candidate span (False: all exact)
        self.expand = True
        # continuous f32 tiles with one split: score in the above kernel (False:
        # always in the finalize stage)
        self.fuse = True

    def _stream(self):
        """The device's current torch stream as a raw hipStream_t (the same
        handle torch.cuda.current_stream(device).cuda_stream gives, without
        building a Stream object: microseconds per suggest)."""
        raw = _RAW_STREAM
        if raw is not None:
            return raw(self._dev_index)
        return torch.cuda.current_stream(self.device).cuda_stream

    def set_precision(self, precision):
        if precision not in ('fp32', 'fp64'):
            raise ValueError("precision must be 'fp32' or 'fp64'")
        self.precision = precision

    # ------------------------------------------------------------ buffers
    def _buf(self, name, n, dtype):
        n = max(int(n), 1)
        t = self._bufs.get(name)
        if t is None or t.numel() < n or t.dtype != dtype:
            cap = max(n, int(1.25 * (t.numel() if t is not None else 0)))
            t = torch.empty(cap, dtype=dtype, device=self.device)
            self._bufs[name] = t
            self._ws = None
        return t

    # ------------------------------------------------------------- tables
    def _build_numpy(self, problems, n_cand, seed, cand_base, n_cand_global):
        """Host-side packing of one level in numpy — the specification that
        the native packer (tpe_host_pack_level) is tested against."""
        f64 = self.precision == 'fp64'
        T = self.tile
        plans = [_tab_plan(lp, n_cand, f64) for lp in problems]
        # sorted (pruned) problems: continuous f32 above mixtures of > PRUNE_MIN_K
        # components that are not tabulated
        pruned_l = [(not f64) and lp.post.family in (N.FAM_GAUSS, N.FAM_LOGGAUSS)
                    and (lp.post.above_dev is not None or len(lp.post.above[0]) > PRUNE_MIN_K)
                    and pl['mode'] == N.TAB_NONE for lp, pl in zip(problems, plans)]
        # a pruned label active for several ids is pooled: one sort slot for all its problems
        pooled_l = [pr and len(lp.ids) >= 2 for lp, pr in zip(problems, pruned_l)]
        S = sum((1 if po else len(lp.ids)) for lp, pr, po in zip(problems, pruned_l, pooled_l) if pr)
        n_sorted = sum(len(lp.ids) for lp, pr in zip(problems, pruned_l) if pr)
        max_slot = max([n_cand * (len(lp.ids) if po else 1) for lp, pr, po in zip(problems, pruned_l, pooled_l)
                        if pr], default=0)
        pbits = int(math.ceil(math.log2(S))) if S > 1 else 0
        key_bits = max(5, 8 - pbits)
        if max_slot >= FINE_KEY_MIN_CAND:
            key_bits = max(key_bits, min(12, 16 - pbits))
        comp32, comp64, samp, grids = [], [], [], []
        n32 = n64 = ns = ngrid = 0
        rows = []                         # per LevelProblem: (table info)
        for lp, pl in zip(problems, plans):
            post = lp.post
            fam = post.family
            klo, khi = _coord_range(post)
            info = dict(wide_off=0, wide_len=0, grid_off=0, grid_n=0, prior_mu=0.0, prior_a=0.0, prior_c=0.0,
                        narrow_cmax=0.0, narrow_amin=0.0, grid_lo=0.0, grid_inv=0.0, key_lo=klo,
                        key_inv=(1 << key_bits) / (khi - klo) if khi > klo else 0.0,
                        family=fam, flags=(N.F_HAS_LOW if post.low is not None else 0)
                        | (N.F_HAS_HIGH if post.high is not None else 0),
                        low=post.low if post.low is not None else 0.0,
                        high=post.high if post.high is not None else 0.0,
                        q=post.q if post.q is not None else 0.0, n_upper=post.upper)
            st = parzen.sampler_table(post)
            info['samp_off'], info['samp_len'] = ns, st.shape[0]
            if fam == N.FAM_CATEGORICAL and 0 < st.shape[0] <= 64 and len(post.above[0]) == st.shape[0]:
                # TPE_F_CAT_LAZY: best-scoring drawable category selected with p >= 2^-16
                c1, s1, p1 = -1, 0.0, 0.0
                for i in range(st.shape[0]):
                    pi = st[i, 0] - (st[i - 1, 0] if i else 0.0)
                    if not pi > 0:
                        continue
                    pa = float(post.above[0][i])
                    sc = math.log(float(post.below[0][i])) - (math.log(pa) if pa > 0 else -math.inf)
                    if c1 < 0 or ((s1 == s1) if sc != sc else sc > s1):
                        c1, s1, p1 = i, sc, pi
                if c1 >= 0 and p1 >= 1.0 / 65536:
                    info['flags'] |= N.F_CAT_LAZY
            samp.append(st)
            ns += st.shape[0]
            if fam == N.FAM_CATEGORICAL:
                for side in ('below', 'above'):
                    p = np.asarray(getattr(post, side)[0], dtype=float)
                    r = np.zeros((len(p), 4))
                    with np.errstate(divide='ignore'):
                        r[:, 0] = np.log(p)
                    r[:, 1] = p
                    info[side + '_off'], info[side + '_len'] = n64, len(p)
                    info[side + '_base'] = 0.0
                    comp64.append(r)
                    n64 += len(p)
            elif fam in (N.FAM_QGAUSS, N.FAM_QLOGGAUSS):
                for side in ('below', 'above'):
                    w, mu, sg = getattr(post, side)
                    m, b, ww, base = parzen.quant_table(w, mu, sg, post)
                    r = np.zeros((len(w), 4))
                    r[:, 0], r[:, 1], r[:, 2] = m, b, ww
                    info[side + '_off'], info[side + '_len'] = n64, len(w)
                    info[side + '_base'] = base
                    comp64.append(r)
                    n64 += len(w)
            else:
                logf = fam == N.FAM_LOGGAUSS
                for side in ('below', 'above'):
                    w, mu, sg = getattr(post, side)
                    m, a, c, base = parzen.gauss_table(w, mu, sg, post, logf)
                    info[side + '_base'] = base
                    if f64:
                        r = np.zeros((len(w), 4))
                        r[:, 0], r[:, 1], r[:, 2] = m, a, c
                        info[side + '_off'], info[side + '_len'] = n64, len(w)
                        comp64.append(r)
                        n64 += len(w)
                    else:
                        meta, wide, cn = None, None, c
                        if side == 'above' and pl['mode'] == N.TAB_NONE:     # tabulated: no pruning
                            cn, wide, meta = parzen.prune_tables(m, a, c)
                        r = _rows32(m, a, cn)
                        info[side + '_off'], info[side + '_len'] = n32, len(w)
                        comp32.append(r)
                        n32 += len(w)
                        if meta is not None:
                            comp32.append(_rows32(m[wide], a[wide], c[wide]))
                            info['wide_off'], info['wide_len'] = n32, len(wide)
                            n32 += len(wide)
                            g = meta.pop('grid')
                            info['grid_off'], info['grid_n'] = ngrid, len(g) - 1
                            grids.append(g)
                            ngrid += len(g)
                            info.update(meta)
            rows.append(info)

        # score tables: 16-B units, a cell row 3 units, a lattice row 1
        units, jobs, blocks, r0 = 0, [], 0, 0
        for lp, pl, info in zip(problems, plans, rows):
            info['tab_mode'], info['tab_off'], info['tab_n'] = pl['mode'], [0, 0], [0, 0]
            info['tab_lo'], info['tab_inv'], info['lat_lo'] = [0.0, 0.0], [0.0, 0.0], 0
            if pl['mode'] == N.TAB_CELLS and pl.get('logpoly'):
                n = pl['n'][0]                  # one table, both sides' polynomials in each row
                info['flags'] = info['flags'] | N.F_LOGPOLY
                for sd in range(2):
                    info['tab_off'][sd], info['tab_n'][sd] = units, n
                    info['tab_lo'][sd] = float(np.float32(pl['lo']))
                    info['tab_inv'][sd] = float(np.float32(n / (pl['hi'] - pl['lo'])))
                units += N.TAB_ROW_UNITS * n
            elif pl['mode'] == N.TAB_CELLS:
                for sd in range(2):
                    n = pl['n'][sd]
                    info['tab_off'][sd], info['tab_n'][sd] = units, n
                    info['tab_lo'][sd] = float(np.float32(pl['lo']))
                    info['tab_inv'][sd] = float(np.float32(n / (pl['hi'] - pl['lo'])))
                    units += N.TAB_ROW_UNITS * n
            elif pl['mode'] == N.TAB_LATTICE:
                info['tab_off'][0], info['tab_n'][0], info['lat_lo'] = units, pl['n'][0], pl['lat_lo']
                units += pl['n'][0] + (pl['n'][0] + 1 + 3) // 4      # rows, then n + 1 f32 entry thresholds
            if pl['mode'] != N.TAB_NONE and len(lp.ids):
                for sd in range(2 if pl['mode'] == N.TAB_CELLS else 1):
                    geo = (0, 0, 0, 0, 0.0, 0.0)
                    if pl['mode'] == N.TAB_CELLS:     # the side's rows and cell geometry
                        side = 'above' if sd else 'below'
                        geo = (info[side + '_off'], info[side + '_len'], info.get('wide_off', 0) if sd else 0,
                               info.get('wide_len', 0) if sd else 0, info['tab_lo'][sd], info['tab_inv'][sd])
                    kind = N.TAB_LOGPOLY if pl.get('logpoly') else pl['mode']
                    jobs.append((r0, sd, kind, info['tab_n'][sd], info['tab_off'][sd], blocks) + geo)
                    n = info['tab_n'][sd]        # cells: TAB_PER_BLOCK rows a block; lattice: a block a value
                    if kind == N.TAB_LOGPOLY and geo[1] >= 0 and geo[1] + geo[3] <= LP_DIRECT_ROWS:
                        blocks += -(-n // (LP_ROWS_PER_WAVE * N.TAB_PER_BLOCK))    # (a short side: direct sums)
                    elif kind == N.TAB_CELLS and geo[1] >= 0 and geo[1] + geo[3] <= MOM_DIRECT_ROWS:
                        blocks += -(-n // (MOM_CELLS_PER_WAVE * N.TAB_PER_BLOCK))  # (a short moment side)
                    else:
                        blocks += -(-n // N.TAB_PER_BLOCK) if pl['mode'] == N.TAB_CELLS else n
            r0 += len(lp.ids)
        tj = np.zeros(len(jobs), dtype=N.TAB_JOB_DTYPE)
        for c, f in enumerate(N.TAB_JOB_DTYPE.names):
            tj[f] = [jb[c] for jb in jobs]

        # problems: one row per (LevelProblem, id)
        counts = np.array([len(lp.ids) for lp in problems], dtype=np.int64)
        P = int(counts.sum())
        prob = np.zeros(P, dtype=N.PROBLEM_DTYPE)
        owner = np.repeat(np.arange(len(problems)), counts)
        for field in ('family', 'flags', 'n_upper', 'samp_off', 'samp_len', 'below_off', 'below_len',
                      'above_off', 'above_len', 'low', 'high', 'q', 'below_base', 'above_base',
                      'wide_off', 'wide_len', 'grid_off', 'grid_n', 'prior_mu', 'prior_a', 'prior_c',
                      'narrow_cmax', 'narrow_amin', 'grid_lo', 'grid_inv', 'key_lo', 'key_inv',
                      'tab_mode', 'tab_off', 'tab_n', 'tab_lo', 'tab_inv', 'lat_lo'):
            prob[field] = np.array([r[field] for r in rows])[owner] if P else 0
        prob['n_cand'] = n_cand
        ids = np.concatenate([lp.ids for lp in problems]) if P else np.zeros(0, np.int64)
        pr = np.repeat(np.array(pruned_l, dtype=bool), counts) if P else np.zeros(0, bool)
        # sorted problems own the candidate range [0, n_sorted * n_cand)
        srank = np.cumsum(pr) - 1
        unslot = np.cumsum(~pr) - 1
        prob['cand_off'] = np.where(pr, srank * n_cand, (n_sorted + unslot) * n_cand)
        slots, pool_first, nxt, r = [], [], 0, 0
        for lp, p_, po in zip(problems, pruned_l, pooled_l):
            k = len(lp.ids)
            if po:
                slots += [nxt] * k
                nxt += 1
            elif p_:
                slots += list(range(nxt, nxt + k))
                nxt += k
            else:
                slots += [-1] * k
            pool_first += [r if po else -1] * k
            r += k
        prob['sort_slot'] = slots if P else -1
        prob['pool_first'] = pool_first if P else -1
        pooled = np.repeat(np.array(pooled_l, dtype=bool), counts) if P else np.zeros(0, bool)
        prob['flags'] = prob['flags'] | np.where(pooled, N.F_POOLED, 0)
        prob['cand_base'] = cand_base
        prob['n_cand_global'] = n_cand if not n_cand_global else int(n_cand_global)
        s64 = int(seed) & 0xFFFFFFFFFFFFFFFF
        prob['key0'] = s64 & 0xFFFFFFFF
        prob['key1'] = s64 >> 32
        prob['ctr2'] = np.array([lp.label_ix for lp in problems], dtype=np.uint32)[owner] if P else 0
        prob['ctr3'] = (ids & 0xFFFFFFFF).astype(np.uint32)
        n_tiles_p = (n_cand + T - 1) // T if n_cand > 0 else 0
        prob['n_tiles'] = n_tiles_p
        prob['tile_off'] = np.arange(P, dtype=np.int64) * n_tiles_p

        # splits of the above mixture per tile: bulk tiles fill the chip (a
        # function of the GLOBAL candidate count); pruned problems with many
        # tiles use one split and geometrically more on their outermost tiles
        fam = prob['family']
        untab = prob['tab_mode'] == N.TAB_NONE
        cont = ((fam == N.FAM_GAUSS) | (fam == N.FAM_LOGGAUSS)) & untab
        qg, ql = (fam == N.FAM_QGAUSS) & untab, (fam == N.FAM_QLOGGAUSS) & untab
        scored = cont | qg | ql
        C_ref = n_cand if not n_cand_global else int(n_cand_global)
        tiles_ref = (C_ref + T - 1) // T
        n_scored_tiles = int(scored.sum()) * tiles_ref
        target = max(1, math.ceil(TARGET_WORK / max(n_scored_tiles, 1)))
        K = prob['above_len'].astype(np.int64)
        tails = pr & (tiles_ref >= TAIL_MIN_TILES)
        splits = np.where(scored, np.where(tails, 1, np.clip(np.minimum(target, (K + MIN_COMPONENTS_PER_SPLIT - 1)
                                                                      // MIN_COMPONENTS_PER_SPLIT), 1, None)), 0)
        prob['n_splits'] = splits
        j = np.arange(n_tiles_p)
        e = np.minimum(j, n_tiles_p - 1 - j)
        tail_ns = np.select([e < 6, e < 8, e < 10, e < 12], [16, 8, 4, 2], 1)     # tpe_host.cpp tail_splits
        ns_tile = np.zeros((P, n_tiles_p), dtype=np.int64)
        for r in range(P):
            if not scored[r]:
                continue
            if tails[r]:
                ns_tile[r] = np.maximum(1, np.minimum(tail_ns, max(1, (K[r] + 63) // 64)))
            else:
                ns_tile[r] = splits[r]

        # tiles
        tiles = np.zeros(P * n_tiles_p, dtype=N.TILE_DTYPE)
        tiles['problem'] = np.repeat(np.arange(P), n_tiles_p)
        tiles['cand_start'] = np.tile(np.arange(n_tiles_p) * T, P)
        tiles['n_splits'] = ns_tile.reshape(-1)

        # work items, grouped [continuous | qgauss | qlog], a tile's items consecutive
        works = []
        counts_w = []
        nw = 0
        for mask in (cont, qg, ql):
            pidx = np.nonzero(mask)[0]
            rows_w = []
            for r in pidx:
                for t in range(n_tiles_p):
                    ti = r * n_tiles_p + t
                    tiles['work_first'][ti] = nw
                    ns = int(ns_tile[r, t])
                    for sp in range(ns):
                        rows_w.append((r, sp, t * T, (K[r] * sp) // ns, (K[r] * (sp + 1)) // ns, ns))
                        nw += 1
            w = np.array(rows_w, dtype=np.int64).reshape(-1, 6)
            wa = np.zeros(len(w), dtype=N.WORK_DTYPE)
            for c, f in enumerate(N.WORK_DTYPE.names):
                wa[f] = w[:, c]
            works.append(wa)
            counts_w.append(len(wa))
        work = np.concatenate(works) if works else np.zeros(0, dtype=N.WORK_DTYPE)
        part_total = nw * T

        return dict(prob=prob, tiles=tiles, work=work, counts_w=counts_w, part_total=part_total, tab_jobs=tj,
                    tab_units=units, tab_blocks=blocks,
                    comp32=np.concatenate(comp32) if comp32 else np.zeros((0, 4), np.float32),
                    comp64=np.concatenate(comp64) if comp64 else np.zeros((0, 4)),
                    grid=np.concatenate(grids) if grids else np.zeros(1, np.int32),
                    samp=np.concatenate(samp) if samp else np.zeros((0, 8)), P=P)

    # ---------------------------------------------------------------- pack
    @staticmethod
    def _labels(problems):
        """tpe_label_in array of one level (LABEL_DTYPE records; returns its
        address) plus the arrays it points into, which the caller keeps alive
        for the native call.  One tuple assignment per label."""
        n = len(problems)
        recs = np.zeros(max(n, 1), dtype=N.LABEL_DTYPE)
        keep = [recs]
        id_addr = {}                              # the level's problems usually share one ids array
        # room for every device-fitted label's merged order first: making room can
        # re-lay out the History's order buffers, which would move addresses
        # already taken (devhist)
        grow = {}
        for lp in problems:
            ad = lp.post.above_dev
            if ad is not None:
                g = grow.setdefault(id(ad[3].group), (ad[3].group, [], []))
                g[1].append(ad[3].slot)
                g[2].append(ad[1])
        for g, slots, ns in grow.values():
            g.ensure(slots, ns)
        for i, lp in enumerate(problems):
            post = lp.post
            flags = (N.F_HAS_LOW if post.low is not None else 0) | (N.F_HAS_HIGH if post.high is not None else 0)
            if lp.inject is not None:        # caller-drawn candidates need not lie on a quantization lattice
                flags |= N.F_NO_TABLE
            ids = lp.ids                          # int64, contiguous (LevelProblem)
            if post.ptrs is not None and post.above_dev is None:
                # native fits: the addresses are known; the posterior owns the arrays
                keep.append(post)
                pt = post.ptrs
                ia = id_addr.get(id(ids))
                if ia is None:
                    ia = id_addr[id(ids)] = ids.ctypes.data
                recs[i] = (post.family, flags, int(post.upper), lp.label_ix,
                           post.low if post.low is not None else 0.0, post.high if post.high is not None else 0.0,
                           post.q if post.q is not None else 0.0,
                           pt[0], pt[1], pt[2], pt[3], pt[4], pt[5], pt[6], pt[7],
                           ia, len(ids), 0, 0, 0, 0, 0, 0.0, 0.0, 0.0, 0, 0, 0, 0, 0)
                continue
            bw = [np.ascontiguousarray(a, dtype=np.float64) for a in post.below]
            ids = np.ascontiguousarray(lp.ids, dtype=np.int64)
            keep.append(bw)
            keep.append(ids)
            bptr = [a.ctypes.data for a in bw] + [0] * (3 - len(bw))
            if post.above_dev is not None:
                col, n_obs, bidx, order = post.above_dev
                bidx = np.ascontiguousarray(bidx, dtype=np.int32)
                keep.append(bidx)
                aptr, ak = [0, 0, 0], n_obs - len(bidx) + 1
                dev = (col.data_ptr(), n_obs, bidx.ctypes.data, len(bidx))
                prior = post.prior
                ordp = order.ptrs(n_obs)          # the label's resident value order (ValueOrder)
            else:
                aw = [np.ascontiguousarray(a, dtype=np.float64) for a in post.above]
                keep.append(aw)
                aptr, ak = [a.ctypes.data for a in aw] + [0] * (3 - len(aw)), len(aw[0])
                dev, prior, ordp = (0, 0, 0, 0), (0.0, 0.0, 0.0, 0), (0, 0, 0, 0, 0)
            recs[i] = (post.family, flags, int(post.upper), lp.label_ix,
                       post.low if post.low is not None else 0.0, post.high if post.high is not None else 0.0,
                       post.q if post.q is not None else 0.0,
                       bptr[0], bptr[1], bptr[2], len(bw[0]), aptr[0], aptr[1], aptr[2], ak,
                       ids.ctypes.data, len(ids), dev[0], dev[1], dev[2], dev[3], prior[3],
                       prior[0], prior[1], prior[2]) + ordp
        return recs.ctypes.data, keep

    @staticmethod
    def _commit_orders(problems):
        """A level with these problems was enqueued: the device-fitted labels'
        merged value orders are now their resident orders (stream order makes
        them valid for every later launch on the stream)."""
        for lp in problems:
            ad = lp.post.above_dev
            if ad is not None:
                ad[3].commit(ad[1])

    def _pack(self, problems, n_cand, seed, cand_base, n_cand_global):
        """Pack one level with the native host runtime straight into the pinned
        staging buffer; returns the PackInfo."""
        n = len(problems)
        labels, keep = self._labels(problems)
        info = N.PackInfo()
        prec = N.PREC_F64 if self.precision == 'fp64' else N.PREC_F32
        seed64 = int(seed) & 0xFFFFFFFFFFFFFFFF
        ncg = int(n_cand_global) if n_cand_global is not None else 0
        for attempt in range(2):
            host = self._pinned
            cap = host.numel() if host is not None else 0
            rc = self.lib.tpe_host_pack_level(labels, n, int(n_cand), seed64, int(cand_base), ncg, prec,
                                              host.data_ptr() if host is not None else None, cap,
                                              ctypes.byref(info))
            if rc == N.E_SPACE:
                self._pinned = torch.empty(max(info.blob_bytes, 2 * cap), dtype=torch.uint8,
                                           pin_memory=torch.cuda.is_available())
                self._ws = None
                continue
            N.check(rc, self.lib, 'tpe_host_pack_level')
            break
        return info

    def _flags(self):
        # (TPE_DEBUG_FLAGS is read per call: tests switch it on around single runs)
        return (0 if self.expand else N.BATCH_NO_EXPAND) | (0 if self.fuse else N.BATCH_NO_FUSE) | \
            int(os.environ.get('TPE_DEBUG_FLAGS', '0'))

    # ----------------------------------------------------- one-call level
    def _level_ws(self):
        """tpe_level_ws over the engine's pools (rebuilt when a pool grows)."""
        ws = self._ws
        if ws is not None:
            return ws
        B = self._bufs
        ws = N.LevelWS()

        def dev(name, itemsize):
            t = B.get(name)
            return (t.data_ptr(), t.numel() * t.element_size() // itemsize) if t is not None else (None, 0)
        pin = self._pinned
        ws.pinned, ws.pinned_bytes = (pin.data_ptr(), pin.numel()) if pin is not None else (None, 0)
        if pin is not None:            # the staging buffer's device address, once per allocation
            dp = ctypes.c_void_p()
            N.check(self.lib.tpe_pinned_device_address(pin.data_ptr(), ctypes.byref(dp)), self.lib,
                    'tpe_pinned_device_address')
            ws.pinned_dev = dp.value
        ws.blob, ws.blob_bytes = dev('blob', 1)
        ws.cand, n1 = dev('cand', 8)
        ws.coord, n2 = dev('coord', 4)
        ws.keys, n3 = dev('keys', 4)
        ws.vals, n4 = dev('vals', 8)
        ws.keys_sorted, n5 = dev('keys_sorted', 4)
        ws.vals_sorted, n6 = dev('vals_sorted', 8)
        ws.cand_cap = min(n1, n2, n3, n4, n5, n6)
        ws.sort_tmp, ws.sort_tmp_bytes = dev('sort_tmp', 1)
        ws.part, ws.part_cap = dev('part', 8)
        ws.tile_best, ws.best_cap = dev('best', 32)
        ws.result, ws.result_cap = dev('result', 48)
        ws.fit_keys, f1 = dev('fit_keys', 8)
        ws.fit_keys_sorted, f2 = dev('fit_keys_sorted', 8)
        ws.fit_vals, f3 = dev('fit_vals', 4)
        ws.fit_vals_sorted, f4 = dev('fit_vals_sorted', 4)
        ws.fit_cap = min(f1, f2, f3, f4)
        ws.draw_pref, ws.draw_pref_cap = dev('draw_pref', 8)
        ws.pool_best, ws.pool_best_cap = dev('pool_best', 8)
        ws.tab, ws.tab_cap = dev('tab', 16)
        self._ws = ws
        return ws

    def _grow(self, need):
        if need.pinned_bytes > (self._pinned.numel() if self._pinned is not None else 0):
            self._pinned = torch.empty(int(need.pinned_bytes * 1.25) + 4096, dtype=torch.uint8,
                                       pin_memory=torch.cuda.is_available())
        self._buf('blob', need.blob_bytes, torch.uint8)
        for name, dt in (('cand', torch.float64), ('coord', torch.float32), ('keys', torch.int32),
                         ('vals', torch.int64), ('keys_sorted', torch.int32), ('vals_sorted', torch.int64)):
            self._buf(name, need.cand, dt)
        self._buf('sort_tmp', need.sort_tmp_bytes, torch.uint8)
        self._buf('part', need.part, torch.float64)
        self._buf('best', need.best * 4, torch.float64)
        self._buf('result', need.result * 6, torch.float64)
        for name, dt in (('fit_keys', torch.float64), ('fit_keys_sorted', torch.float64),
                         ('fit_vals', torch.int32), ('fit_vals_sorted', torch.int32)):
            self._buf(name, need.fit, dt)
        self._buf('draw_pref', need.draw_pref, torch.float64)
        self._buf('pool_best', need.pool_best, torch.int64)
        self._buf('tab', 4 * need.tab, torch.float32)
        self._ws = None

    def run_level(self, problems, n_cand, seed, cand_base=0, n_cand_global=None):
        """``run`` for device-drawn candidates without per-candidate outputs:
        one native call (tpe_level_run) packs, uploads, launches every stage
        and reads the per-problem results back.  Returns RESULT_DTYPE [P]."""
        n_cand = int(n_cand)
        if n_cand < 0 or n_cand >= 2 ** 31:
            raise ValueError('n_EI_candidates out of range: %r' % n_cand)
        labels, keep = self._labels(problems)
        P = sum(len(lp.ids) for lp in problems)
        out = np.empty(P, dtype=N.RESULT_DTYPE)
        need = N.LevelNeed()
        prec = N.PREC_F64 if self.precision == 'fp64' else N.PREC_F32
        seed64 = int(seed) & 0xFFFFFFFFFFFFFFFF
        ncg = int(n_cand_global) if n_cand_global is not None else 0
        stream = self._stream()
        prof = self.profile is not None
        if prof:
            N.check(self.lib.tpe_level_profile(1), self.lib, 'tpe_level_profile')
        for attempt in range(3):
            ws = self._level_ws()
            rc = self.lib.tpe_level_run(labels, len(problems), n_cand, seed64, int(cand_base), ncg, prec,
                                        self._flags(), ctypes.byref(ws),
                                        ctypes.byref(need), stream, out.ctypes.data)
            if rc != N.E_SPACE:
                break
            self._grow(need)
        if prof:
            self.lib.tpe_level_profile(0)
        N.check(rc, self.lib, 'tpe_level_run')
        self._commit_orders(problems)
        del keep
        if prof and P:
            self._record_level_profile()
        return out

    def suggest_tree(self, labels, below_sorted, prior_weight, lf, ids, n_cand, seed, min_draws, flags=0,
                     shard=None, exchange=None, labels_ptr=None):
        """A whole tpe.suggest of a tree space in one native call
        (tpe_suggest_tree): fits, gate prediction and level runs.  ``labels``:
        TREE_LABEL_DTYPE records in label order (``labels_ptr``: their address,
        when the caller keeps it); ``below_sorted``: int64 ascending below
        tids; ``shard`` = (rank, world) with ``exchange`` (a dist._Exchange):
        this rank scores its range of the ``n_cand`` candidates and the native
        call exchanges every level's results.
        Returns (values, active) [n_ids x n_labels] — views of the engine's
        result buffers, valid until its next suggest_tree — or (None,
        need_fit) on TPE_E_FALLBACK: need_fit [n_labels] flags the labels the
        caller must fit and pass back (none: take the general path)."""
        if self.precision != 'fp32':
            return None, np.zeros(len(labels), dtype=np.int8)
        self.tree_calls += 1
        n_cand = int(n_cand)
        if n_cand < 0 or n_cand >= 2 ** 31:
            raise ValueError('n_EI_candidates out of range: %r' % n_cand)
        nl, n, nb = len(labels), len(ids), len(below_sorted)
        io = self._tree_io
        if io is None or io.n_cap < n or io.l_cap < nl or io.b_cap < nb:
            io = self._tree_io = _TreeIO(n, nl, nb, io)
        # arguments into the persistent buffers (their addresses are cached:
        # an ndarray's .ctypes costs microseconds per access)
        io.ids[:n] = ids
        io.below[:nb] = below_sorted
        io.need_fit[:nl] = 0
        if labels_ptr is None:
            labels_ptr = labels.ctypes.data
        path, need = self._tree_out
        seed64 = int(seed) & 0xFFFFFFFFFFFFFFFF
        stream = self._stream()
        prof = self.profile is not None
        if prof:
            N.check(self.lib.tpe_level_profile(1), self.lib, 'tpe_level_profile')
        c_loc, base, c_glob, ex = n_cand, 0, 0, None
        if shard is not None:
            from .dist import shard_range
            base, hi = shard_range(n_cand, shard[0], shard[1])
            c_loc, c_glob = hi - base, n_cand
            ex = exchange.ptr(nl * n, c_loc)
        # an unsharded call through the trampoline (it ORs in TPE_DEBUG_FLAGS);
        # a sharded one through ctypes (the exchange struct is a ctypes object)
        tramp = _CALL_TREE is not None and ex is None
        fl = ((0 if self.expand else N.BATCH_NO_EXPAND) | (0 if self.fuse else N.BATCH_NO_FUSE) | int(flags)) \
            if tramp else self._flags() | int(flags)
        for attempt in range(8):          # a later tree level may need larger pools than the first
            ws = self._level_ws()
            if tramp:
                a_path, a_need, fn = self._tree_addr
                rc = _CALL_TREE(fn, labels_ptr, nl, io.below_ptr, nb, float(prior_weight), int(lf), io.ids_ptr, n,
                                c_loc, base, c_glob, 0, seed64, float(min_draws), int(self.device_fit_min), fl,
                                ctypes.addressof(ws), a_need, stream or 0, io.values_ptr, io.active_ptr, a_path,
                                io.need_fit_ptr)
            else:
                rc = self.lib.tpe_suggest_tree(labels_ptr, nl, io.below_ptr, nb, float(prior_weight), int(lf),
                                               io.ids_ptr, n, c_loc, base, c_glob, ex, seed64, float(min_draws),
                                               int(self.device_fit_min), fl, ctypes.byref(ws), ctypes.byref(need),
                                               stream, io.values_ptr, io.active_ptr, path, io.need_fit_ptr)
            if rc != N.E_SPACE:
                break
            self._grow(need)
        if prof:
            self.lib.tpe_level_profile(0)
        if rc == N.E_FALLBACK:
            return None, io.need_fit[:nl].copy()
        N.check(rc, self.lib, 'tpe_suggest_tree')
        self.last_tree_path = (int(path[0]), int(path[1]))
        if prof and path[1]:
            self._record_level_profile()
        return io.values[:n * nl].reshape(n, nl), io.active[:n * nl].reshape(n, nl)

    def _record_level_profile(self):
        """profile[stage] gets (ms, units, algorithmic CE) of every stage the
        last tpe_level_run launched, timed by the runner's own HIP events on
        its stream (tpe_level_profile): the production flow, stage by stage."""
        recs = (N.StageProf * len(N.STAGES))()
        N.check(self.lib.tpe_level_profile_read(recs, len(N.STAGES)), self.lib, 'tpe_level_profile_read')
        for name, r in zip(N.STAGES, recs):
            if r.launches:
                self.profile.setdefault(name, []).append((float(r.ms), float(r.units), float(r.ce),
                                                          1e-6 * float(r.kernel_ns)))

    # ---------------------------------------------------------------- run
    def run(self, problems, n_cand, seed, cand_base=0, want_lg=False, return_cand=False, n_cand_global=None):
        """Sample, score and select every problem of one level.

        Returns a RESULT_DTYPE array with one row per (LevelProblem, id) in
        order, plus (cand, l, g) float64 [P, n_cand] arrays when requested."""
        n_cand = int(n_cand)
        if n_cand < 0 or n_cand >= 2 ** 31:
            raise ValueError('n_EI_candidates out of range: %r' % n_cand)
        info = self._pack(problems, n_cand, seed, cand_base, n_cand_global)
        self._last_info = info
        P = int(info.n_problems)
        if P == 0:
            return np.zeros(0, dtype=N.RESULT_DTYPE)
        C_total = P * n_cand
        if C_total >= 2 ** 32:
            raise ValueError('more than 2^32 candidates in one level: shard the batch')
        nbytes = int(info.blob_bytes)
        dev = self._buf('blob', nbytes, torch.uint8)
        # host-written ranges only: device-fitted rows are produced by tpe_fit_above
        for i in range(int(info.n_up)):
            o, n = int(info.up_off[i]), int(info.up_len[i])
            dev[o:o + n].copy_(self._pinned[o:o + n], non_blocking=True)
        base = dev.data_ptr()
        prob = np.frombuffer(self._pinned.numpy(), dtype=N.PROBLEM_DTYPE, count=P, offset=int(info.off_problems))
        d_cand = self._buf('cand', C_total, torch.float64)
        d_coord = self._buf('coord', C_total, torch.float32)
        d_part = self._buf('part', info.part_total, torch.float64)
        n_tiles = int(info.n_tiles)
        d_best = self._buf('best', n_tiles * N.BEST_PER_TILE * 4, torch.float64)
        d_res = self._buf('result', P * 6, torch.float64)
        d_keys = self._buf('keys', C_total, torch.int32)
        d_vals = self._buf('vals', C_total, torch.int64)
        # sort only when some problem of the level prunes its above mixture
        sort = info.sort_end_bit > 0
        if sort:
            d_keys_s = self._buf('keys_sorted', C_total, torch.int32)
            d_vals_s = self._buf('vals_sorted', C_total, torch.int64)
            ws = ctypes.c_uint64(0)
            N.check(self.lib.tpe_sort_workspace_bytes(int(info.sort_count), ctypes.byref(ws)), self.lib,
                    'tpe_sort_workspace_bytes')
            d_sort = self._buf('sort_tmp', ws.value, torch.uint8)
        else:
            d_keys_s, d_vals_s, d_sort = d_keys, d_vals, None
        inject = any(lp.inject is not None for lp in problems)
        if inject:
            if not all(lp.inject is not None for lp in problems):
                raise ValueError('either every problem of a level injects candidates or none does')
            cand = np.concatenate([np.asarray(lp.inject, dtype=np.float64).reshape(len(lp.ids), n_cand)
                                   for lp in problems]).reshape(-1)
            fam = np.repeat(prob['family'], n_cand)
            with np.errstate(divide='ignore', invalid='ignore'):
                coord = np.where((fam == N.FAM_LOGGAUSS) | (fam == N.FAM_QLOGGAUSS), np.log(cand), cand)
            cat = fam == N.FAM_CATEGORICAL
            if cat.any():
                upper = np.repeat(prob['n_upper'], n_cand)[cat]
                cv = cand[cat]
                if np.any((cv < 0) | (cv >= upper) | (cv != np.floor(cv))):
                    raise IndexError('categorical candidate out of range')
            # problem r's candidates live at cand_off[r] (sorted problems first)
            at = (prob['cand_off'][:, None] + np.arange(n_cand)[None, :]).reshape(-1)
            placed, placed_t = np.empty(C_total), np.empty(C_total, dtype=np.float32)
            placed[at] = cand
            placed_t[at] = coord.astype(np.float32)
            d_cand[:C_total].copy_(torch.from_numpy(placed))
            d_coord[:C_total].copy_(torch.from_numpy(placed_t))
        d_l = d_g = None
        if want_lg:
            d_l = self._buf('l_out', C_total, torch.float64)
            d_g = self._buf('g_out', C_total, torch.float64)
        b = N.Batch()
        b.problems, b.n_problems = base + info.off_problems, P
        b.precision = N.PREC_F64 if self.precision == 'fp64' else N.PREC_F32
        b.flags = self._flags() | (N.BATCH_WRITE_CAND if (return_cand or want_lg) else 0)
        b.sample = 0 if inject else 1
        b.sort_end_bit, b.key_bits = info.sort_end_bit, info.key_bits
        b.comp32, b.comp64 = base + info.off_comp32, base + info.off_comp64
        b.samp, b.grid = base + info.off_samp, base + info.off_grid
        b.keys, b.vals = d_keys.data_ptr(), d_vals.data_ptr()
        b.keys_sorted, b.vals_sorted = d_keys_s.data_ptr(), d_vals_s.data_ptr()
        if d_sort is not None:
            b.sort_tmp, b.sort_tmp_bytes = d_sort.data_ptr(), d_sort.numel()
        b.total_cand = C_total
        b.sort_count = info.sort_count
        b.cand, b.coord = d_cand.data_ptr(), d_coord.data_ptr()
        b.tiles, b.n_tiles = base + info.off_tiles, n_tiles
        b.fin_tiles, b.n_fin_tiles = base + info.off_fin_tiles, info.n_fin_tiles
        b.work = base + info.off_work
        b.n_work_cont, b.n_work_qgauss, b.n_work_qlog = info.n_work_cont, info.n_work_qgauss, info.n_work_qlog
        b.part = d_part.data_ptr()
        b.l_out = d_l.data_ptr() if d_l is not None else None
        b.g_out = d_g.data_ptr() if d_g is not None else None
        b.tile_best, b.result = d_best.data_ptr(), d_res.data_ptr()
        if info.n_pooled:
            b.pool_best = self._buf('pool_best', P, torch.int64).data_ptr()
        b.samp_tiles, b.n_samp_tiles, b.n_samp_eager = base + info.off_samp_tiles, info.n_samp_tiles, info.n_samp_eager
        b.tab_tiles, b.n_tab_tiles = base + info.off_tab_tiles, info.n_tab_tiles
        if info.n_tab_jobs:
            b.tab_jobs, b.n_tab_jobs, b.tab_blocks = base + info.off_tab_jobs, info.n_tab_jobs, info.tab_blocks
            b.tab = self._buf('tab', 4 * int(info.tab_units), torch.float32).data_ptr()
            b.tab_units = info.tab_units
            b.fgt_max_boxes = info.fgt_max_boxes
            b.fgt_max_cells = info.fgt_max_cells
        if info.n_sorted and not inject and not info.n_pooled:
            b.n_sorted, b.draw_blocks = info.n_sorted, info.draw_blocks
            b.draw_pref = self._buf('draw_pref', int(info.n_sorted) * (int(info.draw_blocks) + 1),
                                    torch.float64).data_ptr()
        if info.n_fit:
            ft = int(info.fit_total)
            d_fk = self._buf('fit_keys', ft, torch.float64)
            d_fks = self._buf('fit_keys_sorted', ft, torch.float64)
            d_fv = self._buf('fit_vals', ft, torch.int32)
            d_fvs = self._buf('fit_vals_sorted', ft, torch.int32)
            b.fit, b.n_fit = base + info.off_fit, info.n_fit
            b.below_idx, b.fit_seg, b.fit_total = base + info.off_below_idx, base + info.off_fit_seg, ft
            b.fit_keys, b.fit_keys_sorted = d_fk.data_ptr(), d_fks.data_ptr()
            b.fit_vals, b.fit_vals_sorted = d_fv.data_ptr(), d_fvs.data_ptr()
            b.fit_max_new, b.fit_max_obs, b.fit_max_merge = info.fit_max_new, info.fit_max_obs, info.fit_max_merge
            b.fit_n_delta = info.fit_n_delta
        stream = self._stream()
        if self.profile is None:
            N.check(self.lib.tpe_run_batch(ctypes.byref(b), ctypes.c_void_p(stream)), self.lib, 'tpe_run_batch')
        else:
            tb = dict(prob=prob.copy(), counts_w=[info.n_work_cont, info.n_work_qgauss, info.n_work_qlog], P=P)
            self._run_profiled(b, stream, tb, n_cand)
        self._commit_orders(problems)
        res = d_res[:P * 6].cpu().numpy().view(N.RESULT_DTYPE).copy()
        if not (want_lg or return_cand):
            return res
        out = [res]
        rows = (prob['cand_off'] // max(n_cand, 1)).astype(np.int64)    # sorted problems come first

        def per_problem(d):
            return d[:C_total].cpu().numpy().reshape(P, n_cand)[rows].copy()
        if return_cand:
            out.append(per_problem(d_cand))
        if want_lg:
            out.append(per_problem(d_l))
            out.append(per_problem(d_g))
        return tuple(out)

    def device_tables(self):
        """(problems, comp32) of the last ``run`` as the device holds them after
        its stages ran — device-fitted above rows and the problem fields the fit
        patches included (tests of the device Parzen fit read them back)."""
        info = self._last_info
        nb = int(info.blob_bytes)
        blob = self._bufs['blob'][:nb].cpu().numpy()
        prob = np.frombuffer(blob, dtype=N.PROBLEM_DTYPE, count=int(info.n_problems),
                             offset=int(info.off_problems)).copy()
        o = int(info.off_comp32)
        comp32 = np.frombuffer(blob[o:o + (nb - o) // 16 * 16], dtype=np.float32).reshape(-1, 4).copy()
        return prob, comp32

    def _run_profiled(self, b, stream, tb, n_cand):
        """The same launches as tpe_run_batch, one stage at a time, bracketed
        by events on the launch stream (bench.py's roofline measurement).
        profile[name] gets (ms, units) per launch: units = algorithmic CE for
        the above kernels (+ exact CE, expanded components and candidates for
        k_above_f32), algorithmic bytes for the sort, candidates otherwise."""
        prob = tb['prob']
        fam = prob['family']
        ce = (prob['above_len'].astype(np.float64) * n_cand)
        groups = [((fam == N.FAM_GAUSS) | (fam == N.FAM_LOGGAUSS),
                   'k_above_f32' if self.precision == 'fp32' else 'k_above_f64'),
                  (fam == N.FAM_QGAUSS, 'k_above_qgauss'), (fam == N.FAM_QLOGGAUSS, 'k_above_qlog')]
        counts = list(tb['counts_w'])
        stages = []
        if b.n_fit:
            stages.append(('fit', self.lib.tpe_fit_above, None, float(b.fit_total)))
        if b.n_tab_jobs:
            stages.append(('k_tables', self.lib.tpe_tables, None, float(b.tab_units)))
        stages.append(('k_sample', self.lib.tpe_sample, None, float(tb['P'] * n_cand)))
        ordered = (bool(b.draw_pref) and b.sample and b.precision == N.PREC_F32 and b.n_sorted > 0
                   and (b.flags & N.BATCH_ORDERED_DRAWS))
        if b.sort_end_bit and b.sort_count and not ordered:     # ordered draws need no sort
            # units: bytes of an LSD radix sort of (u32 key, u64 value) pairs —
            # every 8-bit pass reads and writes both arrays
            passes = (int(b.sort_end_bit) + 7) // 8
            stages.append(('sort', self.lib.tpe_sort, None, float(passes * 2 * 12 * int(b.sort_count))))
        for gi, (mask, name) in enumerate(groups):
            if counts[gi]:
                stages.append((name, self.lib.tpe_score_above, gi, float(ce[mask].sum())))
        stages.append(('k_finalize', self.lib.tpe_finalize, None, float(tb['P'] * n_cand)))
        stages.append(('k_select', self.lib.tpe_select, None, float(tb['P'])))
        cnt = self._buf('ce_count', 2 * max(counts[0], 1), torch.int64)
        cnt.zero_()
        b.ce_count = cnt.data_ptr()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(stages) + 1)]
        cur = torch.cuda.current_stream(self.device)
        evs[0].record(cur)
        work0 = b.work
        rep = max(1, int(self.profile_repeat))
        for i, (name, fn, gi, units) in enumerate(stages):
            arg = b
            if gi is not None:
                arg = N.Batch.from_buffer_copy(b)
                arg.n_work_cont, arg.n_work_qgauss, arg.n_work_qlog = [c if j == gi else 0 for j, c in
                                                                       enumerate(counts)]
                arg.work = work0 + N.WORK_DTYPE.itemsize * sum(counts[:gi])   # this group's first item
            for _ in range(rep):
                N.check(fn(ctypes.byref(arg), ctypes.c_void_p(stream)), self.lib, name)
            evs[i + 1].record(cur)
        evs[-1].synchronize()
        self.last_ce = cnt[:2 * counts[0]].view(-1, 2).cpu().numpy() if counts[0] else None   # per work item
        cc = cnt[:2 * counts[0]].view(-1, 2).sum(0).tolist() if counts[0] else [0, 0]
        executed, expanded = int(cc[0]), int(cc[1])
        b.ce_count = None
        for i, (name, fn, gi, units) in enumerate(stages):
            rec = (evs[i].elapsed_time(evs[i + 1]) / rep, units)
            if name == 'k_sample':
                # algorithmic component evaluations of the tabulated problems (C x K
                # per problem: what the reference evaluates; the tables do not)
                tabp = prob['tab_mode'] != N.TAB_NONE
                rec = rec + (float(((prob['below_len'] + prob['above_len'])[tabp]).astype(np.float64).sum()
                                   * n_cand),)
            if name == 'k_above_f32':
                n_c = float(((fam == N.FAM_GAUSS) | (fam == N.FAM_LOGGAUSS)).sum() * n_cand)
                rec = rec + (float(executed), float(expanded), n_c)
            self.profile.setdefault(name, []).append(rec)


_ENGINES = {}
_CURRENT = {}      # device index -> its engine key (get_engine without a device)


def get_engine(device=None, precision='fp32'):
    """Process-wide engine per device (buffers are reused across suggests)."""
    if torch is None:
        raise N.NativeUnavailable('torch is required for device memory')
    if device is None:
        # (an engine already made for the current device: no availability query per suggest)
        eng = _ENGINES.get(_CURRENT.get(torch.cuda.current_device()) if _CURRENT else None)
        if eng is not None:
            eng.set_precision(precision)
            return eng
        if not torch.cuda.is_available():
            raise N.NativeUnavailable('no HIP device visible: the TPE engine has no CPU fallback')
        device = torch.device('cuda', torch.cuda.current_device())
        _CURRENT[device.index] = str(device)
    key = str(device)
    eng = _ENGINES.get(key)
    if eng is None:
        eng = _ENGINES[key] = Engine(device, precision)
    eng.set_precision(precision)
    return eng
