/*
 * tpe_hip.h — C-ABI of the MI355X TPE suggest engine (libtpe_hip.so).
 *
 * This boundary replaces the numpy operators that gsmafra/hyperopt evaluates
 * through its pyll interpreter on every tpe.suggest call (reference file:line
 * below).  Plain C types only: device pointers, sizes, an opaque hipStream_t.
 * No allocation, no host synchronisation and no C++ exception crosses it; every
 * entry point returns 0 on success or a negative TPE_E* code, and
 * tpe_last_error() gives a thread-local message.
 *
 * One tpe_run_batch() call evaluates a *batch of problems*.  A problem is one
 * (new_id, hyperparameter) pair of one tree level — the unit the reference
 * handles per parameter in build_posterior (tpe.py:663-701):
 *
 *   sample  C candidates from the "below" Parzen mixture     GMM1 / LGMM1 (tpe.py:62-93, 216-250),
 *                                                           categorical (pyll/stochastic.py:104-142)
 *   score   l(x) = lpdf_below(x),  g(x) = lpdf_above(x)      GMM1_lpdf (tpe.py:104-166),
 *                                                           LGMM1_lpdf (tpe.py:259-301),
 *                                                           categorical_lpdf (tpe.py:50-57)
 *   select  argmax_x  l(x) - g(x), first index on ties      broadcast_best (tpe.py:749-759)
 *
 * The Parzen fit (adaptive_parzen_normal, tpe.py:398-475) and the below/above
 * split (ap_filter_trials, tpe.py:613-641) are done by the caller, which
 * uploads the fitted mixtures as the component tables described below — or,
 * for large continuous above mixtures, left to the device: tpe_fit_above()
 * fits them from device-resident observation columns (see tpe_fit_job).
 */
#ifndef TPE_HIP_H
#define TPE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TPE_ABI_VERSION 22

/* finalize slots per candidate tile: tile_best holds n_tiles * TPE_BEST_PER_TILE entries */
#define TPE_BEST_PER_TILE 8

/* categorical problems with at most this many categories are scored by the
 * sample stage itself (device-drawn candidates) */
#define TPE_SAMPLE_LDS_ROWS 1024
/* cell rows a table workgroup computes (one per wave); a lattice value takes
 * a whole workgroup.  A short side (at most 64 component rows + wide rows,
 * rows_n >= 0) is summed directly, several rows a wave: 5 for a log-polynomial
 * job, 4 for a moment-cell job.  tpe_batch.tab_blocks = sum over such
 * log-polynomial jobs of ceil(n / (5 TPE_TAB_PER_BLOCK)) + over such moment
 * jobs of ceil(n / (4 TPE_TAB_PER_BLOCK)) + over the other cell jobs of
 * ceil(n / TPE_TAB_PER_BLOCK) + over lattice jobs of n (a TPE_F_FGT label's
 * above cells: none, the box stage builds them) */
#define TPE_TAB_PER_BLOCK 8
/* 16-B units of one cell row of a TPE_TAB_CELLS table */
#define TPE_TAB_ROW_UNITS 3

/* problem families: {Gaussian, log-Gaussian} x {continuous, quantized} + categorical */
enum {
  TPE_FAM_GAUSS = 0,       /* GMM1_lpdf, q=None   (uniform, normal)            */
  TPE_FAM_LOGGAUSS = 1,    /* LGMM1_lpdf, q=None  (loguniform, lognormal)      */
  TPE_FAM_QGAUSS = 2,      /* GMM1_lpdf, q        (quniform, qnormal)          */
  TPE_FAM_QLOGGAUSS = 3,   /* LGMM1_lpdf, q       (qloguniform, qlognormal)    */
  TPE_FAM_CATEGORICAL = 4  /* categorical_lpdf    (randint, choice, pchoice)   */
};

/* problem flags */
enum {
  TPE_F_HAS_LOW = 1,   /* low bound present (reference: low is not None)   */
  TPE_F_HAS_HIGH = 2,  /* high bound present                                */
  TPE_F_POOLED = 4,    /* candidates pooled with the other ids of the label (see "Pooled labels") */
  TPE_F_CAT_LAZY = 8,  /* categorical, <= 64 categories, best-scoring drawable category with selection
                          probability >= 2^-16: device-drawn batches without per-candidate outputs
                          score it in the select stage by scanning draws in index order until no
                          undrawn category can still win (usually one 1024-draw chunk) */
  TPE_F_NO_TABLE = 16, /* tpe_label_in: score this label per candidate (no lattice table), e.g. when
                          the caller supplies candidates that need not lie on the quantization lattice */
  TPE_F_PREFIT = 32,   /* tpe_tree_label: fit this label up front on the host worker threads (the
                          caller's hint: the labels its previous suggest on the space used); no label
                          flagged: every natively fitted label with enough observations */
  TPE_F_FGT = 64,      /* tpe_problem (set by the packer): a device-fitted TPE_TAB_CELLS label whose
                          above cells are built from Hermite box moments (see "Box moments") */
  TPE_F_REMOTE = 128,  /* tpe_tree_label: another rank evaluates this label (hyperparameter-axis
                          shard, see "Shard axes"): it is neither fitted nor run here; its values
                          are NaN and its activity is the tree's.  Not allowed on a gate. */
  TPE_F_LOGPOLY = 256  /* tpe_problem (set by the packer): a TPE_TAB_CELLS label whose table holds
                          log-polynomial rows of both sides on one cell grid (see "Tabulated
                          scoring"; its two table jobs have kind TPE_TAB_LOGPOLY) */
};

/* box moments (see "Box moments" below): Hermite terms per box, 16-B units per box record */
#define TPE_FGT_P 16
#define TPE_FGT_BOX_UNITS 9

/* tabulated scoring of a problem (tpe_problem.tab_mode, see "Tabulated scoring") */
enum {
  TPE_TAB_NONE = 0,     /* scored by the above / finalize stages (per candidate)                  */
  TPE_TAB_CELLS = 1,    /* continuous f32: per-cell Taylor moment tables of both mixtures          */
  TPE_TAB_LATTICE = 2,  /* quantized: exact {l, g} per lattice value of the candidate range        */
  TPE_TAB_LOGPOLY = 3   /* tpe_tab_job kind of a TPE_F_LOGPOLY label's sides (problems keep
                           TPE_TAB_CELLS)                                                         */
};

/* tpe_batch.flags / tpe_level_run flags */
enum {
  TPE_BATCH_NO_EXPAND = 1,  /* pruned f32 kernel: evaluate every component exactly (no local expansion) */
  TPE_BATCH_WRITE_CAND = 2, /* store every drawn candidate value in cand (else only where a later stage
                               reads it: quantized families and TPE_PREC_F64; the winner's value is
                               re-drawn by the select stage) */
  TPE_BATCH_NO_FUSE = 4,    /* score every continuous tile in the finalize stage (no fused finalize
                               in the above kernel) */
  TPE_BATCH_ORDERED_DRAWS = 8, /* sorted problems draw ordered candidates, no sort (else i.i.d.
                                  draws + sort) — see "Ordered draws" below */
  TPE_BATCH_TAB_EXACT = 16,    /* test hook: flag every table cell, so every candidate of a
                                  TPE_TAB_CELLS problem takes the exact-sum fallback */
  TPE_BATCH_NO_TAB_FAST = 32, /* tpe_level_run: the general sample-stage kernel even where the
                                  specialised one applies (tpe_batch.tab_fast; A/B, tests) */
  TPE_BATCH_NO_FAST2 = 64      /* tpe_level_run: k_sample_tab's 1024-thread FAST pass where
                                  k_sample_fast applies (tab_fast = 1 for log-polynomial levels; tests) */
};

/* precision of the continuous (non-quantized) families; quantized families
 * always evaluate the mixture mass in float64 (cancellation of Phi(ub)-Phi(lb)) */
enum { TPE_PREC_F32 = 0, TPE_PREC_F64 = 1 };

/* error codes */
enum { TPE_OK = 0, TPE_E_ARG = -1, TPE_E_HIP = -2, TPE_E_NODEV = -3, TPE_E_SPACE = -4 };

/*
 * One problem (256 bytes).  Component tables (device, caller-owned):
 *   comp32[k] = float4 {mu_hi, mu_lo, a, c}      families 0/1 at TPE_PREC_F32
 *   comp64[k] = double4 {mu, a, c, 0}            families 0/1 at TPE_PREC_F64
 *   comp64[k] = double4 {mu, b, w, 0}            families 2/3 (b = max(sqrt2*sigma, EPS))
 *   comp64[k] = double4 {log p_k, p_k, 0, 0}     family 4
 * For families 0/1 the mixture log-density is
 *   lpdf(x) = ln2 * log2( sum_k 2^(c_k - (a_k * (t - mu_k))^2) ) + base  [- ln x for LOGGAUSS]
 * with t = x (GAUSS) or ln x (LOGGAUSS); the host folds weights, 1/Z,
 * p_accept and a per-mixture shift (max_k c_k = 0) into c_k and base.
 * Families 2/3:  lpdf(x) = ln( sum_k w_k Phi(zu_k) - w_k Phi(zl_k) ) + base.
 *
 * Pruned above mixture (families 0/1, f32): the above components are sorted by
 * mu; the `wide_len` widest (incl. the prior) are copied to comp32[wide_off..]
 * and set to c = -inf in the sorted list.  A wave of sorted candidates spanning
 * [tmin, tmax] evaluates every wide component plus the sorted components with
 * mu in [tmin - R, tmax + R], R = sqrt(narrow_cmax - lb + 45) / narrow_amin,
 * lb = prior_c - (prior_a * max|t - prior_mu|)^2 a lower bound of log2 s(t):
 * every skipped term is < 2^-45 of the sum.  grid[grid_off .. +grid_n] maps
 * value buckets (grid_lo + g / grid_inv) to the first sorted component with
 * mu >= the bucket edge.  narrow_amin <= 0 disables pruning.  With pruning,
 * work item `split` of a tile evaluates the split-th of its n_splits equal
 * parts of each wave's window (k_start/k_end are ignored).
 *
 * Sorted problems (sort_slot >= 0, the pruned ones) own the candidate range
 * [0, sort_count) of the batch; the sort key is sort_slot << key_bits | value
 * bucket.  Other problems' candidates follow and are never sorted.
 *
 * Pooled labels (a pruned label active for several ids of the level — batched
 * suggest): its problems share the mixtures, so their candidates are sorted as ONE
 * population (one sort slot, key bits sized for n_ids x n_cand) and every wave
 * spans a narrow range however small n_cand is.  A sorted position may then hold
 * any of the label's problems' candidates: the scoring stages fold each candidate
 * into its own problem's pool_best[problem] (atomicMax of a u64 key: the f64 score
 * mapped to an order-preserving integer, its low bits replaced by the
 * complemented candidate index — np.argmax order at ~2^-40 relative score
 * resolution), and k_select re-evaluates the winner's l and g exactly.
 *
 * Ordered draws (TPE_BATCH_ORDERED_DRAWS; device-drawn sorted problems at
 * TPE_PREC_F32): instead of C i.i.d. draws that are then sorted, the
 * sample stage draws the C order statistics of C uniforms,
 * U_g = (E_0 + .. + E_g) / (E_0 + .. + E_Cg), E_i = -ln u_i (Philox counter =
 * global index i), and maps each through the mixture: component k with
 * cum_{k-1} <= U_g < cum_k, then the component's truncated-normal inverse CDF at
 * (U_g - cum_{k-1}) / (cum_k - cum_{k-1}).  The multiset of candidates has the
 * law of C i.i.d. mixture draws (so does its argmax); candidates come out sorted
 * within each component, which is all the pruned kernel needs.  The prefix sums
 * use fixed 64-index blocks of the GLOBAL index (draw_pref: per sorted problem,
 * draw_blocks exclusive block prefixes + the total), so every shard count draws
 * the same values bit for bit.
 *
 * Tabulated scoring (tab_mode != TPE_TAB_NONE): the score of a candidate is a
 * function of its value alone, so each hyperparameter's l and g are tabulated
 * once per level — shared by every new_id of the label — and the sample stage
 * scores each draw from the tables (no candidate stores, no sort, no above or
 * finalize work):
 *   TPE_TAB_CELLS (families 0/1, f32): side s (0 below, 1 above) splits
 *     [tab_lo[s], tab_lo[s] + tab_n[s] / tab_inv[s]) into tab_n[s] cells of
 *     half-width h with a_max * h <= 0.05 (a_max: the narrowest component).
 *     About its centre c a component's term is 2^v exp(B u + G u^2),
 *     u = (t - c) / h, |G| <= 0.0017; a cell row holds the degree-10 Taylor
 *     moments of the sum of the terms within 2^-50 of its largest one
 *     (|B| <= 0.6, truncation < 4e-8 relative) — a 48-B row of floats
 *     {M0..M10, m (log2 shift)}: log2 s(t) = m + log2(sum_n M_n u^n).  Cell j's
 *     centre and half-width are c = fma(j + 0.5, w, tab_lo), h = w / 2 with
 *     w = 1 / tab_inv, all in f32 (the table and the sample stages compute them
 *     alike).  m = NaN (a significant term too narrow to expand) and t outside
 *     the cells fall back to the exact sum.
 *     TPE_F_LOGPOLY (both sides fit the sample stage's LDS on one grid: the
 *     finer side's cells for both): one table of 48-B rows, row j = {b_0, a_0,
 *     b_1, a_1, .., b_5, a_5} (the sides interleaved: one packed Horner chain
 *     evaluates both): the degree-5 polynomials in u of log2 s_below(t) and log2
 *     s_above(t) (shift included) on cell j — the table stage evaluates each
 *     side's moment series in f64 at the 6 Chebyshev nodes of [-1, 1],
 *     interpolates, and checks the polynomial at u = 0, +-1/2, +-1 against the
 *     series (|error| <= 1e-7 (1 + |log2 s|)); a side that fails, or whose
 *     cell is flagged, gets b_0 (a_0) = NaN and its candidates the exact sum.
 *     One row, two degree-5 Horner sums and no log2 per candidate instead of
 *     two rows, two degree-10 sums and two log2.
 *   TPE_TAB_LATTICE (families 2/3): every candidate is x = m q (np.round,
 *     tpe.py:90-93, 248-249); row m - lat_lo of the table (tab_n[0] rows of
 *     double2 {l, g}, float64, reference operation order per component) holds
 *     its scores; other values (injected candidates) are scored directly.
 *     ABI 20: the rows are followed by tab_n[0] + 1 float entry thresholds
 *     (ceil((tab_n[0] + 1) / 4) units): thr[m] = the smallest f32 coordinate t
 *     in the clip range whose np.round(x / q) >= lat_lo + m (+inf: none), so a
 *     device draw t takes row #{m : thr[m] <= t} - 1 with no f64 arithmetic
 *     (k_sample_fast; k_sample_tab quantises directly, with the same result).
 * Tables live in `tab` (16-B units; tab_off[s] = first unit) and are built by
 * the table stage from the problem's component rows (after the device fit).
 *
 * Box moments (TPE_F_FGT: device-fitted above mixtures of a TPE_TAB_CELLS
 * label).  adaptive_parzen_normal clips every bandwidth to >= prior_sigma /
 * min(100, 1 + K) (tpe.py:465-470), so a large history's above components
 * share that narrowest sigma (a = fgt_a in the rows) almost everywhere: their
 * sum is a Gauss transform with one width d = 1 / (fgt_a sqrt(ln 2)).  The
 * box stage (k_boxes) cuts [fgt_lo, fgt_lo + fgt_n d) into boxes of width d
 * and gives each box its Hermite moments A_n = sum_k 2^c_k y_k^n / n!
 * (y_k = (mu_k - centre) / d, n < TPE_FGT_P, f64, fixed-order reductions);
 * a cell then gets its Taylor moments from the boxes within reach,
 * B_m = (-1)^m / m! sum_b sum_n A_bn h_(n+m)(x_b) (h_j(x) = e^-x^2 H_j(x),
 * x_b = (centre_cell - centre_b) / d) — about 16 boxes per cell instead of
 * every component within reach — plus the components of other widths (the
 * wide list, and any "odd" component a box counts) summed directly.  A cell
 * whose truncation bound (Cramer: sum_b 1.09 W_b e^(-x_b^2 / 2) eps_P) is not
 * below 2^-25 of its sum, and every cell of a label whose components do not
 * all lie in the boxes, is built by the direct path instead.  Box records
 * follow the label's above cells in `tab` at fgt_off: one header unit {int32
 * ok, ...} and TPE_FGT_BOX_UNITS units per box {double A[TPE_FGT_P]; int32
 * k_lo, k_hi, n_odd, 0}.
 *
 * samp[k] = double[8] {cum, mu, sigma, fa, fb, flip, 0, 0}: below-mixture
 * sampler table; cum = selection CDF (∝ w_k * mass_k when bounded); fa, fb =
 * Phi of the (mirrored if flip) standardised truncation bounds; family 4 uses cum.
 */
typedef struct tpe_problem {
  int32_t family, flags;
  int32_t n_cand;        /* candidates of this problem on this device          */
  int32_t n_upper;       /* categorical: number of categories                  */
  int64_t cand_off;      /* element offset into cand / coord / keys / l_out    */
  int64_t cand_base;     /* global index of local candidate 0 (shards, RNG)    */
  int64_t n_cand_global; /* candidates of the problem over all shards (= n_cand unsharded) */
  int32_t n_splits;      /* splits of the bulk tiles (tiles carry their own)   */
  int32_t tile_off;      /* first candidate tile of this problem               */
  int32_t n_tiles;       /* candidate tiles of this problem                    */
  int32_t samp_off;
  int32_t samp_len;
  int32_t below_off;
  int32_t below_len;
  int32_t above_off;
  int32_t above_len;
  int32_t wide_off;      /* always-evaluated wide components (pruned mode)     */
  int32_t wide_len;
  int32_t grid_off;
  int32_t grid_n;
  int32_t sort_slot;     /* rank among the batch's sorted problems, -1: unsorted */
  double low, high, q;   /* bounds in sampling space (log space for LGMM1)     */
  double below_base;     /* additive constant of the below lpdf                */
  double above_base;     /* additive constant of the above lpdf                */
  float prior_mu, prior_a, prior_c, narrow_cmax;
  float narrow_amin, grid_lo, grid_inv;
  float key_lo, key_inv; /* sort-key bucket of t: floor((t - key_lo) * key_inv)  */
  int32_t pool_first;    /* pooled: the label's first problem (else -1)         */
  uint32_t key0, key1;   /* Philox-4x32-10 key (suggest seed)                  */
  uint32_t ctr2, ctr3;   /* Philox counter high words (label index, new id)    */
  int32_t tab_mode;      /* TPE_TAB_*                                          */
  int32_t tab_off[2];    /* first 16-B unit of the below / above table in `tab` (lattice: [0]) */
  int32_t tab_n[2];      /* cells per side (lattice: tab_n[0] = lattice values) */
  float tab_lo[2], tab_inv[2];  /* cell j of side s: [tab_lo[s] + j / tab_inv[s], + 1 / tab_inv[s]) */
  float fgt_a;           /* TPE_F_FGT: a of the narrowest (sigma-clipped) components  */
  int64_t lat_lo;        /* lattice: index m of table row 0 (value lat_lo * q) */
  int32_t fgt_off;       /* TPE_F_FGT: first 16-B unit of the box records in `tab`    */
  int32_t fgt_n;         /* TPE_F_FGT: boxes of width 1/(fgt_a sqrt(ln 2)) from fgt_lo */
  double fgt_lo;
} tpe_problem;

/* one table of the table stage: a side of a TPE_TAB_CELLS label (4 cells per
 * 256-thread block) or a TPE_TAB_LATTICE label (1 lattice value per block).
 * `problem` is the label's first problem row (its mixtures are the label's). */
typedef struct tpe_tab_job {
  int32_t problem;
  int32_t side;          /* cells: 0 below, 1 above                             */
  int32_t kind;          /* TPE_TAB_CELLS | TPE_TAB_LATTICE                     */
  int32_t n;             /* cells / lattice values                              */
  int32_t off;           /* first 16-B unit of the table                        */
  int32_t block0;        /* first block of this job in the table stage's grid   */
  /* cells: the side's component rows (comp32 [rows_off, rows_off + rows_n) then
   * [wide_off, wide_off + wide_n)) and cell geometry (the problem's tab_lo /
   * tab_inv of this side), so the table stage reads no problem row; rows_n < 0:
   * read them from the problem (a device-fitted above side: the fit writes them) */
  int32_t rows_off, rows_n, wide_off, wide_n;
  float lo, inv;
} tpe_tab_job;

/* candidate tile: 2048 consecutive candidates of one problem; its above-mixture
 * partial sums are rows work_first .. work_first + n_splits - 1 of `part` */
typedef struct tpe_tile {
  int32_t problem;
  int32_t cand_start;
  int32_t work_first;    /* first work item (= part row) of this tile          */
  int32_t n_splits;      /* its work items (0: no above stage)                 */
} tpe_tile;

/* above-mixture work item: one candidate tile x one component range; writes
 * the tile's partial sums to part[row * 2048 .. + 2048), row = its index in
 * the batch's work list */
typedef struct tpe_work {
  int32_t problem;
  int32_t split;
  int32_t cand_start;
  int32_t k_start;
  int32_t k_end;
  int32_t n_splits;      /* work items of this tile                            */
} tpe_work;

/* best of one finalize slot (TPE_BEST_PER_TILE per tile), written by the finalize stage */
typedef struct tpe_best {
  double score, l, g;
  int64_t idx;           /* local candidate index, -1 if none */
} tpe_best;

/* per-problem result */
typedef struct tpe_result {
  double score, l, g;
  double value;          /* the chosen candidate                               */
  int64_t idx;           /* local candidate index, -1 if the problem is empty  */
  int64_t global_idx;    /* cand_base + idx                                     */
} tpe_result;

/*
 * Device Parzen fit of one continuous above mixture (families 0/1, f32 tables):
 * adaptive_parzen_normal (tpe.py:398-475) of the label's observations that are
 * not in the below set (ap_filter_trials, tpe.py:613-641), written straight
 * into the pruned comp32 layout above.
 *
 * Device value order.  The reference argsorts the above observations on every
 * suggest (tpe.py:427).  Here each device-fitted label keeps a RESIDENT value
 * order of ALL its observations in HBM — (t, i) pairs sorted by t ascending,
 * NaN last, ties by i (t = x, or ln x for LOGGAUSS; i = position in tid
 * order) — owned by the caller and extended, not rebuilt: the history is
 * append-only, so a suggest only merges the observations appended since the
 * order was last written (obs[n_ord_in .. n_obs)).  Stages (tpe_fit_above):
 *   chunks   the new observations, 8192 at a time, sorted in LDS (bitonic)
 *   passes   merge-path merges of the sorted chunks (only when a job has more
 *            than 8192 new observations, i.e. the first suggest)
 *   merge    merge-path merge of the resident order ord_*_in [n_ord_in] with the
 *            sorted new batch into ord_*_out [n_obs] (skipped when nothing is new:
 *            the order is then read from ord_*_in)
 *   compact  the order without the below observations, each with its rank among
 *            the above observations in tid order (the linear-forgetting weight
 *            index) — exactly the stable argsort of the above observations
 *   build    one workgroup per job: prior insertion (searchsorted left), sigma
 *            from neighbour gaps, clip, LF weights, normalisation, {mu, a, c}
 *            rows, wide list, grid; patches the job's problem rows (above_base,
 *            wide_len, prior_*, narrow_*, grid_lo/inv)
 * No sort of the whole history runs after the first suggest.  DELTA MODE: a job
 * with 1 .. TPE_FIT_DELTA_MAX new observations and ord_*_out NULL is not merged:
 * its new observations are sorted and placed among the resident ones (their
 * ranks), and the build reads the resident order and them as one virtual order
 * — the merge pass over the whole order waits until the new ones outgrow the
 * delta (FMinIter's one observation per suggest: one merge every
 * TPE_FIT_DELTA_MAX suggests); ord_*_in stays the caller's order of the first
 * n_ord_in.  A steady-state suggest costs the build (plus, every
 * TPE_FIT_DELTA_MAX appends, one merge pass over each label's order).
 * The host reserves above_off[0 .. K) + wide_off[0 .. 16) rows and grid_n + 1
 * grid entries (K = n_obs - n_below + 1, grid_n = min(4096, 4K)).
 */
#define TPE_FIT_DELTA_MAX 16
typedef struct tpe_fit_job {
  const double* obs;     /* device: the label's observations in tid order, in the kernel
                            coordinate t (x, or the caller's np.log(x) for LOGGAUSS) */
  int64_t n_obs;
  int64_t seg_off;       /* first slot of this job in the fit scratch buffers (fit_seg)   */
  int32_t below_off;     /* below_idx[below_off ..]: ascending indices into obs */
  int32_t n_below;
  int32_t family, flags, lf;
  int32_t problem_first, n_problems;  /* problem rows this mixture serves      */
  int32_t above_off, wide_off, grid_off, grid_n;
  int32_t reserved;
  double prior_mu, prior_sigma, prior_weight, low, high;
  /* resident value order (device, caller-owned): the first n_ord_in observations
   * sorted, and where the order of all n_obs goes when n_ord_in < n_obs */
  const double* ord_key_in; const uint32_t* ord_idx_in; int64_t n_ord_in;
  double* ord_key_out; uint32_t* ord_idx_out;
} tpe_fit_job;

/* all device pointers of one batch (the struct itself lives in host memory) */
typedef struct tpe_batch {
  const tpe_problem* problems; int32_t n_problems;
  int32_t precision;     /* TPE_PREC_F32 | TPE_PREC_F64                         */
  int32_t sample;        /* 1: draw candidates on device (Philox); 0: caller filled cand/coord */
  int32_t sort_end_bit;  /* keys sorted on bits [0, sort_end_bit); 0 = no sort  */
  int32_t key_bits;      /* value-bucket bits of the sort key (problem << key_bits | bucket) */
  int32_t flags;         /* TPE_BATCH_* options (0 = defaults)                  */
  const float* comp32;   /* [n][4]                                             */
  const double* comp64;  /* [n][4]                                             */
  const double* samp;    /* [n][8]                                             */
  const int32_t* grid;   /* pruning grids                                      */
  double* cand;          /* [total_cand] candidate values (see TPE_BATCH_WRITE_CAND) */
  float* coord;          /* [total_cand] kernel coordinate t in f32 (x or ln x) */
  uint32_t* keys;        /* [total_cand] (problem << key_bits | value bucket of t) */
  uint64_t* vals;        /* [total_cand] (position << 32) | f32 bits of t       */
  uint32_t* keys_sorted; /* [total_cand] (== keys when not sorting)            */
  uint64_t* vals_sorted; /* [total_cand] (== vals when not sorting)            */
  void* sort_tmp; uint64_t sort_tmp_bytes;   /* tpe_sort_workspace_bytes()     */
  int64_t total_cand;
  const tpe_tile* tiles; int32_t n_tiles; int32_t n_fin_tiles;
  int64_t sort_count;    /* candidates [0, sort_count) are sorted (sorted problems first) */
  const int32_t* fin_tiles; /* [n_fin_tiles] tiles the finalize stage scores when the candidates
                               are device-drawn (the others are scored by the sample stage —
                               categorical — or the fused above stage — one-split continuous
                               f32);
                               NULL: every tile */
  /* above-mixture work list, ordered [continuous | quantized Gauss | quantized log] */
  const tpe_work* work;
  int32_t n_work_cont, n_work_qgauss, n_work_qlog;
  int32_t fgt_max_boxes; /* most boxes of a TPE_F_FGT problem (0: none; the box stage's grid) */
  double* part;          /* above-mixture partial sums: [n_work][2048]          */
  double* l_out;         /* optional [total_cand] (original order); NULL to skip */
  double* g_out;         /* optional [total_cand]; NULL to skip                 */
  tpe_best* tile_best;   /* [n_tiles * TPE_BEST_PER_TILE]                      */
  tpe_result* result;    /* [n_problems]                                       */
  unsigned long long* ce_count; /* optional [2 * n_work_cont]: per work item of the pruned
                                   kernel, {exactly evaluated component x candidate pairs,
                                   components summed by the local expansion}; NULL to skip */
  /* device Parzen fits (n_fit == 0: none); they patch rows of `problems` */
  const tpe_fit_job* fit; int32_t n_fit;
  int32_t fgt_max_cells; /* most above cells of a TPE_F_FGT problem (built by the box stage) */
  const int32_t* below_idx;   /* below indices of every job                        */
  const int64_t* fit_seg;     /* [n_fit + 1] segment offsets into the fit scratch: a job's
                                 segment holds max(n_obs - n_below, n_obs - n_ord_in, n_below,
                                 64 + 2 * TPE_FIT_DELTA_MAX [+ 2304 per 2048 components of a
                                 delta-mode job]) */
  int64_t fit_total;          /* fit_seg[n_fit]                                    */
  double* fit_keys; double* fit_keys_sorted;        /* [fit_total] scratch (ping-pong) */
  uint32_t* fit_vals; uint32_t* fit_vals_sorted;    /* [fit_total]                */
  int64_t fit_max_new;        /* most new observations of one job (n_obs - n_ord_in) */
  int64_t fit_max_obs;        /* most observations of one job                       */
  int64_t fit_max_merge;      /* most new observations of a job that merges them (0: none) */
  int64_t fit_n_delta;        /* jobs in delta mode (new observations, no ord_*_out) */
  /* ordered draws: [n_sorted][draw_blocks + 1] doubles, draw_blocks = ceil((C_global + 1) / 64) */
  double* draw_pref; int64_t draw_blocks; int32_t n_sorted;
  int32_t tab_fast;      /* >= 1: the candidates are device-drawn at TPE_PREC_F32, early selection is on,
                            nothing per candidate is written and every tabulated problem has
                            1..TPE_SAMPLE_LDS_ROWS sampler rows: the sample stage's specialised kernels —
                            1 + U (ABI 20; every tabulated problem a TPE_F_LOGPOLY cells table of <= 896
                            rows or a lattice of <= 1024 values, <= 64 sampler rows): k_sample_fast in
                            512-thread workgroups taking U 16-B units of LDS (3 per cell row; a lattice
                            value's {l, g} unit plus its 4-B score rank), three a CU; 1: every tabulated
                            problem a TPE_F_LOGPOLY cells table of <= 2048 rows, in 1024-thread
                            workgroups (tpe_level_run sets it; 0: the general kernel) */
  unsigned long long* pool_best;   /* [n_problems] (pooled problems; see "Pooled labels") */
  /* tabulated scoring: table jobs and the table storage (16-B units) */
  const tpe_tab_job* tab_jobs; int32_t n_tab_jobs; int32_t tab_blocks;
  void* tab; int64_t tab_units;
  /* sample-stage tile lists (NULL: every tile through the generic sample kernel):
   * samp_tiles[0 .. n_samp_tiles) = the untabulated tiles, lazy categorical ones
   * last (the first n_samp_eager of them skip those when the lazy scan applies);
   * tab_tiles[0 .. n_tab_tiles) = the tabulated tiles (one 2048-candidate block each) */
  const int32_t* samp_tiles; int32_t n_samp_tiles; int32_t n_samp_eager;
  const int32_t* tab_tiles; int32_t n_tab_tiles;
  /* early selection (needs tables, sampled candidates, tab_tiles and
   * run_best): the sample stage writes, for every run of consecutive tiles of
   * one tabulated problem a workgroup processes, the run's best candidate —
   * score, l, g, index and its drawn value — to run_best[first tile of the run]
   * (host-visible memory; the caller reduces a problem's runs with np.argmax
   * semantics: tpe_level_run does); each lazy categorical problem is selected
   * by the table stage; the select stage runs only for the n_late others (not
   * at all when n_late == 0).  0: the select stage selects every problem. */
  int32_t early_select;
  tpe_result* run_best;  /* [n_tiles], device address of host-visible memory */
  int32_t n_late;
  int32_t tiles_per_problem;   /* > 0: every problem has this many tiles, tile t = {t / tiles_per_problem,
                                  (t % tiles_per_problem) * 2048} (the sample stage then reads no
                                  tile descriptors); 0: read them */
} tpe_batch;

/* ABI version (TPE_ABI_VERSION) of the loaded library */
int tpe_abi_version(void);

/* thread-local message of the last failing call on this thread ("" if none) */
const char* tpe_last_error(void);

/* number of visible HIP devices (0 and TPE_E_NODEV when none) */
int tpe_device_count(int* n);

/* candidates per tile (2048) — the caller sizes tiles / work items with it */
int tpe_tile_size(void);

/* device address of page-locked host memory (NULL when the device cannot
 * address it): look it up once per allocation for tpe_level_ws.pinned_dev */
int tpe_pinned_device_address(void* host, void** dev);

/* device workspace (bytes) the candidate sort needs for `total_cand` candidates */
int tpe_sort_workspace_bytes(int64_t total_cand, uint64_t* bytes);

/* fit (when n_fit > 0) -> tables -> sample (optional) -> sort -> score -> select, enqueued on `stream` (hipStream_t);
 * asynchronous: results are valid once the stream reaches this point. */
int tpe_run_batch(const tpe_batch* batch, void* stream);

/* the stages one by one (same semantics; used by tests and the profiler) */
int tpe_fit_above(const tpe_batch* batch, void* stream);  /* device Parzen fits */
int tpe_tables(const tpe_batch* batch, void* stream);     /* score tables of tabulated labels */
int tpe_sample(const tpe_batch* batch, void* stream);     /* draw + sort keys */
int tpe_sort(const tpe_batch* batch, void* stream);
int tpe_score_above(const tpe_batch* batch, void* stream);
int tpe_finalize(const tpe_batch* batch, void* stream);
int tpe_select(const tpe_batch* batch, void* stream);

/* ------------------------------------------------------------------------
 * Native host runtime (tpe_host.cpp): the Parzen fit and the packing of one
 * tree level into the tables above.  Host pointers only.
 * ---------------------------------------------------------------------- */

/* one hyperparameter of a level: its fitted posterior and the new_ids it is
 * active for (mixtures are float64 host arrays; categorical: below_w / above_w
 * are the probabilities, *_k = number of categories).
 * Device-fitted above mixture (families 0/1, TPE_PREC_F32 only): above_w/mu/
 * sigma NULL, dev_obs = the label's device observation column (n_obs kernel
 * coordinates t in tid order: x, or np.log(x) for LOGGAUSS), below_idx = host array of the n_below ascending indices of the
 * below observations in it, above_k = n_obs - n_below + 1; prior_* and lf are
 * the fit parameters; ord_* = the label's resident value order (tpe_fit_job:
 * ord_*_in may be NULL when n_ord_in = 0, ord_*_out may be NULL when
 * n_ord_in = n_obs or, delta mode, when 0 < n_obs - n_ord_in <= TPE_FIT_DELTA_MAX
 * and n_ord_in > 0).  After the level has run, ord_*_out holds the order of
 * all n_obs observations whenever it was given. */
typedef struct tpe_label_in {
  int32_t family, flags, upper, label_ix;
  double low, high, q;
  const double* below_w; const double* below_mu; const double* below_sigma; int64_t below_k;
  const double* above_w; const double* above_mu; const double* above_sigma; int64_t above_k;
  const int64_t* ids; int64_t n_ids;
  const double* dev_obs; int64_t n_obs;
  const int32_t* below_idx; int32_t n_below; int32_t lf;
  double prior_mu, prior_sigma, prior_weight;
  const double* ord_key_in; const uint32_t* ord_idx_in; int64_t n_ord_in;
  double* ord_key_out; uint32_t* ord_idx_out;
} tpe_label_in;

/* where tpe_host_pack_level put each table in the blob (byte offsets).  The
 * device-fitted rows (end of the grid and comp32 sections) are written by
 * tpe_fit_above: only [0, copy_end) and [off_comp32, off_comp32 + copy2_len)
 * need the host -> device copy. */
typedef struct tpe_pack_info {
  int64_t off_problems, off_tiles, off_work, off_comp32, off_comp64, off_samp, off_grid;
  int64_t n_problems, n_tiles;
  int32_t n_work_cont, n_work_qgauss, n_work_qlog, any_pruned;
  int64_t part_total, blob_bytes;
  int32_t key_bits, sort_end_bit;   /* sort-key layout for tpe_batch (sort_end_bit 0: no sort) */
  int64_t off_fit, off_below_idx, off_fit_seg;
  int32_t n_fit, fgt_max_boxes;     /* device fits; most boxes of a TPE_F_FGT label */
  int64_t fit_total;
  int64_t sort_count;               /* candidates of the sorted (pruned) problems */
  int64_t off_fin_tiles, n_fin_tiles;   /* tpe_batch.fin_tiles */
  int64_t fit_max_new;                  /* tpe_batch.fit_max_new */
  int64_t fit_max_obs;                  /* tpe_batch.fit_max_obs */
  int64_t fit_max_merge;                /* tpe_batch.fit_max_merge */
  int64_t fit_n_delta;                  /* tpe_batch.fit_n_delta */
  int64_t n_sorted, draw_blocks;        /* tpe_batch.n_sorted / draw_blocks */
  int64_t n_pooled;                     /* pooled problems (tpe_batch.pool_best needed) */
  int64_t off_tab_jobs, n_tab_jobs, tab_blocks, tab_units;   /* tabulated scoring (tpe_batch.tab_*) */
  int64_t off_samp_tiles, n_samp_tiles, n_samp_eager, off_tab_tiles, n_tab_tiles;   /* tpe_batch tile lists */
  /* expanded level (see "Expanded levels"; n_expand = 0: not expanded): off_expand holds
   * tpe_problem templates[n_expand], then (at the next 256-B boundary) int32 first[n_expand + 1],
   * then (at the next 256-B boundary) uint32 new_id[n_problems]; the problems and tiles sections
   * (and the tabulated tile list, the identity) are device-only */
  int64_t off_expand, n_expand;
  int64_t fgt_max_cells;                /* most above cells of a TPE_F_FGT label (tpe_batch) */
  /* ABI 20: the blob's host-written byte ranges [up_off[i], up_off[i] + up_len[i]), i < n_up
   * (the upload; everything else is device-only: the device-fitted rows and grid, the fit
   * patches, an expanded level's problems and tiles).  Layout: fit jobs, below positions,
   * fit segments, grid (host | device from a 256-B boundary), comp32 (host | device), fit
   * patches (off_patch: one tpe_problem per problem, the fields the device fit writes,
   * applied to the problem rows after the upload), problems, tiles, comp64, sampler rows,
   * then work, finalize tiles, table jobs, tile lists and the expanded templates. */
  int64_t up_off[4], up_len[4];
  int32_t n_up, pad_;
  int64_t off_patch;                    /* 0: no device fit */
} tpe_pack_info;

/* ------------------------------------------------------------------------
 * Expanded levels.  A batched level (>= 256 problems) whose labels all score
 * from tables (cells or lattice) has problems that differ from their label's
 * only in cand_off (= r * n_cand), ctr3 (the new id) and tile_off (= r *
 * n_tiles), and tiles {r, j * 2048, 0, 0} in order, all of them tabulated.
 * tpe_host_pack_level then writes one problem template per label and the new
 * ids instead of ~270 B per (label, id), and tpe_level_run's device writes the
 * problems and tiles (k_expand) right after the upload: a 20-label x 4096-id
 * level packs and uploads ~0.4 MB of descriptors instead of ~22 MB.
 * ---------------------------------------------------------------------- */

/* adaptive_parzen_normal (tpe.py:398-475) with the caller's sort permutation
 * `order` of obs (np.argsort; may be NULL when n < 2).  Writes n+1 components
 * (w, mu, sigma) sorted by mu; returns the prior's position or a TPE_E* code. */
int64_t tpe_host_fit_parzen(const double* obs, int64_t n, const int64_t* order, double prior_weight,
                            double prior_mu, double prior_sigma, int32_t lf, double* w, double* mu, double* sigma);

/* ap_filter_trials + adaptive_parzen_normal of both sides of one continuous
 * label (tpe.py:613-641, 398-475, 485-568).  x: the label's (transformed)
 * observations, tids strictly ascending; order: a permutation sorting x
 * ascending (the history keeps it incrementally); below_tids ascending.  Each
 * side's permutation is `order` filtered to that side — the permutation
 * np.argsort gives when no value of the side repeats; a side with repeated
 * values or NaN is NOT fitted (out_k[side] = 0): np.argsort's tie order
 * decides its weights, so the caller fits it with tpe_host_fit_parzen and
 * numpy's permutation.  out: 6 rows of n + 1 doubles — below w, mu, sigma,
 * above w, mu, sigma; out_k[0] / out_k[1] = below / above component counts. */
int tpe_host_fit_split(const double* x, const int64_t* tids, const int64_t* order, int64_t n,
                       const int64_t* below_tids, int64_t n_bt, double prior_weight, double prior_mu,
                       double prior_sigma, int32_t lf, double* out, int64_t* out_k);

/* categorical posterior (tpe.py:573-607): p_prior NULL = randint pseudo-counts,
 * else pchoice's counts + upper * prior_weight * p_prior */
int tpe_host_cat_probs(const int64_t* obs, int64_t n, int32_t upper, const double* p_prior, double prior_weight,
                       int32_t lf, double* out);

/* ap_filter_trials + the categorical posteriors of both sides of one label
 * (tpe.py:613-641, 573-607): obs/tids in strictly ascending tid order,
 * below_tids ascending; out_below / out_above: `upper` probabilities each */
int tpe_host_cat_split(const int64_t* obs, const int64_t* tids, int64_t n, const int64_t* below_tids, int64_t n_bt,
                       int32_t upper, const double* p_prior, double prior_weight, int32_t lf, double* out_below,
                       double* out_above);

/* ------------------------------------------------------------------------
 * Exact-replay candidate draws (host): numpy's legacy RandomState stream —
 * MT19937 (the 624-word key and position of RandomState.get_state()),
 * random_sample's 53-bit double, the polar-method gauss with its cached
 * second value, and multinomial(n=1, p) as numpy computes it (a binomial by
 * inversion per category, p_j over the remaining mass, until the draw is
 * placed).  The state is read and written in place, so draws interleave with
 * the caller's own use of the same RandomState.  Reference call sites:
 * tpe.py:73-74 / :224-231 (unbounded: n multinomials, then n normals),
 * tpe.py:82-87 / :240-244 (bounded: multinomial + normal per draw, rejected
 * outside [low, high)), pyll/stochastic.py:126-131 (categorical).
 * ---------------------------------------------------------------------- */
typedef struct tpe_mt_state {
  uint32_t key[624];
  int32_t pos;           /* next key word (624: regenerate first)        */
  int32_t has_gauss;     /* a cached second polar-method value is pending */
  double gauss;
} tpe_mt_state;

/* n draws from the mixture (w, mu, sigma)[k]: the normal deviate d of each
 * accepted draw (bounded: low <= d < high, in the mixture's own coordinate —
 * the caller applies exp / rounding, vectorised, as the reference does);
 * TPE_E_ARG on bad weights (numpy raises ValueError) */
int tpe_replay_mixture(tpe_mt_state* st, const double* w, const double* mu, const double* sigma, int64_t k,
                       int32_t bounded, double low, double high, int64_t n, double* out);

/* n categorical draws (one multinomial(1, p) row each): the chosen index */
int tpe_replay_categorical(tpe_mt_state* st, const double* p, int64_t k, int64_t n, int64_t* out);

/* pack one tree level into `blob` (all tables, 256-B aligned, ready for one
 * host->device copy); TPE_E_SPACE (info->blob_bytes = size needed) if too small */
int tpe_host_pack_level(const tpe_label_in* labels, int32_t n_labels, int32_t n_cand, uint64_t seed,
                        int64_t cand_base, int64_t n_cand_global, int32_t precision, void* blob, int64_t blob_cap,
                        tpe_pack_info* info);

/* ------------------------------------------------------------------------
 * One-call level runner: pack (host) -> H2D -> fit/sample/sort/score/select ->
 * D2H of the per-problem results -> stream synchronise.  This is the whole
 * per-tree-level device round trip of tpe.suggest (tpe.py:663-701 for every
 * active hyperparameter of the level) behind one C call, so the host language
 * pays one foreign call per level.  All memory is caller-owned; the runner
 * never allocates.
 * ---------------------------------------------------------------------- */
typedef struct tpe_level_ws {
  void* pinned; int64_t pinned_bytes;          /* page-locked host staging (tables + result readback) */
  void* pinned_dev;                            /* its device address (tpe_pinned_device_address), or NULL:
                                                  looked up by the call                                 */
  void* blob; int64_t blob_bytes;              /* device copy of the packed tables                      */
  double* cand; float* coord;                  /* device candidate pools, cand_cap elements each        */
  uint32_t* keys; uint64_t* vals; uint32_t* keys_sorted; uint64_t* vals_sorted; int64_t cand_cap;
  void* sort_tmp; int64_t sort_tmp_bytes;
  double* part; int64_t part_cap;              /* elements                                              */
  tpe_best* tile_best; int64_t best_cap;       /* elements                                              */
  tpe_result* result; int64_t result_cap;      /* elements (device)                                     */
  double* fit_keys; double* fit_keys_sorted;
  uint32_t* fit_vals; uint32_t* fit_vals_sorted; int64_t fit_cap;   /* elements                    */
  double* draw_pref; int64_t draw_pref_cap;    /* elements                                              */
  unsigned long long* pool_best; int64_t pool_best_cap;   /* elements                                   */
  void* tab; int64_t tab_cap;                  /* score tables, 16-B units                              */
} tpe_level_ws;

/* what a level needs (written on success and on TPE_E_SPACE) */
typedef struct tpe_level_need {
  int64_t pinned_bytes, blob_bytes, cand, sort_tmp_bytes, part, best, result, fit, draw_pref, pool_best, tab;
} tpe_level_need;

/* Run one tree level: `labels` as for tpe_host_pack_level; `out` receives one
 * tpe_result per (label, id) in order.  TPE_E_SPACE: a workspace is too small —
 * `need` holds every size; grow and call again (nothing was launched). */
int tpe_level_run(const tpe_label_in* labels, int32_t n_labels, int32_t n_cand, uint64_t seed, int64_t cand_base,
                  int64_t n_cand_global, int32_t precision, int32_t flags, const tpe_level_ws* ws,
                  tpe_level_need* need, void* stream, tpe_result* out);

/* ------------------------------------------------------------------------
 * One native call per tpe.suggest of a conditional (hp.choice) tree space:
 * the below/above split and Parzen fit of every label it needs
 * (ap_filter_trials + adaptive_parzen_normal / the categorical posteriors,
 * tpe.py:613-641, 398-607), the speculative fusion of the tree levels (gate
 * winners predicted from the fitted categorical posteriors, every level in one
 * device batch, predictions verified on the results; level by level on a
 * misprediction — the activity rule of vectorize.py:19-37 /
 * pyll/base.py:762-781), and the level runs (tpe_level_run).  The host keeps
 * only the history view and the trial documents.
 *
 * Covered: continuous (GAUSS / LOGGAUSS) and categorical labels fitted on the
 * host at TPE_PREC_F32, categorical gates, and any label whose fit the caller
 * supplies (host_w/mu/sigma/k).  A label the tree needs that it cannot fit —
 * quantized labels and sides with repeated values (numpy's argsort tie order
 * decides their weights), missing value orders (NaN) — is flagged in need_fit
 * and TPE_E_FALLBACK returned: the caller fits those labels (exactly as the
 * reference) and calls again with their fits.  Continuous labels large enough
 * for the device Parzen fit run it (tpe_fit_above) when their record carries
 * the device column; without it, and with non-categorical gates, the call
 * returns TPE_E_FALLBACK with no flag before any fit or run: the caller takes
 * its general path.  (On TPE_E_FALLBACK nothing is written; a device batch may
 * have run when a deeper level flagged a label.)
 * ---------------------------------------------------------------------- */
#define TPE_TREE_MAX_PARENTS 4
enum { TPE_E_FALLBACK = -5 };

/* one hyperparameter of the tree, in label order (label_ix = its position).
 * Quantized labels and continuous sides with repeated values are fitted with
 * numpy's argsort permutation of each side (its tie order decides the linear-
 * forgetting weights of tied observations, tpe.py:427-428): the caller passes
 * those permutations (side_order) with the fit coordinate, or gets need_fit. */
typedef struct tpe_tree_label {
  int32_t family, flags, upper, label_ix;   /* family: TPE_FAM_*; flags: TPE_F_HAS_LOW / TPE_F_HAS_HIGH */
  double low, high;                         /* sampling-space bounds (log space for LOGGAUSS)           */
  double prior_mu, prior_sigma;             /* adaptive_parzen_normal prior (continuous)                */
  const double* p_prior;                    /* categorical: pchoice probabilities (NULL: randint)       */
  const int64_t* tids;                      /* observation tids, strictly ascending                     */
  const void* values;                       /* continuous: f64 kernel coordinate (x, or ln x for
                                               LOGGAUSS); categorical: int64 categories                 */
  const int64_t* order;                     /* continuous: permutation sorting `values` ascending        */
  int64_t n_obs;
  int32_t depth, n_parents;                 /* tree level (roots 0); 0 parents = unconditional           */
  int32_t parent[TPE_TREE_MAX_PARENTS];     /* active iff some parent[j] (a label index) chose          */
  int32_t parent_cat[TPE_TREE_MAX_PARENTS]; /* category parent_cat[j]                                   */
  double q;                                 /* quantum of the quantized families (else 0)                */
  const double* host_w[2];                  /* a caller-made fit, [0] below / [1] above (host_k[0] > 0):  */
  const double* host_mu[2];                 /* used as is (categorical: host_w = the probabilities)     */
  const double* host_sigma[2];
  int64_t host_k[2];
  /* device Parzen fit of the above side (continuous labels with n_obs >= device_fit_min): the
   * label's device column (n_obs kernel coordinates in tid order) and its resident value order
   * (tpe_label_in); NULL dev_obs: such a label sends the space to the caller's general path */
  const double* dev_obs;
  const double* ord_key_in; const uint32_t* ord_idx_in; int64_t n_ord_in;
  double* ord_key_out; uint32_t* ord_idx_out;
  /* the caller's sort of each side (continuous and quantized families): side_order[s] = numpy's
   * np.argsort of side s's coordinates in tid order (s = 0 below, 1 above; `values` = the
   * fit coordinate, e.g. log(max(x, max(EPS, e^low))) for qloguniform, tpe.py:517-568), side_n[s]
   * its length (checked against the split made here).  Both set: the label is fitted here with
   * those permutations — the reference's tie order — instead of being sent to the caller
   * (need_fit).  NULL: the label's own rules above. */
  const int64_t* side_order[2];
  int64_t side_n[2];
} tpe_tree_label;

/* tpe_suggest_tree flags: the tpe_level_run flags, plus */
enum { TPE_TREE_NO_SPECULATE = 1 << 8 };    /* level by level only (no fused batch)                    */

/* ------------------------------------------------------------------------
 * Candidate-shard exchange (multi-GPU, one process per GPU).  A sharded
 * suggest gives every rank the contiguous global candidate range
 * [cand_base, cand_base + n_cand) of each problem (Philox counters are global
 * indices, so the candidates are the ones a single GPU draws there).  After
 * each level run, the ranks all-gather their per-problem results — a header
 * with the rank's status, then P tpe_result records — and every rank reduces
 * them to the global winners with np.argmax semantics (NaN first, then the
 * largest score, then the lowest global index; the reference's per-parameter
 * argmax, tpe.py:749-759), so every rank takes the same tree decisions.  A
 * rank whose level run needs a larger workspace still takes part (status
 * TPE_E_SPACE, empty results) and then every rank returns TPE_E_SPACE: the
 * callers grow and call again in lock-step.
 * The all-gather is an RCCL all-gather over xGMI on the device scratch `dev`
 * when `comm` is set (tpe_comm_init), else the caller's host all-gather.
 * ---------------------------------------------------------------------- */
#define TPE_COMM_ID_BYTES 128
#define TPE_EXCHANGE_HEADER 64   /* bytes before a rank's result records in the exchange */
typedef int (*tpe_gather_fn)(void* ctx, const void* mine, int64_t bytes, void* all);
typedef struct tpe_exchange {
  int32_t rank, world;
  void* comm;             /* RCCL communicator (tpe_comm_init), or NULL                          */
  tpe_gather_fn gather;   /* host all-gather: `bytes` from every rank into all[world * bytes], in
                             rank order; returns 0 on success (used when comm is NULL)          */
  void* ctx;
  void* dev; int64_t dev_bytes;   /* RCCL path: device scratch of world * (TPE_EXCHANGE_HEADER +
                                     P * sizeof(tpe_result)) bytes for the largest level          */
  int32_t always;         /* exchange even when world == 1 (tests of the exchange itself)       */
  int32_t reserved;
} tpe_exchange;

/* RCCL communicator of one process per GPU: rank 0 makes the id, the caller
 * broadcasts its TPE_COMM_ID_BYTES bytes, every rank calls tpe_comm_init on
 * its device.  librccl is loaded on first use (no link-time dependency). */
int tpe_comm_unique_id(void* id);
int tpe_comm_init(int32_t rank, int32_t world, const void* id, int32_t device, void** comm);
int tpe_comm_destroy(void* comm);

/* ------------------------------------------------------------------------
 * Device column store (hyperopt_amd/devhist.py; ABI 22).  The observation
 * columns of device-fitted labels are segments of one flat float64 store.
 * tpe_scatter_f64: dst[pos[i]] = val[i] for the k appended observations of a
 * suggest; `src` is the DEVICE address (tpe_pinned_device_address) of pinned
 * host memory holding k doubles then k int64 positions, read by the kernel
 * itself (no copy): the caller keeps it unchanged until the stream has passed
 * the launch.  tpe_move_ranges: a re-layout of a store (or of the value
 * orders' key / position buffers, elem_bytes 8 / 4): for each of n_ranges
 * {src_off, dst_off, n} int64 triples (pinned, device-addressable, as above)
 * dst[dst_off + i] = src[src_off + i], i < n; src and dst distinct buffers.
 * ---------------------------------------------------------------------- */
int tpe_scatter_f64(const void* src, int64_t k, double* dst, void* stream);
int tpe_move_ranges(const void* ranges, int32_t n_ranges, int32_t elem_bytes, const void* src, void* dst,
                    void* stream);

/* collectives (ncclAllGather calls) this library has issued in this process,
 * in *n: the device combine of candidate-sharded levels and
 * tpe_exchange_allgather over RCCL.  A one-rank exchange (world 1, `always`)
 * issues its in-place all-gather only under TPE_FORCE_COMBINE=1 (the N-rank
 * combine run on one GPU: tests), else the gather is the identity and is
 * skipped.  (ABI 22) */
int tpe_collectives_issued(int64_t* n);

/* the exchange's reduction on the host: all[world][P] -> out[P], np.argmax
 * order over (score, global_idx), empty records (idx < 0) skipped */
int tpe_combine_results(const tpe_result* all, int32_t world, int64_t P, tpe_result* out);

/* ------------------------------------------------------------------------
 * Shard axes.  Besides the candidate axis above, a batched suggest shards
 * with no exchange inside the suggest:
 *   new-id axis          every new id is an independent suggest on the same
 *                        history (the reference's one-id call, tpe.py:812,
 *                        repeated): rank r takes a contiguous block of the ids;
 *   hyperparameter axis  broadcast_best is per hyperparameter
 *                        (tpe.py:749-759): rank r evaluates the non-gate labels
 *                        it owns, every rank evaluates the gates (so every rank
 *                        knows which labels are active), the others are
 *                        TPE_F_REMOTE.
 * Candidates are keyed on (seed, label, new id, global index), so each rank
 * computes exactly what one device computes for its part.  The chosen values
 * are then all-gathered once (tpe_exchange_allgather) and every rank holds
 * the whole result.
 * ---------------------------------------------------------------------- */

/* all-gather of `bytes` host bytes per rank through the exchange: all[world *
 * bytes] in rank order.  RCCL (ex->comm): the bytes go through ex->dev (at
 * least world * bytes) on `stream` — one copy in, an in-place ncclAllGather, one
 * copy out, a stream synchronise; else ex->gather.  Rank-collective. */
int tpe_exchange_allgather(const tpe_exchange* ex, const void* mine, int64_t bytes, void* all, void* stream);

/* below_tids ascending (the n_below best trials, tpe.py:625-629); ids: the
 * n_ids new trial ids; n_cand candidates per problem on this rank, global
 * indices [cand_base, cand_base + n_cand) of n_cand_global (unsharded: 0, 0);
 * ex: the shard exchange (NULL unsharded); speculate_min_draws: a gate is
 * predicted when its predicted category is expected among >= this many of the
 * n_cand_global draws;
 * device_fit_min > 0: continuous labels with that many observations get the
 * device Parzen fit of their above side (their below side, <= 25 observations
 * with equal weights, is fitted here) when the record carries dev_obs, else the
 * space is left to the caller's general path.  values / active: [n_ids x n_labels] — the chosen
 * value (categories as doubles) and whether the label is active; path[0] = 1
 * when the fused batch was used, path[1] = level runs issued; need_fit
 * [n_labels]: set to 1 for the labels the caller must fit (TPE_E_FALLBACK).
 * TPE_E_SPACE: grow the workspace to `need` and call again. */
int tpe_suggest_tree(const tpe_tree_label* labels, int32_t n_labels, const int64_t* below_tids, int64_t n_below,
                     double prior_weight, int32_t lf, const int64_t* ids, int32_t n_ids, int32_t n_cand,
                     int64_t cand_base, int64_t n_cand_global, const tpe_exchange* ex,
                     uint64_t seed, double speculate_min_draws, int64_t device_fit_min, int32_t flags,
                     const tpe_level_ws* ws, tpe_level_need* need, void* stream, double* values, int8_t* active,
                     int32_t* path, int8_t* need_fit);

/* Host worker threads of the native runtime, the calling thread included
 * (default: TPE_HOST_THREADS, else 16 — at most the host's CPUs; at most 16).  tpe_suggest_tree fits the
 * labels of a suggest on them in parallel (each label's fit is the same
 * single-threaded computation wherever it runs, so results do not depend on
 * the count).  n <= 1: everything on the calling thread; n < 0: query only.
 * *previous (if not NULL) gets the count before the call.  Not to be called
 * while another thread is inside tpe_suggest_tree. */
int tpe_host_threads(int32_t n, int32_t* previous);

/* ------------------------------------------------------------------------
 * Stage profiler of tpe_level_run (bench.py's live roofline).  While enabled,
 * the runner brackets each stage it calls with HIP events on its own stream and,
 * after its stream synchronise, keeps the per-stage device times of that run.
 * The stages are timed exactly as the production flow issues them: a stage
 * that launches nothing (no fits, no sort, early selection leaving no late
 * problems for the select stage) reports launches = 0 and ms = 0.
 * Process-wide setting; not meant for concurrent runners.
 * ---------------------------------------------------------------------- */
#define TPE_STAGE_FIT      0
#define TPE_STAGE_TABLES   1
#define TPE_STAGE_SAMPLE   2
#define TPE_STAGE_SORT     3
#define TPE_STAGE_ABOVE    4
#define TPE_STAGE_FINALIZE 5
#define TPE_STAGE_SELECT   6
#define TPE_N_STAGES       7

typedef struct tpe_stage_prof {
  double ms;         /* device time between the stage's bracketing events         */
  double units;      /* stage work: fit scratch slots | table units (16 B) |
                        candidates drawn by the sample kernels (lazy categoricals,
                        scanned by the table stage, excluded) | sort bytes (8-bit
                        LSD passes x 2 x 12 B x keys) | above CE | candidates |
                        problems                                                    */
  double ce;         /* algorithmic component evaluations the stage stands in for:
                        sample = tabulated problems' (K_below + K_above) x C,
                        above = scored problems' K_above x C; else 0                */
  int32_t launches;  /* kernels (and library sorts) the stage launched             */
  int32_t kernel_ns; /* sample stage: its tabulated pass's kernel alone, timed by the
                        start / stop events of its own launch (hipExtLaunchKernel) on
                        the stage's stream, in ns; 0 where not timed               */
} tpe_stage_prof;

/* enable (1) / disable (0) the profiler; creates its events on first use */
int tpe_level_profile(int32_t enable);

/* Debug (tests): while `dev` is set, the sample stage's k_sample_fast pass also
 * writes every candidate's {value, l, g, label index} as four doubles at
 * dev[4 * (cand_off + i)] (device memory, n_records >= the level's candidates;
 * the run records are unchanged).  NULL: the production kernel.  Process-wide. */
int tpe_debug_fast_lg(void* dev, int64_t n_records);

/* the last profiled tpe_level_run: min(n, TPE_N_STAGES) records in stage
 * order; TPE_E_ARG if no run completed since the profiler was enabled */
int tpe_level_profile_read(tpe_stage_prof* out, int32_t n);

/* ------------------------------------------------------------------------
 * Host phase clock of tpe_suggest_tree (tools/native_split.py).  While
 * enabled, a call records the steady-clock microseconds since its entry at
 * each phase below (a tree of several level runs: the last run's phases);
 * phases a call does not reach stay -1.  Process-wide; profiling only.
 * ---------------------------------------------------------------------- */
#define TPE_PHASE_PREFIT   0   /* the up-front fits on the worker threads done   */
#define TPE_PHASE_PACK     1   /* the level packed into the staging buffer       */
#define TPE_PHASE_LAUNCHED 2   /* every kernel of the level issued               */
#define TPE_PHASE_SYNCED   3   /* the stream synchronise returned                */
#define TPE_PHASE_LEVEL    4   /* the level's results assembled                  */
#define TPE_PHASE_RETURN   5   /* tpe_suggest_tree returns                       */
#define TPE_PHASE_RECS     6   /* the level's fits and label records ready (before its pack) */
#define TPE_N_PHASES       7

/* enable (1) / disable (0); *last (if not NULL) gets min(n, TPE_N_PHASES)
 * phase times of the last call (before this one changes the setting) */
int tpe_host_phases(int32_t enable, double* last, int32_t n);

#ifdef __cplusplus
}
#endif

#endif /* TPE_HIP_H */
