// tpe_host.cpp — native host runtime of the TPE suggest engine.
//
// Everything the host does per suggest between the history split and the
// device launch: the adaptive Parzen fit (tpe.py:398-475), the categorical
// pseudo-count posteriors (tpe.py:573-607), and the packing of one tree level
// into the device tables of include/tpe_hip.h (component rows, sampler rows,
// pruning grids, problems, candidate tiles, above-mixture work items) — written
// straight into one staging blob that the caller uploads in a single copy.
//
// Float64 semantics follow numpy exactly where the reference's bits depend on
// them: np.sum's pairwise summation (8192-element buffered chunks), linspace's
// i*step + start with an exact endpoint, np.clip, and no FMA contraction (this
// file is compiled with -ffp-contract=off).  The sort permutation of the fit
// comes from the caller (np.argsort) so tie order is the reference's.
#include <math.h>

#include <chrono>
#include <stdio.h>
#include <cmath>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/tpe_hip.h"
#include "tpe_pool.h"

namespace {

constexpr double kEPS = 1e-12;
constexpr double kLog2e = 1.4426950408889634074;
constexpr double kLn2 = 0.69314718055994530942;
constexpr int kPruneMinK = 64;
constexpr int kPruneWide = 16;
// above-mixture work items per level (>= 8 per CU); TPE_TARGET_WORK overrides (tuning)
int target_work() {
  static int v = [] {
    const char* e = getenv("TPE_TARGET_WORK");
    const int x = e ? atoi(e) : 0;
    return x > 0 ? x : 2048;
  }();
  return v;
}
constexpr int kMinComponentsPerSplit = 128;
constexpr int kFineKeyMinCand = 65536;
// value-bucket bits of large candidate sets; TPE_FINE_KEY_BITS overrides (tuning)
int fine_key_bits() {
  static int v = [] {
    const char* e = getenv("TPE_FINE_KEY_BITS");
    const int x = e ? atoi(e) : 0;
    return x > 0 && x <= 16 ? x : 12;
  }();
  return v;
}
constexpr int kTailMinTiles = 32;      // per-tile tail splits from 32 tiles (64k candidates) on
// tabulated scoring (include/tpe_hip.h "Tabulated scoring")
constexpr double kAScale = 0.84932180028801907;   // sqrt(0.5 * log2(e)): a = kAScale / max(sigma, EPS)
constexpr double kTabEta = 0.05;                  // a_max * h <= kTabEta for every cell of half-width h
constexpr int64_t kTabMaxCells = 65536;           // per side; more: per-candidate scoring
constexpr int64_t kTabRowUnits = 3;               // 16-B units of a cell row (include/tpe_hip.h)
constexpr double kTabMinRatio = 8.0, kTabMinRatioDevFit = 64.0;   // candidates per cell row for tables
constexpr int64_t kTabMaxLattice = 1 << 18;       // lattice values per quantized label
// expanded levels (include/tpe_hip.h): from this many problems the device
// writes the problems and tiles itself; TPE_EXPAND=0 turns it off (A/B, tests)
constexpr int64_t kExpandMinProblems = 256;
bool expand_enabled() {
  const char* e = getenv("TPE_EXPAND");
  return !(e && e[0] == '0');
}
// TPE_TABLES=0 turns tabulated scoring off (A/B and tests); read per call
bool tables_enabled() {
  const char* e = getenv("TPE_TABLES");
  return !(e && e[0] == '0');
}
// box moments for device-fitted labels ("Box moments"); TPE_FGT=0 turns them off (A/B, tests)
bool fgt_enabled() {
  const char* e = getenv("TPE_FGT");
  return !(e && e[0] == '0');
}
constexpr double kTabMinRatioFgt = 1.0;          // candidates per cell row for box-moment tables
// log-polynomial rows (TPE_F_LOGPOLY): both sides on the finer side's grid, one
// 48-B row per cell, at most the sample stage's LDS table rows (kTabLdsCells);
// TPE_LOGPOLY=0: moment rows for every cells label (A/B, tests)
constexpr int64_t kLogpolyMaxCells = 2048;
constexpr int64_t kLpDirectRows = 64;       // a side of <= this many rows: direct sums, no moments
constexpr int64_t kLpRowsPerWave = 5;       // ... kLpRowsPerWave cell rows per table-stage wave
constexpr int64_t kMomDirectRows = 64;      // a moment side of <= this many rows: direct sums,
constexpr int64_t kMomCellsPerWave = 4;     // ... kMomCellsPerWave cell rows per table-stage wave
// a TPE_F_LOGPOLY row in cell rows: its above side's moments (one cell row)
// plus the short below side's direct sums at the nodes (5 rows a wave) and the fit
constexpr double kLpRowCost = 1.25;
bool logpoly_enabled() {
  const char* e = getenv("TPE_LOGPOLY");
  return !(e && e[0] == '0');
}
constexpr int64_t kFgtMaxBoxes = 4096;
// a of the device fit's narrowest components: (float)(sqrt(log2(e) / 2) / max(smin, EPS)),
// smin = prior_sigma / min(100, 1 + K) (tpe.py:465-470), as k_fit_emit rounds it
float fgt_a(double prior_sigma, int64_t K) {
  const double smin = prior_sigma / std::min(100.0, 1.0 + (double)K);
  return (float)(0.84932180028801907 / std::max(smin, kEPS));
}
// the box width d = 1 / (a sqrt(ln 2)): a term 2^-(a (t - mu))^2 = e^-((t - mu) / d)^2
double fgt_width(double prior_sigma, int64_t K) {
  return 1.0 / ((double)fgt_a(prior_sigma, K) * std::sqrt(kLn2));
}
// candidates per cell row from which a device-fitted label tabulates
// (TPE_TAB_DEVFIT_RATIO overrides: A/B of the cost model)
double devfit_ratio() {
  const char* e = getenv("TPE_TAB_DEVFIT_RATIO");
  return e && *e ? atof(e) : kTabMinRatioDevFit;
}
// cells of one side: a_max * h <= kTabEta over [lo, hi) (sig_min: the side's smallest bandwidth)
int64_t tab_cells(double lo, double hi, double sig_min) {
  const double a_max = kAScale / std::max(sig_min, kEPS);
  const double n = std::ceil((hi - lo) * a_max / (2.0 * kTabEta));
  return n >= 1.0 && n < 1e15 ? (int64_t)n : -1;
}
// splits of the tile `e` tiles from either end of a pruned problem's sorted
// range: the sparse tails are where waves span too wide a range for the local
// expansion and evaluate their window exactly (measured on the config-3
// problems: the exact work per tile peaks 1-4 tiles in and fades by ~10)
inline int64_t tail_splits(int64_t e) { return e < 6 ? 16 : e < 8 ? 8 : e < 10 ? 4 : e < 12 ? 2 : 1; }

// numpy's pairwise summation (numpy/_core/src/umath/loops_utils.h.src)
double pairwise(const double* a, int64_t n) {
  if (n < 8) {
    double r = 0.;
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise(a, n2) + pairwise(a + n2, n - n2);
}

// np.sum of a contiguous float64 vector: pairwise within 8192-element buffers
double np_sum(const double* a, int64_t n) {
  const int64_t B = 8192;
  double res = 0.;
  for (int64_t s = 0; s < n; s += B) {
    const double p = pairwise(a + s, std::min(B, n - s));
    res = s == 0 ? p : res + p;
  }
  return res;
}

// np.maximum / np.minimum propagate NaN
inline double np_max(double a, double b) { return (a != a || b != b) ? NAN : (a > b ? a : b); }
inline double np_min(double a, double b) { return (a != a || b != b) ? NAN : (a < b ? a : b); }

// erf(z) bit for bit: libm's erf is exactly +-1 from |z| = 6 on (erfc(6) < 2^-55),
// so the (common) far-from-the-bound components skip the call
inline double erf_fast(double z) { return fabs(z) >= 6.0 ? copysign(1.0, z) : erf(z); }
// erfc(x) bit for bit: libm's erfc is exactly 2 from x = -6 down and exactly 0
// from x = 27.3 up (checked over fine grids of both ranges), so the sampler
// rows of components far from a bound skip the call
inline double erfc_fast(double x) { return x <= -6.0 ? 2.0 : (x >= 27.3 ? 0.0 : erfc(x)); }

// erf(z) for |z| < 6 within ~2e-16 of libm's: 7-term Taylor expansions about
// the centres of 1/128-wide intervals, their coefficients erf^(n)(x0) / n! =
// (-1)^(n-1) 2/sqrt(pi) H_(n-1)(x0) e^(-x0^2) / n! (Hermite H) built once from
// libm's erf and exp — an order of magnitude cheaper than libm's exp-based
// branch for |z| >= 1.25.  Only for values that end up in f32 rows (the
// acceptance mass of a continuous f32 side); exact paths keep libm's erf.
struct ErfTable {
  static constexpr int kN = 768, kDeg = 7;          // 6 * 128 intervals
  double c[kN][kDeg];
  ErfTable() {
    const double k2 = 2.0 / sqrt(M_PI);
    for (int j = 0; j < kN; ++j) {
      const double x0 = (j + 0.5) / 128.0, e = exp(-x0 * x0);
      double h0 = 1.0, h1 = 2.0 * x0, fact = 1.0;   // H_0, H_1; n!
      c[j][0] = erf(x0);
      for (int n = 1; n < kDeg; ++n) {
        fact *= n;
        const double hn = n == 1 ? h0 : h1;          // H_(n-1)
        c[j][n] = ((n - 1) % 2 ? -1.0 : 1.0) * k2 * hn * e / fact;
        if (n >= 2) {                                 // H_n = 2 x H_(n-1) - 2 (n-1) H_(n-2)
          const double h2 = 2.0 * x0 * h1 - 2.0 * (n - 1) * h0;
          h0 = h1; h1 = h2;
        }
      }
    }
  }
};
const ErfTable g_erf_tab;
inline double erf_tab(double z) {
  const double x = fabs(z);
  if (!(x < 6.0)) return erf_fast(z);               // (+-1, NaN)
  const int j = (int)(x * 128.0);
  const double d = x - (j + 0.5) / 128.0;
  const double* c = g_erf_tab.c[j];
  double r = c[6];
  for (int n = 5; n >= 0; --n) r = r * d + c[n];
  return copysign(r, z);
}

// sum_k w_k (Phi_k(hi) - Phi_k(lo)) (tpe.py:130-136): the standardised bounds
// in one vectorisable pass, libm's erf only where it is not exactly +-1 (a
// component within 6 sqrt2 sigma of a bound); the same values as the reference's
// normal_cdf (tpe.py:96-101): 0.5 (1 + erf((x - mu) / max(sqrt2 sigma, EPS)))
// (the terms into a[0, k); p_accept sums them, the packer's parallel pass
// computes a large side's in chunks)
__attribute__((target_clones("avx512f", "avx2", "default")))
void p_accept_terms(const double* w, const double* mu, const double* sg, int64_t k, double lo, double hi,
                    double* __restrict__ a, bool fast) {
  static thread_local std::vector<double> z_tl;
  static thread_local std::vector<unsigned char> near_tl;
  z_tl.resize(2 * (size_t)k);
  near_tl.resize((size_t)k);
  double* __restrict__ za = z_tl.data();
  double* __restrict__ zb = za + k;
  unsigned char* __restrict__ near = near_tl.data();
  const double s2 = sqrt(2.0);
  if (fast)                                          // (one division: within an ulp of the quotients)
    for (int64_t i = 0; i < k; ++i) {
      const double t = s2 * sg[i];
      const double r = 1.0 / (t != t ? t : (t > kEPS ? t : kEPS));
      za[i] = (lo - mu[i]) * r;
      zb[i] = (hi - mu[i]) * r;
    }
  else
    for (int64_t i = 0; i < k; ++i) {
      const double t = s2 * sg[i];
      const double bottom = t != t ? t : (t > kEPS ? t : kEPS);     // np_max(sqrt2 sigma, EPS)
      za[i] = (lo - mu[i]) / bottom;
      zb[i] = (hi - mu[i]) / bottom;
    }
  // the terms whose erfs are both exactly +-1, vectorised; the others (a bound
  // within 6 sqrt2 sigma, or NaN) flagged and made with libm's erf after
  int64_t n_near = 0;
  for (int64_t i = 0; i < k; ++i) {
    const bool sh = fabs(zb[i]) >= 6.0, sl = fabs(za[i]) >= 6.0;
    const double eh = sh ? copysign(1.0, zb[i]) : 0.0, el = sl ? copysign(1.0, za[i]) : 0.0;
    a[i] = w[i] * (0.5 * (1 + eh) - 0.5 * (1 + el));
    near[i] = !(sh & sl);
    n_near += !(sh & sl);
  }
  for (int64_t i = 0; n_near > 0 && i < k; ++i)
    if (near[i]) {
      const double eh = fast ? erf_tab(zb[i]) : erf_fast(zb[i]), el = fast ? erf_tab(za[i]) : erf_fast(za[i]);
      a[i] = w[i] * (0.5 * (1 + eh) - 0.5 * (1 + el));
      --n_near;
    }
}

// (fast: erf_tab for the near terms — an f32 side's mass)
double p_accept(const double* w, const double* mu, const double* sg, int64_t k, bool bounded, double lo, double hi,
                bool fast) {
  if (!bounded) return 1.0;
  static thread_local std::vector<double> zl_tl;
  zl_tl.resize((size_t)k);
  p_accept_terms(w, mu, sg, k, lo, hi, zl_tl.data(), fast);
  return np_sum(zl_tl.data(), k);
}

// log2 of a positive normal double: exponent bits + atanh series of the
// mantissa in [sqrt(1/2), sqrt(2)) (|s| <= 0.1716: truncation < 1e-11).  No
// branches, so a loop of it vectorises; used only for the f32 component tables.
inline double log2_normal(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  double e = (double)((int32_t)((u >> 52) & 0x7FF) - 1023);
  u = (u & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;      // m in [1, 2)
  double m;
  memcpy(&m, &u, 8);
  const bool big = m > 1.4142135623730951;
  m = big ? m * 0.5 : m;
  e = big ? e + 1.0 : e;
  const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
  const double p = s * (2.0 + s2 * (2.0 / 3 + s2 * (2.0 / 5 + s2 * (2.0 / 7 + s2 * (2.0 / 9 + s2 * (2.0 / 11))))));
  return e + p * 1.4426950408889634074;
}

// adaptive_parzen_normal (tpe.py:398-475) of n observations given already
// sorted: sv[i] = obs[order[i]] and rank[i] = order[i] (the observation's
// position in tid order, which indexes the linear-forgetting ramp).  Writes
// n + 1 components; returns the prior's position or TPE_E_ARG.  `clean`: sv
// strictly increasing (no NaN, no repeats) — the neighbour gaps are then
// finite and positive, and np.maximum / np.minimum reduce to branch-free
// max / min that vectorise (same values).
template <bool CLEAN>
__attribute__((always_inline)) inline int64_t fit_sorted(const double* __restrict__ sv,
                                                        const int64_t* __restrict__ rank, int64_t n,
                                                        double prior_weight,
                   double prior_mu, double prior_sigma, int32_t lf, double* __restrict__ w, double* __restrict__ mu,
                   double* __restrict__ sigma) {
  auto mx = [](double a, double b) { return CLEAN ? (a > b ? a : b) : np_max(a, b); };
  auto mn = [](double a, double b) { return CLEAN ? (a < b ? a : b) : np_min(a, b); };
  int64_t pos;
  const int64_t K = n + 1;
  if (n == 0) {
    mu[0] = prior_mu; sigma[0] = prior_sigma; pos = 0;
  } else if (n == 1) {
    if (prior_mu < sv[0]) { pos = 0; mu[0] = prior_mu; mu[1] = sv[0]; sigma[0] = prior_sigma; sigma[1] = prior_sigma * .5; }
    else { pos = 1; mu[0] = sv[0]; mu[1] = prior_mu; sigma[0] = prior_sigma * .5; sigma[1] = prior_sigma; }
  } else {
    // np.searchsorted(sorted, prior_mu, side='left') = number of elements < prior_mu
    pos = std::lower_bound(sv, sv + n, prior_mu) - sv;
    memcpy(mu, sv, (size_t)pos * sizeof(double));
    mu[pos] = prior_mu;
    memcpy(mu + pos + 1, sv + pos, (size_t)(n - pos) * sizeof(double));
    for (int64_t i = 1; i < K - 1; ++i) sigma[i] = mx(mu[i] - mu[i - 1], mu[i + 1] - mu[i]);
    sigma[0] = mu[1] - mu[0];
    sigma[K - 1] = mu[K - 1] - mu[K - 2];
  }
  if (lf && lf < n) {
    // linear_forgetting_weights (tpe.py:381-394): np.linspace(1/n, 1, n - lf)
    // (i * step + start, exact endpoint), then ones — looked up by rank
    const int64_t num = n - lf;
    const double start = 1.0 / (double)n;
    const double step = num > 1 ? (1.0 - start) / (double)(num - 1) : 0.0;
    // (branch-free and vectorisable: a rank r in [0, 2^52) converted exactly
    // as the double with r in its mantissa less 2^52 — an integer or and a
    // subtraction, where the clones' AVX-512F has no int64 -> double)
    const bool last_one = num > 1;
    auto ramp = [&](int64_t r) -> double {
      const double rd = __builtin_bit_cast(double, (uint64_t)r | 0x4330000000000000ull) - 4503599627370496.0;
      double y = rd * step;
      y += start;
      const bool one = (r >= num) | ((r == num - 1) & last_one);
      return one ? 1.0 : y;
    };
    for (int64_t i = 0; i < pos; ++i) w[i] = ramp(rank[i]);
    w[pos] = prior_weight;
    for (int64_t i = pos; i < n; ++i) w[i + 1] = ramp(rank[i]);
  } else {
    for (int64_t i = 0; i < K; ++i) w[i] = 1.0;
    w[pos] = prior_weight;
  }
  const double smin = prior_sigma / std::min(100.0, 1.0 + (double)K);
  const double smax = prior_sigma / 1.0;
  for (int64_t i = 0; i < K; ++i) sigma[i] = mn(mx(sigma[i], smin), smax);   // np.clip
  sigma[pos] = prior_sigma;
  int ok = 1;
  for (int64_t i = 0; i < K; ++i) ok &= sigma[i] > 0;
  if (!ok) return TPE_E_ARG;
  const double tot = np_sum(w, K);
  for (int64_t i = 0; i < K; ++i) w[i] = w[i] / tot;
  return pos;
}

// positions of the below set's members among a label's observation tids
// (both ascending; ap_filter_trials' membership test, tpe.py:629-636), in
// ascending order: binary searches when the below set is small (the usual
// 25 of thousands), else one merge
void below_positions(const int64_t* __restrict__ tids, int64_t n, const int64_t* __restrict__ bt, int64_t n_bt,
                     std::vector<int64_t>& pos) {
  pos.clear();
  if (n_bt * 16 < n) {
    const int64_t* lo = tids;
    for (int64_t j = 0; j < n_bt; ++j) {
      lo = std::lower_bound(lo, tids + n, bt[j]);
      if (lo == tids + n) break;
      if (*lo == bt[j]) pos.push_back(lo - tids);
    }
  } else {
    int64_t b = 0;
    for (int64_t t = 0; t < n; ++t) {
      while (b < n_bt && bt[b] < tids[t]) ++b;
      if (b < n_bt && bt[b] == tids[t]) pos.push_back(t);
    }
  }
}

// tids strictly ascending (one branch-free pass)
bool strictly_ascending(const int64_t* __restrict__ tids, int64_t n) {
  int bad = 0;
  for (int64_t i = 1; i < n; ++i) bad |= tids[i] <= tids[i - 1];
  return !bad;
}

// smallest of n doubles (four independent chains: vectorisable; the values
// are positive bandwidths, so min is order-independent)
inline double min_of(const double* __restrict__ v, int64_t n) {
  double m[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
  int64_t i = 0;
  for (; i + 4 <= n; i += 4)
    for (int j = 0; j < 4; ++j) m[j] = v[i + j] < m[j] ? v[i + j] : m[j];
  for (; i < n; ++i) m[0] = v[i] < m[0] ? v[i] : m[0];
  return std::min(std::min(m[0], m[1]), std::min(m[2], m[3]));
}


// the packer's parallel pass over the large bounded sides' acceptance terms
constexpr int64_t kPaParallelMin = 1024;    // a side of at least this many components
constexpr int64_t kPaChunk = 512;           // ... in chunks of this many
struct PaTask { int32_t li, side; int64_t i0, i1, off; bool fast; };

// per-thread staging of tpe_host_pack_level, reused across calls (no
// first-touch page faults on the large tables of a batched level)
// A large tabulated continuous f32 side (no wide list or grid: its cells sum
// every component) is filled in chunks on the worker threads, two passes:
// terms (a and the unshifted c into scratch, the chunk's largest c), then rows
// once the side's shift (the largest c of all chunks) is known.
constexpr int64_t kFillChunk = 1024;
constexpr int64_t kFitStageStretch = 9 * 256;    // tpe_kernels.hip kFitStretch (a chunk's staged stretch)
constexpr int64_t kFillChunkMinLevel = 16384;   // the level's chunkable components, at least
// (TPE_FILL_CHUNK_MIN: another threshold, A/B)
inline int64_t fill_chunk_min_level() {
  static const int64_t v = [] {
    const char* e = getenv("TPE_FILL_CHUNK_MIN");
    return e && *e ? (int64_t)atoll(e) : kFillChunkMinLevel;
  }();
  return v;
}
struct ChunkTask { int32_t li, side; int64_t i0, i1; int64_t scr; };

struct PackScratch {
  std::vector<float> comp32;
  std::vector<double> comp64, samp;
  std::vector<int32_t> grid, fin_tiles, samp_tiles, tab_tiles;
  std::vector<tpe_problem> prob;
  std::vector<tpe_tile> tiles;
  std::vector<tpe_work> work;
  std::vector<tpe_tab_job> tab_jobs;
  std::vector<tpe_problem> xtmpl;       // expanded levels: one problem template per label
  std::vector<int32_t> xfirst;          // ... each label's first problem (n_labels + 1)
  std::vector<uint32_t> xctr;           // ... each problem's new id (Philox counter word 3)
  std::vector<int64_t> pa_off;          // acceptance terms of the large bounded sides
  std::vector<double> pa_terms;
  std::vector<PaTask> pa_tasks;
  std::vector<char> chunked;            // chunked fills (ChunkTask)
  std::vector<ChunkTask> ch_tasks;
  std::vector<double> ch_a, ch_c, ch_max, side_shift;
  std::vector<int> mass_tasks;          // ... each bounded chunked side's mass task (its first chunk)
};

// value range of a label's kernel coordinate (x, or ln x for log families)
// that its candidates fall in: the bounds, else the below mixture +- 8 sigma
// (f32 draws stay within 5.5 sigma of their component); categories [0, upper)
void coord_range(const tpe_label_in& L, double& klo, double& khi) {
  if (L.family == TPE_FAM_CATEGORICAL) { klo = 0; khi = std::max(L.upper, 1); return; }
  if ((L.flags & TPE_F_HAS_LOW) && (L.flags & TPE_F_HAS_HIGH)) { klo = L.low; khi = L.high; return; }
  klo = INFINITY; khi = -INFINITY;
  for (int64_t i = 0; i < L.below_k; ++i) {
    klo = std::min(klo, L.below_mu[i] - 8 * L.below_sigma[i]);
    khi = std::max(khi, L.below_mu[i] + 8 * L.below_sigma[i]);
  }
}

// the table decision of one label (tpe_host_pack_level): which scoring its
// candidates get — cells (moment rows or TPE_F_LOGPOLY rows), box-moment
// cells, a lattice or none — and the geometry; labels are independent
struct TabCtx {
  const tpe_label_in* labels;
  const char* dev_fit;
  int32_t n_cand;
  bool f64, lp_on, fgt_on;
  double dv_ratio;
  int32_t* tmode;
  int64_t *tn0, *tn1, *tlat;
  double *tklo, *tkhi;
  int64_t* fgt_boxes;
  char* logpoly;
};

constexpr int32_t kTabChunk = 16;

void decide_table(const TabCtx& cx, int32_t li) {
  const tpe_label_in* labels = cx.labels;
  const char* dev_fit = cx.dev_fit;
  const int32_t n_cand = cx.n_cand;
  const bool f64 = cx.f64;
  int32_t* tmode = cx.tmode;
  int64_t *tn0 = cx.tn0, *tn1 = cx.tn1, *tlat = cx.tlat, *fgt_boxes = cx.fgt_boxes;
  double *tklo = cx.tklo, *tkhi = cx.tkhi;
  char* logpoly = cx.logpoly;
  const tpe_label_in& L = labels[li];
  const double ct = (double)L.n_ids * (double)n_cand;     // candidates of the label in this level
  if (L.n_ids <= 0 || L.family == TPE_FAM_CATEGORICAL || L.below_k <= 0) return;
  double klo, khi;
  coord_range(L, klo, khi);
  if (!(std::isfinite(klo) && std::isfinite(khi) && khi > klo)) return;
  tklo[li] = klo; tkhi[li] = khi;
  if ((L.family == TPE_FAM_GAUSS || L.family == TPE_FAM_LOGGAUSS) && !f64) {
    double s0 = INFINITY, s1 = INFINITY;
    s0 = min_of(L.below_sigma, L.below_k);
    if (dev_fit[li])           // the device fit clips every bandwidth to >= prior_sigma / min(100, 1 + K)
      s1 = L.prior_sigma / std::min(100.0, 1.0 + (double)L.above_k);
    else
      s1 = min_of(L.above_sigma, L.above_k);
    const int64_t n0 = tab_cells(klo, khi, s0), n1 = L.above_k > 0 ? tab_cells(klo, khi, s1) : -1;
    // a cell row costs ~10x a candidate's score (two passes plus the f64
    // moments), more against the pruned, locally expanded per-candidate path
    // of a device-fitted mixture: tables pay from kTabMinRatio candidates a cell
    // a device-fitted mixture's above cells built from box moments ("Box
    // moments": ~16 boxes per cell instead of every component within reach)
    // pay from about one candidate a cell
    int64_t nbox = 0;
    if (dev_fit[li] && cx.fgt_on && n1 > 0) {
      const double d = fgt_width(L.prior_sigma, L.above_k);
      const double nb = std::ceil((khi - klo) / d) + 1.0;
      if (d > 0 && nb >= 1.0 && nb <= (double)kFgtMaxBoxes) nbox = (int64_t)nb;
    }
    const double ratio = nbox > 0 ? kTabMinRatioFgt : dev_fit[li] ? cx.dv_ratio : kTabMinRatio;
    const int64_t nl = std::max(n0, n1);
    const double lp_ratio = dev_fit[li] ? cx.dv_ratio : kTabMinRatio;   // (moment cells, no boxes)
    // (box-moment labels keep moment cells: their above cells come from the boxes)
    if (cx.lp_on && nbox == 0 && n0 > 0 && n1 > 0 && nl <= kLogpolyMaxCells &&
        ct >= lp_ratio * kLpRowCost * (double)nl) {
      // both sides' log-polynomials on one grid (the finer side's cells): one
      // row per candidate look-up (include/tpe_hip.h, TPE_F_LOGPOLY)
      tmode[li] = TPE_TAB_CELLS; tn0[li] = tn1[li] = nl;
      logpoly[li] = 1;
    } else if (n0 > 0 && n1 > 0 && n0 <= kTabMaxCells && n1 <= kTabMaxCells && ct >= ratio * (double)(n0 + n1)) {
      tmode[li] = TPE_TAB_CELLS; tn0[li] = n0; tn1[li] = n1;
      fgt_boxes[li] = nbox;
    }
  } else if ((L.family == TPE_FAM_QGAUSS || L.family == TPE_FAM_QLOGGAUSS) && L.q > 0 && L.above_k > 0 &&
             !(L.flags & TPE_F_NO_TABLE)) {
    // every value a device draw can take: bounded draws stay in [low, high];
    // unbounded ones within 8.3 sigma of their component (53-bit uniforms)
    double tlo = klo, thi = khi;
    if (!((L.flags & TPE_F_HAS_LOW) && (L.flags & TPE_F_HAS_HIGH))) {
      tlo = INFINITY; thi = -INFINITY;
      for (int64_t i = 0; i < L.below_k; ++i) {
        tlo = std::min(tlo, L.below_mu[i] - 9 * L.below_sigma[i]);
        thi = std::max(thi, L.below_mu[i] + 9 * L.below_sigma[i]);
      }
    }
    const bool lg = L.family == TPE_FAM_QLOGGAUSS;
    const double xlo = lg ? exp(tlo) : tlo, xhi = lg ? exp(thi) : thi;
    const double mlo = std::floor(xlo / L.q) - 1.0, mhi = std::ceil(xhi / L.q) + 1.0;
    const double nl = mhi - mlo + 1.0;
    if (std::isfinite(nl) && nl >= 1.0 && nl <= (double)kTabMaxLattice && std::fabs(mlo) < 9e15 &&
        ct >= 2.0 * nl) {
      tmode[li] = TPE_TAB_LATTICE; tn0[li] = (int64_t)nl; tlat[li] = (int64_t)mlo;
    }
  }
}

// the largest finite value of c[0, n) (-inf: none) — four lanes at a time in
// GCC vector types, so that every clone vectorises it (the max of finite values
// is exact in any order)
inline __attribute__((always_inline)) double finite_max(const double* __restrict__ c, int64_t n) {
  typedef double v4d __attribute__((vector_size(32)));
  const v4d ninf = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, pinf = {INFINITY, INFINITY, INFINITY, INFINITY};
  v4d m = ninf;
  int64_t i = 0;
  for (; i + 4 <= n; i += 4) {
    v4d v;
    memcpy(&v, c + i, sizeof(v));
    v = (v > ninf) & (v < pinf) ? v : ninf;
    m = v > m ? v : m;
  }
  double r = std::max(std::max(m[0], m[1]), std::max(m[2], m[3]));
  for (; i < n; ++i) {
    const double v = (c[i] > -INFINITY) & (c[i] < INFINITY) ? c[i] : -INFINITY;
    r = v > r ? v : r;
  }
  return r;
}

// f32 component terms of a continuous side's components [0, n) (pointers
// already offset): a = sqrt(log2e / 2) / max(sigma, EPS) and the unshifted
// c = log2(w / (sigma sqrt(2 pi)) / p_accept) (the log family: no p_accept);
// straight-line passes the compiler vectorises, the bit-level log2 for normal
// positive ratios, libm for the rest.  Returns the largest finite c.
inline __attribute__((always_inline)) double comp_terms_f32(const double* __restrict__ w, const double* __restrict__ sg,
                                                            int64_t n, bool logf, double ipa, double* __restrict__ ap,
                                                            double* __restrict__ cp) {
  const double s2pi = sqrt(2 * M_PI), as = sqrt(0.5 * kLog2e);
  // one division per component: 1 / max(sigma, EPS) (the rows are f32; the
  // ratio's double rounding differs from w / (sigma sqrt(2 pi)) by an ulp)
  {
    const double cst = logf ? 1.0 / s2pi : ipa / s2pi;
    int tiny = 0;
    for (int64_t i = 0; i < n; ++i) {
      const double se = sg[i] > kEPS ? sg[i] : kEPS;
      const double inv = 1.0 / se;
      tiny |= !(sg[i] > kEPS);
      cp[i] = w[i] * inv * cst;
      ap[i] = as * inv;
    }
    if (tiny && !logf)       // |sigma| < EPS: the reference divides by |sigma| itself
      for (int64_t i = 0; i < n; ++i)
        if (!(sg[i] > kEPS)) cp[i] = w[i] / (s2pi * fabs(sg[i])) * ipa;
  }
  int odd = 0;
  for (int64_t i = 0; i < n; ++i) {
    const double r = cp[i];
    odd |= !((r >= 2.2250738585072014e-308) & (r <= 1.7976931348623157e308));
    cp[i] = log2_normal(r > 0 ? r : 1.0);
  }
  if (odd)
    for (int64_t i = 0; i < n; ++i) {
      const double r = w[i] / (logf ? ((sg[i] > kEPS ? sg[i] : kEPS) * s2pi) : (s2pi * fabs(sg[i]))) *
                       (logf ? 1.0 : ipa);
      if (!((r >= 2.2250738585072014e-308) & (r <= 1.7976931348623157e308))) cp[i] = log2(r);
    }
  return finite_max(cp, n);
}

// f32 component rows {mu_hi, mu_lo, a, c - shift} of components [0, n)
inline __attribute__((always_inline)) void comp_rows_f32(const double* __restrict__ mu, const double* __restrict__ a,
                                                         const double* __restrict__ c, int64_t n, double shift,
                                                         float* __restrict__ r) {
  for (int64_t i = 0; i < n; ++i, r += 4) {
    const float hi = (float)mu[i];
    r[0] = hi; r[1] = (float)(mu[i] - (double)hi); r[2] = (float)a[i]; r[3] = (float)(c[i] - shift);
  }
}

// one label's sections of tpe_host_pack_level (sampler rows, component rows,
// wide rows, pruning grid) at the offsets the packer assigned; labels are
// independent, so the packer runs this on its worker threads.  (A function of
// its own so that it carries the AVX-512 / AVX2 clones: a lambda would not.)
struct LabelSec { int64_t samp, c64[2], c32[2], wide, grid; };
struct FillCtx {
  const tpe_label_in* labels;
  const LabelSec* sec;
  tpe_problem* lab;
  double* samp;
  double* comp64;
  float* comp32;
  int32_t* grid;
  const char* dev_fit;
  const int32_t* tmode;
  int key_bits;
  bool f64;
  const double* pa_terms;      // a large bounded side's acceptance terms (the packer's parallel pass)
  const int64_t* pa_off;       // [2 * label + side]: their offset in pa_terms, -1: none
  const char* chunked;         // [2 * label + side]: rows filled by chunk tasks (ChunkTask)
};

// the acceptance mass of label li's side: the terms the parallel pass made, or p_accept
inline double side_accept(const FillCtx& cx, int32_t li, int side, const double* w, const double* mu,
                          const double* sg, int64_t k, bool bounded, double lo, double hi, bool fast) {
  const int64_t o = cx.pa_off[2 * (size_t)li + side];
  return o >= 0 ? np_sum(cx.pa_terms + o, k) : p_accept(w, mu, sg, k, bounded, lo, hi, fast);
}

struct PaCtx { const tpe_label_in* labels; const PaTask* tasks; double* terms; };
void pa_chunk(const PaCtx& cx, int t) {
  const PaTask& q = cx.tasks[t];
  const tpe_label_in& L = cx.labels[q.li];
  const double* w = q.side ? L.above_w : L.below_w;
  const double* mu = q.side ? L.above_mu : L.below_mu;
  const double* sg = q.side ? L.above_sigma : L.below_sigma;
  p_accept_terms(w + q.i0, mu + q.i0, sg + q.i0, q.i1 - q.i0, L.low, L.high, cx.terms + q.off + q.i0, q.fast);
}

__attribute__((target_clones("avx512f", "avx2", "default")))
void fill_label(const FillCtx& cx, int32_t li) {
#ifdef TPE_PACK_TRACE
  const auto t_fill0 = std::chrono::steady_clock::now();
  struct Done {
    std::chrono::steady_clock::time_point t0; int32_t li;
    ~Done() {                 // (TPE_PACK_TRACE_LABELS=1: each label's fill time too)
      static const bool on = getenv("TPE_PACK_TRACE_LABELS") != nullptr;
      if (on)
        fprintf(stderr, "fill_label %d %.1f us\n", li,
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
  } done_{t_fill0, li};
#endif
  const tpe_label_in* labels = cx.labels;
  const bool f64 = cx.f64;
  const int key_bits = cx.key_bits;
  const char* dev_fit = cx.dev_fit;
  const int32_t* tmode = cx.tmode;
  const tpe_label_in& L = labels[li];
  const LabelSec& sc = cx.sec[li];
  tpe_problem& p = cx.lab[li];
  memset(&p, 0, sizeof(p));
  p.family = L.family; p.flags = L.flags; p.n_upper = L.upper;
  p.low = L.low; p.high = L.high; p.q = L.q;
  const bool bounded = (L.flags & (TPE_F_HAS_LOW | TPE_F_HAS_HIGH)) != 0;
  // ---- sampler rows (below mixture) ----
  p.samp_off = (int32_t)sc.samp;
  double* srow = cx.samp + 8 * (size_t)sc.samp;
  if (L.family == TPE_FAM_CATEGORICAL) {
    const int64_t k = L.below_k;
    double acc = 0;
    std::vector<double> cum((size_t)k);
    for (int64_t i = 0; i < k; ++i) { acc += L.below_w[i]; cum[i] = acc; }
    for (int64_t i = 0; i < k; ++i) {
      const double row[8] = {i == k - 1 ? 1.0 : cum[i] / acc, 0, 0, 0, 0, 0, 0, 0};
      memcpy(srow + 8 * i, row, sizeof(row));
    }
    p.samp_len = (int32_t)k;
    // lazy scoring (TPE_F_CAT_LAZY): the winner is the best-scoring drawable
    // category (np.argmax order: NaN first, then value, then index)
    if (k <= 64 && L.above_k == k) {
      const double* row0 = srow;
      int64_t c1 = -1;
      double s1 = 0, p1 = 0;
      for (int64_t i = 0; i < k; ++i) {
        const double lo = i ? row0[8 * (i - 1)] : 0.0, pi = row0[8 * i] - lo;
        if (!(pi > 0)) continue;
        const double sc1 = log(L.below_w[i]) - log(L.above_w[i]);
        const bool win = c1 < 0 || (sc1 != sc1 ? s1 == s1 : sc1 > s1);
        if (win) { c1 = i; s1 = sc1; p1 = pi; }
      }
      if (c1 >= 0 && p1 >= 1.0 / 65536) p.flags |= TPE_F_CAT_LAZY;
    }
  } else {
    const int64_t k = L.below_k;
    std::vector<double> sel((size_t)k), fa((size_t)k), fb((size_t)k), flip((size_t)k);
    double tot = 0;
    bool any = false;
    for (int64_t i = 0; i < k; ++i) {
      double za = -INFINITY, zb = INFINITY;
      if (bounded) { za = (L.low - L.below_mu[i]) / L.below_sigma[i]; zb = (L.high - L.below_mu[i]) / L.below_sigma[i]; }
      const bool fl = za > 0;
      const double a = fl ? -zb : za, b = fl ? -za : zb;
      fa[i] = 0.5 * erfc_fast(-a / sqrt(2.0));
      fb[i] = 0.5 * erfc_fast(-b / sqrt(2.0));
      flip[i] = fl ? 1.0 : 0.0;
      sel[i] = bounded ? L.below_w[i] * std::max(fb[i] - fa[i], 0.0) : L.below_w[i];
      any = any || sel[i] > 0;
    }
    if (!any) for (int64_t i = 0; i < k; ++i) sel[i] = L.below_w[i];
    for (int64_t i = 0; i < k; ++i) tot += sel[i];
    double acc = 0;
    for (int64_t i = 0; i < k; ++i) {
      acc += sel[i];
      const double row[8] = {i == k - 1 ? 1.0 : acc / tot, L.below_mu[i], L.below_sigma[i], fa[i], fb[i], flip[i], 0, 0};
      memcpy(srow + 8 * i, row, sizeof(row));
    }
    p.samp_len = (int32_t)k;
  }
  // ---- sort-key range of the kernel coordinate ----
  double klo, khi;
  coord_range(L, klo, khi);
  p.key_lo = (float)klo;
  p.key_inv = khi > klo ? (float)((double)(1 << key_bits) / (khi - klo)) : 0.f;
  // ---- component rows ----
  for (int side = 0; side < 2 - dev_fit[li]; ++side) {
    const double* w = side ? L.above_w : L.below_w;
    const double* mu = side ? L.above_mu : L.below_mu;
    const double* sg = side ? L.above_sigma : L.below_sigma;
    const int64_t k = side ? L.above_k : L.below_k;
    int32_t& off = side ? p.above_off : p.below_off;
    int32_t& len = side ? p.above_len : p.below_len;
    double& base = side ? p.above_base : p.below_base;
    if (L.family == TPE_FAM_CATEGORICAL) {
      off = (int32_t)sc.c64[side]; len = (int32_t)k; base = 0;
      double* r = cx.comp64 + 4 * (size_t)off;
      for (int64_t i = 0; i < k; ++i) {
        const double row[4] = {log(w[i]), w[i], 0, 0};
        memcpy(r + 4 * i, row, sizeof(row));
      }
    } else if (L.family == TPE_FAM_QGAUSS || L.family == TPE_FAM_QLOGGAUSS) {
      off = (int32_t)sc.c64[side]; len = (int32_t)k;
      base = -log(side_accept(cx, li, side, w, mu, sg, k, bounded, L.low, L.high, false));
      double* r = cx.comp64 + 4 * (size_t)off;
      for (int64_t i = 0; i < k; ++i) {
        const double row[4] = {mu[i], np_max(sqrt(2.0) * sg[i], kEPS), w[i], 0};
        memcpy(r + 4 * i, row, sizeof(row));
      }
    } else {
      const bool logf = L.family == TPE_FAM_LOGGAUSS;
      if (cx.chunked[2 * (size_t)li + side]) {      // (its terms and rows: the chunk tasks; its base: the packer)
        off = (int32_t)sc.c32[side]; len = (int32_t)k;
        continue;
      }
      std::vector<double> a((size_t)k), c((size_t)k);
      const double pa = logf ? 1.0 : side_accept(cx, li, side, w, mu, sg, k, bounded, L.low, L.high, !f64);
      double shift = -INFINITY;
      if (f64) {
        for (int64_t i = 0; i < k; ++i) {
          const double se = np_max(sg[i], kEPS);
          const double arg = logf ? w[i] / (se * sqrt(2 * M_PI)) : w[i] / sqrt(2 * M_PI * sg[i] * sg[i]) / pa;
          c[i] = log(arg) * kLog2e;
          a[i] = sqrt(0.5 * kLog2e) / se;
        }
        shift = finite_max(c.data(), k);
      } else {
        shift = comp_terms_f32(w, sg, k, logf, 1.0 / pa, a.data(), c.data());
      }
      if (!std::isfinite(shift)) shift = 0;
      for (int64_t i = 0; i < k; ++i) c[i] -= shift;
      base = shift * kLn2;
      if (f64) {
        off = (int32_t)sc.c64[side]; len = (int32_t)k;
        double* r = cx.comp64 + 4 * (size_t)off;
        for (int64_t i = 0; i < k; ++i) {
          const double row[4] = {mu[i], a[i], c[i], 0};
          memcpy(r + 4 * i, row, sizeof(row));
        }
        continue;
      }
      // pruning (above side, f32, scored per candidate): widest components
      // listed apart, grid over mu.  A tabulated label's cells sum every
      // component (k_tables), so it has neither.
      std::vector<int64_t> wide;
      if (side == 1 && k > kPruneMinK && tmode[li] == TPE_TAB_NONE) {
        // the kPruneWide smallest a (widest sigma), ascending by (a, index): one
        // pass with a small insertion-sorted buffer (= a stable argsort prefix)
        int64_t best[kPruneWide];
        int nb = 0;
        for (int64_t i = 0; i < k; ++i) {
          if (nb == kPruneWide && !(a[i] < a[best[nb - 1]])) continue;   // ties keep the lower index
          int q = nb < kPruneWide ? nb++ : nb - 1;
          while (q > 0 && a[i] < a[best[q - 1]]) { best[q] = best[q - 1]; --q; }
          best[q] = i;
        }
        wide.assign(best, best + nb);
      }
      off = (int32_t)sc.c32[side]; len = (int32_t)k;
      {
        const size_t b0 = 4 * (size_t)sc.c32[side];
        float* r = cx.comp32 + b0;
        for (int64_t i = 0; i < k; ++i, r += 4) {
          const float hi = (float)mu[i];
          r[0] = hi; r[1] = (float)(mu[i] - (double)hi); r[2] = (float)a[i]; r[3] = (float)c[i];
        }
        for (int64_t i : wide) cx.comp32[b0 + 4 * (size_t)i + 3] = -INFINITY;
      }
      std::vector<char> is_wide((size_t)k, 0);
      for (int64_t i : wide) is_wide[i] = 1;
      if (!wide.empty()) {
        p.wide_off = (int32_t)sc.wide;
        p.wide_len = (int32_t)wide.size();
        float* wr = cx.comp32 + 4 * (size_t)sc.wide;
        for (int64_t i : wide) {
          const float hi = (float)mu[i];
          const float row[4] = {hi, (float)(mu[i] - (double)hi), (float)a[i], (float)c[i]};
          memcpy(wr, row, sizeof(row));
          wr += 4;
        }
        const int64_t anchor = wide[0];
        double cmax = -INFINITY, amin = INFINITY;
        for (int64_t i = 0; i < k; ++i)
          if (!is_wide[i]) { cmax = std::max(cmax, c[i]); amin = std::min(amin, a[i]); }
        p.prior_mu = (float)mu[anchor]; p.prior_a = (float)a[anchor]; p.prior_c = (float)c[anchor];
        p.narrow_cmax = (float)cmax; p.narrow_amin = (float)amin;
        const double lo = (double)(float)mu[0], hi = (double)(float)mu[k - 1];
        const int64_t G = std::min<int64_t>(4096, 4 * k);
        const float inv = hi > lo ? (float)((double)G / (hi - lo)) : 0.f;
        p.grid_off = (int32_t)sc.grid; p.grid_n = (int32_t)G;
        p.grid_lo = (float)lo; p.grid_inv = inv;
        // grid[g] = first component with mu32 >= edge_g, edge_g = lo + g * (1 / inv)
        // = #components whose first bucket with edge > mu32 is <= g: a counting
        // pass (bucket estimate + exact edge correction) and a prefix sum —
        // no data-dependent branches in the merge
        const double step = inv > 0 ? 1.0 / (double)inv : 0.0;
        const size_t g0 = (size_t)sc.grid;
        int32_t* __restrict__ gp = cx.grid + g0;
        if (!(inv > 0)) memset(gp, 0, (size_t)G * sizeof(int32_t));
        if (inv > 0) {
          // four interleaved histograms: sorted mu puts neighbours in the same
          // bucket, and one array would chain every increment through memory
          const size_t H = (size_t)G + 1;
          std::vector<int32_t> hist(4 * H, 0);
          const double dinv = (double)inv;
          for (int64_t i = 0; i < k; ++i) {
            const double x = (double)(float)mu[i];
            int64_t g = (int64_t)((x - lo) * dinv) + 1;     // first bucket with edge > x, estimated
            g = g < 0 ? 0 : (g > G ? G : g);
            while (g > 0 && lo + (double)(g - 1) * step > x) --g;
            while (g < G && !(lo + (double)g * step > x)) ++g;
            ++hist[(size_t)(i & 3) * H + (size_t)g];
          }
          int32_t acc = 0;
          for (int64_t g = 0; g < G; ++g) {
            acc += hist[(size_t)g] + hist[H + (size_t)g] + hist[2 * H + (size_t)g] + hist[3 * H + (size_t)g];
            gp[g] = acc;
          }
        }
        gp[G] = (int32_t)k;
      }
    }
  }
}

// the chunk tasks' two passes (ChunkTask; tpe_host_pack_level)
struct ChunkCtx {
  const tpe_label_in* labels;
  const ChunkTask* tasks;
  double* a;                   // scratch: each chunked side's a and unshifted c at ChunkTask.scr
  double* c;
  double* cmax;                // per task: the chunk's largest finite c
  double* pa_terms;            // the bounded sides' acceptance terms (terms pass) ...
  const int64_t* pa_off;       // ... at [2 * label + side] (-1: unbounded or the log family)
  const double* shift;         // [2 * label + side]: the side's shift (rows pass)
  const LabelSec* sec;
  float* comp32;
};

__attribute__((target_clones("avx512f", "avx2", "default")))
void chunk_terms(const ChunkCtx& x, int t) {
  const ChunkTask& q = x.tasks[t];
  const tpe_label_in& L = x.labels[q.li];
  const double* w = q.side ? L.above_w : L.below_w;
  const double* sg = q.side ? L.above_sigma : L.below_sigma;
  const size_t s = 2 * (size_t)q.li + q.side;
  // the chunk's acceptance terms beside (the side's mass is summed after the
  // pass: it only moves the side's base, c - shift is the same)
  if (x.pa_off[s] >= 0) {
    const double* mu = q.side ? L.above_mu : L.below_mu;
    p_accept_terms(w + q.i0, mu + q.i0, sg + q.i0, q.i1 - q.i0, L.low, L.high, x.pa_terms + x.pa_off[s] + q.i0, true);
  }
  x.cmax[t] = comp_terms_f32(w + q.i0, sg + q.i0, q.i1 - q.i0, L.family == TPE_FAM_LOGGAUSS, 1.0,
                             x.a + q.scr + q.i0, x.c + q.scr + q.i0);
}

__attribute__((target_clones("avx512f", "avx2", "default")))
void chunk_rows(const ChunkCtx& x, int t) {
  const ChunkTask& q = x.tasks[t];
  const tpe_label_in& L = x.labels[q.li];
  const double* mu = q.side ? L.above_mu : L.below_mu;
  const size_t s = 2 * (size_t)q.li + q.side;
  comp_rows_f32(mu + q.i0, x.a + q.scr + q.i0, x.c + q.scr + q.i0, q.i1 - q.i0, x.shift[s],
                x.comp32 + 4 * (size_t)(x.sec[q.li].c32[q.side] + q.i0));
}

}  // namespace

extern "C" {

int64_t tpe_host_fit_parzen(const double* obs, int64_t n, const int64_t* order, double prior_weight,
                            double prior_mu, double prior_sigma, int32_t lf, double* w, double* mu,
                            double* sigma) {
  if (n < 0 || (n >= 2 && !order) || !w || !mu || !sigma) return TPE_E_ARG;
  static thread_local std::vector<double> sv;
  static thread_local std::vector<int64_t> rank;
  sv.resize((size_t)n);
  rank.resize((size_t)n);
  double* svp = sv.data();
  int64_t* rkp = rank.data();
  for (int64_t i = 0; i < n; ++i) {
    const int64_t r = n >= 2 ? order[i] : i;
    if (r < 0 || r >= n) return TPE_E_ARG;
    rkp[i] = r;
    svp[i] = obs[r];
  }
  return fit_sorted<false>(svp, rkp, n, prior_weight, prior_mu, prior_sigma, lf, w, mu, sigma);
}

// (AVX-512 / AVX2 clones: -ffp-contract=off holds in all, so the results are identical)
__attribute__((target_clones("avx512f", "avx2", "default")))
int tpe_host_fit_split(const double* x, const int64_t* tids, const int64_t* order, int64_t n,
                       const int64_t* below_tids, int64_t n_bt, double prior_weight, double prior_mu,
                       double prior_sigma, int32_t lf, double* out, int64_t* out_k) {
  if (n < 0 || n_bt < 0 || (n && (!x || !tids || !order)) || (n_bt && !below_tids) || !out || !out_k)
    return TPE_E_ARG;
  if (!strictly_ascending(tids, n)) return TPE_E_ARG;
  // (thread-local staging, looked up once: a TLS access in a loop costs a call)
  static thread_local std::vector<int64_t> pos_tl, code_tl, rk_tl[2];
  static thread_local std::vector<double> sv_tl[2];
  std::vector<int64_t>& pos = pos_tl;
  below_positions(tids, n, below_tids, n_bt, pos);
  // every tid-order position t coded as its rank within its side: r >= 0 above,
  // ~r below (segment fills between the below positions)
  code_tl.resize((size_t)n);
  int64_t* __restrict__ code = code_tl.data();
  const int64_t nb = (int64_t)pos.size(), na = n - nb;
  {
    int64_t t0 = 0;
    for (int64_t j = 0; j <= nb; ++j) {
      const int64_t t1 = j < nb ? pos[(size_t)j] : n;
      for (int64_t t = t0; t < t1; ++t) code[t] = t - j;
      if (j < nb) code[t1] = ~j;
      t0 = t1 + 1;
    }
  }
  // each side in value order (the label's sorting permutation filtered) with
  // its tid-order ranks — the order np.argsort gives when no value repeats
  sv_tl[0].resize((size_t)nb + 1); rk_tl[0].resize((size_t)nb + 1);
  sv_tl[1].resize((size_t)na + 1); rk_tl[1].resize((size_t)na + 1);
  double* __restrict__ sb = sv_tl[0].data();
  double* __restrict__ sa = sv_tl[1].data();
  int64_t* __restrict__ rb = rk_tl[0].data();
  int64_t* __restrict__ ra = rk_tl[1].data();
  int64_t cb = 0, ca = 0;
  int bad = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t t = order[i];
    // (the gather's address depends on order[i] alone: every iteration's loads
    // can be in flight at once — a clamp through `bad` chained them, one cache
    // latency an observation)
    bad |= (uint64_t)t >= (uint64_t)n;
    const int64_t tt = (uint64_t)t < (uint64_t)n ? t : 0;
    const int64_t c = code[tt];
    const double v = x[tt];
    // (the below side is ~25 of them: a predictable branch, half the stores of
    // writing both sides; a count past its side stays on that side's spare slot)
    if (__builtin_expect(c >= 0, 1)) {
      const int64_t wa = ca < na ? ca : na;
      sa[wa] = v; ra[wa] = c; ++ca;
    } else {
      const int64_t wb = cb < nb ? cb : nb;
      sb[wb] = v; rb[wb] = ~c; ++cb;
    }
  }
  bad |= (ca != na) | (cb != nb);
  if (bad) return TPE_E_ARG;                          // not a permutation
  const int64_t cap = n + 1;
  for (int sd = 0; sd < 2; ++sd) {
    const double* __restrict__ v = sd ? sa : sb;
    const int64_t m = sd ? na : nb;
    out_k[sd] = 0;
    // NaN sorts last in `order`; a repeated value leaves the tie order to np.argsort
    int fallback = m >= 1 && v[0] != v[0];
    for (int64_t i = 1; i < m; ++i) fallback |= !(v[i - 1] < v[i]);
    if (fallback) continue;       // the caller refits the side with numpy's permutation
    double* w = out + (3 * sd) * cap;
    const int64_t p = fit_sorted<true>(v, sd ? ra : rb, m, prior_weight, prior_mu, prior_sigma, lf, w, w + cap,
                                       w + 2 * cap);
    if (p < 0) return (int)p;
    out_k[sd] = m + 1;
  }
  return TPE_OK;
}

__attribute__((target_clones("avx512f", "avx2", "default")))
int tpe_host_cat_probs(const int64_t* obs, int64_t n, int32_t upper, const double* p_prior, double prior_weight,
                       int32_t lf, double* out) {
  if (upper <= 0 || n < 0 || !out) return TPE_E_ARG;
  // np.bincount(obs, linear_forgetting_weights(n, lf), upper): per category the
  // weights summed in observation order — four interleaved passes would change
  // that order, so one pass, with the ramp computed on the fly
  static thread_local std::vector<double> counts_tl;
  counts_tl.assign((size_t)upper, 0.0);
  double* counts = counts_tl.data();
  const bool ramp = lf && n >= lf;
  const int64_t num = ramp ? n - lf : 0;
  const double start = n > 0 ? 1.0 / (double)n : 0.0;
  const double step = num > 1 ? (1.0 - start) / (double)(num - 1) : 0.0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t c = obs[i];
    if (c < 0 || c >= upper) return TPE_E_ARG;
    double wi = 1.0;
    if (i < num) {
      if (num == 1) wi = start;
      else if (i < num - 1) { wi = (double)i * step; wi += start; }
    }
    counts[c] += wi;
  }
  for (int32_t k = 0; k < upper; ++k)
    counts[k] = p_prior ? counts[k] + (double)upper * (prior_weight * p_prior[k]) : counts[k] + prior_weight;
  const double tot = np_sum(counts, upper);
  for (int32_t k = 0; k < upper; ++k) out[k] = counts[k] / tot;
  return TPE_OK;
}

int tpe_host_cat_split(const int64_t* obs, const int64_t* tids, int64_t n, const int64_t* below_tids, int64_t n_bt,
                       int32_t upper, const double* p_prior, double prior_weight, int32_t lf, double* out_below,
                       double* out_above) {
  if (n < 0 || n_bt < 0 || (n && (!obs || !tids)) || (n_bt && !below_tids) || !out_below || !out_above)
    return TPE_E_ARG;
  if (!strictly_ascending(tids, n)) return TPE_E_ARG;
  // ap_filter_trials (tpe.py:629-636): the below members' positions, then both
  // sides in tid order (the above side as the segments between them)
  static thread_local std::vector<int64_t> pos_tl, side_tl[2];
  std::vector<int64_t>& pos = pos_tl;
  below_positions(tids, n, below_tids, n_bt, pos);
  const int64_t nb = (int64_t)pos.size();
  std::vector<int64_t>& below = side_tl[0];
  std::vector<int64_t>& above = side_tl[1];
  below.resize((size_t)nb);
  above.resize((size_t)(n - nb));
  int64_t* __restrict__ bp = below.data();
  int64_t* __restrict__ ap = above.data();
  int64_t t0 = 0, k = 0;
  for (int64_t j = 0; j <= nb; ++j) {
    const int64_t t1 = j < nb ? pos[(size_t)j] : n;
    if (t1 > t0) memcpy(ap + k, obs + t0, (size_t)(t1 - t0) * sizeof(int64_t));
    k += t1 - t0;
    if (j < nb) bp[j] = obs[t1];
    t0 = t1 + 1;
  }
  const int rc = tpe_host_cat_probs(bp, nb, upper, p_prior, prior_weight, lf, out_below);
  if (rc) return rc;
  return tpe_host_cat_probs(ap, n - nb, upper, p_prior, prior_weight, lf, out_above);
}

// the level runner's early-fit hook (tpe_level_run): called on the packing
// thread once the blob's leading sections are placed and the fit jobs written,
// before the fill — so the device fit runs while the host fills the rest
static thread_local TpePackHook g_pack_hook = {nullptr, nullptr};

__attribute__((visibility("hidden"))) void tpe_internal_pack_hook(TpePackHook h) { g_pack_hook = h; }

// the pack's straight-line table loops vectorise: an AVX2 clone is picked at
// load time on hosts that have it (-ffp-contract=off holds in both clones, so
// the tables are bit-identical)
__attribute__((target_clones("avx512f", "avx2", "default")))
// (TPE_PACK_TRACE builds, tools/pack_time*.py: the packer's sections timed)
#ifdef TPE_PACK_TRACE
#define PACK_MARK(name) pack_marks.emplace_back(name, std::chrono::steady_clock::now())
#define PACK_DONE()                                                                              \
  do {                                                                                           \
    for (size_t i_ = 1; i_ < pack_marks.size(); ++i_)                                            \
      fprintf(stderr, "pack %-16s %8.1f us\n", pack_marks[i_].first,                             \
              std::chrono::duration<double, std::micro>(pack_marks[i_].second - pack_marks[i_ - 1].second).count()); \
  } while (0)
#else
#define PACK_MARK(name) (void)0
#define PACK_DONE() (void)0
#endif

int tpe_host_pack_level(const tpe_label_in* labels, int32_t n_labels, int32_t n_cand, uint64_t seed,
                        int64_t cand_base, int64_t n_cand_global, int32_t precision, void* blob, int64_t blob_cap,
                        tpe_pack_info* info) {
#ifdef TPE_PACK_TRACE
  std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> pack_marks;
  PACK_MARK("entry");
#endif
  if (!info || n_labels < 0 || n_cand < 0 || (n_labels && !labels)) return TPE_E_ARG;
  const bool f64 = precision == TPE_PREC_F64;
  const int T = 2048;
  // staging tables: per-thread, reused across calls (no first-touch page faults
  // on the large ones — a batched level has ~10^5 problems, tiles and work items)
  // (one thread-local lookup: references to its members stay in registers —
  // a thread_local named inside a loop costs a TLS call per use in a shared object)
  static thread_local PackScratch tls_scratch;
  PackScratch& ps = tls_scratch;
  auto& comp32 = ps.comp32;     // float4 rows
  auto& comp64 = ps.comp64;     // double4 rows
  auto& samp = ps.samp;         // 8 doubles per row
  auto& grid = ps.grid;
  std::vector<tpe_problem> lab((size_t)n_labels);
  int64_t P = 0;
  std::vector<char> dev_fit((size_t)n_labels, 0);   // above mixture fitted on the device
  for (int32_t li = 0; li < n_labels; ++li) {
    const tpe_label_in& L = labels[li];
    P += L.n_ids;
    if (L.dev_obs && !L.above_mu) {
      if ((L.family != TPE_FAM_GAUSS && L.family != TPE_FAM_LOGGAUSS) || f64 || L.n_below < 0 || L.n_below > 64 ||
          (L.n_below > 0 && !L.below_idx) || L.n_obs - L.n_below + 1 != L.above_k || L.above_k <= kPruneMinK ||
          L.n_obs >= ((int64_t)1 << 31) || L.n_ord_in < 0 || L.n_ord_in > L.n_obs ||
          (L.n_ord_in > 0 && (!L.ord_key_in || !L.ord_idx_in)) ||
          (L.n_ord_in < L.n_obs && (!L.ord_key_out || !L.ord_idx_out) &&
           !(L.n_ord_in > 0 && L.n_obs - L.n_ord_in <= TPE_FIT_DELTA_MAX && !L.ord_key_out && !L.ord_idx_out)))
        return TPE_E_ARG;
      dev_fit[li] = 1;
    }
  }
  PACK_MARK("devfit");
  // ---- tabulated scoring: which labels score from tables, and their geometry ----
  const bool tab_on = tables_enabled();
  std::vector<int32_t> tmode((size_t)n_labels, TPE_TAB_NONE);
  std::vector<int64_t> tn0((size_t)n_labels, 0), tn1((size_t)n_labels, 0), tlat((size_t)n_labels, 0);
  std::vector<double> tklo((size_t)n_labels, 0), tkhi((size_t)n_labels, 0);
  std::vector<int64_t> fgt_boxes((size_t)n_labels, 0);   // box-moment labels: their boxes
  std::vector<char> logpoly((size_t)n_labels, 0);         // TPE_F_LOGPOLY labels
  if (tab_on && n_cand > 0) {
    const TabCtx tcx{labels, dev_fit.data(), n_cand, f64, logpoly_enabled(), fgt_enabled(), devfit_ratio(),
                     tmode.data(), tn0.data(), tn1.data(), tlat.data(), tklo.data(), tkhi.data(), fgt_boxes.data(),
                     logpoly.data()};
    // (a label's decision reads its whole above mixture: thousands of
    // components per label make a worker's hand-off worth it; a device-fitted
    // label's reads only its below side — config 5's 125 labels a rank decide in
    // 5 us on one thread, 11-14 us handed out)
    int64_t comps = 0;
    for (int32_t li = 0; li < n_labels; ++li) comps += dev_fit[li] ? labels[li].below_k : labels[li].above_k;
    // (in chunks of up to kTabChunk labels: a thousand-label level's decisions
    // are sub-microsecond each, too small to hand out one by one; a few large
    // labels — config 4's twenty of 10^4 components — one a task)
    struct Chunked { const TabCtx* cx; int32_t n, per; };
    const int32_t per = std::max<int32_t>(1, std::min<int32_t>(kTabChunk, n_labels / (4 * (1 + tpe_pool::workers()))));
    const Chunked ch{&tcx, n_labels, per};
    if (n_labels >= 2 && comps >= 16384)
      tpe_pool::parallel_for((n_labels + per - 1) / per, [](void* c, int k) {
        const Chunked& q = *(const Chunked*)c;
        for (int32_t li = k * q.per; li < std::min(q.n, (k + 1) * q.per); ++li) decide_table(*q.cx, li);
      }, (void*)&ch);
    else
      for (int32_t li = 0; li < n_labels; ++li) decide_table(tcx, li);
  }
  PACK_MARK("tmode");
  // Pruned problems (continuous f32 above mixtures of more than kPruneMinK
  // components, not tabulated) are the only ones whose candidates are sorted; they own the
  // candidate range [0, sort_count).  Sort key = sort_slot << key_bits | value
  // bucket: one 8-bit radix pass up to 8 sorted problems, never below 32
  // buckets per problem.  Large candidate sets get 4096 buckets (two passes):
  // a wave of 512 sorted candidates then spans ~1/8 of a bucket's density,
  // narrow enough for the above kernel's local expansion.
  // A pruned label active for several ids is POOLED: its problems share one
  // sort slot and are sorted as one population (include/tpe_hip.h).
  std::vector<char> pruned((size_t)n_labels, 0), pooled((size_t)n_labels, 0);
  int64_t S = 0, n_sorted_prob = 0, n_pooled = 0, max_slot_cand = 0;   // S: sort slots
  for (int32_t li = 0; li < n_labels; ++li) {
    const tpe_label_in& L = labels[li];
    pruned[li] = !f64 && (L.family == TPE_FAM_GAUSS || L.family == TPE_FAM_LOGGAUSS) &&
                 (dev_fit[li] || L.above_k > kPruneMinK) && tmode[li] == TPE_TAB_NONE;
    pooled[li] = pruned[li] && L.n_ids >= 2;
    if (!pruned[li]) continue;
    S += pooled[li] ? 1 : L.n_ids;
    n_sorted_prob += L.n_ids;
    if (pooled[li]) n_pooled += L.n_ids;
    max_slot_cand = std::max(max_slot_cand, (pooled[li] ? L.n_ids : 1) * (int64_t)n_cand);
  }
  int pbits = 0;
  while (((int64_t)1 << pbits) < S) ++pbits;
  int key_bits = std::max(5, 8 - pbits);
  if (max_slot_cand >= kFineKeyMinCand) key_bits = std::max(key_bits, std::min(fine_key_bits(), 16 - pbits));
  const int sort_end_bit = S > 0 && key_bits + pbits <= 32 ? key_bits + pbits : 0;
  PACK_MARK("prune");
  // ---- per-label sections: every label's sampler rows, component rows, wide
  // rows and pruning grid get their offsets first (label order, as appended
  // one after another), then each label fills its own sections — on the host
  // worker threads when the level has enough components (labels independent) ----
  std::vector<LabelSec> sec((size_t)n_labels);
  int64_t n_samp = 0, n_c64 = 0, n_c32 = 0, n_grid = 0, work_k = 0;
  for (int32_t li = 0; li < n_labels; ++li) {
    const tpe_label_in& L = labels[li];
    LabelSec& q = sec[(size_t)li];
    q.samp = n_samp; n_samp += L.below_k;
    // (a label's fill beyond its rows: the sampler rows' four erfc a below
    // component and a fixed part — a thousand device-fitted labels of 26 host
    // components each are 3.7 us of fill a label, worth the workers)
    work_k += 4 * L.below_k + 64;
    q.c64[0] = q.c64[1] = q.c32[0] = q.c32[1] = q.wide = q.grid = -1;
    const bool rows64 = L.family == TPE_FAM_CATEGORICAL || L.family == TPE_FAM_QGAUSS ||
                        L.family == TPE_FAM_QLOGGAUSS || f64;
    for (int side = 0; side < 2 - dev_fit[li]; ++side) {
      const int64_t k = side ? L.above_k : L.below_k;
      work_k += k;
      if (rows64) { q.c64[side] = n_c64; n_c64 += k; continue; }
      q.c32[side] = n_c32; n_c32 += k;
      if (side == 1 && k > kPruneMinK && tmode[li] == TPE_TAB_NONE) {   // wide rows + grid (pruned)
        q.wide = n_c32; n_c32 += std::min<int64_t>(kPruneWide, k);
        q.grid = n_grid; n_grid += std::min<int64_t>(4096, 4 * k) + 1;
      }
    }
  }
  PACK_MARK("sizing");
  // ---- device-fitted above mixtures: rows and grids after the host ones, fit
  // jobs (before the fill: the level runner may launch the fit right away) ----
  // (the device grid starts 256-B aligned: the host part's upload never
  // touches a word the fit wrote)
  const int64_t host_rows = n_c32, host_grid = std::max<int64_t>(n_grid, 1);
  const int64_t host_grid_pad = (host_grid + 63) & ~(int64_t)63;
  std::vector<tpe_fit_job> fit;
  std::vector<int32_t> below_idx;
  std::vector<int64_t> fit_seg(1, 0);
  std::vector<int32_t> fit_li;          // each fit job's label
  {
    int64_t nf = 0, nb = 0;
    for (int32_t li = 0; li < n_labels; ++li)
      if (dev_fit[li]) { ++nf; nb += std::max<int32_t>(labels[li].n_below, 0); }
    fit.reserve((size_t)nf); below_idx.reserve((size_t)nb + 1); fit_seg.reserve((size_t)nf + 1);
  }
  int64_t dev_rows = 0, dev_grid = 0, fit_max_new = 0, fit_max_obs = 0, fit_max_merge = 0, fit_n_delta = 0;
  {
    int64_t r = 0;
    for (int32_t li = 0; li < n_labels; ++li) {
      const tpe_label_in& L = labels[li];
      if (dev_fit[li]) {
        const int64_t K = L.above_k, G = std::min<int64_t>(4096, 4 * K);
        tpe_fit_job j;
        memset(&j, 0, sizeof(j));
        j.obs = L.dev_obs; j.n_obs = L.n_obs; j.seg_off = fit_seg.back();
        j.below_off = (int32_t)below_idx.size(); j.n_below = L.n_below;
        j.family = L.family; j.flags = L.flags; j.lf = L.lf;
        j.problem_first = (int32_t)r; j.n_problems = (int32_t)L.n_ids;
        j.above_off = (int32_t)(host_rows + dev_rows); j.wide_off = (int32_t)(host_rows + dev_rows + K);
        j.grid_off = (int32_t)(host_grid_pad + dev_grid); j.grid_n = (int32_t)G;
        j.prior_mu = L.prior_mu; j.prior_sigma = L.prior_sigma; j.prior_weight = L.prior_weight;
        j.low = L.low; j.high = L.high;
        j.ord_key_in = L.ord_key_in; j.ord_idx_in = L.ord_idx_in; j.n_ord_in = L.n_ord_in;
        j.ord_key_out = L.ord_key_out; j.ord_idx_out = L.ord_idx_out;
        for (int32_t b = 0; b < L.n_below; ++b) {
          if (L.below_idx[b] < 0 || L.below_idx[b] >= L.n_obs || (b && L.below_idx[b] <= L.below_idx[b - 1]))
            return TPE_E_ARG;
          below_idx.push_back(L.below_idx[b]);
        }
        fit.push_back(j);
        fit_li.push_back(li);
        // scratch segment: the compacted above order, the new observations' merge
        // passes and the below positions all fit in it
        const int64_t n_new = L.n_obs - L.n_ord_in;
        // (delta mode: the delta arrays, then a slot of kFitStageStretch entries per
        // 2048-component chunk for the chunks whose stretch holds a delta entry)
        const int64_t slots = !L.ord_key_out && n_new > 0 ? ((K + 2047) / 2048) * kFitStageStretch : 0;
        fit_seg.push_back(fit_seg.back() + std::max<int64_t>(std::max<int64_t>(K - 1, n_new),
                                                             std::max<int64_t>(L.n_below, 64 + 2 * TPE_FIT_DELTA_MAX + slots)));
        fit_max_new = std::max(fit_max_new, n_new);
        if (L.ord_key_out) fit_max_merge = std::max(fit_max_merge, n_new);
        else fit_n_delta += n_new > 0;          // (delta mode)
        fit_max_obs = std::max<int64_t>(fit_max_obs, L.n_obs);
        dev_rows += K + kPruneWide;
        dev_grid += G + 1;
      }
      r += L.n_ids;
    }
  }
  if (host_rows + dev_rows >= ((int64_t)1 << 31) || host_grid_pad + dev_grid >= ((int64_t)1 << 31)) return TPE_E_ARG;
  if (below_idx.empty()) below_idx.push_back(0);
  PACK_MARK("devrows");
  // ---- expanded levels (include/tpe_hip.h "Expanded levels"): when every label
  // of a large level scores from tables, its problems differ from their label's
  // only in (cand_off, ctr3, tile_off) and its tiles are {problem, j * T, 0, 0}
  // in order: the host writes one template per label and the new ids, the
  // device (k_expand) writes the problems and tiles — ~240 B + 32 B per (label,
  // id) neither packed nor uploaded ----
  const int64_t n_tiles_p = n_cand > 0 ? (n_cand + T - 1) / T : 0;
  bool expand = expand_enabled() && !f64 && P >= kExpandMinProblems && n_tiles_p > 0;
  for (int32_t li = 0; li < n_labels && expand; ++li)
    if (labels[li].n_ids > 0 && tmode[li] == TPE_TAB_NONE) expand = false;
  // ---- the blob's leading sections, placed before the fill (the fill writes
  // its sections in place; the device fit may run while it does):
  //   fit jobs | below positions | fit segments | grid (host | device, 256-B
  //   aligned) | comp32 (host | device) | fit patches (device only: the problem
  //   fields the fit writes, applied after the upload) | problems | tiles
  //   (device only when expanded) | comp64 | sampler rows
  // then the later sections (work, finalize tiles, table jobs, tile lists, the
  // expanded level's templates) after them ----
  const int NL = 10;
  const int64_t len_lead[NL] = {(int64_t)(fit.size() * sizeof(tpe_fit_job)), (int64_t)(below_idx.size() * sizeof(int32_t)),
                                (int64_t)(fit_seg.size() * sizeof(int64_t)), (host_grid_pad + dev_grid) * 4,
                                (host_rows + dev_rows) * 16, fit.empty() ? 0 : P * (int64_t)sizeof(tpe_problem),
                                P * (int64_t)sizeof(tpe_problem), P * n_tiles_p * (int64_t)sizeof(tpe_tile),
                                n_c64 * 32, n_samp * 64};
  int64_t off_lead[NL], lead_end = 0;
  for (int i = 0; i < NL; ++i) {
    off_lead[i] = (lead_end + 255) & ~(int64_t)255;
    lead_end = off_lead[i] + len_lead[i];
  }
  enum { L_FIT, L_BIDX, L_FSEG, L_GRID, L_C32, L_PATCH, L_PROB, L_TILES, L_C64, L_SAMP };
  // the fill's targets: the blob itself when it holds the leading sections,
  // else the scratch (the call then only sizes the level: TPE_E_SPACE)
  const bool direct = blob != nullptr && blob_cap >= lead_end;
  unsigned char* const bb = (unsigned char*)blob;
  float* f_comp32;
  double *f_comp64, *f_samp;
  int32_t* f_grid;
  if (direct) {
    f_comp32 = (float*)(bb + off_lead[L_C32]);
    f_comp64 = (double*)(bb + off_lead[L_C64]);
    f_samp = (double*)(bb + off_lead[L_SAMP]);
    f_grid = (int32_t*)(bb + off_lead[L_GRID]);
  } else {
    // (trivially typed: a resize to the same size as the last call touches nothing)
    comp32.resize((size_t)(4 * n_c32));
    comp64.resize((size_t)(4 * n_c64));
    samp.resize((size_t)(8 * n_samp));
    grid.resize((size_t)host_grid);
    f_comp32 = comp32.data(); f_comp64 = comp64.data(); f_samp = samp.data(); f_grid = grid.data();
  }
  f_grid[0] = 0;
  if (direct && !fit.empty()) {
    memcpy(bb + off_lead[L_FIT], fit.data(), (size_t)len_lead[L_FIT]);
    memcpy(bb + off_lead[L_BIDX], below_idx.data(), (size_t)len_lead[L_BIDX]);
    memcpy(bb + off_lead[L_FSEG], fit_seg.data(), (size_t)len_lead[L_FSEG]);
    if (g_pack_hook.fn) {
      // the level runner uploads the fit sections and launches the device fit
      tpe_pack_info e;
      memset(&e, 0, sizeof(e));
      e.off_fit = off_lead[L_FIT]; e.off_below_idx = off_lead[L_BIDX]; e.off_fit_seg = off_lead[L_FSEG];
      e.off_grid = off_lead[L_GRID]; e.off_comp32 = off_lead[L_C32]; e.off_patch = off_lead[L_PATCH];
      e.n_fit = (int32_t)fit.size(); e.fit_total = fit_seg.back();
      e.fit_max_new = fit_max_new; e.fit_max_obs = fit_max_obs; e.fit_max_merge = fit_max_merge;
      e.fit_n_delta = fit_n_delta; e.n_problems = P;
      e.up_off[0] = 0; e.up_len[0] = off_lead[L_FSEG] + len_lead[L_FSEG]; e.n_up = 1;
      e.blob_bytes = off_lead[L_PATCH] + len_lead[L_PATCH];     // (the device bytes the fit touches)
      g_pack_hook.fn(g_pack_hook.ctx, &e);
    }
  }
  PACK_MARK("lead");
  // large tabulated continuous f32 sides: in chunks (ChunkTask), their
  // acceptance terms in the same tasks as their component terms
  auto& chunked = ps.chunked;
  auto& ch_tasks = ps.ch_tasks;
  auto& side_shift = ps.side_shift;
  chunked.assign(2 * (size_t)n_labels, 0);
  ch_tasks.clear();
  int64_t ch_total = 0;
  // (only a level with many such components: a chunked side costs a second
  // hand-off to the workers, more than it saves on the headline's few thousand)
  int64_t chunkable = 0;
  for (int32_t li = 0; li < n_labels && !f64; ++li) {
    const tpe_label_in& L = labels[li];
    if ((L.family != TPE_FAM_GAUSS && L.family != TPE_FAM_LOGGAUSS) || tmode[li] == TPE_TAB_NONE) continue;
    for (int side = 0; side < 2 - dev_fit[li]; ++side) {
      const int64_t k = side ? L.above_k : L.below_k;
      if (k > kFillChunk) chunkable += k;
    }
  }
  if (chunkable >= fill_chunk_min_level())
    for (int32_t li = 0; li < n_labels; ++li) {
      const tpe_label_in& L = labels[li];
      if ((L.family != TPE_FAM_GAUSS && L.family != TPE_FAM_LOGGAUSS) || tmode[li] == TPE_TAB_NONE) continue;
      for (int side = 0; side < 2 - dev_fit[li]; ++side) {
        const int64_t k = side ? L.above_k : L.below_k;
        if (k <= kFillChunk) continue;
        chunked[2 * (size_t)li + side] = 1;
        const int64_t nch = (k + kFillChunk - 1) / kFillChunk;
        for (int64_t j = 0; j < nch; ++j)
          ch_tasks.push_back(ChunkTask{li, side, k * j / nch, k * (j + 1) / nch, ch_total});
        ch_total += k;
      }
    }
  // the acceptance terms of the large bounded sides in chunks on the workers
  // (libm erf for every component near a bound: the largest label's would
  // otherwise be its fill's critical path); the fill sums them in order
  auto& pa_off = ps.pa_off;
  auto& pa_terms = ps.pa_terms;
  auto& pa_tasks = ps.pa_tasks;
  pa_off.assign(2 * (size_t)n_labels, -1);
  pa_tasks.clear();
  int64_t pa_total = 0;
  for (int32_t li = 0; li < n_labels; ++li) {
    const tpe_label_in& L = labels[li];
    if (!(L.flags & (TPE_F_HAS_LOW | TPE_F_HAS_HIGH)) || L.family == TPE_FAM_CATEGORICAL ||
        L.family == TPE_FAM_LOGGAUSS)
      continue;
    const bool fast = L.family == TPE_FAM_GAUSS && !f64;   // (an f32 side's mass: erf_tab)
    for (int side = 0; side < 2 - dev_fit[li]; ++side) {
      const int64_t k = side ? L.above_k : L.below_k;
      const bool ch = chunked[2 * (size_t)li + side] != 0;     // (its terms: the chunk tasks)
      if (k < kPaParallelMin && !ch) continue;
      pa_off[2 * (size_t)li + side] = pa_total;
      for (int64_t i0 = 0; i0 < k && !ch; i0 += kPaChunk)
        pa_tasks.push_back(PaTask{li, side, i0, std::min(k, i0 + kPaChunk), pa_total, fast});
      pa_total += k;
    }
  }
  pa_terms.resize((size_t)pa_total);
  if (!pa_tasks.empty()) {
    const PaCtx pcx{labels, pa_tasks.data(), pa_terms.data()};
    tpe_pool::parallel_for((int)pa_tasks.size(), [](void* c, int i) { pa_chunk(*(const PaCtx*)c, i); }, (void*)&pcx);
  }
  PACK_MARK("accept");
  const FillCtx fcx{labels, sec.data(), lab.data(), f_samp, f_comp64, f_comp32, f_grid,
                    dev_fit.data(), tmode.data(), key_bits, f64, pa_terms.data(), pa_off.data(), chunked.data()};
  const int n_ch = (int)ch_tasks.size();
  ChunkCtx ccx{labels, ch_tasks.data(), nullptr, nullptr, nullptr, pa_terms.data(), pa_off.data(), nullptr,
               sec.data(), f_comp32};
  if (n_ch) {
    ps.ch_a.resize((size_t)ch_total);
    ps.ch_c.resize((size_t)ch_total);
    ps.ch_max.resize((size_t)n_ch);
    side_shift.assign(2 * (size_t)n_labels, 0.0);
    ccx.a = ps.ch_a.data(); ccx.c = ps.ch_c.data(); ccx.cmax = ps.ch_max.data();
    ccx.shift = side_shift.data();
  }
  {
    // the labels' fills and the chunks' terms, one task each (a few hundred
    // components per label make a worker's hand-off worth it)
    struct Both { const FillCtx* f; const ChunkCtx* c; int32_t n_labels; };
    const Both both{&fcx, &ccx, n_labels};
    auto task = [](void* v, int i) {
      const Both& b = *(const Both*)v;
      if (i < b.n_labels) fill_label(*b.f, (int32_t)i);
      else chunk_terms(*b.c, i - b.n_labels);
    };
    const int n_tasks = n_labels + n_ch;
    if (n_tasks >= 2 && work_k >= 4096) tpe_pool::parallel_for(n_tasks, task, (void*)&both);
    else
      for (int i = 0; i < n_tasks; ++i) task((void*)&both, i);
  }
  PACK_MARK("fill_terms");
  if (n_ch) {
    // each chunked side's shift (the largest finite c of its chunks) and base,
    // then its rows
    for (int t = 0; t < n_ch; ++t) {
      const size_t q = 2 * (size_t)ch_tasks[t].li + ch_tasks[t].side;
      side_shift[q] = ch_tasks[t].i0 == 0 ? ps.ch_max[t] : std::max(side_shift[q], ps.ch_max[t]);
    }
    for (int32_t li = 0; li < n_labels; ++li)
      for (int side = 0; side < 2; ++side) {
        const size_t q = 2 * (size_t)li + side;
        if (!chunked[q]) continue;
        if (!std::isfinite(side_shift[q])) side_shift[q] = 0;
        (side ? lab[li].above_base : lab[li].below_base) = side_shift[q] * kLn2;
      }
    // the rows, and each bounded side's mass (its terms summed in numpy's
    // order) into its base: log2(w / (sigma sqrt(2 pi)) / p) - shift =
    // c' - shift' with shift = shift' + log2(1 / p), one task a side (named by
    // its first chunk)
    auto& mass = ps.mass_tasks;
    mass.clear();
    for (int t = 0; t < n_ch; ++t)
      if (ch_tasks[t].i0 == 0 && pa_off[2 * (size_t)ch_tasks[t].li + ch_tasks[t].side] >= 0) mass.push_back(t);
    struct Rows { const ChunkCtx* c; tpe_problem* lab; const int* mass; int n_ch; };
    const Rows rw{&ccx, lab.data(), mass.data(), n_ch};
    auto rows = [](void* v, int t) {
      const Rows& r = *(const Rows*)v;
      if (t < r.n_ch) { chunk_rows(*r.c, t); return; }
      const ChunkTask& q = r.c->tasks[r.mass[t - r.n_ch]];
      const size_t sd = 2 * (size_t)q.li + q.side;
      const tpe_label_in& L = r.c->labels[q.li];
      const double pa = np_sum(r.c->pa_terms + r.c->pa_off[sd], q.side ? L.above_k : L.below_k);
      double& base = q.side ? r.lab[q.li].above_base : r.lab[q.li].below_base;
      base = pa > 0 && pa < INFINITY ? base - log(pa) : NAN;      // (NaN: refilled below)
    };
    const int n_rows = n_ch + (int)mass.size();
    if (n_rows >= 2) tpe_pool::parallel_for(n_rows, rows, (void*)&rw);
    else rows((void*)&rw, 0);
    // a side whose mass is 0, inf or NaN: its rows with 1 / p inside c, as
    // fill_label makes them (the rows carry the non-finite values, base 0)
    for (int m : mass) {
      const ChunkTask& q0 = ch_tasks[m];
      tpe_problem& p = lab[q0.li];
      double& base = q0.side ? p.above_base : p.below_base;
      if (base == base) continue;
      const tpe_label_in& L = labels[q0.li];
      const size_t sd = 2 * (size_t)q0.li + q0.side;
      const double ipa = 1.0 / np_sum(pa_terms.data() + pa_off[sd], q0.side ? L.above_k : L.below_k);
      const double* w = q0.side ? L.above_w : L.below_w;
      const double* sg = q0.side ? L.above_sigma : L.below_sigma;
      double sh = -INFINITY;
      for (int t = m; t < n_ch && ch_tasks[t].li == q0.li && ch_tasks[t].side == q0.side; ++t) {
        const ChunkTask& q = ch_tasks[t];
        sh = std::max(sh, comp_terms_f32(w + q.i0, sg + q.i0, q.i1 - q.i0, false, ipa, ccx.a + q.scr + q.i0,
                                         ccx.c + q.scr + q.i0));
      }
      side_shift[sd] = std::isfinite(sh) ? sh : 0.0;
      base = side_shift[sd] * kLn2;
      for (int t = m; t < n_ch && ch_tasks[t].li == q0.li && ch_tasks[t].side == q0.side; ++t) chunk_rows(ccx, t);
    }
  }
  PACK_MARK("fill");
  // the device-fitted labels' problem fields (the fill cleared their rows)
  for (size_t k = 0; k < fit.size(); ++k) {
    const tpe_fit_job& j = fit[k];
    tpe_problem& p = lab[fit_li[k]];
    p.above_off = j.above_off; p.above_len = (int32_t)(j.n_obs - j.n_below + 1);
    p.wide_off = j.wide_off;
    p.grid_off = j.grid_off; p.grid_n = j.grid_n;
    p.narrow_amin = 1.f;       // pruned; the fit stage writes the real value
  }
  // ---- score tables: 16-B units (a cell row is 3 units, a lattice row 1) ----
  int64_t tab_units = 0, fgt_max_boxes = 0;
  for (int32_t li = 0; li < n_labels; ++li) {
    tpe_problem& p = lab[li];
    p.tab_mode = tmode[li];
    if (tmode[li] == TPE_TAB_CELLS && logpoly[li]) {
      // one table, both sides' polynomials in each row
      const int64_t n = tn0[li];
      p.flags |= TPE_F_LOGPOLY;
      for (int sd = 0; sd < 2; ++sd) {
        p.tab_off[sd] = (int32_t)tab_units;
        p.tab_n[sd] = (int32_t)n;
        p.tab_lo[sd] = (float)tklo[li];
        p.tab_inv[sd] = (float)((double)n / (tkhi[li] - tklo[li]));
      }
      tab_units += kTabRowUnits * n;
    } else if (tmode[li] == TPE_TAB_CELLS) {
      for (int sd = 0; sd < 2; ++sd) {
        const int64_t n = sd ? tn1[li] : tn0[li];
        p.tab_off[sd] = (int32_t)tab_units;
        p.tab_n[sd] = (int32_t)n;
        p.tab_lo[sd] = (float)tklo[li];
        p.tab_inv[sd] = (float)((double)n / (tkhi[li] - tklo[li]));
        tab_units += kTabRowUnits * n;
      }
      if (fgt_boxes[li] > 0) {              // box records after the label's cells ("Box moments")
        const tpe_label_in& L = labels[li];
        p.flags |= TPE_F_FGT;
        p.fgt_a = fgt_a(L.prior_sigma, L.above_k);
        p.fgt_off = (int32_t)tab_units;
        p.fgt_n = (int32_t)fgt_boxes[li];
        p.fgt_lo = tklo[li];
        tab_units += 1 + TPE_FGT_BOX_UNITS * fgt_boxes[li];
        fgt_max_boxes = std::max(fgt_max_boxes, fgt_boxes[li]);
      }
    } else if (tmode[li] == TPE_TAB_LATTICE) {
      p.tab_off[0] = (int32_t)tab_units;
      p.tab_n[0] = (int32_t)tn0[li];
      p.lat_lo = tlat[li];
      tab_units += tn0[li] + (tn0[li] + 1 + 3) / 4;      // {l, g} rows, then n + 1 f32 entry thresholds
    }
  }
  if (tab_units >= ((int64_t)1 << 31)) return TPE_E_ARG;
  PACK_MARK("tabunits");
  // ---- problems, tiles, work (problem rows and tiles straight into the blob) ----
  int64_t scored = 0;
  const int64_t C_ref = n_cand_global > 0 ? n_cand_global : n_cand;
  auto& xtmpl = ps.xtmpl;
  auto& xfirst = ps.xfirst;
  auto& xctr = ps.xctr;
  xtmpl.clear(); xfirst.clear(); xctr.clear();
  if (expand) {
    xtmpl.resize((size_t)n_labels);
    xfirst.resize((size_t)n_labels + 1);
    xctr.resize((size_t)P);
    int64_t r = 0;
    for (int32_t li = 0; li < n_labels; ++li) {
      tpe_problem q = lab[li];
      q.n_cand = n_cand;
      q.cand_off = 0;                     // k_expand: problem r's candidates at r * n_cand
      q.sort_slot = -1;
      q.pool_first = -1;
      q.cand_base = cand_base;
      q.n_cand_global = C_ref;
      q.key0 = (uint32_t)seed; q.key1 = (uint32_t)(seed >> 32);
      q.ctr2 = (uint32_t)labels[li].label_ix;
      q.ctr3 = 0;                         // k_expand: the problem's new id
      q.n_tiles = (int32_t)n_tiles_p;
      q.tile_off = 0;                     // k_expand: r * n_tiles
      q.n_splits = 0;                     // tabulated: no above stage
      xtmpl[(size_t)li] = q;
      xfirst[(size_t)li] = (int32_t)r;
      for (int64_t j = 0; j < labels[li].n_ids; ++j) xctr[(size_t)r++] = (uint32_t)labels[li].ids[j];
    }
    xfirst[(size_t)n_labels] = (int32_t)r;
  }
  PACK_MARK("expand");
  const int64_t Ph = expand ? 0 : P;      // problems (and their tiles) the host writes
  tpe_problem* prob;
  if (direct) {
    prob = (tpe_problem*)(bb + off_lead[L_PROB]);
  } else {
    ps.prob.resize((size_t)Ph);
    prob = ps.prob.data();
  }
  if (!expand) {
    int64_t r = 0, s_next = 0, u_next = n_sorted_prob * (int64_t)n_cand;
    int32_t slot = 0;
    for (int32_t li = 0; li < n_labels; ++li) {
      const int32_t pool_slot = pooled[li] ? slot++ : -1, pool_first = (int32_t)r;
      for (int64_t j = 0; j < labels[li].n_ids; ++j, ++r) {
        tpe_problem& q = prob[r];
        q = lab[li];
        q.n_cand = n_cand;
        int64_t& next = pruned[li] ? s_next : u_next;
        q.cand_off = next;
        next += n_cand;
        q.sort_slot = pooled[li] ? pool_slot : pruned[li] ? slot++ : -1;
        q.pool_first = pooled[li] ? pool_first : -1;
        if (pooled[li]) q.flags |= TPE_F_POOLED;
        q.cand_base = cand_base;
        q.n_cand_global = C_ref;
        q.key0 = (uint32_t)seed; q.key1 = (uint32_t)(seed >> 32);
        q.ctr2 = (uint32_t)labels[li].label_ix;
        q.ctr3 = (uint32_t)labels[li].ids[j];
        q.n_tiles = (int32_t)n_tiles_p;
        q.tile_off = (int32_t)(r * n_tiles_p);
        if (q.family != TPE_FAM_CATEGORICAL && q.tab_mode == TPE_TAB_NONE) ++scored;
      }
    }
  }
  PACK_MARK("prob");
  // splits of the above mixture per tile.  Bulk tiles: enough work items to fill
  // the chip (a function of the GLOBAL candidate count).  Pruned problems with
  // many tiles: the bulk is cheap (local expansion), so one split, and the
  // outermost tiles of the (local) sorted range — the sparse tails, whose waves
  // span wide windows evaluated exactly — get geometrically more.  A shard sorts
  // and windows only its own candidates and counts its tails in its own tiles,
  // so under candidate sharding the fp32 sums (and near-tie winners) can differ
  // from a single-device run in the last bits: sharded winners agree within the
  // eps-tie set, not bit for bit (the draws themselves are identical).
  const int64_t tiles_ref = (C_ref + T - 1) / T;
  const int64_t scored_tiles = scored * tiles_ref;
  const int64_t target = std::max<int64_t>(1, (target_work() + std::max<int64_t>(scored_tiles, 1) - 1) /
                                                  std::max<int64_t>(scored_tiles, 1));
  bool any_pruned = false;
  for (int64_t r = 0; r < Ph; ++r) {
    tpe_problem& q = prob[r];
    if (q.family == TPE_FAM_CATEGORICAL || q.tab_mode != TPE_TAB_NONE) { q.n_splits = 0; continue; }
    const int64_t ks = (q.above_len + kMinComponentsPerSplit - 1) / kMinComponentsPerSplit;
    const bool tails = q.sort_slot >= 0 && tiles_ref >= kTailMinTiles;
    q.n_splits = tails ? 1 : (int32_t)std::max<int64_t>(1, std::min(target, ks));
    any_pruned = any_pruned || q.sort_slot >= 0;
  }
  auto tile_splits = [&](const tpe_problem& q, int64_t j) -> int32_t {
    if (q.family == TPE_FAM_CATEGORICAL || q.tab_mode != TPE_TAB_NONE) return 0;
    if (!(q.sort_slot >= 0 && tiles_ref >= kTailMinTiles)) return q.n_splits;
    const int64_t e = std::min<int64_t>(j, n_tiles_p - 1 - j);
    const int64_t ns = tail_splits(e);
    const int64_t cap = std::max<int64_t>(1, (q.above_len + 63) / 64);
    return (int32_t)std::max<int64_t>(1, std::min(ns, cap));
  };
  tpe_tile* tiles;
  if (direct) {
    tiles = (tpe_tile*)(bb + off_lead[L_TILES]);
  } else {
    ps.tiles.resize((size_t)(Ph * n_tiles_p));
    tiles = ps.tiles.data();
  }
  {
    tpe_tile* __restrict__ tp = tiles;
    for (int64_t r = 0; r < Ph; ++r) {
      tpe_tile* __restrict__ row = tp + r * n_tiles_p;
      const bool none = prob[r].family == TPE_FAM_CATEGORICAL || prob[r].tab_mode != TPE_TAB_NONE;
      for (int64_t j = 0; j < n_tiles_p; ++j) {
        row[j].problem = (int32_t)r;
        row[j].cand_start = (int32_t)(j * T);
        row[j].work_first = 0;
        row[j].n_splits = none ? 0 : tile_splits(prob[r], j);
      }
    }
  }
  // work items grouped [continuous | quantized Gauss | quantized log]; a tile's
  // items are consecutive, and an item's index is its row of `part`
  auto& work = ps.work;
  work.clear();
  {
    int64_t nw = 0;
    for (int64_t t = 0; t < Ph * n_tiles_p; ++t) nw += tiles[t].n_splits;
    work.reserve((size_t)nw);
  }
  int32_t counts[3] = {0, 0, 0};
  const int fams[3][2] = {{TPE_FAM_GAUSS, TPE_FAM_LOGGAUSS}, {TPE_FAM_QGAUSS, -1}, {TPE_FAM_QLOGGAUSS, -1}};
  for (int gi = 0; gi < 3; ++gi) {
    const size_t before = work.size();
    for (int64_t r = 0; r < Ph; ++r) {
      const tpe_problem& q = prob[r];
      if ((q.family != fams[gi][0] && q.family != fams[gi][1]) || q.tab_mode != TPE_TAB_NONE) continue;
      for (int64_t j = 0; j < n_tiles_p; ++j) {
        tpe_tile& tl = tiles[(size_t)(r * n_tiles_p + j)];
        tl.work_first = (int32_t)work.size();
        for (int32_t sp = 0; sp < tl.n_splits; ++sp) {
          tpe_work w;
          w.problem = (int32_t)r; w.split = sp; w.cand_start = (int32_t)(j * T);
          w.k_start = (int32_t)(((int64_t)q.above_len * sp) / tl.n_splits);
          w.k_end = (int32_t)(((int64_t)q.above_len * (sp + 1)) / tl.n_splits);
          w.n_splits = tl.n_splits;
          work.push_back(w);
        }
      }
    }
    counts[gi] = (int32_t)(work.size() - before);
  }
  if ((int64_t)work.size() >= ((int64_t)1 << 31)) return TPE_E_ARG;
  const int64_t part_total = (int64_t)work.size() * T;
  // tiles the finalize stage scores (device-drawn candidates): not categorical
  // (the sample stage scores those), not one-split continuous f32 (the above
  // stage does)
  auto& fin_tiles = ps.fin_tiles;
  fin_tiles.clear();
  for (int64_t r = 0; r < Ph; ++r) {                 // (per problem: a problem's tiles are consecutive)
    const tpe_problem& q = prob[r];
    if ((q.family == TPE_FAM_CATEGORICAL && q.samp_len <= TPE_SAMPLE_LDS_ROWS) || q.tab_mode != TPE_TAB_NONE) continue;
    const bool cont = !f64 && (q.family == TPE_FAM_GAUSS || q.family == TPE_FAM_LOGGAUSS);
    for (int64_t t = r * n_tiles_p; t < (r + 1) * n_tiles_p; ++t)
      if (!(cont && tiles[t].n_splits == 1)) fin_tiles.push_back((int32_t)t);
  }
  PACK_MARK("tiles_work_fin");
  // table jobs: per tabulated label, one per cell side or one lattice job
  // (TPE_TAB_PER_BLOCK rows per block); `problem` = the label's first row
  auto& tab_jobs = ps.tab_jobs;
  tab_jobs.clear();
  int64_t tab_blocks = 0, fgt_max_cells = 0;
  for (int32_t li = 0, r = 0; li < n_labels; r += (int32_t)labels[li].n_ids, ++li) {
    const tpe_problem& p = lab[li];
    if (p.tab_mode == TPE_TAB_NONE || labels[li].n_ids <= 0) continue;
    const int sides = p.tab_mode == TPE_TAB_CELLS ? 2 : 1;
    for (int sd = 0; sd < sides; ++sd) {
      tpe_tab_job j;
      memset(&j, 0, sizeof(j));
      j.problem = r; j.side = sd; j.kind = p.tab_mode; j.n = p.tab_n[sd]; j.off = p.tab_off[sd];
      j.block0 = (int32_t)tab_blocks;
      if (j.kind == TPE_TAB_CELLS) {
        if (p.flags & TPE_F_LOGPOLY) j.kind = TPE_TAB_LOGPOLY;
        // the rows the side's cells sum (a device-fitted above side: its fit writes them)
        j.rows_off = sd ? p.above_off : p.below_off;
        j.rows_n = sd && dev_fit[li] ? -1 : sd ? p.above_len : p.below_len;
        j.wide_off = sd ? p.wide_off : 0;
        j.wide_n = sd ? p.wide_len : 0;
        j.lo = p.tab_lo[sd];
        j.inv = p.tab_inv[sd];
      }
      // cells: TPE_TAB_PER_BLOCK rows per block; lattice: one block per value
      // (a box-moment label's above cells are built by their own stage: no blocks here)
      if (sd == 1 && (p.flags & TPE_F_FGT)) fgt_max_cells = std::max<int64_t>(fgt_max_cells, j.n);
      else if (j.kind == TPE_TAB_LOGPOLY && j.rows_n >= 0 && j.rows_n + j.wide_n <= kLpDirectRows)
        tab_blocks += (j.n + kLpRowsPerWave * TPE_TAB_PER_BLOCK - 1) / (kLpRowsPerWave * TPE_TAB_PER_BLOCK);
      else if (j.kind == TPE_TAB_CELLS && j.rows_n >= 0 && j.rows_n + j.wide_n <= kMomDirectRows)
        tab_blocks += (j.n + kMomCellsPerWave * TPE_TAB_PER_BLOCK - 1) / (kMomCellsPerWave * TPE_TAB_PER_BLOCK);
      else tab_blocks += j.kind != TPE_TAB_LATTICE ? (j.n + TPE_TAB_PER_BLOCK - 1) / TPE_TAB_PER_BLOCK : j.n;
      tab_jobs.push_back(j);
    }
  }
  if (tab_blocks >= ((int64_t)1 << 31)) return TPE_E_ARG;
  const int64_t n_tab_jobs = (int64_t)tab_jobs.size();
  // sample-stage tile lists: untabulated tiles (lazy categorical last) and tabulated tiles
  auto& samp_tiles = ps.samp_tiles;
  auto& tab_tiles = ps.tab_tiles;
  samp_tiles.clear(); tab_tiles.clear();
  auto append_range = [&](std::vector<int32_t>& v, int64_t r) {
    const size_t b = v.size();
    v.resize(b + (size_t)n_tiles_p);
    int32_t* __restrict__ d = v.data() + b;
    for (int64_t j = 0; j < n_tiles_p; ++j) d[j] = (int32_t)(r * n_tiles_p + j);
  };
  int64_t n_samp_eager = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int64_t r = 0; r < Ph; ++r) {
      const tpe_problem& q = prob[r];
      if (q.tab_mode != TPE_TAB_NONE) {
        if (pass == 0) append_range(tab_tiles, r);
        continue;
      }
      const bool lazy = q.family == TPE_FAM_CATEGORICAL && (q.flags & TPE_F_CAT_LAZY) && q.samp_len <= 64;
      if (lazy == (pass == 1)) append_range(samp_tiles, r);
      if (pass == 0 && !lazy) n_samp_eager += n_tiles_p;
    }
  // (expanded: every tile is tabulated, in order — the identity list, not stored)
  const int64_t n_samp_tiles = (int64_t)samp_tiles.size(),
                n_tab_tiles = expand ? P * n_tiles_p : (int64_t)tab_tiles.size();
  if (samp_tiles.empty()) samp_tiles.push_back(0);
  if (tab_tiles.empty()) tab_tiles.push_back(0);
  if (tab_jobs.empty()) tab_jobs.push_back(tpe_tab_job{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0.f, 0.f});
  const int64_t n_fin = (int64_t)fin_tiles.size();
  if (fin_tiles.empty()) fin_tiles.push_back(0);
  PACK_MARK("jobs_lists");
  // ---- the later sections after the leading ones (256-B aligned) ----
  const int NS = 6;
  // expanded levels: templates, first problems, new ids (one section, 256-B aligned parts)
  const int64_t x_tmpl = (int64_t)(xtmpl.size() * sizeof(tpe_problem));
  const int64_t x_first_off = (x_tmpl + 255) & ~(int64_t)255;
  const int64_t x_ctr_off = (x_first_off + (int64_t)(xfirst.size() * sizeof(int32_t)) + 255) & ~(int64_t)255;
  const int64_t x_len = expand ? x_ctr_off + (int64_t)(xctr.size() * sizeof(uint32_t)) : 0;
  const void* src[NS] = {work.data(), fin_tiles.data(), tab_jobs.data(), samp_tiles.data(), tab_tiles.data(), nullptr};
  const int64_t len[NS] = {(int64_t)(work.size() * sizeof(tpe_work)), (int64_t)(fin_tiles.size() * sizeof(int32_t)),
                           (int64_t)(tab_jobs.size() * sizeof(tpe_tab_job)),
                           (int64_t)(samp_tiles.size() * sizeof(int32_t)),
                           expand ? 0 : (int64_t)(tab_tiles.size() * sizeof(int32_t)), x_len};
  int64_t off[NS], end = lead_end;
  for (int i = 0; i < NS; ++i) {
    off[i] = (end + 255) & ~(int64_t)255;
    end = off[i] + len[i];
  }
  info->off_fit = off_lead[L_FIT]; info->off_below_idx = off_lead[L_BIDX]; info->off_fit_seg = off_lead[L_FSEG];
  info->off_grid = off_lead[L_GRID]; info->off_comp32 = off_lead[L_C32];
  info->off_patch = fit.empty() ? 0 : off_lead[L_PATCH];
  info->off_problems = off_lead[L_PROB]; info->off_tiles = off_lead[L_TILES];
  info->off_comp64 = off_lead[L_C64]; info->off_samp = off_lead[L_SAMP];
  info->off_work = off[0];
  info->off_fin_tiles = off[1]; info->n_fin_tiles = n_fin;
  info->fit_max_new = fit_max_new;
  info->fit_max_merge = fit_max_merge;
  info->fit_n_delta = fit_n_delta;
  info->fit_max_obs = fit_max_obs;
  info->off_tab_jobs = off[2]; info->n_tab_jobs = n_tab_jobs; info->tab_blocks = tab_blocks;
  info->tab_units = tab_units;
  info->off_samp_tiles = off[3]; info->n_samp_tiles = n_samp_tiles; info->n_samp_eager = n_samp_eager;
  info->off_tab_tiles = off[4]; info->n_tab_tiles = n_tab_tiles;
  info->off_expand = expand ? off[5] : 0;
  info->n_expand = expand ? n_labels : 0;
  // host-written ranges (the upload): fit sections + host grid, host comp32
  // rows, then problems (unless expanded: device-only) through the end
  info->n_up = 0;
  auto up = [&](int64_t o, int64_t n) {
    if (n > 0) { info->up_off[info->n_up] = o; info->up_len[info->n_up] = n; ++info->n_up; }
  };
  up(0, off_lead[L_GRID] + host_grid * 4);
  up(off_lead[L_C32], host_rows * 16);
  const int64_t r3 = expand ? off_lead[L_C64] : off_lead[L_PROB];
  up(r3, end - r3);
  info->n_problems = P;
  info->n_tiles = P * n_tiles_p;
  info->n_work_cont = counts[0]; info->n_work_qgauss = counts[1]; info->n_work_qlog = counts[2];
  info->any_pruned = any_pruned ? 1 : 0;
  info->key_bits = key_bits;
  info->sort_end_bit = any_pruned ? sort_end_bit : 0;
  info->part_total = part_total;
  info->n_fit = (int32_t)fit.size();
  info->fgt_max_boxes = (int32_t)fgt_max_boxes;
  info->fgt_max_cells = fgt_max_cells;
  info->fit_total = fit_seg.back();
  info->sort_count = n_sorted_prob * (int64_t)n_cand;
  info->n_sorted = S;
  info->n_pooled = n_pooled;
  info->draw_blocks = (C_ref + 1 + 63) / 64;
  info->blob_bytes = end;
  PACK_MARK("offsets");
  if (!direct || blob_cap < end) return TPE_E_SPACE;
  {
    // the later sections into the blob; a large level's in 64-KiB pieces on the
    // worker pool (a batched level's work items)
    struct Piece { unsigned char* dst; const unsigned char* src; size_t n; };
    static thread_local std::vector<Piece> pieces_tl;
    std::vector<Piece>& pieces = pieces_tl;
    pieces.clear();
    constexpr size_t kPiece = 64 << 10;
    size_t total = 0;
    for (int i = 0; i < NS; ++i) {
      if (!len[i] || !src[i]) continue;
      for (size_t o = 0; o < (size_t)len[i]; o += kPiece)
        pieces.push_back(Piece{bb + off[i] + o, (const unsigned char*)src[i] + o, std::min(kPiece, (size_t)len[i] - o)});
      total += (size_t)len[i];
    }
    auto copy = [](void* c, int k) {
      const Piece& q = (*(const std::vector<Piece>*)c)[(size_t)k];
      memcpy(q.dst, q.src, q.n);
    };
    if (total >= (128u << 10) && pieces.size() > 1) tpe_pool::parallel_for((int)pieces.size(), copy, &pieces);
    else for (size_t k = 0; k < pieces.size(); ++k) copy(&pieces, (int)k);
  }
  PACK_MARK("copy");
  if (expand) {
    unsigned char* x = bb + off[5];
    memcpy(x, xtmpl.data(), (size_t)x_tmpl);
    memcpy(x + x_first_off, xfirst.data(), xfirst.size() * sizeof(int32_t));
    memcpy(x + x_ctr_off, xctr.data(), xctr.size() * sizeof(uint32_t));
  }
  PACK_MARK("xcopy");
  PACK_DONE();
  return TPE_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- replay draws
// numpy legacy RandomState stream (include/tpe_hip.h "Exact-replay candidate
// draws"); compiled with -ffp-contract=off: loc + scale * g and the polar
// method's arithmetic round exactly as numpy's C does
namespace {

constexpr int kMtN = 624, kMtM = 397;

void mt_regen(tpe_mt_state* s) {
  uint32_t* k = s->key;
  auto mix = [](uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  };
  int i = 0;
  for (; i < kMtN - kMtM; ++i) k[i] = mix(k[i], k[i + 1], k[i + kMtM]);
  for (; i < kMtN - 1; ++i) k[i] = mix(k[i], k[i + 1], k[i + kMtM - kMtN]);
  k[kMtN - 1] = mix(k[kMtN - 1], k[0], k[kMtM - 1]);
  s->pos = 0;
}

inline uint32_t mt_next32(tpe_mt_state* s) {
  if (s->pos >= kMtN) mt_regen(s);
  uint32_t y = s->key[s->pos++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// random_sample: 53-bit double from two words
inline double mt_double(tpe_mt_state* s) {
  const int32_t a = (int32_t)(mt_next32(s) >> 5), b = (int32_t)(mt_next32(s) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

// legacy polar-method gauss with the cached second value
double mt_gauss(tpe_mt_state* s) {
  if (s->has_gauss) {
    const double t = s->gauss;
    s->has_gauss = 0;
    s->gauss = 0.0;
    return t;
  }
  double x1, x2, r2;
  do {
    x1 = 2.0 * mt_double(s) - 1.0;
    x2 = 2.0 * mt_double(s) - 1.0;
    r2 = x1 * x1 + x2 * x2;
  } while (r2 >= 1.0 || r2 == 0.0);
  const double f = sqrt(-2.0 * log(r2) / r2);
  s->gauss = f * x1;
  s->has_gauss = 1;
  return f * x2;
}

// multinomial(1, p) as numpy draws it: for j = 0 .. k-2 a binomial(1, p_j /
// remaining) (remaining -= p_j after each), stopping at the first success.
// numpy's binomial(1, p') is an inversion (p' <= 1/2; else 1 - inversion(1 -
// p')) with bound = min(1, np + 10 sqrt(np q + 1)) = 1: X = 0 when U <= qn, X
// = 1 when qn < U and U - qn <= px1, else a fresh U; qn = exp(1 log q) and px1
// = (1 p qn) / (1 q).  Those depend on p alone, so a Multinom1 computes them
// once per mixture and a draw only compares uniforms — the same values and
// the same uniform consumption as numpy's per-call arithmetic.
struct Multinom1 {
  struct Step { double qn, px1; int kind; };   // kind 0: never (p' == 0), 1: inversion, 2: 1 - inversion
  std::vector<Step> steps;
  int64_t k = 0;
  void init(const double* p, int64_t kk) {
    k = kk;
    steps.resize((size_t)std::max<int64_t>(k - 1, 0));
    double remaining = 1.0;
    for (int64_t j = 0; j < k - 1; ++j) {
      const double pj = p[j] / remaining;
      Step st{0.0, 0.0, 0};
      if (pj != 0.0) {
        const double pp = pj <= 0.5 ? pj : 1.0 - pj;
        const double q = 1.0 - pp;
        st.qn = exp(1.0 * log(q));
        st.px1 = ((double)1 * pp * st.qn) / ((double)1 * q);
        st.kind = pj <= 0.5 ? 1 : 2;
      }
      steps[(size_t)j] = st;
      remaining -= p[j];
    }
  }
  // binomial by inversion with n = 1 (see above)
  static int64_t inversion(tpe_mt_state* s, const Step& st) {
    for (;;) {
      double U = mt_double(s);
      if (!(U > st.qn)) return 0;
      U -= st.qn;
      if (!(U > st.px1)) return 1;
    }
  }
  int64_t draw(tpe_mt_state* s) const {
    for (int64_t j = 0; j < k - 1; ++j) {
      const Step& st = steps[(size_t)j];
      if (st.kind == 0) continue;
      const int64_t x = inversion(s, st);
      if ((st.kind == 1 ? x : 1 - x) > 0) return j;
    }
    return k - 1;
  }
};

// numpy's checks on pvals: every p in [0, 1] (no NaN) and a Kahan sum of all
// but the last <= 1 + 1e-12
bool pvals_ok(const double* p, int64_t k) {
  if (k < 1) return false;
  for (int64_t j = 0; j < k; ++j)
    if (!(p[j] >= 0.0 && p[j] <= 1.0)) return false;
  double sum = 0.0, c = 0.0;
  for (int64_t j = 0; j < k - 1; ++j) {
    const double y = p[j] - c;
    const double t = sum + y;
    c = (t - sum) - y;
    sum = t;
  }
  return !(sum > 1.0 + 1e-12);
}

}  // namespace

extern "C" {

int tpe_replay_mixture(tpe_mt_state* st, const double* w, const double* mu, const double* sigma, int64_t k,
                       int32_t bounded, double low, double high, int64_t n, double* out) {
  if (!st || k < 1 || n < 0 || (n && !out) || !w || !mu || !sigma || !pvals_ok(w, k)) return TPE_E_ARG;
  for (int64_t j = 0; j < k; ++j)
    if (!(sigma[j] >= 0.0)) return TPE_E_ARG;                // numpy: scale < 0 raises
  if (st->pos < 0 || st->pos > kMtN) return TPE_E_ARG;
  if (!bounded) {
    // rng.multinomial(1, w, (n,)) then rng.normal(mu[idx], sigma[idx])
    static thread_local std::vector<int64_t> idx_tl;
    std::vector<int64_t>& idx = idx_tl;
    idx.resize((size_t)n);
    Multinom1 m;
    m.init(w, k);
    for (int64_t i = 0; i < n; ++i) idx[(size_t)i] = m.draw(st);
    for (int64_t i = 0; i < n; ++i) {
      const int64_t c = idx[(size_t)i];
      out[i] = mu[c] + sigma[c] * mt_gauss(st);
    }
    return TPE_OK;
  }
  if (!(low < high)) return TPE_E_ARG;
  Multinom1 m;
  m.init(w, k);
  // (the reference rejects forever when [low, high) holds no mass; this stops
  // after 2^40 tries with TPE_E_ARG)
  for (int64_t i = 0, tries = 0; i < n; ++tries) {
    if (tries >= ((int64_t)1 << 40)) return TPE_E_ARG;
    const int64_t c = m.draw(st);
    const double d = mu[c] + sigma[c] * mt_gauss(st);
    if (low <= d && d < high) out[i++] = d;
  }
  return TPE_OK;
}

int tpe_replay_categorical(tpe_mt_state* st, const double* p, int64_t k, int64_t n, int64_t* out) {
  if (!st || n < 0 || (n && !out) || !p || !pvals_ok(p, k) || st->pos < 0 || st->pos > kMtN) return TPE_E_ARG;
  Multinom1 m;
  m.init(p, k);
  for (int64_t i = 0; i < n; ++i) out[i] = m.draw(st);
  return TPE_OK;
}

}  // extern "C"
