// tpe_suggest.cpp — one native call per tpe.suggest of a conditional tree space
// (include/tpe_hip.h, tpe_suggest_tree).
//
// The reference interprets a pyll posterior graph per suggest (tpe.py:804-897):
// for every hyperparameter it splits the history into below/above
// (ap_filter_trials, tpe.py:613-641), fits both Parzen estimators
// (adaptive_parzen_normal tpe.py:398-475, categorical posteriors tpe.py:573-607),
// and evaluates the conditional tree lazily (switch nodes, vectorize.py:19-37,
// pyll/base.py:762-781) so that only the active branch is sampled and scored.
// Here the host side of that is one C++ call: fits of the labels the tree
// needs (tpe_host_fit_split / tpe_host_cat_split), the gate prediction of the
// speculative level fusion, and the level runs (tpe_level_run) — the same
// decisions hyperopt_amd.tpe._choices_fused / _choices_philox make, without a
// Python round trip per label.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/tpe_hip.h"
#include "sort_net.h"
#include "tpe_pool.h"

extern "C" int tpe_internal_fail(int code, const char* what);   // tpe_kernels.hip (hidden)
extern "C" int tpe_internal_exchange(const tpe_exchange* ex, void* stream, int32_t my_status, tpe_result* res,
                                     int64_t P, int32_t* status);     // tpe_kernels.hip (hidden)
extern "C" int tpe_internal_level_run_ex(const tpe_label_in* labels, int32_t n_labels, int32_t n_cand, uint64_t seed,
                                         int64_t cand_base, int64_t n_cand_global, int32_t precision, int32_t flags,
                                         const tpe_level_ws* ws, tpe_level_need* need, void* stream, tpe_result* out,
                                         const tpe_exchange* ex, int64_t P_expected, int32_t* all_status,
                                         int32_t* done);              // tpe_kernels.hip (hidden)

namespace {

using tpe_sort_net::kSortNet;
using tpe_sort_net::sort_small;

// host phase clock (include/tpe_hip.h "Host phase clock")
std::atomic<int> g_ph_on{0};
double g_ph[TPE_N_PHASES];
std::chrono::steady_clock::time_point g_ph_t0;

void phase_start() {
  if (!g_ph_on.load(std::memory_order_relaxed)) return;
  g_ph_t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < TPE_N_PHASES; ++i) g_ph[i] = -1.0;
}

// TPE_TREE_TRACE=1 (with the phase clock on): named marks of tpe_suggest_tree's
// host steps on stderr, us since the call's entry (diagnostic)
void trace_mark(const char* what) {
  static const bool on = [] { const char* e = getenv("TPE_TREE_TRACE"); return e && e[0] == '1'; }();
  if (!on || !g_ph_on.load(std::memory_order_relaxed)) return;
  fprintf(stderr, "[tree] %-12s %8.1f us\n", what,
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g_ph_t0).count());
}

// TPE_DEVICE_COMBINE=0: sharded levels exchange through the host (A/B)
bool device_combine() {
  static const bool on = [] { const char* e = getenv("TPE_DEVICE_COMBINE"); return !(e && e[0] == '0'); }();
  return on;
}

constexpr int kInactive = -2;   // label not active (None)
constexpr int kIdBlock = 512;   // ids per block of a batched suggest's result assembly (worker pool)
constexpr int kActive = -1;     // active label that gates nothing (placeholder)
constexpr int32_t kRemoteRow = -2;   // fused batch: an active label another rank evaluates (TPE_F_REMOTE)

// fitted posterior of one label: continuous (w, mu, sigma) per side or the
// categorical probabilities (mu / sigma null)
struct Fit {
  bool done = false;
  bool dev = false;              // above side: the device Parzen fit (below_idx, the record's column)
  std::vector<double> buf;
  std::vector<double> side_x;      // the two sides' coordinates in tid order (caller-sorted fits)
  std::vector<int32_t> below_idx;
  int64_t k[2] = {0, 0};
  const double* w[2] = {nullptr, nullptr};
  const double* mu[2] = {nullptr, nullptr};
  const double* sg[2] = {nullptr, nullptr};
};

struct Tree {
  const tpe_tree_label* L;
  int32_t n;
  const int64_t* below;
  int64_t n_below;
  double prior_weight;
  int32_t lf;
  int64_t device_fit_min;
  std::vector<Fit>* fits;
  std::vector<char> gate;       // label gates another label
  int32_t max_depth;
  int8_t* need_fit;             // labels the caller must fit (TPE_E_FALLBACK)
};

// each below tid's position among a label's ascending tids (ap_filter_trials,
// tpe.py:629-636), in the below set's (ascending) order.  Tids one apart from
// first to last (every trial observed the label: a flat space's columns) are
// indexed directly instead of searched: 25 searches over a 10^5-tid column
// were most of a device-fitted label's host fit
inline void below_positions(const int64_t* tids, int64_t n, const int64_t* below, int64_t nb,
                            std::vector<int32_t>& out) {
  out.clear();
  if (n <= 0) return;
  const int64_t t0 = tids[0];
  const bool dense = tids[n - 1] - t0 == n - 1;           // (strictly ascending: tids[k] = t0 + k)
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t t = below[b];
    if (dense) {
      if (t >= t0 && t - t0 < n) out.push_back((int32_t)(t - t0));
      continue;
    }
    const int64_t* at = std::lower_bound(tids, tids + n, t);
    if (at != tids + n && *at == t) out.push_back((int32_t)(at - tids));
  }
}

// spec: a speculative fit on a pool worker (prefit): labels the caller must
// fit are left alone (no need_fit flag), and a failure only leaves the fit
// undone — the label's real fit, on the calling thread, reports it
int fit_label(Tree& T, int i, bool spec = false) {
  Fit& f = (*T.fits)[(size_t)i];
  if (f.done) return TPE_OK;
  const tpe_tree_label& L = T.L[i];
  const int64_t n = L.n_obs;
  if (L.host_k[0] > 0) {                      // the caller's fit
    if (L.host_k[1] <= 0 || !L.host_w[0] || !L.host_w[1] ||
        (L.family != TPE_FAM_CATEGORICAL && (!L.host_mu[0] || !L.host_mu[1] || !L.host_sigma[0] || !L.host_sigma[1])))
      return tpe_internal_fail(TPE_E_ARG, "tpe_suggest_tree: incomplete caller fit");
    for (int sd = 0; sd < 2; ++sd) {
      f.k[sd] = L.host_k[sd];
      f.w[sd] = L.host_w[sd];
      f.mu[sd] = L.family == TPE_FAM_CATEGORICAL ? nullptr : L.host_mu[sd];
      f.sg[sd] = L.family == TPE_FAM_CATEGORICAL ? nullptr : L.host_sigma[sd];
    }
    f.done = true;
    return TPE_OK;
  }
  if (L.family != TPE_FAM_CATEGORICAL && (L.side_order[0] || L.side_order[1])) {
    // the caller's per-side sort permutations (numpy's argsort: the reference's
    // tie order, tpe.py:427-428): split here (ap_filter_trials, tpe.py:629-636:
    // below = tid among the below tids, both sides kept in tid order) and fit
    // each side with its permutation (adaptive_parzen_normal, tpe.py:398-475)
    if (!L.side_order[0] || !L.side_order[1] || n < 0 || (n > 0 && (!L.tids || !L.values)))
      return tpe_internal_fail(TPE_E_ARG, "tpe_suggest_tree: a caller-sorted label needs both side orders and columns");
    const double* x = (const double*)L.values;
    f.side_x.resize((size_t)n);
    double* bx = f.side_x.data();
    below_positions(L.tids, n, T.below, T.n_below, f.below_idx);
    const int64_t nb = (int64_t)f.below_idx.size(), na = n - nb;
    if (nb != L.side_n[0] || na != L.side_n[1])
      return tpe_internal_fail(TPE_E_ARG, "tpe_suggest_tree: the caller's side sizes differ from the below split");
    double* ax = bx + nb;
    int64_t q = 0, t0 = 0;
    for (int64_t j = 0; j <= nb; ++j) {                     // above: the runs between the below positions
      const int64_t t1 = j < nb ? f.below_idx[(size_t)j] : n;
      for (int64_t t = t0; t < t1; ++t) ax[q++] = x[t];
      if (j < nb) { bx[j] = x[t1]; t0 = t1 + 1; }
    }
    const size_t cb = (size_t)nb + 1, ca = (size_t)na + 1;
    f.buf.resize(3 * (cb + ca));
    double* o = f.buf.data();
    const int64_t r0 = tpe_host_fit_parzen(bx, nb, nb >= 2 ? L.side_order[0] : nullptr, T.prior_weight, L.prior_mu,
                                           L.prior_sigma, T.lf, o, o + cb, o + 2 * cb);
    const int64_t r1 = tpe_host_fit_parzen(ax, na, na >= 2 ? L.side_order[1] : nullptr, T.prior_weight, L.prior_mu,
                                           L.prior_sigma, T.lf, o + 3 * cb, o + 3 * cb + ca, o + 3 * cb + 2 * ca);
    if (r0 < 0 || r1 < 0)
      return tpe_internal_fail(TPE_E_ARG, "tpe_host_fit_parzen failed on a caller-sorted side (a bad permutation or a "
                                          "non-positive Parzen bandwidth)");
    f.k[0] = nb + 1; f.w[0] = o; f.mu[0] = o + cb; f.sg[0] = o + 2 * cb;
    f.k[1] = na + 1; f.w[1] = o + 3 * cb; f.mu[1] = o + 3 * cb + ca; f.sg[1] = o + 3 * cb + 2 * ca;
    f.done = true;
    return TPE_OK;
  }
  auto host_fit = [&]() {                     // numpy's tie order decides this fit: the caller's
    if (T.need_fit && !spec) T.need_fit[i] = 1;
    return TPE_E_FALLBACK;
  };
  if (n < 0 || (n > 0 && (!L.tids || !L.values))) return tpe_internal_fail(TPE_E_ARG, "tpe_suggest_tree: bad columns");
  if (L.family == TPE_FAM_CATEGORICAL) {
    if (L.upper <= 0) return tpe_internal_fail(TPE_E_ARG, "tpe_suggest_tree: categorical label without categories");
    f.buf.resize(2 * (size_t)L.upper);
    const int rc = tpe_host_cat_split((const int64_t*)L.values, L.tids, n, T.below, T.n_below, L.upper, L.p_prior,
                                      T.prior_weight, T.lf, f.buf.data(), f.buf.data() + L.upper);
    if (rc != TPE_OK)
      return tpe_internal_fail(TPE_E_ARG, "categorical observation out of range or tids not ascending");
    f.k[0] = f.k[1] = L.upper;
    f.w[0] = f.buf.data();
    f.w[1] = f.buf.data() + L.upper;
    f.mu[0] = f.mu[1] = f.sg[0] = f.sg[1] = nullptr;
  } else if ((L.family == TPE_FAM_GAUSS || L.family == TPE_FAM_LOGGAUSS) && L.dev_obs &&
             T.device_fit_min > 0 && n >= std::max<int64_t>(T.device_fit_min, 64)) {
    // device Parzen fit of the above side; the below side (ap_filter_trials,
    // tpe.py:629-636: the observations whose tid is below) fitted here.  It has
    // at most 25 observations, all of weight 1 (no linear-forgetting ramp below
    // 26, tpe.py:381-394), so any sort of it gives numpy's fit: tied values are
    // interchangeable
    const double* x = (const double*)L.values;
    below_positions(L.tids, n, T.below, T.n_below, f.below_idx);
    const int64_t nb = (int64_t)f.below_idx.size();
    if (nb > 64 || n - nb + 1 <= 64) return TPE_E_FALLBACK;
    double bx[64];
    int64_t ord[64];
    for (int64_t q = 0; q < nb; ++q) bx[q] = x[f.below_idx[(size_t)q]];
    if (nb <= kSortNet && (T.lf <= 0 || nb <= T.lf)) {     // (no linear-forgetting ramp: ties interchangeable)
      sort_small(bx, nb, ord);
    } else {                                                // (else: stable insertion sort, NaN last)
      for (int64_t q = 0; q < nb; ++q) ord[q] = q;
      for (int64_t q = 1; q < nb; ++q)
        for (int64_t r = q; r > 0; --r) {
          const double a = bx[ord[r - 1]], c = bx[ord[r]];
          if (!(a > c || (a != a && c == c))) break;
          std::swap(ord[r - 1], ord[r]);
        }
    }
    const size_t cap = (size_t)nb + 1;
    f.buf.resize(3 * cap);
    const int64_t rc = tpe_host_fit_parzen(bx, nb, nb >= 2 ? ord : nullptr, T.prior_weight, L.prior_mu,
                                           L.prior_sigma, T.lf, f.buf.data(), f.buf.data() + cap,
                                           f.buf.data() + 2 * cap);
    if (rc < 0) return tpe_internal_fail(TPE_E_ARG, "tpe_host_fit_parzen failed on a below side");
    f.k[0] = nb + 1;
    f.w[0] = f.buf.data(); f.mu[0] = f.buf.data() + cap; f.sg[0] = f.buf.data() + 2 * cap;
    f.k[1] = n - nb + 1;
    f.w[1] = f.mu[1] = f.sg[1] = nullptr;
    f.dev = true;
  } else if (L.family == TPE_FAM_GAUSS || L.family == TPE_FAM_LOGGAUSS) {
    if (n > 0 && !L.order) return host_fit();                                  // a NaN value
    if (T.device_fit_min > 0 && n >= std::max<int64_t>(T.device_fit_min, 64)) return TPE_E_FALLBACK;
    const size_t cap = (size_t)n + 1;
    f.buf.resize(6 * cap);
    const int rc = tpe_host_fit_split((const double*)L.values, L.tids, L.order, n, T.below, T.n_below, T.prior_weight,
                                      L.prior_mu, L.prior_sigma, T.lf, f.buf.data(), f.k);
    if (rc != TPE_OK)
      return tpe_internal_fail(TPE_E_ARG, "tpe_host_fit_split failed: tids not strictly ascending, a bad order, or a "
                                          "non-positive Parzen bandwidth");
    if (f.k[0] == 0 || f.k[1] == 0) return host_fit();                         // repeated values: numpy's tie order
    for (int sd = 0; sd < 2; ++sd) {
      double* b = f.buf.data() + 3 * (size_t)sd * cap;
      f.w[sd] = b;
      f.mu[sd] = b + cap;
      f.sg[sd] = b + 2 * cap;
    }
  } else {
    return host_fit();                                                         // quantized: numpy's tie order
  }
  f.done = true;
  return TPE_OK;
}

// Labels worth a speculative fit on the pool: the natively fitted ones with
// enough observations for the fit to cost more than a dispatch (categorical,
// continuous with a value order, and the device-fitted ones' host part: the
// below positions among the label's tids and the below side's fit).  Every label of a
// flat space is needed; in a tree the inactive branches' labels are fitted too
// (their observations are the trials that took that branch, so the extra work
// is bounded by the history) — what matters is that the suggest waits for the
// slowest label, not for the sum over the labels the active branch needs.
constexpr int64_t kPrefitMinObs = 256;

bool prefit_worthy(const Tree& T, int i) {
  const tpe_tree_label& L = T.L[i];
  if ((L.flags & TPE_F_REMOTE) || L.host_k[0] > 0 || L.n_obs < kPrefitMinObs || !L.tids || !L.values) return false;
  if (L.family == TPE_FAM_CATEGORICAL) return L.upper > 0;
  if (L.side_order[0] && L.side_order[1]) return true;        // caller-sorted (quantized, repeated values)
  if (L.family != TPE_FAM_GAUSS && L.family != TPE_FAM_LOGGAUSS) return false;
  const bool dev = T.device_fit_min > 0 && L.n_obs >= std::max<int64_t>(T.device_fit_min, 64);
  if (dev) return L.dev_obs != nullptr;         // the below side's fit and its positions among the tids
  return L.order != nullptr;
}

struct PrefitCtx {
  Tree* T;
  const int* ix;
  int n, per;                      // labels; labels a task
};

// a device-fitted label's below values touched before its fit: a task's
// labels issue every such load up front, so their cache and TLB misses (one
// label column of 10^5 values each: ~1 us a label one at a time) overlap
void prefetch_below(const Tree& T, int i) {
  const tpe_tree_label& L = T.L[i];
  if (!L.dev_obs || !L.tids || !L.values || L.n_obs <= 0 || L.family == TPE_FAM_CATEGORICAL) return;
  const int64_t t0 = L.tids[0], n = L.n_obs;
  if (L.tids[n - 1] - t0 != n - 1) return;          // (dense tids only: a position is tid - t0)
  const double* x = (const double*)L.values;
  for (int64_t b = 0; b < T.n_below; ++b) {
    const int64_t t = T.below[b] - t0;
    if (t >= 0 && t < n) __builtin_prefetch(x + t);
  }
}

void prefit_one(void* c, int k) {
  PrefitCtx* p = (PrefitCtx*)c;
  const int j0 = k * p->per, j1 = std::min(p->n, j0 + p->per);
  if (j1 - j0 > 1)
    for (int j = j0; j < j1; ++j) prefetch_below(*p->T, p->ix[j]);
  for (int j = j0; j < j1; ++j) fit_label(*p->T, p->ix[j], true);
}

void prefit(Tree& T) {
  static thread_local std::vector<int> ix_tl;
  std::vector<int>& ix = ix_tl;
  ix.clear();
  bool hinted = false;                  // the caller's hint (TPE_F_PREFIT), else every worthy label
  for (int i = 0; i < T.n && !hinted; ++i) hinted = (T.L[i].flags & TPE_F_PREFIT) != 0;
  for (int i = 0; i < T.n; ++i)
    if ((!hinted || (T.L[i].flags & TPE_F_PREFIT)) && prefit_worthy(T, i)) ix.push_back(i);
  if (ix.size() < 2 || tpe_pool::workers() == 0) return;   // (on demand, on this thread)
  // largest first: the slowest fits start first
  std::sort(ix.begin(), ix.end(), [&](int a, int b) { return T.L[a].n_obs > T.L[b].n_obs; });
  // (a thousand labels: eight a task, their loads issued together; a few: one a task)
  const int n = (int)ix.size(), per = n >= 256 ? 8 : 1;
  PrefitCtx c{&T, ix.data(), n, per};
  tpe_pool::parallel_for((n + per - 1) / per, prefit_one, &c);
}

// ParamTable.active: some parent chose this label's option (`chosen`: the
// per-label codes of one id — a category, kActive or kInactive)
bool is_active(const tpe_tree_label& L, const int* chosen) {
  if (L.n_parents == 0) return true;
  for (int j = 0; j < L.n_parents; ++j) {
    const int c = chosen[L.parent[j]];
    if (c >= 0 && c == L.parent_cat[j]) return true;
  }
  return false;
}

// hyperopt_amd.tpe._predict_activity: per label kInactive / kActive / the
// predicted category of a gate; false when some gate cannot be predicted.  A
// gate's candidates all score log pb[c] - log pa[c] (categorical_lpdf,
// tpe.py:50-57), so its argmax (broadcast_best, tpe.py:749-759) is the best
// drawable category unless it goes undrawn among the C draws.
int predict(Tree& T, int64_t n_cand, double min_draws, std::vector<int>& pred, bool& ok) {
  ok = false;
  pred.assign((size_t)T.n, kInactive);
  for (int d = 0; d <= T.max_depth; ++d) {
    for (int i = 0; i < T.n; ++i) {
      const tpe_tree_label& L = T.L[i];
      if (L.depth != d) continue;
      if (!is_active(L, pred.data())) { pred[(size_t)i] = kInactive; continue; }
      if (!T.gate[(size_t)i]) { pred[(size_t)i] = kActive; continue; }
      if (L.family != TPE_FAM_CATEGORICAL) return TPE_OK;
      const int rc = fit_label(T, i);
      if (rc != TPE_OK) return rc;
      const Fit& f = (*T.fits)[(size_t)i];
      const double* pb = f.w[0];
      const double* pa = f.w[1];
      double tot = 0.0;
      for (int k = 0; k < L.upper; ++k) tot += pb[k];
      if (!(tot > 0)) return TPE_OK;
      int c = -1;
      double best = 0.0;
      for (int k = 0; k < L.upper; ++k) {
        if (!(pb[k] > 0)) continue;
        const double sc = pa[k] > 0 ? std::log(pb[k]) - std::log(pa[k]) : INFINITY;
        // np.argmax: the first maximum, a NaN beats everything
        if (c < 0 || sc > best || (sc != sc && best == best)) { c = k; best = sc; }
      }
      if (c < 0 || (double)n_cand * pb[c] / tot < min_draws) return TPE_OK;
      pred[(size_t)i] = c;
    }
  }
  ok = true;
  return TPE_OK;
}

// one level's label record (tpe_label_in) from a fit
void label_rec(const Tree& T, const tpe_tree_label& L, const Fit& f, const int64_t* ids, int64_t n_ids,
               tpe_label_in& r) {
  memset(&r, 0, sizeof(r));
  r.family = L.family;
  r.flags = L.flags & (TPE_F_HAS_LOW | TPE_F_HAS_HIGH);
  r.upper = L.upper;
  r.label_ix = L.label_ix;
  r.low = L.low;
  r.high = L.high;
  r.q = L.q;
  r.below_w = f.w[0]; r.below_mu = f.mu[0]; r.below_sigma = f.sg[0]; r.below_k = f.k[0];
  r.above_w = f.w[1]; r.above_mu = f.mu[1]; r.above_sigma = f.sg[1]; r.above_k = f.k[1];
  r.ids = ids;
  r.n_ids = n_ids;
  if (f.dev) {                                  // the device fit of the above side (tpe_fit_above)
    r.dev_obs = L.dev_obs;
    r.n_obs = L.n_obs;
    r.below_idx = f.below_idx.data();
    r.n_below = (int32_t)f.below_idx.size();
    r.lf = T.lf;
    r.prior_mu = L.prior_mu; r.prior_sigma = L.prior_sigma; r.prior_weight = T.prior_weight;
    r.ord_key_in = L.ord_key_in; r.ord_idx_in = L.ord_idx_in; r.n_ord_in = L.n_ord_in;
    r.ord_key_out = L.ord_key_out; r.ord_idx_out = L.ord_idx_out;
  }
}

}  // namespace

extern "C" {

// phase mark for tpe_level_run (tpe_kernels.hip)
__attribute__((visibility("hidden"))) void tpe_internal_phase(int i) {
  if (!g_ph_on.load(std::memory_order_relaxed) || i < 0 || i >= TPE_N_PHASES) return;
  g_ph[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g_ph_t0).count();
}

int tpe_host_phases(int32_t enable, double* last, int32_t n) {
  if (last && n > 0) memcpy(last, g_ph, sizeof(double) * (size_t)std::min<int32_t>(n, TPE_N_PHASES));
  if (enable && !g_ph_on.load()) for (int i = 0; i < TPE_N_PHASES; ++i) g_ph[i] = -1.0;
  g_ph_on.store(enable ? 1 : 0);
  return TPE_OK;
}

static int suggest_tree(const tpe_tree_label* labels, int32_t n_labels, const int64_t* below_tids, int64_t n_below,
                        double prior_weight, int32_t lf, const int64_t* ids, int32_t n_ids, int32_t n_cand,
                        int64_t cand_base, int64_t n_cand_global, const tpe_exchange* ex,
                        uint64_t seed, double speculate_min_draws, int64_t device_fit_min, int32_t flags,
                        const tpe_level_ws* ws, tpe_level_need* need, void* stream, double* values, int8_t* active,
                        int32_t* path, int8_t* need_fit) {
  if (n_labels < 0 || n_ids < 0 || n_cand < 0 || n_below < 0 || (n_labels > 0 && !labels) || (n_ids > 0 && !ids) ||
      (n_below > 0 && !below_tids) || !ws || !need || !path || (n_labels > 0 && n_ids > 0 && (!values || !active)) ||
      cand_base < 0 || n_cand_global < 0 || (n_cand_global > 0 && cand_base + n_cand > n_cand_global) ||
      (ex && (ex->world < 1 || ex->rank < 0 || ex->rank >= ex->world)))
    return tpe_internal_fail(TPE_E_ARG, "tpe_suggest_tree: bad arguments");
  // the candidates of the whole suggest (all shards): what the gate prediction counts
  const int64_t c_all = n_cand_global > 0 ? n_cand_global : n_cand;
  const bool exchange = ex && (ex->world > 1 || ex->always);
  path[0] = path[1] = 0;
  if (need_fit) memset(need_fit, 0, (size_t)std::max(n_labels, 0));
  static thread_local std::vector<Fit> fits_tl;
  static thread_local std::vector<tpe_label_in> recs_tl;
  static thread_local std::vector<tpe_result> res_tl;
  static thread_local std::vector<int64_t> ids_tl;
  static thread_local std::vector<int> chosen_tl, pred_tl;
  std::vector<Fit>& fits = fits_tl;
  if (fits.size() < (size_t)n_labels) fits.resize((size_t)n_labels);
  for (int i = 0; i < n_labels; ++i) fits[(size_t)i].done = false;
  Tree T{labels, n_labels, below_tids, n_below, prior_weight, lf, device_fit_min, &fits, {}, 0, need_fit};
  T.gate.assign((size_t)n_labels, 0);
  for (int i = 0; i < n_labels; ++i) {
    const tpe_tree_label& L = labels[i];
    if (L.n_parents < 0 || L.n_parents > TPE_TREE_MAX_PARENTS || L.depth < 0 || L.label_ix != i)
      return tpe_internal_fail(TPE_E_ARG, "tpe_suggest_tree: bad label record");
    for (int j = 0; j < L.n_parents; ++j) {
      if (L.parent[j] < 0 || L.parent[j] >= n_labels || labels[L.parent[j]].depth >= L.depth)
        return tpe_internal_fail(TPE_E_ARG, "tpe_suggest_tree: a parent must be a label of a lower level");
      T.gate[(size_t)L.parent[j]] = 1;
    }
    T.max_depth = std::max(T.max_depth, L.depth);
  }
  for (int i = 0; i < n_labels; ++i)
    if ((labels[i].flags & TPE_F_REMOTE) && T.gate[(size_t)i])
      return tpe_internal_fail(TPE_E_ARG, "tpe_suggest_tree: a gate cannot be remote (every rank evaluates the gates)");
  // spaces for the general path, refused before any fit or run: non-categorical
  // gates, and continuous labels large enough for the device Parzen fit (labels
  // another rank evaluates are never fitted here)
  for (int i = 0; i < n_labels; ++i) {
    const tpe_tree_label& L = labels[i];
    if (T.gate[(size_t)i] && L.family != TPE_FAM_CATEGORICAL) return TPE_E_FALLBACK;
    if (L.flags & TPE_F_REMOTE) continue;
    if ((L.family == TPE_FAM_GAUSS || L.family == TPE_FAM_LOGGAUSS) && L.host_k[0] <= 0 && !L.dev_obs &&
        device_fit_min > 0 && L.n_obs >= std::max<int64_t>(device_fit_min, 64))
      return TPE_E_FALLBACK;
  }
  if (n_labels == 0 || n_ids == 0) return TPE_OK;
  trace_mark("checks");
  prefit(T);
  tpe_internal_phase(TPE_PHASE_PREFIT);
  const int32_t run_flags = flags & ~TPE_TREE_NO_SPECULATE;
  std::vector<tpe_label_in>& recs = recs_tl;
  std::vector<tpe_result>& res = res_tl;
  auto run = [&](int32_t n_recs) -> int {
    tpe_internal_phase(TPE_PHASE_RECS);
    int64_t P = 0;
    for (int32_t r = 0; r < n_recs; ++r) P += recs[(size_t)r].n_ids;
    res.resize((size_t)std::max<int64_t>(P, 1));
    ++path[1];
    if (exchange && ex->comm && device_combine()) {
      // RCCL: the level's runs reduced, gathered and combined on the device, one
      // stream synchronise (falls back to the host exchange below when the level
      // cannot take that path: then nothing was launched or exchanged)
      int32_t all_rc = TPE_OK, done = 0;
      const int rc = tpe_internal_level_run_ex(recs.data(), n_recs, n_cand, seed, cand_base, n_cand_global, TPE_PREC_F32,
                                               run_flags, ws, need, stream, res.data(), ex, P, &all_rc, &done);
      if (done) {
        if (rc != TPE_OK) return rc;
        if (all_rc == TPE_E_SPACE) return tpe_internal_fail(TPE_E_SPACE, "another rank needs a larger workspace");
        if (all_rc != TPE_OK) return tpe_internal_fail(all_rc, "a level run failed on another rank");
        return TPE_OK;
      }
      if (rc != TPE_OK)
        for (int64_t q = 0; q < P; ++q) res[(size_t)q] = tpe_result{0, 0, 0, 0, -1, -1};
      int32_t all2 = TPE_OK;
      const int xrc = tpe_internal_exchange(ex, stream, rc, res.data(), P, &all2);
      if (xrc != TPE_OK) return xrc;
      if (rc != TPE_OK) return rc;
      if (all2 == TPE_E_SPACE) return tpe_internal_fail(TPE_E_SPACE, "another rank needs a larger workspace");
      if (all2 != TPE_OK) return tpe_internal_fail(all2, "a level run failed on another rank");
      return TPE_OK;
    }
    int rc = tpe_level_run(recs.data(), n_recs, n_cand, seed, cand_base, n_cand_global, TPE_PREC_F32, run_flags, ws,
                           need, stream, res.data());
    if (!exchange) return rc;
    // every rank takes part in the exchange, whatever its own status
    if (rc != TPE_OK)
      for (int64_t q = 0; q < P; ++q) res[(size_t)q] = tpe_result{0, 0, 0, 0, -1, -1};
    int32_t all_rc = TPE_OK;
    const int xrc = tpe_internal_exchange(ex, stream, rc, res.data(), P, &all_rc);
    if (xrc != TPE_OK) return xrc;
    if (rc != TPE_OK) return rc;
    if (all_rc == TPE_E_SPACE) return tpe_internal_fail(TPE_E_SPACE, "another rank needs a larger workspace");
    if (all_rc != TPE_OK) return tpe_internal_fail(all_rc, "a level run failed on another rank");
    return TPE_OK;
  };

  // speculative fusion (hyperopt_amd.tpe._choices_fused): every level in one
  // batch under the predicted activity, verified on the gates' results
  if (!(flags & TPE_TREE_NO_SPECULATE) && speculate_min_draws >= 0 && T.max_depth > 0) {
    bool ok = false;
    std::vector<int>& pred = pred_tl;
    int rc = predict(T, c_all, speculate_min_draws, pred, ok);
    if (rc != TPE_OK) return rc;
    if (ok) {
      recs.resize((size_t)n_labels);
      int32_t nr = 0;
      bool pending = false;                 // labels flagged for the caller's fit: all of them at once
      for (int i = 0; i < n_labels; ++i) {
        if (pred[(size_t)i] == kInactive || (labels[i].flags & TPE_F_REMOTE)) continue;
        if ((rc = fit_label(T, i)) != TPE_OK) {
          if (rc == TPE_E_FALLBACK && need_fit && need_fit[i]) { pending = true; continue; }
          return rc;
        }
        label_rec(T, labels[i], fits[(size_t)i], ids, n_ids, recs[(size_t)nr++]);
      }
      if (pending) return TPE_E_FALLBACK;
      if ((rc = run(nr)) != TPE_OK) return rc;
      // the prediction checked and the values written in one pass: ids in
      // blocks (each block's rows of values/active are its own: no cache lines
      // shared between workers; its result reads are runs of consecutive ids
      // per label), a batched suggest's blocks in parallel on the worker pool.
      // A failed check leaves the level-by-level path below, which rewrites
      // every value.  rows[i]: label i's result row (-1: predicted inactive,
      // kRemoteRow: active, evaluated by another rank).
      std::vector<int32_t> rows((size_t)n_labels);
      int32_t r = 0;
      for (int i = 0; i < n_labels; ++i)
        rows[(size_t)i] = pred[(size_t)i] == kInactive ? -1 : (labels[i].flags & TPE_F_REMOTE) ? kRemoteRow : r++;
      const int nb = (n_ids + kIdBlock - 1) / kIdBlock;
      std::vector<int8_t> flag((size_t)std::max(nb, 1), 0);     // per block: 1 misprediction, 2 no candidate
      struct Col {
        const tpe_result* res; const int32_t* rows; const int* pred; double* values; int8_t* active; int8_t* flag;
        int n_ids, n_labels;
      };
      Col cx{res.data(), rows.data(), pred.data(), values, active, flag.data(), n_ids, n_labels};
      auto blk = [](void* c, int k) {
        const Col& q = *(const Col*)c;
        const int j0 = k * kIdBlock, j1 = std::min(q.n_ids, j0 + kIdBlock);
        int8_t f = 0;
        for (int i = 0; i < q.n_labels; ++i) {
          const int32_t rr = q.rows[i];
          const int pd = q.pred[i];
          for (int j = j0; j < j1; ++j) {
            double v = NAN;
            if (rr >= 0) {
              const tpe_result& x = q.res[(size_t)rr * q.n_ids + j];
              if (x.idx < 0) f |= 2;
              if (pd >= 0 && (int64_t)x.value != pd) f |= 1;
              v = x.value;
            }
            q.values[(size_t)j * q.n_labels + i] = v;
            q.active[(size_t)j * q.n_labels + i] = rr >= 0 || rr == kRemoteRow ? 1 : 0;
          }
        }
        q.flag[k] = f;
      };
      if (nb > 1) tpe_pool::parallel_for(nb, blk, &cx);
      else blk(&cx, 0);
      int8_t f = 0;
      for (int k = 0; k < nb; ++k) f |= flag[(size_t)k];
      if (f & 2) return tpe_internal_fail(TPE_E_ARG, "no candidate selected for a label");
      if (!(f & 1)) {
        path[0] = 1;
        return TPE_OK;
      }
    }
  }

  // level by level (hyperopt_amd.tpe._choices_philox)
  trace_mark("level-path");
  std::vector<int>& chosen = chosen_tl;
  chosen.resize((size_t)n_ids * n_labels);
  // every (id, label) inactive, in id blocks on the pool (a batched suggest's
  // rows: 4096 x 20 on config 4)
  struct Init { double* values; int8_t* active; int* chosen; int n_ids, n_labels; };
  Init ini{values, active, chosen.data(), n_ids, n_labels};
  auto init_blk = [](void* c, int k) {
    const Init& q = *(const Init*)c;
    const size_t a = (size_t)k * kIdBlock * q.n_labels,
                 e = (size_t)std::min(q.n_ids, (k + 1) * kIdBlock) * q.n_labels;
    for (size_t t = a; t < e; ++t) { q.values[t] = NAN; q.active[t] = 0; q.chosen[t] = kInactive; }
  };
  const int n_blk = (n_ids + kIdBlock - 1) / kIdBlock;
  // a flat space (one level, every label parentless, no gate): every entry is
  // written below — a local label's by the results pass, a remote one's by the
  // remote pass — and no `chosen` code is ever read: nothing to initialise
  const bool flat = T.max_depth == 0;
  if (!flat) {
    if (n_blk > 1) tpe_pool::parallel_for(n_blk, init_blk, &ini);
    else if (n_blk == 1) init_blk(&ini, 0);
  }
  trace_mark("init");
  std::vector<int64_t>& lvl_ids = ids_tl;
  // a member of a level: its label, its problems' first row in the level's
  // results, their count, and where its id positions start in lvl_ids (-1: every
  // id — a label without parents — whose positions are 0 .. n_ids - 1 and whose
  // records take the caller's id array as it is)
  struct Member { int label; int64_t res_off, count, lvl_first; };
  for (int d = 0; d <= T.max_depth; ++d) {
    recs.clear();
    lvl_ids.clear();
    std::vector<Member> members;
    int64_t n_res = 0;
    bool pending = false;                   // labels flagged for the caller's fit: all of the level's at once
    // the level's labels another rank evaluates: active where the tree says, in
    // one row-major pass over the ids below (a remote label is never a gate, so
    // its `chosen` code is never read; a label a time over 4096 ids strided the
    // rows: 28 us a label on config 4)
    std::vector<int> remote;
    for (int i = 0; i < n_labels; ++i)
      if (labels[i].depth == d && (labels[i].flags & TPE_F_REMOTE)) remote.push_back(i);
    // (a flat space with local members: the remote entries are written by the
    // results pass below, row by row with the members' — one pass over the rows)
    bool any_member = false;
    for (int i = 0; i < n_labels && !any_member; ++i)
      any_member = labels[i].depth == d && !(labels[i].flags & TPE_F_REMOTE);
    const bool rem_in_put = flat && any_member && !remote.empty();
    if (!remote.empty() && !rem_in_put) {
      struct Rem { const tpe_tree_label* labels; const int* remote; int nr; int8_t* active; double* values;
                   const int* chosen; int n_ids, n_labels; bool flat; };
      Rem rm{labels, remote.data(), (int)remote.size(), active, values, chosen.data(), n_ids, n_labels, flat};
      auto rem_blk = [](void* c, int k) {
        const Rem& q = *(const Rem*)c;
        const int j1 = std::min(q.n_ids, (k + 1) * kIdBlock);
        for (int j = k * kIdBlock; j < j1; ++j) {
          int8_t* row = q.active + (size_t)j * q.n_labels;
          double* vrow = q.values + (size_t)j * q.n_labels;
          if (q.flat) {                              // (every remote label active, its value another rank's)
            for (int r = 0; r < q.nr; ++r) { row[q.remote[r]] = 1; vrow[q.remote[r]] = NAN; }
            continue;
          }
          const int* ch = q.chosen + (size_t)j * q.n_labels;
          for (int r = 0; r < q.nr; ++r) {
            const tpe_tree_label& L = q.labels[q.remote[r]];
            if (L.n_parents == 0 || is_active(L, ch)) row[q.remote[r]] = 1;
          }
        }
      };
      if (n_blk > 1) tpe_pool::parallel_for(n_blk, rem_blk, &rm);
      else rem_blk(&rm, 0);
      trace_mark("remote");
    }
    for (int i = 0; i < n_labels; ++i) {
      const tpe_tree_label& L = labels[i];
      if (L.depth != d || (L.flags & TPE_F_REMOTE)) continue;
      Member m{i, n_res, n_ids, -1};
      if (L.n_parents > 0) {
        m.lvl_first = (int64_t)lvl_ids.size();
        for (int j = 0; j < n_ids; ++j)
          if (is_active(L, chosen.data() + (size_t)j * n_labels)) lvl_ids.push_back(j);
        m.count = (int64_t)lvl_ids.size() - m.lvl_first;
        if (m.count == 0) continue;
      }
      const int rc = fit_label(T, i);
      if (rc != TPE_OK) {
        if (rc == TPE_E_FALLBACK && need_fit && need_fit[i]) { pending = true; continue; }
        return rc;
      }
      members.push_back(m);
      n_res += m.count;
    }
    if (pending) return TPE_E_FALLBACK;
    trace_mark("members");
    if (members.empty()) {
      // (a flat space whose local labels all needed nothing: the remote entries still)
      if (rem_in_put)
        for (int j = 0; j < n_ids; ++j)
          for (int r : remote) { active[(size_t)j * n_labels + r] = 1; values[(size_t)j * n_labels + r] = NAN; }
      continue;
    }
    // the gated members' id arrays (positions -> new ids), stable now that lvl_ids is complete
    std::vector<int64_t> lvl_new((size_t)lvl_ids.size());
    for (size_t q = 0; q < lvl_ids.size(); ++q) lvl_new[q] = ids[lvl_ids[q]];
    recs.resize(members.size());
    for (size_t k = 0; k < members.size(); ++k) {
      const Member& m = members[k];
      label_rec(T, labels[m.label], fits[(size_t)m.label], m.lvl_first < 0 ? ids : lvl_new.data() + m.lvl_first,
                m.count, recs[k]);
    }
    const int rc = run((int32_t)members.size());
    if (rc != TPE_OK) return rc;
    // the members' results into their columns, ids in blocks (a block's rows
    // are its own: no cache lines shared between workers); a gated member's
    // positions hold its ids ascending, so a block's are one range, found by
    // bisection.  A problem without a selected candidate flags its block (the
    // check rides along with the one pass over the results)
    struct Mem {
      const Member* members; int n_mem; const int64_t* lvl_ids;
      const tpe_result* res; double* values; int8_t* active; int* chosen; const char* gate; int n_ids, n_labels;
      int8_t* bad;
      const int* rem; int n_rem;     // (flat space: the remote labels, active with another rank's value)
    };
    const int nbk = (n_ids + kIdBlock - 1) / kIdBlock;
    std::vector<int8_t> bad((size_t)std::max(nbk, 1), 0);
    Mem mx{members.data(), (int)members.size(), lvl_ids.data(), res.data(), values, active, chosen.data(),
           T.gate.data(), n_ids, n_labels, bad.data(), remote.data(), rem_in_put ? (int)remote.size() : 0};
    auto put = [](void* c, int k) {
      const Mem& x = *(const Mem*)c;
      const int64_t j0 = (int64_t)k * kIdBlock, j1 = std::min<int64_t>(x.n_ids, j0 + kIdBlock);
      int8_t b = 0;
      for (int mi = 0; mi < x.n_mem; ++mi) {
        const Member& m = x.members[mi];
        const int i = m.label;
        auto set = [&](int64_t q, int64_t j) {
          const tpe_result& r = x.res[(size_t)q];
          const double v = r.value;
          b |= r.idx < 0;
          x.values[(size_t)j * x.n_labels + i] = v;
          x.active[(size_t)j * x.n_labels + i] = 1;
          if (x.gate[i]) x.chosen[(size_t)j * x.n_labels + i] = (int)(int64_t)v;   // (read for a gate only)
        };
        if (m.lvl_first < 0) {
          for (int64_t j = j0; j < j1; ++j) set(m.res_off + j, j);
          continue;
        }
        const int64_t* base = x.lvl_ids + m.lvl_first;
        const int64_t* lo = std::lower_bound(base, base + m.count, j0);
        const int64_t* hi = std::lower_bound(lo, base + m.count, j1);
        for (const int64_t* p = lo; p < hi; ++p) set(m.res_off + (p - base), *p);
      }
      for (int64_t j = j0; j < j1 && x.n_rem; ++j) {
        int8_t* row = x.active + (size_t)j * x.n_labels;
        double* vrow = x.values + (size_t)j * x.n_labels;
        for (int r = 0; r < x.n_rem; ++r) { row[x.rem[r]] = 1; vrow[x.rem[r]] = NAN; }
      }
      x.bad[k] = b;
    };
    if (nbk > 1) tpe_pool::parallel_for(nbk, put, &mx);
    else put(&mx, 0);
    for (int k = 0; k < nbk; ++k)
      if (bad[(size_t)k]) return tpe_internal_fail(TPE_E_ARG, "no candidate selected for a label");
  }
  return TPE_OK;
}

int tpe_suggest_tree(const tpe_tree_label* labels, int32_t n_labels, const int64_t* below_tids, int64_t n_below,
                     double prior_weight, int32_t lf, const int64_t* ids, int32_t n_ids, int32_t n_cand,
                     int64_t cand_base, int64_t n_cand_global, const tpe_exchange* ex,
                     uint64_t seed, double speculate_min_draws, int64_t device_fit_min, int32_t flags,
                     const tpe_level_ws* ws, tpe_level_need* need, void* stream, double* values, int8_t* active,
                     int32_t* path, int8_t* need_fit) {
  phase_start();
  const int rc = suggest_tree(labels, n_labels, below_tids, n_below, prior_weight, lf, ids, n_ids, n_cand, cand_base,
                              n_cand_global, ex, seed, speculate_min_draws, device_fit_min, flags, ws, need, stream,
                              values, active, path, need_fit);
  tpe_internal_phase(TPE_PHASE_RETURN);
  return rc;
}

}  // extern "C"
