// sort_net.h — the below side's sort of a device-fitted label (tpe_suggest.cpp
// fit_label): a branch-free sorting network over at most kSortNet doubles.
//
// A below side's sort (at most kSortNet values: ap_filter_trials caps the
// below count at 25, tpe.py:625-636): Batcher's odd-even merge network over 32
// keys — the values' order-preserving integer images, NaN after every number,
// padding after NaN — with the positions swapped alongside, branch-free (the
// insertion sort it replaces mispredicted its way through ~1.5 us a label on
// config 5's thousand).  Ties come out in any order: a side of at most 25
// observations has every weight 1 (no linear-forgetting ramp, tpe.py:381-394),
// so tied values are interchangeable in the fit.
#pragma once
#include <cstdint>
#include <cstring>

namespace tpe_sort_net {

constexpr int kSortNet = 32;
struct SortNet {
  int n = 0;
  uint8_t a[256], b[256];
  SortNet() {                                        // Batcher's odd-even mergesort comparators
    for (int p = 1; p < kSortNet; p <<= 1)
      for (int k = p; k >= 1; k >>= 1)
        for (int j = k % p; j + k < kSortNet; j += 2 * k)
          for (int i = 0; i < k && i + j + k < kSortNet; ++i)
            if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) { a[n] = (uint8_t)(i + j); b[n] = (uint8_t)(i + j + k); ++n; }
  }
};
const SortNet g_sort_net;

// sorts x[0, n) (n <= kSortNet) into ord: x[ord[0]] <= x[ord[1]] <= .., NaN last
inline void sort_small(const double* x, int64_t n, int64_t* ord) {
  uint64_t k[kSortNet];
  int64_t ix[kSortNet];
  for (int i = 0; i < kSortNet; ++i) {
    uint64_t u = ~0ull;                              // (padding: after everything)
    if (i < n) {
      const double v = x[i];
      memcpy(&u, &v, 8);
      u = v != v ? ~0ull - 1 : (u >> 63 ? ~u : u | (1ull << 63));   // (NaN: after every number)
    }
    k[i] = u;
    ix[i] = i;
  }
  for (int c = 0; c < g_sort_net.n; ++c) {
    const int a = g_sort_net.a[c], b = g_sort_net.b[c];
    const uint64_t ka = k[a], kb = k[b];
    const bool sw = ka > kb;
    const int64_t ia = ix[a], ib = ix[b];
    k[a] = sw ? kb : ka; k[b] = sw ? ka : kb;
    ix[a] = sw ? ib : ia; ix[b] = sw ? ia : ib;
  }
  for (int64_t i = 0; i < n; ++i) ord[i] = ix[i];
}

}  // namespace tpe_sort_net
