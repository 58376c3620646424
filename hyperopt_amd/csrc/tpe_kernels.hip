// tpe_kernels.hip — gfx950 kernels + C-ABI of the TPE suggest engine.
//
// Replaces, per (new_id, hyperparameter) problem, the numpy operators of
// gsmafra/hyperopt's tpe.suggest (see include/tpe_hip.h for the reference
// file:line of each stage).  Five stages, each a batched launch over a flat
// work list so that problems of very different size share one grid:
//
//   tpe_fit_above    (optional) Parzen fit of large continuous above mixtures
//                    from device-resident observation columns
//   tpe_tables       per-label score tables (continuous: Taylor moments per
//                    value cell; quantized: exact l, g per lattice value)
//   tpe_sample       Philox-4x32-10 candidates from the below mixture; tabulated
//                    and categorical labels are scored right here, the others
//                    get sort keys (problem, 4096 value buckets of the coordinate)
//   tpe_sort         radix sort of the keys (rocPRIM) — candidates of one wave
//                    become neighbours in value, which is what lets the hot
//                    loop skip the above-mixture components that cannot matter
//   tpe_score_above  candidate x component log-sum-exp of the above mixture
//                    (the O(C*K) loop; components are wave-uniform scalar
//                    loads, candidates live in VGPRs, 8 per lane)
//   tpe_finalize     below lpdf (<= 26 components), l - g, per-tile argmax
//   tpe_select       per-problem argmax over tiles (first ORIGINAL index on
//                    ties, NaN wins, like np.argmax) and the chosen value
//
// No atomics: every reduction is in a fixed order, so results are bitwise
// reproducible run to run and identical for any candidate sharding.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <type_traits>
#include <vector>

#include "tpe_pool.h"

#include <dlfcn.h>
#include <rccl/rccl.h>
#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/tpe_hip.h"

extern "C" void tpe_internal_phase(int i);   // tpe_suggest.cpp: host phase clock (hidden)

namespace {

constexpr int kThreads = 256;          // 4 waves of 64
constexpr int kR = 8;                  // candidates per lane
constexpr int kWaveCands = 64 * kR;    // 512 consecutive (sorted) candidates per wave
constexpr int kTile = kThreads * kR;   // candidates per tile
constexpr double kEPS = 1e-12;         // tpe.py:25
constexpr double kLn2 = 0.69314718055994530942;
constexpr float kPruneBits = 45.f;     // skipped terms are < 2^-45 of the sum
constexpr int kCumLds = TPE_SAMPLE_LDS_ROWS;   // sampler CDF rows staged in LDS

// onesweep radix sort from 1024 keys up (rocPRIM's default switches to a merge
// sort up to 2^20 keys, ~5x slower here)
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, 1024>;

thread_local char g_err[512];

int fail(int code, const char* what) {
  snprintf(g_err, sizeof(g_err), "%s", what);
  return code;
}

// kernel launches issued by this thread (the stage profiler tells launched
// stages from skipped ones by it)
thread_local int64_t g_launches = 0;
#define TPE_LAUNCH(...)     \
  do {                      \
    ++g_launches;           \
    hipLaunchKernelGGL(__VA_ARGS__); \
  } while (0)

int hip_check(const char* stage) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", stage, hipGetErrorString(e));
    return TPE_E_HIP;
  }
  return TPE_OK;
}

// ---------------------------------------------------------------- Philox
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32 -> 64-bit product per multiplier (v_mad_u64_u32) instead of a
    // mul_hi / mul_lo pair
    const uint64_t p0 = (uint64_t)M0 * (uint64_t)c0, p1 = (uint64_t)M1 * (uint64_t)c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += W0; k1 += W1;
  }
  return U4{c0, c1, c2, c3};
}

// open-interval uniforms
// 23-bit float uniform in [2^-24, 1 - 2^-24]: (k + 0.5) is exact, so never 0 or 1
__device__ __forceinline__ float u01f(uint32_t r) { return ((float)(r >> 9) + 0.5f) * 1.1920928955078125e-07f; }
__device__ __forceinline__ double u01d(uint32_t a, uint32_t b) {
  const uint64_t m = ((uint64_t)a << 21) ^ (uint64_t)(b >> 11);   // 53 bits
  return ((double)m + 0.5) * 1.1102230246251565e-16;
}
// 32-bit uniform as a double in (0, 1) (exact)
__device__ __forceinline__ double u01w(uint32_t a) { return ((double)a + 0.5) * 2.3283064365386963e-10; }

// ---------------------------------------------------------- argmax order
// better() on an f32 key with a 32-bit index (the cells candidates of k_sample_tab)
__device__ __forceinline__ bool better32(float d, int i, float bd, int bi) {
  if (bi < 0) return i >= 0;
  if (i < 0) return false;
  const bool n = d != d, bn = bd != bd;
  if (n || bn) return n && (!bn || i < bi);
  return d > bd || (d == bd && i < bi);
}

// better32's order as one unsigned key, larger = better, 0 = no candidate: the
// f32 key's bits made monotone (every NaN above +inf and equal to each other;
// -0 as +0, which compares equal to it) over the complemented index (the first
// index wins a tie)
__device__ __forceinline__ unsigned long long key32(float d, int i) {
  if (i < 0) return 0ull;
  uint32_t hi = 0xffffffffu;
  if (d == d) {
    const uint32_t b = __float_as_uint(d + 0.f);
    hi = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  }
  return ((unsigned long long)hi << 32) | (unsigned long long)(~(uint32_t)i);
}
// DPP wave reductions of the device libraries (ockl)
extern "C" __device__ unsigned long long __ockl_wfred_max_u64(unsigned long long);
extern "C" __device__ float __ockl_wfred_min_f32(float);
extern "C" __device__ float __ockl_wfred_max_f32(float);

// np.argmax: NaN is the maximum (first NaN wins), otherwise the largest value,
// first index on ties.
__device__ __forceinline__ bool better(double s, int64_t i, double bs, int64_t bi) {
  if (bi < 0) return i >= 0;
  if (i < 0) return false;
  const bool n = s != s, bn = bs != bs;
  if (n || bn) return n && (!bn || i < bi);
  return s > bs || (s == bs && i < bi);
}

// exact max-shifted log-sum-exp (log2 domain) over up to two component ranges
template <typename T, typename C4>
__device__ __forceinline__ T lse2_exact(const C4* __restrict__ comp, int k0, int n, int k1, int n1, T t) {
  T m = -INFINITY;
  for (int r = 0; r < 2; ++r) {
    const int base = r ? k1 : k0, cnt = r ? n1 : n;
    for (int k = 0; k < cnt; ++k) {
      const C4 c = comp[base + k];
      const T d = (t - (T)c.x) - (T)c.y;
      const T z = d * (T)c.z;
      const T v = (T)c.w - z * z;
      m = v > m ? v : m;
    }
  }
  if (!(m > -INFINITY)) return m;      // empty mixture or all -inf
  T s = 0;
  for (int r = 0; r < 2; ++r) {
    const int base = r ? k1 : k0, cnt = r ? n1 : n;
    for (int k = 0; k < cnt; ++k) {
      const C4 c = comp[base + k];
      const T d = (t - (T)c.x) - (T)c.y;
      const T z = d * (T)c.z;
      s += exp2((T)c.w - z * z - m);
    }
  }
  return m + log2(s);
}

// out-of-line copy for rarely taken paths inside register-heavy kernels
__device__ __attribute__((noinline)) float lse2_exact_ool(const float4* __restrict__ comp, int k0, int n, int k1,
                                                          int n1, float t) {
  return lse2_exact<float, float4>(comp, k0, n, k1, n1, t);
}

// the same sum at a wave-uniform t, the wave's lanes striding over the
// components (inline, few registers: the tabulated sample kernel's fallback)
__device__ __forceinline__ float lse2_wave(const float4* __restrict__ comp, int k0, int n0, int k1, int n1, float t) {
  const int lane = threadIdx.x & 63, n = n0 + n1;
  float m = -INFINITY;
#pragma unroll 1
  for (int i = lane; i < n; i += 64) {
    const float4 c = i < n0 ? comp[k0 + i] : comp[k1 + i - n0];
    const float z = ((t - c.x) - c.y) * c.z;
    m = fmaxf(m, c.w - z * z);
  }
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if (!(m > -INFINITY)) return m;
  float s = 0.f;
#pragma unroll 1
  for (int i = lane; i < n; i += 64) {
    const float4 c = i < n0 ? comp[k0 + i] : comp[k1 + i - n0];
    const float z = ((t - c.x) - c.y) * c.z;
    s += exp2f(c.w - z * z - m);
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  return m + log2f(s);
}

// Max-shifted log2-sum of a PRUNED above mixture at t (the fixed-shift sum
// under-flowed: t is far from every component).  m0 = the best term among the
// wide components and t's grid neighbours bounds the sum from below, so a narrow
// component with mu outside t +- sqrt(narrow_cmax - m0 + 45) / narrow_amin is
// under 2^-45 of it — the above kernel's pruning rule with a much tighter bound:
// a few components instead of all K, serially per candidate.
__device__ __attribute__((noinline)) float lse2_pruned(const tpe_problem& p, const float4* __restrict__ comp,
                                                       const int32_t* __restrict__ grid, float t) {
  const float4* __restrict__ C = comp + p.above_off;
  const float4* __restrict__ Wd = comp + p.wide_off;
  const int32_t* __restrict__ G = grid + p.grid_off;
  float m0 = -INFINITY;
  for (int k = 0; k < p.wide_len; ++k) {
    const float4 c = Wd[k];
    const float z = ((t - c.x) - c.y) * c.z;
    m0 = fmaxf(m0, c.w - z * z);
  }
  const int gb = (int)fminf(fmaxf(floorf((t - p.grid_lo) * p.grid_inv), 0.f), (float)p.grid_n);
  const int kc = G[gb];
  for (int k = max(kc - 2, 0); k < min(kc + 2, p.above_len); ++k) {
    const float4 c = C[k];
    const float z = ((t - c.x) - c.y) * c.z;
    m0 = fmaxf(m0, c.w - z * z);
  }
  const float R = sqrtf(fmaxf(p.narrow_cmax - m0 + kPruneBits, 0.f)) / p.narrow_amin;
  const float vlo = t - R, vhi = t + R;
  if (!(m0 > -INFINITY) || !(vlo == vlo && vhi == vhi && R < INFINITY))
    return lse2_exact<float, float4>(comp, p.above_off, p.above_len, p.wide_off, p.wide_len, t);
  const float gl = (vlo - p.grid_lo) * p.grid_inv, gh = (vhi - p.grid_lo) * p.grid_inv;
  const int bl = (int)fminf(fmaxf(floorf(gl) - 1.f, 0.f), (float)p.grid_n);
  const int bh = (int)fminf(fmaxf(floorf(gh) + 2.f, 0.f), (float)p.grid_n);
  const int kl = G[bl], kh = max(G[bh], G[bl]);
  return lse2_exact<float, float4>(comp, p.above_off + kl, kh - kl, p.wide_off, p.wide_len, t);
}

// one-pass fixed-shift sum (every c_k <= 0) with the exact two-pass fallback
// when it under-flows; used for the short below mixture
__device__ __forceinline__ float lse2_fixed(const float4* __restrict__ comp, int k0, int n, float t) {
  float s = 0.f;
#pragma unroll 4
  for (int k = 0; k < n; ++k) {
    const float4 c = comp[k0 + k];
    const float d = (t - c.x) - c.y;
    const float z = d * c.z;
    s += __builtin_amdgcn_exp2f(__builtin_fmaf(-z, z, c.w));
  }
  if (s > 1e-30f) return __log2f(s);
  return lse2_exact<float, float4>(comp, k0, n, 0, 0, t);
}

// double version for comp64 {mu, a, c, 0}
__device__ __forceinline__ double lse2_exact64(const double4* __restrict__ comp, int k0, int n, double t) {
  double m = -INFINITY;
  for (int k = 0; k < n; ++k) {
    const double4 c = comp[k0 + k];
    const double z = (t - c.x) * c.y;
    const double v = c.z - z * z;
    m = v > m ? v : m;
  }
  if (!(m > -INFINITY)) return m;
  double s = 0;
  for (int k = 0; k < n; ++k) {
    const double4 c = comp[k0 + k];
    const double z = (t - c.x) * c.y;
    s += exp2(c.z - z * z - m);
  }
  return m + log2(s);
}

// quantized mixture mass: sum_k w Phi(zu) - w Phi(zl), reference operation order
// (tpe.py:147-159 / :285-298).  LOG selects lognormal_cdf's constant folding.
template <bool LOG>
__device__ __forceinline__ double qterm(const double4& c, double tu, double tl) {
  // (no contraction, as numpy evaluates it: an fma of inc's product with -dec
  // would leave dec's rounding error where tu == tl and the mass is exactly 0 —
  // a tiny negative sum whose log is NaN instead of the reference's -inf)
#pragma clang fp contract(off)
  const double zu = (tu - c.x) / c.y;
  const double zl = (tl - c.x) / c.y;
  double inc, dec;
  if (LOG) { inc = c.z * (.5 + .5 * erf(zu)); dec = c.z * (.5 + .5 * erf(zl)); }
  else     { inc = c.z * (0.5 * (1 + erf(zu))); dec = c.z * (0.5 * (1 + erf(zl))); }
  inc -= dec;
  return inc;
}

template <bool LOG>
__device__ __forceinline__ double qmass(const double4* __restrict__ comp, int k0, int n, double tu, double tl) {
  double prob = 0.0;
  for (int k = 0; k < n; ++k) prob += qterm<LOG>(comp[k0 + k], tu, tl);
  return prob;
}

// quantization interval of one candidate in the kernel coordinate
// (tpe.py:148-155 for GMM1_lpdf, :286-294 + lognormal_cdf :185 for LGMM1_lpdf)
__device__ __forceinline__ void q_bounds(const tpe_problem& p, double x, double& tu, double& tl) {
  double ub = x + p.q / 2.0, lb = x - p.q / 2.0;
  if (p.family == TPE_FAM_QGAUSS) {
    if (p.flags & TPE_F_HAS_HIGH) ub = fmin(ub, p.high);
    if (p.flags & TPE_F_HAS_LOW) lb = fmax(lb, p.low);
    tu = ub; tl = lb;
  } else {
    if (p.flags & TPE_F_HAS_HIGH) ub = fmin(ub, exp(p.high));
    if (p.flags & TPE_F_HAS_LOW) lb = fmax(lb, exp(p.low));
    lb = fmax(0.0, lb);
    tu = log(fmax(ub, kEPS));
    tl = log(fmax(lb, kEPS));
  }
}

typedef float f2 __attribute__((ext_vector_type(2)));

// one component against kR candidates held as kR/2 packed pairs:
// s += 2^(c - (a ((t - mu_hi) - mu_lo))^2)
__device__ __forceinline__ void ce_step(const float4 c, const f2 (&t)[kR / 2], f2 (&s)[kR / 2]) {
  const f2 mh = f2{c.x, c.x}, ml = f2{c.y, c.y}, a = f2{c.z, c.z}, cw = f2{c.w, c.w};
#pragma unroll
  for (int j = 0; j < kR / 2; ++j) {
    const f2 d = (t[j] - mh) - ml;
    const f2 z = d * a;
    const f2 v = __builtin_elementwise_fma(-z, z, cw);     // = lse2_fixed's fmaf(-z, z, c)
    s[j] += f2{__builtin_amdgcn_exp2f(v.x), __builtin_amdgcn_exp2f(v.y)};
  }
}

// sorted position of candidate j (0..kR-1) of this lane inside a tile
__device__ __forceinline__ int tile_pos(int cand_start, int j) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  return cand_start + wave * kWaveCands + lane + 64 * j;
}

// ================================================================= sample
// Phi^-1(pr) in f32 = -sqrt2 erfinv(1 - 2 pr), erfinv by Giles' single-precision
// approximation ("Approximating the erfinv function", GPU Computing Gems 2010)
// with its log argument (1 - x)(1 + x) = 4 pr (1 - pr) formed from pr itself (no
// cancellation in the tails).  Relative error <= 3e-7 over the f32 uniforms
// (checked against scipy.special.ndtri); one v_log_f32, the tail branch adds a
// sqrt.  Every f32 draw inverts through this one function.
__device__ __forceinline__ float ndtri_f32(float pr) {
  const float x = 1.f - 2.f * pr;
  float w = -__logf(4.f * pr * (1.f - pr));
  float q;
  if (w < 5.f) {
    w -= 2.5f;
    q = 2.81022636e-08f;
    q = __builtin_fmaf(q, w, 3.43273939e-07f); q = __builtin_fmaf(q, w, -3.5233877e-06f);
    q = __builtin_fmaf(q, w, -4.39150654e-06f); q = __builtin_fmaf(q, w, 0.00021858087f);
    q = __builtin_fmaf(q, w, -0.00125372503f); q = __builtin_fmaf(q, w, -0.00417768164f);
    q = __builtin_fmaf(q, w, 0.246640727f); q = __builtin_fmaf(q, w, 1.50140941f);
  } else {
    w = __builtin_sqrtf(w) - 3.f;
    q = -0.000200214257f;
    q = __builtin_fmaf(q, w, 0.000100950558f); q = __builtin_fmaf(q, w, 0.00134934322f);
    q = __builtin_fmaf(q, w, -0.00367342844f); q = __builtin_fmaf(q, w, 0.00573950773f);
    q = __builtin_fmaf(q, w, -0.0076224613f); q = __builtin_fmaf(q, w, 0.00943887047f);
    q = __builtin_fmaf(q, w, 1.00167406f); q = __builtin_fmaf(q, w, 2.83297682f);
  }
  return -1.41421356237309505f * (q * x);
}

// The uniforms of candidate i (Philox-4x32-10, counter = its GLOBAL index g, so
// draws do not depend on sharding or on which kernel re-draws them): `us`
// selects the component (category), `uf` / `ud` invert its truncated normal in
// f32 / f64.  f32 draws of the non-categorical families take two candidates per
// Philox block — g even: words (x, y) of block g / 2, g odd: (z, w) — a 32-bit
// selection uniform and 23 bits of inversion; f64 draws and categories take one
// block per candidate (53-bit selection, 53-bit inversion).
struct DrawU { double us; float uf; double ud; uint32_t ws; };   // ws: us's 32-bit word (f32 draws)
__device__ __forceinline__ DrawU draw_uniforms(const tpe_problem& p, int64_t i, int precision) {
  const uint64_t g = (uint64_t)p.cand_base + (uint64_t)i;
  if (precision == TPE_PREC_F32 && p.family != TPE_FAM_CATEGORICAL) {
    const uint64_t blk = g >> 1;
    const U4 r = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), p.ctr2, p.ctr3, p.key0, p.key1);
    const bool odd = g & 1;
    return DrawU{u01w(odd ? r.z : r.x), u01f(odd ? r.w : r.y), 0.0, odd ? r.z : r.x};
  }
  const U4 r = philox4x32_10((uint32_t)g, (uint32_t)(g >> 32), p.ctr2, p.ctr3, p.key0, p.key1);
  return DrawU{u01d(r.x, r.y), u01f(r.z), u01d(r.z, r.w), 0u};
}

// f32 truncation bounds of a problem: smallest float >= low, largest float < high
__device__ __forceinline__ void f32_bounds(const tpe_problem& p, float& lo_f, float& hi_f) {
  lo_f = -INFINITY; hi_f = INFINITY;
  if (p.flags & TPE_F_HAS_LOW) { lo_f = (float)p.low; if ((double)lo_f < p.low) lo_f = nextafterf(lo_f, INFINITY); }
  if (p.flags & TPE_F_HAS_HIGH) {
    hi_f = (float)p.high;
    while ((double)hi_f >= p.high) hi_f = nextafterf(hi_f, -INFINITY);
  }
}

// component (category) choice of candidate i: first k with u < cum_k
__device__ __forceinline__ int draw_category(const tpe_problem& p, const double* __restrict__ cum, int64_t i) {
  const uint64_t g = (uint64_t)p.cand_base + (uint64_t)i;
  const U4 r = philox4x32_10((uint32_t)g, (uint32_t)(g >> 32), p.ctr2, p.ctr3, p.key0, p.key1);
  const double u1 = u01d(r.x, r.y);
  int a = 0, b = p.samp_len - 1;
  while (a < b) { const int m = (a + b) >> 1; if (u1 < cum[m]) b = m; else a = m + 1; }
  return a;
}

// first component k with u < cum_k (binary search; cum stride cs)
__device__ __forceinline__ int find_comp(const tpe_problem& p, const double* __restrict__ cum, int cs, double u) {
  int a = 0, b = p.samp_len - 1;
  while (a < b) { const int m = (a + b) >> 1; if (u < cum[cs * m]) b = m; else a = m + 1; }
  return a;
}

// Value x and kernel coordinate t (x, or ln x before quantisation for log
// families) of a draw from component a of the below mixture, by inversion of its
// truncated normal at the uniform uf (f32) / ud (f64).
// f32 inversion of sampler row s (truncated normal; fa, fb = Phi of the
// mirrored bounds) at the uniform uf: the kernel coordinate of the draw
__device__ __forceinline__ float comp_coord_f32(const double* __restrict__ s, float uf, float lo_f, float hi_f) {
  const float pr = (float)s[3] + uf * ((float)s[4] - (float)s[3]);
  float z = ndtri_f32(pr);
  if (s[5] != 0.0) z = -z;
  float xf = (float)s[1] + (float)s[2] * z;
  if (!(xf == xf)) xf = (float)s[1];
  return fminf(fmaxf(xf, lo_f), hi_f);   // low <= draw < high (tpe.py:86)
}

__device__ __forceinline__ void draw_comp(const tpe_problem& p, const double* __restrict__ S, int a, float uf,
                                          double ud, int precision, float lo_f, float hi_f, double& x, float& t) {
  const double* s = S + 8 * a;
  // truncated normal by inversion; fa, fb = Phi of the (mirrored) bounds
  const double mu = s[1], sg = s[2], fa = s[3], fb = s[4];
  const bool flip = s[5] != 0.0;
  if (precision == TPE_PREC_F32) {
    t = comp_coord_f32(s, uf, lo_f, hi_f);
    x = (double)t;
  } else {
    const double pr = fa + ud * (fb - fa);
    double z = -1.41421356237309505 * erfcinv(2.0 * pr);
    if (flip) z = -z;
    x = mu + sg * z;
    if (!(x == x)) x = mu;
    if ((p.flags & TPE_F_HAS_LOW) && x < p.low) x = p.low;
    if ((p.flags & TPE_F_HAS_HIGH) && x >= p.high) x = nextafter(p.high, -INFINITY);
    t = (float)x;
  }
  if (p.family == TPE_FAM_LOGGAUSS || p.family == TPE_FAM_QLOGGAUSS) x = exp(x);
  if (p.family == TPE_FAM_QGAUSS || p.family == TPE_FAM_QLOGGAUSS) x = rint(x / p.q) * p.q;   // np.round
}

// Candidate i of problem p, i.i.d. (Philox-4x32-10 counter = its GLOBAL index):
// the value x returned to the user and the kernel coordinate t (the category
// for categorical).  `cum` is the selection CDF (LDS copy or the table itself,
// stride `cs`).  k_select calls it again for the winner, so the value never has
// to be stored.
__device__ __forceinline__ void draw_one(const tpe_problem& p, const double* __restrict__ S,
                                         const double* __restrict__ cum, int cs, int64_t i, int precision,
                                         float lo_f, float hi_f, double& x, float& t, int& comp) {
  const DrawU u = draw_uniforms(p, i, precision);
  const int a = find_comp(p, cum, cs, u.us);
  comp = a;
  if (p.family == TPE_FAM_CATEGORICAL) {
    x = (double)a;
    t = (float)a;
    return;
  }
  draw_comp(p, S, a, u.uf, u.ud, precision, lo_f, hi_f, x, t);
}

// draw_one's kernel coordinate alone (f32, continuous families): no f64 value
__device__ __forceinline__ float draw_coord_f32(const tpe_problem& p, const double* __restrict__ S,
                                                const double* __restrict__ cum, int cs, int64_t i, float lo_f,
                                                float hi_f) {
  const DrawU u = draw_uniforms(p, i, TPE_PREC_F32);
  const int a = find_comp(p, cum, cs, u.us);
  return comp_coord_f32(S + 8 * a, u.uf, lo_f, hi_f);
}

// ------------------------------------------------------------ ordered draws
// (include/tpe_hip.h "Ordered draws").  Inclusive prefix sum, in lane order,
// of E_i = -ln u_i over the canonical 64-index block `blk` of problem p (lane l
// <-> global index 64 blk + l; indices past the global count add 0).
// Wave-collective, fixed (Hillis-Steele) order, and not inlined, so the sample,
// block-sum and select kernels compute bit-identical sums.
__device__ __attribute__((noinline)) double exp_block_scan(const tpe_problem& p, int64_t blk) {
  const int lane = threadIdx.x & 63;
  const uint64_t g = (uint64_t)blk * 64 + (uint64_t)lane;
  double e = 0.0;
  if ((int64_t)g <= p.n_cand_global) {
    const U4 r = philox4x32_10((uint32_t)g, (uint32_t)(g >> 32), p.ctr2, p.ctr3, p.key0, p.key1);
    e = -log(u01d(r.x, r.y));
  }
  for (int d = 1; d < 64; d <<= 1) {
    const double o = __shfl_up(e, d);
    if (lane >= d) e += o;
  }
  return e;
}

// The draw at uniform order statistic U: component by the selection CDF, then
// the component's inverse CDF at U's relative position inside the component.
__device__ __forceinline__ void ordered_draw(const tpe_problem& p, const double* __restrict__ S,
                                             const double* __restrict__ cum, int cs, double U, int precision,
                                             float lo_f, float hi_f, double& x, float& t) {
  const int a = find_comp(p, cum, cs, U);
  const double lo = a > 0 ? cum[cs * (a - 1)] : 0.0, hi = cum[cs * a];
  const double w = (U - lo) / (hi - lo);
  const double ud = fmin(fmax(w, 1.1102230246251565e-16), 1.0 - 1.1102230246251565e-16);
  const float uf = fminf(fmaxf((float)w, 5.9604644775390625e-08f), 0.99999994f);
  draw_comp(p, S, a, uf, ud, precision, lo_f, hi_f, x, t);
}

// per sorted problem, the sum of every canonical 64-index block (one wave each)
__global__ __launch_bounds__(kThreads) void k_draw_sums(const tpe_problem* __restrict__ P, int64_t draw_blocks,
                                                        double* __restrict__ pref) {
  const int64_t per = (draw_blocks + kThreads / 64 - 1) / (kThreads / 64);
  const tpe_problem& p = P[blockIdx.x / per];
  if (p.sort_slot < 0 || p.samp_len <= 0) return;
  const int64_t blk = (int64_t)(blockIdx.x % per) * (kThreads / 64) + (threadIdx.x >> 6);
  if (blk >= draw_blocks) return;
  const double s = exp_block_scan(p, blk);
  if ((threadIdx.x & 63) == 63) pref[(int64_t)p.sort_slot * (draw_blocks + 1) + blk] = s;
}

// exclusive prefix of the block sums in place (fixed order: chunk sums, one
// serial pass over them, serial chunks) and the total at [draw_blocks]
__global__ __launch_bounds__(kThreads) void k_draw_scan(const tpe_problem* __restrict__ P, int64_t draw_blocks,
                                                        double* __restrict__ pref) {
  const tpe_problem& p = P[blockIdx.x];
  if (p.sort_slot < 0 || p.samp_len <= 0) return;
  double* row = pref + (int64_t)p.sort_slot * (draw_blocks + 1);
  const int64_t chunk = (draw_blocks + kThreads - 1) / kThreads;
  const int64_t b0 = min(draw_blocks, (int64_t)threadIdx.x * chunk), b1 = min(draw_blocks, b0 + chunk);
  double acc = 0.0;
  for (int64_t b = b0; b < b1; ++b) acc += row[b];
  __shared__ double part[kThreads];
  part[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double run = 0.0;
    for (int q = 0; q < kThreads; ++q) { const double v = part[q]; part[q] = run; run += v; }
    row[draw_blocks] = run;
  }
  __syncthreads();
  double run = part[threadIdx.x];
  for (int64_t b = b0; b < b1; ++b) { const double v = row[b]; row[b] = run; run += v; }
}

// ------------------------------------------------------------ pooled labels
// (include/tpe_hip.h "Pooled labels").  u64 key of (score, candidate index):
// the order-preserving integer of the f64 score (NaN canonicalised: the
// maximum, as in np.argmax) with its low idx_bits replaced by the complemented
// index, so atomicMax keeps the best score and, among equal (truncated) scores,
// the first index.  0 = no candidate.
__device__ __forceinline__ int pool_idx_bits(int n_cand) { return n_cand > 1 ? 32 - __clz(n_cand - 1) : 1; }

__device__ __forceinline__ unsigned long long pool_key(double score, int64_t idx, int idx_bits) {
  if (score != score) score = __longlong_as_double(0x7FF8000000000000ll);
  unsigned long long u = (unsigned long long)__double_as_longlong(score);
  u = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
  const unsigned long long mask = (1ull << idx_bits) - 1;
  return (u & ~mask) | (mask - (unsigned long long)idx);
}

// fold candidate `oo` (absolute position in the candidate arrays) of a pooled
// label into its own problem's best; a relaxed read skips most atomics
__device__ __forceinline__ void pool_update(const tpe_problem* __restrict__ P, const tpe_problem& p,
                                            unsigned long long* __restrict__ pool_best, int64_t oo, double score) {
  const int64_t base = P[p.pool_first].cand_off;
  const int64_t rel = oo - base;
  const int64_t r = p.pool_first + rel / p.n_cand;
  const unsigned long long key = pool_key(score, rel % p.n_cand, pool_idx_bits(p.n_cand));
  if (key > __hip_atomic_load(pool_best + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(pool_best + r, key);
}

// block argmax of (score, original index) into one tile_best slot; the lane
// that holds the winner (unique index) publishes its l and g
__device__ __forceinline__ void block_best(double sc, int64_t orig, double l, double g, tpe_best* __restrict__ slot) {
  double bs = sc;
  int64_t bi = orig;
  for (int off = 32; off > 0; off >>= 1) {
    const double os = __shfl_xor(bs, off);
    const int64_t oi = __shfl_xor(bi, off);
    if (better(os, oi, bs, bi)) { bs = os; bi = oi; }
  }
  __shared__ tpe_best wb[kThreads / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0 && bi < 0) wb[wave] = tpe_best{0, 0, 0, -1};
  if (bi >= 0 && orig == bi) wb[wave] = tpe_best{bs, l, g, bi};
  __syncthreads();
  if (threadIdx.x == 0) {
    tpe_best b = wb[0];
    for (int q = 1; q < kThreads / 64; ++q)
      if (better(wb[q].score, wb[q].idx, b.score, b.idx)) b = wb[q];
    *slot = b;
  }
}

// ----------------------------------------------------------- score tables
// (include/tpe_hip.h "Tabulated scoring").  Cell row: 16 floats {M0..M10, m,
// c, 1/h, flag, 0}.
constexpr int kTabMoments = 11;        // degree-10 Taylor moments per cell
constexpr int kTabStageRowsDecl = 4096; // component rows a table workgroup stages in LDS (k_tables; 64 KiB: two workgroups per CU)
constexpr float kTabDrop = 50.f;       // terms below 2^-50 of the cell's largest are dropped

// Draws (when `draw`) and writes the sort keys: (sorted problem << key_bits) |
// value bucket.  Grid (tiles, TPE_BEST_PER_TILE): block (x, y) handles the y-th
// 256-candidate slice of tile x, one candidate per thread — a 2^20-candidate
// problem runs 4096 workgroups (16 waves per CU).  Categorical problems are
// scored here (categorical_lpdf is a table gather, tpe.py:50-57) and write
// their slice's best straight to tile_best: nothing else of theirs is stored.
// Candidate values are stored only where a later stage reads them (quantized
// and f64 families) or on request (TPE_BATCH_WRITE_CAND).
__global__ __launch_bounds__(kThreads) void k_sample(const tpe_problem* __restrict__ P,
                                                     const tpe_tile* __restrict__ tiles,
                                                     const double* __restrict__ samp,
                                                     const double4* __restrict__ comp64,
                                                     double* __restrict__ cand, float* __restrict__ coord,
                                                     uint32_t* __restrict__ keys, uint64_t* __restrict__ vals,
                                                     uint64_t* __restrict__ vals_sorted,
                                                     tpe_best* __restrict__ tile_best,
                                                     double* __restrict__ l_out, double* __restrict__ g_out,
                                                     int precision, int draw, int key_bits, int flags,
                                                     const double* __restrict__ draw_pref, int64_t draw_blocks,
                                                     int ordered, unsigned long long* __restrict__ pool_best,
                                                     const int32_t* __restrict__ list) {
  const int tile = list ? list[blockIdx.x] : (int)blockIdx.x;
  const tpe_tile tl = tiles[tile];
  const tpe_problem& p = P[tl.problem];
  if (p.tab_mode != TPE_TAB_NONE) return;   // k_sample_tab's
  if (draw && p.family == TPE_FAM_CATEGORICAL && p.samp_len <= kCumLds && (p.flags & TPE_F_CAT_LAZY) &&
      !(flags & TPE_BATCH_WRITE_CAND) && !l_out)
    return;                                // lazy categorical: the select stage scans the first draws itself
  if ((p.flags & TPE_F_POOLED) && tl.cand_start == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    pool_best[tl.problem] = 0ull;          // scored after this kernel: no race
  const bool store_x = (flags & TPE_BATCH_WRITE_CAND) || precision == TPE_PREC_F64 ||
                       p.family == TPE_FAM_QGAUSS || p.family == TPE_FAM_QLOGGAUSS;
  float lo_f, hi_f;
  f32_bounds(p, lo_f, hi_f);
  const double* S = samp + 8 * (int64_t)p.samp_off;
  const uint32_t khi = (uint32_t)p.sort_slot << key_bits;
  const float kmax = (float)((1 << key_bits) - 1);
  // selection CDF staged in LDS: the per-lane binary search then costs no
  // dependent global loads (tables longer than kCumLds search global memory)
  __shared__ double cum_lds[kCumLds];
  const bool in_lds = draw && p.samp_len <= kCumLds;
  if (in_lds)
    for (int q = threadIdx.x; q < p.samp_len; q += kThreads) cum_lds[q] = S[8 * q];
  __syncthreads();
  const int i = tl.cand_start + (int)threadIdx.x + (int)blockIdx.y * kThreads;
  const bool valid = i < p.n_cand;
  const int64_t o = p.cand_off + i;
  if (draw && p.family == TPE_FAM_CATEGORICAL && p.samp_len <= kCumLds) {
    // The score of a categorical candidate depends only on its category, so the
    // slice's argmax (np.argmax: best score, then first index) is the best
    // category among those drawn, at its first draw.  First index per category:
    // wave ballots (the lowest set lane is the earliest candidate) for up to 64
    // categories, LDS atomicMin (order-independent) beyond; then one thread
    // picks the category from LDS.  No per-candidate gathers or shuffles.
    __shared__ int first[kCumLds];
    __shared__ double score[kCumLds];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int base = tl.cand_start + (int)blockIdx.y * kThreads;
    const int c = valid ? draw_category(p, cum_lds, i) : -1;
    if (valid && l_out) { l_out[o] = comp64[p.below_off + c].x; g_out[o] = comp64[p.above_off + c].x; }
    if (valid && (flags & TPE_BATCH_WRITE_CAND)) cand[o] = (double)c;
    const int U = p.samp_len;
    for (int q = threadIdx.x; q < U; q += kThreads) {
      first[q] = INT_MAX;
      score[q] = comp64[p.below_off + q].x - comp64[p.above_off + q].x;
    }
    __syncthreads();
    if (U <= 64) {
      for (int cc = 0; cc < U; ++cc) {
        const unsigned long long m = __ballot(c == cc);
        if (lane == 0 && m) atomicMin(&first[cc], base + wave * 64 + __builtin_ctzll(m));
      }
    } else if (c >= 0) {
      atomicMin(&first[c], i);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      tpe_best b{0, 0, 0, -1};
      for (int cc = 0; cc < U; ++cc)
        if (first[cc] != INT_MAX && better(score[cc], (int64_t)first[cc], b.score, b.idx)) {
          b.score = score[cc];
          b.l = comp64[p.below_off + cc].x;
          b.g = comp64[p.above_off + cc].x;
          b.idx = first[cc];
        }
      tile_best[(int64_t)tile * TPE_BEST_PER_TILE + blockIdx.y] = b;
    }
    return;
  }
  // ordered draws of a sorted problem: no sort follows, candidates go straight
  // to their final place
  const bool od = ordered && draw && p.sort_slot >= 0;
  double Sg = 0.0;                         // E_0 + .. + E_g of this candidate
  if (od && p.samp_len > 0) {
    // whole waves: the block scans are wave-collective
    const int wbase = tl.cand_start + (int)blockIdx.y * kThreads + (int)(threadIdx.x & ~63);
    if (wbase >= p.n_cand) return;
    const int lane = threadIdx.x & 63;
    const int64_t g0 = p.cand_base + wbase;
    const int64_t blk = g0 >> 6;
    const int off = (int)(g0 & 63);
    const double* row = draw_pref + (int64_t)p.sort_slot * (draw_blocks + 1);
    const double sa = exp_block_scan(p, blk);
    if (off == 0) {
      Sg = row[blk] + sa;
    } else {                               // the wave straddles two canonical blocks
      const double sb = exp_block_scan(p, blk + 1);
      const int src = (off + lane) & 63;
      const double a = __shfl(sa, src), bq = __shfl(sb, src);
      Sg = off + lane < 64 ? row[blk] + a : row[blk + 1] + bq;
    }
    Sg /= row[draw_blocks];                // U_g
  }
  if (!valid) return;
  float t;                                 // kernel coordinate of the candidate
  if (!draw) {
    t = coord[o];
  } else if (p.samp_len <= 0) {
    cand[o] = NAN; t = NAN;
  } else if (od) {
    double x;
    ordered_draw(p, S, in_lds ? cum_lds : S, in_lds ? 1 : 8, Sg, precision, lo_f, hi_f, x, t);
    if (store_x) cand[o] = x;
  } else {
    double x;
    int c;
    draw_one(p, S, in_lds ? cum_lds : S, in_lds ? 1 : 8, i, precision, lo_f, hi_f, x, t, c);
    if (store_x) cand[o] = x;
  }
  const uint64_t v = ((uint64_t)o << 32) | (uint64_t)__float_as_uint(t);
  if (p.sort_slot >= 0 && !od) {
    // sort key: (sorted problem, value bucket) — only locality matters for pruning
    const float gb = floorf((t - p.key_lo) * p.key_inv);
    const uint32_t bucket = gb > 0.f ? (uint32_t)fminf(gb, kmax) : 0u;
    keys[o] = khi | bucket;
    vals[o] = v;
  } else {
    vals_sorted[o] = v;                    // never sorted: straight to its final place
  }
}

// Tabulated problems (include/tpe_hip.h "Tabulated scoring").  One 1024-thread
// workgroup per CU-sized group of `per_wg` tabulated tiles (list order: a
// problem's tiles are contiguous).  On entering a problem the workgroup stages
// its selection CDF, a guide table into it, compact f32 sampler rows and —
// when they fit — both cell tables in LDS, so a candidate's draw and score
// issue no global loads: Philox, a guide-started CDF scan, the f32 inverse CDF,
// two table rows and their Horner sums.  Every thread keeps its best; a run of
// tiles of one problem leaves its best in slot 0 of the run's first tile (the
// other slots of its tiles are empty).  Nothing per candidate is stored unless
// asked for (l_out / TPE_BATCH_WRITE_CAND).
constexpr int kTabThreads = 1024;
constexpr int kTabLdsCells = 2048;                  // 96 KiB of 48-B cell rows
static_assert(TPE_TAB_ROW_UNITS == 3 && kTabMoments == 11, "a cell row: 11 moments and the shift in 3 float4");
constexpr int kGuide = 256;                         // CDF guide entries
constexpr int kTabMaxTilesPerWg = 16;
static_assert(kTile % kTabThreads == 0, "tabulated sample tiling");
constexpr int kTabPer = kTile / kTabThreads;         // candidates per thread per tile
static_assert(kTabPer % 2 == 0, "a thread draws its candidates in Philox pairs");

// Guide entry b of a selection CDF: k0 = the first k with cum_k > b / kGuide
// (where the answer for any u in [b, b + 1) / kGuide starts) and its first two
// steps as thresholds on the 32-bit word w the uniform comes from: u = (w +
// 0.5) 2^-32 < c  <=>  w < T(c) = ceil(c 2^32 - 0.5) (both sides exact in
// f64), so a step is passed when w >= T; `never` flags a step past the last
// component or a T of 2^32 (no w reaches it).  One 16-B LDS read per lookup.
struct GuideEnt {
  uint32_t t0, t1;        // T(cum[k0]), T(cum[k0 + 1])
  int32_t k0;
  uint32_t never;         // bit 0: step 0 never passed, bit 1: step 1
};
static_assert(sizeof(GuideEnt) == 16, "guide entries: one 16-B LDS read");

__device__ __forceinline__ uint32_t guide_thresh(double c, uint32_t& never, uint32_t bit) {
  const double t = ceil(c * 4294967296.0 - 0.5);
  if (!(t < 4294967296.0)) { never |= bit; return 0xffffffffu; }
  return t > 0.0 ? (uint32_t)t : 0u;
}

// first k with u < cum_k (k <= len - 1), u = u01w(w): the binary search's
// answer (find_comp) on a non-decreasing CDF.  The guide entry (w's top 8
// bits: floor(u kGuide)) settles it in two steps; `more` flags the (rare) w
// that needs a third (guided_more).
__device__ __forceinline__ int guided_comp(const GuideEnt* __restrict__ guide, uint32_t w, bool& more) {
  const GuideEnt e = guide[w >> 24];
  const bool s0 = !(e.never & 1u) && w >= e.t0, s1 = s0 && !(e.never & 2u) && w >= e.t1;
  more = s1;
  return e.k0 + (int)s0 + (int)s1;
}
// the steps past the guide entry's two (lanes with `more`)
__device__ __forceinline__ int guided_more(const double* __restrict__ cum, int len, double u, int k) {
  while (k < len - 1 && !(u < cum[k])) ++k;
  return k;
}

// log2 of one mixture side's sum at t from its cell rows (LDS), cell_log2_lds
// without branches: the row of a clamped cell index is read and the result
// replaced by NAN when t lies outside the cells, in a flagged cell or the
// series is not positive (the same arithmetic for every t inside)
__device__ __forceinline__ float cell_log2_nb(float lo, float inv, float w, float ih, int n,
                                              const float4* __restrict__ rows, int stride, int step, float t) {
  const float gj = floorf((t - lo) * inv);
  const bool in = gj >= 0.f && gj < (float)n;
  const float4* __restrict__ r = rows + step * (in ? (int)gj : 0);
  const float4 a = r[0], b = r[stride], c = r[2 * stride];
  const float u = (t - __builtin_fmaf(gj + 0.5f, w, lo)) * ih;
  float sm = c.z;
  sm = __builtin_fmaf(sm, u, c.y); sm = __builtin_fmaf(sm, u, c.x);
  sm = __builtin_fmaf(sm, u, b.w); sm = __builtin_fmaf(sm, u, b.z); sm = __builtin_fmaf(sm, u, b.y);
  sm = __builtin_fmaf(sm, u, b.x); sm = __builtin_fmaf(sm, u, a.w); sm = __builtin_fmaf(sm, u, a.z);
  sm = __builtin_fmaf(sm, u, a.y); sm = __builtin_fmaf(sm, u, a.x);
  const float v = c.w + __log2f(sm);
  return in && sm > 0.f ? v : NAN;
}

// log2 of one mixture side's sum at t from its cell rows (LDS or global); NAN
// when t lies outside the cells, in a flagged cell (NaN shift), or the series is
// not positive (the caller then sums the mixture exactly).  w = 1 / inv, ih =
// 1 / h: the cell centre and u as k_tables forms them.
// (row j's k-th float4 at rows[k * stride + j * step]: rows are contiguous,
// stride 1 / step 3, in global memory and LDS alike — a 48-B row j starts at
// 16-B slot 3 j mod 16 of the banks, a permutation of j mod 16, so random rows
// of a wave spread over the banks as planes would)
__device__ __forceinline__ float cell_log2_lds(float lo, float inv, float w, float ih, int n,
                                               const float4* __restrict__ rows, int stride, int step, float t) {
  const float gj = floorf((t - lo) * inv);
  if (!(gj >= 0.f && gj < (float)n)) return NAN;
  const float4* __restrict__ r = rows + step * (int)gj;
  const float4 a = r[0], b = r[stride], c = r[2 * stride];
  const float u = (t - __builtin_fmaf(gj + 0.5f, w, lo)) * ih;
  float sm = c.z;
  sm = __builtin_fmaf(sm, u, c.y); sm = __builtin_fmaf(sm, u, c.x);
  sm = __builtin_fmaf(sm, u, b.w); sm = __builtin_fmaf(sm, u, b.z); sm = __builtin_fmaf(sm, u, b.y);
  sm = __builtin_fmaf(sm, u, b.x); sm = __builtin_fmaf(sm, u, a.w); sm = __builtin_fmaf(sm, u, a.z);
  sm = __builtin_fmaf(sm, u, a.y); sm = __builtin_fmaf(sm, u, a.x);
  return sm > 0.f ? c.w + __log2f(sm) : NAN;
}

// log2 of both mixture sides at t from a TPE_F_LOGPOLY row (include/tpe_hip.h,
// "Tabulated scoring"): {b_0, a_0, .., b_5, a_5}, degree-5 polynomials in u; NAN
// for a side outside the cells or flagged (b_0 / a_0 = NaN).  Cell centre and
// u as cell_log2_lds forms them.
__device__ __forceinline__ void lp_log2(float lo, float inv, float w, float ih, int n, const float4* __restrict__ rows,
                                        float t, float& lb2, float& la2) {
  const float gj = floorf((t - lo) * inv);
  const bool in = gj >= 0.f && gj < (float)n;
  const float4* __restrict__ r = rows + TPE_TAB_ROW_UNITS * (in ? (int)gj : 0);
  const float4 a = r[0], b = r[1], c = r[2];
  const float u = (t - __builtin_fmaf(gj + 0.5f, w, lo)) * ih;
  // the row interleaves the sides, {b_k, a_k} at 2k: both Horner sums as one
  // packed chain (v_pk_fma_f32 on register pairs, the same fma per side)
  const f2 uu = {u, u};
  f2 s = {c.z, c.w};
  s = __builtin_elementwise_fma(s, uu, f2{c.x, c.y});
  s = __builtin_elementwise_fma(s, uu, f2{b.z, b.w});
  s = __builtin_elementwise_fma(s, uu, f2{b.x, b.y});
  s = __builtin_elementwise_fma(s, uu, f2{a.z, a.w});
  s = __builtin_elementwise_fma(s, uu, f2{a.x, a.y});
  lb2 = in ? s.x : NAN;
  la2 = in ? s.y : NAN;
}

// PREC is a template parameter: with the f64 inverse-CDF path reachable, the
// candidate loop needs several times the registers
// f64 exp out of line: inlined, its polynomial's f64 constants were hoisted
// into VGPR pairs at k_sample_tab's start (no literal operands in VOP3) and
// pushed the cells loop into scratch spills
__device__ __noinline__ double exp_call(double x) { return exp(x); }
// (likewise the empty slot's constant, stored out of line)
__device__ __noinline__ void clear_best(tpe_best* d) { *d = tpe_best{0, 0, 0, -1}; }

// FAST: the production case only — f32 cells tables that fit in LDS, device
// draws from the staged sampler, early selection, no per-candidate outputs
// (the host sets tpe_batch.tab_fast when every tabulated problem of the level
// is one).  Its instantiation carries none of the other paths' registers, and
// a label's staging overlaps the first unit's Philox draws (the table rows are
// waited for only before the first cell look-up).
template <int PREC, bool FAST = false>
__global__ __launch_bounds__(kTabThreads) void k_sample_tab(const tpe_problem* __restrict__ P,
                                                            const tpe_tile* __restrict__ tiles,
                                                            const int32_t* __restrict__ list, int n_list,
                                                            int per_wg, const double* __restrict__ samp,
                                                            double* __restrict__ cand,
                                                            const float* __restrict__ coord,
                                                            tpe_best* __restrict__ tile_best,
                                                            double* __restrict__ l_out, double* __restrict__ g_out,
                                                            int draw, int flags,
                                                            const float4* __restrict__ comp32,
                                                            const float4* __restrict__ tab,
                                                            tpe_result* __restrict__ run_best, int tpp) {
  __shared__ float4 tab_lds[TPE_TAB_ROW_UNITS * kTabLdsCells];
  __shared__ double cum_lds[kCumLds];
  __shared__ float4 row_lds[kCumLds];     // {mu, +-sigma (sign = mirrored), Phi(a), Phi(b)} as f32
  __shared__ GuideEnt guide[kGuide];
  __shared__ tpe_best wb[kTabThreads / 64];
  const int lane = threadIdx.x & 63;
  [[maybe_unused]] const int wave = threadIdx.x >> 6;
  const bool need_x = l_out != nullptr || (flags & TPE_BATCH_WRITE_CAND);
  int cur = -1, run_tile = -1;            // problem of the run, first tile of its run
  // what the LDS holds: the sampler and table rows of a label (every problem
  // of a label shares them — a batched suggest's ids run through the same
  // label back to back, and each only flushes its own winner)
  int st_samp = -1, st_len = -1, st_t0 = -1, st_t1 = -1, st_n0 = -1, st_n1 = -1, st_mode = -1;
  bool in_lds = false, tab_in_lds = false;
  double bs = 0.0, bl = 0.0, bg = 0.0, bv = 0.0;
  int64_t bi = -1;
  // bv: the best candidate's draw — its kernel coordinate t for cells (the value
  // is t, or e^t for log families: draw_comp's f32 definition) or its value for
  // the lattice — so the run's winner needs no redraw
  auto emit = [&](int i, int64_t o, double x, double l, double g, double v) {
    if (l_out) { l_out[o] = l; g_out[o] = g; }
    if (flags & TPE_BATCH_WRITE_CAND) cand[o] = x;
    if (better(l - g, i, bs, bi)) { bs = l - g; bl = l; bg = g; bi = i; bv = v; }
  };
  // cells candidates: a thread keeps its best by d = log2 l~ - log2 g~ in f32
  // (the order of l - g up to f32 rounding of d: a near-tie inside the eps-tie
  // set), with the two log2 sums and the coordinate; l, g and the f64 score are
  // formed once per run (flush) — no f64 work per candidate
  float fd = 0.f, flb = 0.f, fla = 0.f, ft = 0.f;
  int fi = -1;
  auto track = [&](int i, float lb2, float la2, float t) {
    const float d = lb2 - la2;
    if (better32(d, i, fd, fi)) { fd = d; fi = i; flb = lb2; fla = la2; ft = t; }
  };
  // the run's problem fields the flush needs (no global reads at the run's end)
  int64_t run_cand_base = 0, run_cand_off = 0;
  double run_bb = 0.0, run_ab = 0.0;
  bool run_logc = false, run_exp = false, run_drawn = false, run_cells = false;
  // a run's record (one lane): l, g and the f64 score of its best -> slot 0 of
  // its first tile, or with early selection its best with the value (the draw
  // it kept — what the select stage's redraw would give) straight to
  // host-visible memory
  auto record_to = [&](int tile_r, int64_t cbase, int64_t coff, bool drawn, bool ex, double s2, double l2,
                       double g2, int64_t i2, double v2) {
    if (run_best) {
      tpe_result r;
      r.score = s2; r.l = l2; r.g = g2; r.idx = i2; r.value = 0.0;
      r.global_idx = i2 >= 0 ? cbase + i2 : -1;
      if (i2 >= 0) r.value = drawn ? (ex ? exp_call(v2) : v2) : cand[coff + i2];
      run_best[tile_r] = r;
    } else {
      tpe_best* __restrict__ d = tile_best + (int64_t)tile_r * TPE_BEST_PER_TILE;
      d->score = s2; d->l = l2; d->g = g2; d->idx = i2;
    }
  };
  auto record = [&](double s2, double l2, double g2, int64_t i2, double v2) {
    record_to(run_tile, run_cand_base, run_cand_off, run_drawn, run_exp, s2, l2, g2, i2, v2);
  };
  // cells runs are combined once, at the workgroup's end (no barrier per run:
  // a batched level's workgroup runs through up to kTabMaxTilesPerWg problems
  // and a per-run barrier exposed each run's slowest wave): each wave leaves
  // its best per run — key, log2 sums, coordinate — and the run's fields
  struct RunRec { int64_t cand_base, cand_off; double bb, ab; int tile, flags; };   // flags: 1 log, 2 exp, 4 drawn
  __shared__ RunRec s_run[kTabMaxTilesPerWg];
  __shared__ unsigned long long s_rk[kTabMaxTilesPerWg][kTabThreads / 64];
  __shared__ float s_rv[kTabMaxTilesPerWg][3][kTabThreads / 64];
  int n_def = 0;                          // cells runs deferred so far (workgroup-uniform)
  // the run's best -> its record (block reduction)
  auto flush = [&]() {
    // lane, wave and their LDS addresses formed here (hoisted to the kernel's
    // start they stayed live across the candidate loops and were spilled)
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wave = tid >> 6;
    if (FAST || run_cells) {
      // cells run: better32's order as one 64-bit key per lane, reduced by the
      // wave's DPP max (no LDS permutes); the winning lane (candidate indices are
      // unique) leaves its log2 sums and draw for the end-of-workgroup combine
      const unsigned long long key = key32(fd, fi);
      const unsigned long long wk = __ockl_wfred_max_u64(key);
      if (wk != 0ull && key == wk) { s_rv[n_def][0][wave] = flb; s_rv[n_def][1][wave] = fla; s_rv[n_def][2][wave] = ft; }
      if (lane == 0) s_rk[n_def][wave] = wk;
      ++n_def;
      fi = -1;
      return;
    }
    for (int off = 32; off > 0; off >>= 1) {
      const double os = __shfl_xor(bs, off), ol = __shfl_xor(bl, off), og = __shfl_xor(bg, off);
      const double ov = __shfl_xor(bv, off);
      const int64_t oi = __shfl_xor(bi, off);
      if (better(os, oi, bs, bi)) { bs = os; bl = ol; bg = og; bi = oi; bv = ov; }
    }
    __shared__ double wv[kTabThreads / 64];
    if (lane == 0) { wb[wave].score = bs; wb[wave].l = bl; wb[wave].g = bg; wb[wave].idx = bi; wv[wave] = bv; }
    __syncthreads();
    if (wave == 0) {                         // lanes 0..15 hold the waves' bests
      const int q = lane < kTabThreads / 64 ? lane : 0;
      double s2 = wb[q].score, l2 = wb[q].l, g2 = wb[q].g, v2 = wv[q];
      int64_t i2 = lane < kTabThreads / 64 ? wb[q].idx : -1;
      for (int off = 8; off > 0; off >>= 1) {
        const double os = __shfl_xor(s2, off), ol = __shfl_xor(l2, off), og = __shfl_xor(g2, off);
        const double ov = __shfl_xor(v2, off);
        const int64_t oi = __shfl_xor(i2, off);
        if (better(os, oi, s2, i2)) { s2 = os; l2 = ol; g2 = og; i2 = oi; v2 = ov; }
      }
      if (lane == 0) record(s2, l2, g2, i2, v2);
    }
    bs = 0.0; bl = 0.0; bg = 0.0; bv = 0.0; bi = -1;
  };
  // this workgroup's tile descriptors, fetched in one round
  __shared__ int s_tile[kTabMaxTilesPerWg], s_prob[kTabMaxTilesPerWg], s_start[kTabMaxTilesPerWg];
  __shared__ int s_unit[kTabMaxTilesPerWg];              // per run: units handed out (dynamic pairs)
  if ((int)threadIdx.x < kTabMaxTilesPerWg) s_unit[threadIdx.x] = 0;
  const int n_my = min(per_wg, n_list - (int)blockIdx.x * per_wg);
  if ((int)threadIdx.x < n_my) {
    const int li = (int)blockIdx.x * per_wg + (int)threadIdx.x;
    const int tile = list ? list[li] : li;
    s_tile[threadIdx.x] = tile;
    if (tpp > 0) {                      // uniform tiles: no descriptor round trip
      const int r = tile / tpp;
      s_prob[threadIdx.x] = r; s_start[threadIdx.x] = (tile - r * tpp) * kTile;
    } else {
      const tpe_tile tl = tiles[tile];
      s_prob[threadIdx.x] = tl.problem; s_start[threadIdx.x] = tl.cand_start;
    }
  }
  __syncthreads();
  if constexpr (FAST) {
    // ---- the production cells loop (see FAST above) ----
    // per unit of a thread: NP consecutive candidates from `first`; phases:
    // uniforms (Philox, no LDS) -> draws (guide, sampler row, ndtri_f32) ->
    // the two cell look-ups, with the exact fallback for the rare candidate
    // outside the cells or in a flagged cell
    for (int gi = 0; gi < n_my; ++gi) {
      const int tile = __builtin_amdgcn_readfirstlane(s_tile[gi]), pid = __builtin_amdgcn_readfirstlane(s_prob[gi]);
      const tpe_problem& p = P[pid];
      bool staged = false;
      double scum = 0.0;
      float4 srow = make_float4(0.f, 0.f, 0.f, 0.f);
      if (pid != cur) {
        if (cur >= 0) flush();
        const bool same = p.samp_off == st_samp && p.samp_len == st_len && p.tab_off[0] == st_t0 &&
                          p.tab_off[1] == st_t1 && p.tab_n[0] == st_n0 && p.tab_n[1] == st_n1;
        if (!same) {
          st_samp = p.samp_off; st_len = p.samp_len; st_t0 = p.tab_off[0]; st_t1 = p.tab_off[1];
          st_n0 = p.tab_n[0]; st_n1 = p.tab_n[1];
          __syncthreads();                               // LDS free for the next label's rows
          // sampler rows into registers first, then the table units by LDS-DMA:
          // every one of the kStageU rounds issued (units past the table: a
          // clamped load into unused slots), so the sampler rows' use below waits
          // for their own loads only, and the tables land while the first unit's
          // Philox draws are computed
          if ((int)threadIdx.x < p.samp_len) {
            const double* sr = samp + 8 * (int64_t)p.samp_off + 8 * (int)threadIdx.x;
            scum = sr[0];
            const float sg = (float)sr[2];
            srow = make_float4((float)sr[1], sr[5] != 0.0 ? -sg : sg, (float)sr[3], (float)sr[4]);
          }
          // (FAST: the label's one TPE_F_LOGPOLY table)
          constexpr int kStageU = TPE_TAB_ROW_UNITS * kTabLdsCells / kTabThreads;
          const int nu = TPE_TAB_ROW_UNITS * p.tab_n[0];
          const int wv = (int)(threadIdx.x >> 6);
#pragma unroll
          for (int u = 0; u < kStageU; ++u) {
            const int q = min(u * kTabThreads + (int)threadIdx.x, nu - 1);
            __builtin_amdgcn_global_load_lds((const void*)(tab + (int64_t)p.tab_off[0] + q),
                                             (__attribute__((address_space(3))) void*)(tab_lds + u * kTabThreads + 64 * wv),
                                             16, 0, 0);
          }
          staged = true;
        }
        cur = pid;
        run_tile = tile;
        run_cand_base = p.cand_base; run_cand_off = p.cand_off;
        run_bb = p.below_base; run_ab = p.above_base;
        run_logc = p.family == TPE_FAM_LOGGAUSS;
        run_exp = run_logc;
        run_drawn = true;
        run_cells = true;
        if (threadIdx.x == 0)
          s_run[n_def] = RunRec{run_cand_base, run_cand_off, run_bb, run_ab, run_tile, (run_logc ? 1 : 0) | (run_exp ? 2 : 0) | 4};
      }
      const int cand_start = __builtin_amdgcn_readfirstlane(s_start[gi]);
      const bool pair = gi + 1 < n_my && __builtin_amdgcn_readfirstlane(s_prob[gi + 1]) == pid &&
                        __builtin_amdgcn_readfirstlane(s_start[gi + 1]) == cand_start + kTile;
      // a run of several tile pairs: (pair, 64-thread slot) units handed out from
      // an LDS counter (waves that run ahead take more; see the general pass)
      int npairs = 0;
      if (pair) {
        int k = gi;
        while (k + 1 < n_my && __builtin_amdgcn_readfirstlane(s_prob[k + 1]) == pid &&
               __builtin_amdgcn_readfirstlane(s_start[k + 1]) == cand_start + (k + 1 - gi) * kTile)
          ++k;
        npairs = (k - gi + 1) / 2;
      }
      const bool dyn = npairs > 1;
      const int nunits = npairs * (kTabThreads / 64);
      float lo_f, hi_f;
      f32_bounds(p, lo_f, hi_f);
      const float lo0 = p.tab_lo[0], inv0 = p.tab_inv[0];
      const float w0 = 1.f / inv0, ih0 = 1.f / (0.5f * w0);
      const int n0 = p.tab_n[0];
      const float4* __restrict__ r0 = tab_lds;
      // the next unit of this wave: false when the run has none left (dynamic)
      int first = 0;
      auto next_unit = [&](bool initial) -> bool {
        if (!dyn) {
          if (!initial) return false;
          first = cand_start + (pair ? 2 * kTabPer : kTabPer) * (int)threadIdx.x;
          return true;
        }
        int u = 0;
        if (lane == 0) u = atomicAdd(&s_unit[n_def], 1);
        u = __builtin_amdgcn_readlane(u, 0);
        if (u >= nunits) return false;
        const int pr = u / (kTabThreads / 64), slot = u - pr * (kTabThreads / 64);
        first = __builtin_amdgcn_readfirstlane(s_start[gi + 2 * pr]) + 2 * kTabPer * (slot * 64 + lane);
        return true;
      };
      auto run_units = [&](auto NPC) {
        constexpr int NP = decltype(NPC)::value;
        // the first unit's uniforms are computed while the label's rows are on
        // their way (every wave has a first unit: a dynamic run has >= 2 pairs,
        // 32 units for 16 waves)
        bool first_unit = true;
        next_unit(true);
        for (;;) {
          uint32_t ws[NP];
          float uf[NP], tj[NP];
          {
            const uint64_t g0 = (uint64_t)p.cand_base + (uint64_t)first;
            if ((g0 & 1) == 0) {
#pragma unroll
              for (int j = 0; j < NP; j += 2) {
                const uint64_t blk = (g0 + (uint64_t)j) >> 1;
                const U4 r = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), p.ctr2, p.ctr3, p.key0, p.key1);
                ws[j] = r.x; uf[j] = u01f(r.y);
                ws[j + 1] = r.z; uf[j + 1] = u01f(r.w);
              }
            } else {
#pragma unroll
              for (int j = 0; j < NP; ++j) {
                const DrawU d = draw_uniforms(p, first + j, TPE_PREC_F32);
                ws[j] = d.ws; uf[j] = d.uf;
              }
            }
          }
          if (first_unit && staged) {
            if ((int)threadIdx.x < p.samp_len) { cum_lds[threadIdx.x] = scum; row_lds[threadIdx.x] = srow; }
            __syncthreads();
            if (threadIdx.x < kGuide) {                  // first k with cum_k > b / kGuide, its two steps
              const double v = (double)threadIdx.x / (double)kGuide;
              const int len = p.samp_len;
              int a = 0, b = len - 1;
              while (a < b) { const int m = (a + b) >> 1; if (v < cum_lds[m]) b = m; else a = m + 1; }
              GuideEnt e;
              e.k0 = a;
              e.never = 0u;
              e.t0 = guide_thresh(a < len - 1 ? cum_lds[a] : INFINITY, e.never, 1u);
              e.t1 = guide_thresh(a + 1 < len - 1 ? cum_lds[a + 1] : INFINITY, e.never, 2u);
              guide[threadIdx.x] = e;
            }
            __syncthreads();
          }
          {
            int kc[NP];
            unsigned more = 0;
#pragma unroll
            for (int j = 0; j < NP; ++j) {
              bool m;
              kc[j] = guided_comp(guide, ws[j], m);
              more |= (unsigned)m << j;
            }
            if (__ballot(more != 0u)) {                 // (rare: a guide slice with 2+ component edges)
#pragma unroll
              for (int j = 0; j < NP; ++j)
                if ((more >> j) & 1u) kc[j] = guided_more(cum_lds, p.samp_len, u01w(ws[j]), kc[j]);
            }
#pragma unroll
            for (int j = 0; j < NP; ++j) {
              const float4 sv = row_lds[kc[j]];
              const float pr = sv.z + uf[j] * (sv.w - sv.z);
              const float z = ndtri_f32(pr);
              const float xf = sv.x + sv.y * z;
              tj[j] = fminf(fmaxf(xf == xf ? xf : sv.x, lo_f), hi_f);
            }
          }
          if (first_unit && staged) {
            __builtin_amdgcn_s_waitcnt(0);               // (the LDS-DMA loads: vmcnt)
            __syncthreads();
          }
          first_unit = false;
          uint32_t exact = 0;
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            const int i = first + j;
            const float t = tj[j];
            float lb2, la2;
            lp_log2(lo0, inv0, w0, ih0, n0, r0, t, lb2, la2);
            const bool valid = i < p.n_cand, ok = lb2 == lb2 && la2 == la2;
            exact |= (unsigned)(valid && !ok) << j;
            if (valid && ok) track(i, lb2, la2, t);
          }
          // outside the cells or in flagged ones: summed exactly by the whole wave
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            unsigned long long need = __ballot((exact >> j) & 1u);
            while (need) {
              const int src = __builtin_ctzll(need);
              need &= need - 1;
              const float t = __shfl(tj[j], src);
              float lb2, la2;
              lp_log2(lo0, inv0, w0, ih0, n0, r0, t, lb2, la2);
              if (!(lb2 == lb2)) lb2 = lse2_wave(comp32, p.below_off, p.below_len, 0, 0, t);
              if (!(la2 == la2)) la2 = lse2_wave(comp32, p.above_off, p.above_len, p.wide_off, p.wide_len, t);
              if (lane == src) track(first + j, lb2, la2, t);
            }
          }
          if (!next_unit(false)) break;
        }
      };
      if (pair) run_units(std::integral_constant<int, 2 * kTabPer>{});
      else run_units(std::integral_constant<int, kTabPer>{});
      gi += dyn ? 2 * npairs - 1 : (pair ? 1 : 0);     // the run's other tiles are done
    }
  }
  for (int gi = 0; gi < n_my && !FAST; ++gi) {
    // (uniform: readfirstlane keeps the problem's fields in scalar registers)
    const int tile = __builtin_amdgcn_readfirstlane(s_tile[gi]), pid = __builtin_amdgcn_readfirstlane(s_prob[gi]);
    const tpe_problem& p = P[pid];
    if (p.tab_mode == TPE_TAB_NONE) continue;        // no list: every tile, k_sample's skipped
    const bool cells = p.tab_mode == TPE_TAB_CELLS;
    if (pid != cur) {
      if (cur >= 0) flush();
      const bool same = p.samp_off == st_samp && p.samp_len == st_len && p.tab_off[0] == st_t0 &&
                        p.tab_off[1] == st_t1 && p.tab_n[0] == st_n0 && p.tab_n[1] == st_n1 && p.tab_mode == st_mode;
      if (!same) {
        st_samp = p.samp_off; st_len = p.samp_len; st_t0 = p.tab_off[0]; st_t1 = p.tab_off[1];
        st_n0 = p.tab_n[0]; st_n1 = p.tab_n[1]; st_mode = p.tab_mode;
        __syncthreads();                               // LDS free for the next label's rows
        const double* S = samp + 8 * (int64_t)p.samp_off;
        in_lds = draw && p.samp_len > 0 && p.samp_len <= kCumLds;
        const bool lpt = (p.flags & TPE_F_LOGPOLY) != 0;       // (one table for both sides)
        tab_in_lds = PREC == TPE_PREC_F32 && cells && (lpt ? p.tab_n[0] : p.tab_n[0] + p.tab_n[1]) <= kTabLdsCells;
        // the table units straight from global memory into LDS (LDS-DMA: no
        // registers, no store instructions; row-major, unit q at tab_lds[q] —
        // a wave's 64 consecutive units land at consecutive 16-B slots), the
        // sampler rows of threads below samp_len through registers; one round
        // of memory latency for all of it
        constexpr int kStageU = TPE_TAB_ROW_UNITS * kTabLdsCells / kTabThreads;
        static_assert(kCumLds <= kTabThreads, "one sampler row per thread");
        if (tab_in_lds) {
          const int n0 = TPE_TAB_ROW_UNITS * p.tab_n[0], nu = lpt ? n0 : n0 + TPE_TAB_ROW_UNITS * p.tab_n[1];
          const int wv = (int)(threadIdx.x >> 6);
#pragma unroll
          for (int u = 0; u < kStageU; ++u) {
            if (u * kTabThreads >= nu) break;          // (uniform; units past nu: a clamped load, unused slots)
            const int q = min(u * kTabThreads + (int)threadIdx.x, nu - 1);
            const float4* src = q < n0 ? tab + (int64_t)p.tab_off[0] + q : tab + (int64_t)p.tab_off[1] + (q - n0);
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(tab_lds + u * kTabThreads + 64 * wv),
                                             16, 0, 0);
          }
        }
        if (in_lds && (int)threadIdx.x < p.samp_len) {
          const double* sr = S + 8 * (int)threadIdx.x;
          cum_lds[threadIdx.x] = sr[0];
          const float sg = (float)sr[2];
          row_lds[threadIdx.x] = make_float4((float)sr[1], sr[5] != 0.0 ? -sg : sg, (float)sr[3], (float)sr[4]);
        }
        __builtin_amdgcn_s_waitcnt(0);                 // (the LDS-DMA loads: vmcnt)
        __syncthreads();
        if (in_lds && threadIdx.x < kGuide) {          // first k with cum_k > b / kGuide, its two steps
          const double v = (double)threadIdx.x / (double)kGuide;
          const int len = p.samp_len;
          int a = 0, b = len - 1;
          while (a < b) { const int m = (a + b) >> 1; if (v < cum_lds[m]) b = m; else a = m + 1; }
          GuideEnt e;
          e.k0 = a;
          e.never = 0u;
          e.t0 = guide_thresh(a < len - 1 ? cum_lds[a] : INFINITY, e.never, 1u);
          e.t1 = guide_thresh(a + 1 < len - 1 ? cum_lds[a + 1] : INFINITY, e.never, 2u);
          guide[threadIdx.x] = e;
        }
        __syncthreads();
      }
      cur = pid;
      run_tile = tile;
      run_cand_base = p.cand_base; run_cand_off = p.cand_off;
      run_bb = p.below_base; run_ab = p.above_base;
      run_logc = p.family == TPE_FAM_LOGGAUSS;
      run_exp = cells && run_logc;
      run_drawn = draw && p.samp_len > 0;
      run_cells = PREC == TPE_PREC_F32 && cells;
      if (run_cells && threadIdx.x == 0)
        s_run[n_def] = RunRec{run_cand_base, run_cand_off, run_bb, run_ab, run_tile,
                              (run_logc ? 1 : 0) | (run_exp ? 2 : 0) | (run_drawn ? 4 : 0)};
    }
    const int cand_start = __builtin_amdgcn_readfirstlane(s_start[gi]);
    // cells: the next listed tile continuing this one is taken along (4
    // candidates per thread in flight instead of 2: more independent chains to
    // hide the LDS and transcendental latencies of one candidate)
    const bool pair = PREC == TPE_PREC_F32 && cells && gi + 1 < n_my &&
                      __builtin_amdgcn_readfirstlane(s_prob[gi + 1]) == pid &&
                      __builtin_amdgcn_readfirstlane(s_start[gi + 1]) == cand_start + kTile;
    if (!run_best && threadIdx.x < TPE_BEST_PER_TILE) {   // (early selection: runs report to run_best)
      clear_best(tile_best + (int64_t)tile * TPE_BEST_PER_TILE + threadIdx.x);
      if (pair) clear_best(tile_best + (int64_t)s_tile[gi + 1] * TPE_BEST_PER_TILE + threadIdx.x);
    }
    float lo_f, hi_f;
    f32_bounds(p, lo_f, hi_f);
    const double* S = samp + 8 * (int64_t)p.samp_off;
    const bool logc = p.family == TPE_FAM_LOGGAUSS;
    // a thread's candidates are consecutive: an f32 Philox block serves two of them
    int first = cand_start + (pair ? 2 * kTabPer : kTabPer) * (int)threadIdx.x;
    int adv = pair ? 1 : 0;                          // tiles done beyond this one
    uint32_t exact = 0;                              // candidates the cell tables do not cover (rare)
    float tj[2 * kTabPer];
    // cells; TL: the tables are in LDS (separate instantiations, so every table
    // read is a plain LDS or global load, never a generic one); NPC: candidates
    // per thread (kTabPer, or 2 kTabPer for a tile pair)
    // FASTC: the production case (tables in LDS, device draws from the staged
    // sampler, no per-candidate outputs) in phases without branches — every
    // candidate's guide lookup, then its sampler row and inverse CDF, then its
    // two cell rows — so the thread's candidates' LDS reads overlap
    auto cells_pass = [&](auto TL, auto NPC, auto FASTC) {
        constexpr int NP = decltype(NPC)::value;
        constexpr bool kFast = decltype(FASTC)::value;
        const float lo0 = p.tab_lo[0], inv0 = p.tab_inv[0], lo1 = p.tab_lo[1], inv1 = p.tab_inv[1];
        const float w0 = 1.f / inv0, w1 = 1.f / inv1, ih0 = 1.f / (0.5f * w0), ih1 = 1.f / (0.5f * w1);
        const int n0 = p.tab_n[0], n1 = p.tab_n[1];
        const bool lpt = (p.flags & TPE_F_LOGPOLY) != 0;
        // both sides' log2 sums at t: a TPE_F_LOGPOLY row, or one moment row per side
        auto sides_nb = [&](const float4* __restrict__ a0, const float4* __restrict__ a1, float t, float& lb2,
                            float& la2) {
          if (lpt) { lp_log2(lo0, inv0, w0, ih0, n0, a0, t, lb2, la2); return; }
          lb2 = cell_log2_nb(lo0, inv0, w0, ih0, n0, a0, 1, TPE_TAB_ROW_UNITS, t);
          la2 = cell_log2_nb(lo1, inv1, w1, ih1, n1, a1, 1, TPE_TAB_ROW_UNITS, t);
        };
        auto sides = [&](const float4* __restrict__ a0, const float4* __restrict__ a1, float t, float& lb2,
                         float& la2) {
          if (lpt) { lp_log2(lo0, inv0, w0, ih0, n0, a0, t, lb2, la2); return; }
          lb2 = cell_log2_lds(lo0, inv0, w0, ih0, n0, a0, 1, TPE_TAB_ROW_UNITS, t);
          la2 = cell_log2_lds(lo1, inv1, w1, ih1, n1, a1, 1, TPE_TAB_ROW_UNITS, t);
        };
        constexpr bool kL = decltype(TL)::value;              // (rows row-major in LDS and global memory)
        const float4* __restrict__ r0;
        const float4* __restrict__ r1;
        if constexpr (kL) { r0 = tab_lds; r1 = tab_lds + TPE_TAB_ROW_UNITS * n0; }
        else { r0 = tab + p.tab_off[0]; r1 = tab + p.tab_off[1]; }
        // the pair's uniforms (draw_uniforms' f32 definition): one Philox block
        // per two candidates when the first one's global index is even
        DrawU du[NP];
        if (draw && in_lds) {
          const uint64_t g0 = (uint64_t)p.cand_base + (uint64_t)first;
          if ((g0 & 1) == 0) {
#pragma unroll
            for (int j = 0; j < NP; j += 2) {
              const uint64_t blk = (g0 + (uint64_t)j) >> 1;
              const U4 r = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), p.ctr2, p.ctr3, p.key0, p.key1);
              du[j] = DrawU{0.0, u01f(r.y), 0.0, r.x};
              du[j + 1] = DrawU{0.0, u01f(r.w), 0.0, r.z};
            }
          } else {
#pragma unroll
            for (int j = 0; j < NP; ++j) du[j] = draw_uniforms(p, first + j, TPE_PREC_F32);
          }
        }
        if constexpr (kFast) {
          static_assert(kL, "the fast cells pass reads LDS tables");
          int kc[NP];
          unsigned more = 0;
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            bool m;
            kc[j] = guided_comp(guide, du[j].ws, m);
            more |= (unsigned)m << j;
          }
          if (__ballot(more != 0u)) {                 // (rare: a guide slice with 2+ component edges)
#pragma unroll
            for (int j = 0; j < NP; ++j)
              if ((more >> j) & 1u) kc[j] = guided_more(cum_lds, p.samp_len, u01w(du[j].ws), kc[j]);
          }
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            const float4 s = row_lds[kc[j]];
            const float pr = s.z + du[j].uf * (s.w - s.z);
            const float z = ndtri_f32(pr);
            const float xf = s.x + s.y * z;
            tj[j] = fminf(fmaxf(xf == xf ? xf : s.x, lo_f), hi_f);
          }
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            const int i = first + j;
            const float t = tj[j];
            float lb2, la2;
            sides_nb(r0, r1, t, lb2, la2);
            const bool valid = i < p.n_cand, ok = lb2 == lb2 && la2 == la2;
            exact |= (unsigned)(valid && !ok) << j;
            if (valid && ok) track(i, lb2, la2, t);
          }
        }
#pragma unroll
        for (int j = 0; j < NP && !kFast; ++j) {
          const int i = first + j;
          tj[j] = NAN;
          if (i >= p.n_cand) continue;
          const int64_t o = p.cand_off + i;
          float t;
          if (!draw) {
            t = coord[o];
          } else if (in_lds) {
            bool more;
            int a = guided_comp(guide, du[j].ws, more);
            if (more) a = guided_more(cum_lds, p.samp_len, u01w(du[j].ws), a);
            const float4 s = row_lds[a];
            const float pr = s.z + du[j].uf * (s.w - s.z);
            const float z = ndtri_f32(pr);
            float xf = s.x + s.y * z;
            if (!(xf == xf)) xf = s.x;
            t = fminf(fmaxf(xf, lo_f), hi_f);
          } else if (p.samp_len > 0) {
            t = draw_coord_f32(p, S, S, 8, i, lo_f, hi_f);
          } else {
            t = NAN;
          }
          tj[j] = t;
          float lb2, la2;
          sides(r0, r1, t, lb2, la2);
          if (!(lb2 == lb2) || !(la2 == la2)) { exact |= 1u << j; continue; }
          track(i, lb2, la2, t);
          if (need_x) {                          // per-candidate outputs on request (tests)
            const double lnx = logc ? (double)t : 0.0;
            const double x = !draw ? cand[o] : logc ? exp_call((double)t) : (double)t;
            if (l_out) { l_out[o] = (double)lb2 * kLn2 + p.below_base - lnx; g_out[o] = (double)la2 * kLn2 + p.above_base - lnx; }
            if (flags & TPE_BATCH_WRITE_CAND) cand[o] = x;
          }
        }
        // candidates outside the cells or in flagged ones: summed exactly by the
        // whole wave, one candidate at a time
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          unsigned long long need = __ballot((exact >> j) & 1u);
          while (need) {
            const int src = __builtin_ctzll(need);
            need &= need - 1;
            const float t = __shfl(tj[j], src);
            float lb2, la2;
            sides(r0, r1, t, lb2, la2);
            if (!(lb2 == lb2)) lb2 = lse2_wave(comp32, p.below_off, p.below_len, 0, 0, t);
            if (!(la2 == la2)) la2 = lse2_wave(comp32, p.above_off, p.above_len, p.wide_off, p.wide_len, t);
            if (lane == src) {
              const int i = first + j;
              const int64_t o = p.cand_off + i;
              track(i, lb2, la2, t);
              if (need_x) {
                const double lnx = logc ? (double)t : 0.0;
                const double x = !draw ? cand[o] : logc ? exp_call((double)t) : (double)t;
                if (l_out) { l_out[o] = (double)lb2 * kLn2 + p.below_base - lnx; g_out[o] = (double)la2 * kLn2 + p.above_base - lnx; }
                if (flags & TPE_BATCH_WRITE_CAND) cand[o] = x;
              }
            }
          }
        }
    };
    if constexpr (PREC == TPE_PREC_F32) {
      if (cells) {
        using P2 = std::integral_constant<int, kTabPer>;
        using P4 = std::integral_constant<int, 2 * kTabPer>;
        using T = std::true_type;
        using F = std::false_type;
        if (tab_in_lds && draw && in_lds && !need_x) {
          // a run of several tile pairs (early selection): its pairs handed out
          // to the waves in units of (pair, 64-thread slot) from an LDS counter,
          // so waves that run ahead take more units and the run ends near the
          // waves' mean instead of their slowest (a thread's best carries over
          // units: the run's combine reduces every thread, whatever it drew)
          int npairs = 0;
          if (pair && run_best) {
            int k = gi;
            while (k + 1 < n_my && __builtin_amdgcn_readfirstlane(s_prob[k + 1]) == pid &&
                   __builtin_amdgcn_readfirstlane(s_start[k + 1]) == cand_start + (k + 1 - gi) * kTile)
              ++k;
            npairs = (k - gi + 1) / 2;
          }
          if (npairs > 1) {
            const int nu = npairs * (kTabThreads / 64);
            for (;;) {
              int u = 0;
              if (lane == 0) u = atomicAdd(&s_unit[n_def], 1);
              u = __builtin_amdgcn_readlane(u, 0);
              if (u >= nu) break;
              const int pr = u / (kTabThreads / 64), slot = u - pr * (kTabThreads / 64);
              first = __builtin_amdgcn_readfirstlane(s_start[gi + 2 * pr]) + 2 * kTabPer * (slot * 64 + lane);
              exact = 0;
              cells_pass(T{}, P4{}, T{});
            }
            adv = 2 * npairs - 1;
          } else if (pair) cells_pass(T{}, P4{}, T{}); else cells_pass(T{}, P2{}, T{});
        }
        else
        if (tab_in_lds) { if (pair) cells_pass(T{}, P4{}, F{}); else cells_pass(T{}, P2{}, F{}); }
        else { if (pair) cells_pass(F{}, P4{}, F{}); else cells_pass(F{}, P2{}, F{}); }
      }
    }
    gi += adv;                                       // the pair's (the run's pairs') other tiles are done
    if (!cells && PREC == TPE_PREC_F32 && draw && in_lds) {
      // lattice, f32 draws: drawn as the cells path draws (draw_uniforms' pairs,
      // the staged sampler rows, ndtri_f32), quantised as draw_comp quantises
      // (np.round(x / q) * q), the lattice row of that multiple looked up
      DrawU du[kTabPer];
      const uint64_t g0 = (uint64_t)p.cand_base + (uint64_t)first;
      if ((g0 & 1) == 0) {
#pragma unroll
        for (int j = 0; j < kTabPer; j += 2) {
          const uint64_t blk = (g0 + (uint64_t)j) >> 1;
          const U4 r = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), p.ctr2, p.ctr3, p.key0, p.key1);
          du[j] = DrawU{0.0, u01f(r.y), 0.0, r.x};
          du[j + 1] = DrawU{0.0, u01f(r.w), 0.0, r.z};
        }
      } else {
#pragma unroll
        for (int j = 0; j < kTabPer; ++j) du[j] = draw_uniforms(p, first + j, TPE_PREC_F32);
      }
      const bool lg = p.family == TPE_FAM_QLOGGAUSS;
      const double2* __restrict__ lat = reinterpret_cast<const double2*>(tab) + p.tab_off[0];
#pragma unroll
      for (int j = 0; j < kTabPer; ++j) {
        const int i = first + j;
        if (i >= p.n_cand) break;
        bool more;
        int a = guided_comp(guide, du[j].ws, more);
        if (more) a = guided_more(cum_lds, p.samp_len, u01w(du[j].ws), a);
        const float4 sr = row_lds[a];
        const float pr = sr.z + du[j].uf * (sr.w - sr.z);
        const float z = ndtri_f32(pr);
        float xf = sr.x + sr.y * z;
        if (!(xf == xf)) xf = sr.x;
        const float t = fminf(fmaxf(xf, lo_f), hi_f);
        const double xu = lg ? exp((double)t) : (double)t;
        const double mq = rint(xu / p.q);
        const double x = mq * p.q;
        const double jq = mq - (double)p.lat_lo;
        double l = -INFINITY, g = 0.0;             // (outside the lattice: unreachable for device draws)
        if (jq >= 0.0 && jq < (double)p.tab_n[0]) {
          const double2 r = lat[(int64_t)jq];
          l = r.x;
          g = r.y;
        }
        emit(i, p.cand_off + i, x, l, g, x);
      }
    } else if (!cells) {                             // lattice: exact {l, g} per quantized value
      for (int j = 0; j < kTabPer; ++j) {
        const int i = first + j;
        if (i >= p.n_cand) break;
        const int64_t o = p.cand_off + i;
        double x, l, g;
        float t;
        if (!draw) {
          x = cand[o];
        } else if (p.samp_len > 0) {
          int c;
          if (in_lds) draw_one(p, S, cum_lds, 1, i, PREC, lo_f, hi_f, x, t, c);
          else draw_one(p, S, S, 8, i, PREC, lo_f, hi_f, x, t, c);
        } else {
          x = NAN;
        }
        const double mq = rint(x / p.q);
        const double jq = mq - (double)p.lat_lo;
        if (mq * p.q == x && jq >= 0.0 && jq < (double)p.tab_n[0]) {
          const double2 r = reinterpret_cast<const double2*>(tab)[p.tab_off[0] + (int64_t)jq];
          l = r.x;
          g = r.y;
        } else {
          // unreachable for device draws (the lattice spans every value they can
          // take; caller-drawn candidates disable the table, TPE_F_NO_TABLE): the
          // candidate drops out (an f64 mass sum here would triple this
          // kernel's registers)
          l = -INFINITY;
          g = 0.0;
        }
        emit(i, o, x, l, g, x);
      }
    }
  }
  if (cur >= 0) flush();
  if (n_def > 0) {                       // the deferred cells runs: wave r combines run r
    __syncthreads();
    for (int r = wave; r < n_def; r += kTabThreads / 64) {
      const unsigned long long k2 = lane < kTabThreads / 64 ? s_rk[r][lane] : 0ull;
      const unsigned long long bk = __ockl_wfred_max_u64(k2);
      const unsigned long long m2 = __ballot(bk != 0ull && k2 == bk);
      const int w2 = m2 ? (int)__builtin_ctzll(m2) : 0;
      const int i2 = bk != 0ull ? (int)~(uint32_t)bk : -1;
      if (lane == 0) {
        const RunRec rr = s_run[r];
        double s2 = 0.0, l2 = 0.0, g2 = 0.0, v2 = 0.0;
        if (i2 >= 0) {
          const float t = s_rv[r][2][w2];
          const double lnx = (rr.flags & 1) ? (double)t : 0.0;
          l2 = (double)s_rv[r][0][w2] * kLn2 + rr.bb - lnx;
          g2 = (double)s_rv[r][1][w2] * kLn2 + rr.ab - lnx;
          s2 = l2 - g2;
          v2 = (double)t;
        }
        record_to(rr.tile, rr.cand_base, rr.cand_off, (rr.flags & 4) != 0, (rr.flags & 2) != 0, s2, l2, g2,
                  (int64_t)i2, v2);
      }
    }
  }
}

// ---- the fast sample kernel, small-workgroup form (k_sample_fast) ----
// The production sample pass of tabulated levels whose labels are TPE_F_LOGPOLY
// cells tables or lattices (device draws at f32, early selection, nothing per
// candidate written), in 512-thread workgroups whose LDS takes only the level's
// largest table (dynamic shared memory, tpe_batch.tab_fast - 1 units of 16 B)
// and whose sampler rows are at most kFastSamp: three workgroups share a CU,
// 24 waves instead of 16, and a workgroup's staging and barriers overlap the
// others' candidate loops.  A thread's unit is NP candidates (NP / 2 Philox
// blocks); a run's units (its consecutive tiles of one problem) are handed to
// the waves statically (wave w: units w, w + 8, ..) or, when its tiles are not
// one candidate range, from an LDS counter.  Cells: the same draws, the same f32
// arithmetic and the same selection order as k_sample_tab's cells passes.
// Lattice (quantized labels): drawn alike, quantised as draw_comp quantises
// (np.round(x / q) * q, after exp for the log family), scored by the value's
// exact f64 {l, g} row; a candidate's f64 score l - g enters the run's argmax
// through its rank among the lattice's scores (lattice_ranks: the same order
// as better() on the f64 scores, so the winner is k_sample_tab's), and the run
// record carries the f64 l, g and score.  LG (debug builds of the stage,
// tpe_debug_fast_lg): every candidate's {value, l, g, label} written besides.
constexpr int kFastThreads = 512;
constexpr int kFastSamp = 64;                  // sampler rows (below components) in LDS
constexpr int kFastWgsPerCu = 3;
constexpr int kFastMaxCells = 896;             // 42 KiB of table rows: three workgroups' LDS in a CU
constexpr int kFastMaxUnits = TPE_TAB_ROW_UNITS * kFastMaxCells;   // 16-B LDS units of the staged table
constexpr int kFastLatMax = 1024;              // lattice values the pass ranks in LDS
// LDS units (16 B) a lattice of n values takes: its {l, g} rows and n + 1 f32
// entry thresholds (the table's, lat_thresh_units), then an int rank per value
__host__ __device__ constexpr int lat_thresh_units(int n) { return (n + 1 + 3) / 4; }
__host__ __device__ constexpr int fast_lat_units(int n) { return n + lat_thresh_units(n) + (n + 3) / 4; }

// rank of each lattice value's score s_j = l_j - g_j, in better()'s order on
// f64 scores: NaN above every number; else #{k : s_k < s_j} + [s_j > -inf] —
// 0 for -inf, the score of a draw outside the lattice (l = -inf, g = 0) — so
// equal scores share a rank and a larger score has a larger one (workgroup-
// collective; O(n) LDS reads per value)
__device__ void lattice_ranks(const double2* __restrict__ rows, int n, int* __restrict__ rank) {
  for (int j = threadIdx.x; j < n; j += kFastThreads) {
    const double2 r = rows[j];
    const double s = r.x - r.y;
    int k = n + 2;
    if (s == s) {
      k = s > -INFINITY ? 1 : 0;
      for (int m = 0; m < n; ++m) {
        const double2 o = rows[m];
        k += (o.x - o.y) < s;
      }
    }
    rank[j] = k;
  }
}

// NP = 2: 80 VGPRs, six waves a SIMD (three workgroups a CU: batched levels);
// NP = 4: two candidate pairs in flight per lane for levels of at most two
// workgroups a CU (config 3's 2^21 candidates), four waves a SIMD
template <int NP, bool LG>
__global__ __launch_bounds__(kFastThreads) __attribute__((amdgpu_waves_per_eu(NP == 2 ? 6 : 4)))
void k_sample_fast(const tpe_problem* __restrict__ P, const tpe_tile* __restrict__ tiles,
                   const int32_t* __restrict__ list, int n_list, int per_wg, const double* __restrict__ samp,
                   const float4* __restrict__ comp32, const float4* __restrict__ tab,
                   tpe_result* __restrict__ run_best, int tpp, double* __restrict__ lg_out) {
  constexpr int kFastUnit = 64 * NP;
  static_assert(NP % 2 == 0 && kTile % kFastUnit == 0, "fast units: Philox pairs tiling the tiles");
  extern __shared__ float4 fast_tab[];                       // the label's table (tab_fast - 1 units at most)
  __shared__ double cum_lds[kFastSamp];
  __shared__ float4 row_lds[kFastSamp];
  __shared__ GuideEnt guide[kGuide];
  constexpr int kW = kFastThreads / 64;
  struct RunRec { int64_t cand_base, lat_lo; double bb, ab, q; int tile, logc, lat, tab_off; };
  __shared__ RunRec s_run[kTabMaxTilesPerWg];
  __shared__ unsigned long long s_rk[kTabMaxTilesPerWg][kW];
  __shared__ float s_rv[kTabMaxTilesPerWg][3][kW];
  __shared__ int s_tile[kTabMaxTilesPerWg], s_prob[kTabMaxTilesPerWg], s_start[kTabMaxTilesPerWg];
  __shared__ int s_unit[kTabMaxTilesPerWg];
  const int lane = threadIdx.x & 63;
  int st_samp = -1, st_len = -1, st_t0 = -1, st_n0 = -1;
  int n_def = 0;                                             // runs so far (workgroup-uniform)
  // the thread's best: cells — score fd (better32 order), index fi, log2 sums
  // flb / fla, draw ft; lattice — index fi, score rank and row (-1: outside the
  // lattice) as the bits of flb and fla, draw ft
  float fd = 0.f, flb = 0.f, fla = 0.f, ft = 0.f;
  int fi = -1;
  if ((int)threadIdx.x < kTabMaxTilesPerWg) s_unit[threadIdx.x] = 0;
  const int n_my = min(per_wg, n_list - (int)blockIdx.x * per_wg);
  if ((int)threadIdx.x < n_my) {
    const int li = (int)blockIdx.x * per_wg + (int)threadIdx.x;
    const int tile = list ? list[li] : li;
    s_tile[threadIdx.x] = tile;
    if (tpp > 0) {
      const int r = tile / tpp;
      s_prob[threadIdx.x] = r; s_start[threadIdx.x] = (tile - r * tpp) * kTile;
    } else {
      const tpe_tile tl = tiles[tile];
      s_prob[threadIdx.x] = tl.problem; s_start[threadIdx.x] = tl.cand_start;
    }
  }
  __syncthreads();
  for (int gi = 0; gi < n_my;) {
    const int tile = __builtin_amdgcn_readfirstlane(s_tile[gi]), pid = __builtin_amdgcn_readfirstlane(s_prob[gi]);
    int gk = gi;                                             // the run: tiles gi .. gk, one problem
    while (gk + 1 < n_my && __builtin_amdgcn_readfirstlane(s_prob[gk + 1]) == pid) ++gk;
    const tpe_problem& p = P[pid];
    const bool lat = p.tab_mode == TPE_TAB_LATTICE;         // (run-uniform)
    const int n0 = p.tab_n[0];
    bool staged = false;
    double scum = 0.0;
    float4 srow = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool same = p.samp_off == st_samp && p.samp_len == st_len && p.tab_off[0] == st_t0 && n0 == st_n0;
    if (!same) {
      st_samp = p.samp_off; st_len = p.samp_len; st_t0 = p.tab_off[0]; st_n0 = n0;
      __syncthreads();                                       // LDS free for the next label's rows
      if ((int)threadIdx.x < p.samp_len) {
        const double* sr = samp + 8 * (int64_t)p.samp_off + 8 * (int)threadIdx.x;
        scum = sr[0];
        const float sg = (float)sr[2];
        srow = make_float4((float)sr[1], sr[5] != 0.0 ? -sg : sg, (float)sr[3], (float)sr[4]);
      }
      // the table rows (cells: 3 units a row; lattice: one {l, g} unit a value) by
      // LDS-DMA, every round's loads issued before the one wait; the last round's
      // lanes past the rows issue nothing (an LDS-DMA lane writes its slot
      // whatever its address: the dynamic LDS holds exactly the rows)
      const int nu = lat ? n0 + lat_thresh_units(n0) : TPE_TAB_ROW_UNITS * n0;
      const int wv = (int)(threadIdx.x >> 6);
      for (int u = 0; u * kFastThreads < nu; ++u) {
        const int q = u * kFastThreads + (int)threadIdx.x;
        if (q < nu)
          __builtin_amdgcn_global_load_lds((const void*)(tab + (int64_t)p.tab_off[0] + q),
                                           (__attribute__((address_space(3))) void*)(fast_tab + u * kFastThreads + 64 * wv),
                                           16, 0, 0);
      }
      staged = true;
    }
    if (threadIdx.x == 0) {
      const bool lgf = p.family == TPE_FAM_LOGGAUSS || p.family == TPE_FAM_QLOGGAUSS;
      s_run[n_def] = RunRec{(int64_t)p.cand_base, p.lat_lo, p.below_base, p.above_base, p.q, tile, lgf ? 1 : 0,
                            lat ? 1 : 0, p.tab_off[0]};
    }
    const int nunits = (gk - gi + 1) * (kTile / kFastUnit);
    float lo_f, hi_f;
    f32_bounds(p, lo_f, hi_f);
    const float lo0 = p.tab_lo[0], inv0 = p.tab_inv[0];
    const float w0 = 1.f / inv0, ih0 = 1.f / (0.5f * w0);
    const double2* __restrict__ lrow = reinterpret_cast<const double2*>(fast_tab);
    const float* __restrict__ lthr = reinterpret_cast<const float*>(fast_tab + n0);
    const int* __restrict__ lrank = reinterpret_cast<const int*>(fast_tab + n0 + lat_thresh_units(n0));
    // a run whose tiles are one candidate range (the packer's order): wave w takes
    // units w, w + kW, ... with no LDS traffic for the hand-out or the addresses
    const int start0 = __builtin_amdgcn_readfirstlane(s_start[gi]);
    const int ntl = gk - gi + 1;
    const int tl = min(lane, ntl - 1);
    const bool contig = __ballot(s_start[gi + tl] != start0 + tl * kTile) == 0ull;
    const int wave0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    bool first_unit = true;
    for (int k = 0;; ++k) {
      int u = wave0 + k * kW;
      if (!contig) {
        int v = 0;
        if (lane == 0) v = atomicAdd(&s_unit[n_def], 1);
        u = __builtin_amdgcn_readlane(v, 0);
      }
      // (a wave without a unit still takes part in the staging barriers below)
      const bool have = u < nunits;
      constexpr int kUnitsPerTile = kTile / kFastUnit;
      const int ut = have ? u / kUnitsPerTile : 0;
      const int first = (contig ? start0 + ut * kTile : __builtin_amdgcn_readfirstlane(s_start[gi + ut])) +
                        kFastUnit * (u - ut * kUnitsPerTile) + NP * lane;
      uint32_t ws[NP];
      float uf[NP], tj[NP];
      if (have) {
        const uint64_t g0 = (uint64_t)p.cand_base + (uint64_t)first;
        if ((g0 & 1) == 0) {
#pragma unroll
          for (int j = 0; j < NP; j += 2) {
            const uint64_t blk = (g0 + (uint64_t)j) >> 1;
            const U4 r = philox4x32_10((uint32_t)blk, (uint32_t)(blk >> 32), p.ctr2, p.ctr3, p.key0, p.key1);
            ws[j] = r.x; uf[j] = u01f(r.y);
            ws[j + 1] = r.z; uf[j + 1] = u01f(r.w);
          }
        } else {
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            const DrawU d = draw_uniforms(p, first + j, TPE_PREC_F32);
            ws[j] = d.ws; uf[j] = d.uf;
          }
        }
      }
      if (first_unit && staged) {
        if ((int)threadIdx.x < p.samp_len) { cum_lds[threadIdx.x] = scum; row_lds[threadIdx.x] = srow; }
        __syncthreads();
        if (threadIdx.x < kGuide) {                  // first k with cum_k > b / kGuide, its two steps
          const double v = (double)threadIdx.x / (double)kGuide;
          const int len = p.samp_len;
          int a = 0, b = len - 1;
          while (a < b) { const int m = (a + b) >> 1; if (v < cum_lds[m]) b = m; else a = m + 1; }
          GuideEnt e;
          e.k0 = a;
          e.never = 0u;
          e.t0 = guide_thresh(a < len - 1 ? cum_lds[a] : INFINITY, e.never, 1u);
          e.t1 = guide_thresh(a + 1 < len - 1 ? cum_lds[a + 1] : INFINITY, e.never, 2u);
          guide[threadIdx.x] = e;
        }
        __builtin_amdgcn_s_waitcnt(0);               // (the LDS-DMA loads: vmcnt)
        __syncthreads();
        if (lat) {                                   // the values' score ranks after the rows
          lattice_ranks(lrow, n0, const_cast<int*>(lrank));
          __syncthreads();
        }
      }
      first_unit = false;
      if (!have) break;
      {
        int kc[NP];
        unsigned more = 0;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          bool m;
          kc[j] = guided_comp(guide, ws[j], m);
          more |= (unsigned)m << j;
        }
        if (__ballot(more != 0u)) {                 // (rare: a guide slice with 2+ component edges)
#pragma unroll
          for (int j = 0; j < NP; ++j)
            if ((more >> j) & 1u) kc[j] = guided_more(cum_lds, p.samp_len, u01w(ws[j]), kc[j]);
        }
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          const float4 sv = row_lds[kc[j]];
          const float pr = sv.z + uf[j] * (sv.w - sv.z);
          const float z = ndtri_f32(pr);
          const float xf = sv.x + sv.y * z;
          tj[j] = fminf(fmaxf(xf == xf ? xf : sv.x, lo_f), hi_f);
        }
      }
      if (lat) {
        // the lattice row of np.round(x / q) (k_sample_tab's quantisation) from the
        // table's entry thresholds: row c - 1 for c = #{m : thr_m <= t}, outside
        // the lattice for c = 0 or n + 1 (no f64 per candidate); the key:
        // (score rank + 1, ~index)
        int c[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) c[j] = 0;
        for (int span = n0 + 1; span > 0;) {       // (the same steps for every lane)
          const int h = span >> 1;
#pragma unroll
          for (int j = 0; j < NP; ++j) c[j] += lthr[c[j] + h] <= tj[j] ? span - h : 0;
          span = h;
        }
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          const int i = first + j;
          const bool in = c[j] >= 1 && c[j] <= n0;
          const int r = in ? c[j] - 1 : -1;
          const int rk = in ? lrank[r] : 0;
          const int brk = __float_as_int(flb);
          if (i < p.n_cand && (fi < 0 || rk > brk || (rk == brk && i < fi))) {
            fi = i; flb = __int_as_float(rk); fla = __int_as_float(r); ft = tj[j];
          }
          if (LG && i < p.n_cand) {
            const double xu = p.family == TPE_FAM_QLOGGAUSS ? exp_call((double)tj[j]) : (double)tj[j];
            const double2 lg = in ? lrow[r] : make_double2(-INFINITY, 0.0);
            double* o = lg_out + 4 * (p.cand_off + i);
            o[0] = rint(xu / p.q) * p.q; o[1] = lg.x; o[2] = lg.y; o[3] = (double)p.ctr2;
          }
        }
        continue;
      }
      uint32_t exact = 0;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int i = first + j;
        float lb2, la2;
        lp_log2(lo0, inv0, w0, ih0, n0, fast_tab, tj[j], lb2, la2);
        const bool valid = i < p.n_cand, ok = lb2 == lb2 && la2 == la2;
        exact |= (unsigned)(valid && !ok) << j;
        const float d = lb2 - la2;
        if (valid && ok && better32(d, i, fd, fi)) { fd = d; fi = i; flb = lb2; fla = la2; ft = tj[j]; }
        if (LG && valid && ok) {
          const bool lgf = p.family == TPE_FAM_LOGGAUSS;
          const double lnx = lgf ? (double)tj[j] : 0.0;
          double* o = lg_out + 4 * (p.cand_off + i);
          o[0] = lgf ? exp_call((double)tj[j]) : (double)tj[j];
          o[1] = (double)lb2 * kLn2 + p.below_base - lnx; o[2] = (double)la2 * kLn2 + p.above_base - lnx;
          o[3] = (double)p.ctr2;
        }
      }
      // outside the cells or in flagged ones: summed exactly by the whole wave
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        unsigned long long need = __ballot((exact >> j) & 1u);
        while (need) {
          const int src = __builtin_ctzll(need);
          need &= need - 1;
          const float t = __shfl(tj[j], src);
          float lb2, la2;
          lp_log2(lo0, inv0, w0, ih0, n0, fast_tab, t, lb2, la2);
          if (!(lb2 == lb2)) lb2 = lse2_wave(comp32, p.below_off, p.below_len, 0, 0, t);
          if (!(la2 == la2)) la2 = lse2_wave(comp32, p.above_off, p.above_len, p.wide_off, p.wide_len, t);
          const int i = __shfl(first, src) + j;
          const float d = lb2 - la2;
          if (lane == src && better32(d, i, fd, fi)) { fd = d; fi = i; flb = lb2; fla = la2; ft = t; }
          if (LG && lane == src) {
            const bool lgf = p.family == TPE_FAM_LOGGAUSS;
            const double lnx = lgf ? (double)t : 0.0;
            double* o = lg_out + 4 * (p.cand_off + i);
            o[0] = lgf ? exp_call((double)t) : (double)t;
            o[1] = (double)lb2 * kLn2 + p.below_base - lnx; o[2] = (double)la2 * kLn2 + p.above_base - lnx;
            o[3] = (double)p.ctr2;
          }
        }
      }
    }
    // the run's best of this wave as one key (DPP max; indices are unique): the
    // winning lane leaves its log2 sums and draw (cells) or its draw and lattice
    // row (lattice)
    {
      int tid = (int)threadIdx.x;
      asm volatile("" : "+v"(tid));
      const int wave = tid >> 6;
      // (lattice: the key of (rank + 1, ~index))
      const unsigned long long key =
          !lat ? key32(fd, fi)
               : fi < 0 ? 0ull
                        : ((unsigned long long)(__float_as_int(flb) + 1) << 32) | (unsigned long long)(~(uint32_t)fi);
      const unsigned long long wk = __ockl_wfred_max_u64(key);
      if (wk != 0ull && key == wk) { s_rv[n_def][0][wave] = flb; s_rv[n_def][1][wave] = fla; s_rv[n_def][2][wave] = ft; }
      if ((tid & 63) == 0) s_rk[n_def][wave] = wk;
      fi = -1;
    }
    ++n_def;
    gi = gk + 1;
  }
  // the runs: wave r combines run r into its record (host-visible)
  __syncthreads();
  const int wave = threadIdx.x >> 6;
  for (int r = wave; r < n_def; r += kW) {
    const unsigned long long k2 = lane < kW ? s_rk[r][lane] : 0ull;
    const unsigned long long bk = __ockl_wfred_max_u64(k2);
    const unsigned long long m2 = __ballot(bk != 0ull && k2 == bk);
    const int w2 = m2 ? (int)__builtin_ctzll(m2) : 0;
    const int i2 = bk != 0ull ? (int)~(uint32_t)bk : -1;
    if (lane == 0) {
      const RunRec rr = s_run[r];
      tpe_result res;
      res.score = 0.0; res.l = 0.0; res.g = 0.0; res.idx = i2; res.value = 0.0; res.global_idx = -1;
      if (i2 >= 0 && rr.lat) {
        // the winner's value and exact {l, g} (the lattice rows in global memory:
        // the LDS holds the last staged label)
        const float t = s_rv[r][2][w2];
        const int jq = __float_as_int(s_rv[r][1][w2]);
        const double xu = rr.logc ? exp_call((double)t) : (double)t;
        const double mq = rint(xu / rr.q);
        const double2 lg = jq >= 0 ? reinterpret_cast<const double2*>(tab)[rr.tab_off + jq]
                                   : make_double2(-INFINITY, 0.0);
        res.l = lg.x;
        res.g = lg.y;
        res.score = lg.x - lg.y;
        res.value = mq * rr.q;
        res.global_idx = rr.cand_base + i2;
      } else if (i2 >= 0) {
        const float t = s_rv[r][2][w2];
        const double lnx = rr.logc ? (double)t : 0.0;
        res.l = (double)s_rv[r][0][w2] * kLn2 + rr.bb - lnx;
        res.g = (double)s_rv[r][1][w2] * kLn2 + rr.ab - lnx;
        res.score = res.l - res.g;
        res.value = rr.logc ? exp_call((double)t) : (double)t;
        res.global_idx = rr.cand_base + i2;
      }
      run_best[rr.tile] = res;
    }
  }
}

// row of `part` a work item writes: its tile's first work item + its split
__device__ __forceinline__ int64_t part_row(const tpe_problem* __restrict__ P, const tpe_tile* __restrict__ tiles,
                                            const tpe_work& w) {
  const tpe_problem& p = P[w.problem];
  return (int64_t)tiles[p.tile_off + w.cand_start / kTile].work_first + w.split;
}

// ============================================================ score above
// Continuous families, f32, pruned: s_i = sum_k 2^(c_k - (a_k ((t_i - mu_hi_k) - mu_lo_k))^2)
// over the wave's window of sorted components plus the wide components.
//
// Local expansion (TPE_BATCH_NO_EXPAND clear): the wave's 512 sorted candidates
// span [t0 - h, t0 + h].  With u = (t - t0) / h and d = t0 - mu, every term is
//   2^(c - a^2 d^2) * exp(B u + G u^2),  B = -2 ln2 a^2 d h,  G = -ln2 a^2 h^2,
// whose Taylor coefficients follow (n+1) e_{n+1} = B e_n + 2 G e_{n-1}.  A
// component with |B| <= kTaylorBMax and |G| <= kTaylorGMax is summed into the
// wave's moments M_n = sum_k 2^(c_k - a_k^2 d_k^2) e_n(k) (one exp2 per
// component per WAVE instead of one per candidate); each candidate then adds
// sum_n M_n u^n.  The coefficients are bounded by those of exp(|B| u + |G| u^2),
// whose tail after degree 10 is < 4e-8 at the box corner (0.6, 0.05), i.e.
// < 1.2e-7 of the term (x e^(2(|B| + |G|))); every term is positive, so the
// bound holds for the sum.  Other components are evaluated exactly for every
// candidate (ce_step).  G grows with the wave's span squared: the bound on it
// is what restricts the expansion to waves narrower than ~0.3 sigma.
constexpr int kTaylorN = 11;
constexpr float kTaylorBMax = 0.6f;
constexpr float kTaylorGMax = 0.05f;
constexpr float kLn2f = 0.693147180559945309f;

__device__ __forceinline__ float4 readlane4(const float4 c, int lane) {
  return make_float4(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.x), lane)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.y), lane)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.z), lane)),
                     __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.w), lane)));
}

// components [kb, ke) (wave-uniform): expandable ones into M, the rest exactly;
// returns the number of exactly evaluated components
__device__ __forceinline__ int expand_range(const float4* __restrict__ C, int kb, int ke, float t0, float h,
                                            float (&M)[kTaylorN], const f2 (&t2)[kR / 2], f2 (&s2)[kR / 2]) {
  const int lane = threadIdx.x & 63;
  int n_exact = 0;
  for (int base = kb; base < ke; base += 64) {
    const int k = base + lane;
    const bool valid = k < ke;
    const float4 c = valid ? C[k] : make_float4(0.f, 0.f, 0.f, -INFINITY);
    const bool live = valid && c.w > -INFINITY;     // wide components sit in the sorted list at c = -inf
    const float d = (t0 - c.x) - c.y;
    const float z = c.z * d;
    const float ah = c.z * h;
    const float B = -2.f * kLn2f * (c.z * z) * h;
    const float G = -kLn2f * ah * ah;
    const bool expand = live && fabsf(B) <= kTaylorBMax && fabsf(G) <= kTaylorGMax;
    const float h0 = expand ? __builtin_amdgcn_exp2f(c.w - z * z) : 0.f;
    float em1 = 0.f, e = h0;
    M[0] += e;
#pragma unroll
    for (int n = 1; n < kTaylorN; ++n) {
      const float en = (B * e + 2.f * G * em1) * (1.f / (float)n);
      em1 = e;
      e = en;
      M[n] += e;
    }
    unsigned long long rest = __ballot(live && !expand);
    n_exact += __popcll(rest);
#ifndef TPE_EXACT_CHUNK_ACC
#define TPE_EXACT_CHUNK_ACC 1
#endif
    if (!TPE_EXACT_CHUNK_ACC) {
      while (rest) {
        const int bl = __builtin_ctzll(rest);
        rest &= rest - 1;
        ce_step(readlane4(c, bl), t2, s2);
      }
    } else if (rest) {
      // this chunk's exact terms summed on their own, then added: small terms
      // are not rounded away one by one against a large running sum
      f2 acc[kR / 2];
#pragma unroll
      for (int j = 0; j < kR / 2; ++j) acc[j] = f2{0.f, 0.f};
      while (rest) {
        const int bl = __builtin_ctzll(rest);
        rest &= rest - 1;
        ce_step(readlane4(c, bl), t2, acc);
      }
#pragma unroll
      for (int j = 0; j < kR / 2; ++j) s2[j] += acc[j];
    }
  }
  return n_exact;
}

// wave-reduce the moments and add sum_n M_n u^n to every candidate's sum
__device__ __forceinline__ void add_moments(float (&M)[kTaylorN], float t0, float h, const f2 (&t2)[kR / 2],
                                            f2 (&s2)[kR / 2]) {
#pragma unroll
  for (int q = 0; q < kTaylorN; ++q)
    for (int off = 32; off > 0; off >>= 1) M[q] += __shfl_xor(M[q], off);
  const float hinv = h > 0.f ? 1.f / h : 0.f;
  const f2 c0 = f2{t0, t0}, hv = f2{hinv, hinv};
#pragma unroll
  for (int j = 0; j < kR / 2; ++j) {
    const f2 u = (t2[j] - c0) * hv;
    f2 acc = f2{M[kTaylorN - 1], M[kTaylorN - 1]};
#pragma unroll
    for (int q = kTaylorN - 2; q >= 0; --q) acc = acc * u + f2{M[q], M[q]};
    s2[j] += acc;
  }
}

// the below mixture (<= 26 components, the widest bandwidths of the problem)
// at the wave's kR x 64 candidates: local expansion (exact fallback) unless
// TPE_BATCH_NO_EXPAND
__device__ __forceinline__ void below_sum(const float4* __restrict__ B, int n, float tmin, float tmax, int flags,
                                          const f2 (&t2)[kR / 2], f2 (&sb2)[kR / 2]) {
  if (flags & TPE_BATCH_NO_EXPAND) {
    for (int k = 0; k < n; ++k) ce_step(B[k], t2, sb2);
    return;
  }
  const float t0 = 0.5f * (tmin + tmax), h = 0.5f * (tmax - tmin);
  float M[kTaylorN];
#pragma unroll
  for (int q = 0; q < kTaylorN; ++q) M[q] = 0.f;
  expand_range(B, 0, n, t0, h, M, t2, sb2);
  add_moments(M, t0, h, t2, sb2);
}

#ifndef TPE_ABOVE_WAVES_PER_EU
#define TPE_ABOVE_WAVES_PER_EU 4   // <= 128 VGPRs: no scratch spills (5 waves spilled 48 B per lane)
#endif
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(TPE_ABOVE_WAVES_PER_EU))) void k_above_f32(const tpe_problem* __restrict__ P,
                                                        const tpe_tile* __restrict__ tiles,
                                                        const tpe_work* __restrict__ W,
                                                        const float4* __restrict__ comp,
                                                        const int32_t* __restrict__ grid,
                                                        const uint64_t* __restrict__ vals,
                                                        double* __restrict__ part,
                                                        tpe_best* __restrict__ tile_best,
                                                        double* __restrict__ l_out, double* __restrict__ g_out,
                                                        unsigned long long* __restrict__ ce_count, int flags,
                                                        int sampled, unsigned long long* __restrict__ pool_best) {
  const tpe_work w = W[blockIdx.x];
  const tpe_problem& p = P[w.problem];
  const int n = p.n_cand;
  float t[kR], s[kR];
  float tmin = INFINITY, tmax = -INFINITY;
#pragma unroll
  for (int j = 0; j < kR; ++j) {
    const int i = tile_pos(w.cand_start, j);
    t[j] = i < n ? __uint_as_float((uint32_t)vals[p.cand_off + i]) : 0.f;
    if (i < n) { tmin = fminf(tmin, t[j]); tmax = fmaxf(tmax, t[j]); }
    s[j] = 0.f;
  }
  // this wave's component window
  for (int off = 32; off > 0; off >>= 1) {
    tmin = fminf(tmin, __shfl_xor(tmin, off));
    tmax = fmaxf(tmax, __shfl_xor(tmax, off));
  }
  int k_lo = w.k_start, k_hi = w.k_end;
  const bool any = tmin <= tmax;
  if (!any) {
    k_hi = k_lo;                       // no valid candidate in this wave
  } else if (p.narrow_amin > 0.f) {
    const float dmax = fmaxf(fabsf(tmin - p.prior_mu), fabsf(tmax - p.prior_mu));
    const float zp = p.prior_a * dmax;
    const float lb = p.prior_c - zp * zp;
    const float R = sqrtf(fmaxf(p.narrow_cmax - lb + kPruneBits, 0.f)) / p.narrow_amin;
    const float vlo = tmin - R, vhi = tmax + R;
    if (vlo == vlo && vhi == vhi && R < INFINITY) {
      const float gl = (vlo - p.grid_lo) * p.grid_inv, gh = (vhi - p.grid_lo) * p.grid_inv;
      const int bl = (int)fminf(fmaxf(floorf(gl) - 1.f, 0.f), (float)p.grid_n);
      const int bh = (int)fminf(fmaxf(floorf(gh) + 2.f, 0.f), (float)p.grid_n);
      const int32_t* G = grid + p.grid_off;
      // pruned problems split the wave's WINDOW (not the whole mixture) over the
      // work items of this tile, so every work item gets an equal share
      const int wl = G[bl], wh = max(G[bh], G[bl]);
      const long long len = wh - wl;
      k_lo = wl + (int)((len * w.split) / w.n_splits);
      k_hi = wl + (int)((len * (w.split + 1)) / w.n_splits);
    }
  }
  k_lo = __builtin_amdgcn_readfirstlane(k_lo);
  k_hi = __builtin_amdgcn_readfirstlane(k_hi);
  const int wide_len = (w.split == 0 && any) ? p.wide_len : 0;   // wide components once per candidate
  // candidate pairs in packed f32 (v_pk_add/mul/fma_f32); v_exp_f32 per lane value
  f2 t2[kR / 2], s2[kR / 2];
#pragma unroll
  for (int j = 0; j < kR / 2; ++j) { t2[j] = f2{t[2 * j], t[2 * j + 1]}; s2[j] = f2{0.f, 0.f}; }
  const float4* __restrict__ C = comp + p.above_off;
  long long n_exact = 0, n_expanded = 0;
  if (!(flags & TPE_BATCH_NO_EXPAND)) {
    const float t0 = 0.5f * (tmin + tmax), h = 0.5f * (tmax - tmin);
    float M[kTaylorN];
#pragma unroll
    for (int q = 0; q < kTaylorN; ++q) M[q] = 0.f;
    n_exact = expand_range(C, k_lo, k_hi, t0, h, M, t2, s2);
    n_exact += expand_range(comp + p.wide_off, 0, wide_len, t0, h, M, t2, s2);
    n_expanded = (long long)(k_hi - k_lo) + wide_len - n_exact;
    add_moments(M, t0, h, t2, s2);
  } else {
    for (int kb = k_lo; kb < k_hi; kb += 64) {      // 64-component chunks, as in expand_range
      f2 acc[kR / 2];
#pragma unroll
      for (int j = 0; j < kR / 2; ++j) acc[j] = f2{0.f, 0.f};
      const int ke = min(kb + 64, k_hi);
#pragma unroll 4
      for (int k = kb; k < ke; ++k) ce_step(C[k], t2, acc);
#pragma unroll
      for (int j = 0; j < kR / 2; ++j) s2[j] += acc[j];
    }
    const float4* __restrict__ Wd = comp + p.wide_off;
    for (int k = 0; k < wide_len; ++k) ce_step(Wd[k], t2, s2);
    n_exact = (long long)(k_hi - k_lo) + wide_len;
  }
#pragma unroll
  for (int j = 0; j < kR / 2; ++j) { s[2 * j] = s2[j].x; s[2 * j + 1] = s2[j].y; }
  // Fused finalize: a one-split work item holds its whole tile's above sums, so
  // it scores l - g for the tile and writes the tile's best to slot 0 (slots
  // 1..7 empty); the packer leaves these tiles out of k_finalize's list.  (Multi-split tiles — the sparse tails — are finalized by
  // k_finalize: a device-wide handshake between their work items would cost an
  // L2 write-back per item on this multi-XCD part.)  The below mixture is summed
  // by the same local expansion (its <= 26 components are the widest of the
  // problem, so they expand over any wave narrow enough for the above side);
  // k_finalize sums it directly, so the two agree to fp32 rounding.
  const bool fin = sampled && !(flags & TPE_BATCH_NO_FUSE) && w.n_splits == 1;
  const int tile = p.tile_off + w.cand_start / kTile;
  if (!fin) {                          // partial sums for k_finalize
    double* __restrict__ out = part + part_row(P, tiles, w) * kTile - w.cand_start;
#pragma unroll
    for (int j = 0; j < kR; ++j) {
      const int i = tile_pos(w.cand_start, j);
      if (i < n) out[i] = (double)s[j];
    }
  }
  if (fin) {
    const bool logsp = p.family == TPE_FAM_LOGGAUSS;
    double bs = 0, bl = 0, bg = 0;
    int64_t bi = -1;
    // below mixture for all kR candidates at once: one pass over its (<= 26)
    // components, each loaded once per wave (component-outer, like the above sum)
    f2 sb2[kR / 2];
    uint32_t oo[kR];                   // original positions: reloaded together (one latency)
#pragma unroll
    for (int j = 0; j < kR; ++j) {
      const int i = tile_pos(w.cand_start, j);
      oo[j] = i < n ? (uint32_t)(vals[p.cand_off + i] >> 32) : 0u;
    }
#pragma unroll
    for (int j = 0; j < kR / 2; ++j) sb2[j] = f2{0.f, 0.f};
    below_sum(comp + p.below_off, p.below_len, tmin, tmax, flags, t2, sb2);
    {
#pragma unroll
    for (int j = 0; j < kR; ++j) {
      const int i = tile_pos(w.cand_start, j);
      if (i >= n) continue;
      const double sa = (double)s[j];
      const float sb = (j & 1) ? sb2[j >> 1].y : sb2[j >> 1].x;
      // an under-flowed fixed-shift sum (either side): max-shifted recompute
      // over the whole mixture, out of line (rare; keeps this loop's registers)
      const double lb2 = sb > 1e-30f ? (double)__log2f(sb)
                                     : (double)lse2_exact_ool(comp, p.below_off, p.below_len, 0, 0, t[j]);
      const double la2 = sa > 1e-30 ? log2(sa)
                         : p.narrow_amin > 0.f ? (double)lse2_pruned(p, comp, grid, t[j])
                                               : (double)lse2_exact_ool(comp, p.above_off, p.above_len, p.wide_off,
                                                                        p.wide_len, t[j]);
      const double lnx = logsp ? (double)t[j] : 0.0;
      const double l = lb2 * kLn2 + p.below_base - lnx;
      const double g = la2 * kLn2 + p.above_base - lnx;
      if (l_out) { l_out[oo[j]] = l; g_out[oo[j]] = g; }
      if (p.flags & TPE_F_POOLED) { pool_update(P, p, pool_best, (int64_t)oo[j], l - g); continue; }
      const int64_t orig = (int64_t)oo[j] - p.cand_off;
      if (better(l - g, orig, bs, bi)) { bs = l - g; bl = l; bg = g; bi = orig; }
    }
    if (!(p.flags & TPE_F_POOLED)) {       // (problem-uniform branch: block_best synchronises)
      tpe_best* __restrict__ slot = tile_best + (int64_t)tile * TPE_BEST_PER_TILE;
      block_best(bs, bi, bl, bg, slot);
      if (threadIdx.x > 0 && threadIdx.x < TPE_BEST_PER_TILE) slot[threadIdx.x] = tpe_best{0, 0, 0, -1};
    }
    }
  }
  if (ce_count) {       // profiling (no atomics): [exact CE, expanded components] of this work item
    __shared__ unsigned long long wce[kThreads / 64][2];
    if ((threadIdx.x & 63) == 0) {
      const int wave_first = w.cand_start + (int)(threadIdx.x >> 6) * kWaveCands;
      const int valid = max(0, min(kWaveCands, n - wave_first));
      wce[threadIdx.x >> 6][0] = (unsigned long long)(n_exact * valid);
      wce[threadIdx.x >> 6][1] = (unsigned long long)n_expanded;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long a0 = 0, a1 = 0;
      for (int q = 0; q < kThreads / 64; ++q) { a0 += wce[q][0]; a1 += wce[q][1]; }
      ce_count[2 * blockIdx.x] = a0;
      ce_count[2 * blockIdx.x + 1] = a1;
    }
  }
}

// Continuous families, f64 (parity precision, unpruned)
__global__ __launch_bounds__(kThreads) void k_above_f64(const tpe_problem* __restrict__ P,
                                                        const tpe_tile* __restrict__ tiles,
                                                        const tpe_work* __restrict__ W,
                                                        const double4* __restrict__ comp,
                                                        const double* __restrict__ cand,
                                                        const uint64_t* __restrict__ vals,
                                                        double* __restrict__ part) {
  const tpe_work w = W[blockIdx.x];
  const tpe_problem& p = P[w.problem];
  const int n = p.n_cand;
  const bool logsp = p.family == TPE_FAM_LOGGAUSS;
  double t[kR], s[kR];
#pragma unroll
  for (int j = 0; j < kR; ++j) {
    const int i = tile_pos(w.cand_start, j);
    const double x = i < n ? cand[vals[p.cand_off + i] >> 32] : 1.0;
    t[j] = logsp ? log(x) : x;
    s[j] = 0.0;
  }
  const double4* __restrict__ C = comp + p.above_off;
  for (int k = w.k_start; k < w.k_end; ++k) {
    const double4 c = C[k];
#pragma unroll
    for (int j = 0; j < kR; ++j) {
      const double z = (t[j] - c.x) * c.y;
      s[j] += exp2(c.z - z * z);
    }
  }
  double* __restrict__ out = part + part_row(P, tiles, w) * kTile - w.cand_start;
#pragma unroll
  for (int j = 0; j < kR; ++j) {
    const int i = tile_pos(w.cand_start, j);
    if (i < n) out[i] = s[j];
  }
}

// Quantized families (always f64): partial mixture mass
template <bool LOG>
__global__ __launch_bounds__(kThreads) void k_above_q(const tpe_problem* __restrict__ P,
                                                      const tpe_tile* __restrict__ tiles,
                                                      const tpe_work* __restrict__ W,
                                                      const double4* __restrict__ comp,
                                                      const double* __restrict__ cand,
                                                      const uint64_t* __restrict__ vals,
                                                      double* __restrict__ part) {
  const tpe_work w = W[blockIdx.x];
  const tpe_problem& p = P[w.problem];
  const int n = p.n_cand;
  constexpr int R = kR / 2;   // two erf per component: keep register use moderate
  for (int h = 0; h < 2; ++h) {
    double tu[R], tl[R], s[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int i = tile_pos(w.cand_start, h * R + j);
      const double x = i < n ? cand[vals[p.cand_off + i] >> 32] : 0.0;
      q_bounds(p, x, tu[j], tl[j]);
      s[j] = 0.0;
    }
    const double4* __restrict__ C = comp + p.above_off;
    for (int k = w.k_start; k < w.k_end; ++k) {
      const double4 c = C[k];
#pragma unroll
      for (int j = 0; j < R; ++j) s[j] += qterm<LOG>(c, tu[j], tl[j]);
    }
    double* __restrict__ out = part + part_row(P, tiles, w) * kTile - w.cand_start;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int i = tile_pos(w.cand_start, h * R + j);
      if (i < n) out[i] = s[j];
    }
  }
}

// =============================================================== finalize
// Grid (tiles, TPE_BEST_PER_TILE): one candidate per thread, 256-thread
// workgroups, so the latency-bound stage (dependent loads, <= 26 below
// components) keeps many workgroups in flight.  Each workgroup writes one
// tile_best slot; candidates may be visited in any order because the argmax
// compares ORIGINAL indices.
static_assert(TPE_BEST_PER_TILE * kThreads == kTile, "finalize slices must cover a tile");

__device__ __forceinline__ void finalize_slice(const tpe_problem* __restrict__ P,
                                               const tpe_tile* __restrict__ tiles,
                                               const float4* __restrict__ comp32,
                                               const double4* __restrict__ comp64,
                                               const int32_t* __restrict__ grid,
                                               const double* __restrict__ cand,
                                               const uint64_t* __restrict__ vals,
                                               const double* __restrict__ part,
                                               double* __restrict__ l_out, double* __restrict__ g_out,
                                               tpe_best* __restrict__ tile_best, int precision,
                                               int sampled, int flags, int tile,
                                               unsigned long long* __restrict__ pool_best) {
  const tpe_tile tl = tiles[tile];
  const tpe_problem& p = P[tl.problem];
  // sampled categorical tiles are finalized by k_sample (one-split continuous
  // f32 tiles by the above kernel: they are never in the finalize list)
  if (sampled && p.family == TPE_FAM_CATEGORICAL && p.samp_len <= kCumLds) return;
  if (p.tab_mode != TPE_TAB_NONE) return;          // scored by the sample stage from its tables

  const int n = p.n_cand;
  const int i = tl.cand_start + (int)threadIdx.x + (int)blockIdx.y * kThreads;
  const bool valid = i < n;
  // device-drawn candidates carry their coordinate t in the sort value: no
  // gather of the candidate value (continuous families at f32, categorical)
  const bool from_t = sampled && ((precision == TPE_PREC_F32 &&
                                   (p.family == TPE_FAM_GAUSS || p.family == TPE_FAM_LOGGAUSS)) ||
                                  p.family == TPE_FAM_CATEGORICAL);
  const uint64_t v = valid ? vals[p.cand_off + i] : 0;
  double sa = 0.0;
  {
    // the tile's partial-sum rows, in split order
    const double* __restrict__ ps = part + (int64_t)tl.work_first * kTile + (i - tl.cand_start);
    const int ns = valid ? tl.n_splits : 0;
    int sp = 0;
    for (; sp + 8 <= ns; sp += 8) {         // eight loads in flight per step
      double a[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] = ps[(int64_t)(sp + q) * kTile];
#pragma unroll
      for (int q = 0; q < 8; ++q) sa += a[q];
    }
    for (; sp < ns; ++sp) sa += ps[(int64_t)sp * kTile];
  }
  const uint32_t oo = (uint32_t)(v >> 32);         // original position
  const int64_t orig = valid ? (int64_t)oo - p.cand_off : -1;
  const float tf = __uint_as_float((uint32_t)v);
  const double x = !valid ? 0.0 : (from_t ? (double)tf : cand[oo]);
  double l = 0, g = 0;
  if (valid) {
    if (p.family == TPE_FAM_CATEGORICAL) {
      const int c = (int)x;
      if (c >= 0 && c < p.n_upper && (double)c == x) {
        l = comp64[p.below_off + c].x;
        g = comp64[p.above_off + c].x;
      } else {
        l = NAN; g = NAN;      // the reference raises IndexError here
      }
    } else if (p.family == TPE_FAM_QGAUSS || p.family == TPE_FAM_QLOGGAUSS) {
      double tu, tlo;
      q_bounds(p, x, tu, tlo);
      const double mb = p.family == TPE_FAM_QGAUSS ? qmass<false>(comp64, p.below_off, p.below_len, tu, tlo)
                                                   : qmass<true>(comp64, p.below_off, p.below_len, tu, tlo);
      l = log(mb) + p.below_base;
      g = log(sa) + p.above_base;
    } else {
      const bool logsp = p.family == TPE_FAM_LOGGAUSS;
      double lb2, la2;
      if (precision == TPE_PREC_F32) {
        const float t = tf;
        lb2 = (double)lse2_fixed(comp32, p.below_off, p.below_len, t);
        // fixed-shift sum; if it under-flowed, redo this candidate max-shifted
        la2 = sa > 1e-30 ? log2(sa)
              : p.narrow_amin > 0.f ? (double)lse2_pruned(p, comp32, grid, t)
                                    : (double)lse2_exact<float, float4>(comp32, p.above_off, p.above_len, p.wide_off,
                                                                        p.wide_len, t);
      } else {
        const double t = logsp ? log(x) : x;
        lb2 = lse2_exact64(comp64, p.below_off, p.below_len, t);
        la2 = sa > 1e-280 ? log2(sa) : lse2_exact64(comp64, p.above_off, p.above_len, t);
      }
      const double lnx = !logsp ? 0.0 : (from_t ? (double)tf : log(x));
      l = lb2 * kLn2 + p.below_base - lnx;
      g = la2 * kLn2 + p.above_base - lnx;
    }
    if (l_out) { l_out[oo] = l; g_out[oo] = g; }
  }
  if (p.flags & TPE_F_POOLED) {            // problem-uniform: no block reduction follows
    if (valid) pool_update(P, p, pool_best, (int64_t)oo, l - g);
    return;
  }
  const double sc = l - g;
  // wave argmax on (score, original index) only; the winning lane (unique
  // index) then publishes its l and g
  double bs = sc;
  int64_t bi = orig;
  for (int off = 32; off > 0; off >>= 1) {
    const double os = __shfl_xor(bs, off);
    const int64_t oi = __shfl_xor(bi, off);
    if (better(os, oi, bs, bi)) { bs = os; bi = oi; }
  }
  __shared__ tpe_best wb[kThreads / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0 && bi < 0) wb[wave] = tpe_best{0, 0, 0, -1};
  if (bi >= 0 && orig == bi) wb[wave] = tpe_best{bs, l, g, bi};
  __syncthreads();
  if (threadIdx.x == 0) {
    tpe_best b = wb[0];
    for (int q = 1; q < kThreads / 64; ++q)
      if (better(wb[q].score, wb[q].idx, b.score, b.idx)) b = wb[q];
    tile_best[(int64_t)tile * TPE_BEST_PER_TILE + blockIdx.y] = b;
  }
}

// grid (n_fin, TPE_BEST_PER_TILE): tile fin_tiles[x] (every tile when fin_tiles
// is NULL).  The packer lists only the tiles no upstream stage finalizes.
__global__ __launch_bounds__(kThreads) void k_finalize(const tpe_problem* __restrict__ P,
                                                       const tpe_tile* __restrict__ tiles,
                                                       const int32_t* __restrict__ fin_tiles,
                                                       const float4* __restrict__ comp32,
                                                       const double4* __restrict__ comp64,
                                                       const int32_t* __restrict__ grid,
                                                       const double* __restrict__ cand,
                                                       const uint64_t* __restrict__ vals,
                                                       const double* __restrict__ part,
                                                       double* __restrict__ l_out, double* __restrict__ g_out,
                                                       tpe_best* __restrict__ tile_best, int precision,
                                                       int sampled, int flags,
                                                       unsigned long long* __restrict__ pool_best) {
  const int tile = fin_tiles ? fin_tiles[blockIdx.x] : (int)blockIdx.x;
  finalize_slice(P, tiles, comp32, comp64, grid, cand, vals, part, l_out, g_out, tile_best, precision, sampled,
                 flags, tile, pool_best);
}

// ================================================================= select
// One 1024-thread workgroup per problem: reads the problem's
// n_tiles * TPE_BEST_PER_TILE slot bests (4096 at 2^20 candidates).
constexpr int kSelThreads = 1024;

// block-wide max / sum over kSelThreads threads (lds: kSelThreads / 64 slots)
template <typename T, bool MAX>
__device__ __forceinline__ T sel_reduce(T v, T* lds) {
  for (int off = 32; off > 0; off >>= 1) {
    const T o = __shfl_xor(v, off);
    v = MAX ? (o > v ? o : v) : v + o;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  v = lds[0];
  for (int q = 1; q < kSelThreads / 64; ++q) v = MAX ? (lds[q] > v ? lds[q] : v) : v + lds[q];
  return v;
}

// exact max-shifted log2-sum of comp rows [k0, k0 + n) and [k1, k1 + n1) at t,
// spread over the workgroup (f64 sum)
__device__ double sel_lse2(const float4* __restrict__ comp, int k0, int n, int k1, int n1, float t, double* lds) {
  float m = -INFINITY;
  for (int k = threadIdx.x; k < n + n1; k += kSelThreads) {
    const float4 c = k < n ? comp[k0 + k] : comp[k1 + k - n];
    const float z = ((t - c.x) - c.y) * c.z;
    m = fmaxf(m, c.w - z * z);
  }
  const double mm = sel_reduce<double, true>((double)m, lds);
  if (!(mm > -INFINITY)) return mm;
  double sum = 0.0;
  for (int k = threadIdx.x; k < n + n1; k += kSelThreads) {
    const float4 c = k < n ? comp[k0 + k] : comp[k1 + k - n];
    const float z = ((t - c.x) - c.y) * c.z;
    sum += exp2((double)(c.w - z * z) - mm);
  }
  return mm + log2(sel_reduce<double, false>(sum, lds));
}

// a lazy categorical problem (TPE_F_CAT_LAZY): selected by a scan of its
// first draws, never by its tiles
__device__ __forceinline__ bool lazy_eligible(const tpe_problem& p) {
  return (p.flags & TPE_F_CAT_LAZY) && p.family == TPE_FAM_CATEGORICAL && p.samp_len <= 64;
}

// lazy categorical (TPE_F_CAT_LAZY): draws scanned in index order, 4096 per
// round (4 per thread), keeping each category's first index; stops once no undrawn drawable
// category could beat the current best (np.argmax order via better(): an
// undrawn category's index would exceed every drawn one) — after the first
// round unless the best-scoring category is rare.
__device__ void select_cat_lazy(const tpe_problem& p, const double* __restrict__ samp,
                                const double4* __restrict__ comp64, tpe_result* __restrict__ out) {
  __shared__ double cum[64], score[64], lsh[64], gsh[64];   // l, g in LDS: no global loads in the serial scan
  __shared__ int first[64];
  __shared__ int done;
  const int K = p.samp_len;
  const double* S = samp + 8 * (int64_t)p.samp_off;
  if ((int)threadIdx.x < K) {
    cum[threadIdx.x] = S[8 * threadIdx.x];
    lsh[threadIdx.x] = comp64[p.below_off + threadIdx.x].x;
    gsh[threadIdx.x] = comp64[p.above_off + threadIdx.x].x;
    score[threadIdx.x] = lsh[threadIdx.x] - gsh[threadIdx.x];
    first[threadIdx.x] = INT_MAX;
  }
  __syncthreads();
  tpe_best b{0, 0, 0, -1};
  // 4096 draws per round whatever the workgroup size (k_select: 1024 threads x 4,
  // the table stage: 512 x 8)
  constexpr int kLazyRound = 4096, kLazyMaxPer = 8;
  const int nt = (int)blockDim.x;
  const int per = kLazyRound / nt;
  for (int base = 0; base < p.n_cand; base += kLazyRound) {
    int c[kLazyMaxPer];
#pragma unroll
    for (int j = 0; j < kLazyMaxPer; ++j) {
      const int i = base + j * nt + (int)threadIdx.x;
      c[j] = j < per && i < p.n_cand ? draw_category(p, cum, i) : -1;
    }
#pragma unroll
    for (int j = 0; j < kLazyMaxPer; ++j)
      for (int cc = 0; cc < K && j < per; ++cc) {     // one LDS atomic per wave and category
        const unsigned long long m = __ballot(c[j] == cc);
        if ((threadIdx.x & 63) == 0 && m)
          atomicMin(&first[cc], base + j * nt + (int)(threadIdx.x & ~63) + __builtin_ctzll(m));
      }
    __syncthreads();
    if (threadIdx.x == 0) {
      b = tpe_best{0, 0, 0, -1};
      for (int c = 0; c < K; ++c)
        if (first[c] != INT_MAX && better(score[c], (int64_t)first[c], b.score, b.idx))
          b = tpe_best{score[c], lsh[c], gsh[c], (int64_t)first[c]};
      int more = b.idx < 0;
      for (int c = 0; c < K && !more; ++c) {
        const bool drawable = cum[c] > (c ? cum[c - 1] : 0.0);
        more = first[c] == INT_MAX && drawable && better(score[c], INT64_MAX, b.score, b.idx);
      }
      done = !more;
    }
    __syncthreads();
    if (done) break;
  }
  if (threadIdx.x == 0) {
    tpe_result r;
    r.score = b.score; r.l = b.l; r.g = b.g; r.idx = b.idx;
    r.value = b.idx >= 0 ? (double)draw_category(p, cum, b.idx) : 0.0;
    r.global_idx = b.idx >= 0 ? p.cand_base + b.idx : -1;
    *out = r;
  }
}

// pooled problem: the winner from pool_best, its value re-drawn, its l and g
// evaluated exactly over the whole mixtures (one workgroup)
__device__ void select_pooled(const tpe_problem& p, int pid, const unsigned long long* __restrict__ pool_best,
                              const float4* __restrict__ comp32, const double* __restrict__ samp,
                              const double* __restrict__ cand, int precision, int sampled,
                              tpe_result* __restrict__ out) {
  __shared__ double lds[kSelThreads / 64];
  const unsigned long long key = pool_best[pid];
  const unsigned long long mask = (1ull << pool_idx_bits(p.n_cand)) - 1;
  const int64_t idx = key ? (int64_t)(mask - (key & mask)) : -1;
  tpe_result r;
  r.score = 0; r.l = 0; r.g = 0; r.value = 0; r.idx = idx; r.global_idx = -1;
  if (idx >= 0) {
    float lo_f, hi_f, t;
    int c;
    if (sampled && p.samp_len > 0) {
      f32_bounds(p, lo_f, hi_f);
      const double* S = samp + 8 * (int64_t)p.samp_off;
      draw_one(p, S, S, 8, idx, precision, lo_f, hi_f, r.value, t, c);
    } else {                               // caller-drawn candidates
      r.value = cand[p.cand_off + idx];
      t = (float)(p.family == TPE_FAM_LOGGAUSS ? log(r.value) : r.value);
    }
    const double lb2 = sel_lse2(comp32, p.below_off, p.below_len, 0, 0, t, lds);
    const double la2 = sel_lse2(comp32, p.above_off, p.above_len, p.wide_off, p.wide_len, t, lds);
    const double lnx = p.family == TPE_FAM_LOGGAUSS ? (double)t : 0.0;
    r.l = lb2 * kLn2 + p.below_base - lnx;
    r.g = la2 * kLn2 + p.above_base - lnx;
    r.score = r.l - r.g;
    r.global_idx = p.cand_base + idx;
  }
  if (threadIdx.x == 0) *out = r;
}
// the winner of a problem scored per tile: the best of its tiles' slots
// (np.argmax order), its value re-drawn (never stored), l and g as scored.
// One kSelThreads workgroup; every thread returns (k_select, and the sample
// stage's last workgroup of a tabulated problem).
__device__ void select_generic(const tpe_problem& p, const tpe_best* __restrict__ tile_best,
                               const double* __restrict__ cand, const double* __restrict__ samp, int precision,
                               int sampled, const double* __restrict__ draw_pref, int64_t draw_blocks, int ordered,
                               tpe_result* __restrict__ out) {
  // the sampler rows of a <= 64-component mixture staged in LDS while the tile
  // bests load, so the winner's redraw needs no dependent global loads
  __shared__ double srow[64 * 8];
  const bool staged = sampled && p.samp_len > 0 && p.samp_len <= 64;
  if (staged) {
    const double* S = samp + 8 * (int64_t)p.samp_off;
    for (int q = threadIdx.x; q < 8 * p.samp_len; q += kSelThreads) srow[q] = S[q];
  }
  tpe_best b{0, 0, 0, -1};
  const int64_t nb = (int64_t)p.n_tiles * TPE_BEST_PER_TILE;
  const tpe_best* __restrict__ tb = tile_best + (int64_t)p.tile_off * TPE_BEST_PER_TILE;
  for (int64_t t = threadIdx.x; t < nb; t += kSelThreads) {
    const tpe_best o = tb[t];
    if (better(o.score, o.idx, b.score, b.idx)) b = o;
  }
  for (int off = 32; off > 0; off >>= 1) {
    tpe_best o;
    o.score = __shfl_xor(b.score, off); o.l = __shfl_xor(b.l, off); o.g = __shfl_xor(b.g, off);
    o.idx = __shfl_xor(b.idx, off);
    if (better(o.score, o.idx, b.score, b.idx)) b = o;
  }
  __shared__ tpe_best wb[kSelThreads / 64];
  if ((threadIdx.x & 63) == 0) wb[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x < 64) {                  // wave 0 finishes (no early return: callers continue)
  b = wb[0];
  for (int q = 1; q < kSelThreads / 64; ++q)
    if (better(wb[q].score, wb[q].idx, b.score, b.idx)) b = wb[q];
  const bool redraw = b.idx >= 0 && sampled && p.samp_len > 0;   // the winner's value was never stored
  const bool od = redraw && ordered && p.sort_slot >= 0;
  double U = 0.0;
  if (od) {                                // wave 0: the winner's canonical block scan
    const int64_t g = p.cand_base + b.idx;
    const double* row = draw_pref + (int64_t)p.sort_slot * (draw_blocks + 1);
    const double sc = exp_block_scan(p, g >> 6);
    U = (row[g >> 6] + __shfl(sc, (int)(g & 63))) / row[draw_blocks];
  }
  // i.i.d. redraw with <= 64 below components: the component search of draw_one
  // as one wave-wide compare + ballot (first k with u < cum_k, else K-1: the
  // binary search's answer on a non-decreasing CDF) instead of a chain of
  // dependent global loads on lane 0
  const bool wave_search = redraw && !od && staged;
  int comp = 0;
  DrawU rw{0.0, 0.f, 0.0};
  if (wave_search) {
    const double* S = srow;
    rw = draw_uniforms(p, b.idx, precision);
    const int lane = (int)threadIdx.x;
    const bool hit = lane < p.samp_len && rw.us < S[8 * lane];
    const unsigned long long m = __ballot(hit);
    comp = m ? __builtin_ctzll(m) : p.samp_len - 1;
  }
  if (threadIdx.x == 0) {
    tpe_result r;
    r.score = b.score; r.l = b.l; r.g = b.g; r.idx = b.idx;
    r.value = 0.0;
    if (redraw) {
      float lo_f, hi_f, t;
      int c;
      f32_bounds(p, lo_f, hi_f);
      const double* S = samp + 8 * (int64_t)p.samp_off;
      if (od) ordered_draw(p, S, S, 8, U, precision, lo_f, hi_f, r.value, t);
      else if (!wave_search) draw_one(p, S, S, 8, b.idx, precision, lo_f, hi_f, r.value, t, c);
      else if (p.family == TPE_FAM_CATEGORICAL) r.value = (double)comp;
      else draw_comp(p, srow, comp, rw.uf, rw.ud, precision, lo_f, hi_f, r.value, t);
    } else if (b.idx >= 0) {
      r.value = cand[p.cand_off + b.idx];
    }
    r.global_idx = b.idx >= 0 ? p.cand_base + b.idx : -1;
    *out = r;
  }
  }
  __syncthreads();                         // (srow / wb reusable by the caller's next selection)
}

__global__ __launch_bounds__(kSelThreads) void k_select(const tpe_problem* __restrict__ P,
                                                     const tpe_best* __restrict__ tile_best,
                                                     const double* __restrict__ cand,
                                                     const double* __restrict__ samp, int precision, int sampled,
                                                     const double* __restrict__ draw_pref, int64_t draw_blocks,
                                                     int ordered, const unsigned long long* __restrict__ pool_best,
                                                     const float4* __restrict__ comp32,
                                                     const double4* __restrict__ comp64, int lazy_ok,
                                                     int early, tpe_result* __restrict__ result) {
  const tpe_problem& p = P[blockIdx.x];
  const bool lazy = lazy_ok && sampled && lazy_eligible(p);
  if (early && (lazy || p.tab_mode != TPE_TAB_NONE)) return;   // selected by the table / sample stage
  if (lazy) {
    select_cat_lazy(p, samp, comp64, result + blockIdx.x);
    return;
  }
  if (p.flags & TPE_F_POOLED) {            // problem-uniform
    select_pooled(p, blockIdx.x, pool_best, comp32, samp, cand, precision, sampled, result + blockIdx.x);
    return;
  }
  select_generic(p, tile_best, cand, samp, precision, sampled, draw_pref, draw_blocks, ordered, result + blockIdx.x);
}

// ============================================================ score tables
// (include/tpe_hip.h "Tabulated scoring")
// the job of table block b, fetched in one load round when there are <= 64
// jobs (each lane loads a whole record; the block's is read out by lane)
static_assert(sizeof(tpe_tab_job) == 48, "a table job: three 16-B loads");
__device__ __forceinline__ tpe_tab_job tab_job_at(const tpe_tab_job* __restrict__ J, int n, int b);
__device__ __forceinline__ int tab_job_of(const tpe_tab_job* __restrict__ J, int n, int b) {
  if (n <= 64) {                                    // one load round: the last job starting at or before b
    const int lane = threadIdx.x & 63;
    const unsigned long long m = __ballot(lane < n && J[lane < n ? lane : 0].block0 <= b);
    return m ? 63 - __builtin_clzll(m) : 0;
  }
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (J[m].block0 <= b) lo = m; else hi = m - 1;
  }
  return lo;
}
__device__ __forceinline__ tpe_tab_job tab_job_at(const tpe_tab_job* __restrict__ J, int n, int b) {
  if (n > 64) return J[tab_job_of(J, n, b)];
  const int lane = threadIdx.x & 63;
  const int4* __restrict__ r = reinterpret_cast<const int4*>(J + (lane < n ? lane : 0));
  const int4 a = r[0], c = r[1], d = r[2];
  const unsigned long long m = __ballot(lane < n && c.y <= b);     // block0 = c.y
  const int k = m ? 63 - __builtin_clzll(m) : 0;
  auto rd = [&](int v) { return __builtin_amdgcn_readlane(v, k); };
  tpe_tab_job j;
  j.problem = rd(a.x); j.side = rd(a.y); j.kind = rd(a.z); j.n = rd(a.w);
  j.off = rd(c.x); j.block0 = rd(c.y); j.rows_off = rd(c.z); j.rows_n = rd(c.w);
  j.wide_off = rd(d.x); j.wide_n = rd(d.y);
  j.lo = __int_as_float(rd(d.z)); j.inv = __int_as_float(rd(d.w));
  return j;
}

// Taylor moments of one significant term (v >= cut) into M
__device__ __forceinline__ void add_moments(double (&M)[kTabMoments], float v, float z, float a, float h, float mx,
                                            bool& bad) {
  const float ah = a * h;
  const float B = -2.f * kLn2f * z * ah;
  const float G = -kLn2f * ah * ah;
  if (fabsf(B) > kTaylorBMax || fabsf(G) > kTaylorGMax) { bad = true; return; }
  float e = __builtin_amdgcn_exp2f(v - mx), em1 = 0.f;
  M[0] += (double)e;
#pragma unroll
  for (int k = 1; k < kTabMoments; ++k) {
    const float en = (B * e + 2.f * G * em1) * (1.f / (float)k);
    em1 = e;
    e = en;
    M[k] += (double)e;
  }
}

// one wave: each lane's share of the Taylor moments of a cell centred at c
// (half-width h) from the component rows r0[0, n0) and r1[0, n1) (LDS or
// global; CONTIG: r1 == r0 + n0, read as one array, four rows in flight per
// lane); mx = the cell's largest term (wave-uniform), bad = some lane's
// significant term lies outside the series' convergence box
template <bool CONTIG>
__device__ __forceinline__ void cell_moments(const float4* __restrict__ r0, int n0, const float4* __restrict__ r1,
                                             int n1, float c, float h, double (&M)[kTabMoments], float& mx_out,
                                             bool& bad_out) {
  const int lane = threadIdx.x & 63;
  const int n = n0 + n1;
  auto at = [&](int i) -> float4 { return CONTIG ? r0[i] : (i < n0 ? r0[i] : r1[i - n0]); };
  // pass 1: the largest term at c
  float mx0 = -INFINITY, mx1 = -INFINITY, mx2 = -INFINITY, mx3 = -INFINITY;
  int i = lane;
  for (; i + 192 < n; i += 256) {
    const float4 q0 = at(i), q1 = at(i + 64), q2 = at(i + 128), q3 = at(i + 192);
    float z;
    z = ((c - q0.x) - q0.y) * q0.z; mx0 = fmaxf(mx0, q0.w - z * z);
    z = ((c - q1.x) - q1.y) * q1.z; mx1 = fmaxf(mx1, q1.w - z * z);
    z = ((c - q2.x) - q2.y) * q2.z; mx2 = fmaxf(mx2, q2.w - z * z);
    z = ((c - q3.x) - q3.y) * q3.z; mx3 = fmaxf(mx3, q3.w - z * z);
  }
  for (; i < n; i += 64) {
    const float4 q = at(i);
    const float z = ((c - q.x) - q.y) * q.z;
    mx0 = fmaxf(mx0, q.w - z * z);
  }
  float mx = fmaxf(fmaxf(mx0, mx1), fmaxf(mx2, mx3));
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  // pass 2: Taylor moments (about c, in u = (t - c) / h) of every term within
  // 2^-50 of it; a significant term outside the series' convergence box flags
  // the cell (its candidates are summed exactly)
#pragma unroll
  for (int q = 0; q < kTabMoments; ++q) M[q] = 0.0;
  bool bad = !(mx > -INFINITY);
  const float cut = mx - kTabDrop;
  i = lane;
  for (; i + 192 < n && !bad; i += 256) {
    const float4 q0 = at(i), q1 = at(i + 64), q2 = at(i + 128), q3 = at(i + 192);
    const float z0 = ((c - q0.x) - q0.y) * q0.z, z1 = ((c - q1.x) - q1.y) * q1.z;
    const float z2 = ((c - q2.x) - q2.y) * q2.z, z3 = ((c - q3.x) - q3.y) * q3.z;
    const float v0 = q0.w - z0 * z0, v1 = q1.w - z1 * z1, v2 = q2.w - z2 * z2, v3 = q3.w - z3 * z3;
    if (v0 >= cut) add_moments(M, v0, z0, q0.z, h, mx, bad);
    if (v1 >= cut) add_moments(M, v1, z1, q1.z, h, mx, bad);
    if (v2 >= cut) add_moments(M, v2, z2, q2.z, h, mx, bad);
    if (v3 >= cut) add_moments(M, v3, z3, q3.z, h, mx, bad);
  }
  for (; i < n && !bad; i += 64) {
    const float4 q = at(i);
    const float z = ((c - q.x) - q.y) * q.z;
    const float v = q.w - z * z;
    if (v >= cut) add_moments(M, v, z, q.z, h, mx, bad);
  }
  mx_out = mx;
  bad_out = __ballot(bad) != 0ull;
}

// Chunked passes over LDS-staged rows: rows [64 g, 64 g + 64) form chunk g,
// summarised by meta[g] = {min mu, max mu, min a, max c}.  No term of chunk g
// at c exceeds bound_g = max c - (min a * dist(c, [min mu, max mu]))^2, so a
// pass visits only the chunks whose bound reaches its threshold (a wave-uniform
// set): pass 1 those that could exceed the best term of the most promising
// chunk, pass 2 those that could be within 2^-50 of the maximum.  kChunkSlack
// (log2 units) covers the f32 rounding of the bounds.  Same results as the
// full scan: the skipped terms are below every threshold.
constexpr int kChunkMax = (kTabStageRowsDecl + 63) / 64;
constexpr float kChunkSlack = 1.f;

__device__ __forceinline__ float chunk_bound(const float4 m, float c) {
  const float d = fmaxf(fmaxf(m.x - c, c - m.y), 0.f);
  const float ad = m.z * d;
  return d > 0.f ? m.w - ad * ad : m.w;
}

// {min mu, max mu, min a, max c} of every chunk, by the whole workgroup: 8
// lanes per chunk (8 rows each, consecutive lanes on consecutive rows)
// combined by three xor shuffles (rows past n: the last row again)
__device__ __forceinline__ void chunk_meta_wg(const float4* __restrict__ rows, int n, float4* __restrict__ meta) {
  const int nch = (n + 63) / 64;
  for (int x = (int)threadIdx.x; x < nch * 8; x += (int)blockDim.x) {    // (whole 8-lane groups)
    const int g = x >> 3, s = x & 7;
    const int last = min(n, g * 64 + 64) - 1;
    float lo = INFINITY, hi = -INFINITY, amin = INFINITY, cmax = -INFINITY;
    float4 q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = rows[min(g * 64 + i * 8 + s, last)];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float mu = q[i].x + q[i].y;
      lo = fminf(lo, mu); hi = fmaxf(hi, mu); amin = fminf(amin, q[i].z); cmax = fmaxf(cmax, q[i].w);
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
      lo = fminf(lo, __shfl_xor(lo, off)); hi = fmaxf(hi, __shfl_xor(hi, off));
      amin = fminf(amin, __shfl_xor(amin, off)); cmax = fmaxf(cmax, __shfl_xor(cmax, off));
    }
    if (s == 0) meta[g] = make_float4(lo, hi, amin, cmax);
  }
}

__device__ __forceinline__ float wave_max(float v) {
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  return v;
}

__device__ __forceinline__ void cell_moments_chunked(const float4* __restrict__ rows, int n,
                                                     const float4* __restrict__ meta, float c, float h,
                                                     double (&M)[kTabMoments], float& mx_out, bool& bad_out) {
  const int lane = threadIdx.x & 63;
  const int nch = (n + 63) / 64;
  // bounds of chunks lane and lane + 64 (kChunkMax <= 128)
  const float b0 = lane < nch ? chunk_bound(meta[lane], c) : -INFINITY;
  const float b1 = lane + 64 < nch ? chunk_bound(meta[lane + 64], c) : -INFINITY;
  auto term = [&](int r) -> float {
    const float4 q = rows[r];
    const float z = ((c - q.x) - q.y) * q.z;
    return q.w - z * z;
  };
  // the most promising chunk first: its best term bounds the maximum from below
  const float bmax = wave_max(fmaxf(b0, b1));
  const unsigned long long h0 = __ballot(b0 == bmax), h1 = __ballot(b1 == bmax);
  const int gbest = h0 ? __builtin_ctzll(h0) : 64 + __builtin_ctzll(h1);
  float m = -INFINITY;
  {
    const int r = gbest * 64 + lane;
    if (r < n) m = term(r);
  }
  const float m0 = wave_max(m);
  // pass 1: chunks that could hold a larger term
  for (int half = 0; half < 2; ++half) {
    unsigned long long set = __ballot((half ? b1 : b0) > m0 - kChunkSlack);
    while (set) {
      const int g = half * 64 + __builtin_ctzll(set);
      set &= set - 1;
      if (g == gbest) continue;
      const int r = g * 64 + lane;
      if (r < n) m = fmaxf(m, term(r));
    }
  }
  const float mx = wave_max(m);
  // pass 2: chunks that could hold a term within 2^-50 of the maximum
  bool bad = !(mx > -INFINITY);
  const float cut = mx - kTabDrop;
  for (int half = 0; half < 2 && !__ballot(bad); ++half) {
    unsigned long long set = __ballot((half ? b1 : b0) >= cut - kChunkSlack);
    while (set) {
      const int g = half * 64 + __builtin_ctzll(set);
      set &= set - 1;
      const int r = g * 64 + lane;
      if (r >= n || bad) continue;
      const float4 q = rows[r];
      const float z = ((c - q.x) - q.y) * q.z;
      const float v = q.w - z * z;
      if (v >= cut) add_moments(M, v, z, q.z, h, mx, bad);
    }
  }
  mx_out = mx;
  bad_out = __ballot(bad) != 0ull;
}

// the above rows of a PRUNED mixture (device-fitted) that can matter at c: m0
// (the best term at c among the wide components and c's grid neighbours)
// bounds the cell's largest term from below, so a narrow component with
// |c - mu| > sqrt(narrow_cmax - m0 + 50) / narrow_amin is under 2^-50 of it
__device__ __forceinline__ void pruned_range(const tpe_problem& p, const float4* __restrict__ comp,
                                             const int32_t* __restrict__ grid, float c, int& k0, int& n0) {
  const int lane = threadIdx.x & 63;
  const int32_t* __restrict__ G = grid + p.grid_off;
  float m0 = -INFINITY;
  if (lane < p.wide_len) {
    const float4 q = comp[p.wide_off + lane];
    const float z = ((c - q.x) - q.y) * q.z;
    m0 = q.w - z * z;
  }
  const int gb = (int)fminf(fmaxf(floorf((c - p.grid_lo) * p.grid_inv), 0.f), (float)p.grid_n);
  const int kn = G[gb] - 2 + (lane - 16);
  if (lane >= 16 && lane < 20 && kn >= 0 && kn < p.above_len) {
    const float4 q = comp[p.above_off + kn];
    const float z = ((c - q.x) - q.y) * q.z;
    m0 = fmaxf(m0, q.w - z * z);
  }
  for (int off = 32; off > 0; off >>= 1) m0 = fmaxf(m0, __shfl_xor(m0, off));
  const float R = sqrtf(fmaxf(p.narrow_cmax - m0 + kTabDrop, 0.f)) / p.narrow_amin;
  if (!(m0 > -INFINITY) || !(R < INFINITY)) {
    k0 = p.above_off; n0 = p.above_len;
  } else {
    const float gl = (c - R - p.grid_lo) * p.grid_inv, gh = (c + R - p.grid_lo) * p.grid_inv;
    const int bl = (int)fminf(fmaxf(floorf(gl) - 1.f, 0.f), (float)p.grid_n);
    const int bh = (int)fminf(fmaxf(floorf(gh) + 2.f, 0.f), (float)p.grid_n);
    const int kl = G[bl], kh = max(G[bh], G[bl]);
    k0 = p.above_off + kl; n0 = kh - kl;
  }
  k0 = __builtin_amdgcn_readfirstlane(k0); n0 = __builtin_amdgcn_readfirstlane(n0);
}

// ---------------------------------------------------------------- box moments
// (include/tpe_hip.h "Box moments").  Widths in d = 1 / (fgt_a sqrt(ln 2)):
// a term 2^(c - (a (t - mu))^2) of the narrowest width is 2^c e^-((t - mu) / d)^2.
constexpr int kFgtP = TPE_FGT_P;
constexpr int kFgtJ = kFgtP + kTabMoments - 1;      // Hermite functions h_0 .. h_(P+9)
// Cramer's 1.0865 times sum_(n >= P) (sqrt2 rho)^n / sqrt(n!), rho = 1/2 (a box's
// half-width in d): a box's truncation error is below this times W_b e^(-x^2 / 2)
constexpr double kFgtEps = 1.0865 * 1.0296e-9;
constexpr double kSqrtLn2 = 0.83255461115769775;
static_assert(kFgtP == 16, "kFgtEps is the P = 16 tail");
static_assert(TPE_FGT_BOX_UNITS * 16 >= kFgtP * 8 + 16, "a box record: the moments and four int32");

__device__ __forceinline__ double fgt_width(const tpe_problem& p) { return 1.0 / ((double)p.fgt_a * kSqrtLn2); }

// One wave per box b of a TPE_F_FGT label: its components [k_lo, k_hi) (f64
// means in [fgt_lo + b d, fgt_lo + (b + 1) d)), A_n = sum 2^c y^n / n! over
// those of the narrowest width (y = (mu - centre) / d), the others counted
// (n_odd: the cells sum them directly); wave butterflies, so a record is the
// same every run.  Block (0, job) also writes the label's header: ok when the
// boxes hold every component.  Grid (ceil(fgt_max_boxes / 4), n_tab_jobs).
__global__ __launch_bounds__(256) void k_boxes(const tpe_problem* __restrict__ P, const tpe_tab_job* __restrict__ J,
                                               const float4* __restrict__ comp32, const int32_t* __restrict__ grid,
                                               float4* __restrict__ tab) {
  const tpe_tab_job jb = J[blockIdx.y];
  if (jb.kind != TPE_TAB_CELLS || jb.side != 1) return;
  const tpe_problem& p = P[jb.problem];
  if (!(p.flags & TPE_F_FGT)) return;
  const int lane = threadIdx.x & 63;
  const int b = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const float4* __restrict__ rows = comp32 + p.above_off;
  const int K = p.above_len;
  const double d = fgt_width(p), lo = p.fgt_lo;
  auto mu_of = [&](int k) { const float4 q = rows[k]; return (double)q.x + (double)q.y; };
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const bool ok = K > 0 && mu_of(0) >= lo && mu_of(K - 1) < lo + (double)p.fgt_n * d;
    reinterpret_cast<int*>(tab + p.fgt_off)[0] = ok ? 1 : 0;
  }
  if (b >= p.fgt_n) return;
  // [k_lo, k_hi): lanes 0 and 1 search the two edges, inside the range the
  // fit's grid over the f32 means gives (a bucket either side of the edge's)
  int kb = 0;
  if (lane < 2) {
    const double edge = lo + (double)(b + lane) * d;
    const int32_t* __restrict__ G = grid + p.grid_off;
    int a = 0, z = K;                               // first k with mu_k >= edge
    if (p.grid_inv > 0.f && p.grid_n > 0) {
      const float gf = floorf(((float)edge - p.grid_lo) * p.grid_inv);
      const int gb = (int)fminf(fmaxf(gf, 0.f), (float)(p.grid_n - 1));
      a = G[max(gb - 1, 0)];
      z = G[min(gb + 2, p.grid_n)];
      if (a > 0 && !(mu_of(a - 1) < edge)) a = 0;   // (outside the bucket bounds: search everything)
      if (z < K && mu_of(z) < edge) z = K;
    }
    while (a < z) {
      const int m = (a + z) >> 1;
      if (mu_of(m) < edge) a = m + 1; else z = m;
    }
    kb = a;
  }
  const int k_lo = __shfl(kb, 0), k_hi = __shfl(kb, 1);
  const double centre = lo + ((double)b + 0.5) * d;
  double A[kFgtP];
#pragma unroll
  for (int n = 0; n < kFgtP; ++n) A[n] = 0.0;
  int odd = 0;
  const double id = 1.0 / d;
  // two components per lane in flight (their terms added in index order);
  // sums of 2^c y^n, the 1 / n! applied once to the reduced sums; 2^c from the
  // f32 exp (c is an f32 row value: its own rounding, up to 2^-19 at |c| >= 16,
  // is larger than the f32 exp's 2^-23)
  // (the next pair's rows loaded before this pair's terms: one row latency per
  // pair instead of one on every pair's critical path)
  float4 n0 = make_float4(0.f, 0.f, 0.f, 0.f), n1 = n0;
  if (k_lo + lane < k_hi) {
    n0 = rows[k_lo + lane];
    n1 = rows[k_lo + lane + 64 < k_hi ? k_lo + lane + 64 : k_lo + lane];
  }
  for (int k = k_lo + lane; k < k_hi; k += 128) {
    const bool two = k + 64 < k_hi;
    const float4 q0 = n0, q1 = n1;
    if (k + 128 < k_hi) {
      n0 = rows[k + 128];
      n1 = rows[k + 192 < k_hi ? k + 192 : k + 128];
    }
    const bool u0 = q0.w > -INFINITY && q0.z == p.fgt_a, u1 = two && q1.w > -INFINITY && q1.z == p.fgt_a;
    odd += (q0.w > -INFINITY && q0.z != p.fgt_a) + (two && q1.w > -INFINITY && q1.z != p.fgt_a);
    const double y0 = ((double)q0.x + (double)q0.y - centre) * id, y1 = ((double)q1.x + (double)q1.y - centre) * id;
    double t0 = u0 ? (double)exp2f(q0.w) : 0.0, t1 = u1 ? (double)exp2f(q1.w) : 0.0;
    A[0] += t0;
    A[0] += t1;
#pragma unroll
    for (int n = 1; n < kFgtP; ++n) {
      t0 *= y0;
      t1 *= y1;
      A[n] += t0;
      A[n] += t1;
    }
  }
#pragma unroll
  for (int n = 0; n < kFgtP; ++n)
    for (int off = 32; off > 0; off >>= 1) A[n] += __shfl_xor(A[n], off);
  for (int off = 32; off > 0; off >>= 1) odd += __shfl_xor(odd, off);
  double* rec = reinterpret_cast<double*>(tab + p.fgt_off + 1 + (int64_t)b * TPE_FGT_BOX_UNITS);
  if (lane < kFgtP) {
    double v = A[0], f = 1.0;                       // f = 1 / lane!
#pragma unroll
    for (int n = 1; n < kFgtP; ++n) {
      v = lane == n ? A[n] : v;
      f = lane >= n ? f / (double)n : f;
    }
    rec[lane] = v * f;
  }
  if (lane == 0) {
    int* ri = reinterpret_cast<int*>(rec + kFgtP);
    ri[0] = k_lo; ri[1] = k_hi; ri[2] = odd; ri[3] = 0;
  }
}

// Cells of the TPE_F_FGT labels' above sides, four per wave (16 lanes each):
// a cell's Taylor moments from the box moments within reach (one box per lane,
// Hermite -> Taylor, reduced over the 16 lanes), plus the wide list and the
// boxes' odd components summed directly at the shift mx = log2 of the boxes'
// sum at the centre.  A cell is built directly instead (pruned window, the
// whole wave) when the label's boxes do not hold every component, the sum is
// not positive, or the truncation bound (boxes within reach, Cramer) plus the
// bound on the boxes out of reach (K e^-(R - 1/2)^2) exceeds 2^-25 of the sum
// (the cells' own Taylor truncation is 4e-8 relative).  Grid
// (ceil(fgt_max_cells / 32), n_tab_jobs), 8 waves per block; the other jobs'
// blocks return at once (k_tables builds those).
constexpr int kFgtCellsPerWave = 4;
constexpr int kFgtLanes = 64 / kFgtCellsPerWave;     // boxes within reach: at most 16
constexpr double kFgtReach = 7.0;                    // box centres within 7 widths of the cell centre
constexpr double kFgtFar = 2.35e-19;                 // e^-(7 - 1/2)^2: a box out of reach, per unit weight

template <int W>
__device__ __forceinline__ double group_sum(double v) {          // over aligned groups of W lanes
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// v of the lane N below within each row of 16 lanes (DPP row_shr: no LDS
// permute; the row's first N lanes read 0)
template <int N>
__device__ __forceinline__ double row_shr(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x110 + N, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x110 + N, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// the sum over each aligned row of 16 lanes, complete in the row's last lane
// (a fixed order: the same bits every run)
__device__ __forceinline__ double row_sum_last(double v) {
  v += row_shr<8>(v);
  v += row_shr<4>(v);
  v += row_shr<2>(v);
  v += row_shr<1>(v);
  return v;
}
static_assert(kFgtLanes == 16, "a cell's lanes are one DPP row");

// (six waves a SIMD: 80 VGPRs, 6 of them spilled — 373-391 us on config 5
// against 410-423 at the four waves its 105 VGPRs allowed, tools/g21.sh)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(6))) void k_cells_fgt(const tpe_problem* __restrict__ P,
                                                   const tpe_tab_job* __restrict__ J,
                                                   const float4* __restrict__ comp32,
                                                   const int32_t* __restrict__ grid, float4* __restrict__ tab,
                                                   bool all_exact) {
  const tpe_tab_job jb = J[blockIdx.y];
  if (jb.kind != TPE_TAB_CELLS || jb.side != 1) return;
  const tpe_problem& p = P[jb.problem];
  if (!(p.flags & TPE_F_FGT)) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane / kFgtLanes, gl = lane % kFgtLanes;            // cell of the wave, lane in its group
  const int j0 = ((int)blockIdx.x * 8 + wave) * kFgtCellsPerWave;     // the wave's first cell
  if (j0 >= jb.n) return;                                              // (wave-uniform)
  const int j = j0 + g;
  const bool live = j < jb.n;
  const bool boxes_ok = reinterpret_cast<const int*>(tab + p.fgt_off)[0] == 1;
  const float w = 1.f / p.tab_inv[1];
  const float c = __builtin_fmaf((float)j + 0.5f, w, p.tab_lo[1]);   // as cell_log2_lds forms them
  const float h = 0.5f * w;
  const double d = fgt_width(p), cd = (double)c;
  double B[kTabMoments];
#pragma unroll
  for (int m = 0; m < kTabMoments; ++m) B[m] = 0.0;
  double err = 0.0;
  const double pos = (cd - p.fgt_lo) / d - 0.5;                      // the cell centre in box-centre units
  const int b0 = max(0, (int)ceil(pos - kFgtReach)), b1 = min(p.fgt_n - 1, (int)floor(pos + kFgtReach));
  if (live && boxes_ok && gl <= b1 - b0) {
    const int b = b0 + gl;
    const double* __restrict__ rec = reinterpret_cast<const double*>(tab + p.fgt_off + 1 + (int64_t)b * TPE_FGT_BOX_UNITS);
    const double x = (cd - (p.fgt_lo + ((double)b + 0.5) * d)) / d;
    const double eh = exp(-0.5 * x * x), e = eh * eh;
    double A[kFgtP];
#pragma unroll
    for (int n = 0; n < kFgtP; ++n) A[n] = rec[n];
    // B_m = sum_n A_n h_(n+m)(x), h_j = e^-x^2 H_j(x) by its recurrence, made
    // one j at a time and added to every B_m it feeds (n = j - m ascending for
    // each m: the same sums in the same order as a table of every h_j, without
    // the 27 doubles that table held: occupancy)
    double h0 = e, h1 = 2.0 * x * e;
#pragma unroll
    for (int jj = 0; jj <= kFgtJ; ++jj) {
      const double hv = jj == 0 ? h0 : h1;
#pragma unroll
      for (int m = 0; m < kTabMoments; ++m)
        if (jj - m >= 0 && jj - m < kFgtP) B[m] += A[jj - m] * hv;
      if (jj >= 1 && jj < kFgtJ) {                    // h_(jj+1) = 2 x h_jj - 2 jj h_(jj-1)
        const double h2 = 2.0 * x * h1 - 2.0 * (double)jj * h0;
        h0 = h1;
        h1 = h2;
      }
    }
    err = A[0] * eh * kFgtEps;
  }
  // the cell's sums in its row's last lane; S0 and the error bound broadcast
#pragma unroll
  for (int m = 0; m < kTabMoments; ++m) B[m] = row_sum_last(B[m]);
  const int last = g * kFgtLanes + kFgtLanes - 1;
  err = __shfl(row_sum_last(err), last) + (double)p.above_len * kFgtFar;
  const double S0 = __shfl(B[0], last);
  const bool ok = live && boxes_ok && S0 > 0.0 && err <= S0 * 0x1p-25;   // (group-uniform)
  float* row = reinterpret_cast<float*>(tab + jb.off + TPE_TAB_ROW_UNITS * j);
  if (ok) {
    const float mx = (float)log2(S0);
    double M[kTabMoments];
#pragma unroll
    for (int m = 0; m < kTabMoments; ++m) M[m] = 0.0;
    if (gl == kFgtLanes - 1) {   // the boxes' part in u = (t - c) / h: B_m (-1)^m / m! (h / d)^m 2^-mx
      const double r = (double)h / d;
      double f = exp2(-(double)mx);
#pragma unroll
      for (int m = 0; m < kTabMoments; ++m) {
        M[m] = B[m] * f;
        f *= -r / (double)(m + 1);
      }
    }
    // directly: the wide list and the boxes' odd components (rare)
    bool bad = false;
    const float cut = mx - kTabDrop;
    for (int i = gl; i < p.wide_len; i += kFgtLanes) {
      const float4 q = comp32[p.wide_off + i];
      const float z = ((c - q.x) - q.y) * q.z;
      const float v = q.w - z * z;
      if (v >= cut) add_moments(M, v, z, q.z, h, mx, bad);
    }
    // odd components reach as far as their own width: boxes within 7 of the
    // label's widest non-wide width (narrow_amin) hold every one that can matter
    const double ro = kFgtReach * fmax((double)p.fgt_a / (double)p.narrow_amin, 1.0) + 1.0;
    const int ob0 = max(0, (int)ceil(pos - ro)), ob1 = min(p.fgt_n - 1, (int)floor(pos + ro));
    for (int bb = ob0; bb <= ob1; bb += kFgtLanes) {
      int no = 0, lo_k = 0, hi_k = 0;
      if (bb + gl <= ob1) {
        const int* __restrict__ ri = reinterpret_cast<const int*>(
            reinterpret_cast<const double*>(tab + p.fgt_off + 1 + (int64_t)(bb + gl) * TPE_FGT_BOX_UNITS) + kFgtP);
        lo_k = ri[0]; hi_k = ri[1]; no = ri[2];
      }
      unsigned long long with_odd = (__ballot(no > 0) >> (g * kFgtLanes)) & ((1ull << kFgtLanes) - 1);
      while (with_odd) {
        const int src = g * kFgtLanes + __builtin_ctzll(with_odd);
        with_odd &= with_odd - 1;
        const int k0 = __shfl(lo_k, src), k1 = __shfl(hi_k, src);
        for (int k = k0 + gl; k < k1; k += kFgtLanes) {
          const float4 q = comp32[p.above_off + k];
          if (!(q.w > -INFINITY) || q.z == p.fgt_a) continue;
          const float z = ((c - q.x) - q.y) * q.z;
          const float v = q.w - z * z;
          if (v >= cut) add_moments(M, v, z, q.z, h, mx, bad);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < kTabMoments; ++m) M[m] = row_sum_last(M[m]);
    bad = ((__ballot(bad) >> (g * kFgtLanes)) & 0xFFFFull) != 0;
    if (gl == kFgtLanes - 1) {                     // the row from the lane holding the sums
      static_assert(kTabMoments == 11 && TPE_TAB_ROW_UNITS == 3, "a moment row: 11 moments and the shift");
      float4* r4 = reinterpret_cast<float4*>(row);
      r4[0] = make_float4((float)M[0], (float)M[1], (float)M[2], (float)M[3]);
      r4[1] = make_float4((float)M[4], (float)M[5], (float)M[6], (float)M[7]);
      r4[2] = make_float4((float)M[8], (float)M[9], (float)M[10], bad || all_exact ? NAN : mx);
    }
  }
  // the cells the boxes cannot build: directly, the whole wave per cell
  const unsigned long long direct = __ballot(live && !ok && gl == 0);
  for (int q = 0; q < kFgtCellsPerWave; ++q) {
    if (!((direct >> (q * kFgtLanes)) & 1ull)) continue;
    const int jq = j0 + q;
    const float cq = __builtin_fmaf((float)jq + 0.5f, w, p.tab_lo[1]);
    double M[kTabMoments];
#pragma unroll
    for (int m = 0; m < kTabMoments; ++m) M[m] = 0.0;
    float mx = -INFINITY;
    bool bad = false;
    int kk, nn;
    pruned_range(p, comp32, grid, cq, kk, nn);
    cell_moments<false>(comp32 + kk, nn, comp32 + p.wide_off, p.wide_len, cq, h, M, mx, bad);
#pragma unroll
    for (int m = 0; m < kTabMoments; ++m) M[m] = group_sum<64>(M[m]);
    float out = 0.f;
#pragma unroll
    for (int m = 0; m < kTabMoments; ++m) out = lane == m ? (float)M[m] : out;
    if (lane == kTabMoments) out = bad || all_exact ? NAN : mx;
    float* rq = reinterpret_cast<float*>(tab + jb.off + TPE_TAB_ROW_UNITS * jq);
    if (lane <= kTabMoments) rq[lane] = out;
  }
}

// one workgroup: {l, g} of lattice value lat_lo + j of a quantized problem, the
// reference's per-component mass terms (tpe.py:147-159 / :285-298) summed in a
// fixed order (thread-strided, a butterfly per wave, the waves' partials in
// wave order) — every wave of the block takes a share of the components (the
// two f64 erf per term make a row long for one wave)
template <bool LOG>
__device__ void lattice_row(const tpe_problem& p, int j, const double4* __restrict__ comp64,
                            double2* __restrict__ rows, double* __restrict__ lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const double x = (double)(p.lat_lo + (int64_t)j) * p.q;
  double tu, tl;
  q_bounds(p, x, tu, tl);
  double sb = 0.0, sa = 0.0;
  for (int k = threadIdx.x; k < p.below_len; k += blockDim.x) sb += qterm<LOG>(comp64[p.below_off + k], tu, tl);
  for (int k = threadIdx.x; k < p.above_len; k += blockDim.x) sa += qterm<LOG>(comp64[p.above_off + k], tu, tl);
  for (int off = 32; off > 0; off >>= 1) { sb += __shfl_xor(sb, off); sa += __shfl_xor(sa, off); }
  if (lane == 0) { lds[2 * wave] = sb; lds[2 * wave + 1] = sa; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double b = 0.0, a = 0.0;
    for (int w = 0; w < nw; ++w) { b += lds[2 * w]; a += lds[2 * w + 1]; }
    rows[j] = make_double2(log(b) + p.below_base, log(a) + p.above_base);
  }
}

// np.round(x / q) of a device draw with coordinate t (k_sample_tab's lattice pass)
__device__ __forceinline__ double lattice_qidx(const tpe_problem& p, float t) {
  const double xu = p.family == TPE_FAM_QLOGGAUSS ? exp((double)t) : (double)t;
  return rint(xu / p.q);
}
// f32 order as an unsigned order (and back)
__device__ __forceinline__ uint32_t f32_okey(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float f32_from_okey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// entry threshold of lattice row m (wave-collective, lane 0 writes thr[m]): the
// smallest f32 coordinate t in the clip range [lo_f, hi_f] whose value
// np.round(x / q) is at least lat_lo + m (lo_f when every t is; +inf when none
// is), so a draw t takes row #{m : thr_m <= t} - 1 (k_sample_fast).  The value
// is non-decreasing in t (consecutive f32 coordinates are far more than an
// ulp of exp apart), so a 64-ary search over the f32 order finds it exactly:
// each round's lanes test 64 evenly spaced points, ~6 rounds.
__device__ void lattice_thresh(const tpe_problem& p, int m, float* __restrict__ thr) {
  const int lane = threadIdx.x & 63;
  float lo_f, hi_f;
  f32_bounds(p, lo_f, hi_f);
  const double target = (double)(p.lat_lo + (int64_t)m);
  float T;
  if (lattice_qidx(p, lo_f) >= target) {
    T = lo_f;
  } else if (!(lattice_qidx(p, hi_f) >= target)) {
    T = INFINITY;
  } else {
    uint32_t a = f32_okey(lo_f), b = f32_okey(hi_f);       // below a: no; at b: yes
    while (b - a > 1u) {
      const uint64_t step = ((uint64_t)(b - a) + 63) / 64;
      const uint64_t kk = (uint64_t)a + (uint64_t)(lane + 1) * step;
      const uint32_t k = kk >= (uint64_t)b ? b : (uint32_t)kk;      // (lane 63 tests b: always yes)
      const unsigned long long yes = __ballot(lattice_qidx(p, f32_from_okey(k)) >= target);
      const int f = (int)__builtin_ctzll(yes);
      const uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)k, f);
      const uint32_t na = f > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)k, f - 1) : a;
      a = na;
      b = nb;
    }
    T = f32_from_okey(b);
  }
  if (lane == 0) thr[m] = T;
}

// ---- TPE_F_LOGPOLY rows (include/tpe_hip.h, "Tabulated scoring") ----
// nodes: the 6 Chebyshev points cos((2i + 1) pi / 12) of [-1, 1] (interpolation),
// then the check points 0, 1/2, -1/2, 1, -1; kLpA: monomial coefficients of the
// degree-5 interpolant from its values at the 6 nodes (the inverse Vandermonde)
__constant__ double kLpNode[11] = {0.96592582628906831, 0.70710678118654757, 0.25881904510252074, -0.25881904510252063, -0.70710678118654746, -0.9659258262890682, 0, 0.5, -0.5, 1, -1};
__constant__ double kLpA[6][6] = {
    {0.044658198738520241, -0.1666666666666663, 0.62200846792814679, 0.62200846792814635, -0.16666666666666655, 0.04465819873852047},
    {0.046233569414010529, -0.23570226039551737, 2.4032561733691682, -2.4032561733691673, 0.2357022603955134, -0.046233569414008954},
    {-0.75598306414370686, 2.6666666666666647, -1.9106836025229559, -1.9106836025229608, 2.666666666666667, -0.75598306414370731},
    {-0.7826512591014102, 3.771236166328257, -7.3823145501758516, 7.3823145501758454, -3.7712361663282445, 0.78265125910140476},
    {1.3333333333333324, -2.6666666666666647, 1.3333333333333304, 1.333333333333335, -2.666666666666667, 1.3333333333333333},
    {1.3803682405467783, -3.7712361663282552, 5.1516044068750295, -5.1516044068750251, 3.7712361663282468, -1.3803682405467748}};
constexpr double kLpTol = 5e-7;        // |fit - value| <= kLpTol (1 + |log2 s|) at the check points
// a side of at most this many component rows (the below side: <= 26) gets its
// log-polynomials from direct sums at the nodes, one cell row per thread
// (tpe_host.cpp kLpDirectRows: its job's blocks hold 512 rows, not 8)
constexpr int kLpDirectRows = 64;
constexpr int kLpRowsPerWave = 5;      // (5 rows x 11 nodes = 55 lanes; tpe_host.cpp kLpRowsPerWave)

// log2 of a positive normal double to ~1e-7 absolute (exponent + f32 log2 of the mantissa)
__device__ __forceinline__ double log2_fast(double x) {
  int e;
  const double m = frexp(x, &e);                  // x = m 2^e, m in [0.5, 1)
  return (double)e + (double)__log2f((float)m);
}

// one side's log-polynomial from its reduced cell moments (wave-collective):
// lane 4q holds moment q's f64 sum; m = the cell's log2 shift; flagged: the
// side takes the exact sum for its candidates.  Lanes 0..5 write c_0..c_5 to
// out[0], out[2], .. out[10] (f32; the row interleaves the two sides), NaN in
// all six when the side is flagged or fails the check.
__device__ __forceinline__ void logpoly_side(double sum, float m, bool flagged, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  double M[kTabMoments];
#pragma unroll
  for (int q = 0; q < kTabMoments; ++q) M[q] = __shfl(sum, 4 * q);
  // the moment series and its log2 at this lane's node (lanes 0..10)
  const double u = kLpNode[lane < 11 ? lane : 0];
  double sr = M[kTabMoments - 1];
#pragma unroll
  for (int q = kTabMoments - 2; q >= 0; --q) sr = __builtin_fma(sr, u, M[q]);
  const bool pos = sr > 0.0 && sr < INFINITY;
  const double y = (double)m + log2_fast(pos ? sr : 1.0);
  // interpolant coefficients (lanes 0..5) and its value at every node
  const int r = lane < 6 ? lane : 0;
  double c = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) c = __builtin_fma(kLpA[r][i], __shfl(y, i), c);
  double C[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) C[k] = __shfl(c, k);
  double pv = C[5];
#pragma unroll
  for (int k = 4; k >= 0; --k) pv = __builtin_fma(pv, u, C[k]);
  const bool bad = lane < 11 && (!pos || !(fabs(pv - y) <= kLpTol * (1.0 + fabs(y))));
  const bool any = __ballot(bad) != 0ull || flagged || !(m == m);
  if (lane < 6) out[2 * lane] = any ? NAN : (float)c;         // (the sides interleaved: {b_k, a_k} at 2k)
}

// a moment-cell side of at most this many component rows (the below side: <=
// 26) is summed directly, kMomCellsPerWave cell rows per wave, 16 lanes each
// (tpe_host.cpp kMomDirectRows: its job's blocks hold 32 rows, not 8)
constexpr int kMomDirectRows = 64;
constexpr int kMomCellsPerWave = 4;

// the max over each aligned row of 16 lanes, in every lane of the row (DPP:
// quad xor 1 and 2, then row rotations by 4 and 8)
__device__ __forceinline__ float row_max_all(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false)));
  return v;
}

// 512-thread workgroups, one wave per cell row / lattice value
// (TPE_TAB_PER_BLOCK per workgroup).  A cell job's workgroup first stages its
// side's component rows in LDS (unless pruned or too many), so both passes of
// every cell read LDS only.
constexpr int kTabTblThreads = 64 * TPE_TAB_PER_BLOCK;
constexpr int kTabStageRows = kTabStageRowsDecl;    // 64 KiB of float4 rows
static_assert(TPE_TAB_PER_BLOCK * kTabMoments * 64 * 8 <= kTabStageRows * 16, "moment reduction fits the staging LDS");
__global__ __launch_bounds__(kTabTblThreads) void k_tables(const tpe_problem* __restrict__ P,
                                                          const tpe_tab_job* __restrict__ J, int n_jobs,
                                                          const float4* __restrict__ comp32,
                                                          const double4* __restrict__ comp64,
                                                          const int32_t* __restrict__ grid,
                                                          float4* __restrict__ tab, bool all_exact,
                                                          int tab_blocks, const double* __restrict__ samp,
                                                          int lazy_ok, tpe_result* __restrict__ result) {
  __shared__ float4 rows_lds[kTabStageRows];
  if ((int)blockIdx.x >= tab_blocks) {
    // early selection: one block per problem selects a lazy categorical
    // problem right here (it needs no tables)
    const tpe_problem& q = P[(int)blockIdx.x - tab_blocks];
    if (lazy_ok && lazy_eligible(q)) select_cat_lazy(q, samp, comp64, result + ((int)blockIdx.x - tab_blocks));
    return;
  }
  const tpe_tab_job jb = tab_job_at(J, n_jobs, (int)blockIdx.x);
  const tpe_problem& p = P[jb.problem];
  const int b = (int)blockIdx.x - jb.block0;
  const int j = b * TPE_TAB_PER_BLOCK + (int)(threadIdx.x >> 6);
  if (jb.kind == TPE_TAB_LOGPOLY && jb.rows_n >= 0 && jb.rows_n + jb.wide_n <= kLpDirectRows) {
    // a short side (the below mixture): its log-polynomials from the exact
    // max-shifted sums at the nodes, no moments — a wave holds kLpRowsPerWave
    // cell rows, one lane per (row, node); node positions and exponents in f64
    // (an f32 t would move a node of a narrow cell by a sizeable part of it)
    const int nr = jb.rows_n + jb.wide_n;
    if ((int)threadIdx.x < nr)
      rows_lds[threadIdx.x] = (int)threadIdx.x < jb.rows_n ? comp32[jb.rows_off + threadIdx.x]
                                                           : comp32[jb.wide_off + threadIdx.x - jb.rows_n];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int rl = lane / 11, k = lane - 11 * rl;               // (row of the wave, node)
    const int jr = (b * TPE_TAB_PER_BLOCK + wave) * kLpRowsPerWave + rl;
    const bool live = rl < kLpRowsPerWave && jr < jb.n;
    const float w = 1.f / jb.inv;
    const double c = (double)__builtin_fmaf((float)(live ? jr : 0) + 0.5f, w, jb.lo);   // (as the sample stage forms it)
    const double h = 0.5 * (double)w;
    const double t = c + h * kLpNode[live ? k : 0];
    double m = -INFINITY;
    for (int q = 0; q < nr; ++q) {
      const float4 r = rows_lds[q];
      const double z = ((t - (double)r.x) - (double)r.y) * (double)r.z;
      m = fmax(m, (double)r.w - z * z);
    }
    double sm = 0.0;
    for (int q = 0; q < nr; ++q) {
      const float4 r = rows_lds[q];
      const double z = ((t - (double)r.x) - (double)r.y) * (double)r.z;
      sm += (double)__builtin_amdgcn_exp2f((float)((double)r.w - z * z - m));
    }
    const bool ok = !all_exact && m > -INFINITY && m < INFINITY && sm > 0.0;
    const double y = m + log2_fast(sm > 0.0 ? sm : 1.0);
    // the row's interpolant: lane (rl, k < 6) forms c_k, lanes (rl, k >= 6) check it
    const int b0 = 11 * (rl < kLpRowsPerWave ? rl : 0);
    double cf = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) cf = __builtin_fma(kLpA[k < 6 ? k : 0][i], __shfl(y, b0 + i), cf);
    double pv = __shfl(cf, b0 + 5);
#pragma unroll
    for (int n = 4; n >= 0; --n) pv = __builtin_fma(pv, kLpNode[live ? k : 0], __shfl(cf, b0 + n));
    const bool bad = live && (!ok || (k >= 6 && !(fabs(pv - y) <= kLpTol * (1.0 + fabs(y)))));
    const unsigned long long bm = __ballot(bad);
    const bool row_bad = rl < kLpRowsPerWave && ((bm >> b0) & 0x7FFull) != 0ull;
    if (live && k < 6)
      reinterpret_cast<float*>(tab + jb.off + TPE_TAB_ROW_UNITS * jr)[2 * k + jb.side] = row_bad ? NAN : (float)cf;
    return;
  }
  if (jb.kind == TPE_TAB_CELLS && jb.rows_n >= 0 && jb.rows_n + jb.wide_n <= kMomDirectRows) {
    // a short moment side (the below mixture of a box-moment label): a cell
    // per 16 lanes, its rows' passes as cell_moments makes them (the largest
    // term, then the moments of the terms within 2^-kTabDrop of it), the sums
    // by DPP row shifts into the row's last lane, which writes the row
    const int nr = jb.rows_n + jb.wide_n;
    if ((int)threadIdx.x < nr)
      rows_lds[threadIdx.x] = (int)threadIdx.x < jb.rows_n ? comp32[jb.rows_off + threadIdx.x]
                                                           : comp32[jb.wide_off + threadIdx.x - jb.rows_n];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, gl = lane & 15;
    const int jr = (b * TPE_TAB_PER_BLOCK + wave) * kMomCellsPerWave + g;
    const bool live = jr < jb.n;
    const float w = 1.f / jb.inv;
    const float c = __builtin_fmaf((float)(live ? jr : 0) + 0.5f, w, jb.lo);   // as cell_log2_lds forms it
    const float h = 0.5f * w;
    float mx = -INFINITY;
    for (int q = gl; q < nr; q += 16) {
      const float4 r = rows_lds[q];
      const float z = ((c - r.x) - r.y) * r.z;
      mx = fmaxf(mx, r.w - z * z);
    }
    mx = row_max_all(mx);
    double M[kTabMoments];
#pragma unroll
    for (int q = 0; q < kTabMoments; ++q) M[q] = 0.0;
    bool bad = !(mx > -INFINITY);
    const float cut = mx - kTabDrop;
    for (int q = gl; q < nr && !bad; q += 16) {
      const float4 r = rows_lds[q];
      const float z = ((c - r.x) - r.y) * r.z;
      const float v = r.w - z * z;
      if (v >= cut) add_moments(M, v, z, r.z, h, mx, bad);
    }
#pragma unroll
    for (int q = 0; q < kTabMoments; ++q) M[q] = row_sum_last(M[q]);
    bad = ((__ballot(bad) >> (g * 16)) & 0xFFFFull) != 0;
    if (live && gl == 15) {
      float4* r4 = reinterpret_cast<float4*>(tab + jb.off + TPE_TAB_ROW_UNITS * jr);
      r4[0] = make_float4((float)M[0], (float)M[1], (float)M[2], (float)M[3]);
      r4[1] = make_float4((float)M[4], (float)M[5], (float)M[6], (float)M[7]);
      r4[2] = make_float4((float)M[8], (float)M[9], (float)M[10], bad || all_exact ? NAN : mx);
    }
    return;
  }
  if (jb.kind == TPE_TAB_CELLS || jb.kind == TPE_TAB_LOGPOLY) {
    // (the job carries the rows and geometry: no problem row on this path, but
    // for a device-fitted above side, rows_n < 0, whose fit wrote them there)
    [[maybe_unused]] const int side = jb.side;
    const bool pruned = jb.rows_n < 0;
    const int k0 = pruned ? p.above_off : jb.rows_off, n0 = pruned ? p.above_len : jb.rows_n;
    const int k1 = pruned ? p.wide_off : jb.wide_off, n1 = pruned ? p.wide_len : jb.wide_n;
    const bool stage = !pruned && n0 + n1 <= kTabStageRows;      // workgroup-uniform
    __shared__ float4 meta_lds[kChunkMax];
    if (stage) {
      // the rows by LDS-DMA: every round's loads issued before the one wait
      // (rounds past the rows: clamped loads into unused slots)
      const int nr = n0 + n1, wv = (int)(threadIdx.x >> 6);
      for (int u = 0; u * kTabTblThreads < nr; ++u) {
        const int q = min(u * kTabTblThreads + (int)threadIdx.x, nr - 1);
        const float4* src = q < n0 ? comp32 + k0 + q : comp32 + k1 + (q - n0);
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(rows_lds + u * kTabTblThreads + 64 * wv),
                                         16, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      chunk_meta_wg(rows_lds, nr, meta_lds);
      __syncthreads();
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool live = j < jb.n;                                   // wave-uniform
    // cell centre and half-width exactly as the sample stage forms them (cell_log2_lds)
    const float w = 1.f / jb.inv;
    const float c = __builtin_fmaf((float)j + 0.5f, w, jb.lo);
    const float h = 0.5f * w;
    double M[kTabMoments];
#pragma unroll
    for (int q = 0; q < kTabMoments; ++q) M[q] = 0.0;
    float mx = -INFINITY;
    bool bad = false;
    if (live) {
      if (stage) {
        cell_moments_chunked(rows_lds, n0 + n1, meta_lds, c, h, M, mx, bad);
      } else if (!pruned) {
        cell_moments<false>(comp32 + k0, n0, comp32 + k1, n1, c, h, M, mx, bad);
      } else {
        int kk, nn;
        pruned_range(p, comp32, grid, c, kk, nn);
        cell_moments<false>(comp32 + kk, nn, comp32 + k1, n1, c, h, M, mx, bad);
      }
    }
    // every wave is past its passes: the staged rows' LDS takes each wave's
    // per-lane moments, and 4 lanes per moment sum them (16 lanes each, then
    // two shuffles) — no 64-lane butterflies of 11 doubles
    __syncthreads();
    double* red = reinterpret_cast<double*>(rows_lds) + wave * (kTabMoments * 64);
    if (!live) return;
#pragma unroll
    for (int q = 0; q < kTabMoments; ++q) red[q * 64 + lane] = M[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int q = lane >> 2, part = lane & 3;
    double sum = 0.0;
    if (q < kTabMoments)
      for (int i = 0; i < 16; ++i) sum += red[q * 64 + part * 16 + i];
    sum += __shfl_xor(sum, 1);
    sum += __shfl_xor(sum, 2);
    float* row = reinterpret_cast<float*>(tab + jb.off + TPE_TAB_ROW_UNITS * j);
    if (jb.kind == TPE_TAB_LOGPOLY) {
      // this side's half of the label's row: its log-polynomial (lane 11's
      // shift and flag, as the moment row takes them)
      const float m = __shfl(mx, kTabMoments);
      const bool fl = __shfl(bad || all_exact ? 1 : 0, kTabMoments) != 0;
      logpoly_side(sum, m, fl, row + jb.side);
      return;
    }
    float val = 0.f;
    if (part == 0 && q < kTabMoments) val = (float)sum;
    // row lanes: moment q from lane 4q, then the shift mx (NaN: the cell is flagged)
    const float mv = __shfl(val, 4 * (lane < kTabMoments ? lane : 0));
    float out = lane < kTabMoments ? mv : 0.f;
    if (lane == kTabMoments) out = bad || all_exact ? NAN : mx;
    if (lane <= kTabMoments) row[lane] = out;
  } else if (b < jb.n) {                             // lattice: block b computes value b
    double* lds = reinterpret_cast<double*>(rows_lds);
    if (p.family == TPE_FAM_QLOGGAUSS) lattice_row<true>(p, b, comp64, reinterpret_cast<double2*>(tab + jb.off), lds);
    else lattice_row<false>(p, b, comp64, reinterpret_cast<double2*>(tab + jb.off), lds);
    // ... and its entry threshold after the rows (the last block: the exit too)
    if (threadIdx.x < 64) {
      float* thr = reinterpret_cast<float*>(tab + jb.off + jb.n);
      lattice_thresh(p, b, thr);
      if (b == jb.n - 1) lattice_thresh(p, jb.n, thr);
    }
  }
}

// ============================================================ shard combine on the device
// A candidate-sharded level (tpe_suggest_tree over RCCL, include/tpe_hip.h
// "Candidate-shard exchange") combined without a host round trip: the
// early-selection run records (device memory) reduced per problem straight
// into this rank's exchange slot, an in-place ncclAllGather, and k_combine
// reducing the ranks' records per problem (np.argmax order: NaN, score, lowest
// global index, tpe.py:749-759) into the host-visible results, the worst
// status beside them — one stream synchronise per level.
constexpr int kCombThreads = 256;

// (host-written pinned memory: system-scope loads, as k_upload)
__device__ __forceinline__ int32_t sys_load_i32(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one wave per problem: span[2p] = the list position of its first tabulated
// tile, span[2p + 1] = its tabulated tiles (0: its result is res_dev[p]); a
// run starts at the problem's first position and at every multiple of `per`
// (the sample stage's workgroup partition); list = NULL: the identity.
// span = NULL (a level of at most kRunsDevMax problems): the spans from the
// packer's layout instead — every problem tpp tiles, the tile list the
// tabulated problems' tiles in problem order — so no host memory is read and
// a run's first tile is p * tpp + (pos - a): the wave's chain is one load of
// the problems' modes, one of its runs' records, the record itself carried
// through the reduction
constexpr int64_t kRunsDevMax = 256;
__global__ __launch_bounds__(kCombThreads) void k_runs_reduce(const int32_t* __restrict__ span,
                                                               const int32_t* __restrict__ list, int per,
                                                               const tpe_problem* __restrict__ prob, int tpp,
                                                               const tpe_result* __restrict__ run_best,
                                                               const tpe_result* __restrict__ res_dev, int64_t P,
                                                               unsigned char* __restrict__ slot, int32_t status,
                                                               tpe_result* __restrict__ out1,
                                                               int32_t* __restrict__ status1) {
  // (one rank: the gather is the identity and the combine a copy — the records
  // go straight to the results, out1 / status1, instead of the slot)
  if (blockIdx.x == 0 && threadIdx.x == 0) *(status1 ? status1 : reinterpret_cast<int32_t*>(slot)) = status;
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * (kCombThreads / 64) + (threadIdx.x >> 6);
  if (p >= P) return;
  tpe_result* dst = out1 ? out1 + p : reinterpret_cast<tpe_result*>(slot + TPE_EXCHANGE_HEADER) + p;
  int32_t a, n;
  if (span) {
    a = sys_load_i32(span + 2 * p);
    n = sys_load_i32(span + 2 * p + 1);
  } else {
    int before = 0;                                // tabulated problems before p
    for (int64_t q0 = 0; q0 < p; q0 += 64) {
      const int64_t q = q0 + lane;
      before += __popcll(__ballot(q < p && prob[q].tab_mode != TPE_TAB_NONE));
    }
    a = before * tpp;
    n = prob[p].tab_mode != TPE_TAB_NONE ? tpp : 0;
  }
  if (n == 0) {
    if (lane == 0) *dst = res_dev[p];
    return;
  }
  tpe_result w{0, 0, 0, 0, -1, -1};
  // the runs' first positions: a, then every multiple of per in (a, a + n) —
  // one lane a run, so a wave's record loads are all in flight at once
  const int b0 = (a / per + 1) * per;
  const int n_runs = 1 + (a + n > b0 ? (a + n - b0 + per - 1) / per : 0);
  for (int j = lane; j < n_runs; j += 64) {
    const int pos = j == 0 ? a : b0 + (j - 1) * per;
    const int t = span ? (list ? list[pos] : pos) : (int)(p * tpp + (pos - a));
    const tpe_result c = run_best[t];
    if (better(c.score, c.idx, w.score, w.idx)) w = c;
  }
  for (int off = 32; off > 0; off >>= 1) {         // (np.argmax order: unique indices, any order of reduction)
    tpe_result o;
    o.score = __shfl_xor(w.score, off); o.l = __shfl_xor(w.l, off); o.g = __shfl_xor(w.g, off);
    o.value = __shfl_xor(w.value, off); o.idx = __shfl_xor(w.idx, off); o.global_idx = __shfl_xor(w.global_idx, off);
    if (better(o.score, o.idx, w.score, w.idx)) w = o;
  }
  if (lane == 0) *dst = w;
}

__global__ __launch_bounds__(kCombThreads) void k_combine(const unsigned char* __restrict__ all, int W, int64_t per,
                                                           int64_t P, tpe_result* __restrict__ out,
                                                           int32_t* __restrict__ status) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int32_t worst = TPE_OK;                        // a hard error outranks a workspace retry
    for (int r = 0; r < W; ++r) {
      const int32_t st = *reinterpret_cast<const int32_t*>(all + (int64_t)r * per);
      if (st != TPE_OK && (worst == TPE_OK || worst == TPE_E_SPACE)) worst = st;
    }
    *status = worst;
  }
  const int64_t p = (int64_t)blockIdx.x * kCombThreads + threadIdx.x;
  if (p >= P) return;
  auto rec = [&](int r) { return reinterpret_cast<const tpe_result*>(all + (int64_t)r * per + TPE_EXCHANGE_HEADER)[p]; };
  tpe_result w = rec(0);
  for (int r = 1; r < W; ++r) {                    // tpe_combine_results' order
    const tpe_result c = rec(r);
    if (c.idx < 0) continue;
    if (w.idx < 0 || better(c.score, c.global_idx, w.score, w.global_idx)) w = c;
  }
  out[p] = w;
}

// ============================================================ level upload
// The packed level (pinned host memory, device-addressable) copied into the
// device blob by the compute queue itself: the first stage then follows in
// queue order, without the copy engine's hand-off to the compute queue (the
// ~10 us gap an hipMemcpyAsync upload left before the first kernel of a level).
// System-scope loads: the host rewrites the staging buffer every level.
constexpr int kUploadThreads = 256;

// the blob's host-written ranges (tpe_pack_info.up_off / up_len, in 8-byte words)
struct UploadRanges {
  int64_t w0[4], n8[4];
  int32_t n;
};

__global__ __launch_bounds__(kUploadThreads) void k_upload(const unsigned long long* __restrict__ src,
                                                           unsigned long long* __restrict__ dst, UploadRanges r) {
  int64_t total = 0;
  for (int k = 0; k < r.n; ++k) total += r.n8[k];
  const int64_t stride = (int64_t)gridDim.x * kUploadThreads;
  for (int64_t i = (int64_t)blockIdx.x * kUploadThreads + threadIdx.x; i < total; i += stride) {
    int k = 0;
    int64_t j = i;
    while (k < r.n - 1 && j >= r.n8[k]) { j -= r.n8[k]; ++k; }
    const int64_t w = r.w0[k] + j;
    dst[w] = __hip_atomic_load(src + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ============================================================ column store
// (include/tpe_hip.h "Device column store").  k_scatter_f64: the appended
// observations of a history's device columns, k values then k int64 positions
// in pinned host memory (system-scope loads, as k_upload), stored into the
// flat column store; k_move_ranges: a store re-layout, every segment's live
// prefix moved to its new offset (element size 4 or 8), the ranges' {src, dst,
// n} triples in pinned host memory, one range per workgroup-stride.
constexpr int kColThreads = 256;

__global__ __launch_bounds__(kColThreads) void k_scatter_f64(const unsigned long long* __restrict__ src, int64_t k,
                                                             double* __restrict__ dst) {
  const int64_t stride = (int64_t)gridDim.x * kColThreads;
  for (int64_t i = (int64_t)blockIdx.x * kColThreads + threadIdx.x; i < k; i += stride) {
    const unsigned long long v = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const long long pos = (long long)__hip_atomic_load(src + k + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    dst[pos] = __longlong_as_double((long long)v);
  }
}

template <typename T>
__global__ __launch_bounds__(kColThreads) void k_move_ranges(const long long* __restrict__ ranges, int32_t n_ranges,
                                                             const T* __restrict__ src, T* __restrict__ dst) {
  for (int r = blockIdx.x; r < n_ranges; r += gridDim.x) {
    const long long so = __hip_atomic_load(ranges + 3 * r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const long long d0 = __hip_atomic_load(ranges + 3 * r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const long long n = __hip_atomic_load(ranges + 3 * r + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (long long i = threadIdx.x; i < n; i += kColThreads) dst[d0 + i] = src[so + i];
  }
}

// a device fit that ran before the upload (tpe_level_run's early fit) wrote its
// problem fields into the patch rows: copied into the problem rows here (the
// fields k_fit_wide writes), after the upload and k_expand
__global__ __launch_bounds__(64) void k_fit_patch(const tpe_fit_job* __restrict__ J,
                                                  const tpe_problem* __restrict__ patch,
                                                  tpe_problem* __restrict__ prob) {
  const tpe_fit_job& j = J[blockIdx.x];
  for (int t = threadIdx.x; t < j.n_problems; t += 64) {
    const tpe_problem& s = patch[j.problem_first + t];
    tpe_problem& d = prob[j.problem_first + t];
    d.above_base = s.above_base;
    d.wide_len = s.wide_len;
    d.prior_mu = s.prior_mu; d.prior_a = s.prior_a; d.prior_c = s.prior_c;
    d.narrow_cmax = s.narrow_cmax; d.narrow_amin = s.narrow_amin;
    d.grid_lo = s.grid_lo; d.grid_inv = s.grid_inv;
  }
}

// ============================================================ expanded levels
// (include/tpe_hip.h "Expanded levels").  The problems of an expanded level
// differ from their label's template only in cand_off, tile_off and ctr3, and
// its tiles are {r, j * kTile, 0, 0} in order.  One thread per 8-byte word of
// the problem rows (consecutive threads write consecutive words) and one per
// tile.
constexpr int kExpandThreads = 256;
constexpr int kProbWords = (int)(sizeof(tpe_problem) / 8);
static_assert(sizeof(tpe_problem) % 8 == 0, "problem rows in 8-byte words");

__global__ __launch_bounds__(kExpandThreads) void k_expand(const tpe_problem* __restrict__ tmpl,
                                                           const int32_t* __restrict__ first, int n_lab,
                                                           const uint32_t* __restrict__ new_id,
                                                           tpe_problem* __restrict__ prob, tpe_tile* __restrict__ tiles,
                                                           int64_t P, int32_t n_tiles, int32_t n_cand) {
  const int64_t i = (int64_t)blockIdx.x * kExpandThreads + threadIdx.x;
  if (i < P * kProbWords) {
    const int64_t r = i / kProbWords;
    const int w = (int)(i - r * kProbWords);
    int a = 0, b = n_lab - 1;                    // the last label whose first problem is <= r
    while (a < b) {
      const int m = (a + b + 1) >> 1;
      if ((int64_t)first[m] <= r) a = m; else b = m - 1;
    }
    uint64_t v = reinterpret_cast<const uint64_t*>(tmpl + a)[w];
    const int byte = 8 * w;
    auto put32 = [&](int off, uint32_t x) {
      if (off >= byte && off < byte + 8) {
        const int sh = 8 * (off - byte);
        v = (v & ~(0xffffffffull << sh)) | ((uint64_t)x << sh);
      }
    };
    if (byte == (int)offsetof(tpe_problem, cand_off)) v = (uint64_t)(r * (int64_t)n_cand);
    put32((int)offsetof(tpe_problem, tile_off), (uint32_t)(r * (int64_t)n_tiles));
    put32((int)offsetof(tpe_problem, ctr3), new_id[r]);
    reinterpret_cast<uint64_t*>(prob + r)[w] = v;
  }
  if (i < P * (int64_t)n_tiles) {
    const int64_t r = i / n_tiles;
    tiles[i] = tpe_tile{(int32_t)r, (int32_t)((i - r * n_tiles) * kTile), 0, 0};
  }
}

// ============================================================ device Parzen fit
// adaptive_parzen_normal (tpe.py:398-475) of the above observations of a label
// (ap_filter_trials, tpe.py:613-641), directly into the pruned f32 layout.
constexpr int kPruneWide = 16;
constexpr double kAScale = 0.84932180028801907;   // sqrt(0.5 * log2(e))

// ---- resident value order (include/tpe_hip.h "Device value order") ----
constexpr int kFitMaxBelow_ = 64;               // (kFitMaxBelow, below)
// The order of the reference's argsort of the above observations (tpe.py:427),
// stable: t ascending, NaN last (np.argsort), equal t by position in tid order.
__device__ __forceinline__ bool ord_lt(double ka, uint32_t ia, double kb, uint32_t ib) {
  if (ka < kb) return true;
  if (ka > kb) return false;
  const bool na = ka != ka, nb = kb != kb;           // (equal or unordered)
  if (na != nb) return nb;
  return ia < ib;
}

// the column holds the kernel coordinate itself (the host's np.log for the log
// families, tpe.py:523 / :556), so the order and the rows see numpy's values
__device__ __forceinline__ double fit_coord(const tpe_fit_job& j, int64_t i) { return j.obs[i]; }

// Delta mode (include/tpe_hip.h "Device value order"): a job whose few new
// observations (at most kFitMaxDelta) are not merged into its resident order
// (no ord_key_out) reads the order and its sorted new observations as one
// VIRTUAL order: new observation k (k-th smallest) at position dp[k] = its rank
// among the resident ones + k, resident entry e at e + #{k : dp[k] <= e + k}.
// The merge — a pass over the whole order for a handful of values — waits
// until the new ones outgrow the delta.  Its arrays in the fit scratch: keys in
// fit_keys_sorted[seg_off ..], indices and positions in fit_vals_sorted after
// the below positions (adj).
constexpr int kFitMaxDelta = TPE_FIT_DELTA_MAX;
__device__ __forceinline__ bool fit_delta(const tpe_fit_job& j) { return j.n_ord_in < j.n_obs && !j.ord_key_out; }
__device__ __forceinline__ double* delta_keys(const tpe_fit_job& j, double* fks) { return fks + j.seg_off; }
__device__ __forceinline__ uint32_t* delta_idx(const tpe_fit_job& j, uint32_t* fvs) {
  return fvs + j.seg_off + kFitMaxBelow_;
}
__device__ __forceinline__ uint32_t* delta_pos(const tpe_fit_job& j, uint32_t* fvs) {
  return fvs + j.seg_off + kFitMaxBelow_ + kFitMaxDelta;
}

// chunks: the new observations obs[n_ord_in ..] of each job, kOrdChunk at a
// time, sorted in LDS by a bitonic network on (t, i) -> fit scratch buffer 0
// (delta mode: -> the delta arrays, with each one's virtual position)
constexpr int kOrdChunk = 8192;
constexpr int kOrdChunkThreads = 1024;
__global__ __launch_bounds__(kOrdChunkThreads) void k_ord_chunks(const tpe_fit_job* __restrict__ J,
                                                                 double* __restrict__ keys,
                                                                 uint32_t* __restrict__ idx,
                                                                 double* __restrict__ dkeys,
                                                                 uint32_t* __restrict__ dvals) {
  const tpe_fit_job& j = J[blockIdx.y];
  const int64_t m = j.n_ord_in, k = j.n_obs - m, c0 = (int64_t)blockIdx.x * kOrdChunk;
  if (c0 >= k) return;
  __shared__ double sk[kOrdChunk];
  __shared__ uint32_t sv[kOrdChunk];
  const int n = (int)min<int64_t>(kOrdChunk, k - c0);
  int N = 1;
  while (N < n) N <<= 1;
  for (int i = threadIdx.x; i < N; i += kOrdChunkThreads) {   // padding sorts after every element
    const bool in = i < n;
    sk[i] = in ? fit_coord(j, m + c0 + i) : NAN;
    sv[i] = in ? (uint32_t)(m + c0 + i) : 0xFFFFFFFFu;
  }
  __syncthreads();
  for (int w = 2; w <= N; w <<= 1) {
    for (int h = w >> 1; h > 0; h >>= 1) {
      for (int i = threadIdx.x; i < N; i += kOrdChunkThreads) {
        const int p = i ^ h;
        if (p > i) {
          const double ka = sk[i], kb = sk[p];
          const uint32_t va = sv[i], vb = sv[p];
          if (ord_lt(kb, vb, ka, va) == ((i & w) == 0)) { sk[i] = kb; sk[p] = ka; sv[i] = vb; sv[p] = va; }
        }
      }
      __syncthreads();
    }
  }
  if (fit_delta(j)) {                               // (k <= kFitMaxDelta: one chunk)
    const int i = threadIdx.x;
    if (i < n) {
      const double t = sk[i];
      const uint32_t v = sv[i];
      int64_t lo = 0, hi = m;                       // resident entries before it
      while (lo < hi) {
        const int64_t md = (lo + hi) >> 1;
        if (ord_lt(j.ord_key_in[md], j.ord_idx_in[md], t, v)) lo = md + 1;
        else hi = md;
      }
      delta_keys(j, dkeys)[i] = t;
      delta_idx(j, dvals)[i] = v;
      delta_pos(j, dvals)[i] = (uint32_t)(lo + i);
    }
    return;
  }
  double* __restrict__ ok = keys + j.seg_off + c0;
  uint32_t* __restrict__ ov = idx + j.seg_off + c0;
  for (int i = threadIdx.x; i < n; i += kOrdChunkThreads) { ok[i] = sk[i]; ov[i] = sv[i]; }
}

// delta mode only (no job of the level merges): each job's few new
// observations sorted by rank (one wave; every pair compared) and placed among
// the resident ones (their virtual positions) — k_ord_chunks' delta branch
// without its 96-KiB LDS sort
__global__ __launch_bounds__(64) void k_ord_delta(const tpe_fit_job* __restrict__ J, double* __restrict__ dkeys,
                                                  uint32_t* __restrict__ dvals) {
  const tpe_fit_job& j = J[blockIdx.x];
  if (!fit_delta(j)) return;
  const int n = (int)(j.n_obs - j.n_ord_in), i = threadIdx.x;
  __shared__ double sk[kFitMaxDelta];
  if (i < n) sk[i] = fit_coord(j, j.n_ord_in + i);
  __syncthreads();
  if (i >= n) return;
  const double t = sk[i];
  const uint32_t v = (uint32_t)(j.n_ord_in + i);
  int r = 0;                                          // its rank among the new ones (indices break ties)
  for (int q = 0; q < n; ++q) r += ord_lt(sk[q], (uint32_t)(j.n_ord_in + q), t, v);
  int64_t lo = 0, hi = j.n_ord_in;                    // resident entries before it
  while (lo < hi) {
    const int64_t md = (lo + hi) >> 1;
    if (ord_lt(j.ord_key_in[md], j.ord_idx_in[md], t, v)) lo = md + 1;
    else hi = md;
  }
  delta_keys(j, dkeys)[r] = t;
  delta_idx(j, dvals)[r] = v;
  delta_pos(j, dvals)[r] = (uint32_t)(lo + r);
}

// merge-path merge, one tile of kMergeTile outputs per workgroup: the tile's
// A and B ranges (found by a binary search on each tile edge's diagonal) are
// staged in LDS, each thread merges kMergePer outputs from its own diagonal,
// and the merged tile is written back coalesced.
//   L > 0: a pass over each job's sorted new batch (runs of L, pairs merged)
//          in src -> dst at the job's scratch segment
//   L = 0: the resident order ord_in [n_ord_in] with the sorted batch in src
//          -> ord_out [n_obs]
constexpr int kMergeThreads = 256;
constexpr int kMergePer = 8;
constexpr int kMergeTile = kMergeThreads * kMergePer;
static_assert(kOrdChunk % kMergeTile == 0, "merge tiles never straddle a run pair");
__global__ __launch_bounds__(kMergeThreads) void k_ord_merge(const tpe_fit_job* __restrict__ J,
                                                             const double* __restrict__ sk,
                                                             const uint32_t* __restrict__ sv,
                                                             double* __restrict__ dk, uint32_t* __restrict__ dv,
                                                             int64_t L) {
  const tpe_fit_job& j = J[blockIdx.y];
  const int64_t k = j.n_obs - j.n_ord_in, t0 = (int64_t)blockIdx.x * kMergeTile;
  if (k <= 0 || fit_delta(j)) return;
  const double *ak, *bk;
  const uint32_t *av, *bv;
  double* ok;
  uint32_t* ov;
  int64_t na, nb, d0;
  if (L > 0) {
    if (t0 >= k) return;
    const int64_t base = t0 / (2 * L) * (2 * L), mid = min(base + L, k), end = min(base + 2 * L, k);
    ak = sk + j.seg_off + base; av = sv + j.seg_off + base; na = mid - base;
    bk = sk + j.seg_off + mid; bv = sv + j.seg_off + mid; nb = end - mid;
    ok = dk + j.seg_off + base; ov = dv + j.seg_off + base;
    d0 = t0 - base;
  } else {
    if (t0 >= j.n_obs) return;
    ak = j.ord_key_in; av = j.ord_idx_in; na = j.n_ord_in;
    bk = sk + j.seg_off; bv = sv + j.seg_off; nb = k;
    ok = j.ord_key_out; ov = j.ord_idx_out;
    d0 = t0;
  }
  const int64_t d1 = min(d0 + kMergeTile, na + nb);
  __shared__ int64_t split[2];
  if (threadIdx.x < 2) {              // A elements among the first d outputs
    const int64_t d = threadIdx.x ? d1 : d0;
    int64_t lo = max<int64_t>(0, d - nb), hi = min(d, na);
    while (lo < hi) {
      const int64_t md = (lo + hi) >> 1;
      if (ord_lt(ak[md], av[md], bk[d - 1 - md], bv[d - 1 - md])) lo = md + 1;
      else hi = md;
    }
    split[threadIdx.x] = lo;
  }
  __syncthreads();
  const int64_t a0 = split[0], b0 = d0 - a0;
  const int nA = (int)(split[1] - a0), n = (int)(d1 - d0), nB = n - nA;
  // a tile drawn from one input only is a straight coalesced copy, no LDS
  // merge (a level that merges a few new observations into a resident order
  // of 10^5 leaves almost every tile pure A: the merge's LDS bank conflicts
  // were most of its time)
  if (nA == 0 || nB == 0) {                          // (block-uniform)
    const double* ck = nB == 0 ? ak + a0 : bk + b0;
    const uint32_t* cv = nB == 0 ? av + a0 : bv + b0;
    double tk[kMergePer];
    uint32_t tv[kMergePer];
#pragma unroll
    for (int e = 0; e < kMergePer; ++e) {            // every load issued before the stores
      const int i = (int)threadIdx.x + e * kMergeThreads;
      if (i < n) { tk[e] = ck[i]; tv[e] = cv[i]; }
    }
#pragma unroll
    for (int e = 0; e < kMergePer; ++e) {
      const int i = (int)threadIdx.x + e * kMergeThreads;
      if (i < n) { ok[d0 + i] = tk[e]; ov[d0 + i] = tv[e]; }
    }
    return;
  }
  __shared__ double lk[kMergeTile];
  __shared__ uint32_t lv[kMergeTile];
  {
    double tk[kMergePer];
    uint32_t tv[kMergePer];
#pragma unroll
    for (int e = 0; e < kMergePer; ++e) {            // every load issued before the LDS stores
      const int i = (int)threadIdx.x + e * kMergeThreads;
      if (i < n) {
        tk[e] = i < nA ? ak[a0 + i] : bk[b0 + i - nA];
        tv[e] = i < nA ? av[a0 + i] : bv[b0 + i - nA];
      }
    }
#pragma unroll
    for (int e = 0; e < kMergePer; ++e) {
      const int i = (int)threadIdx.x + e * kMergeThreads;
      if (i < n) { lk[i] = tk[e]; lv[i] = tv[e]; }
    }
  }
  __syncthreads();
  const int dd = min(threadIdx.x * kMergePer, n);
  int lo = max(0, dd - nB), hi = min(dd, nA);
  while (lo < hi) {
    const int md = (lo + hi) >> 1;
    if (ord_lt(lk[md], lv[md], lk[nA + dd - 1 - md], lv[nA + dd - 1 - md])) lo = md + 1;
    else hi = md;
  }
  int ia = lo, ib = dd - lo;
  const int cnt = min(kMergePer, n - dd);
  double rk[kMergePer];
  uint32_t rv[kMergePer];
#pragma unroll
  for (int e = 0; e < kMergePer; ++e) {
    if (e < cnt) {
      const bool take_a = ia < nA && (ib >= nB || ord_lt(lk[ia], lv[ia], lk[nA + ib], lv[nA + ib]));
      const int at = take_a ? ia : nA + ib;
      rk[e] = lk[at];
      rv[e] = lv[at];
      ia += take_a;
      ib += !take_a;
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kMergePer; ++e)
    if (e < cnt) { lk[dd + e] = rk[e]; lv[dd + e] = rv[e]; }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += kMergeThreads) { ok[d0 + i] = lk[i]; ov[d0 + i] = lv[i]; }
}

// the job's current order (merged this level, or the resident one)
__device__ __forceinline__ const double* ord_keys(const tpe_fit_job& j) {
  return j.n_ord_in < j.n_obs && j.ord_key_out ? j.ord_key_out : j.ord_key_in;
}
__device__ __forceinline__ const uint32_t* ord_idx(const tpe_fit_job& j) {
  return j.n_ord_in < j.n_obs && j.ord_key_out ? j.ord_idx_out : j.ord_idx_in;
}

// the job's virtual order (delta mode) or its order as it is (nd = 0): entry f
// of the n_obs sorted (t, i) pairs
struct VOrd {
  const double* ok;
  const uint32_t* ov;
  const double* dk;          // the delta (LDS): keys, indices, virtual positions
  const uint32_t* dv;
  const uint32_t* dp;
  int nd;
  __device__ __forceinline__ int before(int64_t f) const {      // delta entries at positions < f
    int lo = 0, hi = nd;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if ((int64_t)dp[m] < f) lo = m + 1; else hi = m;
    }
    return lo;
  }
  __device__ __forceinline__ double key(int64_t f) const {
    const int c = before(f);
    return c < nd && (int64_t)dp[c] == f ? dk[c] : ok[f - c];
  }
  __device__ __forceinline__ uint32_t idx(int64_t f) const {
    const int c = before(f);
    return c < nd && (int64_t)dp[c] == f ? dv[c] : ov[f - c];
  }
};

// the job's delta into LDS (block-wide, at least kFitMaxDelta threads; the
// caller synchronises) and its virtual order
__device__ __forceinline__ VOrd vord_lds(const tpe_fit_job& j, const double* __restrict__ dkeys,
                                         const uint32_t* __restrict__ dvals, double* l_dk, uint32_t* l_dv,
                                         uint32_t* l_dp) {
  const int nd = fit_delta(j) ? (int)(j.n_obs - j.n_ord_in) : 0;
  if ((int)threadIdx.x < nd) {
    l_dk[threadIdx.x] = dkeys[j.seg_off + threadIdx.x];
    l_dv[threadIdx.x] = dvals[j.seg_off + kFitMaxBelow_ + threadIdx.x];
    l_dp[threadIdx.x] = dvals[j.seg_off + kFitMaxBelow_ + kFitMaxDelta + threadIdx.x];
  }
  return VOrd{ord_keys(j), ord_idx(j), l_dk, l_dv, l_dp, nd};
}

// Per-job scalars of the build, at the head of the job's fit_keys segment
// (free once the merge has run): the prior's position, the combined chunk
// statistics, then the chunks' statistics (FitPart, 12 doubles each).
constexpr int kFitHdrPos = 0, kFitHdrStats = 1, kFitHdrGrid = 6, kFitHdrParts = 8;

// position of each below observation in the job's order (binary search for its
// own (t, i) pair), written SORTED and as adj[k] = pos_k - k (pos_k: the k-th
// smallest position) -> adj[seg_off + k]: the above observation q of the order
// (the compacted index) sits at position q + #{k : adj[k] <= q}; and the
// prior's position among the above observations (np.searchsorted(side='left')
// of prior_mu, tpe.py:427-431): the observations < prior_mu in the whole order
// less the below ones
constexpr int kFitMaxBelow = 64;
static_assert(kFitMaxBelow == kFitMaxBelow_ && kFitMaxDelta <= kFitMaxBelow && kFitMaxDelta <= 64,
              "one delta entry per thread");
__global__ __launch_bounds__(kFitMaxBelow) void k_ord_below(const tpe_fit_job* __restrict__ J,
                                                            const int32_t* __restrict__ below_idx,
                                                            uint32_t* __restrict__ adj, double* __restrict__ hdr,
                                                            const double* __restrict__ dkeys) {
  const tpe_fit_job& j = J[blockIdx.x];
  const int b = threadIdx.x;
  __shared__ double l_dk[kFitMaxDelta];
  __shared__ uint32_t l_dv[kFitMaxDelta], l_dp[kFitMaxDelta];
  const VOrd V = vord_lds(j, dkeys, adj, l_dk, l_dv, l_dp);
  __syncthreads();
  bool under = false;
  uint32_t mine = 0xFFFFFFFFu;
  if (b < j.n_below) {
    const uint32_t i = (uint32_t)below_idx[j.below_off + b];
    const double t = fit_coord(j, i);
    under = t < j.prior_mu;
    int64_t lo = 0, hi = j.n_obs;
    while (lo < hi) {
      const int64_t md = (lo + hi) >> 1;
      if (ord_lt(V.key(md), V.idx(md), t, i)) lo = md + 1;
      else hi = md;
    }
    mine = (uint32_t)lo;
  }
  int r = 0;                                        // rank of this position (positions are distinct)
  for (int q = 0; q < j.n_below; ++q) r += __shfl(mine, q) < mine;
  if (b < j.n_below) adj[j.seg_off + r] = mine - (uint32_t)r;
  const int n_under = __popcll(__ballot(under));
  // the first and last above observations' positions: past the below positions
  // that open the order (positions 0, 1, ..) and before those that close it
  const int nb = j.n_below;
  const int head = __popcll(__ballot(b < nb && mine == (uint32_t)r));
  const int tail = __popcll(__ballot(b < nb && (int64_t)mine == j.n_obs - nb + r));
  if (b == 0) {
    int64_t lo = 0, hi = j.n_obs;                   // observations with t < prior_mu (NaN last)
    while (lo < hi) {
      const int64_t md = (lo + hi) >> 1;
      if (V.key(md) < j.prior_mu) lo = md + 1;
      else hi = md;
    }
    const int64_t pos = lo - n_under, n = j.n_obs - nb;
    hdr[j.seg_off + kFitHdrPos] = (double)pos;
    // the grid's bounds: the f32 means of the first and last component (the prior inserted)
    const double m0 = pos == 0 ? j.prior_mu : V.key(head);
    const double m1 = pos == n ? j.prior_mu : V.key(j.n_obs - 1 - tail);
    hdr[j.seg_off + kFitHdrGrid] = (double)(float)m0;
    hdr[j.seg_off + kFitHdrGrid + 1] = (double)(float)m1;
  }
}

// ---- build: adaptive_parzen_normal over the above observations of the order ----
// The order holds every observation; the above ones are those at positions not
// in the job's below list (k_ord_below).  Nothing is compacted in HBM: each
// chunk's workgroup stages its above observations — keys, and their ranks among
// the above observations in tid order (the linear-forgetting weight index) —
// into LDS from the contiguous stretch of the order that holds them.  Launches
// over (chunk of kFitChunk components) x job, so a 100k-component mixture
// spreads over ~50 workgroups instead of one:
//   k_fit_main    per chunk, one pass: its {mu, a, c} rows (c shifted by an
//                 upper bound of max log2(w / sigma), so no pass waits for the
//                 data's maximum), its wide candidates, its statistics (W, the
//                 acceptance mass M, the wide-threshold counts), its grid buckets
//   k_fit_combine the job's chunk statistics combined (fixed chunk order)
//   k_fit_wide    the wide list (fixed index order), c = -inf for its members in
//                 the sorted rows, the problem rows
constexpr int kFitChunk = 2048;
constexpr int kFitThreads = 256;
constexpr int kFitPer = kFitChunk / kFitThreads;
// positions of the order a staging thread reads: the stretch holding a chunk's
// above observations and their neighbours (kFitChunk + 3) holds at most
// kFitMaxBelow below ones too
constexpr int kFitStagePer = 9;
static_assert(kFitStagePer * 256 >= kFitChunk + 3 + 64, "staging covers the stretch");
constexpr int kThr = 5;                          // wide if sigma > smin * 2^(m+1), m < kThr
struct FitPart {                                 // one chunk's statistics (fit scratch, 8-B aligned)
  double W, M;
  double rmax;                                   // max w / max(sigma, EPS): cm = log2(rmax) (log2 is monotone)
  double sm_all;
  double sm[kThr];
  int32_t cnt[kThr];
  int32_t pad;
};

// above observation q of a job (its order index among the above observations)
// read through the sorted below positions in global memory: position q +
// #{k : adj[k] <= q} of the order (the wide list, the grid bounds)
struct AboveSrc {
  VOrd V;                    // the job's (virtual) order
  const uint32_t* adj;       // k_ord_below
  const int32_t* bidx;       // the job's below indices into obs, ascending
  int nb;
  __device__ __forceinline__ int64_t at(int64_t q) const {
    int lo = 0, hi = nb;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if ((int64_t)adj[m] <= q) lo = m + 1; else hi = m;
    }
    return q + lo;
  }
  __device__ __forceinline__ double key(int64_t q) const { return V.key(at(q)); }
  __device__ __forceinline__ uint32_t rank(int64_t q) const {   // its index in obs less the older below ones
    const uint32_t i = V.idx(at(q));
    int lo = 0, hi = nb;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if ((uint32_t)bidx[m] < i) lo = m + 1; else hi = m;
    }
    return i - (uint32_t)lo;
  }
};

// the view of one job's sorted above observations with the prior inserted at
// pos (np.searchsorted(side='left'), tpe.py:427-431) and its bandwidth rules
template <class Src>
struct FitCtx {
  Src src;               // sorted above observations and their ranks in tid order
  int64_t n, K, pos;
  double pmu, psig, pw, smin, smax, start, step;
  int64_t num;
  bool ramp, bounded;
  double low, high;
  __device__ __forceinline__ double mu(int64_t i) const {
    return i < pos ? src.key(i) : (i == pos ? pmu : src.key(i - 1));
  }
  __device__ __forceinline__ double sigma(int64_t i) const {          // tpe.py:441-470
    if (i == pos) return psig;
    double sg;
    if (i == 0) sg = mu(1) - mu(0);
    else if (i == K - 1) sg = mu(K - 1) - mu(K - 2);
    else sg = fmax(mu(i) - mu(i - 1), mu(i + 1) - mu(i));
    return fmin(fmax(sg, smin), smax);
  }
  __device__ __forceinline__ double weight(int64_t i) const {         // tpe.py:381-394, 454-460
    if (i == pos) return pw;
    if (!ramp) return 1.0;
    const int64_t r = src.rank(i < pos ? i : i - 1);
    if (r >= num) return 1.0;
    if (r == num - 1) return 1.0;
    if (num == 1) return start;
    return __dadd_rn(__dmul_rn((double)r, step), start);        // linspace: i * step + start
  }
};

// (f64 erf out of line: inlined twice, its polynomial constants were hoisted
// into VGPR pairs and took the stats kernel to 143 VGPRs)
// |z| >= 6: erf(z) rounds to +-1 in f64 (1 - erf(6) = 2.2e-17 < half an ulp of 1)
__device__ __noinline__ double erf_call(double z) { return erf(z); }

template <class Src>
__device__ __forceinline__ FitCtx<Src> fit_ctx(const tpe_fit_job& j, Src src, int64_t pos) {
  FitCtx<Src> c;
  c.src = src;
  c.n = j.n_obs - j.n_below;
  c.K = c.n + 1;
  c.pos = pos;
  c.pmu = j.prior_mu; c.psig = j.prior_sigma; c.pw = j.prior_weight;
  c.smax = j.prior_sigma;
  c.smin = j.prior_sigma / fmin(100.0, 1.0 + (double)c.K);                   // tpe.py:465-470
  c.ramp = j.lf > 0 && j.lf < c.n;
  c.num = c.n - j.lf;
  c.start = 1.0 / (double)c.n;
  c.step = c.num > 1 ? (1.0 - c.start) / (double)(c.num - 1) : 0.0;
  c.bounded = j.family != TPE_FAM_LOGGAUSS && (j.flags & (TPE_F_HAS_LOW | TPE_F_HAS_HIGH));
  c.low = j.low; c.high = j.high;
  return c;
}

__device__ __forceinline__ AboveSrc above_src(const tpe_fit_job& j, const int32_t* __restrict__ below_idx,
                                              const uint32_t* __restrict__ adj, const VOrd& V) {
  return AboveSrc{V, adj + j.seg_off, below_idx + j.below_off, j.n_below};
}

// Below indices per bucket of the observation indices (bucket b = i >> bsh,
// at most kFitBuckets of them): s_bk[b] = #{k : s_bi[k] < b << bsh}, so an
// observation's count of older below ones is s_bk[b] plus a scan of its own
// bucket's few (usually no) entries instead of a search of the whole list.
constexpr int kFitBuckets = 256;
__device__ __forceinline__ int fit_bucket_shift(int64_t n_obs) {
  int s = 0;
  while (((n_obs - 1) >> s) >= kFitBuckets) ++s;
  return s;
}
__device__ __forceinline__ void fit_rank_buckets(int nb, const uint32_t* s_bi, int bsh, uint32_t* s_bk) {
  for (int b = threadIdx.x; b <= kFitBuckets; b += kFitThreads) {
    const uint64_t edge = (uint64_t)b << bsh;
    int lo = 0, hi = nb;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if ((uint64_t)s_bi[m] < edge) lo = m + 1; else hi = m;
    }
    s_bk[b] = (uint32_t)lo;
  }
}

// Stages components [c0 - 1, c1] of job j (the chunk's and one neighbour on
// each side; the prior inserted at pos) into lmu (means) and lrk (an
// observation's rank among the above ones in tid order: its LF weight index),
// indexed by i - c0 + 1.  They come from the order's stretch holding above
// observations [qa, qb), less the below positions in it (s_bp, sorted: the
// stretch holds entries [la, lb) of it, usually none), loads first.
// Block-wide; the caller synchronises.
// one staged entry f of the stretch: below ones skipped, the rest into lmu / lrk
__device__ __forceinline__ void fit_stage_put(int64_t f, double kv, uint32_t o, const uint32_t* s_bp,
                                              const uint32_t* s_bi, const uint32_t* s_bk, int bsh, int64_t c0,
                                              int64_t c1, int64_t pos, int la, int lb, double* lmu, uint32_t* lrk) {
  int lo = la;
  bool below = false;
  for (int k = la; k < lb; ++k) {                     // uniform trip count
    const int64_t p = s_bp[k];
    lo += p < f;
    below |= p == f;
  }
  if (below) return;
  const int64_t q = f - lo;
  const int64_t i = q + (q >= pos);
  if (i < c0 - 1 || i > c1) return;
  uint32_t k = s_bk[o >> bsh];
  const uint32_t ke = s_bk[(o >> bsh) + 1];
  while (k < ke && s_bi[k] < o) ++k;
  lmu[i - c0 + 1] = kv;
  lrk[i - c0 + 1] = o - k;
}

// the stretch's entries from ok[f], ov[f] (f in [fa, fb)): every load issued first
__device__ __forceinline__ void fit_stage_plain(const double* __restrict__ ok, const uint32_t* __restrict__ ov,
                                                const uint32_t* s_bp, const uint32_t* s_bi, const uint32_t* s_bk,
                                                int bsh, int64_t c0, int64_t c1, int64_t pos, int la, int lb,
                                                int64_t fa, int64_t fb, double* lmu, uint32_t* lrk) {
  double kv[kFitStagePer];
  uint32_t iv[kFitStagePer];
#pragma unroll
  for (int e = 0; e < kFitStagePer; ++e) {
    const int64_t f = fa + e * kFitThreads + threadIdx.x;
    if (f < fb) { kv[e] = ok[f]; iv[e] = ov[f]; }
  }
#pragma unroll
  for (int e = 0; e < kFitStagePer; ++e) {
    const int64_t f = fa + e * kFitThreads + threadIdx.x;
    if (f >= fb) break;
    fit_stage_put(f, kv[e], iv[e], s_bp, s_bi, s_bk, bsh, c0, c1, pos, la, lb, lmu, lrk);
  }
}

// a stretch holding delta entries (a few chunks of a job in delta mode): the
// virtual order's entries [fa, fb) gathered into the job's fit scratch (the
// chunk's slot, see fit_slot) by k_fit_gather, where k_fit_main's staging then
// reads them — so the staging stays the common case's code and registers.
constexpr int kFitStretch = kFitStagePer * kFitThreads;
static_assert(kFitStretch == 2304 && kFitChunk == 2048, "tpe_host.cpp sizes the delta slots (kFitStageStretch)");
__device__ __forceinline__ void fit_gather_stretch(const VOrd& V, int64_t fa, int64_t fb, int da, int db,
                                                   double* __restrict__ sk, uint32_t* __restrict__ sv) {
  double kv[kFitStagePer];
  uint32_t iv[kFitStagePer];
#pragma unroll
  for (int e = 0; e < kFitStagePer; ++e) {            // every load issued first
    const int64_t f = fa + e * kFitThreads + threadIdx.x;
    if (f < fb) {
      int c = da;
      bool in_delta = false;
      for (int k = da; k < db; ++k) {                 // uniform trip count
        const int64_t p = V.dp[k];
        c += p < f;
        in_delta |= p == f;
      }
      kv[e] = in_delta ? V.dk[c] : V.ok[f - c];
      iv[e] = in_delta ? V.dv[c] : V.ov[f - c];
    }
  }
#pragma unroll
  for (int e = 0; e < kFitStagePer; ++e) {
    const int64_t f = fa + e * kFitThreads + threadIdx.x;
    if (f < fb) { sk[f - fa] = kv[e]; sv[f - fa] = iv[e]; }
  }
}

// a delta-mode job's chunk slot for its gathered stretch: in its fit scratch
// segment after the delta arrays (fit_keys_sorted / fit_vals_sorted; the host
// sizes the segment for one slot per chunk)
__device__ __forceinline__ int64_t fit_slot(const tpe_fit_job& j, int64_t chunk) {
  return j.seg_off + kFitMaxBelow_ + 2 * kFitMaxDelta + chunk * kFitStretch;
}

// The stretch of the (virtual) order holding a chunk's above observations
// [c0 - 2, c1 + 1): positions [fa, fb), its below entries [la, lb) of s_bp and
// its delta entries [da, db) (usually none).  Workgroup-uniform (scalars).
struct FitStretch {
  int la, lb, da, db;
  int64_t fa, fb;
};
__device__ __forceinline__ FitStretch fit_stretch(const tpe_fit_job& j, const VOrd& V, const uint32_t* s_bp, int64_t c0,
                                                  int64_t c1, int64_t n) {
  const int nb = j.n_below;
  const int64_t qa = max<int64_t>(0, c0 - 2), qb = min<int64_t>(n, c1 + 1);
  auto n_before = [&](int64_t q) {                    // below positions before above observation q
    int lo = 0, hi = nb;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if ((int64_t)s_bp[m] - m <= q) lo = m + 1; else hi = m;
    }
    return lo;
  };
  FitStretch t;
  t.la = __builtin_amdgcn_readfirstlane(n_before(qa));
  t.lb = __builtin_amdgcn_readfirstlane(n_before(qb - 1));
  t.fa = qa + t.la;
  t.fb = qb + t.lb;
  t.da = __builtin_amdgcn_readfirstlane(V.before(t.fa));
  t.db = __builtin_amdgcn_readfirstlane(V.before(t.fb));
  return t;
}

template <bool DELTA>
__device__ void fit_stage_rows(const tpe_fit_job& j, const VOrd& V, const FitStretch& t, const uint32_t* s_bp,
                               const uint32_t* s_bi, const uint32_t* s_bk, int bsh, int64_t c0, int64_t c1,
                               int64_t pos, double* lmu, uint32_t* lrk, const double* dkeys, const uint32_t* dvals) {
  const double* ok = V.ok - t.da;                    // (the order shifted by the delta entries before the stretch)
  const uint32_t* ov = V.ov - t.da;
  if (DELTA && t.da != t.db) {                       // (the stretch k_fit_gather gathered)
    ok = dkeys + fit_slot(j, (int64_t)blockIdx.x) - t.fa;
    ov = dvals + fit_slot(j, (int64_t)blockIdx.x) - t.fa;
  }
  fit_stage_plain(ok, ov, s_bp, s_bi, s_bk, bsh, c0, c1, pos, t.la, t.lb, t.fa, t.fb, lmu, lrk);
  if (threadIdx.x == 0 && pos >= c0 - 1 && pos <= c1) lmu[pos - c0 + 1] = j.prior_mu;
}

// log2 of a positive finite double: its exponent exactly plus the f32 log2 of
// its mantissa (in [-1, 0): |error| < 3e-7, under the f32 rounding of a row's c
// at |c| >= 4)
__device__ __forceinline__ double log2_rows(double x) {
  return (double)__builtin_amdgcn_frexp_exp(x) + (double)__builtin_amdgcn_logf((float)__builtin_amdgcn_frexp_mant(x));
}

// a component's row {mu_hi, mu_lo, a, c}: a = A / max(sigma, EPS) rounded from
// f64 (the pruning bound narrow_amin is rounded the same way), c = log2(w / se)
// - cm, at most 0 (cm bounds it).  k_fit_main writes the same bits (its
// smallest-sigma shortcut takes the same values precomputed).
__device__ __forceinline__ float4 fit_row(double mu, double se, double w, double cm) {
  const float hi = (float)mu;
  return make_float4(hi, (float)(mu - (double)hi), (float)(kAScale / se),
                     fminf((float)(log2_rows(w) - log2_rows(se) - cm), 0.f));
}

// 0.5 * (1 + erf((x - mu) / max(sqrt2 sigma, EPS))) (tpe.py:96-101); |z| >= 6
// tested as |x - mu| >= 6 den, so a wave whose lanes all saturate divides
// nothing (where the two tests disagree z rounds to within an ulp of 6 and
// erf(z) rounds to +-1 all the same)
__device__ __forceinline__ double ncdf_fit(double x, double mu, double sigma) {
  const double d = x - mu, den = fmax(1.4142135623730951 * sigma, kEPS);
  double e = copysign(1.0, d);
  if (!(fabs(d) >= 6.0 * den)) e = erf_call(d / den);
  return 0.5 * (1.0 + e);
}

// the job's sorted below positions and below indices into LDS (block-wide)
__device__ __forceinline__ void fit_below_lds(const tpe_fit_job& j, const int32_t* __restrict__ below_idx,
                                              const uint32_t* __restrict__ adj, uint32_t* s_bp, uint32_t* s_bi) {
  if ((int)threadIdx.x < j.n_below) {
    s_bp[threadIdx.x] = adj[j.seg_off + threadIdx.x] + threadIdx.x;
    s_bi[threadIdx.x] = (uint32_t)below_idx[j.below_off + threadIdx.x];
  }
}

__device__ __forceinline__ FitPart* fit_parts(const tpe_fit_job& j, double* scratch) {
  return reinterpret_cast<FitPart*>(scratch + j.seg_off + kFitHdrParts);
}
static_assert(sizeof(FitPart) == 12 * sizeof(double), "FitPart: 12 doubles");
static_assert(kFitThreads >= kFitMaxBelow, "a fit workgroup stages the below list in one round");

struct FitStats {
  double W, M, cm, thr, s_narrow;
};

// the wide candidates' counter of every job (k_fit_main appends to it)
__global__ __launch_bounds__(256) void k_fit_wide_reset(const tpe_fit_job* __restrict__ J, int n_fit,
                                                        uint32_t* __restrict__ wide_scratch) {
  const int q = (int)(blockIdx.x * 256 + threadIdx.x);
  if (q < n_fit) wide_scratch[J[q].seg_off] = 0u;
}

// the shift of the rows' c: an upper bound of max log2(w / sigma) (LF weights
// <= 1, the prior's pw; every sigma >= smin), so every c <= 0 without waiting
// for the data's maximum — the rows and the statistics come out of one pass
__device__ __forceinline__ double fit_cm_bound(const tpe_fit_job& j, int64_t K) {
  const double smin = j.prior_sigma / fmin(100.0, 1.0 + (double)K);
  return log2(fmax(1.0, j.prior_weight) / fmax(smin, kEPS));
}

// wide candidates of a job: sigma above the lowest wide threshold (2 smin) or
// the prior — their indices in wide_scratch[seg_off + 1 ..] (counter at
// [seg_off]), their sigmas in the fit scratch after the chunk statistics
constexpr int kWideCap = 8192;
__device__ __forceinline__ double* wide_sigmas(const tpe_fit_job& j, double* scratch, int64_t K) {
  const int64_t nc = (K + kFitChunk - 1) / kFitChunk;
  return scratch + j.seg_off + kFitHdrParts + 12 * nc;
}

// Delta mode: the stretches of the chunks that hold delta entries gathered
// into their slots, before k_fit_main.  Workgroup (k, job): delta entry k's
// chunk by its above index and the two beside it (the stretches overlap), each
// gathered when k is the first delta entry of its stretch — every such chunk
// exactly once.
__global__ __launch_bounds__(kFitThreads) void k_fit_gather(const tpe_fit_job* __restrict__ J,
                                                            const int32_t* __restrict__ below_idx,
                                                            const uint32_t* __restrict__ adj,
                                                            const double* __restrict__ scratch,
                                                            double* __restrict__ dkeys, uint32_t* __restrict__ dvals) {
  const tpe_fit_job& j = J[blockIdx.y];
  if (!fit_delta(j)) return;
  const int nd = (int)(j.n_obs - j.n_ord_in), k = (int)blockIdx.x;
  if (k >= nd) return;
  __shared__ uint32_t s_bp[kFitMaxBelow], s_bi[kFitMaxBelow];
  __shared__ double l_dk[kFitMaxDelta];
  __shared__ uint32_t l_dv[kFitMaxDelta], l_dp[kFitMaxDelta];
  fit_below_lds(j, below_idx, adj, s_bp, s_bi);
  const VOrd V = vord_lds(j, dkeys, dvals, l_dk, l_dv, l_dp);
  __syncthreads();
  const int64_t n = j.n_obs - j.n_below, K = n + 1;
  const int64_t pos = (int64_t)scratch[j.seg_off + kFitHdrPos];
  const int64_t p = V.dp[k];
  int lo = 0, hi = j.n_below;                       // below positions before p
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if ((int64_t)s_bp[m] < p) lo = m + 1; else hi = m;
  }
  const int64_t q = p - lo, i = q + (q >= pos);
  for (int side = -1; side <= 1; ++side) {
    const int64_t c = i / kFitChunk + side;
    if (c < 0 || c * kFitChunk >= K) continue;
    const int64_t c0 = c * kFitChunk, c1 = min(c0 + kFitChunk, K);
    const FitStretch t = fit_stretch(j, V, s_bp, c0, c1, n);
    if (t.da != k || t.db == t.da) continue;        // (another workgroup's chunk, or none)
    fit_gather_stretch(V, t.fa, t.fb, t.da, t.db, dkeys + fit_slot(j, c), dvals + fit_slot(j, c));
  }
}

// One pass per chunk: its rows {mu_hi, mu_lo, a, c = log2(w / sigma) - shift}
// (every one finite; k_fit_wide marks the wide ones), its wide candidates, its
// statistics (normaliser W, acceptance mass M, the wide-threshold counts) and
// its grid buckets.  Grid over the f32 means: grid[g] = the first component
// with mu32 >= edge_g, edge_g = glo + g / ginv (grid[G] = K); the chunk writes
// the buckets whose answer lies in it (a binary search over its staged means) —
// the buckets g with mu32[c0 - 1] < edge_g <= mu32[c1 - 1] (the last chunk:
// every g from there up, K when no mean reaches edge_g).
// (DELTA: a level with delta-mode jobs; the instance for one without keeps the
// common case's code)
template <bool DELTA>
__global__ __launch_bounds__(kFitThreads) __attribute__((amdgpu_waves_per_eu(6))) void k_fit_main(const tpe_fit_job* __restrict__ J,
                                                          const int32_t* __restrict__ below_idx,
                                                          const uint32_t* __restrict__ adj,
                                                          double* __restrict__ scratch,
                                                          uint32_t* __restrict__ wide_scratch,
                                                          float4* __restrict__ comp, int32_t* __restrict__ grid,
                                                          const double* __restrict__ dkeys, const uint32_t* __restrict__ dvals) {
  const tpe_fit_job& j = J[blockIdx.y];
  const int64_t n = j.n_obs - j.n_below, K = n + 1, c0 = (int64_t)blockIdx.x * kFitChunk;
  if (c0 >= K) return;
  const int64_t c1 = min(c0 + kFitChunk, K);
  __shared__ uint32_t s_bp[kFitMaxBelow], s_bi[kFitMaxBelow];
  __shared__ uint32_t s_bk[kFitBuckets + 1];
  __shared__ double lmu[kFitChunk + 2];
  __shared__ uint32_t lrk[kFitChunk + 2];
  __shared__ double l_dk[kFitMaxDelta];
  __shared__ uint32_t l_dv[kFitMaxDelta], l_dp[kFitMaxDelta];
  fit_below_lds(j, below_idx, adj, s_bp, s_bi);
  const VOrd V = DELTA ? vord_lds(j, dkeys, dvals, l_dk, l_dv, l_dp) : VOrd{ord_keys(j), ord_idx(j), l_dk, l_dv, l_dp, 0};
  __syncthreads();
  const FitStretch t = fit_stretch(j, V, s_bp, c0, c1, n);
  const int bsh = fit_bucket_shift(j.n_obs);
  fit_rank_buckets(j.n_below, s_bi, bsh, s_bk);
  __syncthreads();
  const double* __restrict__ hdr = scratch + j.seg_off;
  const int64_t pos = (int64_t)hdr[kFitHdrPos];
  fit_stage_rows<DELTA>(j, V, t, s_bp, s_bi, s_bk, bsh, c0, c1, pos, lmu, lrk, dkeys, dvals);
  __syncthreads();
  // the bandwidth and weight rules of fit_ctx (tpe.py:381-394, 441-470) over
  // the staged means, the prior already in place
  const double smin = j.prior_sigma / fmin(100.0, 1.0 + (double)K), smax = j.prior_sigma;
  const bool ramp = j.lf > 0 && j.lf < n;
  const int64_t num = n - j.lf;
  const double start = 1.0 / (double)n, step = num > 1 ? (1.0 - start) / (double)(num - 1) : 0.0;
  const bool bounded = j.family != TPE_FAM_LOGGAUSS && (j.flags & (TPE_F_HAS_LOW | TPE_F_HAS_HIGH));
  const double cm = fit_cm_bound(j, K), thr0 = 2.0 * smin;
  // most components sit at the clip: their a and log2(se) once (fit_row's values)
  const double se_min = fmax(smin, kEPS), ls_min = log2_rows(se_min);
  const float a_min = (float)(kAScale / se_min);
  float4* __restrict__ C = comp + j.above_off;
  uint32_t* __restrict__ wl = wide_scratch + j.seg_off;
  double* __restrict__ wsg = wide_sigmas(j, scratch, K);
  double W = 0, M = 0, sm_all = 0, s_lo = 0;
  double sm[kThr];
  int cnt[kThr];
#pragma unroll
  for (int m = 0; m < kThr; ++m) { sm[m] = 0; cnt[m] = 0; }
#pragma unroll 1
  for (int e = 0; e < kFitPer; ++e) {
    const int64_t i = c0 + e * kFitThreads + threadIdx.x;
    if (i >= c1) break;
    const int li = (int)(i - c0) + 1;
    const double mu = lmu[li];
    double sg, w;
    if (i == pos) {
      sg = j.prior_sigma;
      w = j.prior_weight;
    } else {
      // an edge component has one gap (-inf for the missing one: the clip
      // below gives what the one-gap rule gives, NaN gaps included)
      const double gl = i > 0 ? mu - lmu[li - 1] : -INFINITY;
      const double gr = i < K - 1 ? lmu[li + 1] - mu : -INFINITY;
      sg = fmin(fmax(fmax(gl, gr), smin), smax);
      w = 1.0;
      if (ramp) {
        const int64_t r = lrk[li];
        if (r < num - 1) w = __dadd_rn(__dmul_rn((double)r, step), start);    // linspace: i * step + start
      }
    }
    const double se = fmax(sg, kEPS);
    float a = a_min;
    double ls = ls_min;
    if (__ballot(se != se_min)) {                   // (a wave-uniform branch: no division when all clip)
      if (se != se_min) {
        a = (float)(kAScale / se);
        ls = log2_rows(se);
      }
    }
    const float hi = (float)mu;
    C[i] = make_float4(hi, (float)(mu - (double)hi), a, fminf((float)(log2_rows(w) - ls - cm), 0.f));
    W += w;
    if (bounded) M += w * (ncdf_fit(j.high, mu, sg) - ncdf_fit(j.low, mu, sg));
    if (i == pos || sg > thr0) {
      const uint32_t slot = atomicAdd(&wl[0], 1u);
      if (slot < (uint32_t)kWideCap) { wl[1 + slot] = (uint32_t)i; wsg[slot] = i == pos ? INFINITY : sg; }
    }
    if (i != pos) {
      sm_all = fmax(sm_all, sg);
      if (sg > thr0) {
#pragma unroll
        for (int m = 0; m < kThr; ++m) {
          const double thr = smin * (double)(2 << m);
          if (sg > thr) ++cnt[m]; else sm[m] = fmax(sm[m], sg);
        }
      } else {
        s_lo = fmax(s_lo, sg);                      // under every threshold
      }
    }
  }
#pragma unroll
  for (int m = 0; m < kThr; ++m) sm[m] = fmax(sm[m], s_lo);
  for (int o = 32; o > 0; o >>= 1) {
    W += __shfl_xor(W, o); M += __shfl_xor(M, o); sm_all = fmax(sm_all, __shfl_xor(sm_all, o));
#pragma unroll
    for (int m = 0; m < kThr; ++m) { sm[m] = fmax(sm[m], __shfl_xor(sm[m], o)); cnt[m] += __shfl_xor(cnt[m], o); }
  }
  __shared__ FitPart wp[kFitThreads / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    wp[wave].W = W; wp[wave].M = M; wp[wave].rmax = 0.0; wp[wave].sm_all = sm_all;
#pragma unroll
    for (int m = 0; m < kThr; ++m) { wp[wave].sm[m] = sm[m]; wp[wave].cnt[m] = cnt[m]; }
  }
  // ---- grid buckets of this chunk ----
  const int G = j.grid_n;
  int32_t* __restrict__ Gp = grid + j.grid_off;
  __shared__ int s_ga, s_gb;
  __shared__ double s_glo;
  __shared__ float s_ginv;
  if (threadIdx.x == 0) {
    const double glo = hdr[kFitHdrGrid], ghi = hdr[kFitHdrGrid + 1];
    const float ginv = ghi > glo ? (float)((double)G / (ghi - glo)) : 0.f;
    int ga, gb;
    if (!(ginv > 0.f)) {
      ga = 0; gb = c0 == 0 ? G : 0;                  // every bucket 0, written by the first chunk
    } else {
      auto first_above = [&](double m) {             // first g in [0, G] with edge_g > m (G: none)
        int lo = 0, hi = G;
        while (lo < hi) {
          const int md = (lo + hi) >> 1;
          if (glo + (double)md / (double)ginv > m) hi = md; else lo = md + 1;
        }
        return lo;
      };
      ga = c0 == 0 ? 0 : first_above((double)(float)lmu[0]);
      gb = c1 == K ? G : first_above((double)(float)lmu[c1 - c0]);
    }
    s_ga = ga; s_gb = gb; s_glo = glo; s_ginv = ginv;
    if (c0 == 0) Gp[G] = (int32_t)K;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    FitPart r = wp[0];
    for (int w2 = 1; w2 < kFitThreads / 64; ++w2) {
      r.W += wp[w2].W; r.M += wp[w2].M; r.sm_all = fmax(r.sm_all, wp[w2].sm_all);
#pragma unroll
      for (int m = 0; m < kThr; ++m) { r.sm[m] = fmax(r.sm[m], wp[w2].sm[m]); r.cnt[m] += wp[w2].cnt[m]; }
    }
    r.pad = 0;
    fit_parts(j, scratch)[blockIdx.x] = r;
  }
  const int ga = s_ga, gb = s_gb;
  const double glo = s_glo;
  const float ginv = s_ginv;
  for (int g = ga + (int)threadIdx.x; g < gb; g += kFitThreads) {
    if (!(ginv > 0.f)) { Gp[g] = 0; continue; }
    const double edge = glo + (double)g / (double)ginv;
    int64_t lo = c0, hi = c1;                      // first i with !(mu32[i] < edge) (c1: none in the chunk)
    while (lo < hi) {
      const int64_t md = (lo + hi) >> 1;
      if ((double)(float)lmu[md - c0 + 1] < edge) lo = md + 1;
      else hi = md;
    }
    Gp[g] = (int32_t)lo;
  }
}

// the job's chunk statistics combined once (fixed chunk order) into the header
__global__ __launch_bounds__(64) void k_fit_combine(const tpe_fit_job* __restrict__ J, double* __restrict__ scratch) {
  const tpe_fit_job& j = J[blockIdx.x];
  const int64_t K = j.n_obs - j.n_below + 1;
  const int nc = (int)((K + kFitChunk - 1) / kFitChunk);
  const FitPart* __restrict__ parts = fit_parts(j, scratch);
  __shared__ FitPart lp[64];
  __shared__ FitPart acc;
  for (int c0 = 0; c0 < nc; c0 += 64) {
    const int m = min(64, nc - c0);
    if ((int)threadIdx.x < m) lp[threadIdx.x] = parts[c0 + threadIdx.x];      // one round of loads
    __syncthreads();
    if (threadIdx.x == 0) {
      FitPart r = c0 ? acc : lp[0];
      for (int q = c0 ? 0 : 1; q < m; ++q) {
        const FitPart& p = lp[q];
        r.W += p.W; r.M += p.M; r.sm_all = fmax(r.sm_all, p.sm_all);
#pragma unroll
        for (int t = 0; t < kThr; ++t) { r.sm[t] = fmax(r.sm[t], p.sm[t]); r.cnt[t] += p.cnt[t]; }
      }
      acc = r;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double smin = j.prior_sigma / fmin(100.0, 1.0 + (double)K);
    double thr = INFINITY, s_narrow = acc.sm_all;
    for (int m = 0; m < kThr; ++m)
      if (thr == INFINITY && acc.cnt[m] <= kPruneWide - 1) { thr = smin * (double)(2 << m); s_narrow = acc.sm[m]; }
    double* __restrict__ hdr = scratch + j.seg_off + kFitHdrStats;
    hdr[0] = acc.W; hdr[1] = acc.M; hdr[2] = fit_cm_bound(j, K); hdr[3] = thr; hdr[4] = s_narrow;
  }
}

// the wide list (the prior and sigma > thr, index order): its rows, c = -inf
// for them in the sorted list, and the job's problem rows:
// lpdf = ln2 * log2(sum) + base; base = ln2*cm - ln(W sqrt(2 pi) p_accept)
__global__ __launch_bounds__(64) void k_fit_wide(const tpe_fit_job* __restrict__ J,
                                                 const int32_t* __restrict__ below_idx,
                                                 const uint32_t* __restrict__ adj,
                                                 double* __restrict__ scratch,
                                                 const uint32_t* __restrict__ wide_scratch,
                                                 tpe_problem* __restrict__ P, float4* __restrict__ comp,
                                                 const double* __restrict__ dkeys) {
  const tpe_fit_job& j = J[blockIdx.x];
  const int64_t K = j.n_obs - j.n_below + 1;
  __shared__ int64_t wide_ix[kPruneWide];
  __shared__ int s_nw;
  __shared__ double l_dk[kFitMaxDelta];
  __shared__ uint32_t l_dv[kFitMaxDelta], l_dp[kFitMaxDelta];
  const VOrd V = vord_lds(j, dkeys, adj, l_dk, l_dv, l_dp);
  const uint32_t* __restrict__ wl = wide_scratch + j.seg_off;
  const double* __restrict__ hdr = scratch + j.seg_off;
  const double thr = hdr[kFitHdrStats + 3];
  const FitCtx<AboveSrc> c = fit_ctx(j, above_src(j, below_idx, adj, V), (int64_t)hdr[kFitHdrPos]);
  const uint32_t n_cand = wl[0];
  const double* __restrict__ wsg = wide_sigmas(j, scratch, K);
  if (threadIdx.x == 0) s_nw = 0;
  __syncthreads();
  // the candidates above thr (at most 15 and the prior: thr's definition); past
  // the candidate list's capacity every component is examined
  const int64_t m = n_cand <= (uint32_t)kWideCap ? (int64_t)n_cand : K;
  for (int64_t q = threadIdx.x; q < m; q += 64) {
    const int64_t i = n_cand <= (uint32_t)kWideCap ? (int64_t)wl[1 + q] : q;
    const double sg = n_cand <= (uint32_t)kWideCap ? wsg[q] : (i == c.pos ? INFINITY : c.sigma(i));
    if (sg > thr) {
      const int slot = atomicAdd(&s_nw, 1);
      if (slot < kPruneWide) wide_ix[slot] = i;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = min(s_nw, kPruneWide);
    for (int a = 1; a < nw; ++a)                  // fixed order of the wide list
      for (int b = a; b > 0 && wide_ix[b - 1] > wide_ix[b]; --b) {
        const int64_t t = wide_ix[b]; wide_ix[b] = wide_ix[b - 1]; wide_ix[b - 1] = t;
      }
    s_nw = nw;
  }
  __syncthreads();
  const FitStats st{hdr[kFitHdrStats], hdr[kFitHdrStats + 1], hdr[kFitHdrStats + 2], hdr[kFitHdrStats + 3],
                    hdr[kFitHdrStats + 4]};
  const int nw = s_nw;
  if ((int)threadIdx.x < nw) {
    const int64_t i = wide_ix[threadIdx.x];
    const double sg = c.sigma(i), w = c.weight(i), mu = c.mu(i), se = fmax(sg, kEPS);
    comp[j.wide_off + threadIdx.x] = fit_row(mu, se, w, st.cm);
    comp[j.above_off + i].w = -INFINITY;          // listed apart
  }
  // every problem of the job (a batched level: one per active id, any count)
  for (int t = threadIdx.x; t < j.n_problems; t += 64) {
    const double glo = hdr[kFitHdrGrid], ghi = hdr[kFitHdrGrid + 1];
    const float ginv = ghi > glo ? (float)((double)j.grid_n / (ghi - glo)) : 0.f;
    const double pa = c.bounded ? st.M / st.W : 1.0;
    tpe_problem& p = P[j.problem_first + t];     // (these fields: k_fit_patch copies them too)
    p.above_base = kLn2 * st.cm - log(st.W) - 0.91893853320467274 - log(pa);
    p.wide_len = nw;
    const double pse = fmax(j.prior_sigma, kEPS);
    p.prior_mu = (float)j.prior_mu;
    p.prior_a = (float)(kAScale / pse);
    p.prior_c = (float)(log2(j.prior_weight / pse) - st.cm);
    p.narrow_cmax = 0.f;                           // every c <= 0 (the shift is an upper bound)
    p.narrow_amin = (float)(kAScale / fmax(st.s_narrow, kEPS));
    p.grid_lo = (float)glo;
    p.grid_inv = ginv;
  }
}

// device-drawn sorted problems at f32 draw ordered (include/tpe_hip.h "Ordered draws")
// the select stage may scan a lazy categorical problem's first draws (nothing
// per candidate requested)
bool lazy_ok(const tpe_batch* b) {
  return b->sample && !(b->flags & TPE_BATCH_WRITE_CAND) && !b->l_out;
}

bool ordered_draws(const tpe_batch* b) {
  return b->sample && b->precision == TPE_PREC_F32 && (b->flags & TPE_BATCH_ORDERED_DRAWS) && b->n_sorted > 0 &&
         b->sort_count > 0;
}

int check_batch(const tpe_batch* b) {
  if (!b) return fail(TPE_E_ARG, "null batch");
  if (b->n_problems < 0 || b->n_tiles < 0 || b->n_work_cont < 0 || b->n_work_qgauss < 0 || b->n_work_qlog < 0 ||
      b->total_cand < 0)
    return fail(TPE_E_ARG, "negative count");
  const int64_t n_work = (int64_t)b->n_work_cont + b->n_work_qgauss + b->n_work_qlog;
  if (b->precision != TPE_PREC_F32 && b->precision != TPE_PREC_F64) return fail(TPE_E_ARG, "bad precision");
  if (b->n_problems > 0 && (!b->problems || !b->result)) return fail(TPE_E_ARG, "null problems/result");
  if (b->n_tiles > 0 && (!b->tiles || !b->tile_best || !b->cand || !b->coord || !b->keys || !b->vals ||
                         !b->keys_sorted || !b->vals_sorted))
    return fail(TPE_E_ARG, "null candidate buffers");
  if (n_work > 0 && (!b->work || !b->part)) return fail(TPE_E_ARG, "null work buffers");
  if (b->n_work_cont > 0 && b->precision == TPE_PREC_F32 && (!b->comp32 || !b->grid))
    return fail(TPE_E_ARG, "null comp32/grid");
  if ((n_work > 0 || b->n_tiles > 0) && !b->comp64 && b->precision == TPE_PREC_F64)
    return fail(TPE_E_ARG, "null comp64");
  if ((b->l_out == nullptr) != (b->g_out == nullptr)) return fail(TPE_E_ARG, "l_out and g_out go together");
  if (b->total_cand >= ((int64_t)1 << 32)) return fail(TPE_E_ARG, "more than 2^32 candidates in one batch");
  if (b->sort_end_bit < 0 || b->sort_end_bit > 32) return fail(TPE_E_ARG, "bad sort_end_bit");
  if (b->sort_count < 0 || b->sort_count > b->total_cand) return fail(TPE_E_ARG, "bad sort_count");
  if (b->key_bits < 0 || b->key_bits > 16) return fail(TPE_E_ARG, "bad key_bits");
  if (b->sort_end_bit == 0 && (b->keys_sorted != b->keys || b->vals_sorted != b->vals))
    return fail(TPE_E_ARG, "unsorted batch must alias keys_sorted/vals_sorted to keys/vals");
  if (b->n_fit < 0 || b->fit_total < 0) return fail(TPE_E_ARG, "negative fit count");
  if (b->n_fit > 0 && (!b->fit || !b->below_idx || !b->fit_seg || !b->fit_keys || !b->fit_keys_sorted ||
                       !b->fit_vals || !b->fit_vals_sorted || !b->comp32 || !b->grid || !b->problems))
    return fail(TPE_E_ARG, "null fit buffers");
  if (b->n_fit > 0 && b->precision != TPE_PREC_F32) return fail(TPE_E_ARG, "device fit needs TPE_PREC_F32");
  if (b->n_sorted < 0 || b->draw_blocks < 0) return fail(TPE_E_ARG, "negative n_sorted/draw_blocks");
  if (ordered_draws(b) && (!b->draw_pref || b->draw_blocks < 1))
    return fail(TPE_E_ARG, "ordered draws need draw_pref and draw_blocks");
  if (b->n_tab_jobs < 0 || b->tab_blocks < 0 || b->tab_units < 0) return fail(TPE_E_ARG, "negative table count");
  if (b->n_tab_jobs > 0 && (!b->tab_jobs || !b->tab || !b->comp32 || !b->comp64))
    return fail(TPE_E_ARG, "null table buffers");
  // (no tabulated tile list: every tile is tabulated, in order — an expanded level)
  if (b->early_select && (!b->run_best || b->n_tab_jobs <= 0 || !b->sample || !b->samp ||
                          (!b->tab_tiles && b->n_tab_tiles != b->n_tiles) || b->n_late < 0 ||
                          b->n_late > b->n_problems))
    return fail(TPE_E_ARG, "early selection needs tables, device draws, tile lists and run_best");
  return TPE_OK;
}

// TPE_EARLY_FIT=0: a level's device fit runs after its upload (else it starts
// while the host packs the rest of the level: early_fit_hook; A/B, tests)
bool early_fit_enabled() {           // (read per level: the tests switch it)
  const char* v = getenv("TPE_EARLY_FIT");
  return !(v && v[0] == '0');
}

// TPE_RESULT_COPY=1: read the results back with a copy (else the select stage
// writes them into the pinned buffer directly)
bool direct_results() {
  const char* v = getenv("TPE_RESULT_COPY");
  return !(v && v[0] == '1');
}

// TPE_UPLOAD_COPY=1: upload a level with hipMemcpyAsync (else the k_upload
// kernel copies it from the device-addressable staging buffer)
bool kernel_upload() {
  static const int on = [] {
    const char* v = getenv("TPE_UPLOAD_COPY");
    return !(v && v[0] == '1');
  }();
  return on != 0;
}

// device address of a pinned host buffer, or nullptr when it is not
// device-addressable pinned memory (no cache: callers pass the address they
// looked up once per allocation in tpe_level_ws.pinned_dev)
char* device_alias(void* host) {
  hipPointerAttribute_t a;
  char* d = nullptr;
  if (hipPointerGetAttributes(&a, host) == hipSuccess && a.type == hipMemoryTypeHost && a.devicePointer)
    d = (char*)a.devicePointer;
  (void)hipGetLastError();
  return d;
}

// compute units of the current device (cached per device; 256 on MI355X)
int cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) { (void)hipGetLastError(); return 256; }
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) {
      (void)hipGetLastError();
      n = 256;
    }
    cache[dev] = n;
  }
  return cache[dev];
}

// TPE_TAB_FAST=0: the general sample-stage kernel for every level (A/B, tests)
bool tab_fast_disabled() {
  static const int v = [] { const char* e = getenv("TPE_TAB_FAST"); return e && e[0] == '0' ? 1 : 0; }();
  return v != 0;
}

// tabulated tiles per sample-stage workgroup (the early selection's run
// enumeration on the host uses the same partition)
int tab_tiles_per_wg(int n_tab, int wgs_per_cu) {
  const int slots = cu_count() * wgs_per_cu;
  return std::min(kTabMaxTilesPerWg, std::max(1, (n_tab + slots - 1) / slots));
}
// sample-stage workgroups a CU holds: k_sample_fast's three (tab_fast >= 2), else one
int tab_wgs_per_cu(const tpe_batch* b) { return b->tab_fast >= 2 ? kFastWgsPerCu : 1; }

// TPE_FAST_NP2=1: k_sample_fast's two-candidate units on every level (A/B)
bool fast_np2_forced() {
  static const int v = [] { const char* e = getenv("TPE_FAST_NP2"); return e && e[0] == '1' ? 1 : 0; }();
  return v != 0;
}

// TPE_SAMPLE_FAST2=0: k_sample_tab's FAST pass instead of k_sample_fast (A/B, tests)
bool fast2_disabled() {
  static const int v = [] { const char* e = getenv("TPE_SAMPLE_FAST2"); return e && e[0] == '0' ? 1 : 0; }();
  return v != 0;
}

// np.argmax order of (score, index) on the host: better() of the kernels
bool host_better(double s, int64_t i, double bs, int64_t bi) {
  if (bi < 0) return i >= 0;
  if (i < 0) return false;
  const bool n = s != s, bn = bs != bs;
  if (n || bn) return n && (!bn || i < bi);
  return s > bs || (s == bs && i < bi);
}

}  // namespace

extern "C" {

int tpe_abi_version(void) { return TPE_ABI_VERSION; }

// error hand-off for the library's other host translation units (tpe_suggest.cpp)
__attribute__((visibility("hidden"))) int tpe_internal_fail(int code, const char* what) { return fail(code, what); }

const char* tpe_last_error(void) { return g_err; }

int tpe_device_count(int* n) {
  int c = 0;
  if (!n) return fail(TPE_E_ARG, "null out pointer");
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess || c == 0) { *n = 0; (void)hipGetLastError(); return fail(TPE_E_NODEV, "no HIP device"); }
  *n = c;
  return TPE_OK;
}

int tpe_tile_size(void) { return kTile; }

int tpe_pinned_device_address(void* host, void** dev) {
  if (!host || !dev) return fail(TPE_E_ARG, "tpe_pinned_device_address: null pointer");
  *dev = device_alias(host);
  return TPE_OK;
}

int tpe_sort_workspace_bytes(int64_t total_cand, uint64_t* bytes) {
  if (!bytes || total_cand < 0) return fail(TPE_E_ARG, "bad arguments");
  size_t sz = 0;
  hipError_t e = rocprim::radix_sort_pairs<SortConfig>(
      nullptr, sz, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const uint64_t*)nullptr, (uint64_t*)nullptr,
      (size_t)total_cand, 0u, 32u, (hipStream_t)0);
  if (e != hipSuccess) return fail(TPE_E_HIP, hipGetErrorString(e));
  *bytes = (uint64_t)sz;
  return TPE_OK;
}

int tpe_fit_above(const tpe_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  if (b->n_fit == 0) return TPE_OK;
  if (b->fit_total >= ((int64_t)1 << 32)) return fail(TPE_E_ARG, "more than 2^32 fit observations");
  if (b->fit_max_new < 0 || b->fit_max_obs < b->fit_max_new || b->fit_max_obs >= ((int64_t)1 << 31) ||
      b->fit_max_merge < 0 || b->fit_max_merge > b->fit_max_new || b->fit_n_delta < 0 || b->fit_n_delta > b->n_fit)
    return fail(TPE_E_ARG, "bad fit_max_new / fit_max_obs / fit_max_merge");
  hipStream_t s = (hipStream_t)stream;
  if (b->fit_max_new > 0) {
    // the observations appended since each order was written: sorted chunks,
    // merged pairwise until one run per job, then merged into the resident order
    const int64_t chunks = (b->fit_max_new + kOrdChunk - 1) / kOrdChunk;
    if (b->fit_max_merge == 0)                // (every job with new observations in delta mode)
      TPE_LAUNCH(k_ord_delta, dim3(b->n_fit), dim3(64), 0, s, b->fit, b->fit_keys_sorted, b->fit_vals_sorted);
    else
      TPE_LAUNCH(k_ord_chunks, dim3((unsigned)chunks, b->n_fit), dim3(kOrdChunkThreads), 0, s, b->fit, b->fit_keys,
                 b->fit_vals, b->fit_keys_sorted, b->fit_vals_sorted);
    if ((rc = hip_check("tpe_fit_above/chunks"))) return rc;
    double* src_k = b->fit_keys;
    uint32_t* src_v = b->fit_vals;
    double* dst_k = b->fit_keys_sorted;
    uint32_t* dst_v = b->fit_vals_sorted;
    if (b->fit_max_merge > 0) {               // (none when every job with new observations is in delta mode)
      const unsigned tiles_new = (unsigned)((b->fit_max_merge + kMergeTile - 1) / kMergeTile);
      for (int64_t L = kOrdChunk; L < b->fit_max_merge; L *= 2) {
        TPE_LAUNCH(k_ord_merge, dim3(tiles_new, b->n_fit), dim3(kMergeThreads), 0, s, b->fit, src_k, src_v, dst_k,
                   dst_v, L);
        std::swap(src_k, dst_k);
        std::swap(src_v, dst_v);
      }
      const unsigned tiles_obs = (unsigned)((b->fit_max_obs + kMergeTile - 1) / kMergeTile);
      TPE_LAUNCH(k_ord_merge, dim3(tiles_obs, b->n_fit), dim3(kMergeThreads), 0, s, b->fit, src_k, src_v,
                 (double*)nullptr, (uint32_t*)nullptr, (int64_t)0);
      if ((rc = hip_check("tpe_fit_above/merge"))) return rc;
    }
  }
  // the sorted below positions (adj) in fit_vals_sorted (free once the merge
  // has run), then the build over the order itself (no compaction): chunk
  // statistics (into fit_keys, free once the merge has run), rows + grid
  // buckets, the wide list (its counter and indices in fit_vals) and the
  // problem rows
  uint32_t* adj = b->fit_vals_sorted;
  TPE_LAUNCH(k_ord_below, dim3(b->n_fit), dim3(kFitMaxBelow), 0, s, b->fit, b->below_idx, adj, b->fit_keys,
             (const double*)b->fit_keys_sorted);
  const unsigned chunks_k = (unsigned)((b->fit_max_obs + 1 + kFitChunk - 1) / kFitChunk);
  // the wide candidates' counters (one per job, at its segment's head)
  TPE_LAUNCH(k_fit_wide_reset, dim3((unsigned)((b->n_fit + 255) / 256)), dim3(256), 0, s, b->fit, b->n_fit, b->fit_vals);
  if (b->fit_n_delta > 0) {                   // (jobs in delta mode: their delta chunks' stretches first)
    const unsigned nd = (unsigned)std::min<int64_t>(b->fit_max_new, kFitMaxDelta);
    TPE_LAUNCH(k_fit_gather, dim3(nd, b->n_fit), dim3(kFitThreads), 0, s, b->fit, b->below_idx, adj,
               (const double*)b->fit_keys, b->fit_keys_sorted, b->fit_vals_sorted);
    TPE_LAUNCH(k_fit_main<true>, dim3(chunks_k, b->n_fit), dim3(kFitThreads), 0, s, b->fit, b->below_idx, adj,
               b->fit_keys, b->fit_vals, (float4*)b->comp32, const_cast<int32_t*>(b->grid), b->fit_keys_sorted,
               b->fit_vals_sorted);
  } else {
    TPE_LAUNCH(k_fit_main<false>, dim3(chunks_k, b->n_fit), dim3(kFitThreads), 0, s, b->fit, b->below_idx, adj,
               b->fit_keys, b->fit_vals, (float4*)b->comp32, const_cast<int32_t*>(b->grid), b->fit_keys_sorted,
               b->fit_vals_sorted);
  }
  TPE_LAUNCH(k_fit_combine, dim3(b->n_fit), dim3(64), 0, s, b->fit, b->fit_keys);
  TPE_LAUNCH(k_fit_wide, dim3(b->n_fit), dim3(64), 0, s, b->fit, b->below_idx, adj, b->fit_keys, b->fit_vals,
             const_cast<tpe_problem*>(b->problems), (float4*)b->comp32, (const double*)b->fit_keys_sorted);
  return hip_check("tpe_fit_above/build");
}

int tpe_tables(const tpe_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  if (b->n_tab_jobs == 0 || (b->tab_blocks == 0 && b->fgt_max_cells == 0)) return TPE_OK;
  const int extra = b->early_select ? b->n_problems : 0;
  if (b->fgt_max_boxes > 0 && b->fgt_max_cells > 0) {
    // the TPE_F_FGT labels' above cells: box moments, then the cells from them
    TPE_LAUNCH(k_boxes, dim3((unsigned)((b->fgt_max_boxes + 3) / 4), b->n_tab_jobs), dim3(256), 0,
               (hipStream_t)stream, b->problems, b->tab_jobs, (const float4*)b->comp32, b->grid, (float4*)b->tab);
    TPE_LAUNCH(k_cells_fgt, dim3((unsigned)((b->fgt_max_cells + 8 * kFgtCellsPerWave - 1) / (8 * kFgtCellsPerWave)),
                                 b->n_tab_jobs), dim3(512), 0, (hipStream_t)stream, b->problems, b->tab_jobs,
               (const float4*)b->comp32, b->grid, (float4*)b->tab, (b->flags & TPE_BATCH_TAB_EXACT) != 0);
  }
  if (b->tab_blocks == 0 && extra == 0) return hip_check("tpe_tables");
  TPE_LAUNCH(k_tables, dim3(b->tab_blocks + extra), dim3(kTabTblThreads), 0, (hipStream_t)stream,
                       b->problems, b->tab_jobs, b->n_tab_jobs, (const float4*)b->comp32, (const double4*)b->comp64,
                       b->grid, (float4*)b->tab, (b->flags & TPE_BATCH_TAB_EXACT) != 0, b->tab_blocks, b->samp,
                       lazy_ok(b) ? 1 : 0, b->result);
  return hip_check("tpe_tables");
}

// the stage profiler's kernel-bracketing events (tpe_stage_prof.kernel_ns): set
// by run_batch_profiled around the sample stage, null otherwise
static hipEvent_t g_kev[2] = {nullptr, nullptr};
static bool g_kev_on = false;

// the sample stage's tabulated pass: timed by its own launch's start / stop
// events while the profiler brackets the stage
#define TPE_LAUNCH_TIMED(kern, grid, block, shmem, stream, ...)                                           \
  do {                                                                                                  \
    ++g_launches;                                                                                       \
    if (g_kev_on)                                                                                       \
      hipExtLaunchKernelGGL(kern, grid, block, (std::uint32_t)(shmem), stream, g_kev[0], g_kev[1], 0u,  \
                            __VA_ARGS__);                                                               \
    else                                                                                                \
      hipLaunchKernelGGL(kern, grid, block, shmem, stream, __VA_ARGS__);                                \
  } while (0)

// tpe_debug_fast_lg's buffer: k_sample_fast writes {value, l, g, label} of every
// candidate there (null: the production kernel, nothing per candidate)
static struct { double* dev; int64_t n; } g_fast_lg = {nullptr, 0};

int tpe_debug_fast_lg(void* dev, int64_t n_records) {
  if (dev && n_records <= 0) return fail(TPE_E_ARG, "tpe_debug_fast_lg: no records");
  g_fast_lg.dev = (double*)dev;
  g_fast_lg.n = dev ? n_records : 0;
  return TPE_OK;
}

extern "C++" {
// k_sample_fast<NP, LG> over the level's tabulated tiles
template <int NP, bool LG>
void launch_fast(const tpe_batch* b, int wgs, size_t lds, hipStream_t s, int n_tab, int per, tpe_result* run_best,
                 double* lg) {
  TPE_LAUNCH_TIMED((k_sample_fast<NP, LG>), dim3(wgs), dim3(kFastThreads), lds, s, b->problems, b->tiles,
                   b->tab_tiles, n_tab, per, b->samp, (const float4*)b->comp32, (const float4*)b->tab, run_best,
                   b->tiles_per_problem, lg);
}
}

int tpe_sample(const tpe_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  if (b->sample && !b->samp && b->n_tiles) return fail(TPE_E_ARG, "null sampler table");
  if (b->n_tiles == 0) return TPE_OK;
  const bool od = ordered_draws(b);
  if (od) {
    const int64_t per = (b->draw_blocks + kThreads / 64 - 1) / (kThreads / 64);
    if ((int64_t)b->n_problems * per >= ((int64_t)1 << 31)) return fail(TPE_E_ARG, "ordered-draw grid too large");
    TPE_LAUNCH(k_draw_sums, dim3((unsigned)(b->n_problems * per)), dim3(kThreads), 0, (hipStream_t)stream,
                       b->problems, b->draw_blocks, b->draw_pref);
    TPE_LAUNCH(k_draw_scan, dim3(b->n_problems), dim3(kThreads), 0, (hipStream_t)stream, b->problems,
                       b->draw_blocks, b->draw_pref);
    if ((rc = hip_check("tpe_sample/prefix"))) return rc;
  }
  // generic kernel over the untabulated tiles (without the lazy categorical
  // ones when the select stage scans those), tabulated tiles apart; no lists:
  // both kernels over every tile, each skipping the other's
  const bool lazy = b->sample && !(b->flags & TPE_BATCH_WRITE_CAND) && !b->l_out;
  const int n_gen = b->samp_tiles ? (lazy ? b->n_samp_eager : b->n_samp_tiles) : b->n_tiles;
  const int n_tab = b->tab_tiles ? b->n_tab_tiles : (b->n_tab_jobs > 0 ? b->n_tiles : 0);
  if (n_gen > 0)
    TPE_LAUNCH(k_sample, dim3(n_gen, TPE_BEST_PER_TILE), dim3(kThreads), 0, (hipStream_t)stream,
                       b->problems, b->tiles, b->samp, (const double4*)b->comp64, b->cand, b->coord, b->keys, b->vals,
                       b->vals_sorted, b->tile_best, b->l_out, b->g_out, b->precision, b->sample, b->key_bits,
                       b->flags, b->draw_pref, b->draw_blocks, od ? 1 : 0, b->pool_best,
                       b->samp_tiles);
  if (n_tab > 0) {
    if (!b->tab) return fail(TPE_E_ARG, "tabulated tiles without score tables");
    // one workgroup per CU-sized group of tiles (each stages its problem once)
    const int per = tab_tiles_per_wg(n_tab, tab_wgs_per_cu(b));
    const int wgs = (n_tab + per - 1) / per;
    tpe_result* run_best = b->early_select ? b->run_best : nullptr;
    const bool fast = b->tab_fast && run_best && b->precision == TPE_PREC_F32 && b->sample && !b->l_out &&
                      !(b->flags & TPE_BATCH_WRITE_CAND);
    if (fast && b->tab_fast >= 2) {
      if (b->tab_fast - 1 > kFastMaxUnits) return fail(TPE_E_ARG, "tpe_sample: tab_fast units past the fast kernel's LDS");
      double* lg = g_fast_lg.dev;                  // (debug: every candidate's value, l, g)
      if (lg && g_fast_lg.n < b->total_cand) return fail(TPE_E_ARG, "tpe_sample: tpe_debug_fast_lg buffer too small");
      const size_t lds = (size_t)(b->tab_fast - 1) * 16;
      // (two candidate pairs per lane when the level fills at most two workgroups a CU)
      const bool np4 = wgs <= 2 * cu_count() && !fast_np2_forced();
      if (lg && np4) launch_fast<4, true>(b, wgs, lds, (hipStream_t)stream, n_tab, per, run_best, lg);
      else if (lg) launch_fast<2, true>(b, wgs, lds, (hipStream_t)stream, n_tab, per, run_best, lg);
      else if (np4) launch_fast<4, false>(b, wgs, lds, (hipStream_t)stream, n_tab, per, run_best, nullptr);
      else launch_fast<2, false>(b, wgs, lds, (hipStream_t)stream, n_tab, per, run_best, nullptr);
    } else if (fast)
      TPE_LAUNCH_TIMED((k_sample_tab<TPE_PREC_F32, true>), dim3(wgs), dim3(kTabThreads), 0, (hipStream_t)stream,
                         b->problems, b->tiles, b->tab_tiles, n_tab, per, b->samp, b->cand, b->coord, b->tile_best,
                         b->l_out, b->g_out, b->sample, b->flags, (const float4*)b->comp32, (const float4*)b->tab,
                         run_best, b->tiles_per_problem);
    else if (b->precision == TPE_PREC_F64)
      TPE_LAUNCH(k_sample_tab<TPE_PREC_F64>, dim3(wgs), dim3(kTabThreads), 0, (hipStream_t)stream,
                         b->problems, b->tiles, b->tab_tiles, n_tab, per, b->samp, b->cand, b->coord, b->tile_best,
                         b->l_out, b->g_out, b->sample, b->flags, (const float4*)b->comp32, (const float4*)b->tab,
                         run_best, b->tiles_per_problem);
    else
      TPE_LAUNCH(k_sample_tab<TPE_PREC_F32>, dim3(wgs), dim3(kTabThreads), 0, (hipStream_t)stream,
                         b->problems, b->tiles, b->tab_tiles, n_tab, per, b->samp, b->cand, b->coord, b->tile_best,
                         b->l_out, b->g_out, b->sample, b->flags, (const float4*)b->comp32, (const float4*)b->tab,
                         run_best, b->tiles_per_problem);
  }
  return hip_check("tpe_sample");
}

int tpe_sort(const tpe_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  // sort_end_bit == 0: no sort; the caller aliases keys_sorted/vals_sorted to keys/vals.
  // Ordered draws: the sample stage already wrote the final order.
  if (b->n_tiles == 0 || b->sort_count == 0 || b->sort_end_bit == 0 || ordered_draws(b)) return TPE_OK;
  size_t sz = (size_t)b->sort_tmp_bytes;
  hipError_t e = rocprim::radix_sort_pairs<SortConfig>(
      b->sort_tmp, sz, (const uint32_t*)b->keys, b->keys_sorted, (const uint64_t*)b->vals, b->vals_sorted,
      (size_t)b->sort_count, 0u, (unsigned)b->sort_end_bit, (hipStream_t)stream);
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "tpe_sort: %s (workspace %llu bytes)", hipGetErrorString(e),
             (unsigned long long)b->sort_tmp_bytes);
    return TPE_E_HIP;
  }
  ++g_launches;
  return hip_check("tpe_sort");
}

int tpe_score_above(const tpe_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  const int n_cont = b->n_work_cont, n_qg = b->n_work_qgauss, n_ql = b->n_work_qlog;
  hipStream_t s = (hipStream_t)stream;
  if (n_cont) {
    if (b->precision == TPE_PREC_F32)
      TPE_LAUNCH(k_above_f32, dim3(n_cont), dim3(kThreads), 0, s, b->problems, b->tiles, b->work,
                         (const float4*)b->comp32, b->grid, b->vals_sorted, b->part, b->tile_best,
                         b->l_out, b->g_out, b->ce_count, b->flags, b->sample, b->pool_best);
    else
      TPE_LAUNCH(k_above_f64, dim3(n_cont), dim3(kThreads), 0, s, b->problems, b->tiles, b->work,
                         (const double4*)b->comp64, b->cand, b->vals_sorted, b->part);
  }
  if (n_qg)
    TPE_LAUNCH((k_above_q<false>), dim3(n_qg), dim3(kThreads), 0, s, b->problems, b->tiles, b->work + n_cont,
                       (const double4*)b->comp64, b->cand, b->vals_sorted, b->part);
  if (n_ql)
    TPE_LAUNCH((k_above_q<true>), dim3(n_ql), dim3(kThreads), 0, s, b->problems, b->tiles,
                       b->work + n_cont + n_qg,
                       (const double4*)b->comp64, b->cand, b->vals_sorted, b->part);
  return hip_check("tpe_score_above");
}

int tpe_finalize(const tpe_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  if (b->n_tiles == 0) return TPE_OK;
  // only the listed tiles, unless every tile may need this stage (caller-drawn
  // candidates, no fused finalize)
  const bool listed = b->fin_tiles && b->sample && !(b->flags & TPE_BATCH_NO_FUSE);
  const int n_fin = listed ? b->n_fin_tiles : b->n_tiles;
  if (n_fin == 0) return TPE_OK;
  TPE_LAUNCH(k_finalize, dim3(n_fin, TPE_BEST_PER_TILE), dim3(kThreads), 0,
                     (hipStream_t)stream, b->problems, b->tiles, listed ? b->fin_tiles : nullptr,
                     (const float4*)b->comp32, (const double4*)b->comp64, b->grid, b->cand, b->vals_sorted,
                     b->part, b->l_out, b->g_out, b->tile_best, b->precision, b->sample, b->flags, b->pool_best);
  return hip_check("tpe_finalize");
}

int tpe_select(const tpe_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  if (b->n_problems == 0 || (b->early_select && b->n_late == 0)) return TPE_OK;
  TPE_LAUNCH(k_select, dim3(b->n_problems), dim3(kSelThreads), 0, (hipStream_t)stream, b->problems,
                     b->tile_best, b->cand, b->samp, b->precision, b->sample, b->draw_pref, b->draw_blocks,
                     ordered_draws(b) ? 1 : 0, b->pool_best, (const float4*)b->comp32, (const double4*)b->comp64,
                     lazy_ok(b) ? 1 : 0, b->early_select ? 1 : 0, b->result);
  return hip_check("tpe_select");
}

int tpe_run_batch(const tpe_batch* b, void* stream) {
  int rc = check_batch(b);
  if (rc) return rc;
  if ((rc = tpe_fit_above(b, stream))) return rc;
  if ((rc = tpe_tables(b, stream))) return rc;
  if ((rc = tpe_sample(b, stream))) return rc;
  if ((rc = tpe_sort(b, stream))) return rc;
  if ((rc = tpe_score_above(b, stream))) return rc;
  if ((rc = tpe_finalize(b, stream))) return rc;
  return tpe_select(b, stream);
}

// ---------------------------------------------------------------- stage profiler
// HIP events between the stages tpe_level_run issues, on its stream; read after
// the runner's own stream synchronise (include/tpe_hip.h)
static struct {
  int on;
  int valid;
  hipEvent_t ev[TPE_N_STAGES + 1];
  tpe_stage_prof last[TPE_N_STAGES];
  int kev_used;                           // the sample stage's pass was launched with g_kev
} g_prof;

int tpe_level_profile(int32_t enable) {
  if (enable && !g_prof.ev[0]) {
    for (int i = 0; i <= TPE_N_STAGES; ++i) {
      hipError_t e = hipEventCreate(&g_prof.ev[i]);
      if (e != hipSuccess) return fail(TPE_E_HIP, hipGetErrorString(e));
    }
    for (int i = 0; i < 2; ++i) {
      hipError_t e = hipEventCreate(&g_kev[i]);
      if (e != hipSuccess) return fail(TPE_E_HIP, hipGetErrorString(e));
    }
  }
  g_prof.on = enable ? 1 : 0;
  if (enable) g_prof.valid = 0;         // (disabling keeps the last run readable)
  return TPE_OK;
}

int tpe_level_profile_read(tpe_stage_prof* out, int32_t n) {
  if (!out || n < 0) return fail(TPE_E_ARG, "tpe_level_profile_read: null output");
  if (!g_prof.valid) return fail(TPE_E_ARG, "tpe_level_profile_read: no profiled level run");
  memcpy(out, g_prof.last, sizeof(tpe_stage_prof) * (size_t)std::min<int32_t>(n, TPE_N_STAGES));
  return TPE_OK;
}

// tpe_run_batch's stages, each followed by an event
static int run_batch_profiled(const tpe_batch* b, void* stream) {
  typedef int (*stage_fn)(const tpe_batch*, void*);
  static const stage_fn fns[TPE_N_STAGES] = {tpe_fit_above, tpe_tables, tpe_sample, tpe_sort,
                                             tpe_score_above, tpe_finalize, tpe_select};
  hipStream_t s = (hipStream_t)stream;
  if (hipEventRecord(g_prof.ev[0], s) != hipSuccess) return hip_check("tpe_level_profile");
  g_prof.kev_used = 0;
  for (int i = 0; i < TPE_N_STAGES; ++i) {
    const int64_t n0 = g_launches;
    g_kev_on = i == TPE_STAGE_SAMPLE && b->n_tab_jobs > 0 && b->early_select && b->tab_fast;
    int rc = fns[i](b, stream);
    if (g_kev_on) g_prof.kev_used = 1;
    g_kev_on = false;
    if (rc) return rc;
    g_prof.last[i].launches = (int32_t)(g_launches - n0);
    if (hipEventRecord(g_prof.ev[i + 1], s) != hipSuccess) return hip_check("tpe_level_profile");
  }
  return TPE_OK;
}

// after the stream synchronise: event times and each stage's work
// hp: the host-written problems, or (expanded level) the label templates with
// the first problem of each label in xfirst
static int profile_collect(const tpe_batch& b, const tpe_pack_info& info, const tpe_problem* hp,
                           const int32_t* xfirst, int64_t n_cand) {
  const int64_t P = info.n_problems;
  double ce_tab = 0, ce_above = 0, drawn = 0;
  const bool lz = b.early_select && !(b.flags & TPE_BATCH_WRITE_CAND);
  const int64_t rows = xfirst ? info.n_expand : P;
  for (int64_t r = 0; r < rows; ++r) {
    const double n = xfirst ? (double)(xfirst[r + 1] - xfirst[r]) : 1.0;   // problems of this row
    if (hp[r].tab_mode != TPE_TAB_NONE)
      ce_tab += n * (double)(hp[r].below_len + hp[r].above_len) * (double)n_cand;
    else if (hp[r].family != TPE_FAM_CATEGORICAL)
      ce_above += n * (double)hp[r].above_len * (double)n_cand;
    // candidates the sample stage draws (lazy categoricals are scanned by the table stage)
    const bool lazy = lz && (hp[r].flags & TPE_F_CAT_LAZY) && hp[r].family == TPE_FAM_CATEGORICAL &&
                      hp[r].samp_len <= 64;
    if (!lazy) drawn += n * (double)n_cand;
  }
  const double C = (double)P * (double)n_cand;
  const double units[TPE_N_STAGES] = {
      (double)info.fit_total, (double)info.tab_units, drawn,
      (double)((b.sort_end_bit + 7) / 8) * 2.0 * 12.0 * (double)b.sort_count, ce_above, C, (double)P};
  for (int i = 0; i < TPE_N_STAGES; ++i) {
    tpe_stage_prof& q = g_prof.last[i];
    float ms = 0.f;
    if (q.launches > 0) {
      hipError_t e = hipEventElapsedTime(&ms, g_prof.ev[i], g_prof.ev[i + 1]);
      if (e != hipSuccess) return fail(TPE_E_HIP, hipGetErrorString(e));
    }
    q.ms = ms;
    q.units = units[i];
    q.ce = i == TPE_STAGE_SAMPLE ? ce_tab : (i == TPE_STAGE_ABOVE ? ce_above : 0.0);
    q.kernel_ns = 0;
    if (i == TPE_STAGE_SAMPLE && g_prof.kev_used) {
      float kms = 0.f;
      if (hipEventElapsedTime(&kms, g_kev[0], g_kev[1]) == hipSuccess) q.kernel_ns = (int32_t)(kms * 1e6f);
    }
  }
  g_prof.valid = 1;
  return TPE_OK;
}

// the device exchange of a sharded level (tpe_internal_level_run_ex): the
// exchange, the problems every rank runs, and where the outcome goes
struct LevelEx {
  const tpe_exchange* ex;
  int64_t P;
  int32_t* all_status;   // the worst status over the ranks
  int32_t* done;         // 1: the exchange ran (out holds the global winners); 0: the caller exchanges
};

static int level_run_impl(const tpe_label_in* labels, int32_t n_labels, int32_t n_cand, uint64_t seed,
                          int64_t cand_base, int64_t n_cand_global, int32_t precision, int32_t flags,
                          const tpe_level_ws* ws, tpe_level_need* need, void* stream, tpe_result* out,
                          const LevelEx* lx);

int tpe_level_run(const tpe_label_in* labels, int32_t n_labels, int32_t n_cand, uint64_t seed, int64_t cand_base,
                  int64_t n_cand_global, int32_t precision, int32_t flags, const tpe_level_ws* ws,
                  tpe_level_need* need, void* stream, tpe_result* out) {
  return level_run_impl(labels, n_labels, n_cand, seed, cand_base, n_cand_global, precision, flags, ws, need, stream,
                        out, nullptr);
}

// tpe_level_run of one rank of a candidate-sharded suggest with the RCCL
// exchange done on the device (see k_runs_reduce / k_combine); *done = 0 when
// the level could not take that path (nothing launched, no exchange made:
// the caller exchanges on the host as before)
__attribute__((visibility("hidden"))) int tpe_internal_level_run_ex(
    const tpe_label_in* labels, int32_t n_labels, int32_t n_cand, uint64_t seed, int64_t cand_base,
    int64_t n_cand_global, int32_t precision, int32_t flags, const tpe_level_ws* ws, tpe_level_need* need,
    void* stream, tpe_result* out, const tpe_exchange* ex, int64_t P_expected, int32_t* all_status, int32_t* done) {
  *done = 0;
  const LevelEx lx{ex, P_expected, all_status, done};
  return level_run_impl(labels, n_labels, n_cand, seed, cand_base, n_cand_global, precision, flags, ws, need, stream,
                        out, &lx);
}

__attribute__((visibility("hidden"))) int rccl_allgather_inplace(const tpe_exchange* ex, int64_t per,
                                                                 hipStream_t s);   // (after the RCCL loader)

// TPE_FORCE_COMBINE=1: a one-rank exchange takes the N-rank device combine
// (read per call: the tests switch it around single suggests)
static bool force_combine() {
  const char* e = getenv("TPE_FORCE_COMBINE");
  return e && e[0] == '1';
}

// host-written byte ranges of the packed level as k_upload's 8-byte words; false
// when a rounded range would pass the device blob (the caller copies instead)
static bool upload_ranges(const tpe_pack_info& info, int64_t blob_cap, UploadRanges& r, int64_t& words) {
  memset(&r, 0, sizeof(r));
  words = 0;
  for (int k = 0; k < info.n_up && k < 4; ++k) {
    const int64_t o = info.up_off[k], n = (info.up_len[k] + 7) & ~(int64_t)7;
    if ((o & 7) || o + n > blob_cap) return false;
    r.w0[r.n] = o / 8;
    r.n8[r.n] = n / 8;
    words += n / 8;
    ++r.n;
  }
  return true;
}

// the early device fit (tpe_host_pack_level's hook): the fit sections uploaded
// and tpe_fit_above launched — its problem fields into the patch rows — while
// the host packs the rest of the level; k_fit_patch applies them after the
// level's upload.  Nothing happens (the fit stage runs after the upload, as
// without the hook) unless the workspace holds what it touches.
struct EarlyFit {
  const tpe_level_ws* ws;
  hipStream_t s;
  const char* dbase;            // the pinned staging buffer's device address
  int launched;
  int rc;
};

static void early_fit_hook(void* c, const tpe_pack_info* e) {
  EarlyFit& x = *(EarlyFit*)c;
  const tpe_level_ws* ws = x.ws;
  if (x.launched || e->n_fit <= 0 || !x.dbase || !kernel_upload() || e->fit_total > ws->fit_cap ||
      e->blob_bytes > ws->blob_bytes || e->n_problems <= 0)
    return;
  UploadRanges r;
  int64_t words;
  if (!upload_ranges(*e, ws->blob_bytes, r, words) || words * 8 > ws->pinned_bytes) return;
  unsigned char* dev = (unsigned char*)ws->blob;
  const int grid = (int)std::min<int64_t>(std::max<int64_t>((words + kUploadThreads - 1) / kUploadThreads, 1), 2048);
  TPE_LAUNCH(k_upload, dim3(grid), dim3(kUploadThreads), 0, x.s, (const unsigned long long*)x.dbase,
             (unsigned long long*)dev, r);
  if ((x.rc = hip_check("k_upload (early fit)"))) return;
  tpe_batch b;
  memset(&b, 0, sizeof(b));
  b.problems = (const tpe_problem*)(dev + e->off_patch);      // (the fit's problem fields: patch rows)
  b.n_problems = (int32_t)e->n_problems;
  b.result = (tpe_result*)dev;                                // (unused by the fit)
  b.precision = TPE_PREC_F32;
  b.comp32 = (const float*)(dev + e->off_comp32);
  b.grid = (const int32_t*)(dev + e->off_grid);
  b.keys_sorted = b.keys; b.vals_sorted = b.vals;
  b.fit = (const tpe_fit_job*)(dev + e->off_fit);
  b.n_fit = e->n_fit;
  b.below_idx = (const int32_t*)(dev + e->off_below_idx);
  b.fit_seg = (const int64_t*)(dev + e->off_fit_seg);
  b.fit_total = e->fit_total;
  b.fit_keys = ws->fit_keys; b.fit_keys_sorted = ws->fit_keys_sorted;
  b.fit_vals = ws->fit_vals; b.fit_vals_sorted = ws->fit_vals_sorted;
  b.fit_max_new = e->fit_max_new; b.fit_max_obs = e->fit_max_obs; b.fit_max_merge = e->fit_max_merge;
  b.fit_n_delta = e->fit_n_delta;
  x.rc = tpe_fit_above(&b, x.s);
  x.launched = x.rc == TPE_OK;
}

static int level_run_impl(const tpe_label_in* labels, int32_t n_labels, int32_t n_cand, uint64_t seed,
                          int64_t cand_base, int64_t n_cand_global, int32_t precision, int32_t flags,
                          const tpe_level_ws* ws, tpe_level_need* need, void* stream, tpe_result* out,
                          const LevelEx* lx) {
  if (!ws || !need || (n_labels > 0 && !out)) return fail(TPE_E_ARG, "null workspace/need/out");
  memset(need, 0, sizeof(*need));
  tpe_pack_info info;
  memset(&info, 0, sizeof(info));
  // pack straight into the pinned staging buffer; the result readback area
  // follows the blob.  A level with device fits launches them from inside the
  // pack, as soon as their jobs are placed (early_fit_hook), unless profiling
  EarlyFit ef{ws, (hipStream_t)stream, nullptr, 0, TPE_OK};
  const bool hook = !g_prof.on && precision == TPE_PREC_F32 && direct_results() && early_fit_enabled();
  if (hook) {
    ef.dbase = ws->pinned_dev ? (const char*)ws->pinned_dev : device_alias(ws->pinned);
    tpe_internal_pack_hook(TpePackHook{early_fit_hook, &ef});
  }
  int rc = tpe_host_pack_level(labels, n_labels, n_cand, seed, cand_base, n_cand_global, precision, ws->pinned,
                               ws->pinned_bytes, &info);
  if (hook) tpe_internal_pack_hook(TpePackHook{nullptr, nullptr});
  if (ef.rc != TPE_OK) return ef.rc;
  if (rc != TPE_OK && rc != TPE_E_SPACE) return fail(rc, "tpe_host_pack_level: bad level description");
  tpe_internal_phase(TPE_PHASE_PACK);
  const int64_t P = info.n_problems, C = P * (int64_t)n_cand;
  const int64_t res_off = (info.blob_bytes + 255) & ~(int64_t)255;
  // early selection's per-run bests follow the results (host-visible)
  // (+ 64: the device exchange's status word between them)
  const int64_t rb_off = (res_off + P * (int64_t)sizeof(tpe_result) + 64 + 255) & ~(int64_t)255;
  need->pinned_bytes = rb_off + (info.n_tab_jobs > 0 ? info.n_tiles * (int64_t)sizeof(tpe_result) : 0);
  need->blob_bytes = info.blob_bytes;
  need->cand = C;
  need->part = info.part_total;
  need->best = info.n_tiles * TPE_BEST_PER_TILE;
  need->result = P;
  need->fit = info.fit_total;
  if (C >= ((int64_t)1 << 32)) return fail(TPE_E_ARG, "more than 2^32 candidates in one level: shard the batch");
  uint64_t sz = 0;
  // ordered draws replace the sort of the pruned problems' candidates
  const bool od = precision == TPE_PREC_F32 && (flags & TPE_BATCH_ORDERED_DRAWS) && info.n_sorted > 0 &&
                  info.sort_count > 0 && info.n_pooled == 0;
  if (info.n_pooled > 0) need->pool_best = P;
  need->tab = info.tab_units;
  if (od) need->draw_pref = info.n_sorted * (info.draw_blocks + 1);
  if (!od && info.sort_end_bit > 0 && info.sort_count > 0) {
    if ((rc = tpe_sort_workspace_bytes(info.sort_count, &sz))) return rc;
    need->sort_tmp_bytes = (int64_t)sz;
  }
  if (rc == TPE_E_SPACE || need->pinned_bytes > ws->pinned_bytes || need->blob_bytes > ws->blob_bytes ||
      need->cand > ws->cand_cap || need->part > ws->part_cap || need->best > ws->best_cap ||
      need->result > ws->result_cap || need->fit > ws->fit_cap || need->sort_tmp_bytes > ws->sort_tmp_bytes ||
      need->draw_pref > ws->draw_pref_cap ||
      need->pool_best > ws->pool_best_cap || need->tab > ws->tab_cap)
    return fail(TPE_E_SPACE, "level workspace too small (see tpe_level_need)");
  if (P == 0) return TPE_OK;
  hipStream_t s = (hipStream_t)stream;
  unsigned char* host = (unsigned char*)ws->pinned;
  unsigned char* dev = (unsigned char*)ws->blob;
  // the host-written ranges (tpe_pack_info.up_*): by k_upload, a copy kernel on
  // the compute queue, or by the copy engine (TPE_UPLOAD_COPY=1)
  hipError_t e = hipSuccess;
  char* dbase = !direct_results() ? nullptr : (ws->pinned_dev ? (char*)ws->pinned_dev : device_alias(ws->pinned));
  {
    UploadRanges r;
    int64_t words = 0;
    if (dbase && kernel_upload() && upload_ranges(info, ws->blob_bytes, r, words) && words <= ((int64_t)8 << 20)) {
      const int grid = (int)std::min<int64_t>(std::max<int64_t>((words + kUploadThreads - 1) / kUploadThreads, 1),
                                              2048);
      TPE_LAUNCH(k_upload, dim3(grid), dim3(kUploadThreads), 0, s, (const unsigned long long*)dbase,
                 (unsigned long long*)dev, r);
      if ((rc = hip_check("k_upload"))) return rc;
    } else {
      for (int k = 0; k < info.n_up && e == hipSuccess; ++k)
        e = hipMemcpyAsync(dev + info.up_off[k], host + info.up_off[k], (size_t)info.up_len[k], hipMemcpyHostToDevice,
                           s);
    }
  }
  if (e != hipSuccess) return fail(TPE_E_HIP, hipGetErrorString(e));
  // expanded level: the templates, first problems and new ids (uploaded above)
  const tpe_problem* xtmpl = nullptr;
  const int32_t* xfirst = nullptr;
  const int64_t n_tiles_p = P > 0 ? info.n_tiles / P : 0;
  if (info.n_expand > 0) {
    const int64_t nl = info.n_expand;
    const int64_t first_off = ((int64_t)(nl * sizeof(tpe_problem)) + 255) & ~(int64_t)255;
    const int64_t ctr_off = (first_off + (nl + 1) * (int64_t)sizeof(int32_t) + 255) & ~(int64_t)255;
    xtmpl = (const tpe_problem*)(host + info.off_expand);
    xfirst = (const int32_t*)(host + info.off_expand + first_off);
    if (nl >= ((int64_t)1 << 31) || xfirst[0] != 0 || xfirst[nl] != P || n_tiles_p * P != info.n_tiles ||
        n_tiles_p < 1 || n_cand > n_tiles_p * kTile || info.n_tab_tiles != info.n_tiles)
      return fail(TPE_E_ARG, "tpe_level_run: bad expanded level");
    for (int64_t l = 0; l < nl; ++l)
      if (xfirst[l + 1] < xfirst[l] || xtmpl[l].tab_mode == TPE_TAB_NONE)
        return fail(TPE_E_ARG, "tpe_level_run: bad expanded level");
    const int64_t n_thr = std::max<int64_t>(P * kProbWords, info.n_tiles);
    TPE_LAUNCH(k_expand, dim3((unsigned)((n_thr + kExpandThreads - 1) / kExpandThreads)), dim3(kExpandThreads), 0, s,
               (const tpe_problem*)(dev + info.off_expand), (const int32_t*)(dev + info.off_expand + first_off),
               (int)nl, (const uint32_t*)(dev + info.off_expand + ctr_off), (tpe_problem*)(dev + info.off_problems),
               (tpe_tile*)(dev + info.off_tiles), P, (int32_t)n_tiles_p, n_cand);
    if ((rc = hip_check("k_expand"))) return rc;
  }
  if (ef.launched) {                           // the early fit's problem fields into the rows
    TPE_LAUNCH(k_fit_patch, dim3(info.n_fit), dim3(64), 0, s, (const tpe_fit_job*)(dev + info.off_fit),
               (const tpe_problem*)(dev + info.off_patch), (tpe_problem*)(dev + info.off_problems));
    if ((rc = hip_check("k_fit_patch"))) return rc;
  }
  tpe_batch b;
  memset(&b, 0, sizeof(b));
  b.problems = (const tpe_problem*)(dev + info.off_problems);
  b.n_problems = (int32_t)P;
  b.precision = precision;
  b.flags = flags;
  b.sample = 1;
  b.sort_end_bit = info.sort_end_bit;
  b.key_bits = info.key_bits;
  b.comp32 = (const float*)(dev + info.off_comp32);
  b.comp64 = (const double*)(dev + info.off_comp64);
  b.samp = (const double*)(dev + info.off_samp);
  b.grid = (const int32_t*)(dev + info.off_grid);
  b.cand = ws->cand; b.coord = ws->coord; b.keys = ws->keys; b.vals = ws->vals;
  if (od) {
    b.keys_sorted = ws->keys; b.vals_sorted = ws->vals;
    b.draw_pref = ws->draw_pref; b.draw_blocks = info.draw_blocks; b.n_sorted = (int32_t)info.n_sorted;
  } else if (info.sort_end_bit > 0) {
    b.keys_sorted = ws->keys_sorted; b.vals_sorted = ws->vals_sorted;
    b.sort_tmp = ws->sort_tmp; b.sort_tmp_bytes = (uint64_t)ws->sort_tmp_bytes;
  } else {
    b.keys_sorted = ws->keys; b.vals_sorted = ws->vals;
  }
  b.total_cand = C;
  b.sort_count = info.sort_count;
  b.tiles = (const tpe_tile*)(dev + info.off_tiles);
  b.n_tiles = (int32_t)info.n_tiles;
  // (the packer gives every problem n_tiles_p tiles {r, j * kTile}, in order)
  b.tiles_per_problem = n_tiles_p * P == info.n_tiles ? (int32_t)n_tiles_p : 0;
  b.fin_tiles = (const int32_t*)(dev + info.off_fin_tiles);
  b.n_fin_tiles = (int32_t)info.n_fin_tiles;
  b.work = (const tpe_work*)(dev + info.off_work);
  b.n_work_cont = info.n_work_cont; b.n_work_qgauss = info.n_work_qgauss; b.n_work_qlog = info.n_work_qlog;
  b.part = ws->part;
  b.tile_best = ws->tile_best;
  if (info.n_pooled > 0) b.pool_best = ws->pool_best;
  b.samp_tiles = (const int32_t*)(dev + info.off_samp_tiles);
  b.n_samp_tiles = (int32_t)info.n_samp_tiles;
  b.n_samp_eager = (int32_t)info.n_samp_eager;
  b.tab_tiles = xtmpl ? nullptr : (const int32_t*)(dev + info.off_tab_tiles);   // (expanded: every tile, in order)
  b.n_tab_tiles = (int32_t)info.n_tab_tiles;
  if (info.n_tab_jobs > 0) {
    b.tab_jobs = (const tpe_tab_job*)(dev + info.off_tab_jobs);
    b.n_tab_jobs = (int32_t)info.n_tab_jobs;
    b.tab_blocks = (int32_t)info.tab_blocks;
    b.tab = ws->tab;
    b.tab_units = info.tab_units;
    b.fgt_max_boxes = info.fgt_max_boxes;
    b.fgt_max_cells = (int32_t)info.fgt_max_cells;
  }
  // the select stage writes the results straight into the pinned staging
  // buffer when the device can address it (no readback copy)
  tpe_result* rh = (tpe_result*)(host + res_off);
  tpe_result* rd = dbase ? (tpe_result*)(dbase + res_off) : nullptr;
  // early selection (include/tpe_hip.h): the sample stage reports each run of
  // tabulated tiles to host-visible memory, the table stage selects the lazy
  // categoricals, and only the rest go through the select stage
  // (expanded level: no host-written problems; every problem is tabulated)
  const tpe_problem* hp = xtmpl ? nullptr : (const tpe_problem*)(host + info.off_problems);
  if (info.n_tab_jobs > 0 && dbase) {
    b.early_select = 1;
    b.run_best = (tpe_result*)(dbase + rb_off);
    const bool lz = !(flags & TPE_BATCH_WRITE_CAND);
    int32_t late = 0;
    for (int64_t r = 0; hp && r < P; ++r) {
      const tpe_problem& q = hp[r];
      const bool lazy = lz && (q.flags & TPE_F_CAT_LAZY) && q.family == TPE_FAM_CATEGORICAL && q.samp_len <= 64;
      late += !(lazy || q.tab_mode != TPE_TAB_NONE);
    }
    b.n_late = late;
    // the sample stage's specialised kernel: every tabulated problem cells with
    // both tables within its LDS and a staged sampler (the problem rows: the
    // host's, or an expanded level's label templates)
    const bool fast_ok = precision == TPE_PREC_F32 && !(flags & (TPE_BATCH_WRITE_CAND | TPE_BATCH_NO_TAB_FAST)) &&
                         !tab_fast_disabled();
    // k_sample_fast: every tabulated problem a log-polynomial cells table or a
    // lattice within its LDS; k_sample_tab's FAST pass: log-polynomial cells only
    bool fast = fast_ok, fast_lp = fast_ok;
    const tpe_problem* rows = hp ? hp : xtmpl;
    const int64_t n_rows = hp ? P : (xtmpl ? info.n_expand : 0);
    int max_cells = 0, max_units = 0, max_samp = 0;
    for (int64_t r = 0; (fast || fast_lp) && r < n_rows; ++r) {
      const tpe_problem& q = rows[r];
      if (q.tab_mode == TPE_TAB_NONE) continue;
      const bool samp_ok = q.samp_len > 0 && q.samp_len <= kCumLds;
      const bool lp = q.tab_mode == TPE_TAB_CELLS && (q.flags & TPE_F_LOGPOLY) && q.tab_n[0] <= kTabLdsCells && samp_ok;
      const bool lat = q.tab_mode == TPE_TAB_LATTICE && q.tab_n[0] <= kFastLatMax && samp_ok;
      fast_lp = fast_lp && lp;
      fast = fast && (lp || lat);
      max_cells = std::max(max_cells, lp ? q.tab_n[0] : 0);
      max_units = std::max(max_units, lp ? TPE_TAB_ROW_UNITS * q.tab_n[0] : fast_lat_units(q.tab_n[0]));
      max_samp = std::max(max_samp, q.samp_len);
    }
    // (the small-workgroup kernel when the level's tables and sampler rows fit its LDS)
    const bool fast2 = fast && !fast2_disabled() && !(flags & TPE_BATCH_NO_FAST2) && max_cells <= kFastMaxCells &&
                       max_units <= kFastMaxUnits &&
                       max_samp <= kFastSamp;
    b.tab_fast = n_rows > 0 ? (fast2 ? 1 + max_units : fast_lp ? 1 : 0) : 0;
  }
  b.result = rd ? rd : ws->result;
  // device exchange (sharded level over RCCL): run records and results in
  // device scratch after the exchange slots, combined on the device
  const int64_t xper = TPE_EXCHANGE_HEADER + P * (int64_t)sizeof(tpe_result);
  unsigned char* xrun = nullptr;
  bool dex = false;
  if (lx && lx->ex && lx->ex->comm && dbase && b.early_select && lx->P == P) {
    const int64_t base = ((int64_t)lx->ex->world * xper + 255) & ~(int64_t)255;
    const int64_t need_x = base + (info.n_tiles + P) * (int64_t)sizeof(tpe_result);
    const int64_t runs_bytes = 2 * P * (int64_t)sizeof(int32_t);
    if (lx->ex->dev && lx->ex->dev_bytes >= need_x && runs_bytes <= info.n_tiles * (int64_t)sizeof(tpe_result)) {
      dex = true;
      xrun = (unsigned char*)lx->ex->dev + base;
      b.run_best = (tpe_result*)xrun;
      b.result = (tpe_result*)(xrun + info.n_tiles * (int64_t)sizeof(tpe_result));
    }
  }
  if (info.n_fit > 0 && !ef.launched) {
    b.fit = (const tpe_fit_job*)(dev + info.off_fit);
    b.n_fit = info.n_fit;
    b.below_idx = (const int32_t*)(dev + info.off_below_idx);
    b.fit_seg = (const int64_t*)(dev + info.off_fit_seg);
    b.fit_total = info.fit_total;
    b.fit_keys = ws->fit_keys; b.fit_keys_sorted = ws->fit_keys_sorted;
    b.fit_vals = ws->fit_vals; b.fit_vals_sorted = ws->fit_vals_sorted;
    b.fit_max_new = info.fit_max_new; b.fit_max_obs = info.fit_max_obs; b.fit_max_merge = info.fit_max_merge;
    b.fit_n_delta = info.fit_n_delta;
  }
  if (g_prof.on) {
    g_prof.valid = 0;
    if ((rc = check_batch(&b)) || (rc = run_batch_profiled(&b, stream))) return rc;
  } else if ((rc = tpe_run_batch(&b, stream))) {
    return rc;
  }
  if (dex) {
    // each problem's span of the tabulated tile list: from the packer's layout
    // on the device (a level of at most kRunsDevMax problems with tpp tiles
    // each), else written by the host (host-visible: the run-record area is
    // free in this mode) — its runs are enumerated on the device as the host
    // reduction below enumerates them
    const int n_tab = (int)info.n_tab_tiles, per = tab_tiles_per_wg(n_tab, tab_wgs_per_cu(&b));
    const int tpp = b.tiles_per_problem;
    const int32_t* d_span = nullptr;
    if (P > kRunsDevMax || tpp <= 0) {
      int32_t* span = (int32_t*)(host + rb_off);
      if (xtmpl) {                                   // expanded: every problem's tiles, in order
        for (int64_t r = 0; r < P; ++r) { span[2 * r] = (int32_t)(r * n_tiles_p); span[2 * r + 1] = (int32_t)n_tiles_p; }
      } else {
        for (int64_t r = 0; r < P; ++r) span[2 * r] = span[2 * r + 1] = 0;
        const int32_t* list = (const int32_t*)(host + info.off_tab_tiles);
        const tpe_tile* tl = (const tpe_tile*)(host + info.off_tiles);
        for (int i = 0; i < n_tab; ++i) {
          const int pr = tl[list[i]].problem;
          if (span[2 * pr + 1]++ == 0) span[2 * pr] = i;
        }
      }
      d_span = (const int32_t*)(dbase + rb_off);
    }
    const unsigned int blocks = (unsigned int)((P + kCombThreads / 64 - 1) / (kCombThreads / 64));
    unsigned char* slot = (unsigned char*)lx->ex->dev + (int64_t)lx->ex->rank * xper;
    int32_t* st_host = (int32_t*)(host + res_off + P * (int64_t)sizeof(tpe_result));   // (the pad before rb_off)
    int32_t* st_dev = (int32_t*)(dbase + res_off + P * (int64_t)sizeof(tpe_result));
    // (forced exchange on one rank: no gather, no combine — unless
    // TPE_FORCE_COMBINE=1, the tests' way to run the N > 1 device combine,
    // slot → in-place all-gather → k_combine, on the box's one GPU)
    const bool one = lx->ex->world == 1 && !force_combine();
    TPE_LAUNCH(k_runs_reduce, dim3(blocks), dim3(kCombThreads), 0, s, d_span, xtmpl ? nullptr : b.tab_tiles, per,
               b.problems, tpp, (const tpe_result*)b.run_best, (const tpe_result*)b.result, P, slot, (int32_t)TPE_OK,
               one ? rd : (tpe_result*)nullptr, one ? st_dev : (int32_t*)nullptr);
    if ((rc = hip_check("k_runs_reduce"))) return rc;
    if ((rc = rccl_allgather_inplace(lx->ex, xper, s))) return rc;
    // the level's collective is issued: from here every failure is this level's
    // status (done = 1), so the caller never issues a second collective for it
    // that the other ranks would not join
    auto gathered_fail = [&](int code) {
      *lx->all_status = code;
      *lx->done = 1;
      return code;
    };
    if (!one) {
      const unsigned int cblocks = (unsigned int)((P + kCombThreads - 1) / kCombThreads);   // (a thread a problem)
      TPE_LAUNCH(k_combine, dim3(cblocks), dim3(kCombThreads), 0, s, (const unsigned char*)lx->ex->dev,
                 lx->ex->world, xper, P, rd, st_dev);
      if ((rc = hip_check("k_combine"))) return gathered_fail(rc);
    }
    tpe_internal_phase(TPE_PHASE_LAUNCHED);
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return gathered_fail(fail(TPE_E_HIP, hipGetErrorString(e)));
    tpe_internal_phase(TPE_PHASE_SYNCED);
    memcpy(out, rh, (size_t)P * sizeof(tpe_result));
    *lx->all_status = *(volatile int32_t*)st_host;
    *lx->done = 1;
    tpe_internal_phase(TPE_PHASE_LEVEL);
    return g_prof.on ? profile_collect(b, info, xtmpl ? xtmpl : hp, xfirst, n_cand) : TPE_OK;
  }
  e = rd ? hipSuccess : hipMemcpyAsync(rh, ws->result, (size_t)P * sizeof(tpe_result), hipMemcpyDeviceToHost, s);
  tpe_internal_phase(TPE_PHASE_LAUNCHED);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return fail(TPE_E_HIP, hipGetErrorString(e));
  tpe_internal_phase(TPE_PHASE_SYNCED);
  if (b.early_select) {
    // each tabulated problem: the best of its runs (np.argmax order), runs
    // enumerated exactly as the sample stage partitions the tile list
    // (expanded level: the identity list, tile t of problem t / n_tiles_p)
    const tpe_result* rb = (const tpe_result*)(host + rb_off);
    const int32_t* list = xtmpl ? nullptr : (const int32_t*)(host + info.off_tab_tiles);
    const tpe_tile* tl = xtmpl ? nullptr : (const tpe_tile*)(host + info.off_tiles);
    auto tile_of = [&](int i) { return list ? list[i] : i; };
    auto prob_of = [&](int t) { return tl ? tl[t].problem : (int)(t / n_tiles_p); };
    const int n_tab = (int)info.n_tab_tiles, per = tab_tiles_per_wg(n_tab, tab_wgs_per_cu(&b));
    if (xtmpl && n_tiles_p > 0 && per % n_tiles_p == 0) {
      // expanded level (every problem tabulated, tiles in order) whose workgroups
      // hold whole problems: each problem is one run, recorded at its first
      // tile — gathered straight into `out`, in slices on the worker pool (a
      // batched level has ~10^5 of them)
      struct Gather { const tpe_result* rb; tpe_result* out; int64_t P, ntp, slice; } g{rb, out, P, n_tiles_p, 4096};
      tpe_pool::parallel_for((int)((P + g.slice - 1) / g.slice), [](void* c, int k) {
        const Gather& q = *(const Gather*)c;
        const int64_t r1 = std::min(q.P, (k + 1) * q.slice);
        for (int64_t r = k * q.slice; r < r1; ++r) q.out[r] = q.rb[r * q.ntp];
      }, &g);
      tpe_internal_phase(TPE_PHASE_LEVEL);
      return g_prof.on ? profile_collect(b, info, xtmpl, xfirst, n_cand) : TPE_OK;
    }
    const int tpp = b.tiles_per_problem;
    if (tpp > 0) {
      // the packer's layout (every problem tpp tiles, the list the tabulated
      // problems' tiles in problem order): a problem's runs start at its first
      // list position and at every multiple of per after it — visited directly,
      // not found by a scan of the whole list (the headline's 5 problems have
      // ~5000 tabulated tiles and a few hundred runs)
      int rank = 0;
      for (int64_t r = 0; r < P; ++r) {
        if (hp && hp[r].tab_mode == TPE_TAB_NONE) continue;
        tpe_result w{0, 0, 0, 0, -1, -1};
        const int a = rank * tpp, e = a + tpp;
        for (int pos = a; pos < e; pos = (pos / per + 1) * per) {
          const tpe_result& c = rb[r * tpp + (pos - a)];
          if (host_better(c.score, c.idx, w.score, w.idx)) w = c;
        }
        rh[r] = w;
        ++rank;
      }
    } else {
      for (int64_t r = 0; r < P; ++r)
        if (!hp || hp[r].tab_mode != TPE_TAB_NONE) { rh[r] = tpe_result{0, 0, 0, 0, -1, -1}; }
      for (int i = 0; i < n_tab; ++i) {
        const int t = tile_of(i), pr = prob_of(t);
        if (i % per != 0 && prob_of(tile_of(i - 1)) == pr) continue;      // not a run's first tile
        const tpe_result& c = rb[t];
        tpe_result& w = rh[pr];
        if (host_better(c.score, c.idx, w.score, w.idx)) w = c;
      }
    }
  }
  memcpy(out, rh, (size_t)P * sizeof(tpe_result));
  tpe_internal_phase(TPE_PHASE_LEVEL);
  return g_prof.on ? profile_collect(b, info, xtmpl ? xtmpl : hp, xfirst, n_cand) : TPE_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- shard exchange
// RCCL entry points, resolved from librccl on first use (include/tpe_hip.h)
namespace {
struct Rccl {
  bool tried = false, ok = false;
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
};
Rccl& rccl() {
  static Rccl r;
  if (!r.tried) {
    r.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (h) {
      r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
      r.init = (decltype(r.init))dlsym(h, "ncclCommInitRank");
      r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
      r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
      r.err = (decltype(r.err))dlsym(h, "ncclGetErrorString");
      r.ok = r.get_id && r.init && r.all_gather && r.destroy && r.err;
    }
  }
  return r;
}
int rccl_fail(const char* what, ncclResult_t e) {
  snprintf(g_err, sizeof(g_err), "%s: %s", what, rccl().err ? rccl().err(e) : "rccl error");
  return TPE_E_HIP;
}
}  // namespace



extern "C" {

static std::atomic<int64_t> g_collectives{0};       // ncclAllGather calls issued (tpe_collectives_issued)

// every rank's `per` bytes at its slot of ex->dev gathered in place on stream s
// (one rank: the identity, skipped — unless TPE_FORCE_COMBINE=1 runs the
// N-rank combine on one GPU, where the collective itself is issued too)
__attribute__((visibility("hidden"))) int rccl_allgather_inplace(const tpe_exchange* ex, int64_t per, hipStream_t s) {
  if (ex->world == 1 && !(force_combine() && ex->comm)) return TPE_OK;
  Rccl& r = rccl();
  if (!r.ok) return fail(TPE_E_HIP, "librccl not found");
  unsigned char* d = (unsigned char*)ex->dev;
  const ncclResult_t ne = r.all_gather(d + (size_t)per * ex->rank, d, (size_t)per, ncclUint8, (ncclComm_t)ex->comm, s);
  if (ne != ncclSuccess) return rccl_fail("ncclAllGather", ne);
  g_collectives.fetch_add(1, std::memory_order_relaxed);
  return TPE_OK;
}

int tpe_scatter_f64(const void* src, int64_t k, double* dst, void* stream) {
  if (k < 0 || (k > 0 && (!src || !dst))) return fail(TPE_E_ARG, "tpe_scatter_f64: bad arguments");
  if (k == 0) return TPE_OK;
  const unsigned int grid = (unsigned int)std::min<int64_t>((k + kColThreads - 1) / kColThreads, 1024);
  TPE_LAUNCH(k_scatter_f64, dim3(grid), dim3(kColThreads), 0, (hipStream_t)stream,
             (const unsigned long long*)src, k, dst);
  return hip_check("k_scatter_f64");
}

int tpe_move_ranges(const void* ranges, int32_t n_ranges, int32_t elem_bytes, const void* src, void* dst,
                    void* stream) {
  if (n_ranges < 0 || (elem_bytes != 4 && elem_bytes != 8) || (n_ranges > 0 && (!ranges || !src || !dst)) ||
      src == dst)
    return fail(TPE_E_ARG, "tpe_move_ranges: bad arguments");
  if (n_ranges == 0) return TPE_OK;
  const unsigned int grid = (unsigned int)std::min<int32_t>(n_ranges, 2048);
  if (elem_bytes == 8)
    TPE_LAUNCH(k_move_ranges<unsigned long long>, dim3(grid), dim3(kColThreads), 0, (hipStream_t)stream,
               (const long long*)ranges, n_ranges, (const unsigned long long*)src, (unsigned long long*)dst);
  else
    TPE_LAUNCH(k_move_ranges<uint32_t>, dim3(grid), dim3(kColThreads), 0, (hipStream_t)stream,
               (const long long*)ranges, n_ranges, (const uint32_t*)src, (uint32_t*)dst);
  return hip_check("k_move_ranges");
}

int tpe_collectives_issued(int64_t* n) {
  if (!n) return fail(TPE_E_ARG, "tpe_collectives_issued: null");
  *n = g_collectives.load(std::memory_order_relaxed);
  return TPE_OK;
}

int tpe_comm_unique_id(void* id) {
  if (!id) return fail(TPE_E_ARG, "tpe_comm_unique_id: null id");
  Rccl& r = rccl();
  if (!r.ok) return fail(TPE_E_HIP, "librccl not found");
  ncclUniqueId u;
  const ncclResult_t e = r.get_id(&u);
  if (e != ncclSuccess) return rccl_fail("ncclGetUniqueId", e);
  static_assert(sizeof(u) == TPE_COMM_ID_BYTES, "unique id size");
  memcpy(id, &u, sizeof(u));
  return TPE_OK;
}

int tpe_comm_init(int32_t rank, int32_t world, const void* id, int32_t device, void** comm) {
  if (!id || !comm || world < 1 || rank < 0 || rank >= world) return fail(TPE_E_ARG, "tpe_comm_init: bad arguments");
  Rccl& r = rccl();
  if (!r.ok) return fail(TPE_E_HIP, "librccl not found");
  if (hipSetDevice(device) != hipSuccess) return hip_check("tpe_comm_init/hipSetDevice");
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  const ncclResult_t e = r.init(&c, world, u, rank);
  if (e != ncclSuccess) return rccl_fail("ncclCommInitRank", e);
  *comm = (void*)c;
  return TPE_OK;
}

int tpe_comm_destroy(void* comm) {
  if (!comm) return TPE_OK;
  Rccl& r = rccl();
  if (!r.ok) return fail(TPE_E_HIP, "librccl not found");
  const ncclResult_t e = r.destroy((ncclComm_t)comm);
  return e == ncclSuccess ? TPE_OK : rccl_fail("ncclCommDestroy", e);
}

int tpe_combine_results(const tpe_result* all, int32_t world, int64_t P, tpe_result* out) {
  if (world < 1 || P < 0 || (P > 0 && (!all || !out))) return fail(TPE_E_ARG, "tpe_combine_results: bad arguments");
  for (int64_t p = 0; p < P; ++p) {
    tpe_result w = all[p];
    for (int32_t r = 1; r < world; ++r) {
      const tpe_result& c = all[(size_t)r * P + p];
      if (c.idx < 0) continue;
      if (w.idx < 0 || host_better(c.score, c.global_idx, w.score, w.global_idx)) w = c;
    }
    out[p] = w;
  }
  return TPE_OK;
}

int tpe_exchange_allgather(const tpe_exchange* ex, const void* mine, int64_t bytes, void* all, void* stream) {
  if (!ex || bytes < 0 || (bytes > 0 && (!mine || !all)) || ex->world < 1 || ex->rank < 0 || ex->rank >= ex->world)
    return fail(TPE_E_ARG, "tpe_exchange_allgather: bad arguments");
  const int W = ex->world;
  if (ex->comm) {
    Rccl& r = rccl();
    if (!r.ok) return fail(TPE_E_HIP, "librccl not found");
    if (!ex->dev || ex->dev_bytes < bytes * W) return fail(TPE_E_ARG, "tpe_exchange: device scratch too small");
    if (bytes == 0) return TPE_OK;
    hipStream_t s = (hipStream_t)stream;
    unsigned char* d = (unsigned char*)ex->dev;
    hipError_t e = hipMemcpyAsync(d + (size_t)bytes * ex->rank, mine, (size_t)bytes, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return fail(TPE_E_HIP, hipGetErrorString(e));
    // in place: rank r's block already sits at its slot of the receive buffer
    const ncclResult_t ne = r.all_gather(d + (size_t)bytes * ex->rank, d, (size_t)bytes, ncclUint8,
                                         (ncclComm_t)ex->comm, s);
    if (ne != ncclSuccess) return rccl_fail("ncclAllGather", ne);
    g_collectives.fetch_add(1, std::memory_order_relaxed);
    e = hipMemcpyAsync(all, d, (size_t)bytes * W, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(TPE_E_HIP, hipGetErrorString(e));
    return TPE_OK;
  }
  if (!ex->gather) return fail(TPE_E_ARG, "tpe_exchange: neither a communicator nor a gather function");
  if (ex->gather(ex->ctx, mine, bytes, all) != 0) return fail(TPE_E_HIP, "tpe_exchange: gather failed");
  return TPE_OK;
}

// one exchange of a sharded level (tpe_suggest.cpp): every rank's status and
// P results -> the global winners in res, the worst status in *status
__attribute__((visibility("hidden"))) int tpe_internal_exchange(const tpe_exchange* ex, void* stream, int32_t my_status,
                                                                tpe_result* res, int64_t P, int32_t* status) {
  const int64_t per = TPE_EXCHANGE_HEADER + P * (int64_t)sizeof(tpe_result);
  const int W = ex->world;
  static thread_local std::vector<unsigned char> mine, all;
  mine.assign((size_t)per, 0);
  all.resize((size_t)per * W);
  memcpy(mine.data(), &my_status, sizeof(my_status));
  if (P > 0) memcpy(mine.data() + TPE_EXCHANGE_HEADER, res, (size_t)P * sizeof(tpe_result));
  const int xrc = tpe_exchange_allgather(ex, mine.data(), per, all.data(), stream);
  if (xrc != TPE_OK) return xrc;
  int32_t worst = TPE_OK;
  static thread_local std::vector<tpe_result> recs;
  recs.resize((size_t)std::max<int64_t>(P * W, 1));
  for (int r = 0; r < W; ++r) {
    int32_t st;
    memcpy(&st, all.data() + (size_t)per * r, sizeof(st));
    // a hard error outranks a workspace retry (every rank then fails, none waits)
    if (st != TPE_OK && (worst == TPE_OK || worst == TPE_E_SPACE)) worst = st;
    if (P > 0) memcpy(recs.data() + (size_t)r * P, all.data() + (size_t)per * r + TPE_EXCHANGE_HEADER,
                      (size_t)P * sizeof(tpe_result));
  }
  *status = worst;
  if (worst != TPE_OK || P == 0) return TPE_OK;
  return tpe_combine_results(recs.data(), W, P, res);
}

}  // extern "C"
