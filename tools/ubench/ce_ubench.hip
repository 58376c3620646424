// Microbenchmark: ceiling of one "component evaluation" (CE) on gfx950.
//
// A CE is the inner step of the TPE mixture log-density:
//   t = c_k - (a_k * ((x - mu_hi_k) - mu_lo_k))^2 ;  s += exp2(t)
// i.e. sub, sub, mul, fma, v_exp_f32, add.  Components are wave-uniform and
// are read through the scalar cache; candidates live in VGPRs (R per lane).
// Variants isolate the VALU part, the transcendental part and a packed-f32
// form so the roofline used by bench.py is a measured ceiling, not a guess.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <chrono>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE, int R>
__global__ __launch_bounds__(256) void ce_kernel(const float4* __restrict__ comp, int K,
                                                 const float* __restrict__ xin, float* __restrict__ out) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  float x[R], s[R];
#pragma unroll
  for (int r = 0; r < R; ++r) { x[r] = xin[tid * R + r]; s[r] = 0.f; }
#pragma unroll 8
  for (int k = 0; k < K; ++k) {
    const float4 c = comp[k];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (MODE == 0 || MODE == 3) {         // full CE
        float d = (x[r] - c.x) - c.y;
        float z = d * c.z;
        float t = __builtin_fmaf(-z, z, c.w);
        s[r] += __builtin_amdgcn_exp2f(t);
      } else if (MODE == 1) {  // VALU only (exp replaced by nothing)
        float d = (x[r] - c.x) - c.y;
        float z = d * c.z;
        float t = __builtin_fmaf(-z, z, c.w);
        s[r] += t;
      } else if (MODE == 2) {  // exp only + add
        s[r] += __builtin_amdgcn_exp2f(x[r] - c.x);
      }
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) acc += s[r];
  out[tid] = acc;
}

// packed-f32 form: two candidates per v_pk_* instruction
template <int R2>
__global__ __launch_bounds__(256) void ce_kernel_pk(const float4* __restrict__ comp, int K,
                                                    const float* __restrict__ xin, float* __restrict__ out) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  f2 x[R2], s[R2];
#pragma unroll
  for (int r = 0; r < R2; ++r) { x[r] = f2{xin[tid * 2 * R2 + 2 * r], xin[tid * 2 * R2 + 2 * r + 1]}; s[r] = f2{0.f, 0.f}; }
  for (int k = 0; k < K; ++k) {
    const float4 c = comp[k];
    const f2 mh = f2{c.x, c.x}, ml = f2{c.y, c.y}, a = f2{c.z, c.z}, cw = f2{c.w, c.w};
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      f2 d = (x[r] - mh) - ml;
      f2 z = d * a;
      f2 t = cw - z * z;
      f2 e = f2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
      s[r] += e;
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < R2; ++r) acc += s[r].x + s[r].y;
  out[tid] = acc;
}


// exp2 by range reduction + degree-5 minimax polynomial (packed f32), t <= 0.
// rint via the 1.5*2^23 magic constant: no v_rndne / v_cvt, the integer part is
// read from the low mantissa bits and shifted straight into the exponent.
__device__ __forceinline__ f2 exp2_poly(f2 t) {
  const f2 M = f2{12582912.0f, 12582912.0f};
  f2 r = t + M;
  f2 n = r - M;
  f2 f = t - n;                       // [-0.5, 0.5]
  f2 p = f2{1.32764655e-3f, 1.32764655e-3f};
  p = p * f + f2{9.67554096e-3f, 9.67554096e-3f};
  p = p * f + f2{5.55071346e-2f, 5.55071346e-2f};
  p = p * f + f2{2.40221202e-1f, 2.40221202e-1f};
  p = p * f + f2{6.93146944e-1f, 6.93146944e-1f};
  p = p * f + f2{1.00000012f, 1.00000012f};
  int ix = __float_as_int(p.x) + (__float_as_int(r.x) << 23);
  int iy = __float_as_int(p.y) + (__float_as_int(r.y) << 23);
  return f2{__int_as_float(ix), __int_as_float(iy)};
}

// MODE 0: all v_exp_f32; MODE 1: all polynomial; MODE 2: 1 of every R2 pairs polynomial
template <int R2, int MODE>
__global__ __launch_bounds__(256) void ce_kernel_mix(const float4* __restrict__ comp, int K,
                                                     const float* __restrict__ xin, float* __restrict__ out) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  f2 x[R2], s[R2];
#pragma unroll
  for (int r = 0; r < R2; ++r) { x[r] = f2{xin[tid * 2 * R2 + 2 * r], xin[tid * 2 * R2 + 2 * r + 1]}; s[r] = f2{0.f, 0.f}; }
#pragma unroll 2
  for (int k = 0; k < K; ++k) {
    const float4 c = comp[k];
    const f2 mh = f2{c.x, c.x}, ml = f2{c.y, c.y}, a = f2{c.z, c.z}, cw = f2{c.w, c.w};
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      f2 d = (x[r] - mh) - ml;
      f2 z = d * a;
      f2 t = cw - z * z;
      f2 e;
      if (MODE == 1 || (MODE == 2 && r == 0) || (MODE == 3 && r < 2))
        e = exp2_poly(t);
      else
        e = f2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
      s[r] += e;
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < R2; ++r) acc += s[r].x + s[r].y;
  out[tid] = acc;
}

// fp64 quantized CE: w * (Phi(ub) - Phi(lb)) with two erf evaluations
template <int R>
__global__ __launch_bounds__(256) void qce_kernel(const double4* __restrict__ comp, int K,
                                                  const double* __restrict__ xin, double* __restrict__ out) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  double u[R], l[R], s[R];
#pragma unroll
  for (int r = 0; r < R; ++r) { u[r] = xin[tid * R + r] + 0.5; l[r] = xin[tid * R + r] - 0.5; s[r] = 0.0; }
  for (int k = 0; k < K; ++k) {
    const double4 c = comp[k];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      double pu = erf((u[r] - c.x) * c.y);
      double pl = erf((l[r] - c.x) * c.y);
      s[r] += c.z * (pu - pl);
    }
  }
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) acc += s[r];
  out[tid] = acc;
}

template <typename F>
static double time_ms(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int K = 4096;
  const int threads = 256;
  const int blocks = 256 * 8;     // 8 WGs per CU
  const int R = 8;
  const size_t nthr = (size_t)threads * blocks;
  std::vector<float4> hc(K);
  std::vector<double4> hq(K);
  for (int k = 0; k < K; ++k) {
    hc[k] = make_float4(0.001f * k, 1e-9f, 0.5f, -1.0f);
    hq[k] = make_double4(0.001 * k, 0.7, 1.0 / K, 0.0);
  }
  std::vector<float> hx(nthr * R);
  std::vector<double> hxd(nthr * R);
  for (size_t i = 0; i < hx.size(); ++i) { hx[i] = (float)((i * 2654435761u) % 10000) * 1e-3f; hxd[i] = hx[i]; }
  float4* dc; double4* dq; float* dx; float* dout; double* dxd; double* doutd;
  CHECK(hipMalloc(&dc, K * sizeof(float4)));
  CHECK(hipMalloc(&dq, K * sizeof(double4)));
  CHECK(hipMalloc(&dx, hx.size() * sizeof(float)));
  CHECK(hipMalloc(&dxd, hxd.size() * sizeof(double)));
  CHECK(hipMalloc(&dout, 2 * nthr * sizeof(float)));  // R4 variant runs 2x the threads
  CHECK(hipMalloc(&doutd, nthr * sizeof(double)));
  CHECK(hipMemcpy(dc, hc.data(), K * sizeof(float4), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dq, hq.data(), K * sizeof(double4), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dx, hx.data(), hx.size() * sizeof(float), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dxd, hxd.data(), hxd.size() * sizeof(double), hipMemcpyHostToDevice));

  const double ce = (double)nthr * R * K;
  double ms;
  ms = time_ms([&] { ce_kernel<0, R><<<blocks, threads>>>(dc, K, dx, dout); }, 10);
  printf("{\"variant\":\"full_ce_f32\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
  ms = time_ms([&] { ce_kernel<3, R><<<blocks, threads>>>(dc, K, dx, dout); }, 10);
  printf("{\"variant\":\"full_ce_f32_unroll8\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
  ms = time_ms([&] { ce_kernel<1, R><<<blocks, threads>>>(dc, K, dx, dout); }, 10);
  printf("{\"variant\":\"valu_only_f32\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
  ms = time_ms([&] { ce_kernel<2, R><<<blocks, threads>>>(dc, K, dx, dout); }, 10);
  printf("{\"variant\":\"exp_add_only_f32\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
  ms = time_ms([&] { ce_kernel_pk<R / 2><<<blocks, threads>>>(dc, K, dx, dout); }, 10);
  printf("{\"variant\":\"full_ce_pk_f32\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
  for (int rr = 0; rr < 1; ++rr) {
    ms = time_ms([&] { ce_kernel<0, 4><<<blocks * 2, threads>>>(dc, K, dx, dout); }, 10);
    printf("{\"variant\":\"full_ce_f32_R4\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
    ms = time_ms([&] { ce_kernel<0, 16><<<blocks / 2, threads>>>(dc, K, dx, dout); }, 10);
    printf("{\"variant\":\"full_ce_f32_R16\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
  }
  for (int rep = 0; rep < 2; ++rep) {
    ms = time_ms([&] { ce_kernel_mix<R / 2, 0><<<blocks, threads>>>(dc, K, dx, dout); }, 10);
    printf("{\"variant\":\"mix_all_vexp_pk\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
    ms = time_ms([&] { ce_kernel_mix<R / 2, 1><<<blocks, threads>>>(dc, K, dx, dout); }, 10);
    printf("{\"variant\":\"mix_all_poly_pk\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
    ms = time_ms([&] { ce_kernel_mix<R / 2, 2><<<blocks, threads>>>(dc, K, dx, dout); }, 10);
    printf("{\"variant\":\"mix_1of4_poly_pk\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
    ms = time_ms([&] { ce_kernel_mix<R / 2, 3><<<blocks, threads>>>(dc, K, dx, dout); }, 10);
    printf("{\"variant\":\"mix_2of4_poly_pk\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, ce / (ms * 1e-3));
  }
  const int Kq = 512;
  ms = time_ms([&] { qce_kernel<4><<<blocks, threads>>>(dq, Kq, dxd, doutd); }, 5);
  printf("{\"variant\":\"quant_ce_f64\",\"ms\":%.4f,\"ce_per_s\":%.4e}\n", ms, (double)nthr * 4 * Kq / (ms * 1e-3));
  CHECK(hipDeviceSynchronize());
  return 0;
}
