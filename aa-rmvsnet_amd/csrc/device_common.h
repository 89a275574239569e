// Device-side helpers shared by the kernels: wave/block reductions, GroupNorm
// statistics in fp64 atomic slots, activation functions.
#pragma once

#include <hip/hip_runtime.h>

#include "aarmvs_internal.h"

namespace aarmvs {

// Buffer-descriptor loads for the streaming kernels: 32-bit byte offsets instead of
// 64-bit addresses (VGPR pressure), and the hardware range check does the zero padding:
// an offset at or past num_records loads 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const float* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
  void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)n, 0x00020000);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float4 ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}
__device__ __forceinline__ float2 ld2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
}
__device__ __forceinline__ float ld1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Gate activations of the LSTM epilogue on the hardware exp / rcp (v_exp_f32, v_rcp_f32).
// Fast forms (the inference sweep): rcp(1 + exp(-x)) and 1 - 2 rcp(exp(2x) + 1), ~1 ulp but
// biased: +0.30 ulp and, for |tanh| arguments below 0.5, -0.84 ulp on average
// (tools/microbench/gate_fn_bias.cpp) -- harmless for the depth maps, not for the BPTT, whose
// 192-plane recurrence and long cancelling parameter-gradient sums turn a drift into errors
// well above float32's.  Unbiased forms (the training sweep, PRECISE cells):
//   exp_u: v_exp_f32 of x log2e with the rounding error of the fp32 constant log2e corrected
//          (it made __expf's error grow as -1.3e-8 |x| relative: the sigmoid's +0.3 ulp);
//   rcp_nr: one Newton step on the reciprocal (the division to ~0.5 ulp);
//   tanh: for |x| < 0.625 the odd minimax polynomial x + x^3 P(x^2) (no cancellation).
__device__ __forceinline__ float fast_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float fast_tanh(float x) {
  // tanh(x) = 1 - 2 / (exp(2x) + 1); saturates cleanly for large |x| (exp -> inf / 0)
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * x) + 1.0f);
}
__device__ __forceinline__ float exp_u(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 1.44269502f);
  const float c = fmaf(e, x * 1.3349758e-8f, e);   // x (log2e - fp32(log2e)) ln 2
  // no correction at e = 0, inf or NaN (x = -inf would give fmaf(0, -inf, 0) = NaN)
  return (e > 0.0f && e < INFINITY) ? c : e;
}
__device__ __forceinline__ float rcp_nr(float d) {   // 1 / d for d >= 1 (d = inf -> 0, NaN -> NaN)
  const float r = __builtin_amdgcn_rcpf(d);
  return d < INFINITY ? fmaf(fmaf(-d, r, 1.0f), r, r) : (d != d ? d : 0.0f);
}
__device__ __forceinline__ float precise_sigmoid(float x) { return rcp_nr(1.0f + exp_u(-x)); }
__device__ __forceinline__ float precise_tanh(float x) {
  const float ax = fabsf(x), z = x * x;
  const float p = fmaf(fmaf(fmaf(fmaf(-5.70498872745e-3f, z, 2.06390887954e-2f), z, -5.37397155531e-2f), z,
                            1.33314422036e-1f), z, -3.33332819422e-1f);
  const float small = fmaf(p * z, x, x);
  const float big = copysignf(1.0f - 2.0f * rcp_nr(exp_u(2.0f * ax) + 1.0f), x);
  return ax < 0.625f ? small : big;
}

// Wave-wide reductions on DPP (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror,
// row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3): plain VALU operations,
// no LDS round trips (a __shfl_xor butterfly is six dependent ds_bpermute_b32 per dword).
// The 64 lanes combine in a fixed order; the result is lane 63's, returned wave-uniform.
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_i32(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWS, 0xF, false);
}
template <class Op>
__device__ __forceinline__ int wave_reduce_i32(int v, int ident, Op op) {
  v = op(v, dpp_i32<0xB1, 0xF>(ident, v));
  v = op(v, dpp_i32<0x4E, 0xF>(ident, v));
  v = op(v, dpp_i32<0x141, 0xF>(ident, v));
  v = op(v, dpp_i32<0x140, 0xF>(ident, v));
  v = op(v, dpp_i32<0x142, 0xA>(ident, v));
  v = op(v, dpp_i32<0x143, 0xC>(ident, v));
  return __builtin_amdgcn_readlane(v, 63);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double v) {   // lanes not written read +0.0
  const long long b = __double_as_longlong(v);
  const int lo = dpp_i32<CTRL, ROWS>(0, (int)(b & 0xffffffffll));
  const int hi = dpp_i32<CTRL, ROWS>(0, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_f64<0xB1, 0xF>(v);
  v += dpp_f64<0x4E, 0xF>(v);
  v += dpp_f64<0x141, 0xF>(v);
  v += dpp_f64<0x140, 0xF>(v);
  v += dpp_f64<0x142, 0xA>(v);
  v += dpp_f64<0x143, 0xC>(v);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum of NV values per thread; result valid in thread 0.
// `red` is LDS scratch of at least NV * (blockDim.x / 64) floats.
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[i * nw + wid] = v[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float s = 0.f;
      for (int w = 0; w < nw; ++w) s += red[i * nw + w];
      v[i] = s;
    }
  }
  __syncthreads();
}

// block_sum in fp64 (parameter-gradient partials: long cancelling sums)
template <int NV>
__device__ __forceinline__ void block_sum_d(double (&v)[NV], double* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum_d(v[i]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[i * nw + wid] = v[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      double s = 0.0;
      for (int w = 0; w < nw; ++w) s += red[i * nw + w];
      v[i] = s;
    }
  }
  __syncthreads();
}

// block_sum_d whose block totals go straight to out[0 .. NV): thread i < NV sums value i over
// the waves (same order as block_sum_d, so the same bits), instead of one thread summing all
// NV values serially.
template <int NV>
__device__ __forceinline__ void block_sum_d_store(double (&v)[NV], double* red, double* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum_d(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[i * nw + wid] = v[i];
  }
  __syncthreads();
  if ((int)threadIdx.x < NV) {
    double s = 0.0;
    for (int w = 0; w < nw; ++w) s += red[threadIdx.x * nw + w];
    out[threadIdx.x] = s;
  }
}

// Bound on |relu(gamma_c xhat + beta_c)| over the 16 channels of a GroupNorm(2,16)+ReLU output
// (deConvGnReLU, module.py:286-287) with n values per group: |xhat| <= sqrt(n - 1) (Samuelson),
// 1% margin for the fp32 evaluation.  Uniform loads: every lane computes the same value.
__device__ __forceinline__ float gn_relu_bound(const float* gamma, const float* beta, double n) {
  const float s = 1.01f * (float)sqrt(n > 1.0 ? n - 1.0 : 0.0);
  float m = 0.0f;
#pragma unroll
  for (int c = 0; c < 16; ++c) m = fmaxf(m, fabsf(gamma[c]) * s + fabsf(beta[c]));
  return m;
}

// GroupNorm fused parameters from fp64 slot sums: y = x * a + b with
// a = rstd * gamma, b = beta - mean * a  (the ATen CPU group_norm form).
struct GnStat {
  float mean, rstd;
};
__device__ __forceinline__ GnStat gn_stat_from(double s, double ss, double n) {
  const double mean = s / n;
  double var = ss / n - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  GnStat r;
  r.mean = (float)mean;
  r.rstd = (float)(1.0 / sqrt(var + (double)kGnEps));
  return r;
}
__device__ __forceinline__ GnStat stat_read(const double* stat, double n) {
  // slots summed in index order; the loads are issued 16 slots at a time (two round trips)
  static_assert(kSlots % 16 == 0, "slot batches");
  const double2* p = reinterpret_cast<const double2*>(stat);
  double s = 0.0, ss = 0.0;
#pragma unroll
  for (int h = 0; h < kSlots; h += 16) {
    double2 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = p[h + i];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s += v[i].x;
      ss += v[i].y;
    }
  }
  return gn_stat_from(s, ss, n);
}

}  // namespace aarmvs
