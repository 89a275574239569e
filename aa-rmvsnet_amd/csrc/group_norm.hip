// GroupNorm forward and backward for the PyTorch-side modules (FeatNet, and the BPTT
// recompute of the omega chain and the U-Net deconvs: module.py:98-103, 245-287 via
// models.module.GroupNorm) on gfx950.
//
// x is NCHW fp32, [B][C][HW], G groups of C/G channels.  Every statistic is a fixed-order
// reduction: per (b, c) channel plane, blocks of kGnThreads threads take fixed HW ranges
// and accumulate in fp64, their partials are summed by one block per (b, g) in a fixed tree,
// so results are bit-reproducible run to run.  ATen's ROCm group_norm reduces a whole
// (b, g) row in one thread block (one busy CU per group at B = 1).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "aarmvs_internal.h"
#include "device_common.h"

namespace aarmvs {

constexpr int kGnThreads = 256;
constexpr int kGnPerThread = 16;   // elements per thread per partial block
constexpr int kGnSpan = kGnThreads * kGnPerThread;

// blocks per channel plane
static inline int gn_nb(int HW) { return (HW + kGnSpan - 1) / kGnSpan; }

template <int NV>
__device__ __forceinline__ void block_sum_d(double (&v)[NV], double (*red)[kGnThreads]) {
#pragma unroll
  for (int i = 0; i < NV; ++i) red[i][threadIdx.x] = v[i];
  __syncthreads();
  for (int o = kGnThreads / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
#pragma unroll
      for (int i = 0; i < NV; ++i) red[i][threadIdx.x] += red[i][threadIdx.x + o];
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = red[i][0];
}

// forward partials: (sum x, sum x^2) of one HW range of channel plane (b, c)
__global__ void __launch_bounds__(kGnThreads) gn_fwd_partial_kernel(const float* __restrict__ x,
                                                                    int C, int HW,
                                                                    double* __restrict__ part) {
  __shared__ double red[2][kGnThreads];
  const int blk = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
  const float* xp = x + ((size_t)b * C + c) * HW;
  double v[2] = {0.0, 0.0};
  const int i0 = blk * kGnSpan + threadIdx.x;
#pragma unroll 4
  for (int k = 0; k < kGnPerThread; ++k) {
    const int i = i0 + k * kGnThreads;
    if (i < HW) {
      const double t = xp[i];
      v[0] += t;
      v[1] += t * t;
    }
  }
  block_sum_d<2>(v, red);
  if (threadIdx.x == 0) {
    double* pp = part + 2 * (((size_t)b * C + c) * gridDim.x + blk);
    pp[0] = v[0];
    pp[1] = v[1];
  }
}

// per (b, g): mean and rstd from the group's partials (channels in order, blocks in order)
__global__ void __launch_bounds__(kGnThreads) gn_fwd_stats_kernel(const double* __restrict__ part,
                                                                  int C, int HW, int G, int nb,
                                                                  float eps,
                                                                  float* __restrict__ mean_rstd) {
  __shared__ double red[2][kGnThreads];
  const int g = blockIdx.x, b = blockIdx.y, cg = C / G;
  const double* pp = part + 2 * (((size_t)b * C + (size_t)g * cg) * nb);
  const int n = cg * nb;
  double v[2] = {0.0, 0.0};
  for (int i = threadIdx.x; i < n; i += kGnThreads) {
    v[0] += pp[2 * i];
    v[1] += pp[2 * i + 1];
  }
  block_sum_d<2>(v, red);
  if (threadIdx.x == 0) {
    const double cnt = (double)cg * HW;
    const double mean = v[0] / cnt;
    double var = v[1] / cnt - mean * mean;
    var = var < 0.0 ? 0.0 : var;
    mean_rstd[2 * (b * G + g)] = (float)mean;
    mean_rstd[2 * (b * G + g) + 1] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

// y = x * a + (beta - mean * a), a = rstd * gamma (ATen's form)
__global__ void __launch_bounds__(kGnThreads) gn_fwd_apply_kernel(
    const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean_rstd, int C, int HW, int G, float* __restrict__ y) {
  const int c = blockIdx.y, b = blockIdx.z, g = c / (C / G);
  const float mean = mean_rstd[2 * (b * G + g)], rstd = mean_rstd[2 * (b * G + g) + 1];
  const float a = gamma ? rstd * gamma[c] : rstd;
  const float sh = (beta ? beta[c] : 0.0f) - mean * a;
  const size_t base = ((size_t)b * C + c) * HW;
  for (int i = blockIdx.x * kGnThreads + threadIdx.x; i < HW; i += gridDim.x * kGnThreads)
    y[base + i] = fmaf(x[base + i], a, sh);
}

// backward partials of channel plane (b, c): (sum dy * xhat, sum dy)
__global__ void __launch_bounds__(kGnThreads) gn_bwd_partial_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ mean_rstd,
    int C, int HW, int G, double* __restrict__ part) {
  __shared__ double red[2][kGnThreads];
  const int blk = blockIdx.x, c = blockIdx.y, b = blockIdx.z, g = c / (C / G);
  const float mean = mean_rstd[2 * (b * G + g)], rstd = mean_rstd[2 * (b * G + g) + 1];
  const size_t base = ((size_t)b * C + c) * HW;
  double v[2] = {0.0, 0.0};
  const int i0 = blk * kGnSpan + threadIdx.x;
#pragma unroll 4
  for (int k = 0; k < kGnPerThread; ++k) {
    const int i = i0 + k * kGnThreads;
    if (i < HW) {
      const double d = dy[base + i];
      v[0] += d * (double)((x[base + i] - mean) * rstd);
      v[1] += d;
    }
  }
  block_sum_d<2>(v, red);
  if (threadIdx.x == 0) {
    double* pp = part + 2 * (((size_t)b * C + c) * gridDim.x + blk);
    pp[0] = v[0];
    pp[1] = v[1];
  }
}

// per (b, c): s1 = sum dy * xhat, s2 = sum dy (the dgamma / dbeta terms of sample b); per
// (b, g): the two group means of the input gradient, (sum gamma_c s2) / n and
// (sum gamma_c s1) / n, into coef.  One block per (b, g), channels in order.
__global__ void __launch_bounds__(kGnThreads) gn_bwd_stats_kernel(
    const double* __restrict__ part, const float* __restrict__ gamma, int C, int HW, int G, int nb,
    float* __restrict__ s1, float* __restrict__ s2, float* __restrict__ coef) {
  __shared__ double red[2][kGnThreads];
  const int g = blockIdx.x, b = blockIdx.y, cg = C / G;
  double gs[2] = {0.0, 0.0};
  for (int cc = 0; cc < cg; ++cc) {
    const int c = g * cg + cc;
    const double* pp = part + 2 * (((size_t)b * C + c) * nb);
    double v[2] = {0.0, 0.0};
    for (int i = threadIdx.x; i < nb; i += kGnThreads) {
      v[0] += pp[2 * i];
      v[1] += pp[2 * i + 1];
    }
    block_sum_d<2>(v, red);
    __syncthreads();   // red is reused by the next channel
    if (threadIdx.x == 0) {
      s1[b * C + c] = (float)v[0];
      s2[b * C + c] = (float)v[1];
    }
    const double gm = gamma ? (double)gamma[c] : 1.0;
    gs[0] += gm * v[1];   // sum dyhat
    gs[1] += gm * v[0];   // sum dyhat * xhat
  }
  if (threadIdx.x == 0) {
    const double cnt = (double)cg * HW;
    coef[2 * (b * G + g)] = (float)(gs[0] / cnt);
    coef[2 * (b * G + g) + 1] = (float)(gs[1] / cnt);
  }
}

// dx = rstd (gamma dy - mean(dyhat) - xhat mean(dyhat xhat))
__global__ void __launch_bounds__(kGnThreads) gn_bwd_apply_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ mean_rstd, const float* __restrict__ coef, int C, int HW, int G,
    float* __restrict__ dx) {
  const int c = blockIdx.y, b = blockIdx.z, g = c / (C / G);
  const float mean = mean_rstd[2 * (b * G + g)], rstd = mean_rstd[2 * (b * G + g) + 1];
  const float m1 = coef[2 * (b * G + g)], m2 = coef[2 * (b * G + g) + 1];
  const float gm = gamma ? gamma[c] : 1.0f;
  const size_t base = ((size_t)b * C + c) * HW;
  for (int i = blockIdx.x * kGnThreads + threadIdx.x; i < HW; i += gridDim.x * kGnThreads) {
    const float xh = (x[base + i] - mean) * rstd;
    dx[base + i] = rstd * (gm * dy[base + i] - m1 - xh * m2);
  }
}

static inline unsigned gn_apply_blocks(int HW) {
  return (unsigned)std::max(1, std::min((HW + kGnThreads - 1) / kGnThreads, 64));
}

size_t gn_scratch_bytes(int B, int C, int HW) {
  return (size_t)B * C * gn_nb(HW) * 2 * sizeof(double) + (size_t)B * C * 2 * sizeof(float);
}

hipError_t launch_group_norm_fwd(const float* x, const float* gamma, const float* beta, int B,
                                 int C, int HW, int G, float eps, float* y, float* mean_rstd,
                                 void* scratch, hipStream_t s) {
  const int nb = gn_nb(HW);
  double* part = static_cast<double*>(scratch);
  hipLaunchKernelGGL(gn_fwd_partial_kernel, dim3(nb, C, B), dim3(kGnThreads), 0, s, x, C, HW, part);
  hipError_t e;
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(gn_fwd_stats_kernel, dim3(G, B), dim3(kGnThreads), 0, s, part, C, HW, G, nb,
                     eps, mean_rstd);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(gn_fwd_apply_kernel, dim3(gn_apply_blocks(HW), C, B), dim3(kGnThreads), 0, s,
                     x, gamma, beta, mean_rstd, C, HW, G, y);
  return hipGetLastError();
}

hipError_t launch_group_norm_bwd(const float* dy, const float* x, const float* gamma,
                                 const float* mean_rstd, int B, int C, int HW, int G, float* dx,
                                 float* s1, float* s2, void* scratch, hipStream_t s) {
  const int nb = gn_nb(HW);
  double* part = static_cast<double*>(scratch);
  float* coef = reinterpret_cast<float*>(part + (size_t)B * C * nb * 2);
  hipLaunchKernelGGL(gn_bwd_partial_kernel, dim3(nb, C, B), dim3(kGnThreads), 0, s, dy, x,
                     mean_rstd, C, HW, G, part);
  hipError_t e;
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(gn_bwd_stats_kernel, dim3(G, B), dim3(kGnThreads), 0, s, part, gamma, C, HW,
                     G, nb, s1, s2, coef);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(gn_bwd_apply_kernel, dim3(gn_apply_blocks(HW), C, B), dim3(kGnThreads), 0, s,
                     dy, x, gamma, mean_rstd, coef, C, HW, G, dx);
  return hipGetLastError();
}

}  // namespace aarmvs
