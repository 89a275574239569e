// The sampling half of FeatNet's modulated deformable convolution (models/module.py:105-236 of
// the reference, DeformConv2d.forward) on gfx950, forward and backward; the contraction with the
// conv weights is a plain GEMM left to hipBLASLt by the caller (aarmvs.ops.deform_conv2d).
//
// For output pixel (i, j) and kernel tap n = 3 a' + b' (a = a' - 1, b = b' - 1) the sampling
// point in the zero-padded input is
//   pr = (i s + 1 + a) + offset[n],  pc = (j s + 1 + b) + offset[9 + n]   (p_0 + p_n + offset)
// r0 = floor(pr), c0 = floor(pc) (no gradient), the corner rows / columns clamped to the padded
// image, pr / pc clamped likewise, and
//   val[c] = m[n] (g_lt x[r0c, c0c] + g_rb x[r1c, c1c] + g_lb x[r0c, c1c] + g_rt x[r1c, c0c])
// with g_lt = (1 + (r0c - pr)) (1 + (c0c - pc)), g_rb = (1 - (r1c - pr)) (1 - (c1c - pc)),
// g_lb = (1 + (r0c - pr)) (1 - (c1c - pc)), g_rt = (1 - (r1c - pr)) (1 + (c0c - pc)); a padded
// position outside the image reads 0.  Every operation is one IEEE fp32 rounding in the
// reference's order (the file is compiled without contraction), so val equals the PyTorch
// expression of models.module.DeformConv2d bit for bit.
//
// Layout: x is NHWC [B][H][W][C] (a corner's C channels are one 128-byte row), val is
// [B][h w][9][C] (the GEMM's A operand, row = pixel).  One half-wave per (pixel, tap), lane =
// channel: every corner read, val write and dL/dx atomic is one contiguous 128-byte row.  The
// backward recomputes the corners and writes dL/dx (atomically, into an NHWC buffer the caller
// zeroes), dL/d offset and dL/d m (32-lane shuffle sums).
#include <hip/hip_runtime.h>

#include "aarmvs_internal.h"

namespace aarmvs {

constexpr int kDfC = 32;   // channels (FeatNet's deformable convs are 32 -> 32)
constexpr int kDfTaps = 9;


struct DfPos {
  float prc, pcc;              // clamped sampling point
  float r0c, r1c, c0c, c1c;    // clamped corner rows / columns
  bool rin, cin;               // pr / pc inside the clamp range (their gradient passes)
  int ro[2], co[2];            // image row / column of the corner rows / columns, -1 outside
};

__device__ __forceinline__ DfPos df_pos(const DfArgs& a, int b, int i, int j, int n) {
  const int hw = a.h * a.w, px = i * a.w + j;
  const float* o = a.off + (size_t)b * 2 * kDfTaps * hw + px;
  const float Hp1 = (float)(a.H + 2 * a.pad - 1), Wp1 = (float)(a.W + 2 * a.pad - 1);
  const float pr = __fadd_rn((float)(i * a.stride + 1 + n / 3 - 1), o[(size_t)n * hw]);
  const float pc = __fadd_rn((float)(j * a.stride + 1 + n % 3 - 1), o[(size_t)(kDfTaps + n) * hw]);
  const float r0 = floorf(pr), c0 = floorf(pc);
  DfPos p;
  p.r0c = fminf(fmaxf(r0, 0.0f), Hp1);
  p.r1c = fminf(fmaxf(__fadd_rn(r0, 1.0f), 0.0f), Hp1);
  p.c0c = fminf(fmaxf(c0, 0.0f), Wp1);
  p.c1c = fminf(fmaxf(__fadd_rn(c0, 1.0f), 0.0f), Wp1);
  p.prc = fminf(fmaxf(pr, 0.0f), Hp1);
  p.pcc = fminf(fmaxf(pc, 0.0f), Wp1);
  p.rin = pr >= 0.0f && pr <= Hp1;
  p.cin = pc >= 0.0f && pc <= Wp1;
  const float rr[2] = {p.r0c, p.r1c}, cc[2] = {p.c0c, p.c1c};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int r = (int)rr[k] - a.pad, c = (int)cc[k] - a.pad;
    p.ro[k] = r >= 0 && r < a.H ? r : -1;
    p.co[k] = c >= 0 && c < a.W ? c : -1;
  }
  return p;
}

// the four corner factors: g_lt, g_rb, g_lb, g_rt (module.py's order)
struct DfFac {
  float ar0, ar1, ac0, ac1;    // 1 + (r0c - pr), 1 - (r1c - pr), 1 + (c0c - pc), 1 - (c1c - pc)
  float g[4];
};
__device__ __forceinline__ DfFac df_fac(const DfPos& p) {
  DfFac f;
  f.ar0 = __fadd_rn(1.0f, __fsub_rn(p.r0c, p.prc));
  f.ar1 = __fsub_rn(1.0f, __fsub_rn(p.r1c, p.prc));
  f.ac0 = __fadd_rn(1.0f, __fsub_rn(p.c0c, p.pcc));
  f.ac1 = __fsub_rn(1.0f, __fsub_rn(p.c1c, p.pcc));
  f.g[0] = __fmul_rn(f.ar0, f.ac0);
  f.g[1] = __fmul_rn(f.ar1, f.ac1);
  f.g[2] = __fmul_rn(f.ar0, f.ac1);
  f.g[3] = __fmul_rn(f.ar1, f.ac0);
  return f;
}

// corner k (lt, rb, lb, rt) -> (row index, column index) into DfPos::ro / co
__device__ __forceinline__ int df_kr(int k) { return (k == 1 || k == 3) ? 1 : 0; }
__device__ __forceinline__ int df_kc(int k) { return (k == 1 || k == 2) ? 1 : 0; }

__device__ __forceinline__ float df_sum32(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
  return v;
}

template <bool BWD>
__global__ void __launch_bounds__(256) deform_sample_kernel(DfArgs a) {
  const int lane = threadIdx.x & 31;
  const long long item = (long long)blockIdx.x * 8 + (threadIdx.x >> 5);   // (b, pixel, tap)
  const int hw = a.h * a.w;
  if (item >= (long long)a.B * hw * kDfTaps) return;   // whole half-waves
  const int n = (int)(item % kDfTaps);
  const long long bp = item / kDfTaps;
  const int px = (int)(bp % hw), b = (int)(bp / hw);
  const int i = px / a.w, j = px - i * a.w;
  const DfPos p = df_pos(a, b, i, j, n);
  const DfFac f = df_fac(p);
  const float* xb = a.x + (size_t)b * a.H * a.W * kDfC;
  float t[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = p.ro[df_kr(k)], c = p.co[df_kc(k)];
    t[k] = (r >= 0 && c >= 0) ? xb[((size_t)r * a.W + c) * kDfC + lane] : 0.0f;
  }
  const float vu = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(f.g[0], t[0]), __fmul_rn(f.g[1], t[1])),
                                       __fmul_rn(f.g[2], t[2])),
                             __fmul_rn(f.g[3], t[3]));
  const size_t mi = ((size_t)b * kDfTaps + n) * hw + px;
  const float m = a.m ? a.m[mi] : 1.0f;
  if constexpr (!BWD) {
    a.val[(size_t)item * kDfC + lane] = a.m ? __fmul_rn(vu, m) : vu;
  } else {
    const float gv = a.gval[(size_t)item * kDfC + lane];
    const float gu = a.m ? __fmul_rn(gv, m) : gv;   // dL/d (unmodulated val)
    // dL/dx: the four corners (coinciding clamped corners each add their own share)
    float* gxb = a.gx + (size_t)b * a.H * a.W * kDfC;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = p.ro[df_kr(k)], c = p.co[df_kc(k)];
      if (r >= 0 && c >= 0) unsafeAtomicAdd(gxb + ((size_t)r * a.W + c) * kDfC + lane, gu * f.g[k]);
    }
    // dL/d g_k = sum_c gu t_k; g_lt = ar0 ac0, g_rb = ar1 ac1, g_lb = ar0 ac1, g_rt = ar1 ac0 with
    // d ar0 / d pr = -1, d ar1 / d pr = +1, d ac0 / d pc = -1, d ac1 / d pc = +1
    const float dpr = gu * (-(f.ac0 * t[0]) + f.ac1 * t[1] - f.ac1 * t[2] + f.ac0 * t[3]);
    const float dpc = gu * (-(f.ar0 * t[0]) + f.ar1 * t[1] + f.ar0 * t[2] - f.ar1 * t[3]);
    const float sr = df_sum32(dpr), sc = df_sum32(dpc);
    const float sm = a.gm ? df_sum32(gv * vu) : 0.0f;
    if (lane == 0) {
      const size_t oi = ((size_t)b * 2 * kDfTaps + n) * hw + px;
      a.goff[oi] = p.rin ? sr : 0.0f;
      a.goff[oi + (size_t)kDfTaps * hw] = p.cin ? sc : 0.0f;
      if (a.gm) a.gm[mi] = sm;
    }
  }
}

hipError_t launch_deform_sample(const DfArgs& a, bool bwd, hipStream_t s) {
  ProfScope ps(s, K_DEFORM);
  const long long items = (long long)a.B * a.h * a.w * kDfTaps;
  const long long blocks = (items + 7) / 8;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  if (bwd)
    hipLaunchKernelGGL(deform_sample_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(deform_sample_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace aarmvs
