// The evidential head's epilogue (evidential/models.py:385-459, ELFNet-style NIG mixture) on
// gfx950: for each of the three classifier outputs (classif0/1/2, [1][4][D][H][W]: cost, log nu,
// log alpha, log beta per plane, already at the head's full [maxdisp, H, W] resolution, so the
// align_corners=True trilinear "upsample" of get_pred / get_logits (:418-430) is the identity)
//   prob_i  = softmax_D(cost_i)                                   (get_pred, :421)
//   pred_i  = sum_d prob_i[d] depth_values[d]                     (disparity_regression, :40-45)
//   la_i, alpha_i, beta_i = softplus(sum_d prob_i[d] logit_i[d]) (+1 for alpha)
//                                                                 (get_logits :426-430, :281-285)
// then the mixture moe_nig(moe_nig(e0, e1), e2)                   (:287-304)
// and prob_combine = mean_i prob_i                               (:457-458).
// One thread per pixel; every load and store of a (head, channel, plane) is one coalesced
// row of the [D][H*W] plane: the kernel is a single streaming pass (HBM-bound: 3 x 4 x D floats
// in, 4 + D floats out per pixel), all the per-pixel state in registers.
//
// The backward (for train.py's loss_der through the head, :517-558) recomputes the forward of
// its pixel and differentiates it in closed form, in the order autograd applies the chain rule
// to the reference's expressions; dL/d the three classifier outputs, no gradient to the depths.
#include <hip/hip_runtime.h>

#include "aarmvs_internal.h"

namespace aarmvs {

constexpr int kEvD = 32;   // maxdisp (evidential/models.py:245): the reference's only working D

__device__ __forceinline__ float ev_softplus(float x) {   // F.softplus(beta=1, threshold=20)
  return x > 20.0f ? x : log1pf(expf(x));
}
__device__ __forceinline__ float ev_softplus_grad(float x) {   // d softplus / dx
  if (x > 20.0f) return 1.0f;
  const float z = expf(x);
  return z / (z + 1.0f);
}

struct NigEst {
  float u, la, al, be;
};

// moe_nig (evidential/models.py:287-296)
__device__ __forceinline__ NigEst moe_nig(const NigEst& a, const NigEst& b) {
  NigEst r;
  r.la = a.la + b.la;
  r.u = (a.la * a.u + b.u * b.la) / r.la;
  r.al = a.al + b.al + 0.5f;
  const float d1 = a.u - r.u, d2 = b.u - r.u;
  r.be = a.be + b.be + 0.5f * (a.la * (d1 * d1) + b.la * (d2 * d2));
  return r;
}

// backward of moe_nig: g (dL/d the result) -> ga, gb (dL/d the two inputs, overwritten)
__device__ __forceinline__ void moe_nig_bwd(const NigEst& a, const NigEst& b, const NigEst& g,
                                            NigEst& ga, NigEst& gb) {
  const float la = a.la + b.la;
  const float n = a.la * a.u + b.u * b.la;
  const float u = n / la;
  const float d1 = a.u - u, d2 = b.u - u;
  const float gq = 0.5f * g.be;
  ga.al = g.al;
  gb.al = g.al;
  ga.be = g.be;
  gb.be = g.be;
  const float gd1 = gq * (a.la * (2.0f * d1)), gd2 = gq * (b.la * (2.0f * d2));
  ga.u = gd1;
  gb.u = gd2;
  ga.la = gq * (d1 * d1);
  gb.la = gq * (d2 * d2);
  const float gu = g.u - gd1 - gd2;   // u also enters through d1, d2
  const float gn = gu / la;
  const float gla = g.la - gu * n / (la * la);
  ga.la += gla + gn * a.u;
  gb.la += gla + gn * b.u;
  ga.u += gn * a.la;
  gb.u += gn * b.la;
}

struct EvArgs {
  const float* head[3];   // [4][D][HW] each
  const float* dv;        // [D]
  int HW;
  float* ev;              // [4][HW]
  float* pc;              // [D][HW]
  const float* g_ev;      // backward: [4][HW] or null
  const float* g_pc;      // backward: [D][HW] or null
  float* g_head[3];       // backward: [4][D][HW] each
};

// softmax over D of one head's cost channel at pixel p (max-subtracted, as F.softmax)
__device__ __forceinline__ void ev_softmax(const float* __restrict__ c, int HW, int p, float (&pr)[kEvD]) {
  float m = -INFINITY;
#pragma unroll
  for (int d = 0; d < kEvD; ++d) {
    pr[d] = c[(size_t)d * HW + p];
    m = fmaxf(m, pr[d]);
  }
  float s = 0.0f;
#pragma unroll
  for (int d = 0; d < kEvD; ++d) {
    pr[d] = expf(pr[d] - m);
    s += pr[d];
  }
  const float inv = 1.0f / s;
#pragma unroll
  for (int d = 0; d < kEvD; ++d) pr[d] *= inv;
}

// one head's estimate (pred, la, alpha, beta) and the three pre-softplus logits
__device__ __forceinline__ NigEst ev_head(const float* __restrict__ h, const float* __restrict__ dv,
                                          int HW, int p, const float (&pr)[kEvD], float (&lg)[3]) {
  const size_t cs = (size_t)kEvD * HW;
  float pred = 0.0f, l0 = 0.0f, l1 = 0.0f, l2 = 0.0f;
#pragma unroll
  for (int d = 0; d < kEvD; ++d) {
    const size_t o = (size_t)d * HW + p;
    pred += pr[d] * dv[d];
    l0 += h[cs + o] * pr[d];
    l1 += h[2 * cs + o] * pr[d];
    l2 += h[3 * cs + o] * pr[d];
  }
  lg[0] = l0;
  lg[1] = l1;
  lg[2] = l2;
  return NigEst{pred, ev_softplus(l0), ev_softplus(l1) + 1.0f, ev_softplus(l2)};
}

__global__ void __launch_bounds__(256) evidential_fwd_kernel(EvArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.HW) return;
  float pc[kEvD];
#pragma unroll
  for (int d = 0; d < kEvD; ++d) pc[d] = 0.0f;
  NigEst e[3];
#pragma unroll 1
  for (int i = 0; i < 3; ++i) {
    float pr[kEvD], lg[3];
    ev_softmax(a.head[i], a.HW, p, pr);
    e[i] = ev_head(a.head[i], a.dv, a.HW, p, pr, lg);
#pragma unroll
    for (int d = 0; d < kEvD; ++d) pc[d] += pr[d];
  }
  const NigEst r = moe_nig(moe_nig(e[0], e[1]), e[2]);
  a.ev[p] = r.u;
  a.ev[a.HW + p] = r.la;
  a.ev[2 * a.HW + p] = r.al;
  a.ev[3 * a.HW + p] = r.be;
#pragma unroll
  for (int d = 0; d < kEvD; ++d) a.pc[(size_t)d * a.HW + p] = pc[d] / 3.0f;
}

__global__ void __launch_bounds__(256) evidential_bwd_kernel(EvArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.HW) return;
  const int HW = a.HW;
  // forward of the pixel: the three estimates and their logits
  NigEst e[3];
  float lg[3][3];
#pragma unroll 1
  for (int i = 0; i < 3; ++i) {
    float pr[kEvD];
    ev_softmax(a.head[i], HW, p, pr);
    e[i] = ev_head(a.head[i], a.dv, HW, p, pr, lg[i]);
  }
  const NigEst e01 = moe_nig(e[0], e[1]);
  NigEst g{0.0f, 0.0f, 0.0f, 0.0f};
  if (a.g_ev) g = NigEst{a.g_ev[p], a.g_ev[HW + p], a.g_ev[2 * HW + p], a.g_ev[3 * HW + p]};
  NigEst g01, g2, g0, g1;
  moe_nig_bwd(e01, e[2], g, g01, g2);
  moe_nig_bwd(e[0], e[1], g01, g0, g1);
  const NigEst ge[3] = {g0, g1, g2};
  const size_t cs = (size_t)kEvD * HW;
#pragma unroll 1
  for (int i = 0; i < 3; ++i) {
    const float* __restrict__ h = a.head[i];
    float* __restrict__ gh = a.g_head[i];
    float pr[kEvD];
    ev_softmax(h, HW, p, pr);
    // dL/d the logits through softplus; dL/d pred through disparity_regression
    const float gl0 = ge[i].la * ev_softplus_grad(lg[i][0]);
    const float gl1 = ge[i].al * ev_softplus_grad(lg[i][1]);
    const float gl2 = ge[i].be * ev_softplus_grad(lg[i][2]);
    const float gpred = ge[i].u;
    float gp[kEvD];
    float dot = 0.0f;
#pragma unroll
    for (int d = 0; d < kEvD; ++d) {
      const size_t o = (size_t)d * HW + p;
      const float v0 = h[cs + o], v1 = h[2 * cs + o], v2 = h[3 * cs + o];
      gh[cs + o] = gl0 * pr[d];
      gh[2 * cs + o] = gl1 * pr[d];
      gh[3 * cs + o] = gl2 * pr[d];
      float q = gpred * a.dv[d] + gl0 * v0 + gl1 * v1 + gl2 * v2;
      if (a.g_pc) q += a.g_pc[o] / 3.0f;
      gp[d] = q;
      dot += pr[d] * q;
    }
#pragma unroll
    for (int d = 0; d < kEvD; ++d) gh[(size_t)d * HW + p] = pr[d] * (gp[d] - dot);   // softmax backward
  }
}

hipError_t launch_evidential(const float* const head[3], const float* dv, int D, int HW, float* ev,
                             float* pc, const float* g_ev, const float* g_pc, float* const g_head[3],
                             hipStream_t s) {
  if (D != kEvD) return hipErrorInvalidValue;
  EvArgs a{};
  for (int i = 0; i < 3; ++i) {
    a.head[i] = head[i];
    a.g_head[i] = g_head ? g_head[i] : nullptr;
  }
  a.dv = dv;
  a.HW = HW;
  a.ev = ev;
  a.pc = pc;
  a.g_ev = g_ev;
  a.g_pc = g_pc;
  const int blocks = (HW + 255) / 256;
  ProfScope ps(s, K_EVIDENTIAL);
  if (g_head)
    hipLaunchKernelGGL(evidential_bwd_kernel, dim3(blocks), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(evidential_fwd_kernel, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace aarmvs
