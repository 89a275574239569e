// Homography warp, inter-view adaptive aggregation (omega) and the per-plane cost
// slice for gfx950.
//
// Reference: models/module.py:6-38 (homo_warping_depthwise),
//            models/drmvsnet.py:27-38 (InterViewAAModule), :307-319 (accumulation).
//
// Per plane and batch element the cost slice needs three grid-wide GroupNorm
// reductions per source view, so it is produced by four launches:
//   K1 cost_t1       warp + (warp-ref)^2 over a haloed tile in LDS, 3x3 conv 32->4
//                    (t1, 16 B/px/view) and GN#0 partial sums
//   K2 omega_stats<1> t1 -> a -> 1x1 conv -> GN#1 partial sums
//   K3 omega_stats<2> ...  -> 1x1 conv -> GN#2 partial sums
//   K4 cost_final    re-warp every view, w_v from t1 and the three GN stats,
//                    x = -(sum_v (1+w_v)(warp_v-ref)^2)/nsrc  -> [B,32,H,W]
// K1 and K4 stream the source features (HBM-bound); K2/K3 read only t1.
#include <hip/hip_runtime.h>

#include "device_common.h"

namespace aarmvs {

// ---------------------------------------------------------------------------
// Sampling position of reference pixel (x, y) in the source view, in source
// pixel units, following module.py:26-33 then grid_sample's align_corners=False
// unnormalisation.  The grid itself is built by separate torch ops in the
// reference (explicit _rn ops here: no contraction); grid_sample's CPU kernel is
// FMA-contracted by its compiler: ix = fma(g + 1, size/2, -0.5).  This pair of
// choices reproduces the reference's sampling positions bit for bit.
// ---------------------------------------------------------------------------
struct Proj12 {
  float r[12];
};

__device__ __forceinline__ void sample_pos(const float* __restrict__ m, float depth, float x,
                                           float y, int H, int W, float& ix, float& iy) {
  float p[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float rx = __fadd_rn(__fadd_rn(__fmul_rn(m[4 * k + 0], x), __fmul_rn(m[4 * k + 1], y)),
                               m[4 * k + 2]);                     // rot @ [x,y,1]   :26
    p[k] = __fadd_rn(__fmul_rn(rx, depth), m[4 * k + 3]);         // * depth + t     :27-28
  }
  float z = p[2];
  if (z == 0.0f) z = __fadd_rn(z, 1e-4f);                         // :29
  const float px = __fdiv_rn(p[0], z), py = __fdiv_rn(p[1], z);   // :30
  const float gx = __fsub_rn(__fdiv_rn(px, (float)(W - 1) * 0.5f), 1.0f);  // :31
  const float gy = __fsub_rn(__fdiv_rn(py, (float)(H - 1) * 0.5f), 1.0f);  // :32
  ix = __fmaf_rn(__fadd_rn(gx, 1.0f), (float)W * 0.5f, -0.5f);
  iy = __fmaf_rn(__fadd_rn(gy, 1.0f), (float)H * 0.5f, -0.5f);
}

// Bilinear taps with zero padding.  Invalid taps get index 0 and weight 0.
struct Taps {
  int idx[4];
  float wt[4];
  bool ok[4];
};

__device__ __forceinline__ Taps make_taps(float ix, float iy, int H, int W) {
  Taps t;
  const float x0 = floorf(ix), y0 = floorf(iy);
  const float wx = __fsub_rn(ix, x0), wy = __fsub_rn(iy, y0);
  const float ex = __fsub_rn(1.0f, wx), sy = __fsub_rn(1.0f, wy);
  const float wts[4] = {__fmul_rn(sy, ex), __fmul_rn(sy, wx), __fmul_rn(wy, ex), __fmul_rn(wy, wx)};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float xf = x0 + (float)(k & 1), yf = y0 + (float)(k >> 1);
    const bool ok = (xf > -1.0f) && (xf < (float)W) && (yf > -1.0f) && (yf < (float)H);
    t.ok[k] = ok;
    t.idx[k] = ok ? ((int)yf * W + (int)xf) : 0;
    t.wt[k] = wts[k];
  }
  return t;
}

__device__ __forceinline__ float bilinear(const float* __restrict__ plane, const Taps& t) {
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = t.ok[k] ? plane[t.idx[k]] : 0.0f;
  // nw*wnw + ne*wne + sw*wsw + se*wse as the compiled ATen CPU kernel evaluates it
  // (left to right, contracted into an fma chain)
  return __fmaf_rn(v[3], t.wt[3],
                   __fmaf_rn(v[2], t.wt[2], __fmaf_rn(v[1], t.wt[1], __fmul_rn(v[0], t.wt[0]))));
}

// ---------------------------------------------------------------------------
// Standalone warp (aarmvs_homo_warp): one thread per (b, pixel), all channels.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) homo_warp_kernel(const float* __restrict__ src,
                                                        const float* __restrict__ rel,
                                                        const float* __restrict__ depth, int C,
                                                        int H, int W, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int HW = H * W;
  const float* m = rel + 12 * b;
  const float dep = depth[b];
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    float ix, iy;
    sample_pos(m, dep, (float)(p % W), (float)(p / W), H, W, ix, iy);
    const Taps t = make_taps(ix, iy, H, W);
    const float* s = src + (size_t)b * C * HW;
    float* o = out + (size_t)b * C * HW + p;
    for (int c = 0; c < C; ++c) o[(size_t)c * HW] = bilinear(s + (size_t)c * HW, t);
  }
}

hipError_t launch_homo_warp(const float* src, const float* rel, const float* depth, int B, int C,
                            int H, int W, float* out, hipStream_t s) {
  const int HW = H * W;
  dim3 grid((unsigned)std::min((HW + 255) / 256, 4096), (unsigned)B);
  ProfScope ps(s, K_WARP);
  hipLaunchKernelGGL(homo_warp_kernel, grid, dim3(256), 0, s, src, rel, depth, C, H, W, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Backward of the warp w.r.t. the source features (aarmvs_homo_warp_backward):
// grid_sample's bilinear backward as a scatter-add of the output gradient into the
// four taps (no-return fp32 atomics; out-of-range taps receive nothing).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) homo_warp_bwd_kernel(const float* __restrict__ gout,
                                                            const float* __restrict__ rel,
                                                            const float* __restrict__ depth,
                                                            int C, int H, int W,
                                                            float* __restrict__ gsrc) {
  const int b = blockIdx.y;
  const int HW = H * W;
  const float* m = rel + 12 * b;
  const float dep = depth[b];
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    float ix, iy;
    sample_pos(m, dep, (float)(p % W), (float)(p / W), H, W, ix, iy);
    const Taps t = make_taps(ix, iy, H, W);
    const float* g = gout + (size_t)b * C * HW + p;
    float* s = gsrc + (size_t)b * C * HW;
    for (int c = 0; c < C; ++c) {
      const float gv = g[(size_t)c * HW];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (t.ok[k]) atomicAdd(s + (size_t)c * HW + t.idx[k], t.wt[k] * gv);
    }
  }
}

hipError_t launch_homo_warp_bwd(const float* gout, const float* rel, const float* depth, int B,
                                int C, int H, int W, float* gsrc, hipStream_t s) {
  const int HW = H * W;
  dim3 grid((unsigned)std::min((HW + 255) / 256, 4096), (unsigned)B);
  ProfScope ps(s, K_WARP);
  hipLaunchKernelGGL(homo_warp_bwd_kernel, grid, dim3(256), 0, s, gout, rel, depth, C, H, W, gsrc);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K1: warp + sqdiff on a haloed tile, omega conv3x3 32->4, GN#0 partial sums.
// Tile = 8 rows x 32 cols of output pixels; LDS holds sq for the 10x34 halo tile.
// ---------------------------------------------------------------------------
constexpr int T1_TH = 8, T1_TW = 32, T1_HH = T1_TH + 2, T1_HW = T1_TW + 2;
constexpr int T1_NPIX = T1_HH * T1_HW;  // 340

struct CostKArgs {
  const float* ref;
  const float* src[AARMVS_MAX_SRC];
  const float* rel;
  const float* depth_values;
  int d, D;
  const float* params;
  float* t1;
  double* stats;
  float* x;
  float* omega_out;
  int B, H, W, nsrc;
  size_t off_ow0, off_ob0, off_og0w, off_og0b, off_ow1, off_ob1, off_og1w, off_og1b, off_ow2,
      off_ob2, off_og2w, off_og2b, off_owo, off_obo;
};

__global__ void __launch_bounds__(256) cost_t1_kernel(CostKArgs a) {
  __shared__ float sq[kC * T1_NPIX];
  __shared__ float red[2 * 4];
  __shared__ double vstat[AARMVS_MAX_SRC][2];
  const int H = a.H, W = a.W, HW = H * W;
  const int tiles_x = (W + T1_TW - 1) / T1_TW, tiles_y = (H + T1_TH - 1) / T1_TH;
  const int ntiles = tiles_x * tiles_y;
  const int b = blockIdx.y;
  const float dep = a.depth_values[b * a.D + a.d];
  const float* ref = a.ref + (size_t)b * kC * HW;
  const float* w0 = a.params + a.off_ow0;   // [4][32][9]
  const float* b0 = a.params + a.off_ob0;
  if (threadIdx.x < AARMVS_MAX_SRC * 2) vstat[threadIdx.x >> 1][threadIdx.x & 1] = 0.0;
  __syncthreads();
  const int ty = threadIdx.x / T1_TW, tx = threadIdx.x % T1_TW;

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int y0 = (tile / tiles_x) * T1_TH, x0 = (tile % tiles_x) * T1_TW;
    for (int v = 0; v < a.nsrc; ++v) {
      const float* m = a.rel + 12 * (v * a.B + b);
      const float* src = a.src[v] + (size_t)b * kC * HW;
      // stage sq = (warp - ref)^2 on the halo tile (zero outside the image: conv padding)
      for (int i = threadIdx.x; i < T1_NPIX; i += blockDim.x) {
        const int gy = y0 - 1 + i / T1_HW, gx = x0 - 1 + i % T1_HW;
        if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
          float ix, iy;
          sample_pos(m, dep, (float)gx, (float)gy, H, W, ix, iy);
          const Taps t = make_taps(ix, iy, H, W);
          const int p = gy * W + gx;
#pragma unroll 4
          for (int c = 0; c < kC; ++c) {
            const float d = __fsub_rn(bilinear(src + (size_t)c * HW, t), ref[(size_t)c * HW + p]);
            sq[c * T1_NPIX + i] = __fmul_rn(d, d);
          }
        } else {
#pragma unroll 4
          for (int c = 0; c < kC; ++c) sq[c * T1_NPIX + i] = 0.0f;
        }
      }
      __syncthreads();
      // omega.reweight_network.0.0: conv3x3 32->4, pad 1
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int ci = 0; ci < kC; ++ci) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const float s = sq[ci * T1_NPIX + (ty + tap / 3) * T1_HW + tx + tap % 3];
#pragma unroll
          for (int co = 0; co < 4; ++co) acc[co] = fmaf(s, w0[(co * kC + ci) * 9 + tap], acc[co]);
        }
      }
      const int gy = y0 + ty, gx = x0 + tx;
      float part[2] = {0.f, 0.f};
      if (gy < H && gx < W) {
        float4 o;
        o.x = acc[0] + b0[0];
        o.y = acc[1] + b0[1];
        o.z = acc[2] + b0[2];
        o.w = acc[3] + b0[3];
        reinterpret_cast<float4*>(a.t1)[((size_t)b * a.nsrc + v) * HW + gy * W + gx] = o;
        part[0] = (o.x + o.y) + (o.z + o.w);
        part[1] = (o.x * o.x + o.y * o.y) + (o.z * o.z + o.w * o.w);
      }
      block_sum<2>(part, red);   // contains __syncthreads (also guards sq reuse)
      if (threadIdx.x == 0) {
        vstat[v][0] += part[0];
        vstat[v][1] += part[1];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < a.nsrc) {
    double* st = a.stats + ((size_t)b * nstat(a.nsrc) + stat_omega(threadIdx.x, 0)) * kSlots * 2;
    stat_add(st, vstat[threadIdx.x][0], vstat[threadIdx.x][1]);
  }
}

// omega pointwise chain helpers (ResnetBlockGn, module.py:252-264)
struct OmegaP {
  float w1[16], b1[4], w2[16], b2[4], wo[4], bo;
  float g0w[4], g0b[4], g1w[4], g1b[4], g2w[4], g2b[4];
};

__device__ __forceinline__ void load_omega(const CostKArgs& a, OmegaP& o) {
  const float* P = a.params;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    o.w1[i] = P[a.off_ow1 + i];
    o.w2[i] = P[a.off_ow2 + i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o.b1[i] = P[a.off_ob1 + i];
    o.b2[i] = P[a.off_ob2 + i];
    o.wo[i] = P[a.off_owo + i];
    o.g0w[i] = P[a.off_og0w + i];
    o.g0b[i] = P[a.off_og0b + i];
    o.g1w[i] = P[a.off_og1w + i];
    o.g1b[i] = P[a.off_og1b + i];
    o.g2w[i] = P[a.off_og2w + i];
    o.g2b[i] = P[a.off_og2b + i];
  }
  o.bo = P[a.off_obo];
}

__device__ __forceinline__ void gn_relu4(const float (&x)[4], const GnStat& s, const float* gw,
                                         const float* gb, bool relu, float (&y)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float sc = s.rstd * gw[c];
    const float sh = gb[c] - s.mean * sc;
    const float v = x[c] * sc + sh;
    y[c] = relu ? fmaxf(v, 0.0f) : v;
  }
}

__device__ __forceinline__ void conv1x1_4(const float (&x)[4], const float* w, const float* bias,
                                          float (&y)[4]) {
#pragma unroll
  for (int co = 0; co < 4; ++co) {
    float s = 0.f;
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) s = fmaf(w[co * 4 + ci], x[ci], s);
    y[co] = s + bias[co];
  }
}

// K2/K3: GN#STAGE partial sums of the stage's conv1x1 output.
template <int STAGE>
__global__ void __launch_bounds__(256) omega_stats_kernel(CostKArgs a) {
  __shared__ float red[2 * 4];
  __shared__ GnStat gs[2];
  const int v = blockIdx.y, b = blockIdx.z;
  const int HW = a.H * a.W;
  const double n = 4.0 * HW;
  const double* st = a.stats + ((size_t)b * nstat(a.nsrc) + stat_omega(v, 0)) * kSlots * 2;
  if (threadIdx.x < STAGE) gs[threadIdx.x] = stat_read(st + threadIdx.x * kSlots * 2, n);
  __syncthreads();
  OmegaP o;
  load_omega(a, o);
  const float4* t1 = reinterpret_cast<const float4*>(a.t1) + ((size_t)b * a.nsrc + v) * HW;
  float part[2] = {0.f, 0.f};
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    const float4 q = t1[p];
    const float t[4] = {q.x, q.y, q.z, q.w};
    float aa[4], t2[4];
    gn_relu4(t, gs[0], o.g0w, o.g0b, true, aa);
    conv1x1_4(aa, o.w1, o.b1, t2);
    float r[4];
    if (STAGE == 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c) r[c] = t2[c];
    } else {
      float bb[4];
      gn_relu4(t2, gs[1], o.g1w, o.g1b, true, bb);
      conv1x1_4(bb, o.w2, o.b2, r);
    }
    part[0] += (r[0] + r[1]) + (r[2] + r[3]);
    part[1] += (r[0] * r[0] + r[1] * r[1]) + (r[2] * r[2] + r[3] * r[3]);
  }
  block_sum<2>(part, red);
  if (threadIdx.x == 0) {
    stat_add(a.stats + ((size_t)b * nstat(a.nsrc) + stat_omega(v, STAGE)) * kSlots * 2, part[0],
             part[1]);
  }
}

// K4: final cost slice.  One thread per pixel, all views, all 32 channels.
__global__ void __launch_bounds__(256) cost_final_kernel(CostKArgs a) {
  __shared__ GnStat gs[AARMVS_MAX_SRC][3];
  const int b = blockIdx.y;
  const int H = a.H, W = a.W, HW = H * W;
  const double n = 4.0 * HW;
  if (threadIdx.x < 3 * a.nsrc) {
    const int v = threadIdx.x / 3, k = threadIdx.x % 3;
    gs[v][k] = stat_read(
        a.stats + ((size_t)b * nstat(a.nsrc) + stat_omega(v, k)) * kSlots * 2, n);
  }
  __syncthreads();
  OmegaP o;
  load_omega(a, o);
  const float dep = a.depth_values[b * a.D + a.d];
  const float* ref = a.ref + (size_t)b * kC * HW;
  const float inv_n = (float)a.nsrc;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    float acc[kC];
    float r[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      acc[c] = 0.f;
      r[c] = ref[(size_t)c * HW + p];
    }
    const float x = (float)(p % W), y = (float)(p / W);
    for (int v = 0; v < a.nsrc; ++v) {
      // omega weight of this view at this pixel
      const float4 q = reinterpret_cast<const float4*>(a.t1)[((size_t)b * a.nsrc + v) * HW + p];
      const float t[4] = {q.x, q.y, q.z, q.w};
      float aa[4], t2[4], bb[4], t3[4], g3[4];
      gn_relu4(t, gs[v][0], o.g0w, o.g0b, true, aa);
      conv1x1_4(aa, o.w1, o.b1, t2);
      gn_relu4(t2, gs[v][1], o.g1w, o.g1b, true, bb);
      conv1x1_4(bb, o.w2, o.b2, t3);
      gn_relu4(t3, gs[v][2], o.g2w, o.g2b, false, g3);
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) s = fmaf(o.wo[c], fmaxf(g3[c] + aa[c], 0.0f), s);
      const float wv = sigmoidf_(s + o.bo);
      if (a.omega_out) a.omega_out[((size_t)v * a.B + b) * HW + p] = wv;
      const float wp1 = __fadd_rn(wv, 1.0f);
      float ix, iy;
      sample_pos(a.rel + 12 * (v * a.B + b), dep, x, y, H, W, ix, iy);
      const Taps tp = make_taps(ix, iy, H, W);
      const float* src = a.src[v] + (size_t)b * kC * HW;
#pragma unroll 8
      for (int c = 0; c < kC; ++c) {
        const float d = __fsub_rn(bilinear(src + (size_t)c * HW, tp), r[c]);
        acc[c] = __fadd_rn(acc[c], __fmul_rn(wp1, __fmul_rn(d, d)));
      }
    }
    float* xo = a.x + (size_t)b * kC * HW + p;
#pragma unroll
    for (int c = 0; c < kC; ++c) xo[(size_t)c * HW] = -1.0f * __fdiv_rn(acc[c], inv_n);
  }
}

hipError_t launch_cost_slice(const CostArgs& ca, const SweepGeom& g, const Workspace& ws,
                             float* omega_out, hipStream_t s) {
  const ParamLayout& L = param_layout();
  CostKArgs a;
  a.ref = ca.ref;
  for (int v = 0; v < AARMVS_MAX_SRC; ++v) a.src[v] = v < g.nsrc ? ca.src[v] : nullptr;
  a.rel = ca.rel;
  a.depth_values = ca.depth_values;
  a.d = ca.d;
  a.D = g.D;
  a.params = ca.params;
  a.t1 = ws.t1;
  a.stats = ws.stats;
  a.x = ws.x;
  a.omega_out = omega_out;
  a.B = g.B;
  a.H = g.H;
  a.W = g.W;
  a.nsrc = g.nsrc;
  a.off_ow0 = L.pk_off[P_OW0];
  a.off_ob0 = L.pk_off[P_OB0];
  a.off_og0w = L.pk_off[P_OG0W];
  a.off_og0b = L.pk_off[P_OG0B];
  a.off_ow1 = L.pk_off[P_OW1];
  a.off_ob1 = L.pk_off[P_OB1];
  a.off_og1w = L.pk_off[P_OG1W];
  a.off_og1b = L.pk_off[P_OG1B];
  a.off_ow2 = L.pk_off[P_OW2];
  a.off_ob2 = L.pk_off[P_OB2];
  a.off_og2w = L.pk_off[P_OG2W];
  a.off_og2b = L.pk_off[P_OG2B];
  a.off_owo = L.pk_off[P_OWO];
  a.off_obo = L.pk_off[P_OBO];

  const int HW = g.H * g.W;
  const int ntiles = ((g.W + T1_TW - 1) / T1_TW) * ((g.H + T1_TH - 1) / T1_TH);
  const int per_b = std::max(1, std::min(ntiles, 4 * g.cu_count / std::max(1, g.B)));
  {
    ProfScope ps(s, K_COST_T1);
    hipLaunchKernelGGL(cost_t1_kernel, dim3(per_b, g.B), dim3(256), 0, s, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int pblk = std::max(1, std::min((HW + 255) / 256, 2 * g.cu_count / std::max(1, g.B * g.nsrc) + 1));
  {
    ProfScope ps(s, K_OMEGA1);
    hipLaunchKernelGGL(omega_stats_kernel<1>, dim3(pblk, g.nsrc, g.B), dim3(256), 0, s, a);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  {
    ProfScope ps(s, K_OMEGA2);
    hipLaunchKernelGGL(omega_stats_kernel<2>, dim3(pblk, g.nsrc, g.B), dim3(256), 0, s, a);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int fblk = std::max(1, std::min((HW + 255) / 256, 8 * g.cu_count / std::max(1, g.B)));
  {
    ProfScope ps(s, K_COST_FINAL);
    hipLaunchKernelGGL(cost_final_kernel, dim3(fblk, g.B), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace aarmvs
