// Homography warp, inter-view adaptive aggregation (omega) and the per-plane cost
// slice for gfx950.
//
// Reference: models/module.py:6-38 (homo_warping_depthwise),
//            models/drmvsnet.py:27-38 (InterViewAAModule), :307-319 (accumulation).
//
// Per plane and batch element the cost slice needs three grid-wide GroupNorm
// reductions per source view.  They are met by a one-plane-ahead pipeline
// (see cost_pipe_kernel below): per plane one streaming launch over the source
// features plus two small statistics launches over the 16-B/px/view omega conv output.
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
  unsigned idx[4];
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
    t.idx[k] = ok ? (unsigned)((int)yf * W + (int)xf) : 0u;
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

// Buffer-descriptor gathers for the streaming kernels: 32-bit byte offsets instead of
// 64-bit addresses (VGPR pressure), and the hardware range check does the zero padding:
// an out-of-range tap gets offset = num_records and loads 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const float* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
  void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)n, 0x00020000);
}

struct BTaps {
  uint32_t off[4];   // byte offset within one channel plane, or `oob`
  float wt[4];
};

__device__ __forceinline__ BTaps make_btaps(float ix, float iy, int H, int W, uint32_t oob) {
  BTaps t;
  const float x0 = floorf(ix), y0 = floorf(iy);
  const float wx = __fsub_rn(ix, x0), wy = __fsub_rn(iy, y0);
  const float ex = __fsub_rn(1.0f, wx), sy = __fsub_rn(1.0f, wy);
  t.wt[0] = __fmul_rn(sy, ex);
  t.wt[1] = __fmul_rn(sy, wx);
  t.wt[2] = __fmul_rn(wy, ex);
  t.wt[3] = __fmul_rn(wy, wx);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float xf = x0 + (float)(k & 1), yf = y0 + (float)(k >> 1);
    const bool ok = (xf > -1.0f) && (xf < (float)W) && (yf > -1.0f) && (yf < (float)H);
    t.off[k] = ok ? (uint32_t)((int)yf * W + (int)xf) * 4u : oob;
  }
  return t;
}

// bilinear sample of channel plane at byte offset `coff` (same fma chain as bilinear())
__device__ __forceinline__ float bilinear_b(__amdgpu_buffer_rsrc_t r, const BTaps& t, uint32_t coff) {
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    v[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, t.off[k], coff, 0));
  return __fmaf_rn(v[3], t.wt[3],
                   __fmaf_rn(v[2], t.wt[2], __fmaf_rn(v[1], t.wt[1], __fmul_rn(v[0], t.wt[0]))));
}

__device__ __forceinline__ float load_b(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t coff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, coff, 0));
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
// Cost-slice pipeline.
//
// The cost slice of plane d does not depend on the recurrence, so the sweep runs it
// one plane ahead: launch P(d) = cost_pipe(prev = d, next = d + 1) does, per tile,
//   prev part  x_d = -(sum_v (1 + w_v) (warp_v(d) - ref)^2) / nsrc, with w_v from the
//              omega conv output t1_d and plane d's three GroupNorm statistics;
//   next part  sq_v(d+1) = (warp_v(d+1) - ref)^2 on a haloed tile in LDS, the omega
//              conv3x3 32->4 -> t1_{d+1} (16 B/px/view), GroupNorm #0 partial sums.
// Both parts sample the same source neighbourhood (adjacent depths), so the second
// gather of a (pixel, view) hits in L1/L2: the source features stream from HBM about
// once per plane.  omega_stats<1>/<2> then complete plane d+1's GN #1/#2 statistics
// from t1_{d+1} alone.
// ---------------------------------------------------------------------------
struct PipeArgs {
  const float* ref;
  const float* src[AARMVS_MAX_SRC];
  const float* rel;           // [nsrc][B][12]
  const float* dvals;         // [B][D]
  int D;
  int d_prev, d_next;         // -1: part disabled
  const float4* t1_prev;      // [B][nsrc][HW]
  float4* t1_next;
  const double* st_prev;      // [B][nsrc][3][kSlots][2]
  double* st_next;
  float* x;                   // [B,32,H,W]
  float* omega_out;           // [nsrc,B,H,W] (prev plane) or null
  const float* params;
  size_t off_ow0, off_ob0, off_og0w, off_og0b, off_ow1, off_ob1, off_og1w, off_og1b, off_ow2,
      off_ob2, off_og2w, off_og2b, off_owo, off_obo;
  int B, H, W, nsrc;
  double* zero_ptr;           // omega_stats<1>: stale statistics to clear (or null)
  int zero_n;
};

// omega pointwise chain helpers (ResnetBlockGn, module.py:252-264)
struct OmegaP {
  float w1[16], b1[4], w2[16], b2[4], wo[4], bo;
  float g0w[4], g0b[4], g1w[4], g1b[4], g2w[4], g2b[4];
};

__device__ __forceinline__ void load_omega(const PipeArgs& a, const float* __restrict__ P,
                                           OmegaP& o) {
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

// omega weight of one (pixel, view) from its conv3x3 output t and the three GN stats
// (drmvsnet.py:30-35 after the first conv)
__device__ __forceinline__ float omega_weight(const float4 q, const GnStat* gs, const PipeArgs& a,
                                              const float* __restrict__ P) {
  OmegaP o;
  load_omega(a, P, o);
  const float t[4] = {q.x, q.y, q.z, q.w};
  float aa[4], t2[4], bb[4], t3[4], g3[4];
  gn_relu4(t, gs[0], o.g0w, o.g0b, true, aa);
  conv1x1_4(aa, o.w1, o.b1, t2);
  gn_relu4(t2, gs[1], o.g1w, o.g1b, true, bb);
  conv1x1_4(bb, o.w2, o.b2, t3);
  gn_relu4(t3, gs[2], o.g2w, o.g2b, false, g3);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) s = fmaf(o.wo[c], fmaxf(g3[c] + aa[c], 0.0f), s);
  return sigmoidf_(s + o.bo);
}

__device__ __forceinline__ size_t st_index(int b, int v, int k, int nsrc) {
  return (((size_t)b * nsrc + v) * 3 + k) * kSlots * 2;
}

constexpr int kPipeTW = 32;

template <int TH>
struct PipeCfg {
  static constexpr int THREADS = TH * kPipeTW;
  static constexpr int HH = TH + 2, HW = kPipeTW + 2, NPIX = HH * HW;
  static constexpr int RING = 2 * HW + 2 * TH;
  static constexpr int WAVES = THREADS / 64;
};

// XCD-aware contiguous tile range of this block: blocks are dealt round-robin over the
// 8 XCDs, so logical block l = xcd * (G/8) + slot gives every XCD one contiguous band of
// tiles (neighbouring tiles share source rows in that XCD's L2).  Speed only.
__device__ __forceinline__ void tile_range(int ntiles, int& t0, int& t1) {
  const int G = gridDim.x;
  int l = blockIdx.x;
  if ((G & 7) == 0) l = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int chunk = (ntiles + G - 1) / G;
  t0 = min(ntiles, l * chunk);
  t1 = min(ntiles, t0 + chunk);
}

template <int TH>
__global__ void __launch_bounds__(TH * kPipeTW) cost_pipe_kernel(PipeArgs a,
                                                                 const float* __restrict__ P) {
  using Cfg = PipeCfg<TH>;
  __shared__ float sq[kC * Cfg::NPIX];
  __shared__ float wsum[Cfg::WAVES][AARMVS_MAX_SRC][2];
  __shared__ GnStat gs[AARMVS_MAX_SRC][3];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.y;
  const int H = a.H, W = a.W, HW = H * W, nsrc = a.nsrc;
  const bool prev = a.d_prev >= 0, next = a.d_next >= 0;
  for (int i = tid; i < Cfg::WAVES * AARMVS_MAX_SRC * 2; i += Cfg::THREADS)
    (&wsum[0][0][0])[i] = 0.f;
  if (prev && tid < 3 * nsrc) {
    const int v = tid / 3, k = tid % 3;
    gs[v][k] = stat_read(a.st_prev + st_index(b, v, k, nsrc), 4.0 * HW);
  }
  __syncthreads();
  // parameters come through a __restrict__ argument so that their uniform loads can be
  // scalar (s_load) despite the kernel's vector stores
  const float* __restrict__ w0 = P + a.off_ow0;   // [4][32][9]
  const float* __restrict__ b0 = P + a.off_ob0;
  const float dprev = prev ? a.dvals[b * a.D + a.d_prev] : 0.f;
  const float dnext = next ? a.dvals[b * a.D + a.d_next] : 0.f;
  const uint32_t fbytes = (uint32_t)((size_t)kC * HW * 4);   // one view's [32,H,W] map
  const __amdgpu_buffer_rsrc_t rref = uniform_rsrc(a.ref + (size_t)b * kC * HW, fbytes);
  const uint32_t cstride = (uint32_t)HW * 4u;
  const float inv_n = (float)nsrc;

  // ring (halo-only) pixel of this thread, in halo-tile coordinates
  int rhy = -1, rhx = -1;
  if (tid < Cfg::RING) {
    const int i = tid;
    if (i < Cfg::HW) { rhy = 0; rhx = i; }
    else if (i < 2 * Cfg::HW) { rhy = TH + 1; rhx = i - Cfg::HW; }
    else if (i < 2 * Cfg::HW + TH) { rhy = 1 + i - 2 * Cfg::HW; rhx = 0; }
    else { rhy = 1 + i - 2 * Cfg::HW - TH; rhx = Cfg::HW - 1; }
  }
  const int ty = tid / kPipeTW, tx = tid % kPipeTW;

  const int tiles_x = (W + kPipeTW - 1) / kPipeTW, tiles_y = (H + TH - 1) / TH;
  int tb, te;
  tile_range(tiles_x * tiles_y, tb, te);
  for (int tile = tb; tile < te; ++tile) {
    const int y0 = (tile / tiles_x) * TH, x0 = (tile % tiles_x) * kPipeTW;
    const int gy = y0 + ty, gx = x0 + tx;
    const bool inside = gy < H && gx < W;
    const int p = gy * W + gx;
    const uint32_t pofs = inside ? (uint32_t)p * 4u : fbytes;   // reference pixel (re-read: L1/L2)
    float acc[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c) acc[c] = 0.f;
    const int ry = y0 - 1 + rhy, rx = x0 - 1 + rhx;
    const bool ring_in = rhy >= 0 && ry >= 0 && ry < H && rx >= 0 && rx < W;
    for (int v = 0; v < nsrc; ++v) {
      const float* m = a.rel + 12 * (v * a.B + b);
      const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(a.src[v] + (size_t)b * kC * HW, fbytes);
      if (prev && inside) {
        const float wv =
            omega_weight(a.t1_prev[((size_t)b * nsrc + v) * HW + p], gs[v], a, P);
        if (a.omega_out) a.omega_out[((size_t)v * a.B + b) * HW + p] = wv;
        const float wp1 = __fadd_rn(wv, 1.0f);
        float ix, iy;
        sample_pos(m, dprev, (float)gx, (float)gy, H, W, ix, iy);
        const BTaps t = make_btaps(ix, iy, H, W, fbytes);
#pragma unroll 8
        for (int c = 0; c < kC; ++c) {
          const float d = __fsub_rn(bilinear_b(rsrc, t, c * cstride), load_b(rref, pofs, c * cstride));
          acc[c] = __fadd_rn(acc[c], __fmul_rn(wp1, __fmul_rn(d, d)));
        }
      }
      if (next) {
        // own (interior) pixel
        {
          const int hidx = (ty + 1) * Cfg::HW + tx + 1;
          if (inside) {
            float ix, iy;
            sample_pos(m, dnext, (float)gx, (float)gy, H, W, ix, iy);
            const BTaps t = make_btaps(ix, iy, H, W, fbytes);
#pragma unroll 8
            for (int c = 0; c < kC; ++c) {
              const float d = __fsub_rn(bilinear_b(rsrc, t, c * cstride), load_b(rref, pofs, c * cstride));
              sq[c * Cfg::NPIX + hidx] = __fmul_rn(d, d);
            }
          } else {
#pragma unroll
            for (int c = 0; c < kC; ++c) sq[c * Cfg::NPIX + hidx] = 0.f;
          }
        }
        // ring pixel (zero outside the image: the conv's zero padding)
        if (rhy >= 0) {
          const int hidx = rhy * Cfg::HW + rhx;
          if (ring_in) {
            float ix, iy;
            sample_pos(m, dnext, (float)rx, (float)ry, H, W, ix, iy);
            const BTaps t = make_btaps(ix, iy, H, W, fbytes);
            const uint32_t qofs = (uint32_t)(ry * W + rx) * 4u;
#pragma unroll 8
            for (int c = 0; c < kC; ++c) {
              const float d = __fsub_rn(bilinear_b(rsrc, t, c * cstride), load_b(rref, qofs, c * cstride));
              sq[c * Cfg::NPIX + hidx] = __fmul_rn(d, d);
            }
          } else {
#pragma unroll
            for (int c = 0; c < kC; ++c) sq[c * Cfg::NPIX + hidx] = 0.f;
          }
        }
        __syncthreads();
        // omega.reweight_network.0.0: conv3x3 32->4, pad 1
        float o4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int ci = 0; ci < kC; ++ci) {
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) {
            const float s = sq[ci * Cfg::NPIX + (ty + tap / 3) * Cfg::HW + tx + tap % 3];
#pragma unroll
            for (int co = 0; co < 4; ++co) o4[co] = fmaf(s, w0[(co * kC + ci) * 9 + tap], o4[co]);
          }
        }
        float ps = 0.f, pss = 0.f;
        if (inside) {
          float4 out;
          out.x = o4[0] + b0[0];
          out.y = o4[1] + b0[1];
          out.z = o4[2] + b0[2];
          out.w = o4[3] + b0[3];
          a.t1_next[((size_t)b * nsrc + v) * HW + p] = out;
          ps = (out.x + out.y) + (out.z + out.w);
          pss = (out.x * out.x + out.y * out.y) + (out.z * out.z + out.w * out.w);
        }
        ps = wave_sum(ps);
        pss = wave_sum(pss);
        if (lane == 0) {
          wsum[wave][v][0] += ps;
          wsum[wave][v][1] += pss;
        }
        __syncthreads();   // sq is rewritten by the next view
      }
    }
    if (prev && inside) {
      float* xo = a.x + (size_t)b * kC * HW + p;
#pragma unroll
      for (int c = 0; c < kC; ++c) xo[(size_t)c * HW] = -1.0f * __fdiv_rn(acc[c], inv_n);
    }
  }
  if (next) {
    __syncthreads();
    if (tid < nsrc) {
      double s = 0.0, ss = 0.0;
      for (int w = 0; w < Cfg::WAVES; ++w) {
        s += wsum[w][tid][0];
        ss += wsum[w][tid][1];
      }
      stat_add(a.st_next + st_index(b, tid, 0, nsrc), s, ss);
    }
  }
}

// GN #STAGE (1 or 2) partial sums of the omega chain on t1 (plane d_next).  Stage 1
// also clears the statistics of the plane before (their last reader has finished).
template <int STAGE>
__global__ void __launch_bounds__(256) omega_stats_kernel(PipeArgs a,
                                                          const float* __restrict__ P) {
  __shared__ float red[2 * 4];
  __shared__ GnStat gs[2];
  const int v = blockIdx.y, b = blockIdx.z;
  const int HW = a.H * a.W;
  if (STAGE == 1 && a.zero_ptr && v == 0 && b == 0)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.zero_n; i += gridDim.x * blockDim.x)
      a.zero_ptr[i] = 0.0;
  if (threadIdx.x < STAGE)
    gs[threadIdx.x] = stat_read(a.st_next + st_index(b, v, threadIdx.x, a.nsrc), 4.0 * HW);
  __syncthreads();
  OmegaP o;
  load_omega(a, P, o);
  const float4* t1 = a.t1_next + ((size_t)b * a.nsrc + v) * HW;
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
  if (threadIdx.x == 0) stat_add(a.st_next + st_index(b, v, STAGE, a.nsrc), part[0], part[1]);
}

static PipeArgs pipe_args(const CostArgs& ca, const SweepGeom& g, const Workspace& ws) {
  const ParamLayout& L = param_layout();
  PipeArgs a{};
  a.ref = ca.ref;
  for (int v = 0; v < AARMVS_MAX_SRC; ++v) a.src[v] = v < g.nsrc ? ca.src[v] : nullptr;
  a.rel = ca.rel;
  a.dvals = ca.depth_values;
  a.D = g.D;
  a.params = ca.params;
  a.x = ws.x;
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
  return a;
}

constexpr int kPipeTH = 8;

hipError_t launch_cost_pipe(const CostArgs& ca, const SweepGeom& g, const Workspace& ws,
                            int d_prev, int d_next, float* omega_out, hipStream_t s) {
  PipeArgs a = pipe_args(ca, g, ws);
  a.d_prev = d_prev;
  a.d_next = d_next;
  if (d_prev >= 0) {
    a.t1_prev = reinterpret_cast<const float4*>(ws.t1[d_prev & 1]);
    a.st_prev = ws.omega_stats[d_prev & 1];
  }
  if (d_next >= 0) {
    a.t1_next = reinterpret_cast<float4*>(ws.t1[d_next & 1]);
    a.st_next = ws.omega_stats[d_next & 1];
  }
  a.omega_out = omega_out;
  using Cfg = PipeCfg<kPipeTH>;
  const int ntiles = ((g.W + kPipeTW - 1) / kPipeTW) * ((g.H + kPipeTH - 1) / kPipeTH);
  int blocks = std::max(1, std::min(ntiles, 4 * g.cu_count / std::max(1, g.B)));
  if (blocks >= 64) blocks &= ~7;   // multiple of 8 for the XCD-aware tile mapping
  hipError_t e;
  {
    ProfScope ps(s, K_COST_PIPE);
    hipLaunchKernelGGL(cost_pipe_kernel<kPipeTH>, dim3(blocks, g.B), dim3(Cfg::THREADS), 0, s, a,
                       a.params);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (d_next < 0) return hipSuccess;
  // GN #1 / #2 statistics of plane d_next; stage 1 clears plane d_prev's statistics
  if (d_prev >= 0) {
    a.zero_ptr = ws.omega_stats[d_prev & 1];
    a.zero_n = (int)(ws.omega_stats_bytes / sizeof(double));
  }
  const int HW = g.H * g.W;
  const int pblk =
      std::max(1, std::min((HW + 255) / 256, 2 * g.cu_count / std::max(1, g.B * g.nsrc) + 1));
  {
    ProfScope ps(s, K_OMEGA1);
    hipLaunchKernelGGL(omega_stats_kernel<1>, dim3(pblk, g.nsrc, g.B), dim3(256), 0, s, a, a.params);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  {
    ProfScope ps(s, K_OMEGA2);
    hipLaunchKernelGGL(omega_stats_kernel<2>, dim3(pblk, g.nsrc, g.B), dim3(256), 0, s, a, a.params);
  }
  return hipGetLastError();
}

}  // namespace aarmvs
