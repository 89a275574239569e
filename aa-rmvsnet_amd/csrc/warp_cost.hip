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
  size_t off_ow0t, off_ow0, off_ob0, off_og0w, off_og0b, off_ow1, off_ob1, off_og1w, off_og1b, off_ow2,
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

// NHWC gathers: a tap of one pixel is 32 contiguous channels (128 B); lane k of an
// 8-lane pixel group loads channels 4k..4k+3 with one dwordx4 (the per-CU address rate,
// not HBM, limits dword gathers).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}

// byte offsets of the 4 taps (pixel * 128 B, or `oob`) + weights
__device__ __forceinline__ BTaps make_ntaps(float ix, float iy, int H, int W, uint32_t oob) {
  BTaps t = make_btaps(ix, iy, H, W, oob);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (t.off[k] != oob) t.off[k] *= 32u;   // dword offset of the pixel * 4 B -> * 128 B
  return t;
}

// bilinear sample of 4 channels (byte offset `coff` within the pixel), same fma chain
__device__ __forceinline__ float4 bilinear4(__amdgpu_buffer_rsrc_t r, const BTaps& t, uint32_t coff) {
  const float4 v0 = ld4(r, t.off[0] + coff), v1 = ld4(r, t.off[1] + coff);
  const float4 v2 = ld4(r, t.off[2] + coff), v3 = ld4(r, t.off[3] + coff);
  auto one = [&](float a0, float a1, float a2, float a3) {
    return __fmaf_rn(a3, t.wt[3], __fmaf_rn(a2, t.wt[2], __fmaf_rn(a1, t.wt[1], __fmul_rn(a0, t.wt[0]))));
  };
  return make_float4(one(v0.x, v1.x, v2.x, v3.x), one(v0.y, v1.y, v2.y, v3.y),
                     one(v0.z, v1.z, v2.z, v3.z), one(v0.w, v1.w, v2.w, v3.w));
}

struct RingTap {
  BTaps t;
  uint32_t qofs;   // reference pixel byte offset (or out of range)
  int hidx;        // position in the halo tile
};

constexpr int kPipeTW = 32;
constexpr int kPipeThreads = 256;   // 32 pixel columns x 8 lanes
constexpr int kSqStride = 36;       // floats per pixel in the LDS tile: conflict-free b128 reads

template <int TH>
struct PipeCfg {
  static constexpr int HH = TH + 2, HW = kPipeTW + 2, NPIX = HH * HW;
  static constexpr int RING = 2 * HW + 2 * TH;
  static constexpr int PIX = TH * kPipeTW;
  static constexpr int WAVES = kPipeThreads / 64;
  static constexpr int SQ_FLOATS = NPIX * kSqStride;
  static constexpr int WT_FLOATS = AARMVS_MAX_SRC * PIX;
  static constexpr int LDS_FLOATS = SQ_FLOATS > WT_FLOATS ? SQ_FLOATS : WT_FLOATS;
};

// ABL: ablation bits for the diagnostic harness (tools/microbench/pipe_bench.cpp); the
// library only instantiates ABL = 0.  1: no prev part, 2: no next-part own gathers,
// 4: no ring gathers, 8: no conv.
template <int TH, int ABL = 0>
__global__ void __launch_bounds__(kPipeThreads) cost_pipe_kernel(PipeArgs a,
                                                                 const float* __restrict__ P,
                                                                 const float* __restrict__ Rel) {
  using Cfg = PipeCfg<TH>;
  // sq tile (next part) and the omega-weight table (prev part) share the LDS
  __shared__ __attribute__((aligned(16))) float lds[Cfg::LDS_FLOATS];
  __shared__ RingTap ring[Cfg::RING];
  __shared__ float wsum[Cfg::WAVES][AARMVS_MAX_SRC][2];
  __shared__ GnStat gs[AARMVS_MAX_SRC][3];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = tid >> 3, k = tid & 7;        // 8-lane pixel groups
  const uint32_t koff = 16u * k;                // this lane's 4 channels within a pixel
  const int b = blockIdx.y;
  const int H = a.H, W = a.W, HW = H * W, nsrc = a.nsrc;
  const bool prev = a.d_prev >= 0 && !(ABL & 1), next = a.d_next >= 0;
  for (int i = tid; i < Cfg::WAVES * AARMVS_MAX_SRC * 2; i += kPipeThreads)
    (&wsum[0][0][0])[i] = 0.f;
  if (prev && tid < 3 * nsrc) {
    const int v = tid / 3, kk = tid % 3;
    gs[v][kk] = stat_read(a.st_prev + st_index(b, v, kk, nsrc), 4.0 * HW);
  }
  __syncthreads();
  // parameters come through a __restrict__ argument so that their uniform loads can be
  // scalar (s_load) despite the kernel's vector stores
  const float* __restrict__ w0t = P + a.off_ow0t;   // [9][32][4]
  const float* __restrict__ b0 = P + a.off_ob0;
  const float dprev = prev ? a.dvals[b * a.D + a.d_prev] : 0.f;
  const float dnext = next ? a.dvals[b * a.D + a.d_next] : 0.f;
  const uint32_t fbytes = (uint32_t)((size_t)kC * HW * 4);   // one view's [H,W,32] map
  const __amdgpu_buffer_rsrc_t rref = uniform_rsrc(a.ref + (size_t)b * kC * HW, fbytes);
  const float inv_n = (float)nsrc;
  const int tiles_x = (W + kPipeTW - 1) / kPipeTW;
  const int tile = blockIdx.x;
  const int y0 = (tile / tiles_x) * TH, x0 = (tile % tiles_x) * kPipeTW;

  if (prev) {
    // omega weights w_v of the tile's pixels (one pixel per thread) -> LDS; two views
    // per step so that two t1 loads are in flight
    float* wtab = lds;
    for (int i = tid; i < Cfg::PIX; i += kPipeThreads) {
      const int gy = y0 + i / kPipeTW, gx = x0 + i % kPipeTW;
      const bool inside = gy < H && gx < W;
      const size_t p = inside ? (size_t)gy * W + gx : 0;
      for (int v = 0; v < nsrc; v += 2) {
        const bool two = v + 1 < nsrc;
        const float4 q0 = a.t1_prev[((size_t)b * nsrc + v) * HW + p];
        const float4 q1 = two ? a.t1_prev[((size_t)b * nsrc + v + 1) * HW + p] : q0;
        const float w0v = inside ? omega_weight(q0, gs[v], a, P) : 0.f;
        wtab[v * Cfg::PIX + i] = __fadd_rn(w0v, 1.0f);
        if (inside && a.omega_out) a.omega_out[((size_t)v * a.B + b) * HW + p] = w0v;
        if (two) {
          const float w1v = inside ? omega_weight(q1, gs[v + 1], a, P) : 0.f;
          wtab[(v + 1) * Cfg::PIX + i] = __fadd_rn(w1v, 1.0f);
          if (inside && a.omega_out) a.omega_out[((size_t)(v + 1) * a.B + b) * HW + p] = w1v;
        }
      }
    }
    __syncthreads();
    // x = -(sum_v (1 + w_v) (warp_v - ref)^2) / nsrc, 4 channels per lane; RB rows and
    // two views per step keep 2 x RB x 4 tap loads in flight (the view order of the
    // accumulation is kept)
    constexpr int RB = 2;
    static_assert(TH % RB == 0, "rows per step must divide the tile height");
    for (int r0 = 0; r0 < TH; r0 += RB) {
      int gy[RB], gx = x0 + col, p[RB];
      bool inside[RB];
      float4 rf[RB], acc[RB];
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        gy[j] = y0 + r0 + j;
        inside[j] = gy[j] < H && gx < W;
        p[j] = gy[j] * W + gx;
        rf[j] = ld4(rref, (inside[j] ? (uint32_t)p[j] * 128u : fbytes) + koff);
        acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      for (int v = 0; v < nsrc; v += 2) {
        const int nv = v + 1 < nsrc ? 2 : 1;
        float4 g[2][RB];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (u < nv) {
            const __amdgpu_buffer_rsrc_t rsrc =
                uniform_rsrc(a.src[v + u] + (size_t)b * kC * HW, fbytes);
#pragma unroll
            for (int j = 0; j < RB; ++j) {
              float ix, iy;
              sample_pos(Rel + 12 * ((v + u) * a.B + b), dprev, (float)gx, (float)gy[j], H, W,
                         ix, iy);
              const BTaps t = make_ntaps(ix, iy, H, W, fbytes);
              g[u][j] = bilinear4(rsrc, t, koff);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (u < nv) {
#pragma unroll
            for (int j = 0; j < RB; ++j) {
              const float wp1 = wtab[(v + u) * Cfg::PIX + (r0 + j) * kPipeTW + col];
              const float dx = __fsub_rn(g[u][j].x, rf[j].x), dy = __fsub_rn(g[u][j].y, rf[j].y);
              const float dz = __fsub_rn(g[u][j].z, rf[j].z), dw = __fsub_rn(g[u][j].w, rf[j].w);
              acc[j].x = __fadd_rn(acc[j].x, __fmul_rn(wp1, __fmul_rn(dx, dx)));
              acc[j].y = __fadd_rn(acc[j].y, __fmul_rn(wp1, __fmul_rn(dy, dy)));
              acc[j].z = __fadd_rn(acc[j].z, __fmul_rn(wp1, __fmul_rn(dz, dz)));
              acc[j].w = __fadd_rn(acc[j].w, __fmul_rn(wp1, __fmul_rn(dw, dw)));
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        if (inside[j]) {
          float* xo = a.x + (size_t)b * kC * HW + (size_t)(4 * k) * HW + p[j];   // NCHW
          xo[0] = -1.0f * __fdiv_rn(acc[j].x, inv_n);
          xo[(size_t)HW] = -1.0f * __fdiv_rn(acc[j].y, inv_n);
          xo[(size_t)2 * HW] = -1.0f * __fdiv_rn(acc[j].z, inv_n);
          xo[(size_t)3 * HW] = -1.0f * __fdiv_rn(acc[j].w, inv_n);
        }
      }
    }
    __syncthreads();   // the weight table's LDS becomes the sq tile
  }

  if (next) {
    float* sq = lds;
    for (int v = 0; v < nsrc; ++v) {
      const float* m = Rel + 12 * (v * a.B + b);
      const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(a.src[v] + (size_t)b * kC * HW, fbytes);
      if (tid < Cfg::RING) {
        // taps of this thread's ring (halo-only) pixel, shared through LDS
        int hy, hx;
        if (tid < Cfg::HW) { hy = 0; hx = tid; }
        else if (tid < 2 * Cfg::HW) { hy = TH + 1; hx = tid - Cfg::HW; }
        else if (tid < 2 * Cfg::HW + TH) { hy = 1 + tid - 2 * Cfg::HW; hx = 0; }
        else { hy = 1 + tid - 2 * Cfg::HW - TH; hx = Cfg::HW - 1; }
        const int ry = y0 - 1 + hy, rx = x0 - 1 + hx;
        RingTap rt;
        rt.hidx = hy * Cfg::HW + hx;
        if (ry >= 0 && ry < H && rx >= 0 && rx < W && !(ABL & 4)) {
          float ix, iy;
          sample_pos(m, dnext, (float)rx, (float)ry, H, W, ix, iy);
          rt.t = make_ntaps(ix, iy, H, W, fbytes);
          rt.qofs = (uint32_t)(ry * W + rx) * 128u;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            rt.t.off[q] = fbytes;
            rt.t.wt[q] = 0.f;
          }
          rt.qofs = fbytes;
        }
        ring[tid] = rt;
      }
      // own rows: squared difference at d_next -> LDS tile (zero outside the image)
      for (int r = 0; r < TH; ++r) {
        const int gy = y0 + r, gx = x0 + col;
        const bool inside = gy < H && gx < W && !(ABL & 2);
        float ix, iy;
        sample_pos(m, dnext, (float)gx, (float)gy, H, W, ix, iy);
        BTaps t = make_ntaps(ix, iy, H, W, fbytes);
        if (!inside)
#pragma unroll
          for (int q = 0; q < 4; ++q) t.off[q] = fbytes;
        const float4 g = bilinear4(rsrc, t, koff);
        const float4 rf = ld4(rref, (inside ? (uint32_t)(gy * W + gx) * 128u : fbytes) + koff);
        const float dx = __fsub_rn(g.x, rf.x), dy = __fsub_rn(g.y, rf.y);
        const float dz = __fsub_rn(g.z, rf.z), dw = __fsub_rn(g.w, rf.w);
        *reinterpret_cast<float4*>(&sq[((r + 1) * Cfg::HW + col + 1) * kSqStride + 4 * k]) =
            make_float4(__fmul_rn(dx, dx), __fmul_rn(dy, dy), __fmul_rn(dz, dz), __fmul_rn(dw, dw));
      }
      __syncthreads();   // ring tap table ready
      for (int i = tid; i < Cfg::RING * 8; i += kPipeThreads) {
        const RingTap& rt = ring[i >> 3];   // (i & 7) == k
        const float4 g = bilinear4(rsrc, rt.t, koff);
        const float4 rf = ld4(rref, rt.qofs + koff);
        const float dx = __fsub_rn(g.x, rf.x), dy = __fsub_rn(g.y, rf.y);
        const float dz = __fsub_rn(g.z, rf.z), dw = __fsub_rn(g.w, rf.w);
        *reinterpret_cast<float4*>(&sq[rt.hidx * kSqStride + 4 * k]) =
            make_float4(__fmul_rn(dx, dx), __fmul_rn(dy, dy), __fmul_rn(dz, dz), __fmul_rn(dw, dw));
      }
      __syncthreads();
      // omega.reweight_network.0.0: conv3x3 32->4, pad 1; one output pixel per thread
      float ps = 0.f, pss = 0.f;
      for (int i = tid; i < Cfg::PIX; i += kPipeThreads) {
        const int py = i / kPipeTW, px = i % kPipeTW;
        float o4[4] = {0.f, 0.f, 0.f, 0.f};
        if (!(ABL & 8)) {
#pragma unroll 1
          for (int tap = 0; tap < 9; ++tap) {
            const float4* s4 = reinterpret_cast<const float4*>(
                &sq[((py + tap / 3) * Cfg::HW + px + tap % 3) * kSqStride]);
#pragma unroll 2
            for (int c4 = 0; c4 < 8; ++c4) {
              const float4 q = s4[c4];
              const float qq[4] = {q.x, q.y, q.z, q.w};
              const float* wt = w0t + (tap * kC + 4 * c4) * 4;   // [j][co], contiguous
#pragma unroll
              for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int co = 0; co < 4; ++co) o4[co] = fmaf(qq[j], wt[j * 4 + co], o4[co]);
            }
          }
        }
        const int gy = y0 + py, gx = x0 + px;
        if (gy < H && gx < W) {
          float4 out;
          out.x = o4[0] + b0[0];
          out.y = o4[1] + b0[1];
          out.z = o4[2] + b0[2];
          out.w = o4[3] + b0[3];
          a.t1_next[((size_t)b * nsrc + v) * HW + gy * W + gx] = out;
          ps += (out.x + out.y) + (out.z + out.w);
          pss += (out.x * out.x + out.y * out.y) + (out.z * out.z + out.w * out.w);
        }
      }
      ps = wave_sum(ps);
      pss = wave_sum(pss);
      if (lane == 0) {
        wsum[wave][v][0] = ps;
        wsum[wave][v][1] = pss;
      }
      __syncthreads();   // sq and the ring table are rewritten for the next view
    }
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
  a.off_ow0t = L.ow0t_off;
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
  // the pipeline gathers from the NHWC copies of the features in the workspace
  a.ref = ws.nhwc[0];
  for (int v = 0; v < g.nsrc; ++v) a.src[v] = ws.nhwc[1 + v];
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
  const int ntiles = ((g.W + kPipeTW - 1) / kPipeTW) * ((g.H + kPipeTH - 1) / kPipeTH);
  hipError_t e;
  {
    ProfScope ps(s, K_COST_PIPE);
    hipLaunchKernelGGL(cost_pipe_kernel<kPipeTH>, dim3(ntiles, g.B), dim3(kPipeThreads), 0, s, a,
                       a.params, a.rel);
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

// NCHW [B][32][HW] -> NHWC [B][HW][32] (once per sweep, so that a bilinear tap is one
// 128-B line).  64 pixels per block through LDS: coalesced reads and 16-B writes.
__global__ void __launch_bounds__(256) nchw_to_nhwc_kernel(const float* __restrict__ src,
                                                           float* __restrict__ dst, int HW) {
  __shared__ float t[kC][65];
  const int b = blockIdx.y, p0 = blockIdx.x * 64;
  const float* s = src + (size_t)b * kC * HW;
  float* d = dst + (size_t)b * kC * HW;
  const int px = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = (threadIdx.x >> 6) + 4 * j;
    t[c][px] = p0 + px < HW ? s[(size_t)c * HW + p0 + px] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + 256 * j, q = idx >> 3, c4 = idx & 7;
    if (p0 + q < HW)
      reinterpret_cast<float4*>(d)[(size_t)(p0 + q) * 8 + c4] =
          make_float4(t[4 * c4][q], t[4 * c4 + 1][q], t[4 * c4 + 2][q], t[4 * c4 + 3][q]);
  }
}

hipError_t launch_to_nhwc(const float* src, float* dst, int B, int HW, hipStream_t s) {
  ProfScope ps(s, K_TO_NHWC);
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3((HW + 63) / 64, B), dim3(256), 0, s, src, dst, HW);
  return hipGetLastError();
}

}  // namespace aarmvs
