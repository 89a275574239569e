// Homography warp, inter-view adaptive aggregation (omega) and the per-plane cost
// slice for gfx950.
//
// Reference: models/module.py:6-38 (homo_warping_depthwise),
//            models/drmvsnet.py:27-38 (InterViewAAModule), :307-319 (accumulation).
//
// Per plane and batch element the cost slice needs three grid-wide GroupNorm
// reductions per source view.  The slices do not depend on the recurrence, so
// they are computed a plane group at a time (kPlaneGroup): one omega conv launch over the
// group's planes, two statistics launches over its 16-B/px/view omega conv output (each
// statistic reduced in a fixed order), then one cost_x launch writing the group's slices.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cstdlib>
#include <cstring>

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
// Backward of the warp w.r.t. the source features (aarmvs_homo_warp_backward, the gradient of
// grid_sample at module.py:36): a scatter-add of the output gradient into the four bilinear
// taps, many reference pixels into one source pixel.  fp32 atomics would make each sum depend on
// the order the atomics are served in, so the sums are formed in 64-bit fixed point instead
// (integer adds are associative: bit-reproducible), as the sweep's own dL/dsrc (cbw_feat):
//   1. warp_bwd_max: max |grad_out| per batch element (float bits, order-independent max; a NaN
//      counts as +inf);
//   2. warp_bwd_scatter: each contribution wt * g scaled by 2^k_b (exact) and rounded to an
//      integer, k_b such that any source pixel's total (<= HW max|g|: the bilinear weights of
//      one reference pixel sum to <= 1) stays below 2^61; quantum 2^-k_b ~ HW max|g| 2^-62;
//   3. warp_bwd_fold: grad_src += (float)(sum 2^-k_b), one rounding.
// A batch element whose grad_out holds a NaN or an infinity has no fixed-point scale: its
// contributions go to grad_src as fp32 atomics, which carry the NaN / infinity to exactly the
// source pixels grid_sample's backward carries them to, and leave the others finite (not
// bit-reproducible, like the reference's own scatter); the fold skips it.
// Batch elements are processed 64 at a time.  Workspace: 64 exponents' source words (256 B) +
// [min(B, 64)][C][HW] int64 accumulators (zeroed here per chunk of batch elements).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) warp_bwd_max_kernel(const float* __restrict__ gout, size_t n_per_b,
                                                           unsigned* __restrict__ gmax) {
  const int b = blockIdx.y;
  const float* g = gout + (size_t)b * n_per_b;
  float m = 0.f;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n_per_b; i += (size_t)gridDim.x * 256) {
    const float v = fabsf(g[i]);
    m = (v > m || v != v) ? (v != v ? INFINITY : v) : m;
  }
  const int w = wave_reduce_i32(__float_as_int(m), 0, [](int x, int y) { return x > y ? x : y; });
  if ((threadIdx.x & 63) == 0 && (unsigned)w > __hip_atomic_load(gmax + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(gmax + b, (unsigned)w);
}

// the fixed-point exponent of a batch element; false: its grad_out is not finite
__device__ __forceinline__ bool warp_bwd_exp(unsigned maxbits, int HW, int& k) {
  const float mx = __uint_as_float(maxbits);
  k = 0;
  if (!(mx <= FLT_MAX)) return false;
  const double tot = (double)mx * (double)HW;
  if (!(tot > 0.0)) return true;
  const int kk = 61 - ilogb(tot) - 1;
  k = kk > 120 ? 120 : (kk < -120 ? -120 : kk);
  return true;
}

__global__ void __launch_bounds__(256) homo_warp_bwd_kernel(const float* __restrict__ gout,
                                                            const float* __restrict__ rel,
                                                            const float* __restrict__ depth,
                                                            const unsigned* __restrict__ gmax,
                                                            int C, int H, int W,
                                                            unsigned long long* __restrict__ acc,
                                                            float* __restrict__ gsrc) {
  const int b = blockIdx.y;
  const int HW = H * W;
  const float* m = rel + 12 * b;
  const float dep = depth[b];
  int k;
  const bool fixed = warp_bwd_exp(gmax[b], HW, k);
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    float ix, iy;
    sample_pos(m, dep, (float)(p % W), (float)(p / W), H, W, ix, iy);
    const Taps t = make_taps(ix, iy, H, W);
    const float* g = gout + (size_t)b * C * HW + p;
    unsigned long long* s = acc + (size_t)b * C * HW;
    float* gs = gsrc + (size_t)b * C * HW;
    for (int c = 0; c < C; ++c) {
      const float gv = g[(size_t)c * HW];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (t.ok[q]) {
          if (fixed) {
            const long long f = (long long)rint(ldexp((double)(t.wt[q] * gv), k));
            if (f != 0) atomicAdd(s + (size_t)c * HW + t.idx[q], (unsigned long long)f);
          } else {
            atomicAdd(gs + (size_t)c * HW + t.idx[q], t.wt[q] * gv);
          }
        }
    }
  }
}

__global__ void __launch_bounds__(256) warp_bwd_fold_kernel(const unsigned long long* __restrict__ acc,
                                                            const unsigned* __restrict__ gmax, size_t n_per_b,
                                                            int HW, float* __restrict__ gsrc) {
  const int b = blockIdx.y;
  int k;
  if (!warp_bwd_exp(gmax[b], HW, k)) return;   // non-finite grad_out: scattered in fp32
  const unsigned long long* a = acc + (size_t)b * n_per_b;
  float* o = gsrc + (size_t)b * n_per_b;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n_per_b; i += (size_t)gridDim.x * 256) {
    const long long q = (long long)a[i];
    if (q != 0) o[i] += (float)ldexp((double)q, -k);
  }
}

constexpr int kWarpBwdChunk = 64;   // batch elements per pass (the 256-B exponent header)

size_t homo_warp_bwd_workspace_bytes(int B, int C, int H, int W) {
  return 256 + (size_t)std::min(B, kWarpBwdChunk) * C * H * W * 8;
}

hipError_t launch_homo_warp_bwd(const float* gout, const float* rel, const float* depth, int B,
                                int C, int H, int W, float* gsrc, void* workspace, hipStream_t s) {
  const int HW = H * W;
  const size_t nb = (size_t)C * HW;
  unsigned* gmax = static_cast<unsigned*>(workspace);
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(static_cast<char*>(workspace) + 256);
  ProfScope ps(s, K_WARP);
  hipError_t e = hipSuccess;
  for (int b0 = 0; b0 < B; b0 += kWarpBwdChunk) {
    const int nbt = std::min(B - b0, kWarpBwdChunk);
    if ((e = hipMemsetAsync(workspace, 0, homo_warp_bwd_workspace_bytes(nbt, C, H, W), s)) != hipSuccess)
      return e;
    const float* go = gout + (size_t)b0 * nb;
    float* gsb = gsrc + (size_t)b0 * nb;
    const unsigned gb = (unsigned)std::min<size_t>((nb + 255) / 256, 1024);
    hipLaunchKernelGGL(warp_bwd_max_kernel, dim3(gb, nbt), dim3(256), 0, s, go, nb, gmax);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    dim3 grid((unsigned)std::min((HW + 255) / 256, 4096), (unsigned)nbt);
    hipLaunchKernelGGL(homo_warp_bwd_kernel, grid, dim3(256), 0, s, go, rel + 12 * (size_t)b0, depth + b0,
                       gmax, C, H, W, acc, gsb);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(warp_bwd_fold_kernel, dim3(gb, nbt), dim3(256), 0, s, acc, gmax, nb, HW, gsb);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return e;
}

// ---------------------------------------------------------------------------
// Cost-slice stage, per plane group d0 .. d0 + n - 1 (launch_omega_group, launch_cost_x_group):
//   omega_conv         sq_v(d) = (warp_v(d) - ref)^2 on a haloed tile in LDS, the omega
//                      conv3x3 32->4 -> t1_d (16 B/px/view), GN #0 partial sums;
//   omega_stats<1>/<2> GN #1/#2 partial sums from t1_d alone (each followed by a fixed-order
//                      stat_reduce);
//   cost_x             x_d = -(sum_v (1 + w_v) (warp_v(d) - ref)^2) / nsrc, with w_v from
//                      t1_d and plane d's three GroupNorm statistics (drmvsnet.py:307-319).
// Both gather their bilinear taps straight from the "c8" feature copies
// ([B][4][H][W][8], to_c8_kernel): one tap of one 8-channel chunk is a 32-B segment,
// and neighbouring output pixels share taps in L1/L2.
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
  float* x;                   // [B,H,W,32] (NHWC)
  float* omega_out;           // [nsrc,B,H,W] (prev plane) or null
  const float* params;
  size_t off_owb_scale;            // the omega conv fragments' scale
  size_t off_owm, off_owm_scale;   // omega_mfma's 32x32x16 fragments, their scale
  size_t off_ow0t, off_ow0, off_ob0, off_og0w, off_og0b, off_ow1, off_ob1, off_og1w, off_og1b, off_ow2,
      off_ob2, off_og2w, off_og2b, off_owo, off_obo;
  int B, H, W, nsrc;
  int box_cap;                // LDS source-box capacity in pixels (diagnostic override, <= the kernel's)
  // plane batching: one launch covers planes d .. d + npl - 1 (d = d_prev or d_next), plane
  // k's t1 / statistics / x at k times these strides from the plane-0 pointers
  int npl;
  size_t t1_kstride;          // float4s
  size_t st_kstride;          // doubles
  size_t x_kstride;           // floats
  int omega_k;                // cost_x: the plane (0 .. npl-1) whose omega weights go to omega_out
  // GroupNorm partial sums: one (sum, sumsq) per producing block, [npl][B][nsrc][part_n],
  // reduced in a fixed order by stat_reduce_kernel (deterministic statistics, independent of
  // the launch's grouping and of block timing)
  double* part;
  int part_n;
  int omega_ipb;              // omega_mfma: items per block (AARMVS_OMEGA_IPB, default 1)
};

template <typename PA>
__device__ __forceinline__ void part_put(PA& a, int kp, int b, int v, int i, double s,
                                         double ss) {
  const size_t k = (((size_t)kp * a.B + b) * a.nsrc + v) * a.part_n + i;
  a.part[2 * k] = s;
  a.part[2 * k + 1] = ss;
}

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
__device__ __forceinline__ float omega_weight(const float4 q, const GnStat* gs, const OmegaP& o) {
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

// omega_conv tiles are 32 pixels wide, 16 rows (one thread per pixel).
constexpr int kTileW = 32, kTileH = 16, kTileThreads = kTileW * kTileH;
constexpr int kTileWaves = kTileThreads / 64;

// XCD-aware tile order: blocks are dealt to the 8 XCDs round-robin, so XCD k takes the
// k-th contiguous band of tiles and neighbouring tiles (which share source rows) share
// its L2
__device__ __forceinline__ int xcd_tile(int bid, int nb) {
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// A sampling position reduced to what the taps need: the top-left tap's floor
// coordinates and the four bilinear weights (make_taps' arithmetic).
struct TapF {
  float xf, yf;
  float wt[4];
};

__device__ __forceinline__ TapF tap_f(const float* __restrict__ m, float dep, int x, int y, int H,
                                      int W) {
  float ix, iy;
  sample_pos(m, dep, (float)x, (float)y, H, W, ix, iy);
  TapF t;
  t.xf = floorf(ix);
  t.yf = floorf(iy);
  const float wx = __fsub_rn(ix, t.xf), wy = __fsub_rn(iy, t.yf);
  const float ex = __fsub_rn(1.0f, wx), sy = __fsub_rn(1.0f, wy);
  t.wt[0] = __fmul_rn(sy, ex);
  t.wt[1] = __fmul_rn(sy, wx);
  t.wt[2] = __fmul_rn(wy, ex);
  t.wt[3] = __fmul_rn(wy, wx);
  return t;
}

// Source box of a block: the bounding box of every in-image bilinear tap its threads
// need.  Each thread extends (lx, ly, hx, hy) by its positions, then box_reduce()
// combines the block (one barrier) and returns the box in wave-uniform registers.
__device__ __forceinline__ void box_extend(const TapF& t, int H, int W, int& lx, int& ly, int& hx,
                                           int& hy) {
  if (!(t.xf == t.xf) || !(t.yf == t.yf)) return;   // NaN position: all taps read zero
  const float xl = fmaxf(t.xf, 0.f), xh = fminf(t.xf + 1.f, (float)(W - 1));
  const float yl = fmaxf(t.yf, 0.f), yh = fminf(t.yf + 1.f, (float)(H - 1));
  if (xl <= xh && yl <= yh) {
    lx = min(lx, (int)xl);
    hx = max(hx, (int)xh);
    ly = min(ly, (int)yl);
    hy = max(hy, (int)yh);
  }
}

struct Box {
  int x0, y0, nx, ny;
};

// red: LDS scratch [NW][4] (NW: the block's waves); must not be read by anyone before the
// barrier here
template <int NW = kTileWaves>
__device__ __forceinline__ Box box_reduce(int lx, int ly, int hx, int hy, int (*red)[4]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  auto mn = [](int a, int b) { return min(a, b); };
  auto mx = [](int a, int b) { return max(a, b); };
  lx = wave_reduce_i32(lx, INT_MAX, mn);
  ly = wave_reduce_i32(ly, INT_MAX, mn);
  hx = wave_reduce_i32(hx, INT_MIN, mx);
  hy = wave_reduce_i32(hy, INT_MIN, mx);
  if (lane == 0) {
    red[wave][0] = lx;
    red[wave][1] = ly;
    red[wave][2] = hx;
    red[wave][3] = hy;
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    lx = min(lx, red[w][0]);
    ly = min(ly, red[w][1]);
    hx = max(hx, red[w][2]);
    hy = max(hy, red[w][3]);
  }
  Box bx;
  bx.x0 = __builtin_amdgcn_readfirstlane(lx);
  bx.y0 = __builtin_amdgcn_readfirstlane(ly);
  bx.nx = __builtin_amdgcn_readfirstlane(hx >= lx ? hx - lx + 1 : 0);
  bx.ny = __builtin_amdgcn_readfirstlane(hy >= ly ? hy - ly + 1 : 0);
  return bx;
}

// row of box pixel p: umulhi(p, ceil(2^32 / nx)), exact for p, nx < 2^16
// ceil(2^32 / nx) = floor((2^32 - 1) / nx) + 1: a 32-bit division (the 64-bit form cost ~110
// scalar instructions per omega item)
__device__ __forceinline__ uint32_t box_magic(int nx) {
  return nx > 1 ? 0xFFFFFFFFu / (uint32_t)nx + 1u : 0u;
}
__device__ __forceinline__ int box_row(int p, int nx, uint32_t mg) {
  return nx > 1 ? (int)__umulhi((uint32_t)p, mg) : p;
}

// The four taps of a position: pixel indices (into the LDS box, or image pixels for
// the global path) and weights; out-of-image taps get `zpix` (the box's zero pixel, or
// a pixel index whose byte offset lies past the buffer: loads 0).
struct TapP {
  uint32_t pix[4];
  float wt[4];
};

__device__ __forceinline__ TapP tap_p(const TapF& t, bool valid, int H, int W, bool lds,
                                      const Box& bx, uint32_t zpix) {
  TapP o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    o.wt[k] = t.wt[k];
    const float xf = t.xf + (float)(k & 1), yf = t.yf + (float)(k >> 1);
    const bool ok = valid && (xf > -1.0f) && (xf < (float)W) && (yf > -1.0f) && (yf < (float)H);
    const int xi = ok ? (int)xf : bx.x0, yi = ok ? (int)yf : bx.y0;
    // 24-bit multiplies (full rate): coordinates and extents are < 2^24
    const uint32_t p = lds ? __umul24((uint32_t)(yi - bx.y0), (uint32_t)bx.nx) + (uint32_t)(xi - bx.x0)
                           : __umul24((uint32_t)yi, (uint32_t)W) + (uint32_t)xi;
    o.pix[k] = ok ? p : zpix;
  }
  return o;
}

__device__ __forceinline__ TapP tap_p4(const TapF& t, bool valid, int H, int W, bool lds,
                                      const Box& bx, uint32_t zpix) {
  TapP o;
#pragma unroll
  for (int k = 0; k < 4; ++k) o.wt[k] = t.wt[k];
  // tap_p's result (omega_mfma): the four taps' validity from two column and two row tests (make_taps' tests on the same
  // float coordinates), and their indices from the top-left one: one signed 24-bit multiply
  // (a tap row or column may be -1; coordinates and extents are < 2^23 wherever a tap is
  // valid, and an invalid tap's index is selected away)
  const float xf1 = t.xf + 1.0f, yf1 = t.yf + 1.0f;
  const bool cx0 = t.xf > -1.0f && t.xf < (float)W, cx1 = xf1 > -1.0f && xf1 < (float)W;
  const bool cy0 = valid && t.yf > -1.0f && t.yf < (float)H;
  const bool cy1 = valid && yf1 > -1.0f && yf1 < (float)H;
  const int ox = lds ? bx.x0 : 0, oy = lds ? bx.y0 : 0, rs = lds ? bx.nx : W;
  const int p00 = __mul24((int)t.yf - oy, rs) + ((int)t.xf - ox);
  o.pix[0] = cy0 && cx0 ? (uint32_t)p00 : zpix;
  o.pix[1] = cy0 && cx1 ? (uint32_t)(p00 + 1) : zpix;
  o.pix[2] = cy1 && cx0 ? (uint32_t)(p00 + rs) : zpix;
  o.pix[3] = cy1 && cx1 ? (uint32_t)(p00 + rs + 1) : zpix;
  return o;
}

__device__ __forceinline__ float bil1(float v0, float v1, float v2, float v3, const TapP& t) {
  return __fmaf_rn(v3, t.wt[3], __fmaf_rn(v2, t.wt[2], __fmaf_rn(v1, t.wt[1], __fmul_rn(v0, t.wt[0]))));
}

// the fma chain of bilinear() on 4 channels
__device__ __forceinline__ float4 bil4(float4 v0, float4 v1, float4 v2, float4 v3, const TapP& t) {
  return make_float4(bil1(v0.x, v1.x, v2.x, v3.x, t), bil1(v0.y, v1.y, v2.y, v3.y, t),
                     bil1(v0.z, v1.z, v2.z, v3.z, t), bil1(v0.w, v1.w, v2.w, v3.w, t));
}

__device__ __forceinline__ float4 sqdiff4(float4 g, float4 r) {
  const float dx = __fsub_rn(g.x, r.x), dy = __fsub_rn(g.y, r.y);
  const float dz = __fsub_rn(g.z, r.z), dw = __fsub_rn(g.w, r.w);
  return make_float4(__fmul_rn(dx, dx), __fmul_rn(dy, dy), __fmul_rn(dz, dz), __fmul_rn(dw, dw));
}

// 16-B slot s of c8 pixel p (chunk c = s >> 1, half h = s & 1) in global memory
__device__ __forceinline__ float4 ld_c8(__amdgpu_buffer_rsrc_t r, uint32_t p, int s, int HW) {
  return ld4(r, (uint32_t)(s >> 1) * (uint32_t)HW * 32u + p * 32u + 16u * (uint32_t)(s & 1));
}

// sample_pos split over the two lanes of a pixel: lane h computes coordinate h (x for 0,
// y for 1) with exactly sample_pos's operations, and the pair swaps results (DPP
// quad_perm [1,0,3,2]): one numerator division chain per lane instead of two.
__device__ __forceinline__ float swap_pair(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ void sample_pos_pair(const float* __restrict__ m, float depth, float x,
                                                float y, int H, int W, int h, float& ix,
                                                float& iy) {
  auto row = [&](int k) {
    const float rx = __fadd_rn(__fadd_rn(__fmul_rn(m[4 * k + 0], x), __fmul_rn(m[4 * k + 1], y)),
                               m[4 * k + 2]);
    return __fadd_rn(__fmul_rn(rx, depth), m[4 * k + 3]);
  };
  const float ph = h ? row(1) : row(0);
  float z = row(2);
  if (z == 0.0f) z = __fadd_rn(z, 1e-4f);
  const int dim = h ? H : W;
  const float g = __fsub_rn(__fdiv_rn(__fdiv_rn(ph, z), (float)(dim - 1) * 0.5f), 1.0f);
  const float i = __fmaf_rn(__fadd_rn(g, 1.0f), (float)dim * 0.5f, -0.5f);
  const float o = swap_pair(i);
  ix = h ? o : i;
  iy = h ? i : o;
}

// cost_x: x_d on an 8 x 32 tile, two lanes per reference pixel (lane h holds channels
// 8c + 4h .. 8c + 4h + 3 of every chunk c), so that one wave-wide tap load covers 32
// pixels x 32 B of a chunk image: contiguous 1-KiB requests.  The views are
// accumulated in view order in registers.
// XV: bit 2 (the library's) the omega weights split over the lane pair (view v by lane
// v & 1, swapped by DPP) and computed before the view loop: 0.46 vs 0.50 ms per plane;
// bit 1 (microbenchmark variant) the sampling position split over the pair as well
// (sample_pos_pair): no further gain; bits 4 / 8 (microbenchmark) 5 / 6 waves per SIMD
// instead of 4: 0.485 / 0.578 ms (6 spills) vs 0.482 ms, so occupancy is not the limit
// (the measured HBM traffic, 2.1 GB per plane, is close to the algorithmic 1.94 GB).
constexpr int kXRows = 4;   // the library's tile rows (XR): 256-thread blocks (339 vs 347 us with 8)
template <int XV = 0, int XR = kXRows>
__global__ void __launch_bounds__(2 * XR * kTileW)
__attribute__((amdgpu_waves_per_eu((XV & 8) ? 6 : (XV & 4) ? 5 : 4))) cost_x_kernel(PipeArgs a,
                                                              const float* __restrict__ P,
                                                              const float* __restrict__ Rel) {
  __shared__ GnStat gs[AARMVS_MAX_SRC][3];
  const int tid = threadIdx.x, b = blockIdx.y;
  const int H = a.H, W = a.W, HW = H * W, nsrc = a.nsrc;
  // the npl planes of a tile are consecutive blocks of one XCD: their taps share its L2
  const int seq = xcd_tile(blockIdx.x, gridDim.x);
  const int tile = seq / a.npl, kp = seq - tile * a.npl;
  const int tiles_x = (W + kTileW - 1) / kTileW;
  const int h = tid & 1, q = tid >> 1;
  const int gy = (tile / tiles_x) * XR + q / kTileW, gx = (tile % tiles_x) * kTileW + q % kTileW;
  if (tid < 3 * nsrc) {
    const int v = tid / 3, k = tid % 3;
    gs[v][k] = stat_read(a.st_prev + kp * a.st_kstride + st_index(b, v, k, nsrc), 4.0 * HW);
  }
  __syncthreads();
  if (gy >= H || gx >= W) return;
  const float4* __restrict__ t1p = a.t1_prev + kp * a.t1_kstride;
  float* const omega_out = kp == a.omega_k ? a.omega_out : nullptr;
  // parameters come through a __restrict__ argument so that their uniform loads are
  // scalar (s_load) despite the kernel's vector stores
  OmegaP o;
  load_omega(a, P, o);
  const float dep = a.dvals[b * a.D + a.d_prev + kp];
  const uint32_t fbytes = (uint32_t)((size_t)kC * HW * 4);   // one view's c8 image
  const __amdgpu_buffer_rsrc_t rref = uniform_rsrc(a.ref + (size_t)b * kC * HW, fbytes);
  const size_t p = (size_t)gy * W + gx;
  // this lane's half of the reference feature (16 channels), read once for all views
  float4 rf[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) rf[c] = ld_c8(rref, (uint32_t)p, 2 * c + h, HW);
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  // omega weights of all views, each computed by one lane of the pair (view v by lane
  // v & 1) and swapped
  float wv[AARMVS_MAX_SRC];
#pragma unroll
  for (int vp = 0; vp < AARMVS_MAX_SRC; vp += 2) {
    if ((XV & 2) && vp < nsrc) {
      const int vm = min(vp + h, nsrc - 1);
      // 32-bit element offsets (B * nsrc * HW < 2^31, checked on the host): a wave-uniform
      // base (scalar) plus this lane's view step
      const uint32_t p32 = (uint32_t)p, hw = (uint32_t)HW;
      const float w = omega_weight(
          t1p[(uint32_t)(b * nsrc + vp) * hw + (uint32_t)(vm - vp) * hw + p32], gs[vm], o);
      if (omega_out && vp + h < nsrc)
        omega_out[(uint32_t)(vp * a.B + b) * hw + (uint32_t)(h * a.B) * hw + p32] = w;
      const float ws = swap_pair(w);
      wv[vp] = h ? ws : w;
      if (vp + 1 < AARMVS_MAX_SRC) wv[vp + 1] = h ? w : ws;
    }
  }
  for (int v = 0; v < nsrc; ++v) {
    const float* __restrict__ m = Rel + 12 * (v * a.B + b);
    const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(a.src[v] + (size_t)b * kC * HW, fbytes);
    float w;
    if constexpr ((XV & 2) != 0) {
      w = wv[0];
#pragma unroll
      for (int k = 1; k < AARMVS_MAX_SRC; ++k) w = v == k ? wv[k] : w;
    } else {
      w = omega_weight(t1p[((size_t)b * nsrc + v) * HW + p], gs[v], o);
      if (omega_out && h == 0) omega_out[((size_t)v * a.B + b) * HW + p] = w;
    }
    const float wp1 = __fadd_rn(w, 1.0f);
    const Box none{0, 0, 0, 0};
    TapF tf;
    if constexpr ((XV & 1) == 0) {
      tf = tap_f(m, dep, gx, gy, H, W);
    } else {
      float ix, iy;
      sample_pos_pair(m, dep, (float)gx, (float)gy, H, W, h, ix, iy);
      tf.xf = floorf(ix);
      tf.yf = floorf(iy);
      const float wx = __fsub_rn(ix, tf.xf), wy = __fsub_rn(iy, tf.yf);
      const float ex = __fsub_rn(1.0f, wx), sy = __fsub_rn(1.0f, wy);
      tf.wt[0] = __fmul_rn(sy, ex);
      tf.wt[1] = __fmul_rn(sy, wx);
      tf.wt[2] = __fmul_rn(wy, ex);
      tf.wt[3] = __fmul_rn(wy, wx);
    }
    const TapP t = tap_p(tf, true, H, W, false, none, fbytes / 32u);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int s = 2 * c + h;
      const float4 g = bil4(ld_c8(rsrc, t.pix[0], s, HW), ld_c8(rsrc, t.pix[1], s, HW),
                            ld_c8(rsrc, t.pix[2], s, HW), ld_c8(rsrc, t.pix[3], s, HW), t);
      // x accumulation in view order (drmvsnet.py:311-316)
      const float4 sq = sqdiff4(g, rf[c]);
      float* ac = &acc[4 * c];
      ac[0] = __fadd_rn(ac[0], __fmul_rn(wp1, sq.x));
      ac[1] = __fadd_rn(ac[1], __fmul_rn(wp1, sq.y));
      ac[2] = __fadd_rn(ac[2], __fmul_rn(wp1, sq.z));
      ac[3] = __fadd_rn(ac[3], __fmul_rn(wp1, sq.w));
    }
  }
  // NHWC: this lane's channels 8c + 4h .. +3 of pixel p, one 16-B store per chunk
  float* xo = a.x + kp * a.x_kstride + ((size_t)b * HW + p) * kC + 4 * h;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = -1.0f * __fdiv_rn(acc[4 * c + j], (float)nsrc);
    *reinterpret_cast<float4*>(xo + 8 * c) = make_float4(r[0], r[1], r[2], r[3]);
  }
}

// omega_conv LDS images (source box, reference tile, sq tile): 32-B pixels (one chunk),
// the two 16-B halves of pixel p swapped when bit 3 of p is set, so that 16 consecutive
// pixels' reads of one half cover all banks.  Piece i of an image (pixel i >> 1, slot
// i & 1) sits at byte 16 i: images are lane-linear and filled by LDS-DMA.
__device__ __forceinline__ uint32_t img_slot(uint32_t p, int h) {
  return p * 8u + ((uint32_t)(h ^ (int)((p >> 3) & 1u)) << 2);
}
__device__ __forceinline__ float4 img_ld(const float* img, uint32_t p, int h) {
  return *reinterpret_cast<const float4*>(img + img_slot(p, h));
}
__device__ __forceinline__ void img_st(float* img, uint32_t p, int h, float4 v) {
  *reinterpret_cast<float4*>(img + img_slot(p, h)) = v;
}
// the half of pixel p held in slot s of its image: slot ^ swizzle bit
__device__ __forceinline__ int img_half(uint32_t p, int s) { return s ^ (int)((p >> 3) & 1u); }

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

typedef __attribute__((address_space(3))) void* lds_void_ptr;
// LDS-DMA, 16 B per lane: lane l of the wave lands at wave_dst + 16 l (wave_dst uniform);
// an offset past the buffer's range loads zeros.  soff: a wave-uniform byte offset (the chunk's
// plane) in the instruction's scalar offset, so the per-lane offset stays loop-invariant
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, float* wave_dst, uint32_t off,
                                      uint32_t soff = 0) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_ptr)wave_dst, 16, off, soff, 0, 0);
}
// hi = fp16(x) for a pair, lo = fp16(x - hi): the difference on v_fma_mix_f32 straight from
// the packed fp16 hi (x - hi is exact in fp32, so this is the same value as the convert-back
// and subtract it replaces: 4 instructions per pair instead of 6)
__device__ __forceinline__ uint32_t split_pair(float a, float b, uint32_t& lo_bits) {
  const uint32_t hb = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){a, b}, half2_t));
  float la, lb;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(la) : "v"(hb), "v"(a));
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(lb) : "v"(hb), "v"(b));
  lo_bits = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){la, lb}, half2_t));
  return hb;
}
__device__ __forceinline__ void dma_wait() {
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
}


// ---------------------------------------------------------------------------
// omega_mfma: t1 of plane d_next for one (tile, view) per block with the conv3x3 32->4 on
// the matrix cores as a GEMM followed by a shifted gather.
//
// The block owns a haloed 16 x 32 pixel tile (output: its 14 x 30 interior); wave w owns
// haloed rows 2w (lanes 0-31) and 2w+1 (lanes 32-63), one pixel per lane.  Per 8-channel
// chunk the source box arrives in LDS by LDS-DMA (as in omega_conv); each lane samples its
// own pixel (8 channels), forms sq = (warp - ref)^2 (the reference feature straight from
// the c8 image: one pixel per lane, no LDS), and splits sq 2^-e into fp16 hi + lo.  One
// v_permlane32_swap per dword pair turns the 64 lanes' (hi, lo) into the A operands of
// two v_mfma_f32_32x32x16_f16 row groups (rows = the 32 pixels of a haloed row; K =
// [8 ch hi | 8 ch lo]), and
//   Y[px][u, co] += A x [W_hi ; W_hi]  +  A x [W_lo ; 0]  +  A x [W_lo2 ; W_lo]   (u: 8 off-centre taps)
// gives hi W_hi + lo W_hi + hi W_lo + hi W_lo2 + lo W_lo (the split-fp16 product with the weights
// in three fp16 terms, DESIGN.md §Precision: no systematic per-weight error) over
// the 32 N columns (tap slot u, output channel co).  The centre tap stays an fp32 VALU
// chain on the lane's own sq.  After the 4 chunks Y goes to LDS (pixel stride 36 floats:
// conflict-free float4 reads) and each interior pixel sums its 8 neighbours' Y[., u, co].
// sq is staged x 2^-e (e from the sweep's |x| bound, ws.xbound: sq <= 4 max|feature|^2
// <= bound) so that fp16 cannot overflow; the weights carry their own power-of-two scale.
// ---------------------------------------------------------------------------
// TW: haloed tile width (32, or 16 for 256-thread blocks: 4 blocks per CU by LDS instead of 2).
// Lane l of wave w holds haloed pixel 64 w + l = (hy, hx) = ((64 w + l) / TW, (64 w + l) % TW);
// MFMA row group 0 / 1 of the wave is its lanes 0-31 / 32-63.
constexpr int kMTileH = 16;
template <int TW>
struct OmegaTile {
  static constexpr int NT = kMTileH * TW;   // threads = haloed pixels
  static constexpr int OUTH = kMTileH - 2, OUTW = TW - 2;
  static constexpr int BOXPX = 2 * NT;      // LDS source-box capacity (32-B pixels)
  static int tiles(int H, int W) { return ((W + OUTW - 1) / OUTW) * ((H + OUTH - 1) / OUTH); }
  __device__ static int tiles_d(int H, int W) { return ((W + OUTW - 1) / OUTW) * ((H + OUTH - 1) / OUTH); }
};
// the library's tile width (AARMVS_OMEGA_TW = 32: 16 x 32 haloed tiles, 512 threads; A/B builds)
#ifndef AARMVS_OMEGA_TW
#define AARMVS_OMEGA_TW 16
#endif
constexpr int kOmegaTW = AARMVS_OMEGA_TW;

// ABL: ablation bits for the diagnostic harness only (tools/microbench/pipe_bench.cpp; the
// library instantiates ABL = 0): 1 no MFMAs, 2 no box DMA, 4 no box sampling, 8 no reference
// loads, 16 sampling positions without the homography divisions (the own pixel), 32 no Y
// image / gather (t1 from the row sums of the own lanes), 64 no statistics atomics, 128 no
// fragment loads
// BAL: sign-balanced accumulation, for the training sweep only: +9% time
// wave_sum_d (device_common.h) of two values at once, in the same order and so with the same
// result, on DPP moves with an undefined `old` operand: only lane 63's value is used, and every
// lane it depends on is written at every step, so the zero fills of update_dpp are not needed
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64_u(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, ROWS, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ void wave_sum2_d(double& u, double& w) {
  u += dpp_f64_u<0xB1, 0xF>(u);
  w += dpp_f64_u<0xB1, 0xF>(w);
  u += dpp_f64_u<0x4E, 0xF>(u);
  w += dpp_f64_u<0x4E, 0xF>(w);
  u += dpp_f64_u<0x141, 0xF>(u);
  w += dpp_f64_u<0x141, 0xF>(w);
  u += dpp_f64_u<0x140, 0xF>(u);
  w += dpp_f64_u<0x140, 0xF>(w);
  u += dpp_f64_u<0x142, 0xA>(u);
  w += dpp_f64_u<0x142, 0xA>(w);
  u += dpp_f64_u<0x143, 0xC>(u);
  w += dpp_f64_u<0x143, 0xC>(w);
  auto rl = [](double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  };
  u = rl(u);
  w = rl(w);
}

// one (tile, view, plane) item of omega_mfma_kernel (seq: its index in the launch's order)
// OmegaPos: the item's tile (index, row and column of tiles), source view and plane, advanced
// item by item by the kernel (no per-item integer divisions)
struct OmegaPos {
  int tile, ty, tx, v, kp;
};
// The block's GroupNorm partial of an item is summed over the block's waves one item later (by
// thread 0, after the next item's first barrier; the kernel sums the last item's after its
// loop): no barrier of its own.  wsum[par][wave] holds item parity par's wave sums.
template <int NW>
__device__ __forceinline__ void omega_block_sum(const double (*ws)[2], double& s0, double& s1) {
  s0 = 0.0;
  s1 = 0.0;
  for (int w = 0; w < NW; ++w) {
    s0 += ws[w][0];
    s1 += ws[w][1];
  }
}

template <int ABL, int TW, bool BAL, typename PA>
__device__ __forceinline__ void omega_item(PA& a, const float* __restrict__ P,
                                           const float* __restrict__ Rel,
                                           const unsigned* __restrict__ xbound, const OmegaPos ip,
                                           double (*wsum)[OmegaTile<TW>::NT / 64][2], int par,
                                           bool has_prev, const OmegaPos pv) {
  using T = OmegaTile<TW>;
  constexpr int kMThreads = T::NT, kMBoxPx = T::BOXPX, kMOutH = T::OUTH, kMOutW = T::OUTW;
  constexpr int NB = (2 * kMBoxPx + kMThreads - 1) / kMThreads;   // box pieces per thread
  static_assert(TW == 16 || TW == 32, "the row sums shift by DPP along one haloed row");
  // LDS: chunk c's source box and reference pixels, then (after the last chunk) the row-sum
  // images zm, zp (16 B per haloed pixel each)
  constexpr int kRefFl = (kMBoxPx + 1) * 8;
  constexpr int YFL = kRefFl + 2 * kMThreads * 4;
  static_assert(2 * kMThreads * 4 <= YFL, "the row-sum images fit in the box space");
  __shared__ __attribute__((aligned(16))) float smem[YFL];
  float* const box = smem;
  float4* const zms = reinterpret_cast<float4*>(smem);
  float4* const zps = zms + kMThreads;
  __shared__ int red[kMThreads / 64][4];
  int tid;
  asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));   // see omega_mfma_kernel
  const int lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.z;
  const int H = a.H, W = a.W, HW = H * W, nsrc = a.nsrc;
  const int v = ip.v, kp = ip.kp;
  const int y0 = ip.ty * kMOutH, x0 = ip.tx * kMOutW;
  const int hy = tid / TW, hx = tid % TW;   // haloed pixel of this lane
  const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
  const bool in_img = gy >= 0 && gy < H && gx >= 0 && gx < W;
  const bool interior = in_img && hy >= 1 && hy <= kMOutH && hx >= 1 && hx <= kMOutW;
  // chunk c's reference pixels: one 16-B half per lane and DMA, half h of haloed pixel t at
  // rimg[(h NT + t) 4], after the box (conflict-free, lane-linear reads)
  float* const rimg = smem + kRefFl;

  const float dep = a.dvals[b * a.D + a.d_next + kp];
  const float* __restrict__ m = Rel + 12 * (v * a.B + b);
  const uint32_t fbytes = (uint32_t)((size_t)kC * HW * 4);
  const uint32_t cbytes = (uint32_t)HW * 32u;
  const __amdgpu_buffer_rsrc_t rref = uniform_rsrc(a.ref + (size_t)b * kC * HW, fbytes);
  const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(a.src[v] + (size_t)b * kC * HW, fbytes);
  TapF tf{};
  int lx = INT_MAX, ly = INT_MAX, bhx = INT_MIN, bhy = INT_MIN;
  if (in_img) {
    if constexpr ((ABL & 16) != 0) {
      tf.xf = (float)gx + 0.25f * dep * 1e-3f;
      tf.yf = (float)gy;
      tf.wt[0] = tf.wt[1] = tf.wt[2] = tf.wt[3] = 0.25f;
      tf.xf = floorf(tf.xf);
    } else {
      tf = tap_f(m, dep, gx, gy, H, W);
    }
    box_extend(tf, H, W, lx, ly, bhx, bhy);
  }
  const Box bx = box_reduce<kMThreads / 64>(lx, ly, bhx, bhy, red);
  // after box_reduce's barrier: every wave is past the previous item's row-sum reads and wave sums
  if (tid < 8) box[kMBoxPx * 8 + tid] = 0.f;   // the zero pixel
  if (has_prev && tid == 0) {
    double s0, s1;
    omega_block_sum<kMThreads / 64>(wsum[par ^ 1], s0, s1);
    if (!(ABL & 64)) part_put(a, pv.kp, b, pv.v, pv.tile, s0, s1);
  }
  const bool lds = bx.nx * bx.ny <= min(kMBoxPx, a.box_cap);
  const uint32_t zp = lds ? (uint32_t)kMBoxPx : fbytes / 32u;
  TapP tp = tap_p4(tf, in_img, H, W, lds, bx, zp);
  const int items = lds ? bx.nx * bx.ny * 2 : 0;
  const uint32_t mg = box_magic(bx.nx);
  uint32_t boff[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int i = tid + j * kMThreads, p = i >> 1, r = box_row(p, bx.nx, mg);
    const uint32_t gp = __umul24((uint32_t)(bx.y0 + r), (uint32_t)W) + (uint32_t)bx.x0 +
                        ((uint32_t)p - __umul24((uint32_t)r, (uint32_t)bx.nx));
    boff[j] = gp * 32u + 16u * (uint32_t)img_half((uint32_t)p, i & 1);
  }
  const uint32_t rpix = in_img ? (uint32_t)(gy * W + gx) * 32u : fbytes;
  // the wave's LDS destinations in scalar registers (m0 without a readfirstlane per DMA)
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  auto stage = [&](int c) {
    const uint32_t cb = (uint32_t)c * cbytes;
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (!(ABL & 2) && tid + j * kMThreads < items)
        dma16(rsrc, box + (j * kMThreads + wave_s * 64) * 4, boff[j], cb);
    // this lane's reference pixel in the c8 image (past the buffer: zeros)
    if (!(ABL & 8)) {
      dma16(rref, rimg + (wave_s * 64) * 4, rpix, cb);
      dma16(rref, rimg + (kMThreads + wave_s * 64) * 4, rpix + 16u, cb);
    }
  };
  // sq staging scale: bound 2^-e in [2^13, 2^15) (sq <= 4 max|f|^2 <= bound), e even and of
  // either sign, so that fp16 cannot overflow and the lo parts of small sq stay normal numbers.
  // The scale is applied as 2^(-e/2) to the difference: the bilinear weights carry it (the
  // sample is 2^(-e/2) g exactly) and the reference is subtracted by one fma with -2^(-e/2),
  // so sq arrives scaled with no multiply of its own; the centre tap accumulates the scaled sq
  // and is scaled back by 2^e at the end (all exact power-of-two scalings)
  int e = 0;
  {
    const float bound = __uint_as_float(*xbound);
    if (bound > 0.0f) {
      const int k = ilogbf(bound);
      e = k >= 134 ? 120 : (k < -100 ? -114 : k - 14);
      e += e & 1;
    }
  }
  const float dsc = ldexpf(1.0f, -(e / 2));
#pragma unroll
  for (int k = 0; k < 4; ++k) tp.wt[k] = __fmul_rn(tp.wt[k], dsc);
  const float* __restrict__ w0t = P + a.off_ow0t;   // [9][32][4]: centre tap = tap 4
  const half8* __restrict__ owm = reinterpret_cast<const half8*>(P + a.off_owm);
  floatx16 acc0, acc1;   // first written by chunk 0's MFMAs (ABL 1: zero here)
  if constexpr ((ABL & 1) != 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
  }
  float o4[4] = {0.f, 0.f, 0.f, 0.f};

  stage(0);
  dma_wait();
  __syncthreads();
#pragma unroll 1
  for (int c = 0; c < 4; ++c) {
    const float* const bx_c = box;
    // sample the own pixel (8 channels) and form sq
    float4 g0, g1;
    if (ABL & 4) {
      g0 = g1 = make_float4(tp.wt[0], tp.wt[1], tp.wt[2], tp.wt[3]);
    } else if (lds) {
      g0 = bil4(img_ld(bx_c, tp.pix[0], 0), img_ld(bx_c, tp.pix[1], 0), img_ld(bx_c, tp.pix[2], 0),
                img_ld(bx_c, tp.pix[3], 0), tp);
      g1 = bil4(img_ld(bx_c, tp.pix[0], 1), img_ld(bx_c, tp.pix[1], 1), img_ld(bx_c, tp.pix[2], 1),
                img_ld(bx_c, tp.pix[3], 1), tp);
    } else {
      g0 = bil4(ld_c8(rsrc, tp.pix[0], 2 * c, HW), ld_c8(rsrc, tp.pix[1], 2 * c, HW),
                ld_c8(rsrc, tp.pix[2], 2 * c, HW), ld_c8(rsrc, tp.pix[3], 2 * c, HW), tp);
      g1 = bil4(ld_c8(rsrc, tp.pix[0], 2 * c + 1, HW), ld_c8(rsrc, tp.pix[1], 2 * c + 1, HW),
                ld_c8(rsrc, tp.pix[2], 2 * c + 1, HW), ld_c8(rsrc, tp.pix[3], 2 * c + 1, HW), tp);
    }
    // the reference pixel from LDS (DMA'd with the box: a register prefetch carried across
    // the chunk loop cost 16 register copies per chunk)
    const float4 rf0 = *reinterpret_cast<const float4*>(rimg + tid * 4);
    const float4 rf1 = *reinterpret_cast<const float4*>(rimg + (kMThreads + tid) * 4);
    // sq 2^-e: (2^(-e/2) g - 2^(-e/2) r)^2, the difference rounded once as in sqdiff4
    auto dsq = [&](float g, float r) {
      const float dd = __fmaf_rn(r, -dsc, g);
      return __fmul_rn(dd, dd);
    };
    const float sq[8] = {dsq(g0.x, rf0.x), dsq(g0.y, rf0.y), dsq(g0.z, rf0.z), dsq(g0.w, rf0.w),
                         dsq(g1.x, rf1.x), dsq(g1.y, rf1.y), dsq(g1.z, rf1.z), dsq(g1.w, rf1.w)};
    // this chunk's B fragments, issued before the barrier: their L1/L2 latency is hidden
    // behind it and the centre-tap chain (2.5% of the kernel against loading them after;
    // DMA'ing all 12 to LDS once per item instead was 1.8%)
    half8 Bd, Bl, Bl2;
    if constexpr ((ABL & 128) == 0) {
      Bd = owm[(c * 3 + 0) * 64 + lane];
      Bl = owm[(c * 3 + 1) * 64 + lane];
      Bl2 = owm[(c * 3 + 2) * 64 + lane];
    }
    __syncthreads();   // every lane's box and reference reads of chunk c are done
    if (c < 3) stage(c + 1);
    // centre tap (omega.reweight_network.0.0, tap 4) on the own pixel, fp32 (BAL)
    {
      const float* wt = w0t + (4 * kC + 8 * c) * 4;
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int co = 0; co < 4; ++co) o4[co] = fmaf(sq[j], wt[j * 4 + co], o4[co]);
    }
    // split sq 2^-e into fp16 hi + lo.  Out-of-image pixels (the conv's zero padding) already
    // have sq = 0: zero bilinear weights on the box's zero pixel (or past the buffer) and a
    // reference read past the buffer.  Two values per v_cvt_pk_f16_f32.
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) hw[i] = split_pair(sq[2 * i], sq[2 * i + 1], lw[i]);
    // after the swaps, (hw, lw) are the pixel operands of the wave's pixels 0-31 (lanes 0-31 hi,
    // 32-63 lo of pixel lane & 31) and of its pixels 32-63
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto r = __builtin_amdgcn_permlane32_swap(hw[i], lw[i], false, false);
      hw[i] = r[0];
      lw[i] = r[1];
    }
    // BAL: odd chunks accumulate the negated sum (accumulators and A negated), so the matrix
    // cores' downward rounding alternates sign
    if (BAL && (c & 1)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        hw[i] ^= 0x80008000u;
        lw[i] ^= 0x80008000u;
      }
    }
    if (BAL && c > 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc0[r] = -acc0[r];
        acc1[r] = -acc1[r];
      }
    }
    const half8 A0 = __builtin_bit_cast(half8, u32x4{hw[0], hw[1], hw[2], hw[3]});
    const half8 A1 = __builtin_bit_cast(half8, u32x4{lw[0], lw[1], lw[2], lw[3]});
    if constexpr ((ABL & 128) != 0) {
      Bd = A1;
      Bl = A0;
      Bl2 = A1;
    }
    // D^T = W x [sq hi | sq lo]^T: the weight fragments as the A operand, so that a lane holds
    // its pixel's tap slots (rows) rather than a slot's pixels: row r of lane l is slot
    // 2 (r >> 2) + (l >> 5), output channel r & 3 (the row sums below)
    if (!(ABL & 1)) {
      if (c == 0) {   // the accumulators start from the MFMA's inline-zero C operand (no zero fill)
        const floatx16 z = {};
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bd, A0, z, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bd, A1, z, 0, 0, 0);
      } else {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bd, A0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bd, A1, acc1, 0, 0, 0);
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bl, A0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bl, A1, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bl2, A0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(Bl2, A1, acc1, 0, 0, 0);
    } else {
      acc0[0] += (float)A0[0] + (float)Bd[1];
      acc1[0] += (float)A1[0] + (float)Bl[1];
    }
    if (c < 3) {
      dma_wait();
      __syncthreads();   // chunk c+1's box and reference visible
    }
  }
  // The 3x3 conv's off-centre taps as row sums, in registers.  acc0 / acc1 hold the wave's
  // pixels 0-31 / 32-63 (pixel lane & 31 in lanes l and l + 32); register group g (registers
  // 4 g .. 4 g + 3, output channels 0-3) holds tap slot 2 g in lanes 0-31 and 2 g + 1 in lanes
  // 32-63, slots -> taps 0, 6 | 1, 7 | 2, 8 | 3, 5 (pack_omega_conv_kernel): the groups 0-2 are
  // the taps of dx = -1, 0, +1 of row dy = -1 (lanes 0-31) and dy = +1 (lanes 32-63).  A 16-lane
  // DPP row is one haloed row (TW = 16), so the dx neighbours are one lane away:
  //   Z_dy[q] = Y(dy,-1)[q - 1] + Y(dy,0)[q] + Y(dy,+1)[q + 1]          (row_shr / row_shl)
  //   Z_0[q]  = Y(0,-1)[q - 1] + Y(0,+1)[q + 1]
  //   t1[p]   = Z_-1[p - TW] + Z_0[p] + Z_+1[p + TW]                    (via LDS: other waves)
  // (the edge lanes of a row get zeros from the DPP bound: they are halo pixels, never output).
  // TW = 32: a haloed row is a lane half, two DPP rows; wave_shr / wave_shl shift across them,
  // and the lanes a shift carries across a half or the wave's end are halo columns too.
  static constexpr int kShr = TW == 16 ? 0x111 : 0x138, kShl = TW == 16 ? 0x101 : 0x130;
  auto shr1 = [](float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), kShr, 0xF, 0xF, true));
  };
  auto shl1 = [](float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), kShl, 0xF, 0xF, true));
  };
  float zmr[4], zpr[4], z0[4];
#pragma unroll
  for (int co = 0; co < 4; ++co) {
    const float r0 = (shr1(acc0[co]) + acc0[4 + co]) + shl1(acc0[8 + co]);
    const float r1 = (shr1(acc1[co]) + acc1[4 + co]) + shl1(acc1[8 + co]);
    // -> Z_-1 of the wave's pixel `lane` in zmr, Z_+1 in zpr
    const auto zz = __builtin_amdgcn_permlane32_swap(__float_as_uint(r0), __float_as_uint(r1), false, false);
    zmr[co] = __uint_as_float(zz[0]);
    zpr[co] = __uint_as_float(zz[1]);
    // -> tap 3 and tap 5 of pixel `lane`
    const auto t35 = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc0[12 + co]),
                                                      __float_as_uint(acc1[12 + co]), false, false);
    z0[co] = shr1(__uint_as_float(t35[0])) + shl1(__uint_as_float(t35[1]));
  }
  // the row-sum images over the box space: every lane passed chunk 3's box reads before the
  // barrier in the loop
  if constexpr ((ABL & 32) == 0) {
    zms[tid] = make_float4(zmr[0], zmr[1], zmr[2], zmr[3]);
    zps[tid] = make_float4(zpr[0], zpr[1], zpr[2], zpr[3]);
  }
  __syncthreads();
  // GroupNorm partials in fp64 from the first addition on (var = E[x^2] - E[x]^2 cancels)
  double ps = 0.0, pss = 0.0;
  if (interior) {
    float g4[4];
    if constexpr ((ABL & 32) != 0) {
#pragma unroll
      for (int co = 0; co < 4; ++co) g4[co] = (zmr[co] + z0[co]) + zpr[co];
    } else {
      const float4 up = zms[tid - TW], dn = zps[tid + TW];
      g4[0] = (up.x + z0[0]) + dn.x;
      g4[1] = (up.y + z0[1]) + dn.y;
      g4[2] = (up.z + z0[2]) + dn.z;
      g4[3] = (up.w + z0[3]) + dn.w;
    }
    if (BAL) {   // chunk 3 left -sum in the accumulators
#pragma unroll
      for (int co = 0; co < 4; ++co) g4[co] = -g4[co];
    }
    const float pe = ldexpf(1.0f, e);
    const float isc = P[a.off_owm_scale] * pe;
    const float* __restrict__ b0 = P + a.off_ob0;
    float4 out;
    out.x = fmaf(g4[0], isc, o4[0] * pe) + b0[0];
    out.y = fmaf(g4[1], isc, o4[1] * pe) + b0[1];
    out.z = fmaf(g4[2], isc, o4[2] * pe) + b0[2];
    out.w = fmaf(g4[3], isc, o4[3] * pe) + b0[3];
    a.t1_next[kp * a.t1_kstride + ((size_t)b * nsrc + v) * HW + gy * W + gx] = out;
    ps = ((double)out.x + (double)out.y) + ((double)out.z + (double)out.w);
    pss = ((double)out.x * out.x + (double)out.y * out.y) + ((double)out.z * out.z + (double)out.w * out.w);
  }
  wave_sum2_d(ps, pss);
  if (lane == 0) {
    wsum[par][wave][0] = ps;
    wsum[par][wave][1] = pss;
  }
}

// The kernel: a block takes a.omega_ipb consecutive items (omega_ipb()).  A tile's (view, plane)
// items are consecutive on one XCD (xcd_tile): the reference tile, and a view's source box
// across the npl neighbouring planes, come from its L2.
// (AARMVS_OMEGA_WAVES: the minimum waves per SIMD the compiler is held to; A/B builds only)
#ifndef AARMVS_OMEGA_WAVES
#define AARMVS_OMEGA_WAVES 4
#endif
template <int ABL = 0, int TW = kOmegaTW, bool BAL = false>
__global__ void __launch_bounds__(OmegaTile<TW>::NT) __attribute__((amdgpu_waves_per_eu(AARMVS_OMEGA_WAVES)))
omega_mfma_kernel(PipeArgs a, const float* __restrict__ P, const float* __restrict__ Rel,
                  const unsigned* __restrict__ xbound) {
  if (blockDim.x != OmegaTile<TW>::NT) return;   // LDS images are sized for exactly this block
  const int ipb = a.omega_ipb > 1 ? a.omega_ipb : 1;
  const int npl = a.npl, nsrc = a.nsrc;
  const int tiles_x = (a.W + OmegaTile<TW>::OUTW - 1) / OmegaTile<TW>::OUTW;
  const int total = OmegaTile<TW>::tiles_d(a.H, a.W) * nsrc * npl;
  const int seq0 = xcd_tile(blockIdx.x, gridDim.x) * ipb;
  // seq = (tile * nsrc + v) * npl + kp, decomposed once and then advanced
  OmegaPos ip;
  ip.tile = seq0 / (nsrc * npl);
  {
    const int vk = seq0 - ip.tile * (nsrc * npl);
    ip.v = vk / npl;
    ip.kp = vk - ip.v * npl;
    ip.ty = ip.tile / tiles_x;
    ip.tx = ip.tile - ip.ty * tiles_x;
  }
  constexpr int NW = OmegaTile<TW>::NT / 64;
  __shared__ double wsum[2][NW][2];
  OmegaPos pv = ip;
  int it = 0;
#pragma unroll 1
  for (; it < ipb; ++it) {
    if (seq0 + it >= total) break;
    // (no barrier between items: the next item's LDS writes all follow box_reduce's barrier,
    // which every wave reaches after the previous item's last LDS read)
    if (it) {
      pv = ip;
      if (++ip.kp == npl) {
        ip.kp = 0;
        if (++ip.v == nsrc) {
          ip.v = 0;
          ++ip.tile;
          if (++ip.tx == tiles_x) {
            ip.tx = 0;
            ++ip.ty;
          }
        }
      }
    }
    // the item reads the arguments through a pointer the compiler cannot prove invariant
    // across items: otherwise it hoists every argument load out of the loop (SGPR spills)
    uint32_t z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    typedef const __attribute__((address_space(4))) PipeArgs KPipeArgs;
    KPipeArgs& ka = *(KPipeArgs*)((const __attribute__((address_space(4))) char*)&a + z);
    omega_item<ABL, TW, BAL>(ka, P, Rel, xbound, ip, wsum, it & 1, it > 0, pv);
  }
  if (it > 0) {   // the last item's block sum
    __syncthreads();
    if (threadIdx.x == 0) {
      double s0, s1;
      omega_block_sum<NW>(wsum[(it - 1) & 1], s0, s1);
      if (!(ABL & 64)) part_put(a, ip.kp, (int)blockIdx.z, ip.v, ip.tile, s0, s1);
    }
  }
}

// GN #STAGE (1 or 2) partial sums of the omega chain on t1 (plane d_next).
template <int STAGE>
__global__ void __launch_bounds__(256) omega_stats_kernel(PipeArgs a,
                                                          const float* __restrict__ P) {
  __shared__ double red[2 * 4];
  __shared__ GnStat gs[2];
  const int v = blockIdx.y, b = blockIdx.z / a.npl, kp = blockIdx.z - b * a.npl;
  const int HW = a.H * a.W;
  double* const st = a.st_next + kp * a.st_kstride;
  if (threadIdx.x < STAGE)
    gs[threadIdx.x] = stat_read(st + st_index(b, v, threadIdx.x, a.nsrc), 4.0 * HW);
  __syncthreads();
  OmegaP o;
  load_omega(a, P, o);
  const float4* t1 = a.t1_next + kp * a.t1_kstride + ((size_t)b * a.nsrc + v) * HW;
  double part[2] = {0.0, 0.0};   // fp64: var = E[x^2] - E[x]^2 cancels
  // four independent 16-B loads in flight per thread per iteration
  const int gstride = gridDim.x * blockDim.x;
  for (int p0 = blockIdx.x * blockDim.x + threadIdx.x; p0 < HW; p0 += 4 * gstride) {
    float4 qs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + u * gstride;
      qs[u] = p < HW ? t1[p] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
    if (p0 + u * gstride >= HW) break;
    const float4 q = qs[u];
    const float t[4] = {q.x, q.y, q.z, q.w};
    float aa[4], t2[4];
    gn_relu4(t, gs[0], o.g0w, o.g0b, true, aa);
    conv1x1_4(aa, o.w1, o.b1, t2);
    float r[4];
    if constexpr (STAGE == 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c) r[c] = t2[c];
    } else {
      float bb[4];
      gn_relu4(t2, gs[1], o.g1w, o.g1b, true, bb);
      conv1x1_4(bb, o.w2, o.b2, r);
    }
    part[0] += ((double)r[0] + (double)r[1]) + ((double)r[2] + (double)r[3]);
    part[1] += ((double)r[0] * r[0] + (double)r[1] * r[1]) + ((double)r[2] * r[2] + (double)r[3] * r[3]);
    }
  }
  block_sum_d<2>(part, red);
  if (threadIdx.x == 0) part_put(a, kp, b, v, blockIdx.x, part[0], part[1]);
}

// Statistic STAGE of every (plane, batch element, view) of a group from the per-block
// partials: one block per (plane, b, v), each thread a strided sequential sum, then a fixed
// tree; the result goes to slot 0 of the statistic (the other slots stay zero).
__global__ void __launch_bounds__(256) stat_reduce_kernel(PipeArgs a, int stage) {
  __shared__ double red[2][256];
  const int g = blockIdx.x, v = g % a.nsrc, b = (g / a.nsrc) % a.B, kp = g / (a.nsrc * a.B);
  const double* pp = a.part + 2 * (size_t)g * a.part_n;
  double s = 0.0, ss = 0.0;
  for (int i = threadIdx.x; i < a.part_n; i += 256) {
    s += pp[2 * i];
    ss += pp[2 * i + 1];
  }
  red[0][threadIdx.x] = s;
  red[1][threadIdx.x] = ss;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double* st = a.st_next + kp * a.st_kstride + st_index(b, v, stage, a.nsrc);
    st[0] = red[0][0];
    st[1] = red[1][0];
  }
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
  a.box_cap = INT_MAX;
  a.npl = 1;
  a.omega_k = 0;
  a.off_ow0 = L.pk_off[P_OW0];
  a.off_ow0t = L.ow0t_off;
  a.off_owb_scale = L.owb_scale_off;
  a.off_owm = L.owm_off;
  a.off_owm_scale = L.owb_scale_off;
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

// LDS source-box capacity override: AARMVS_PIPE_BOX_CAP=n (pixels) forces smaller boxes,
// i.e. cost_x's region subdivision and omega_conv's global-gather fallback (a diagnostic
// for the parity tests; results are bit-identical)
static int pipe_box_cap() {
  const char* s = std::getenv("AARMVS_PIPE_BOX_CAP");
  return (s && *s) ? std::max(4, std::atoi(s)) : INT_MAX;
}

// omega_mfma items per block: a block walks ipb consecutive (plane) items of one (tile, view),
// so its fixed cost (prologue, box set-up, statistics hand-off) is paid once per ipb items:
// -3..10% omega time at the headline geometry.  Default 4, halved while the
// grid would hold fewer than 8 blocks per CU; AARMVS_OMEGA_IPB=n forces n (results are
// bit-identical for every n: the items' arithmetic does not change).
static int omega_ipb(int items, int cu_count) {
  const char* s = std::getenv("AARMVS_OMEGA_IPB");
  if (s && *s) return std::max(1, std::min(8, std::atoi(s)));
  // 8 items per block where the grid stays >= 8 blocks per CU (round 6, second session: 7.58-7.61
  // against 7.65-7.67 ms per headline launch at 4, profiles/r06s14_omega_ipb.txt)
  int ipb = 8;
  while (ipb > 1 && (items + ipb - 1) / ipb < 8 * std::max(1, cu_count)) ipb >>= 1;
  return ipb;
}

static PipeArgs pipe_args_c8(const CostArgs& ca, const SweepGeom& g, const Workspace& ws) {
  PipeArgs a = pipe_args(ca, g, ws);
  // the pipeline reads the c8 copies of the features in the workspace
  a.ref = ws.feat8[0];
  for (int v = 0; v < g.nsrc; ++v) a.src[v] = ws.feat8[1 + v];
  a.box_cap = pipe_box_cap();
  return a;
}

static void group_strides(PipeArgs& a, const Workspace& ws, int n) {
  a.npl = n;
  a.t1_kstride = ws.t1_plane;
  a.st_kstride = ws.omega_stats_bytes / sizeof(double);
  a.x_kstride = ws.x_plane;
}

hipError_t launch_cost_x_group(const CostArgs& ca, const SweepGeom& g, const Workspace& ws, int d0,
                               int n, float* x0, float* omega_out, int omega_k, hipStream_t s) {
  PipeArgs a = pipe_args_c8(ca, g, ws);
  group_strides(a, ws, n);
  a.d_prev = d0;
  a.d_next = -1;
  a.x = x0;
  a.t1_prev = reinterpret_cast<const float4*>(ws.t1);
  a.st_prev = ws.omega_stats;
  a.omega_out = omega_out;
  a.omega_k = omega_out ? omega_k : -1;
  const int ntiles = ((g.W + kTileW - 1) / kTileW) * ((g.H + kXRows - 1) / kXRows);
  ProfScope ps(s, K_COST_X);
  hipLaunchKernelGGL(cost_x_kernel<2>, dim3(ntiles * n, g.B), dim3(2 * kXRows * kTileW), 0, s, a,
                     a.params, a.rel);
  return hipGetLastError();
}

hipError_t launch_omega_group(const CostArgs& ca, const SweepGeom& g, const Workspace& ws, int d0,
                              int n, hipStream_t s, bool balanced) {
  PipeArgs a = pipe_args_c8(ca, g, ws);
  group_strides(a, ws, n);
  a.d_prev = -1;
  a.d_next = d0;
  a.t1_next = reinterpret_cast<float4*>(ws.t1);
  a.st_next = ws.omega_stats;
  a.part = ws.omega_part;
  hipError_t e;
  const int nred = n * g.B * g.nsrc;   // reduce blocks
  // the group's statistics accumulate from zero
  if ((e = hipMemsetAsync(ws.omega_stats, 0, (size_t)n * ws.omega_stats_bytes, s)) != hipSuccess)
    return e;
  {
    const int ntiles = OmegaTile<kOmegaTW>::tiles(g.H, g.W);
    ProfScope ps(s, K_OMEGA_CONV);
    a.part_n = ntiles;
    a.omega_ipb = omega_ipb(ntiles * g.nsrc * n * g.B, g.cu_count);
    const int nblk = (ntiles * g.nsrc * n + a.omega_ipb - 1) / a.omega_ipb;
    if (balanced)
      hipLaunchKernelGGL((omega_mfma_kernel<0, kOmegaTW, true>), dim3(nblk, 1, g.B),
                         dim3(OmegaTile<kOmegaTW>::NT), 0, s, a, a.params, a.rel, ws.xbound);
    else
      hipLaunchKernelGGL((omega_mfma_kernel<0, kOmegaTW>), dim3(nblk, 1, g.B),
                         dim3(OmegaTile<kOmegaTW>::NT), 0, s, a, a.params, a.rel, ws.xbound);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  {
    ProfScope ps(s, K_STAT_REDUCE);
    hipLaunchKernelGGL(stat_reduce_kernel, dim3(nred), dim3(256), 0, s, a, 0);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // GN #1 / #2 statistics of every plane of the group.  The blocks per (plane, view) must
  // not depend on n: the fp32 per-thread partial sums follow the grid stride, and a plane's
  // statistics are bit-identical however the sweep is grouped or split into d_range calls.
  const int HW = g.H * g.W;
  const int pblk =
      std::max(1, std::min((HW + 1023) / 1024, 8 * g.cu_count / std::max(1, g.B * g.nsrc) + 1));
  a.part_n = pblk;
  {
    ProfScope ps(s, K_OMEGA1);
    hipLaunchKernelGGL(omega_stats_kernel<1>, dim3(pblk, g.nsrc, g.B * n), dim3(256), 0, s, a,
                       a.params);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  {
    ProfScope ps(s, K_STAT_REDUCE);
    hipLaunchKernelGGL(stat_reduce_kernel, dim3(nred), dim3(256), 0, s, a, 1);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  {
    ProfScope ps(s, K_OMEGA2);
    hipLaunchKernelGGL(omega_stats_kernel<2>, dim3(pblk, g.nsrc, g.B * n), dim3(256), 0, s, a,
                       a.params);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  {
    ProfScope ps(s, K_STAT_REDUCE);
    hipLaunchKernelGGL(stat_reduce_kernel, dim3(nred), dim3(256), 0, s, a, 2);
  }
  return hipGetLastError();
}

// NCHW [B][32][HW] -> c8 [B][4][HW][8] (once per sweep): four 8-channel chunk images of
// 32-B pixels.  64 pixels per block through LDS: coalesced reads and 16-B writes.
__global__ void __launch_bounds__(256) nchw_to_c8_kernel(const float* __restrict__ src,
                                                         float* __restrict__ dst, int HW,
                                                         unsigned* __restrict__ xbound) {
  __shared__ float t[kC][65];
  __shared__ float wmax[4];
  const int b = blockIdx.y, p0 = blockIdx.x * 64;
  const float* s = src + (size_t)b * kC * HW;
  float4* d = reinterpret_cast<float4*>(dst + (size_t)b * kC * HW);
  const int px = threadIdx.x & 63;
  float mx = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = (threadIdx.x >> 6) + 4 * j;
    const float v = p0 + px < HW ? s[(size_t)c * HW + p0 + px] : 0.f;
    t[c][px] = v;
    // NaN-propagating max of |v| (a NaN feature forces the largest fp16 guard scale)
    const float av = fabsf(v);
    mx = (av > mx || av != av) ? av : mx;
  }
  if (xbound) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float q = __shfl_xor(mx, o, 64);
      mx = (q > mx || q != q) ? q : mx;
    }
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (xbound && threadIdx.x == 0) {
    float m = 0.f;
    for (int w = 0; w < 4; ++w) m = (wmax[w] > m || wmax[w] != wmax[w]) ? wmax[w] : m;
    const float bound = 8.0f * m * m;   // non-negative: float bits order like unsigned
    const unsigned bits = __float_as_uint(bound != bound ? INFINITY : bound);
    // one address for the whole grid: read first, so that only blocks that raise the bound
    // pay a (serialised) atomic
    if (bits > __hip_atomic_load(xbound, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(xbound, bits);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + 256 * j, ch = idx >> 7, q = (idx & 127) >> 1, h = idx & 1;
    const int c0 = 8 * ch + 4 * h;
    if (p0 + q < HW)
      d[((size_t)ch * HW + p0 + q) * 2 + h] =
          make_float4(t[c0][q], t[c0 + 1][q], t[c0 + 2][q], t[c0 + 3][q]);
  }
}

hipError_t launch_to_c8(const float* src, float* dst, int B, int HW, hipStream_t s,
                        unsigned* xbound) {
  ProfScope ps(s, K_TO_C8);
  hipLaunchKernelGGL(nchw_to_c8_kernel, dim3((HW + 63) / 64, B), dim3(256), 0, s, src, dst, HW,
                     xbound);
  return hipGetLastError();
}

}  // namespace aarmvs

// ===========================================================================
// Backward of the cost-slice stage (the BPTT's drmvsnet.py:307-319 part): from dL/dx of a
// group of planes to the omega.* parameter gradients and dL/d(reference, source features).
//   x = -(1/nsrc) sum_v (1 + w_v) sq_v,  sq_v = (warp_v - ref)^2,  w_v = omega(sq_v)
//   dL/dsq_v = -(1 + w_v)/nsrc dL/dx + conv3x3^T(dL/dt1_v);  dL/dw_v = -(1/nsrc) sum_c dL/dx sq_v
//   omega chain backward (sigmoid, 1x1 conv, ReLU, ResnetBlockGn with three GroupNorm(1,4)
//   backwards, each needing a grid-wide sum per (plane, sample, view))
//   dL/dwarp_v = 2 (warp_v - ref) dL/dsq_v;  dL/dref = -sum_v dL/dwarp_v;
//   dL/dsrc_v = bilinear scatter of dL/dwarp_v (module.py:36: grid_sample's backward).
// The forward's t1 and GroupNorm statistics come from the training record (the forward copies
// them there per group); every pixel's warp, sq and omega chain is recomputed with the
// forward's own arithmetic (same helpers, contraction off), so the ReLU masks are the forward's.
// Stages per group: cbw_chain<1> (dL/dw from the warp, dL/do; GN3 sums), <2> (GN2 sums),
// <3> (GN1 sums), <4> (dL/dt1), each with a fixed-order reduce; cbw_feat (dL/dsq, the
// feature gradients, the conv3x3 weight gradient).  Source gradients are scattered into an
// LDS box per (tile, view) over the group's planes and flushed with global atomics.
// ===========================================================================

namespace aarmvs {

// omega chain of one (pixel, view) with its intermediates (omega_weight's operations)
struct OmegaChain {
  float t[4], v1[4], aa[4], t2[4], v2[4], bb[4], t3[4], g3[4], s3[4], w;
};
__device__ __forceinline__ void omega_chain(const float4 q, const GnStat* gs, const OmegaP& o,
                                            OmegaChain& c) {
  c.t[0] = q.x;
  c.t[1] = q.y;
  c.t[2] = q.z;
  c.t[3] = q.w;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float sc = gs[0].rstd * o.g0w[i];
    const float sh = o.g0b[i] - gs[0].mean * sc;
    c.v1[i] = c.t[i] * sc + sh;
    c.aa[i] = fmaxf(c.v1[i], 0.0f);
  }
  conv1x1_4(c.aa, o.w1, o.b1, c.t2);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float sc = gs[1].rstd * o.g1w[i];
    const float sh = o.g1b[i] - gs[1].mean * sc;
    c.v2[i] = c.t2[i] * sc + sh;
    c.bb[i] = fmaxf(c.v2[i], 0.0f);
  }
  conv1x1_4(c.bb, o.w2, o.b2, c.t3);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float sc = gs[2].rstd * o.g2w[i];
    const float sh = o.g2b[i] - gs[2].mean * sc;
    c.g3[i] = c.t3[i] * sc + sh;
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    c.s3[i] = c.g3[i] + c.aa[i];
    s = fmaf(o.wo[i], fmaxf(c.s3[i], 0.0f), s);
  }
  c.w = sigmoidf_(s + o.bo);
}

struct CbwArgs {
  PipeArgs p;            // forward pipeline arguments (c8 features, rel, depths, params, t1, stats)
  const float* gx;       // [n][B][HW][32] dL/dx of the group's planes
  float* go;             // [n][B][nsrc][HW] dL/do (stage 1 out, later in)
  float* wo;             // [n][B][nsrc][HW] the omega weights w (stage 1 out, for cbw_feat)
  float4* gt1;           // [n][B][nsrc][HW] dL/dt1 (stage 4 out)
  const double* gsum;    // [n][B][nsrc][3][2] GroupNorm backward sums (stage 1: GN3, 2: GN2, 3: GN1)
  double* part;          // [n][B][nsrc][pblk][32] per-block partial sums
  unsigned* gmax;        // float bits: [0] max |dL/dx| (stage 1), [1] max |dL/dt1| (stage 4)
  int d0, pblk;
};

// max |v| of a wave folded into *dst (float bits: non-negative floats order as unsigned; an
// order-independent, hence deterministic, reduction)
__device__ __forceinline__ void wave_absmax_bits(float m, unsigned* dst) {
  const int b = wave_reduce_i32(__float_as_int(m != m ? INFINITY : m), 0,
                                [](int x, int y) { return x > y ? x : y; });
  if ((threadIdx.x & 63) == 0 && (unsigned)b > __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(dst, (unsigned)b);
}

// columns of each stage's partial rows: 0, 1 = the GroupNorm sums of the stage's statistic;
// then parameter-gradient sums (cbw_param_cols)
template <int STAGE>
__global__ void __launch_bounds__(256) cbw_chain_kernel(CbwArgs a, const float* __restrict__ P,
                                                        const float* __restrict__ Rel) {
  constexpr int NCOL = STAGE == 1 ? 15 : STAGE == 4 ? 4 : 30;
  __shared__ double red[NCOL * 4];
  __shared__ GnStat gs[3];
  __shared__ float gm[3][2];   // per statistic: mean(g_xhat), mean(g_xhat xhat)
  const PipeArgs& pa = a.p;
  const int v = blockIdx.y, bk = blockIdx.z, b = bk % pa.B, k = bk / pa.B;
  const int H = pa.H, W = pa.W, HW = H * W, nsrc = pa.nsrc;
  const size_t kbv = ((size_t)k * pa.B + b) * nsrc + v;
  if (threadIdx.x < 3)
    gs[threadIdx.x] = stat_read(pa.st_prev + k * pa.st_kstride + st_index(b, v, threadIdx.x, nsrc), 4.0 * HW);
  if (threadIdx.x >= 32 && threadIdx.x < 38) {
    const int i = threadIdx.x - 32;   // statistic 2 - (i >> 1)... (GN3 = stat 2, GN2 = 1, GN1 = 0)
    const int st = i >> 1;
    gm[st][i & 1] = (float)(a.gsum[kbv * 6 + 2 * st + (i & 1)] / (4.0 * HW));
  }
  __syncthreads();
  OmegaP o;
  load_omega(pa, P, o);
  double s[NCOL];   // fp64: the parameter gradients are long cancelling sums
#pragma unroll
  for (int i = 0; i < NCOL; ++i) s[i] = 0.0;
  const float* m = Rel + 12 * (v * pa.B + b);
  const float dep = pa.dvals[b * pa.D + a.d0 + k];
  const uint32_t fbytes = (uint32_t)((size_t)kC * HW * 4);
  const __amdgpu_buffer_rsrc_t rref = uniform_rsrc(pa.ref + (size_t)b * kC * HW, fbytes);
  const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(pa.src[v] + (size_t)b * kC * HW, fbytes);
  const float4* t1p = pa.t1_prev + k * pa.t1_kstride + ((size_t)b * nsrc + v) * HW;
  float* gop = a.go + kbv * HW;
  float amax = 0.f;   // stage 1: max |dL/dx|, stage 4: max |dL/dt1| (the dL/dsrc fixed-point scale)
  for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += gridDim.x * 256) {
    OmegaChain c;
    omega_chain(t1p[p], gs, o, c);
    float g_o;
    if constexpr (STAGE == 1) {
      // dL/dw = -(1/nsrc) sum_c dL/dx sq (the warp and sq recomputed as cost_x does)
      const int x = p % W, y = p / W;
      const TapF tf = tap_f(m, dep, x, y, H, W);
      const Box none{0, 0, 0, 0};
      const TapP t = tap_p(tf, true, H, W, false, none, fbytes / 32u);
      const float* gxp = a.gx + (((size_t)k * pa.B + b) * HW + p) * kC;
      float dw = 0.f;
#pragma unroll
      for (int sl = 0; sl < 8; ++sl) {
        const float4 g = bil4(ld_c8(rsrc, t.pix[0], sl, HW), ld_c8(rsrc, t.pix[1], sl, HW),
                              ld_c8(rsrc, t.pix[2], sl, HW), ld_c8(rsrc, t.pix[3], sl, HW), t);
        const float4 sq = sqdiff4(g, ld_c8(rref, (uint32_t)p, sl, HW));
        const float4 gg = *reinterpret_cast<const float4*>(gxp + 4 * sl);
        dw += gg.x * sq.x + gg.y * sq.y + gg.z * sq.z + gg.w * sq.w;
        amax = fmaxf(amax, fmaxf(fmaxf(fabsf(gg.x), fabsf(gg.y)), fmaxf(fabsf(gg.z), fabsf(gg.w))));
      }
      dw = -dw / (float)nsrc;
      g_o = dw * c.w * (1.0f - c.w);
      gop[p] = g_o;
      a.wo[kbv * HW + p] = c.w;
    } else {
      g_o = gop[p];
    }
    float g_r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) g_r[i] = c.s3[i] > 0.f ? o.wo[i] * g_o : 0.f;
    // GN3 (statistic 2): y = g3 = gamma xhat + beta, dL/dy = g_r
    float xh3[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xh3[i] = (c.t3[i] - gs[2].mean) * gs[2].rstd;
    if constexpr (STAGE == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gx3 = g_r[i] * o.g2w[i];
        s[0] += gx3;
        s[1] += gx3 * xh3[i];
        s[2 + i] += g_o * fmaxf(c.s3[i], 0.0f);   // Wo
        s[7 + i] += g_r[i] * xh3[i];               // gamma3
        s[11 + i] += g_r[i];                       // beta3
      }
      s[6] += g_o;                                 // bo
      continue;
    }
    float g_t3[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) g_t3[i] = gs[2].rstd * (g_r[i] * o.g2w[i] - gm[2][0] - xh3[i] * gm[2][1]);
    // t3 = W2 bb + b2
    float g_n2[4], xh2[4];
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
      float ga = 0.f;
#pragma unroll
      for (int co = 0; co < 4; ++co) ga = fmaf(o.w2[co * 4 + ci], g_t3[co], ga);
      g_n2[ci] = c.v2[ci] > 0.f ? ga : 0.f;
      xh2[ci] = (c.t2[ci] - gs[1].mean) * gs[1].rstd;
    }
    if constexpr (STAGE == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gx2 = g_n2[i] * o.g1w[i];
        s[0] += gx2;
        s[1] += gx2 * xh2[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) s[2 + i * 4 + j] += g_t3[i] * c.bb[j];   // W2[i][j]
        s[18 + i] += g_t3[i];                                              // b2
        s[22 + i] += g_n2[i] * xh2[i];                                     // gamma2
        s[26 + i] += g_n2[i];                                              // beta2
      }
      continue;
    }
    float g_t2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) g_t2[i] = gs[1].rstd * (g_n2[i] * o.g1w[i] - gm[1][0] - xh2[i] * gm[1][1]);
    // t2 = W1 aa + b1; aa also feeds the residual (r = relu(g3 + aa))
    float g_n1[4], xh1[4];
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
      float ga = g_r[ci];
#pragma unroll
      for (int co = 0; co < 4; ++co) ga = fmaf(o.w1[co * 4 + ci], g_t2[co], ga);
      g_n1[ci] = c.v1[ci] > 0.f ? ga : 0.f;
      xh1[ci] = (c.t[ci] - gs[0].mean) * gs[0].rstd;
    }
    if constexpr (STAGE == 3) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gx1 = g_n1[i] * o.g0w[i];
        s[0] += gx1;
        s[1] += gx1 * xh1[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) s[2 + i * 4 + j] += g_t2[i] * c.aa[j];   // W1[i][j]
        s[18 + i] += g_t2[i];                                              // b1
        s[22 + i] += g_n1[i] * xh1[i];                                     // gamma1
        s[26 + i] += g_n1[i];                                              // beta1
      }
      continue;
    }
    float g_t1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      g_t1[i] = gs[0].rstd * (g_n1[i] * o.g0w[i] - gm[0][0] - xh1[i] * gm[0][1]);
      s[i] += g_t1[i];   // b0
    }
    a.gt1[kbv * HW + p] = make_float4(g_t1[0], g_t1[1], g_t1[2], g_t1[3]);
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(g_t1[0]), fabsf(g_t1[1])), fmaxf(fabsf(g_t1[2]), fabsf(g_t1[3]))));
  }
  if constexpr (STAGE == 1 || STAGE == 4) wave_absmax_bits(amax, a.gmax + (STAGE == 1 ? 0 : 1));
  block_sum_d_store<NCOL>(s, red, a.part + (kbv * a.pblk + blockIdx.x) * 32);
}

// GroupNorm-backward sums per (plane, b, v): columns 0, 1 of the stage's partial rows
__global__ void cbw_gsum_kernel(const double* __restrict__ part, int pblk, double* __restrict__ gsum,
                                int st) {
  const size_t kbv = blockIdx.x;
  const int c = threadIdx.x;
  if (c >= 2) return;
  double s = 0.0;
  for (int i = 0; i < pblk; ++i) s += part[(kbv * pblk + i) * 32 + c];
  gsum[kbv * 6 + 2 * st + c] = s;
}

// parameter columns -> gacc: one block per column, strided per-thread sums then a fixed tree
struct CbwCols {
  int c0, ncol;
  int off[30];   // gacc index of column c0 + j
};
__global__ void __launch_bounds__(256) cbw_param_kernel(const double* __restrict__ part, int nrow,
                                                        CbwCols cols, double* __restrict__ gacc) {
  __shared__ double red[256];
  const int t = threadIdx.x, j = blockIdx.x;
  double s = 0.0;
  for (int r = t; r < nrow; r += 256) s += part[(size_t)r * 32 + cols.c0 + j];
  red[t] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) gacc[cols.off[j]] += red[0];
}

// dL/dsrc in fixed point: the scatter of grid_sample's backward adds contributions from many
// blocks into one source pixel, and fp32 atomics would make the sum depend on their order.  Each
// contribution (an fp32 value, or a block's fp32 register sum over its own gathers, formed in a
// fixed order) is scaled by 2^k (exact) and rounded to a 64-bit integer; integer atomics are
// associative, so the group's sums are bit-reproducible.  k is chosen per group from a bound on
// any source pixel's total (cbw_scale_kernel), so nothing overflows and the fixed-point quantum
// is ~2^-40 of that bound (far below float32's resolution of the values).
__device__ __forceinline__ unsigned long long to_fixed(float v, int k) {
  return (unsigned long long)(long long)rintf(ldexpf(v, k));
}

// k from the group's maxima: |dL/dwarp| = |2 (warp - ref) dL/dsq| <= 4 max|f| (2/nsrc max|dL/dx| +
// 36 max|w0| max|dL/dt1|) =: G (|warp|, |ref| <= max|f| = sqrt(xbound / 8)), every reference pixel
// and plane contributes at most G in total (bilinear weights sum to <= 1), so any source pixel's
// sum over the group is <= HW n G; 2^k HW n G <= 2^61.
__global__ void cbw_scale_kernel(const unsigned* __restrict__ gmax, const unsigned* __restrict__ xbound,
                                 const float* __restrict__ w0, int HW, int n, int nsrc, int* __restrict__ fxk) {
  __shared__ float red[64];
  float mw = 0.f;
  for (int i = threadIdx.x; i < 4 * 32 * 9; i += 64) mw = fmaxf(mw, fabsf(w0[i]));
  red[threadIdx.x] = mw;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 64; ++i) mw = fmaxf(mw, red[i]);
    const double mf = sqrt((double)__uint_as_float(*xbound) / 8.0);
    const double g = 4.0 * mf * (2.0 / nsrc * (double)__uint_as_float(gmax[0]) +
                                 36.0 * (double)mw * (double)__uint_as_float(gmax[1]));
    const double tot = g * (double)HW * (double)n;
    int k = 0;
    if (tot > 0.0 && tot < 1e300) {
      k = 61 - ilogb(tot) - 1;
      k = k > 120 ? 120 : (k < -120 ? -120 : k);
    }
    *fxk = k;
  }
}

// gsrc8 += the group's fixed-point sums (value 2^-k), which are cleared for the next group:
// the groups are folded in their fixed (reverse plane) order
// AARMVS_COH (diagnostic builds only, tools/bwd_nondet.py): the cost-slice backward's reads of
// buffers written by earlier kernels as agent-scope atomic loads, its read-modify-writes as
// agent-scope atomic loads and stores (L2-coherent across XCDs); the library is built with 0
#ifndef AARMVS_COH
#define AARMVS_COH 0
#endif
template <typename T>
__device__ __forceinline__ T coh_ld(const T* p) {
  if constexpr (AARMVS_COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <typename T>
__device__ __forceinline__ void coh_st(T* p, T v) {
  if constexpr (AARMVS_COH) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
__device__ __forceinline__ float4 coh_ld4(const float* p) {
  if constexpr (AARMVS_COH) return make_float4(coh_ld(p), coh_ld(p + 1), coh_ld(p + 2), coh_ld(p + 3));
  else return *reinterpret_cast<const float4*>(p);
}
__global__ void __launch_bounds__(256) cbw_fold_kernel(unsigned long long* __restrict__ g64,
                                                       float* __restrict__ gsrc8, size_t n,
                                                       const int* __restrict__ fxk) {
  const int k = *fxk;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const long long q = (long long)coh_ld(g64 + i);
    if (q != 0) {
      coh_st(gsrc8 + i, coh_ld(gsrc8 + i) + (float)ldexp((double)q, -k));
      coh_st(g64 + i, 0ull);
    }
  }
}

// dL/dsq, the feature gradients and the conv3x3 weight gradient.  Block: a 16 x 16 tile of one
// sample, one source view and one 8-channel chunk, all planes of the group; thread = pixel.
//   dL/dsq = -(1 + w)/nsrc dL/dx + conv3x3^T(dL/dt1)   (this chunk's 8 channels)
//   dL/dwarp = 2 (warp - ref) dL/dsq;  dL/dref -= dL/dwarp (per view, summed in view order by
//   cost_bwd_end: one writer per (view, pixel, channel));
//   dL/dsrc: grid_sample's bilinear scatter of dL/dwarp, done as a gather.  The source box (the
//   bounding box of the tile's taps over the group's planes: corner positions bound them, the
//   plane homography and the position along a depth ray being monotone while z > 0) is owned
//   pixel by pixel by the block's threads, which accumulate in registers over the planes.  Per
//   plane every reference pixel files its index under the box cell of its top-left tap (one
//   integer LDS atomic for the slot); each owned source pixel then reads the cells of its four
//   possible top-left taps and adds wt[corner] * dL/dwarp of the pixels filed there.  After the
//   group the owned pixels are flushed with global atomics (neighbouring tiles' boxes overlap).
//   A cell with more than kFbSlots pixels, a tap outside the box, or a box that does not fit
//   (kFbOwn pixels per thread) uses global atomics directly.  (The LDS box of float atomics this
//   replaces took half of the kernel: 32 ds_add_f32 per pixel and plane.)
//   gW0[co][c][tap] = sum_q dL/dt1[q - off(tap)][co] sq[q][c]: thread t < 252 owns (half of the
//   chunk's channels, tap) pair t % 18 for all four co (16 sums: one float4 read of sq and one of
//   dL/dt1 per 16 FMAs) over the tile pixels q = t / 18 + 14 i; the 14 pixel subsets are summed in
//   order at the end.
constexpr int kFbT = 16, kFbOwn = 3, kFbBoxPx = kFbOwn * 256, kFbCells = 1280, kFbSlots = 2;
constexpr int kWgPairs = 18, kWgSubs = 14;
// LDS scratch of the plane loop (gather cells, filed dL/dwarp and weights), reused after the
// loop for the weight-gradient subset sums
constexpr int kFbGwOff = 0, kFbWtOff = 256 * 32, kFbCntOff = kFbWtOff + 256 * 16,
              kFbLstOff = kFbCntOff + kFbCells * 4, kFbScratch = kFbLstOff + kFbCells * kFbSlots * 2;
static_assert(kFbScratch >= kWgPairs * kWgSubs * 16 * 4, "subset sums fit the scratch");
struct CbfArgs {
  PipeArgs p;
  const float* gx;          // [n][B][HW][32]
  const float4* gt1;        // [n][B][nsrc][HW]
  const float* w;           // [n][B][nsrc][HW] omega weights (cbw_chain<1>'s)
  unsigned long long* gsrc64;   // [nsrc][B][4][HW][8] the group's dL/dsrc (c8 layout) in fixed point
  const int* fxk;           // the fixed-point exponent k: value = integer 2^-k (cbw_scale_kernel)
  float* grefv;             // [nsrc][B][32][HW] dL/dref per view (NCHW) accumulated
  float* wpart;             // [4 chunks][nsrc][B][tiles][288] conv3x3 weight-gradient partials
  int d0, n;
};

#ifndef AARMVS_CBF_MINB
#define AARMVS_CBF_MINB 2
#endif
// diagnostic builds only (tools/cbf_ab.sh): 1 no weight-gradient loop, 2 no scatter, 4 no source
// gathers, 8 no box flush, 16 no conv3x3^T; the library is built with 0
#ifndef AARMVS_CBF_ABL
#define AARMVS_CBF_ABL 0
#endif
__global__ void __launch_bounds__(256, AARMVS_CBF_MINB) cbw_feat_kernel(CbfArgs a, const float* __restrict__ P,
                                                       const float* __restrict__ Rel) {
  __shared__ float4 w0q[9][8];                    // this chunk's conv3x3 weights [tap][c] (co in .xyzw)
  __shared__ float4 gts[18 * 18];                 // dL/dt1 of the haloed tile (one plane)
  __shared__ float4 sq4[256][2];                  // the tile's sq (8 channels)
  __shared__ __attribute__((aligned(16))) char fbs[kFbScratch];
  float4 (*const gwim)[2] = reinterpret_cast<float4 (*)[2]>(fbs + kFbGwOff);   // dL/dwarp (8 ch)
  float4* const wtim = reinterpret_cast<float4*>(fbs + kFbWtOff);              // bilinear weights
  int* const cnt = reinterpret_cast<int*>(fbs + kFbCntOff);   // pixels filed per top-left-tap cell
  unsigned short (*const lst)[kFbSlots] =
      reinterpret_cast<unsigned short (*)[kFbSlots]>(fbs + kFbLstOff);         // their tile indices
  float (*const wsum)[kWgSubs][16] = reinterpret_cast<float (*)[kWgSubs][16]>(fbs);   // after the loop
  __shared__ int bred[4][4];
  __shared__ int bad;
  const PipeArgs& pa = a.p;
  const int tid = threadIdx.x, b = blockIdx.z;
  // one block per (tile, view, chunk), chunk fastest, XCD-aware (xcd_tile): the 4 nsrc blocks
  // of a tile, which read the same dL/dx (and per view the same dL/dt1 halo) lines, and the
  // neighbouring tiles, which share source taps, run together on one XCD's L2
  const int seq = xcd_tile(blockIdx.x, gridDim.x);
  const int tile = seq / (4 * pa.nsrc), vc = seq - tile * (4 * pa.nsrc);
  const int v = vc >> 2, c = vc & 3;
  const int fxk = *a.fxk;
  const int H = pa.H, W = pa.W, HW = H * W, nsrc = pa.nsrc;
  const int tiles_x = (W + kFbT - 1) / kFbT;
  const int tx0 = (tile % tiles_x) * kFbT, ty0 = (tile / tiles_x) * kFbT;
  const int lx = tid & 15, ly = tid >> 4;
  const int x = tx0 + lx, y = ty0 + ly;
  const bool in = x < W && y < H;
  const int p = in ? y * W + x : 0;
  if (tid < 72) {   // raw [co][32][tap]
    const int tap = tid % 9, j = tid / 9;
    const float* w = P + pa.off_ow0 + (8 * c + j) * 9 + tap;
    w0q[tap][j] = make_float4(w[0], w[288], w[576], w[864]);
  }
  if (tid == 0) bad = 0;
  const uint32_t fbytes = (uint32_t)((size_t)kC * HW * 4);
  const __amdgpu_buffer_rsrc_t rref = uniform_rsrc(pa.ref + (size_t)b * kC * HW, fbytes);
  const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(pa.src[v] + (size_t)b * kC * HW, fbytes);
  const float* m = Rel + 12 * (v * pa.B + b);
  const int pair = tid % kWgPairs, sub = tid / kWgPairs;   // weight-gradient role (tid < 252)
  const int pcg = pair / 9, ptap = pair % 9;
  float gref[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float wacc[16];   // [co][4 channels of half pcg]
#pragma unroll
  for (int i = 0; i < 16; ++i) wacc[i] = 0.f;
  const float4 rf0 = in ? ld_c8(rref, (uint32_t)p, 2 * c, HW) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 rf1 = in ? ld_c8(rref, (uint32_t)p, 2 * c + 1, HW) : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  // the source box over the group's planes: tile corners x planes
  int bx0 = INT_MAX, by0 = INT_MAX, bx1 = -1, by1 = -1;
  if (tid < 4 * a.n) {
    const int cx = (tid & 1) ? min(tx0 + kFbT - 1, W - 1) : tx0;
    const int cy = (tid & 2) ? min(ty0 + kFbT - 1, H - 1) : ty0;
    const float dep = pa.dvals[b * pa.D + a.d0 + (tid >> 2)];
    const float zc = (m[8] * (float)cx + m[9] * (float)cy + m[10]) * dep + m[11];
    const TapF tf = tap_f(m, dep, cx, cy, H, W);
    if (!(zc > 0.f) || !(tf.xf == tf.xf) || !(tf.yf == tf.yf) || fabsf(tf.xf) > 1e6f ||
        fabsf(tf.yf) > 1e6f) {
      bad = 1;
    } else {
      bx0 = max(0, (int)tf.xf);
      by0 = max(0, (int)tf.yf);
      bx1 = min(W - 1, (int)tf.xf + 1);
      by1 = min(H - 1, (int)tf.yf + 1);
    }
  }
  const Box bxr = box_reduce<4>(bx0, by0, bx1, by1, bred);
  // cells: top-left tap positions x0 - 1 .. x0 + nx - 1 (and likewise in y), row stride cw
  const int cw = bxr.nx + 1;
  const bool use_box = !bad && bxr.nx > 0 && bxr.ny > 0 && bxr.nx * bxr.ny <= kFbBoxPx &&
                       cw * (bxr.ny + 1) <= kFbCells;
  if (use_box)
    for (int i = tid; i < cw * (bxr.ny + 1); i += 256) cnt[i] = 0;
  float own[kFbOwn][8];   // owned source-box pixels tid + 256 j: dL/dsrc over the group's planes
#pragma unroll
  for (int j = 0; j < kFbOwn; ++j)
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) own[j][ch] = 0.f;
  int mycell = -1;        // the cell this thread's pixel was filed under (reset next plane)
  int obase[kFbOwn];      // cell of owned pixel j's own position (its corner-0 cell), or -1
#pragma unroll
  for (int j = 0; j < kFbOwn; ++j) {
    const int i = tid + 256 * j;
    obase[j] = -1;
    if (use_box && i < bxr.nx * bxr.ny) {
      const int ry = i / bxr.nx, rx = i - ry * bxr.nx;
      obase[j] = (ry + 1) * cw + rx + 1;
    }
  }
  const float* gxb = a.gx + 8 * c;
  // software pipeline: the global operands of plane k + 1 (dL/dt1 halo, t1, dL/dx, the source
  // gathers) are loaded while plane k is computed
  const int hi0 = tid, hi1 = tid + 256;
  auto halo = [&](int i, size_t kbv) {
    const int hy = i / 18, hx = i % 18, gy = ty0 - 1 + hy, gxx = tx0 - 1 + hx;
    return (i < 18 * 18 && gy >= 0 && gy < H && gxx >= 0 && gxx < W)
               ? coh_ld4(reinterpret_cast<const float*>(a.gt1 + kbv * HW + gy * W + gxx))
               : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  float4 nh0, nh1, ngx0, ngx1, ns[4][2];
  float nw = 0.f;
  TapF ntf;
  auto fetch = [&](int k) {
    const size_t kbv = ((size_t)k * pa.B + b) * nsrc + v;
    nh0 = halo(hi0, kbv);
    nh1 = halo(hi1, kbv);
    if (in) {
      nw = coh_ld(a.w + kbv * HW + p);
      const float* gxp = gxb + (((size_t)k * pa.B + b) * HW + p) * kC;
      ngx0 = coh_ld4(gxp);
      ngx1 = coh_ld4(gxp + 4);
      ntf = tap_f(m, pa.dvals[b * pa.D + a.d0 + k], x, y, H, W);
      const Box none{0, 0, 0, 0};
      const TapP t = tap_p(ntf, true, H, W, false, none, fbytes / 32u);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (AARMVS_CBF_ABL & 4) {
          ns[q][0] = ns[q][1] = make_float4(ntf.wt[0], ntf.wt[1], (float)t.pix[q], 0.f);
          continue;
        }
        ns[q][0] = ld_c8(rsrc, t.pix[q], 2 * c, HW);
        ns[q][1] = ld_c8(rsrc, t.pix[q], 2 * c + 1, HW);
      }
    }
  };
  fetch(0);
#pragma unroll 1
  for (int k = 0; k < a.n; ++k) {
    __syncthreads();   // cells zeroed / previous plane's LDS reads done
    gts[hi0] = nh0;
    if (hi1 < 18 * 18) gts[hi1] = nh1;
    if (mycell >= 0) cnt[mycell] = 0;
    mycell = -1;
    __syncthreads();
    const float wk = nw;
    const float4 gx0 = ngx0, gx1 = ngx1;
    const TapF tf = ntf;
    float4 sv4[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sv4[q][0] = ns[q][0];
      sv4[q][1] = ns[q][1];
    }
    if (k + 1 < a.n) fetch(k + 1);
    float sqv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float gw[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (in) {
      const Box none{0, 0, 0, 0};
      const TapP t = tap_p(tf, true, H, W, false, none, fbytes / 32u);
      const float4 g0 = bil4(sv4[0][0], sv4[1][0], sv4[2][0], sv4[3][0], t);
      const float4 g1 = bil4(sv4[0][1], sv4[1][1], sv4[2][1], sv4[3][1], t);
      const float4 s0 = sqdiff4(g0, rf0), s1 = sqdiff4(g1, rf1);
      const float wv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float rv[8] = {rf0.x, rf0.y, rf0.z, rf0.w, rf1.x, rf1.y, rf1.z, rf1.w};
      sqv[0] = s0.x; sqv[1] = s0.y; sqv[2] = s0.z; sqv[3] = s0.w;
      sqv[4] = s1.x; sqv[5] = s1.y; sqv[6] = s1.z; sqv[7] = s1.w;
      const float gxv[8] = {gx0.x, gx0.y, gx0.z, gx0.w, gx1.x, gx1.y, gx1.z, gx1.w};
      const float dsc = -(wk + 1.0f) / (float)nsrc;
      float gsq[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) gsq[j] = dsc * gxv[j];
#pragma unroll 3
      for (int tap = 0; tap < ((AARMVS_CBF_ABL & 16) ? 1 : 9); ++tap) {
        const float4 gt = gts[(ly + 2 - tap / 3) * 18 + lx + 2 - tap % 3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float4 w = w0q[tap][j];
          gsq[j] = fmaf(w.x, gt.x, gsq[j]);
          gsq[j] = fmaf(w.y, gt.y, gsq[j]);
          gsq[j] = fmaf(w.z, gt.z, gsq[j]);
          gsq[j] = fmaf(w.w, gt.w, gsq[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        gw[j] = 2.0f * (wv[j] - rv[j]) * gsq[j];
        gref[j] -= gw[j];
      }
    }
    // grid_sample backward: file the pixel under its top-left tap's cell for the gather below;
    // taps that are never gathered (in-image corners outside the box, every corner of a pixel
    // outside the cells) are scattered with fixed-point global atomics here.  Whether a filed
    // pixel is gathered depends only on its cell's final count (read after the barrier), so the
    // result does not depend on the order the LDS atomics were served in.
    int kx = 0, ky = 0;
    if (in && !(AARMVS_CBF_ABL & 2) && tf.xf == tf.xf && tf.yf == tf.yf) {
      kx = (int)fminf(fmaxf(tf.xf, -8.f), (float)W + 8.f);
      ky = (int)fminf(fmaxf(tf.yf, -8.f), (float)H + 8.f);
      const int cx = kx - bxr.x0 + 1, cy = ky - bxr.y0 + 1;
      if (use_box && cx >= 0 && cx < cw && cy >= 0 && cy <= bxr.ny) {
        const int cell = cy * cw + cx;
        const int slot = atomicAdd(&cnt[cell], 1);
        mycell = cell;
        if (slot < kFbSlots) lst[cell][slot] = (unsigned short)tid;
        gwim[tid][0] = make_float4(gw[0], gw[1], gw[2], gw[3]);
        gwim[tid][1] = make_float4(gw[4], gw[5], gw[6], gw[7]);
        wtim[tid] = make_float4(tf.wt[0], tf.wt[1], tf.wt[2], tf.wt[3]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int xi = kx + (q & 1), yi = ky + (q >> 1);
        if (xi < 0 || xi >= W || yi < 0 || yi >= H) continue;   // zero padding
        const bool inbox = xi >= bxr.x0 && xi < bxr.x0 + bxr.nx && yi >= bxr.y0 && yi < bxr.y0 + bxr.ny;
        if (mycell >= 0 && inbox) continue;
        unsigned long long* gp = a.gsrc64 + ((((size_t)v * pa.B + b) * 4 + c) * HW + (size_t)yi * W + xi) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(gp + j, to_fixed(tf.wt[q] * gw[j], fxk));
      }
    }
    sq4[tid][0] = make_float4(sqv[0], sqv[1], sqv[2], sqv[3]);
    sq4[tid][1] = make_float4(sqv[4], sqv[5], sqv[6], sqv[7]);
    __syncthreads();
    if (tid < kWgPairs * kWgSubs && !(AARMVS_CBF_ABL & 1)) {
      const int dy = ptap / 3, dx = ptap % 3;
#pragma unroll 4
      for (int qq = sub; qq < 256; qq += kWgSubs) {
        const float4 sv = sq4[qq][pcg];
        const float4 gt = gts[((qq >> 4) + 2 - dy) * 18 + (qq & 15) + 2 - dx];
        const float g4[4] = {gt.x, gt.y, gt.z, gt.w}, s4[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
        for (int co = 0; co < 4; ++co)
#pragma unroll
          for (int j = 0; j < 4; ++j) wacc[co * 4 + j] = fmaf(g4[co], s4[j], wacc[co * 4 + j]);
      }
    }
    // a cell holding more than kFbSlots pixels is not gathered: its pixels scatter their in-box
    // corners with the fixed-point atomics
    if (mycell >= 0 && cnt[mycell] > kFbSlots) {
      const float4 wq = wtim[tid], g0 = gwim[tid][0], g1 = gwim[tid][1];
      const float wt4[4] = {wq.x, wq.y, wq.z, wq.w};
      const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int xi = kx + (q & 1), yi = ky + (q >> 1);
        if (xi < 0 || xi >= W || yi < 0 || yi >= H) continue;
        const bool inbox = xi >= bxr.x0 && xi < bxr.x0 + bxr.nx && yi >= bxr.y0 && yi < bxr.y0 + bxr.ny;
        if (!inbox) continue;
        unsigned long long* gp = a.gsrc64 + ((((size_t)v * pa.B + b) * 4 + c) * HW + (size_t)yi * W + xi) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(gp + j, to_fixed(wt4[q] * gv[j], fxk));
      }
    }
    // the gather: owned source pixel s takes corner q of the pixels filed under cell s - q, in
    // ascending tile-index order
    if (use_box && !(AARMVS_CBF_ABL & 2)) {
#pragma unroll
      for (int j = 0; j < kFbOwn; ++j) {
        if (obase[j] < 0) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cell = obase[j] - (q >> 1) * cw - (q & 1);
          const int n = cnt[cell];
          if (n > kFbSlots) continue;
          // ascending tile index by min / max: written for exactly two slots
          static_assert(kFbSlots == 2, "the fixed-order gather below sorts two slots");
          const int l0 = lst[cell][0], l1 = lst[cell][1];
          for (int sl = 0; sl < n; ++sl) {
            const int pp = n == 1 ? l0 : (sl == 0 ? min(l0, l1) : max(l0, l1));
            const float4 wq = wtim[pp];
            const float w = q == 0 ? wq.x : q == 1 ? wq.y : q == 2 ? wq.z : wq.w;
            const float4 g0 = gwim[pp][0], g1 = gwim[pp][1];
            own[j][0] += w * g0.x;
            own[j][1] += w * g0.y;
            own[j][2] += w * g0.z;
            own[j][3] += w * g0.w;
            own[j][4] += w * g1.x;
            own[j][5] += w * g1.y;
            own[j][6] += w * g1.z;
            own[j][7] += w * g1.w;
          }
        }
      }
    }
  }
  if (in) {
    float* gr = a.grefv + ((size_t)v * pa.B + b) * kC * HW + p;
#pragma unroll
    for (int j = 0; j < 8; ++j) coh_st(gr + (size_t)(8 * c + j) * HW, coh_ld(gr + (size_t)(8 * c + j) * HW) + gref[j]);
  }
  __syncthreads();   // every gather of the last plane done: the scratch becomes the subset sums
  if (tid < kWgPairs * kWgSubs) {
#pragma unroll
    for (int i = 0; i < 16; ++i) wsum[pair][sub][i] = wacc[i];
  }
  __syncthreads();
  if (use_box && !(AARMVS_CBF_ABL & 8)) {   // flush the owned box pixels (8 channels each)
    // through LDS (sq4's 8 KB, free after the last plane) so that consecutive lanes add to
    // consecutive channels: a wave-wide atomic covers 8 pixels x 64 B instead of 64 pixels'
    // separate lines
    unsigned long long* gb = a.gsrc64 + (((size_t)v * pa.B + b) * 4 + c) * HW * 8;
    float* fl = reinterpret_cast<float*>(sq4);
    const int nbox = bxr.nx * bxr.ny;
#pragma unroll
    for (int j = 0; j < kFbOwn; ++j) {
      if (256 * j >= nbox) break;   // block-uniform
      if (j > 0) __syncthreads();   // the previous round's reads done
      *reinterpret_cast<float4*>(fl + 8 * tid) = make_float4(own[j][0], own[j][1], own[j][2], own[j][3]);
      *reinterpret_cast<float4*>(fl + 8 * tid + 4) = make_float4(own[j][4], own[j][5], own[j][6], own[j][7]);
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = tid + 256 * k, i = (e >> 3) + 256 * j, ch = e & 7;
        const float val = fl[e];
        if (i < nbox && val != 0.f) {
          const int ry = i / bxr.nx, rx = i - ry * bxr.nx;
          atomicAdd(gb + ((size_t)(bxr.y0 + ry) * W + bxr.x0 + rx) * 8 + ch, to_fixed(val, fxk));
        }
      }
    }
  }
  const int ntiles = tiles_x * ((H + kFbT - 1) / kFbT);
  const size_t blk = (((size_t)c * nsrc + v) * pa.B + b) * ntiles + tile;
  float* wp = a.wpart + blk * 288;
  for (int i = tid; i < 288; i += 256) {   // i = (co * 8 + j) * 9 + tap
    const int tap = i % 9, j = (i / 9) % 8, co = i / 72;
    const int pr = (j >> 2) * 9 + tap, col = co * 4 + (j & 3);
    float sum = wsum[pr][0][col];
#pragma unroll
    for (int k = 1; k < kWgSubs; ++k) sum += wsum[pr][k][col];
    wp[i] = sum;
  }
}

// per chunk c: sum the (view, b, tile) partials in a fixed order -> gW0[co][8c + j][tap], in
// two passes: 64 contiguous segments of the partials (blockIdx.y), then the segments in order.
constexpr int kW0Seg = 64;
__global__ void __launch_bounds__(256) cbw_w0_seg_kernel(const float* __restrict__ wpart, int nblk,
                                                         double* __restrict__ wseg) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 1152) return;
  const int tap = i % 9, cc = (i / 9) % 32, co = i / 288;
  const int c = cc >> 3, j = cc & 7;
  const float* src = wpart + (size_t)c * nblk * 288 + (co * 8 + j) * 9 + tap;
  const int k0 = (int)((long)blockIdx.y * nblk / kW0Seg), k1 = (int)((long)(blockIdx.y + 1) * nblk / kW0Seg);
  double s = 0.0;
  for (int k = k0; k < k1; ++k) s += src[(size_t)k * 288];
  wseg[(size_t)blockIdx.y * 1152 + i] = s;
}

__global__ void __launch_bounds__(256) cbw_w0_reduce_kernel(const double* __restrict__ wseg,
                                                            double* __restrict__ gw) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 1152) return;
  double s = 0.0;
  for (int k = 0; k < kW0Seg; ++k) s += wseg[(size_t)k * 1152 + i];
  gw[i] += s;
}

// dL/dref = sum over views (in view order) of the per-view accumulators
__global__ void __launch_bounds__(256) cbw_ref_sum_kernel(const float* __restrict__ grefv, int nsrc,
                                                          size_t n, float* __restrict__ gref) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    float s = grefv[i];
    for (int v = 1; v < nsrc; ++v) s += grefv[(size_t)v * n + i];
    gref[i] = s;
  }
}

// c8 [B][4][HW][8] -> NCHW [B][32][HW]
__global__ void __launch_bounds__(256) c8_to_nchw_kernel(const float* __restrict__ src,
                                                         float* __restrict__ dst, int HW) {
  const int b = blockIdx.y;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < 32 * HW; i += gridDim.x * 256) {
    const int p = i % HW, ch = i / HW;
    dst[(size_t)b * 32 * HW + i] = src[(((size_t)b * 4 + (ch >> 3)) * HW + p) * 8 + (ch & 7)];
  }
}

// ---- host side ----
struct CostBwdLayout {
  float* go;
  float* wo;
  float4* gt1;
  double* gsum;
  double* part;
  float* wpart;
  double* wseg;
  float* gsrc8;
  float* grefv;
  unsigned long long* gsrc64;   // the current group's dL/dsrc in fixed point (cbw_feat_kernel)
  unsigned* gmax;               // [0] max |dL/dx|, [1] max |dL/dt1| of the group (float bits); then
  int* fxk;                     // the fixed-point exponent
  size_t bytes;
  int pblk, ntiles16;
};

static CostBwdLayout cost_bwd_layout(void* base, int B, int H, int W, int nsrc) {
  CostBwdLayout L{};
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = p ? p + off : nullptr;
    off = (off + bytes + 255) / 256 * 256;
    return r;
  };
  const size_t HW = (size_t)H * W;
  const int G = kPlaneGroup;
  // blocks per (plane, b, view) of the chain kernels: a group launch has G x B x nsrc x pblk
  L.pblk = std::max(1, std::min((int)((HW + 4095) / 4096), 64));
  L.ntiles16 = ((W + kFbT - 1) / kFbT) * ((H + kFbT - 1) / kFbT);
  L.go = reinterpret_cast<float*>(take((size_t)G * B * nsrc * HW * 4));
  L.wo = reinterpret_cast<float*>(take((size_t)G * B * nsrc * HW * 4));
  L.gt1 = reinterpret_cast<float4*>(take((size_t)G * B * nsrc * HW * 16));
  L.gsum = reinterpret_cast<double*>(take((size_t)G * B * nsrc * 6 * 8));
  L.part = reinterpret_cast<double*>(take((size_t)G * B * nsrc * L.pblk * 32 * 8));
  L.wpart = reinterpret_cast<float*>(take((size_t)4 * nsrc * B * L.ntiles16 * 288 * 4));
  L.wseg = reinterpret_cast<double*>(take((size_t)kW0Seg * 1152 * 8));
  L.gsrc8 = reinterpret_cast<float*>(take((size_t)nsrc * B * 32 * HW * 4));
  L.grefv = reinterpret_cast<float*>(take((size_t)nsrc * B * 32 * HW * 4));
  L.gsrc64 = reinterpret_cast<unsigned long long*>(take((size_t)nsrc * B * 32 * HW * 8));
  L.gmax = reinterpret_cast<unsigned*>(take(256));
  L.fxk = reinterpret_cast<int*>(L.gmax ? L.gmax + 4 : nullptr);
  L.bytes = off;
  return L;
}

size_t cost_bwd_scratch_bytes(int B, int H, int W, int nsrc) {
  return cost_bwd_layout(nullptr, B, H, W, nsrc).bytes;
}

static CostArgs cost_args_of(const aarmvs_backward_args* a) {
  CostArgs ca{};
  ca.ref = a->ref_fea;
  for (int v = 0; v < a->nsrc; ++v) ca.src[v] = a->src_fea[v];
  ca.rel = a->rel_proj;
  ca.depth_values = a->depth_values;
  ca.params = static_cast<const float*>(a->packed_params);
  return ca;
}

hipError_t cost_bwd_begin(CostBwdCtx& c, hipStream_t s) {
  const aarmvs_backward_args* a = c.a;
  CostBwdLayout L = cost_bwd_layout(c.scratch, a->B, a->H, a->W, a->nsrc);
  hipError_t e;
  const size_t HW = (size_t)a->H * a->W;
  if ((e = hipMemsetAsync(L.gsrc8, 0, (size_t)a->nsrc * a->B * 32 * HW * 4, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(L.gsrc64, 0, (size_t)a->nsrc * a->B * 32 * HW * 8, s)) != hipSuccess) return e;
  return hipMemsetAsync(L.grefv, 0, (size_t)a->nsrc * a->B * 32 * HW * 4, s);
}

hipError_t cost_bwd_group(void* ctx, int g0, int n, const float* gx, hipStream_t s) {
  CostBwdCtx& c = *static_cast<CostBwdCtx*>(ctx);
  const aarmvs_backward_args* a = c.a;
  const ParamLayout& PL = param_layout();
  CostBwdLayout L = cost_bwd_layout(c.scratch, a->B, a->H, a->W, a->nsrc);
  const SweepGeom g{a->B, a->H, a->W, a->nsrc, a->D, cu_count()};
  const CostArgs ca = cost_args_of(a);
  hipError_t e;
  // the forward's omega conv output and GroupNorm statistics of the group's planes, read where
  // the recorded forward wrote them (the record's per-plane layout is the workspace slots')
  Workspace ws = c.ws;
  ws.t1 = a->record->t1 + (size_t)g0 * c.ws.t1_plane * 4;
  ws.omega_stats = a->record->ostats + (size_t)g0 * (c.ws.omega_stats_bytes / 8);
  CbwArgs ba{};
  ba.p = pipe_args_c8(ca, g, ws);
  group_strides(ba.p, ws, n);
  ba.p.t1_prev = reinterpret_cast<const float4*>(ws.t1);
  ba.p.st_prev = ws.omega_stats;
  ba.gx = gx;
  ba.go = L.go;
  ba.wo = L.wo;
  ba.gt1 = L.gt1;
  ba.gsum = L.gsum;
  ba.part = L.part;
  ba.gmax = L.gmax;
  ba.d0 = g0;
  ba.pblk = L.pblk;
  if ((e = hipMemsetAsync(L.gmax, 0, 8, s)) != hipSuccess) return e;
  const dim3 grid(L.pblk, a->nsrc, a->B * n);
  const int nkbv = n * a->B * a->nsrc, nrow = nkbv * L.pblk;
  auto cols = [&](int c0, std::initializer_list<std::pair<int, int>> ranges) {
    CbwCols cc{};
    cc.c0 = c0;
    int j = 0;
    for (const auto& r : ranges)
      for (int i = 0; i < r.second; ++i) cc.off[j++] = (int)PL.raw_off[r.first] + i;
    cc.ncol = j;
    return cc;
  };
  // stage 1: dL/do, GN3 sums; Wo, bo, gamma3, beta3
  {
    ProfScope ps(s, K_CBW_CHAIN);
    hipLaunchKernelGGL(cbw_chain_kernel<1>, grid, dim3(256), 0, s, ba, ba.p.params, ba.p.rel);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  { ProfScope ps_(s, K_CBW_SMALL);
  hipLaunchKernelGGL(cbw_gsum_kernel, dim3(nkbv), dim3(64), 0, s, L.part, L.pblk, L.gsum, 2);
  }
  {
    const CbwCols cc = cols(2, {{P_OWO, 4}, {P_OBO, 1}, {P_OG2W, 4}, {P_OG2B, 4}});
    { ProfScope ps_(s, K_CBW_SMALL);
    hipLaunchKernelGGL(cbw_param_kernel, dim3(cc.ncol), dim3(256), 0, s, L.part, nrow, cc, c.gacc);
    }
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // stage 2: GN2 sums; W2, b2, gamma2, beta2
  {
    ProfScope ps(s, K_CBW_CHAIN);
    hipLaunchKernelGGL(cbw_chain_kernel<2>, grid, dim3(256), 0, s, ba, ba.p.params, ba.p.rel);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  { ProfScope ps_(s, K_CBW_SMALL);
  hipLaunchKernelGGL(cbw_gsum_kernel, dim3(nkbv), dim3(64), 0, s, L.part, L.pblk, L.gsum, 1);
  }
  {
    const CbwCols cc = cols(2, {{P_OW2, 16}, {P_OB2, 4}, {P_OG1W, 4}, {P_OG1B, 4}});
    { ProfScope ps_(s, K_CBW_SMALL);
    hipLaunchKernelGGL(cbw_param_kernel, dim3(cc.ncol), dim3(256), 0, s, L.part, nrow, cc, c.gacc);
    }
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // stage 3: GN1 sums; W1, b1, gamma1, beta1
  {
    ProfScope ps(s, K_CBW_CHAIN);
    hipLaunchKernelGGL(cbw_chain_kernel<3>, grid, dim3(256), 0, s, ba, ba.p.params, ba.p.rel);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  { ProfScope ps_(s, K_CBW_SMALL);
  hipLaunchKernelGGL(cbw_gsum_kernel, dim3(nkbv), dim3(64), 0, s, L.part, L.pblk, L.gsum, 0);
  }
  {
    const CbwCols cc = cols(2, {{P_OW1, 16}, {P_OB1, 4}, {P_OG0W, 4}, {P_OG0B, 4}});
    { ProfScope ps_(s, K_CBW_SMALL);
    hipLaunchKernelGGL(cbw_param_kernel, dim3(cc.ncol), dim3(256), 0, s, L.part, nrow, cc, c.gacc);
    }
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // stage 4: dL/dt1; b0
  {
    ProfScope ps(s, K_CBW_CHAIN);
    hipLaunchKernelGGL(cbw_chain_kernel<4>, grid, dim3(256), 0, s, ba, ba.p.params, ba.p.rel);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  {
    const CbwCols cc = cols(0, {{P_OB0, 4}});
    { ProfScope ps_(s, K_CBW_SMALL);
    hipLaunchKernelGGL(cbw_param_kernel, dim3(cc.ncol), dim3(256), 0, s, L.part, nrow, cc, c.gacc);
    }
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // dL/dsq -> features, conv3x3 weights
  CbfArgs fa{};
  fa.p = ba.p;
  fa.gx = gx;
  fa.gt1 = L.gt1;
  fa.w = L.wo;
  fa.gsrc64 = L.gsrc64;
  fa.fxk = L.fxk;
  fa.grefv = L.grefv;
  {
    ProfScope ps_(s, K_CBW_SMALL);
    hipLaunchKernelGGL(cbw_scale_kernel, dim3(1), dim3(64), 0, s, L.gmax, c.ws.xbound,
                       ba.p.params + ba.p.off_ow0, a->H * a->W, n, a->nsrc, L.fxk);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  fa.wpart = L.wpart;
  fa.d0 = g0;
  fa.n = n;
  {
    ProfScope ps(s, K_CBW_FEAT);
    hipLaunchKernelGGL(cbw_feat_kernel, dim3(L.ntiles16 * 4 * a->nsrc, 1, a->B), dim3(256), 0, s, fa,
                       ba.p.params, ba.p.rel);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  { ProfScope ps_(s, K_CBW_SMALL);
  hipLaunchKernelGGL(cbw_w0_seg_kernel, dim3(5, kW0Seg), dim3(256), 0, s, L.wpart,
                     a->nsrc * a->B * L.ntiles16, L.wseg);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  { ProfScope ps_(s, K_CBW_SMALL);
  hipLaunchKernelGGL(cbw_w0_reduce_kernel, dim3(5), dim3(256), 0, s, L.wseg, c.gacc + PL.raw_off[P_OW0]);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  {
    const size_t nel = (size_t)a->nsrc * a->B * 32 * a->H * a->W;
    ProfScope ps_(s, K_CBW_SMALL);
    hipLaunchKernelGGL(cbw_fold_kernel, dim3((unsigned)std::min<size_t>(4096, (nel + 255) / 256)), dim3(256), 0, s,
                       L.gsrc64, L.gsrc8, nel, L.fxk);
  }
  }
  return hipGetLastError();
}

hipError_t cost_bwd_end(CostBwdCtx& c, hipStream_t s) {
  const aarmvs_backward_args* a = c.a;
  CostBwdLayout L = cost_bwd_layout(c.scratch, a->B, a->H, a->W, a->nsrc);
  const int HW = a->H * a->W;
  {
    const size_t n = (size_t)a->B * 32 * HW;
    hipLaunchKernelGGL(cbw_ref_sum_kernel, dim3((unsigned)std::min<size_t>(4096, (n + 255) / 256)), dim3(256),
                       0, s, L.grefv, a->nsrc, n, a->grad_ref);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  for (int v = 0; v < a->nsrc; ++v) {
    if (!a->grad_src[v]) continue;
    hipLaunchKernelGGL(c8_to_nchw_kernel, dim3(std::min(4096, (32 * HW + 255) / 256), a->B), dim3(256), 0, s,
                       L.gsrc8 + (size_t)v * a->B * 32 * HW, a->grad_src[v], HW);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace aarmvs
