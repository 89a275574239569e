// Backpropagation through the recurrent regulariser (UNetConvLSTM, models/drmvsnet.py:119-167,
// ConvLSTMCell module.py:76-92, deConvGnReLU module.py:264-287, conv_0 drmvsnet.py:117) for
// gfx950: the BPTT of EMVSNet's training sweep (drmvsnet.py:273-291) on the tensors the forward
// kept in its training record (aarmvs_train_record).
//
// Per plane d, last plane first (the recurrence), the input gradients only:
//   cell 4 gates  <- dL/dcost (conv_0 transposed, fused) + dL/dh4 carried from plane d+1
//   cell 4 dgrad  -> dL/d relu(GN(u1)), dL/dh0' (added), dL/dh4 of plane d-1
//   GN(2,16) backward sums of deconv_1, then deconv_1 transposed -> dL/dh3' (added)
//   cell 3 gates, cell 3 dgrad, deconv_0 likewise, cell 2 gates / dgrad (-> dL/d maxpool(h1'))
//   cell 1 gates (+ max-pool routing), cell 1 dgrad, cell 0 gates (+ routing), cell 0 dgrad
//   -> dL/dx of plane d (the cost slice's gradient) and dL/dh0 of plane d-1.
// The gate gradients dL/dz of every cell and the deconvs' output gradients are kept for a group
// of planes; the weight gradients (sums over pixels and planes) run once per group: cells on the
// matrix cores (split-fp16, four products), deconvs / head / biases / GroupNorm affines on VALU,
// per-block partials reduced in a fixed order into fp64 accumulators -> deterministic.
//
// The input-gradient convs (dgrad) are the forward 3x3 convs transposed and flipped, on the
// same split-fp16 v_mfma_f32_32x32x16_f16 implicit GEMM as the forward cells (three products,
// DESIGN.md §7); the gate gradients carry a per-plane power-of-two scale (max |dL/dz| -> 2^14)
// so that fp16's range holds them whatever their magnitude.
// All tensors NHWC ([B][H][W][C]) fp32, as in the forward record.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <initializer_list>

#include "device_common.h"

namespace aarmvs {

typedef _Float16 bhalf8 __attribute__((ext_vector_type(8)));
typedef float bfloatx16 __attribute__((ext_vector_type(16)));
typedef float bfloatx4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float acc_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }

// power-of-two exponent e with max * 2^-e in [2^14, 2^15) (0 for an all-zero tensor)
__device__ __forceinline__ int scale_exp(unsigned bits) {
  const float m = __uint_as_float(bits);
  if (!(m > 0.0f)) return 0;
  if (!(m < INFINITY)) return 120;
  return ilogbf(m) - 14;
}

// a pair (a, b) split the same way: the hi pair as one v_cvt_pk_f16_f32 read back for the lo
// parts (6 instructions per pair instead of 8 for two split16)
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split16x2(float a, float b, half2v& hi, half2v& lo) {
  hi = __builtin_convertvector((float2v){a, b}, half2v);
  lo = __builtin_convertvector((float2v){a - (float)hi[0], b - (float)hi[1]}, half2v);
}

// max |v| of a wave folded into *dst (float bits: non-negative floats order as unsigned)
// The block's max |v| (NaN as +inf) as float bits, one plain store per block: the scale maxima
// are per-block partials reduced by their consumers in a fixed way, no atomics (deterministic
// whatever the schedule).
__device__ __forceinline__ void block_absmax_store(float m, unsigned* dst) {
  __shared__ float wm[16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float q = __shfl_xor(m, o, 64);
    m = (q > m || q != q) ? q : m;
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) wm[w] = m != m ? INFINITY : fabsf(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = 0.f;
    for (int i = 0; i < nw; ++i) b = fmaxf(b, wm[i]);
    *dst = __float_as_uint(b);
  }
}

// max over n partial maxima (float bits) by the whole block; every thread gets the result
__device__ __forceinline__ unsigned block_max_of(const unsigned* p, int n) {
  __shared__ unsigned wm[16];
  unsigned m = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) m = max(m, p[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) wm[w] = m;
  __syncthreads();
  unsigned r = 0;
  for (int i = 0; i < nw; ++i) r = max(r, wm[i]);
  return r;
}

// ---------------------------------------------------------------------------
// Scratch layout of aarmvs_sweep_backward (all regions 256-B aligned).
// ---------------------------------------------------------------------------
constexpr int kWgBlocks = 256;   // wgrad blocks per launch (= partials per reduce)

struct BpttLayout {
  float* gh[5];        // dL/dh of the state the current plane leaves [Pk][hid]
  float* gc[5];        // dL/dc likewise
  float* gz[5];        // [G][Pk][4 hid] gate gradients of the group's planes
  unsigned* zmax;      // [5][G] float bits of max |gz| per (cell, group plane), after zmax_group
  unsigned* zpart;     // [5][G][zp_n] per-gate-block maxima of |gz| (float bits), plain stores
  int zp_n;            // partial slots per (cell, plane): the gate kernel's largest grid
  float* gr[2];        // dL/d relu(GN(u_j)) of the current plane [B][Hu][Wu][16]
  float* gr0b;         // gr[0]'s second buffer (odd planes: stage A writes it, stage B reads it)
  float* gskip[2][2];  // [plane parity][cell 0, 1] cells 4 and 3's skip-input dL/dh0, dL/dh1 [Pk][16]
  float* gpool[2];     // dL/d maxpool(h0'), maxpool(h1') [B][H/2^(j+1)][.][16]
  float* gu[2];        // [G][B][Hu][Wu][16] dL/du_j (deconv outputs) of the group's planes
  float* gx;           // [G][B][H][W][32] dL/dx of the group's planes
  double* gnb_part[2]; // per deconv [G][B][nblk][36] GroupNorm-backward partial sums of the group's planes
  double* gacc;        // [raw param count] fp64 parameter-gradient accumulators
  float* wpart;        // [kWgBlocks][kWgPartMax] wgrad partials
  double* rseg;        // [kRedSeg][kWgPartMax] segment sums of the partials
  // the per-group buffers above (gz, zmax, gu, gx, gnb_part) exist twice, one set per group
  // parity, so that a group's weight-gradient and cost-slice stage can run beside the next
  // group's planes; use_set(p) points the fields at set p
  struct GroupSet {
    float* gz[5];
    unsigned* zmax;
    unsigned* zpart;
    float* gu[2];
    float* gx;
    double* gnb_part[2];
  } set[2];
  void use_set(int p) {
    const GroupSet& g = set[p];
    for (int k = 0; k < 5; ++k) gz[k] = g.gz[k];
    zmax = g.zmax;
    zpart = g.zpart;
    gu[0] = g.gu[0];
    gu[1] = g.gu[1];
    gx = g.gx;
    gnb_part[0] = g.gnb_part[0];
    gnb_part[1] = g.gnb_part[1];
  }
  size_t bytes;
  size_t cell_px[5];
  int gnb_nblk;
};
constexpr size_t kWgPartMax = 64 * 64 * 9 + 64;
constexpr int kRedSeg = 64;      // segments of the two-pass partial reduction

static inline size_t al256(size_t x) { return (x + 255) / 256 * 256; }

BpttLayout bptt_layout(void* base, int B, int H, int W) {
  BpttLayout L{};
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = p ? p + off : nullptr;
    off = al256(off + bytes);
    return r;
  };
  const size_t HW = (size_t)H * W;
  const size_t px[5] = {HW, HW / 4, HW / 16, HW / 4, HW};
  const int G = kPlaneGroup;
  for (int k = 0; k < 5; ++k) {
    L.cell_px[k] = (size_t)B * px[k];
    L.gh[k] = reinterpret_cast<float*>(take(L.cell_px[k] * kCellHid[k] * 4));
    L.gc[k] = reinterpret_cast<float*>(take(L.cell_px[k] * kCellHid[k] * 4));
  }
  L.gnb_nblk = (int)std::min<size_t>(512, (HW + 1023) / 1024);
  L.zp_n = (int)((L.cell_px[0] * 4 + 255) / 256);   // gate blocks of the largest cell (hid / 4 lanes per px)
  for (int q = 0; q < 2; ++q) {
    BpttLayout::GroupSet& g = L.set[q];
    for (int k = 0; k < 5; ++k)
      g.gz[k] = reinterpret_cast<float*>(take((size_t)G * L.cell_px[k] * 4 * kCellHid[k] * 4));
    g.zmax = reinterpret_cast<unsigned*>(take(5 * G * 4));
    g.zpart = reinterpret_cast<unsigned*>(take((size_t)5 * G * L.zp_n * 4));
    g.gu[0] = reinterpret_cast<float*>(take((size_t)G * B * (HW / 4) * 16 * 4));
    g.gu[1] = reinterpret_cast<float*>(take((size_t)G * B * HW * 16 * 4));
    g.gx = reinterpret_cast<float*>(take((size_t)G * B * HW * kC * 4));
    for (int j = 0; j < 2; ++j)
      g.gnb_part[j] = reinterpret_cast<double*>(take((size_t)G * B * L.gnb_nblk * 36 * 8));
  }
  L.use_set(0);
  L.gr[0] = reinterpret_cast<float*>(take((size_t)B * (HW / 4) * 16 * 4));
  L.gr[1] = reinterpret_cast<float*>(take((size_t)B * HW * 16 * 4));
  L.gr0b = reinterpret_cast<float*>(take((size_t)B * (HW / 4) * 16 * 4));
  for (int q = 0; q < 2; ++q)
    for (int k = 0; k < 2; ++k) L.gskip[q][k] = reinterpret_cast<float*>(take(L.cell_px[k] * 16 * 4));
  L.gpool[0] = reinterpret_cast<float*>(take((size_t)B * (HW / 4) * 16 * 4));
  L.gpool[1] = reinterpret_cast<float*>(take((size_t)B * (HW / 16) * 16 * 4));
  L.gacc = reinterpret_cast<double*>(take(param_layout().raw_total * 8));
  L.wpart = reinterpret_cast<float*>(take((size_t)kWgBlocks * kWgPartMax * 4));
  L.rseg = reinterpret_cast<double*>(take((size_t)kRedSeg * kWgPartMax * 8));
  L.bytes = off;
  return L;
}

// ---------------------------------------------------------------------------
// Gate backward of one cell at one plane (module.py:83-90 differentiated):
//   dh = dL/dh' (+ conv_0 transposed of dL/dcost for cell 4, + max-pool routing for cells
//   0 and 1), dc = dL/dc' ->
//   dz_o = dh tanh(c') s_o (1 - s_o), dc' += dh s_o (1 - tanh(c')^2),
//   dz_i = dc' tanh(g) s_i (1 - s_i), dz_f = dc' c s_f (1 - s_f), dz_g = dc' s_i (1 - tanh(g)^2),
//   dL/dc (previous plane) = dc' s_f.
// One thread per (pixel, 4 hidden channels).
// ---------------------------------------------------------------------------
struct GateBwdArgs {
  const float* z;        // pre-activations (i, f, o, g), the record's [B][hid/4][4][H*W][4]
  const float* c_prev;   // [P][hid]
  const float* c_new;    // [P][hid]
  const float* gh;       // [P][hid] dL/dh'
  const float* gh_add;   // null or [P][hid]: a second term of dL/dh' (the skip input's), added to gh
  float* gc;             // [P][hid] dL/dc' in, dL/dc (previous plane) out
  float* gz;             // [P][4 hid] out
  unsigned* zpart;       // per-block max |gz| (float bits) at [blockIdx.x]
  int mode;              // 0: none, 1: cell 4 head, 2: max-pool routing
  const float* gcost;    // mode 1: dL/dcost of this plane, [B][D][H][W] at plane d
  int gcost_bstride;     // D * H * W
  const float* whead;    // mode 1: conv_0 weight [8][3][3] (raw)
  const float* gpool;    // mode 2: dL/d maxpool(h') [B][H/2][W/2][hid]
  const float* hnew;     // mode 2: h' [P][hid]
  int B, H, W, hid;
};

__global__ void __launch_bounds__(256) gate_bwd_kernel(GateBwdArgs a) {
  // 32-bit index arithmetic (B H W hid < 2^31, checked by the caller): 64-bit divisions by
  // the runtime W, H were most of this streaming kernel's instructions
  const int hid = a.hid, qs = hid == 16 ? 2 : 1;   // log2(hid / 4): hid is 16 or 8
  const uint32_t HWc = (uint32_t)a.H * (uint32_t)a.W, P = (uint32_t)a.B * HWc;
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  float m = 0.f;
  if (t < (P << qs)) {
    const uint32_t p = t >> qs;
    const int c0 = (int)(t & ((1u << qs) - 1u)) * 4;
    const uint32_t b32 = p / HWc, pl = p - b32 * HWc, y32 = pl / (uint32_t)a.W;
    const int b = (int)b32, y = (int)y32, x = (int)(pl - y32 * (uint32_t)a.W);
    float4 dh4 = *reinterpret_cast<const float4*>(a.gh + p * hid + c0);
    if (a.gh_add) {
      const float4 s4 = *reinterpret_cast<const float4*>(a.gh_add + p * hid + c0);
      dh4.x += s4.x;
      dh4.y += s4.y;
      dh4.z += s4.z;
      dh4.w += s4.w;
    }
    float dh[4] = {dh4.x, dh4.y, dh4.z, dh4.w};
    if (a.mode == 1) {
      // cost[q] = sum_{ci,tap} w[ci][tap] h4[q + off(tap)] + b  ->  dh4[p][ci] = sum_tap w[ci][tap] gcost[p - off(tap)]
      const float* gcb = a.gcost + (size_t)b * a.gcost_bstride;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int qy = y - (tap / 3 - 1), qx = x - (tap % 3 - 1);
        if (qy >= 0 && qy < a.H && qx >= 0 && qx < a.W) {
          const float g = gcb[(size_t)qy * a.W + qx];
#pragma unroll
          for (int i = 0; i < 4; ++i) {   // hid 8: c0 is 0 or 4 (wave-uniform loads, then a select)
            const float w0 = a.whead[i * 9 + tap], w4 = a.whead[(4 + i) * 9 + tap];
            dh[i] = fmaf(c0 ? w4 : w0, g, dh[i]);
          }
        }
      }
    } else if (a.mode == 2) {
      // F.max_pool2d(2, 2) backward: the window's first maximum (row-major scan) takes the gradient
      const int y0 = y & ~1, x0 = x & ~1;
      const int Wc = a.W / 2, Hc = a.H / 2;
      if (y0 + 1 < a.H + 0 && (y >> 1) < Hc && (x >> 1) < Wc) {
        const size_t base = ((size_t)b * a.H + y0) * a.W + x0;
        const float4 v00 = *reinterpret_cast<const float4*>(a.hnew + base * hid + c0);
        const float4 v01 = *reinterpret_cast<const float4*>(a.hnew + (base + 1) * hid + c0);
        const float4 v10 = *reinterpret_cast<const float4*>(a.hnew + (base + a.W) * hid + c0);
        const float4 v11 = *reinterpret_cast<const float4*>(a.hnew + (base + a.W + 1) * hid + c0);
        const float4 gp = *reinterpret_cast<const float4*>(
            a.gpool + (((size_t)b * Hc + (y >> 1)) * Wc + (x >> 1)) * hid + c0);
        const int me = (y - y0) * 2 + (x - x0);
        const float w0[4] = {v00.x, v00.y, v00.z, v00.w}, w1[4] = {v01.x, v01.y, v01.z, v01.w};
        const float w2[4] = {v10.x, v10.y, v10.z, v10.w}, w3[4] = {v11.x, v11.y, v11.z, v11.w};
        const float gg[4] = {gp.x, gp.y, gp.z, gp.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int am = 0;
          float mv = w0[i];
          if (w1[i] > mv) { mv = w1[i]; am = 1; }
          if (w2[i] > mv) { mv = w2[i]; am = 2; }
          if (w3[i] > mv) { mv = w3[i]; am = 3; }
          if (am == me) dh[i] += gg[i];
        }
      }
    }
    // the record's planar gate layout [B][hid/4 quads][4 gates][H*W][4] (CellArgs::z_out)
    const float* zp = a.z + (size_t)b * 4 * hid * HWc + ((size_t)(c0 >> 2) * 4 * HWc + pl) * 4;
    const float4 zi = *reinterpret_cast<const float4*>(zp);
    const float4 zf = *reinterpret_cast<const float4*>(zp + (size_t)HWc * 4);
    const float4 zo = *reinterpret_cast<const float4*>(zp + (size_t)HWc * 8);
    const float4 zg = *reinterpret_cast<const float4*>(zp + (size_t)HWc * 12);
    const float4 cp = *reinterpret_cast<const float4*>(a.c_prev + p * hid + c0);
    const float4 cn = *reinterpret_cast<const float4*>(a.c_new + p * hid + c0);
    const float4 gc4 = *reinterpret_cast<const float4*>(a.gc + p * hid + c0);
    const float ZI[4] = {zi.x, zi.y, zi.z, zi.w}, ZF[4] = {zf.x, zf.y, zf.z, zf.w};
    const float ZO[4] = {zo.x, zo.y, zo.z, zo.w}, ZG[4] = {zg.x, zg.y, zg.z, zg.w};
    const float CP[4] = {cp.x, cp.y, cp.z, cp.w}, CN[4] = {cn.x, cn.y, cn.z, cn.w};
    const float GC[4] = {gc4.x, gc4.y, gc4.z, gc4.w};
    float di[4], df[4], dO[4], dg[4], dcp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float si = acc_sigmoid(ZI[i]), sf = acc_sigmoid(ZF[i]), so = acc_sigmoid(ZO[i]);
      const float tg = tanhf(ZG[i]), tc = tanhf(CN[i]);
      dO[i] = dh[i] * tc * so * (1.0f - so);
      const float dcn = GC[i] + dh[i] * so * (1.0f - tc * tc);
      di[i] = dcn * tg * si * (1.0f - si);
      df[i] = dcn * CP[i] * sf * (1.0f - sf);
      dg[i] = dcn * si * (1.0f - tg * tg);
      dcp[i] = dcn * sf;
      m = fmaxf(m, fmaxf(fmaxf(fabsf(di[i]), fabsf(df[i])), fmaxf(fabsf(dO[i]), fabsf(dg[i]))));
      if (di[i] != di[i] || df[i] != df[i] || dO[i] != dO[i] || dg[i] != dg[i]) m = INFINITY;
    }
    float* gzp = a.gz + p * (4 * hid) + c0;
    *reinterpret_cast<float4*>(gzp) = make_float4(di[0], di[1], di[2], di[3]);
    *reinterpret_cast<float4*>(gzp + hid) = make_float4(df[0], df[1], df[2], df[3]);
    *reinterpret_cast<float4*>(gzp + 2 * hid) = make_float4(dO[0], dO[1], dO[2], dO[3]);
    *reinterpret_cast<float4*>(gzp + 3 * hid) = make_float4(dg[0], dg[1], dg[2], dg[3]);
    *reinterpret_cast<float4*>(a.gc + p * hid + c0) = make_float4(dcp[0], dcp[1], dcp[2], dcp[3]);
  }
  block_absmax_store(m, a.zpart + blockIdx.x);
}

// ---------------------------------------------------------------------------
// Input-gradient conv (dgrad) of a cell: out[p][ci] = sum_{tap, cz} A[ci][cz, tap] gz[p + off(tap)][cz]
// with A the packed transposed/flipped weights (pack_dgrad_kernel).  Implicit GEMM on
// v_mfma_f32_32x32x16_f16: M = 32 output channels (one m-tile per block, blockIdx.y), N = the
// 32 pixels of a tile row (one wave per row, 8 rows), K = 9 taps x 16 gate channels per chunk.
// gz is staged per 16-channel chunk as fp16 hi/lo (scaled by the plane's 2^-e) into the
// forward cells' LDS pixel layout (h3_pix); the block's A fragments stay in LDS.
// Output channels go to up to three destinations (the cell input's parts), stored or added.
// ---------------------------------------------------------------------------
struct DgPart {
  float* dst;    // [P][nch]
  int c0, nch;   // output channels c0 .. c0 + nch - 1 of the conv
  int add;       // 1: dst += , 0: dst =
};
struct DgradArgs {
  const float* gz;          // [B][H][W][CZ]
  const unsigned* zpart;    // the gate kernel's per-block maxima of |gz| (float bits)
  int nzp;
  const float* wfrag;       // this cell's packed fragments (all m-tiles)
  const float* wscale;      // 1 / 2^e of the fragments
  DgPart part[3];
  int nparts;
  int cout;                 // valid output channels (cin of the forward conv)
  int B, H, W;
};

constexpr int kDgTH = 8, kDgTW = 32, kDgW2 = kDgTW + 2, kDgNPIX = (kDgTH + 2) * kDgW2;

__device__ __forceinline__ int dg_pix(int p, int h) { return p * 32 + ((h ^ ((p >> 3) & 1)) << 4); }

// Persistent: a block keeps its m-tile's fragments in LDS and walks the tiles (stride gridDim.x);
// the next chunk's gz (this tile's, or the next tile's first) is loaded into registers while the
// current chunk's MFMAs run.
template <int CZ>
__global__ void __launch_bounds__(512) dgrad_kernel(DgradArgs a) {
  constexpr int NCHK = CZ / 16;
  constexpr int AH = NCHK * 9 * 2 * 512;   // halves of this m-tile's fragments (hi and lo)
  constexpr int NI = (2 * kDgNPIX + 511) / 512;   // staging items per thread
  extern __shared__ __attribute__((aligned(16))) char lds_dg[];
  char* wl = lds_dg;                        // [chunk][tap][hi, lo][64 lanes][8]
  char* in_hi = wl + AH * 2;
  char* in_lo = in_hi + kDgNPIX * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mt = blockIdx.y;
  const int tiles_x = (a.W + kDgTW - 1) / kDgTW, tiles_y = (a.H + kDgTH - 1) / kDgTH;
  const int ntiles = a.B * tiles_x * tiles_y;
  int tile = blockIdx.x;
  if (tile >= ntiles) return;   // whole block
  {
    const float4* s = reinterpret_cast<const float4*>(a.wfrag + (size_t)mt * (AH / 2));
    float4* d = reinterpret_cast<float4*>(wl);
    for (int i = tid; i < AH * 2 / 16; i += 512) d[i] = s[i];
  }
  const int ez = scale_exp(block_max_of(a.zpart, a.nzp));
  const float zs = ldexpf(1.0f, -ez);
  const float inv = *a.wscale * ldexpf(1.0f, ez);
  auto coords = [&](int t, int& b, int& y0, int& x0) {
    b = t / (tiles_x * tiles_y);
    const int rem = t % (tiles_x * tiles_y);
    y0 = (rem / tiles_x) * kDgTH;
    x0 = (rem % tiles_x) * kDgTW;
  };
  // two prefetched chunks in flight (register buffers by chunk parity): chunk i + 2's loads are
  // issued when chunk i is staged, so a chunk's global latency spans two chunks' MFMAs
  float4 pv[2][NI][2];   // [buffer][item j = (half hh, haloed pixel p) of e = tid + 512 j]
  auto load = [&](int t, int c, int buf) {
    int b, y0, x0;
    coords(t, b, y0, x0);
    const float* gzb = a.gz + (size_t)b * a.H * a.W * CZ;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int e = tid + 512 * j;
      const int hh = e >= kDgNPIX ? 1 : 0, p = e - hh * kDgNPIX;
      const int row = p / kDgW2, cc = p - row * kDgW2;
      const int gy = y0 - 1 + row, gx = x0 - 1 + cc;
      pv[buf][j][0] = pv[buf][j][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < 2 * kDgNPIX && gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
        const float4* s = reinterpret_cast<const float4*>(gzb + ((size_t)gy * a.W + gx) * CZ + 16 * c + 8 * hh);
        pv[buf][j][0] = s[0];
        pv[buf][j][1] = s[1];
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int e = tid + 512 * j;
      if (e >= 2 * kDgNPIX) continue;
      const int hh = e >= kDgNPIX ? 1 : 0, p = e - hh * kDgNPIX;
      const float4 q0 = pv[buf][j][0], q1 = pv[buf][j][1];
      const float v[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
      bhalf8 hv, lv;
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        half2v hi, lo;
        split16x2(v[k] * zs, v[k + 1] * zs, hi, lo);
        hv[k] = hi[0];
        hv[k + 1] = hi[1];
        lv[k] = lo[0];
        lv[k + 1] = lo[1];
      }
      *reinterpret_cast<bhalf8*>(in_hi + dg_pix(p, hh)) = hv;
      *reinterpret_cast<bhalf8*>(in_lo + dg_pix(p, hh)) = lv;
    }
  };
  const int col = lane & 31, h = lane >> 5;
  load(tile, 0, 0);
  load(tile, 1, 1);   // (NCHK >= 2)
  for (; tile < ntiles; tile += gridDim.x) {
    int b, y0, x0;
    coords(tile, b, y0, x0);
    const int next = tile + (int)gridDim.x;
    // sign-balanced accumulation (convlstm.hip h3_mfma_chunk): taps with (tap + chunk) odd
    // carry negated fragments (pack_dgrad_kernel) and go to accn; the result is acc - accn
    bfloatx16 acc, accn;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = accn[j] = 0.f;
    static_assert(NCHK % 2 == 0, "chunk pairs (the accumulators' sign pattern)");
    auto chunk = [&](int c, auto PAR) {
      constexpr int CP = decltype(PAR)::value;   // c & 1
      __syncthreads();   // previous chunk's fragment reads done (fragments visible the first time)
      store(CP);
      __syncthreads();
      if (c + 2 < NCHK)
        load(tile, c + 2, CP);
      else if (next < ntiles)
        load(next, c + 2 - NCHK, CP);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int p = (wave + tap / 3) * kDgW2 + col + tap % 3;
        const bhalf8 bh = *reinterpret_cast<const bhalf8*>(in_hi + dg_pix(p, h));
        const bhalf8 bl = *reinterpret_cast<const bhalf8*>(in_lo + dg_pix(p, h));
        const char* af = wl + (size_t)(((c * 9 + tap) * 2) * 512 + lane * 8) * 2;
        const bhalf8 ah = *reinterpret_cast<const bhalf8*>(af);
        const bhalf8 alo = *reinterpret_cast<const bhalf8*>(af + 512 * 2);
        bfloatx16& d = ((tap + CP) & 1) ? accn : acc;
        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bh, d, 0, 0, 0);
      }
    };
#pragma unroll 1
    for (int c = 0; c < NCHK; c += 2) {
      chunk(c, std::integral_constant<int, 0>{});
      chunk(c + 1, std::integral_constant<int, 1>{});
    }
    acc -= accn;
    const int y = y0 + wave, x = x0 + col;
    if (y < a.H && x < a.W) {
      const size_t p = ((size_t)b * a.H + y) * a.W + x;
      // D row m = 8 (j >> 2) + 4 h + (j & 3) -> output channel 32 mt + m
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int co = 32 * mt + 8 * g + 4 * h;
        if (co >= a.cout) continue;
#pragma unroll
        for (int pi = 0; pi < 3; ++pi) {
          if (pi >= a.nparts) break;
          const DgPart& pt = a.part[pi];
          if (co >= pt.c0 && co < pt.c0 + pt.nch) {
            float4* d = reinterpret_cast<float4*>(pt.dst + p * pt.nch + (co - pt.c0));
            float4 v = make_float4(acc[4 * g] * inv, acc[4 * g + 1] * inv, acc[4 * g + 2] * inv,
                                   acc[4 * g + 3] * inv);
            if (pt.add) {
              const float4 o = *d;
              v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
            }
            *d = v;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// deConvGnReLU backward (module.py:286-287): y = relu(GN(u)).  Per (b, group) the sums
// S1 = sum g_xhat, S2 = sum g_xhat xhat with g_xhat = [y > 0] g gamma, and per channel the
// affine gradients sum [y > 0] g xhat (gamma) and sum [y > 0] g (beta).  Per-block partials,
// then a fixed-order reduce (the affine sums go straight into the fp64 accumulators).
// ---------------------------------------------------------------------------
struct GnbArgs {
  const float* gr;       // [B][HW][16] dL/dy
  const float* u;        // [B][HW][16]
  const double* stats;   // the plane's reg stats (reg_stat_index(b, j, g))
  const float* gamma;
  const float* beta;
  double* part;          // [B][nblk][36]
  int j, HW;
};

__global__ void __launch_bounds__(256) gnb_partial_kernel(GnbArgs a) {
  __shared__ double red[36 * 4];
  __shared__ float coef[2][16];   // a = rstd gamma, b = beta - mean a
  __shared__ float mr[2][2];
  const int b = blockIdx.y;
  if (threadIdx.x < 16) {
    const int c = threadIdx.x, g = c >> 3;
    const GnStat st = stat_read(a.stats + reg_stat_index(b, a.j, g), 8.0 * a.HW);
    const float sc = st.rstd * a.gamma[c];
    coef[0][c] = sc;
    coef[1][c] = a.beta[c] - st.mean * sc;
    if ((c & 7) == 0) {
      mr[g][0] = st.mean;
      mr[g][1] = st.rstd;
    }
  }
  __syncthreads();
  // the 36 block-uniform coefficients in scalar registers (read from LDS into VGPRs they held
  // 36 more VGPRs through the loop: 176, two waves per SIMD)
  float ca[16], cb[16], mrs[2][2];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    ca[c] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(coef[0][c])));
    cb[c] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(coef[1][c])));
  }
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int k = 0; k < 2; ++k) mrs[g][k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(mr[g][k])));
  double s[36];   // fp64: cancelling sums
#pragma unroll
  for (int i = 0; i < 36; ++i) s[i] = 0.0;
  const float* grb = a.gr + (size_t)b * a.HW * 16;
  const float* ub = a.u + (size_t)b * a.HW * 16;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < a.HW; p += gridDim.x * 256) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 g4 = *reinterpret_cast<const float4*>(grb + (size_t)p * 16 + 4 * q);
      const float4 u4 = *reinterpret_cast<const float4*>(ub + (size_t)p * 16 + 4 * q);
      const float G[4] = {g4.x, g4.y, g4.z, g4.w}, U[4] = {u4.x, u4.y, u4.z, u4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 4 * q + i, grp = c >> 3;
        const float yv = fmaf(U[i], ca[c], cb[c]);
        const float gn = yv > 0.f ? G[i] : 0.f;
        const float xh = (U[i] - mrs[grp][0]) * mrs[grp][1];
        const float gxh = gn * a.gamma[c];
        s[2 * grp] += gxh;
        s[2 * grp + 1] += gxh * xh;
        s[4 + c] += gn * xh;
        s[20 + c] += gn;
      }
    }
  }
  block_sum_d_store<36>(s, red, a.part + ((size_t)b * gridDim.x + blockIdx.x) * 36);
}

// The affine sums of a group's planes -> gacc, once per group (one block per column 4 .. 35):
// plane by plane in the backward's order (last first), per plane the samples in order, per
// sample strided per-thread sums and a fixed tree -- the order a per-plane reduce would use.
__global__ void __launch_bounds__(256) gnb_affine_kernel(const double* __restrict__ part, int n, int nblk,
                                                         int B, double* __restrict__ gacc_gamma,
                                                         double* __restrict__ gacc_beta) {
  __shared__ double red[256];
  const int i = 4 + blockIdx.x, t = threadIdx.x;
  for (int k = n - 1; k >= 0; --k) {
    double tot = 0.0;
    for (int b = 0; b < B; ++b) {
      double s = 0.0;
      for (int m = t; m < nblk; m += 256) s += part[(((size_t)k * B + b) * nblk + m) * 36 + i];
      red[t] = s;
      __syncthreads();
      for (int o = 128; o > 0; o >>= 1) {
        if (t < o) red[t] += red[t + o];
        __syncthreads();
      }
      if (t == 0) tot += red[0];
      __syncthreads();
    }
    if (t == 0) {
      if (i < 20) gacc_gamma[i - 4] += tot;
      else gacc_beta[i - 20] += tot;
    }
  }
}

// ---------------------------------------------------------------------------
// deconv_j backward (ConvTranspose2d(16,16,3,s2,p1,op1), module.py:281): per coarse pixel
// dL/dh[ci] = sum_{ky,kx,co} gu[2y-1+ky][2x-1+kx][co] W[ci][co][ky][kx], with the GroupNorm+ReLU
// backward applied on the fly: gu = rstd (g_xhat - S1/n - xhat S2/n).  The coarse pixel's own
// 2 x 2 output quad's gu is stored (weight and bias gradients).  dL/dh is added into gh.
// Four lanes per coarse pixel (one output-channel quarter each); weights [tap][co][ci] in LDS.
// ---------------------------------------------------------------------------
struct DcbArgs {
  const float* gr;       // [B][Ho][Wo][16]
  const float* u;        // [B][Ho][Wo][16]
  const double* stats;   // plane's reg stats
  const double* part;    // the plane's GroupNorm-backward partials [B][nblk][36]
  int nblk;
  const float* gamma;
  const float* beta;
  const float* w;        // raw ConvTranspose2d weight [ci][co][3][3]
  float* gu;             // [B][Ho][Wo][16] out (owned quads)
  float* gh;             // [B][Hi][Wi][16] += dL/dh
  int j, Hi, Wi;
};

__global__ void __launch_bounds__(256) deconv_bwd_kernel(DcbArgs a) {
  __shared__ float4 wsh[9 * 16 * 4];   // [tap][co & 3][co >> 2][ci / 4]: the 4 lanes of a quad (co >> 2)
                                       // read 4 distinct float4s in distinct banks
  __shared__ float coef[4][16];        // y = u a + b; xhat = (u - mean) rstd
  __shared__ float gco[2][2];          // per group: S1 / n, S2 / n
  __shared__ double gred[4][256];
  const int b = blockIdx.y, tid = threadIdx.x;
  // S1, S2 of both groups from the partials: strided per-thread sums and a fixed tree (every
  // block computes the same values)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double sum = 0.0;
    for (int m = tid; m < a.nblk; m += 256) sum += a.part[((size_t)b * a.nblk + m) * 36 + i];
    gred[i][tid] = sum;
  }
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
#pragma unroll
      for (int i = 0; i < 4; ++i) gred[i][tid] += gred[i][tid + o];
    }
    __syncthreads();
  }
  const int Ho = 2 * a.Hi, Wo = 2 * a.Wi;
  for (int i = tid; i < 9 * 16 * 16; i += 256) {
    const int ci = i & 15, co = (i >> 4) & 15, tap = i >> 8;
    reinterpret_cast<float*>(wsh)[((((tap * 4 + (co & 3)) * 4 + (co >> 2)) * 4) + (ci >> 2)) * 4 + (ci & 3)] =
        a.w[(ci * 16 + co) * 9 + tap];
  }
  if (tid < 16) {
    const int c = tid, g = c >> 3;
    const GnStat st = stat_read(a.stats + reg_stat_index(b, a.j, g), 8.0 * Ho * Wo);
    const float sc = st.rstd * a.gamma[c];
    coef[0][c] = sc;
    coef[1][c] = a.beta[c] - st.mean * sc;
    coef[2][c] = st.mean;
    coef[3][c] = st.rstd;
    if ((c & 7) == 0) {
      const double n = 8.0 * Ho * Wo;
      gco[g][0] = (float)(gred[2 * g][0] / n);
      gco[g][1] = (float)(gred[2 * g + 1][0] / n);
    }
  }
  __syncthreads();
  // four lanes per coarse pixel, lane q the output channels 4q .. 4q + 3: its dL/dy and u
  // loads are one float4 each per tap, its dL/dh partial over those channels is summed over
  // the quad on DPP, and lane q adds input channels 4q .. 4q + 3 into gh
  const int pidx = blockIdx.x * 64 + (tid >> 2), q = tid & 3;
  if (pidx >= a.Hi * a.Wi) return;   // whole quads leave together
  const int iy = pidx / a.Wi, ix = pidx % a.Wi;
  const float* grb = a.gr + (size_t)b * Ho * Wo * 16 + 4 * q;
  const float* ub = a.u + (size_t)b * Ho * Wo * 16 + 4 * q;
  const int grp = q >> 1;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll 3
  for (int tap = 0; tap < 9; ++tap) {
    const int oy = 2 * iy - 1 + tap / 3, ox = 2 * ix - 1 + tap % 3;
    if (oy < 0 || oy >= Ho || ox < 0 || ox >= Wo) continue;
    const size_t o = ((size_t)oy * Wo + ox) * 16;
    const float4 g4 = *reinterpret_cast<const float4*>(grb + o);
    const float4 u4 = *reinterpret_cast<const float4*>(ub + o);
    const float G[4] = {g4.x, g4.y, g4.z, g4.w}, U[4] = {u4.x, u4.y, u4.z, u4.w};
    float gu[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 4 * q + i;
      const float yv = fmaf(U[i], coef[0][c], coef[1][c]);
      const float gxh = (yv > 0.f ? G[i] : 0.f) * a.gamma[c];
      const float xh = (U[i] - coef[2][c]) * coef[3][c];
      gu[i] = coef[3][c] * (gxh - gco[grp][0] - xh * gco[grp][1]);
    }
    if (tap == 4 || tap == 5 || tap == 7 || tap == 8)   // the owned quad (2y + a, 2x + b)
      *reinterpret_cast<float4*>(a.gu + (size_t)b * Ho * Wo * 16 + o + 4 * q) = make_float4(gu[0], gu[1], gu[2], gu[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float g = gu[i];
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) {
        const float4 wv = wsh[((tap * 4 + i) * 4 + q) * 4 + c4];
        acc[4 * c4 + 0] = fmaf(g, wv.x, acc[4 * c4 + 0]);
        acc[4 * c4 + 1] = fmaf(g, wv.y, acc[4 * c4 + 1]);
        acc[4 * c4 + 2] = fmaf(g, wv.z, acc[4 * c4 + 2]);
        acc[4 * c4 + 3] = fmaf(g, wv.w, acc[4 * c4 + 3]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {   // (a0 + a1) + (a2 + a3) in every lane of the quad
    float v = acc[i];
    v += __int_as_float(dpp_i32<0xB1, 0xF>(0, __float_as_int(v)));
    v += __int_as_float(dpp_i32<0x4E, 0xF>(0, __float_as_int(v)));
    acc[i] = v;
  }
  float4 mine = make_float4(acc[0], acc[1], acc[2], acc[3]);
  if (q == 1) mine = make_float4(acc[4], acc[5], acc[6], acc[7]);
  if (q == 2) mine = make_float4(acc[8], acc[9], acc[10], acc[11]);
  if (q == 3) mine = make_float4(acc[12], acc[13], acc[14], acc[15]);
  float4* gh = reinterpret_cast<float4*>(a.gh + (((size_t)b * a.Hi + iy) * a.Wi + ix) * 16 + 4 * q);
  float4 o = *gh;
  o.x += mine.x;
  o.y += mine.y;
  o.z += mine.z;
  o.w += mine.w;
  *gh = o;
}

// ---------------------------------------------------------------------------
// Cell weight gradient over a group of planes: gW[cz][ci][tap] = sum_{d,p} gz_d[p][cz] in_d[p +
// off(tap)][ci], gb[cz] = sum gz.  v_mfma_f32_16x16x32_f16 with K = the 32 pixels of a tile
// row: A = gz^T (16 gate channels x 32 px, from a channel-major LDS image), B = the cell input
// at the tap's offset (32 px x 16 input channels).  Four split-fp16 products per MFMA step
// (hi hi, hi lo, lo hi, lo lo: ~fp32 products).  Blocks stride over the group's (plane, tile)
// items and write one partial each, reduced in a fixed order (reduce_partials).
// ---------------------------------------------------------------------------
enum WgMode : int { WG_PLAIN = 0, WG_POOL = 1, WG_GNRELU = 2 };
struct WgPart {
  const float* ptr;     // plane 0's tensor; plane d at ptr + d * dstride
  size_t dstride;       // floats between planes (record slab)
  int nch, mode;
  const double* stats;  // GNRELU: plane 0's reg stats (+ d * sstride), deconv j
  size_t sstride;
  int j;
  const float* gamma;
  const float* beta;
  float scale;          // staging scale (power of two)
  const unsigned* bound;// if set: scale = 2^-e with *bound 2^-e in [2^14, 2^15) (the cost slice x)
};
struct WgChunk {         // one 16-channel input chunk (wgrad2), resolved on the host
  const float* ptr;     // plane 0's tensor at the chunk's first channel; plane d at + d * dstride
  size_t dstride;
  int nch, mode;        // the part's channel count (pixel stride), mode
  int nv;               // valid channels of the chunk (16 or 8)
  int j;                // GNRELU: deconv index
  const double* stats;  // GNRELU: plane 0's reg stats (+ d * sstride)
  size_t sstride;
  const float* gamma;   // GNRELU: at the chunk's first channel
  const float* beta;
  int gn0;              // GNRELU: GroupNorm group of the chunk's first channel
  float scale;
  const unsigned* bound;
};
struct WgradArgs {
  const float* gz;        // [G][P][CZ]
  const unsigned* zmax;   // [G] per-plane scales of gz
  WgPart part[3];
  WgChunk chunk[3];
  int gn_chunk;           // wgrad2: the GNRELU chunk (its statistics tabled in LDS), or -1
  double* rseg;           // reduction segments (BpttLayout::rseg)
  int nparts, cin;        // input channels (valid)
  int nplanes, d0;        // group planes: record plane d0 + k  <->  gz slot k
  int B, H, W;            // cell resolution
  float* wpart;           // [gridDim.x][kWgPartMax]: [CZ][cin_pad][9] then bias [CZ]
};

// ---------------------------------------------------------------------------
// wgrad2: all input chunks in one block: each (plane, 4 x 32 tile) item is staged once for
// every input chunk, and the next item's global operands are loaded into registers while the
// current item's MFMAs run.  The input is staged once per channel, column c of a row at half 8 + c; a
// lane's B fragment for tap column dx is its aligned 8 columns shifted by dx - 1, assembled
// from the aligned 16 B and one neighbouring dword with v_alignbit (no shifted copies).
// LDS rows are padded so that the 16 lanes of a fragment read hit 16 different bank groups.
// 512 threads: wave w owns gate m-tile w % (CZ/16) and a share of the (chunk, tap row) combos.
// ---------------------------------------------------------------------------
constexpr int kW2TH = 4;                          // tile rows (x 32 columns)
constexpr int kW2ZS = kW2TH * 32 + 8;             // halves per gate channel
constexpr int kW2RL = 48;                         // halves per input row (columns -2 .. 33 at 6 .. 41)
constexpr int kW2IS = (kW2TH + 2) * kW2RL + 8;    // halves per input channel

template <int CZ, int NCH>
constexpr size_t wgrad2_lds() {
  return (size_t)2 * CZ * kW2ZS * 2 + (size_t)2 * NCH * 16 * kW2IS * 2;
}

template <int CZ, int NCH>
__global__ void __launch_bounds__(512) wgrad2_kernel(WgradArgs a) {
  constexpr int MT = CZ / 16, NS = 8 / MT;
  constexpr int NCOMBO = NCH * 3, CPW = (NCOMBO + NS - 1) / NS;
  constexpr int CIN = NCH * 16, NG = CZ / 8;
  constexpr int NU = (kW2TH + 2) * 18 * NCH;               // input staging units (2 px x 16 ch)
  static_assert(NU <= 512, "one input unit per thread");
  extern __shared__ __attribute__((aligned(16))) char lds_w2[];
  _Float16* zt = reinterpret_cast<_Float16*>(lds_w2);       // [2][CZ][kW2ZS]
  _Float16* it = zt + 2 * CZ * kW2ZS;                         // [2][CIN][kW2IS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_x = (a.W + 31) / 32, tiles_y = (a.H + kW2TH - 1) / kW2TH;
  const int ntile = a.B * tiles_x * tiles_y;
  const int nitem = ntile * a.nplanes;
  // staging scale of a chunk
  // GroupNorm+ReLU chunks: bound 2^-e in [2^14, 2^15) (the forward cells' staging scale,
  // gn_relu_bound), so that neither fp16 overflows nor the lo parts of small values go subnormal
  auto chunk_scale = [&](const WgChunk& ch) {
    if (ch.bound) return ldexpf(1.0f, -scale_exp(*ch.bound));
    if (ch.mode == WG_GNRELU) {
      const float bnd = gn_relu_bound(ch.gamma - 8 * ch.gn0, ch.beta - 8 * ch.gn0, 8.0 * a.H * a.W);
      if (bnd > 0.0f) {
        const int k = ilogbf(bnd);
        return ldexpf(1.0f, -(k >= 134 ? 120 : (k < -100 ? -114 : k - 14)));
      }
    }
    return ch.scale;
  };
  auto item_pos = [&](int item, int& k, int& b, int& y0, int& x0) {
    k = item / ntile;
    const int tile = item % ntile;
    b = tile / (tiles_x * tiles_y);
    const int rem = tile % (tiles_x * tiles_y);
    y0 = (rem / tiles_x) * kW2TH;
    x0 = (rem % tiles_x) * 32;
  };
  // staging roles
  const bool zrole = tid < 64 * NG;
  const int zpp = tid / NG, zcg = tid % NG;                  // pixel pair (row zpp / 16), channel group
  const int zr = zpp >> 4, zx = 2 * (zpp & 15);
  struct Pre {
    float4 z[4];
    float4 in[2][2][2];   // [8-channel half][pixel][float4]
  };
  float bacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) bacc[i] = 0.f;
  // input unit of this thread: chunk uc, tile row rr - 1, columns 2 ucp - 2, 2 ucp - 1
  const bool irole = tid < NU;
  const int uc = tid % NCH, ucp = (tid / NCH) % 18, urr = tid / (NCH * 18);
  const WgChunk uch = a.chunk[uc];            // this thread's chunk, for every item
  // GroupNorm statistics of the GNRELU chunk for the group's planes: [k][b][group]
  float2* gst = reinterpret_cast<float2*>(it + 2 * CIN * kW2IS);
  if (a.gn_chunk >= 0) {
    const WgChunk& gc = a.chunk[a.gn_chunk];
    for (int e = tid; e < a.nplanes * a.B * 2; e += 512) {
      const int kk = e / (2 * a.B), bb = (e >> 1) % a.B, g = e & 1;
      const GnStat st = stat_read(gc.stats + (size_t)(a.d0 + kk) * gc.sstride + reg_stat_index(bb, gc.j, g),
                                  8.0 * a.H * a.W);
      gst[e] = make_float2(st.mean, st.rstd);
    }
  }
  const float usc = chunk_scale(uch);
  const float zs = ldexpf(1.0f, -scale_exp(a.zmax[0]));   // the group's slots share one exponent
  auto fetch = [&](int item) {
    Pre pf;
    float4(&zq)[4] = pf.z;
    int k, b, y0, x0;
    item_pos(item, k, b, y0, x0);
    if (zrole) {
      const float* gzp = a.gz + (size_t)k * a.B * a.H * a.W * CZ;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int gy = y0 + zr, gx = x0 + zx + h;
        if (gy < a.H && gx < a.W) {
          const float4* s4 = reinterpret_cast<const float4*>(gzp + (((size_t)b * a.H + gy) * a.W + gx) * CZ + 8 * zcg);
          zq[2 * h] = s4[0];
          zq[2 * h + 1] = s4[1];
        } else {
          zq[2 * h] = zq[2 * h + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int h = 0; h < 2; ++h) pf.in[hh][h][0] = pf.in[hh][h][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (irole) {
      const int gy = y0 - 1 + urr;
      if (uch.mode != WG_POOL && gy >= 0 && gy < a.H) {
        const float* bb = uch.ptr + (size_t)(a.d0 + k) * uch.dstride + (size_t)b * a.H * a.W * uch.nch;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          if (8 * hh >= uch.nv) continue;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int gx = x0 + 2 * ucp - 2 + h;
            if (gx >= 0 && gx < a.W) {
              const float4* s4 = reinterpret_cast<const float4*>(bb + ((size_t)gy * a.W + gx) * uch.nch + 8 * hh);
              pf.in[hh][h][0] = s4[0];
              pf.in[hh][h][1] = s4[1];
            }
          }
        }
      }
    }
    return pf;
  };
  // D accumulators: combo i (chunk c = q / 3, tap row dy = q % 3, q = s + NS i) x tap column dx
  const int mt = wave % MT, sgrp = wave / MT;
  bfloatx4 acc[CPW][3];
#pragma unroll
  for (int i = 0; i < CPW; ++i)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) acc[i][dx] = bfloatx4{0.f, 0.f, 0.f, 0.f};
  const int item0 = blockIdx.x;
  Pre pre;
  if (item0 < nitem) pre = fetch(item0);
  // sign-balanced accumulation (convlstm.hip h3_mfma_chunk): odd items stage -gz and the
  // accumulators are negated between items, so they hold (-1)^item x the running sums and the
  // MFMAs' low-side drift alternates sign
  float zsg = zs;
#pragma unroll 1
  for (int item = item0; item < nitem; item += gridDim.x) {
    int k, b, y0, x0;
    item_pos(item, k, b, y0, x0);
    if (item != item0) {
      zsg = -zsg;
#pragma unroll
      for (int i = 0; i < CPW; ++i)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) acc[i][dx] = -acc[i][dx];
    }
    __syncthreads();   // the previous item's fragment reads are done
    const float4(&zq)[4] = pre.z;
    if (zrole) {
      const float v0[8] = {zq[0].x, zq[0].y, zq[0].z, zq[0].w, zq[1].x, zq[1].y, zq[1].z, zq[1].w};
      const float v1[8] = {zq[2].x, zq[2].y, zq[2].z, zq[2].w, zq[3].x, zq[3].y, zq[3].z, zq[3].w};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        bacc[i] += v0[i] + v1[i];
        half2v hp, lp;
        split16x2(v0[i] * zsg, v1[i] * zsg, hp, lp);
        const int o = (8 * zcg + i) * kW2ZS + zr * 32 + zx;
        *reinterpret_cast<unsigned*>(zt + o) = __builtin_bit_cast(unsigned, hp);
        *reinterpret_cast<unsigned*>(zt + CZ * kW2ZS + o) = __builtin_bit_cast(unsigned, lp);
      }
    }
    if (irole) {
      const int c = uc, cp = ucp, rr = urr;
      const int gy = y0 - 1 + rr;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const bool valid = 8 * hh < uch.nv;
        float v[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4* q = pre.in[hh][h];
          v[h][0] = q[0].x; v[h][1] = q[0].y; v[h][2] = q[0].z; v[h][3] = q[0].w;
          v[h][4] = q[1].x; v[h][5] = q[1].y; v[h][6] = q[1].z; v[h][7] = q[1].w;
        }
        if (uch.mode == WG_POOL && valid) {
          // 2x2 max-pool of the finer state, loaded here (cells 1 and 2)
          const int Ws = 2 * a.W;
          const float* bb = uch.ptr + (size_t)(a.d0 + k) * uch.dstride + (size_t)b * 4 * a.H * a.W * uch.nch;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int gx = x0 + 2 * cp - 2 + h;
            if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
              const float* s0 = bb + ((size_t)(2 * gy) * Ws + 2 * gx) * uch.nch + 8 * hh;
#pragma unroll 1
              for (int w = 0; w < 4; ++w) {
                const float4* s4 = reinterpret_cast<const float4*>(s0 + ((w >> 1) * Ws + (w & 1)) * uch.nch);
                const float4 a0 = s4[0], a1 = s4[1];
                const float qq[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
                for (int i = 0; i < 8; ++i) v[h][i] = w == 0 ? qq[i] : fmaxf(v[h][i], qq[i]);
              }
            }
          }
        } else if (uch.mode == WG_GNRELU && valid) {
          const float2 ms = gst[(k * a.B + b) * 2 + uch.gn0 + hh];
          const GnStat gs{ms.x, ms.y};
          const bool in0 = gy >= 0 && gy < a.H && x0 + 2 * cp - 2 >= 0 && x0 + 2 * cp - 2 < a.W;
          const bool in1 = gy >= 0 && gy < a.H && x0 + 2 * cp - 1 >= 0 && x0 + 2 * cp - 1 < a.W;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float gsc = gs.rstd * uch.gamma[8 * hh + i];
            const float gsh = uch.beta[8 * hh + i] - gs.mean * gsc;
            v[0][i] = in0 ? fmaxf(fmaf(v[0][i], gsc, gsh), 0.0f) : 0.0f;
            v[1][i] = in1 ? fmaxf(fmaf(v[1][i], gsc, gsh), 0.0f) : 0.0f;
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          half2v hp, lp;
          split16x2(v[0][i] * usc, v[1][i] * usc, hp, lp);
          const int o = (16 * c + 8 * hh + i) * kW2IS + rr * kW2RL + 6 + 2 * cp;
          *reinterpret_cast<unsigned*>(it + o) = __builtin_bit_cast(unsigned, hp);
          *reinterpret_cast<unsigned*>(it + CIN * kW2IS + o) = __builtin_bit_cast(unsigned, lp);
        }
        __builtin_amdgcn_sched_barrier(0);   // one half's values live at a time
      }
    }
    __syncthreads();
    if (item + (int)gridDim.x < nitem) pre = fetch(item + gridDim.x);   // in flight during the MFMAs
    const int ar = lane & 15, g = lane >> 4;
#pragma unroll 1
    for (int r = 0; r < kW2TH; ++r) {
      const int ao = (16 * mt + ar) * kW2ZS + r * 32 + 8 * g;
      const bhalf8 zh = *reinterpret_cast<const bhalf8*>(zt + ao);
      const bhalf8 zl = *reinterpret_cast<const bhalf8*>(zt + CZ * kW2ZS + ao);
#pragma unroll
      for (int i = 0; i < CPW; ++i) {
        const int q = sgrp + NS * i;
        if (q < NCOMBO) {
          const int c = q / 3, dy = q % 3;
          const int bo = (16 * c + ar) * kW2IS + (r + dy) * kW2RL + 8 + 8 * g;
          bhalf8 bf[2][3];
#pragma unroll
          for (int hl = 0; hl < 2; ++hl) {
            const _Float16* src = it + hl * CIN * kW2IS + bo;
            const uint4 U = *reinterpret_cast<const uint4*>(src);
            const unsigned pv = *reinterpret_cast<const unsigned*>(src - 2);
            const unsigned nx = *reinterpret_cast<const unsigned*>(src + 8);
            const unsigned s0 = __builtin_amdgcn_alignbit(U.x, pv, 16);
            const unsigned s1 = __builtin_amdgcn_alignbit(U.y, U.x, 16);
            const unsigned s2 = __builtin_amdgcn_alignbit(U.z, U.y, 16);
            const unsigned s3 = __builtin_amdgcn_alignbit(U.w, U.z, 16);
            const unsigned s4 = __builtin_amdgcn_alignbit(nx, U.w, 16);
            bf[hl][0] = __builtin_bit_cast(bhalf8, make_uint4(s0, s1, s2, s3));
            bf[hl][1] = __builtin_bit_cast(bhalf8, U);
            bf[hl][2] = __builtin_bit_cast(bhalf8, make_uint4(s1, s2, s3, s4));
          }
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) {
            acc[i][dx] = __builtin_amdgcn_mfma_f32_16x16x32_f16(zh, bf[0][dx], acc[i][dx], 0, 0, 0);
            acc[i][dx] = __builtin_amdgcn_mfma_f32_16x16x32_f16(zh, bf[1][dx], acc[i][dx], 0, 0, 0);
            acc[i][dx] = __builtin_amdgcn_mfma_f32_16x16x32_f16(zl, bf[0][dx], acc[i][dx], 0, 0, 0);
            acc[i][dx] = __builtin_amdgcn_mfma_f32_16x16x32_f16(zl, bf[1][dx], acc[i][dx], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);   // one combo's fragments live at a time
      }
    }
  }
  // the group's zmax slots share one exponent (zmax_group_kernel); the accumulators' sign
  const float zinv = zsg < 0.f ? -ldexpf(1.0f, scale_exp(a.zmax[0])) : ldexpf(1.0f, scale_exp(a.zmax[0]));
  float* wp = a.wpart + (size_t)blockIdx.x * kWgPartMax;
  const int cinp = 16 * ((a.cin + 15) / 16);
#pragma unroll
  for (int i = 0; i < CPW; ++i) {
    const int q = sgrp + NS * i;
    if (q < NCOMBO) {
      const int c = q / 3, dy = q % 3;
      const float inv = zinv / chunk_scale(a.chunk[c]);
      const int ci = 16 * c + (lane & 15);
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          const int cz = 16 * mt + 4 * (lane >> 4) + rg;
          wp[((size_t)cz * cinp + ci) * 9 + 3 * dy + dx] = acc[i][dx][rg] * inv;
        }
    }
  }
  // bias: thread tid staged channel group tid % NG of pixel pair tid / NG in every item
  __syncthreads();
  float* bred = reinterpret_cast<float*>(lds_w2);   // [64 NG][8]
  if (zrole) {
#pragma unroll
    for (int i = 0; i < 8; ++i) bred[tid * 8 + i] = bacc[i];
  }
  __syncthreads();
  if (tid < CZ) {
    const int cg = tid / 8, i = tid % 8;
    float sb = 0.f;
    for (int t = cg; t < 64 * NG; t += NG) sb += bred[t * 8 + i];
    wp[(size_t)CZ * cinp * 9 + tid] = sb;
  }
}

// Partials -> fp64 accumulators, deterministic, in two passes: pass 1 sums each entry over
// kRedSeg contiguous segments of the nblk partials (blockIdx.y = segment), pass 2 sums the
// segments in order into the destination (wgrad: raw layout [cz][cin][3][3] then bias [cz],
// from the partials' [cz][cin_pad][9] + bias; identity: entries < nw to gw, the rest to gb).
__global__ void __launch_bounds__(256) seg_reduce_kernel(const float* __restrict__ part, int nblk,
                                                         int stride, int n, double* __restrict__ seg) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const int k0 = (int)((long)blockIdx.y * nblk / kRedSeg), k1 = (int)((long)(blockIdx.y + 1) * nblk / kRedSeg);
  double s = 0.0;
  for (int k = k0; k < k1; ++k) s += part[(size_t)k * stride + e];
  seg[(size_t)blockIdx.y * n + e] = s;
}

__global__ void __launch_bounds__(256) seg_final_kernel(const double* __restrict__ seg, int n_src, int cz,
                                                        int cin, int n, int nw, double* __restrict__ gw,
                                                        double* __restrict__ gb) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  int src = e;
  if (cz > 0) {   // wgrad layout
    const int cinp = 16 * ((cin + 15) / 16);
    if (e < cz * cin * 9) {
      const int tap = e % 9, ci = (e / 9) % cin, z = e / (9 * cin);
      src = (z * cinp + ci) * 9 + tap;
    } else {
      src = cz * cinp * 9 + (e - cz * cin * 9);
    }
  }
  double s = 0.0;
  for (int k = 0; k < kRedSeg; ++k) s += seg[(size_t)k * n_src + src];
  if (e < nw)
    gw[e] += s;
  else
    gb[e - nw] += s;
}

static hipError_t reduce_partials(const float* part, int nblk, int stride, int n_src, int cz, int cin, int n,
                                  int nw, double* rseg, double* gw, double* gb, hipStream_t s) {
  hipLaunchKernelGGL(seg_reduce_kernel, dim3((n_src + 255) / 256, kRedSeg), dim3(256), 0, s, part, nblk,
                     stride, n_src, rseg);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(seg_final_kernel, dim3((n + 255) / 256), dim3(256), 0, s, rseg, n_src, cz, cin, n, nw,
                     gw, gb);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// deconv_j weight / bias gradient over a group: gW[ci][co][ky][kx] = sum_{d, iy, ix}
// h[iy][ix][ci] gu[2iy-1+ky][2ix-1+kx][co], gb[co] = sum gu.  Per tap a 16 x 16 GEMM over the
// pixels on v_mfma_f32_16x16x4_f32 (fp32 operands: the products are exact as in the
// reference's fp32 conv): A = h^T (16 ci x 4 px), B = gu at the tap (4 px x 16 co).  Blocks
// stride over 64-pixel runs of the coarse image (per plane), with the run's h and its gu rows
// staged in LDS; wave w owns taps w, w + 4, w + 8; one partial per block (2304 + 16 floats).
// ---------------------------------------------------------------------------
constexpr int kDcwBlocks = 1024, kDcwPart = 2320;
struct DcwArgs {
  const float* h;       // coarse input plane 0 (record state slab of d0 + 1: h' of the
  size_t hstride;       //   deconv's source cell), + k * hstride
  const float* gu;      // [G][B][Ho][Wo][16]
  int nplanes, B, Hi, Wi;
  float* wpart;         // [gridDim.x][kDcwPart]
};

__global__ void __launch_bounds__(256) deconv_wgrad_kernel(DcwArgs a) {
  __shared__ float hs[64][17];
  __shared__ float gs[3][130][17];   // fine rows 2y-1 .. 2y+1, cols 2x0-1 .. 2x0+128
  __shared__ float bred[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Ho = 2 * a.Hi, Wo = 2 * a.Wi;
  const int runs_x = (a.Wi + 63) / 64;
  const int nrun = a.nplanes * a.B * a.Hi * runs_x;
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 acc[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;
  const int m = lane & 15, kq = lane >> 4;
#pragma unroll 1
  for (int run = blockIdx.x; run < nrun; run += gridDim.x) {
    int t = run;
    const int rx = t % runs_x;
    t /= runs_x;
    const int iy = t % a.Hi;
    t /= a.Hi;
    const int b = t % a.B, k = t / a.B;
    const int x0 = rx * 64;
    __syncthreads();
    // staging: one float4 (4 channels of a pixel) per load
    const float* hp = a.h + (size_t)k * a.hstride + ((size_t)b * a.Hi + iy) * a.Wi * 16;
    {
      const int px = tid >> 2, c4 = (tid & 3) * 4;   // 64 px x 4 quads = 256 threads
      const float4 v = x0 + px < a.Wi ? *reinterpret_cast<const float4*>(hp + (size_t)(x0 + px) * 16 + c4)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
      hs[px][c4] = v.x;
      hs[px][c4 + 1] = v.y;
      hs[px][c4 + 2] = v.z;
      hs[px][c4 + 3] = v.w;
    }
    const float* gp = a.gu + ((size_t)k * a.B + b) * Ho * Wo * 16;
    for (int e = tid; e < 3 * 130 * 4; e += 256) {
      const int c4 = (e & 3) * 4, pc = e >> 2, rr = pc / 130, cc = pc - rr * 130;
      const int oy = 2 * iy - 1 + rr, ox = 2 * x0 - 1 + cc;
      const float4 v = (oy >= 0 && oy < Ho && ox >= 0 && ox < Wo)
                           ? *reinterpret_cast<const float4*>(gp + ((size_t)oy * Wo + ox) * 16 + c4)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      gs[rr][cc][c4] = v.x;
      gs[rr][cc][c4 + 1] = v.y;
      gs[rr][cc][c4 + 2] = v.z;
      gs[rr][cc][c4 + 3] = v.w;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int tap = wave + 4 * i;
      if (tap < 9) {
        const int dy = tap / 3, dx = tap % 3;
#pragma unroll 4
        for (int p0 = 0; p0 < 64; p0 += 4) {
          const int px = p0 + kq;
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(hs[px][m], gs[dy][2 * px + dx][m], acc[i], 0, 0, 0);
        }
      }
    }
    if (tid < 64) {   // bias: each fine pixel of the run's owned quads once; lane phase tid >> 4
      const int co = tid & 15, ph = tid >> 4;
      const int npx = min(64, a.Wi - x0);
      float s = 0.f;
      for (int px = ph; px < npx; px += 4)
        s += gs[1][2 * px + 1][co] + gs[1][2 * px + 2][co] + gs[2][2 * px + 1][co] + gs[2][2 * px + 2][co];
      bacc += s;
    }
  }
  float* wp = a.wpart + (size_t)blockIdx.x * kDcwPart;
  // D: row = ci = 4 (lane >> 4) + r, col = co = lane & 15; entry (ci * 16 + co) * 9 + tap
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int tap = wave + 4 * i;
    if (tap < 9)
#pragma unroll
      for (int r = 0; r < 4; ++r) wp[((4 * kq + r) * 16 + m) * 9 + tap] = acc[i][r];
  }
  if (tid < 64) bred[tid] = bacc;
  __syncthreads();
  if (tid < 16) wp[2304 + tid] = (bred[tid] + bred[16 + tid]) + (bred[32 + tid] + bred[48 + tid]);
}

// conv_0 (head) weight / bias gradient over a group: gW[ci][tap] = sum gcost[p] h4[p + off][ci],
// gb = sum gcost.  A lane pair per (sample, pixel) walks the group's planes, lane h taking input
// channels 4 h .. 4 h + 3 (one 16-B load per tap, 36 sums): the tap offsets and their in-image
// tests are formed once, and every plane's 9 loads are unconditional (a tap outside the image
// reads its clamped neighbour with a zero weight), so they issue together.  Block reduce of the
// 73 sums through LDS, one partial of kHwPart floats per block.  (Round 6, second session: the thread-per-
// (plane, pixel) form -- three runtime divisions per pixel and a branch around every tap's loads
// -- took 432 us per 16-plane group at 640x512, latency-bound on the loads one tap at a time; the
// transposed form 454 us.)
constexpr int kHwBlocks = 1024, kHwPart = 80;
static_assert((size_t)kHwBlocks * kHwPart <= (size_t)kWgBlocks * kWgPartMax, "head partials fit wpart");
struct HwArgs {
  const float* gcost;   // [B][D][H][W]
  const float* h4;      // record: h4' of plane d0 (state slab d0 + 1) + k * hstride
  size_t hstride;
  int nplanes, d0, D, B, H, W;
  float* wpart;
};

__global__ void __launch_bounds__(256) head_wgrad_kernel(HwArgs a) {
  __shared__ float part[256][37];   // the threads' sums (odd row stride: conflict-free)
  float s[37];   // [c][tap] for channels 4 h + c, then (h = 0) the bias sum
#pragma unroll
  for (int i = 0; i < 37; ++i) s[i] = 0.f;
  const uint32_t HW = (uint32_t)a.H * (uint32_t)a.W, W = (uint32_t)a.W;
  const uint32_t n = 2u * (uint32_t)a.B * HW;
  const uint32_t h = threadIdx.x & 1u;
  for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < n; t += gridDim.x * 256u) {
    const uint32_t bp = t >> 1, b = bp / HW, p = bp - b * HW;
    const int y = (int)(p / W), x = (int)(p - (uint32_t)y * W);
    uint32_t off[9];
    unsigned ok = 0u;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int qy = y + tap / 3 - 1, qx = x + tap % 3 - 1;
      if (qy >= 0 && qy < a.H && qx >= 0 && qx < a.W) ok |= 1u << tap;
      const int cy = min(max(qy, 0), a.H - 1), cx = min(max(qx, 0), a.W - 1);
      off[tap] = ((uint32_t)cy * W + (uint32_t)cx) * 8u + 4u * h;
    }
    const float* gp = a.gcost + ((size_t)b * a.D + a.d0) * HW + p;
    const float* hb = a.h4 + (size_t)b * HW * 8;
#pragma unroll 1
    for (int k = 0; k < a.nplanes; ++k) {
      const float g = gp[(size_t)k * HW];
      const float* hk = hb + (size_t)k * a.hstride;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const float4 q = *reinterpret_cast<const float4*>(hk + off[tap]);
        const float gt = (ok >> tap) & 1u ? g : 0.f;
        s[0 * 9 + tap] = fmaf(gt, q.x, s[0 * 9 + tap]);
        s[1 * 9 + tap] = fmaf(gt, q.y, s[1 * 9 + tap]);
        s[2 * 9 + tap] = fmaf(gt, q.z, s[2 * 9 + tap]);
        s[3 * 9 + tap] = fmaf(gt, q.w, s[3 * 9 + tap]);
      }
      s[36] += h ? 0.f : g;
    }
  }
  // block reduce in LDS, in a fixed order: sum t of this block's threads of parity hh for sum i
  // (a register butterfly over 73 values took the kernel to 256 VGPRs, one wave per SIMD)
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 37; ++i) part[threadIdx.x][i] = s[i];
  __syncthreads();
  if (threadIdx.x < 74) {
    const int hh = threadIdx.x / 37, i = threadIdx.x - 37 * hh;
    float acc = 0.f;
#pragma unroll 8
    for (int t = hh; t < 256; t += 2) acc += part[t][i];
    float* wp = a.wpart + (size_t)blockIdx.x * kHwPart;
    if (i < 36)
      wp[36 * hh + i] = acc;   // [ci = 4 hh + i / 9][tap = i % 9]
    else if (hh == 0)
      wp[72] = acc;            // the bias sum (lanes of parity 0 hold it)
  }
}

__global__ void gacc_to_float_kernel(const double* __restrict__ gacc, float* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = (float)gacc[i];
}

// Diagnostic trace (AARMVS_BWD_TRACE=1): after every kernel of the plane chain a position-
// weighted checksum of what it wrote, at [plane][slot] of a device log that
// aarmvs_debug_bwd_trace (not part of the ABI) copies out.  Runs of a schedule are compared
// entry by entry: the first differing entry names the kernel whose output first differs.
constexpr int kTraceSlots = 32;
static unsigned long long* g_trace = nullptr;
static int g_trace_planes = 0;
__global__ void __launch_bounds__(256) cksum_kernel(const unsigned* __restrict__ p, size_t n,
                                                   unsigned long long* out) {
  __shared__ unsigned long long red[256];
  unsigned long long acc = 0;
  for (size_t i = threadIdx.x; i < n; i += 256) acc += (unsigned long long)p[i] * (1 + (i % 61));
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

// every plane of a group shares the largest scale exponent: zmax[slot] <- max over the slots
__global__ void __launch_bounds__(256) zmax_group_kernel(const unsigned* zpart, int stride, int nb, int n,
                                                         unsigned* zmax) {
  unsigned m = 0;
  for (int i = 0; i < n; ++i) m = max(m, block_max_of(zpart + (size_t)i * stride, nb));
  if ((int)threadIdx.x < n) zmax[threadIdx.x] = m;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static hipError_t run_gate_bwd(const GateBwdArgs& a, hipStream_t s, int kid) {
  const size_t n = (size_t)a.B * a.H * a.W * (a.hid / 4);
  if ((size_t)a.B * a.H * a.W * a.hid >= (1ull << 31)) return hipErrorInvalidValue;   // 32-bit indices
  ProfScope ps(s, kid);
  hipLaunchKernelGGL(gate_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int CZ>
static hipError_t run_dgrad(const DgradArgs& a, hipStream_t s, int kid) {
  constexpr size_t lds = (size_t)(CZ / 16) * 9 * 2 * 512 * 2 + 2 * kDgNPIX * 32;
  static bool attr[kMaxDevices] = {};
  if (hipError_t e = ensure_dyn_lds((const void*)dgrad_kernel<CZ>, (int)lds, attr); e != hipSuccess)
    return e;
  const int tiles = a.B * ((a.W + kDgTW - 1) / kDgTW) * ((a.H + kDgTH - 1) / kDgTH);
  const int mtn = (a.cout + 31) / 32;
  // persistent blocks: as many as the CUs hold (LDS-bound), split over the m-tiles
  const int cu = cu_count();
  const int per_cu = std::max(1, (int)((160 * 1024) / lds));
  const int grid = std::max(1, std::min(tiles, std::max(1, cu * per_cu / mtn)));
  ProfScope ps(s, kid);
  hipLaunchKernelGGL(dgrad_kernel<CZ>, dim3(grid, mtn), dim3(512), lds, s, a);
  return hipGetLastError();
}

// the 16-channel input chunks of a cell conv's parts
static void fill_chunks(WgradArgs& a) {
  int c = 0;
  for (int pi = 0; pi < a.nparts; ++pi) {
    const WgPart& p = a.part[pi];
    for (int lc = 0; lc < p.nch && c < 3; lc += 16, ++c) {
      WgChunk& ch = a.chunk[c];
      ch.ptr = p.ptr + lc;
      ch.dstride = p.dstride;
      ch.nch = p.nch;
      ch.mode = p.mode;
      ch.nv = std::min(16, p.nch - lc);
      ch.j = p.j;
      ch.stats = p.stats;
      ch.sstride = p.sstride;
      ch.gamma = p.gamma ? p.gamma + lc : nullptr;
      ch.beta = p.beta ? p.beta + lc : nullptr;
      ch.gn0 = lc / 8;
      ch.scale = p.scale;
      ch.bound = p.bound;
    }
  }
}

template <int CZ, int NCH>
static hipError_t run_wgrad(WgradArgs a, double* gw, double* gb, hipStream_t s, int kid) {
  fill_chunks(a);
  a.gn_chunk = -1;
  for (int c = 0; c < NCH; ++c)
    if (a.chunk[c].mode == WG_GNRELU) a.gn_chunk = c;
  const size_t lds = wgrad2_lds<CZ, NCH>() + (size_t)kPlaneGroup * a.B * 2 * sizeof(float2);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static bool attr[kMaxDevices] = {};
  if (hipError_t e = ensure_dyn_lds((const void*)wgrad2_kernel<CZ, NCH>, 160 * 1024, attr); e != hipSuccess)
    return e;
  {
    ProfScope ps(s, kid);
    hipLaunchKernelGGL((wgrad2_kernel<CZ, NCH>), dim3(kWgBlocks), dim3(512), lds, s, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  ProfScope ps(s, K_BWD_SMALL);
  return reduce_partials(a.wpart, kWgBlocks, (int)kWgPartMax, CZ * 16 * NCH * 9 + CZ, CZ, a.cin,
                         CZ * a.cin * 9 + CZ, CZ * a.cin * 9, a.rseg, gw, gb, s);
}

}  // namespace aarmvs

namespace aarmvs {

size_t bptt_scratch_bytes(int B, int H, int W) { return bptt_layout(nullptr, B, H, W).bytes; }

// A cross-stream dependency of the backward's schedules.  AARMVS_BWD_HOSTSYNC=1 (diagnostic)
// makes the host wait for the event instead of the consumer stream (same ordering, no device-side
// wait), to tell a missing dependency from a device-side event problem.
static hipError_t xwait(hipStream_t consumer, hipEvent_t ev) {
  static const bool host = [] {
    const char* v = getenv("AARMVS_BWD_HOSTSYNC");
    return v && atoi(v) != 0;
  }();
  return host ? hipEventSynchronize(ev) : hipStreamWaitEvent(consumer, ev, 0);
}

// The regulariser's backward over every plane (last first), in groups of kPlaneGroup planes:
// per plane the gate / dgrad / GroupNorm / deconv chain; per group the weight gradients and
// then `group_done(g0, n, gx)` (the cost-slice backward of the group's dL/dx, or a copy-out).
hipError_t bptt_regulariser(const BpttRun& r, hipStream_t s) {
  const ParamLayout& PL = param_layout();
  const int B = r.B, H = r.H, W = r.W, D = r.D;
  const TrainLayout T = train_layout(B, H, W);
  BpttLayout L = bptt_layout(r.scratch, B, H, W);
  const float* pk = r.packed;
  const aarmvs_train_record& rec = *r.rec;
  const int G = kPlaneGroup;
  const size_t HW = (size_t)H * W;
  hipError_t e;
#define CK(x)                             \
  do {                                    \
    if ((e = (x)) != hipSuccess) return e; \
  } while (0)
  // state gradients start at zero after the last plane; parameter accumulators at zero
  for (int k = 0; k < 5; ++k) {
    CK(hipMemsetAsync(L.gh[k], 0, L.cell_px[k] * kCellHid[k] * 4, s));
    CK(hipMemsetAsync(L.gc[k], 0, L.cell_px[k] * kCellHid[k] * 4, s));
  }
  CK(hipMemsetAsync(L.gacc, 0, PL.raw_total * 8, s));
  const int res_div[5] = {1, 2, 4, 2, 1};
  auto zslot = [&](int k, int slot) { return L.gz[k] + (size_t)slot * L.cell_px[k] * 4 * kCellHid[k]; };
  // blocks of cell k's gate kernel (run_gate_bwd): hid / 4 threads per cell pixel
  auto gate_blocks = [&](int k) { return (int)((L.cell_px[k] * (kCellHid[k] / 4) + 255) / 256); };
  auto gate = [&](hipStream_t s, int k, int slot, const UnetIO& io, int mode, int d, const float* gh_add = nullptr) {
    GateBwdArgs a{};
    a.z = io.z[k];
    a.c_prev = io.c_prev[k];
    a.c_new = io.c_new[k];
    a.gh = L.gh[k];
    a.gh_add = gh_add;
    a.gc = L.gc[k];
    a.gz = zslot(k, slot);
    a.zpart = L.zpart + ((size_t)k * G + slot) * L.zp_n;
    a.mode = mode;
    a.B = B;
    a.H = H / res_div[k];
    a.W = W / res_div[k];
    a.hid = kCellHid[k];
    if (mode == 1) {
      a.gcost = r.grad_cost + (size_t)d * HW;
      a.gcost_bstride = (int)((size_t)D * HW);
      a.whead = pk + PL.pk_off[P_HW];
    } else if (mode == 2) {
      a.gpool = L.gpool[k];
      a.hnew = io.h_new[k];
    }
    return run_gate_bwd(a, s, K_GATE_BWD0 + k);
  };
  auto dgrad = [&](hipStream_t s, int k, int slot, std::initializer_list<DgPart> parts) {
    DgradArgs a{};
    a.gz = zslot(k, slot);
    a.zpart = L.zpart + ((size_t)k * G + slot) * L.zp_n;
    a.nzp = gate_blocks(k);
    a.wfrag = pk + PL.dg_off[k];
    a.wscale = pk + PL.dg_scale_off + k;
    int i = 0;
    for (const DgPart& p : parts) a.part[i++] = p;
    a.nparts = i;
    a.cout = cell_cin(k);
    a.B = B;
    a.H = H / res_div[k];
    a.W = W / res_div[k];
    return kCellHid[k] == 16 ? run_dgrad<64>(a, s, K_DGRAD0 + k) : run_dgrad<32>(a, s, K_DGRAD0 + k);
  };
  // GroupNorm-backward partial blocks per (plane, sample) of deconv j's output
  auto gnb_nblk = [&](int j) {
    const size_t hwo = (size_t)(j ? H : H / 2) * (j ? W : W / 2);
    return std::max(1, std::min(L.gnb_nblk, (int)((hwo + 1023) / 1024)));
  };
  auto deconv_bwd = [&](hipStream_t s, int j, int slot, const UnetIO& io, float* gr) {
    const int Ho = j ? H : H / 2, Wo = j ? W : W / 2;
    const size_t hwo = (size_t)Ho * Wo;
    GnbArgs g{};
    g.gr = gr;
    g.u = j ? io.u1 : io.u0;
    g.stats = io.reg_stats;
    g.gamma = pk + PL.pk_off[j ? P_D1GW : P_D0GW];
    g.beta = pk + PL.pk_off[j ? P_D1GB : P_D0GB];
    const int nblk = gnb_nblk(j);
    g.part = L.gnb_part[j] + (size_t)slot * B * nblk * 36;
    g.j = j;
    g.HW = (int)hwo;
    {
      ProfScope ps(s, K_GNB_PARTIAL);
      hipLaunchKernelGGL(gnb_partial_kernel, dim3(nblk, B), dim3(256), 0, s, g);
    }
    CK(hipGetLastError());
    DcbArgs a{};
    a.gr = gr;
    a.u = g.u;
    a.stats = io.reg_stats;
    a.part = g.part;
    a.nblk = nblk;
    a.gamma = g.gamma;
    a.beta = g.beta;
    a.w = pk + PL.pk_off[j ? P_D1W : P_D0W];
    a.gu = L.gu[j] + (size_t)slot * B * hwo * 16;
    a.gh = L.gh[j ? 3 : 2];
    a.j = j;
    a.Hi = Ho / 2;
    a.Wi = Wo / 2;
    ProfScope ps(s, K_DECONV_BWD);
    hipLaunchKernelGGL(deconv_bwd_kernel, dim3((a.Hi * a.Wi + 63) / 64, B), dim3(256), 0, s, a);
    return hipGetLastError();
  };
  const size_t xs = T.x_plane;   // floats per plane of gx
  // Two-stage plane pipeline on two streams: stage A of plane d (cells 4 and 3 and the
  // deconv_1 backward) on the aux stream beside stage B of plane d + 1 (the deconv_0 backward,
  // cells 2, 1, 0) on the caller's stream.  The only values crossing from A to B are cell 3's
  // dL/d relu(GN(u_0)) and cells 4 and 3's skip-input gradients dL/dh0, dL/dh1: stored (not
  // added into gh[0], gh[1], which stage B of plane d + 1 still owns) into per-parity buffers
  // and added by cells 0 and 1's gate backward (the same single fp32 add: the same bits in
  // either schedule).  Events: evA[p] "stage A of a parity-p plane done" (aux -> main),
  // evB[p] "stage B of a parity-p plane done" (main -> aux: its parity buffers are free).
  // The group stage (weight gradients, dL/dx copy-out, the cost-slice backward of the group)
  // runs on a third stream beside the next group's planes: it reads only the group's buffer
  // set (gz, zmax, gu, gx, GroupNorm partials; two sets, by group parity) and the record, and
  // writes only the parameter accumulators and the cost-slice scratch, which the plane chain
  // never touches.  Events: evP "the group's planes done" (main -> group stream), evG[p] "the
  // group stage of a parity-p group done" (its set is free again).
  // AARMVS_BWD_PIPE: 1 the plane pipeline and the group overlap (default), 0 everything on the
  // caller's stream, 3 the plane pipeline alone, 2 the plane stages on two streams in order;
  // diagnostics: 4 the group stage on its stream but waited for at once, 5 the group overlap
  // without the plane pipeline.  Every schedule gives bit-identical gradients (every reduction
  // has a fixed order; tests/test_gpu_bptt.py::test_backward_schedules_are_bit_identical).  Until
  // round 5 the multi-stream ones did not: packed-fp32 device code (since disabled in the
  // Makefile) gave results that depended on what ran beside it.
  struct PipeSet {
    int dev = -1;
    hipStream_t aux = nullptr, grp = nullptr;   // the library's streams 1 and 2 (library_stream)
    hipEvent_t ev[9] = {};   // evA[2], evB[2], fork, evP, evG[2], group join
  };
  static thread_local PipeSet ps_dev[kMaxDevices];   // aux streams + events per device
  const int pipe_mode = [] {   // read per call (bench.py times the schedules side by side)
    const char* v = getenv("AARMVS_BWD_PIPE");
    return v ? atoi(v) : 1;
  }();
  // (under stream capture the backward stays on the caller's stream, as the sweep does)
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  CK(hipStreamIsCapturing(s, &cap));
  const bool pipe_on = pipe_mode != 0 && cap == hipStreamCaptureStatusNone;
  int dev = 0;
  CK(current_device(dev));
  PipeSet& ps = ps_dev[dev];
  hipStream_t sa = s, sg = s;
  const hipStream_t sg0 = s;   // the caller's stream
  if (pipe_on && !g_prof_on) {   // (per-kernel timing runs on one stream: isolated kernel spans)
    if (ps.dev != dev) {
      CK(library_stream(dev, 1, ps.aux));
      CK(library_stream(dev, 2, ps.grp));
      for (hipEvent_t& x : ps.ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
      ps.dev = dev;
    }
    if (pipe_mode != 5) sa = ps.aux;
    if (pipe_mode == 1 || pipe_mode == 4 || pipe_mode == 5) sg = ps.grp;
  }
  // every return from here on (errors included) leaves the aux streams' work ordered on s
  StreamJoin join{s, sa, ps.ev[4]};
  StreamJoin join_g{s, sg, ps.ev[8]};
  hipEvent_t* evA = ps.ev;
  hipEvent_t* evB = ps.ev + 2;
  hipEvent_t evP = ps.ev[5];
  hipEvent_t* evG = ps.ev + 6;
  auto gr0_of = [&](int d) { return (d & 1) ? L.gr0b : L.gr[0]; };
  static const bool trace = [] {
    const char* v = getenv("AARMVS_BWD_TRACE");
    return v && atoi(v) != 0;
  }();
  if (trace && g_trace_planes < D) {
    if (g_trace) CK(hipFree(g_trace));
    CK(hipMalloc(&g_trace, (size_t)D * kTraceSlots * 8));
    g_trace_planes = D;
  }
  if (trace) CK(hipMemsetAsync(g_trace, 0, (size_t)D * kTraceSlots * 8, s));
  auto tr = [&](hipStream_t st, int d, int slot, const void* ptr, size_t nfloats) -> hipError_t {
    if (!trace) return hipSuccess;
    hipLaunchKernelGGL(cksum_kernel, dim3(1), dim3(256), 0, st, static_cast<const unsigned*>(ptr), nfloats,
                       g_trace + (size_t)d * kTraceSlots + slot);
    return hipGetLastError();
  };
  const size_t hw4 = (size_t)B * (HW / 4) * 16, hw1 = (size_t)B * HW * 16;
  auto zsz = [&](int k) { return L.cell_px[k] * 4 * kCellHid[k]; };
  auto hsz = [&](int k) { return L.cell_px[k] * kCellHid[k]; };
  int gi = 0;
  for (int g0 = ((D - 1) / G) * G; g0 >= 0; g0 -= G, ++gi) {
    const int n = std::min(G, D - g0);
    L.use_set(gi & 1);
    if (sg != s && gi >= 2) CK(xwait(s, evG[gi & 1]));   // set free again
    if (sa != s) {   // the aux stream starts after everything the group's stage A overwrites is consumed
      CK(hipEventRecord(ps.ev[4], s));
      CK(xwait(sa, ps.ev[4]));
    }
    auto stage_a = [&](int d) -> hipError_t {
      const int k = d - g0, q = d & 1;
      const UnetIO io = unet_io_record(T, rec, d);
      CK(gate(sa, 4, k, io, 1, d));
      CK(tr(sa, d, 0, zslot(4, k), zsz(4)));
      CK(tr(sa, d, 1, L.gc[4], hsz(4)));
      CK(tr(sa, d, 2, L.zpart + ((size_t)4 * G + k) * L.zp_n, gate_blocks(4)));
      CK(dgrad(sa, 4, k, {{L.gr[1], 0, 16, 0}, {L.gskip[q][0], 16, 16, 0}, {L.gh[4], 32, 8, 0}}));
      CK(tr(sa, d, 3, L.gr[1], hw1));
      CK(tr(sa, d, 4, L.gskip[q][0], L.cell_px[0] * 16));
      CK(tr(sa, d, 5, L.gh[4], hsz(4)));
      CK(deconv_bwd(sa, 1, k, io, L.gr[1]));
      CK(tr(sa, d, 6, L.gu[1] + (size_t)k * hw1, hw1));
      CK(tr(sa, d, 7, L.gh[3], hsz(3)));
      CK(gate(sa, 3, k, io, 0, d));
      CK(tr(sa, d, 8, zslot(3, k), zsz(3)));
      CK(tr(sa, d, 9, L.gc[3], hsz(3)));
      CK(dgrad(sa, 3, k, {{gr0_of(d), 0, 16, 0}, {L.gskip[q][1], 16, 16, 0}, {L.gh[3], 32, 16, 0}}));
      CK(tr(sa, d, 10, gr0_of(d), hw4));
      CK(tr(sa, d, 11, L.gskip[q][1], L.cell_px[1] * 16));
      CK(tr(sa, d, 12, L.gh[3], hsz(3)));
      return hipSuccess;
    };
    auto stage_b = [&](int d) -> hipError_t {
      const int k = d - g0, q = d & 1;
      const UnetIO io = unet_io_record(T, rec, d);
      CK(deconv_bwd(s, 0, k, io, gr0_of(d)));
      CK(tr(s, d, 13, L.gu[0] + (size_t)k * hw4, hw4));
      CK(tr(s, d, 14, L.gh[2], hsz(2)));
      CK(gate(s, 2, k, io, 0, d));
      CK(tr(s, d, 15, zslot(2, k), zsz(2)));
      CK(tr(s, d, 16, L.gc[2], hsz(2)));
      CK(dgrad(s, 2, k, {{L.gpool[1], 0, 16, 0}, {L.gh[2], 16, 16, 0}}));
      CK(tr(s, d, 17, L.gpool[1], (size_t)B * (HW / 16) * 16));
      CK(tr(s, d, 18, L.gh[2], hsz(2)));
      CK(gate(s, 1, k, io, 2, d, L.gskip[q][1]));
      CK(tr(s, d, 19, zslot(1, k), zsz(1)));
      CK(tr(s, d, 20, L.gc[1], hsz(1)));
      CK(dgrad(s, 1, k, {{L.gpool[0], 0, 16, 0}, {L.gh[1], 16, 16, 0}}));
      CK(tr(s, d, 21, L.gpool[0], hw4));
      CK(tr(s, d, 22, L.gh[1], hsz(1)));
      CK(gate(s, 0, k, io, 2, d, L.gskip[q][0]));
      CK(tr(s, d, 23, zslot(0, k), zsz(0)));
      CK(tr(s, d, 24, L.gc[0], hsz(0)));
      CK(tr(s, d, 27, L.zpart + ((size_t)0 * G + k) * L.zp_n, gate_blocks(0)));
      CK(tr(s, d, 28, L.zpart + ((size_t)1 * G + k) * L.zp_n, gate_blocks(1)));
      CK(tr(s, d, 29, L.zpart + ((size_t)2 * G + k) * L.zp_n, gate_blocks(2)));
      CK(tr(s, d, 30, L.zpart + ((size_t)3 * G + k) * L.zp_n, gate_blocks(3)));
      CK(dgrad(s, 0, k, {{L.gx + (size_t)k * xs, 0, 32, 0}, {L.gh[0], 32, 16, 0}}));
      CK(tr(s, d, 25, L.gx + (size_t)k * xs, xs));
      CK(tr(s, d, 26, L.gh[0], hsz(0)));
      return hipSuccess;
    };
    // step i: stage A of plane g0 + n - 1 - i, stage B of the plane after it
    for (int i = 0; i <= n; ++i) {
      const int d = g0 + n - 1 - i;
      if (pipe_mode == 2 && sa != s) {   // diagnostic: B(d + 1), then A(d) after it (no overlap)
        if (i >= 1) {
          CK(xwait(s, evA[(d + 1) & 1]));
          CK(stage_b(d + 1));
        }
        if (i < n) {
          CK(hipEventRecord(evB[d & 1], s));
          CK(xwait(sa, evB[d & 1]));
          CK(stage_a(d));
          CK(hipEventRecord(evA[d & 1], sa));
        }
        continue;
      }
      if (i < n) {
        if (sa != s && i >= 2) CK(xwait(sa, evB[d & 1]));   // B(d + 2) done
        CK(stage_a(d));
        if (sa != s) CK(hipEventRecord(evA[d & 1], sa));
      }
      if (i >= 1) {
        if (sa != s) CK(xwait(s, evA[(d + 1) & 1]));
        CK(stage_b(d + 1));
        if (sa != s) CK(hipEventRecord(evB[(d + 1) & 1], s));
      }
    }
    // ---- the group stage: weight gradients of the group, then its cost-slice backward ----
    if (sg != s) {
      CK(hipEventRecord(evP, s));
      CK(xwait(sg, evP));
    }
    {
    const hipStream_t s = sg;   // (the group stage's launches below)
    for (int k = 0; k < 5; ++k) {
      {
        ProfScope ps(s, K_BWD_SMALL);
        hipLaunchKernelGGL(zmax_group_kernel, dim3(1), dim3(256), 0, s, L.zpart + (size_t)k * G * L.zp_n,
                           L.zp_n, gate_blocks(k), n, L.zmax + k * G);
      }
      CK(hipGetLastError());
    }
    const float hsc = 16384.0f;   // |h| < 1
    auto wpart = [&](const float* ptr, size_t dstride, int nch, int mode, float scale, int j = 0) {
      WgPart p{};
      p.ptr = ptr;
      p.dstride = dstride;
      p.nch = nch;
      p.mode = mode;
      p.scale = scale;
      if (mode == WG_GNRELU) {
        p.stats = rec.stats;
        p.sstride = T.stats_slab;
        p.j = j;
        p.gamma = pk + PL.pk_off[j ? P_D1GW : P_D0GW];
        p.beta = pk + PL.pk_off[j ? P_D1GB : P_D0GB];
      }
      return p;
    };
    const float* st0 = rec.state;                 // slab d: state before plane d
    const float* st1 = rec.state + T.state_slab;  // slab d + 1: after plane d
    for (int k = 0; k < 5; ++k) {
      WgradArgs a{};
      a.gz = L.gz[k];
      a.zmax = L.zmax + k * G;
      a.cin = cell_cin(k);
      a.nplanes = n;
      a.d0 = g0;
      a.B = B;
      a.H = H / res_div[k];
      a.W = W / res_div[k];
      a.wpart = L.wpart;
      a.rseg = L.rseg;
      const size_t S = T.state_slab;
      switch (k) {
        case 0:
          a.part[0] = wpart(rec.x, T.x_plane, 32, WG_PLAIN, 1.0f);
          a.part[0].bound = r.xbound;
          a.part[1] = wpart(st0 + T.h_off[0], S, 16, WG_PLAIN, hsc);
          a.nparts = 2;
          break;
        case 1:
          a.part[0] = wpart(st1 + T.h_off[0], S, 16, WG_POOL, hsc);
          a.part[1] = wpart(st0 + T.h_off[1], S, 16, WG_PLAIN, hsc);
          a.nparts = 2;
          break;
        case 2:
          a.part[0] = wpart(st1 + T.h_off[1], S, 16, WG_POOL, hsc);
          a.part[1] = wpart(st0 + T.h_off[2], S, 16, WG_PLAIN, hsc);
          a.nparts = 2;
          break;
        case 3:
          a.part[0] = wpart(rec.u + T.u0_off, T.u_slab, 16, WG_GNRELU, 16.0f, 0);
          a.part[1] = wpart(st1 + T.h_off[1], S, 16, WG_PLAIN, hsc);
          a.part[2] = wpart(st0 + T.h_off[3], S, 16, WG_PLAIN, hsc);
          a.nparts = 3;
          break;
        default:
          a.part[0] = wpart(rec.u + T.u1_off, T.u_slab, 16, WG_GNRELU, 16.0f, 1);
          a.part[1] = wpart(st1 + T.h_off[0], S, 16, WG_PLAIN, hsc);
          a.part[2] = wpart(st0 + T.h_off[4], S, 8, WG_PLAIN, hsc);
          a.nparts = 3;
          break;
      }
      double* gw = L.gacc + PL.raw_off[P_C0W + 2 * k];
      double* gb = L.gacc + PL.raw_off[P_C0B + 2 * k];
      const int nch = (a.cin + 15) / 16;
      const hipError_t we = kCellHid[k] == 8 ? run_wgrad<32, 3>(a, gw, gb, s, K_WGRAD0 + k)
                            : nch == 3     ? run_wgrad<64, 3>(a, gw, gb, s, K_WGRAD0 + k)
                                           : run_wgrad<64, 2>(a, gw, gb, s, K_WGRAD0 + k);
      CK(we);
    }
    for (int j = 0; j < 2; ++j) {   // the deconvs' GroupNorm affine gradients of the group
      ProfScope ps(s, K_BWD_SMALL);
      hipLaunchKernelGGL(gnb_affine_kernel, dim3(32), dim3(256), 0, s, L.gnb_part[j], n, gnb_nblk(j), B,
                         L.gacc + PL.raw_off[j ? P_D1GW : P_D0GW], L.gacc + PL.raw_off[j ? P_D1GB : P_D0GB]);
      CK(hipGetLastError());
    }
    for (int j = 0; j < 2; ++j) {
      DcwArgs a{};
      a.h = st1 + T.h_off[j ? 3 : 2] + (size_t)g0 * T.state_slab;
      a.hstride = T.state_slab;
      a.gu = L.gu[j];
      a.nplanes = n;
      a.B = B;
      a.Hi = j ? H / 2 : H / 4;
      a.Wi = j ? W / 2 : W / 4;
      a.wpart = L.wpart;
      {
        ProfScope ps(s, K_DECONV_WGRAD);
        hipLaunchKernelGGL(deconv_wgrad_kernel, dim3(kDcwBlocks), dim3(256), 0, s, a);
      }
      CK(hipGetLastError());
      CK(reduce_partials(L.wpart, kDcwBlocks, kDcwPart, 2320, 0, 0, 2320, 2304, L.rseg,
                         L.gacc + PL.raw_off[j ? P_D1W : P_D0W], L.gacc + PL.raw_off[j ? P_D1B : P_D0B], s));
    }
    {
      HwArgs a{};
      a.gcost = r.grad_cost;
      a.h4 = st1 + T.h_off[4] + (size_t)g0 * T.state_slab;
      a.hstride = T.state_slab;
      a.nplanes = n;
      a.d0 = g0;
      a.D = D;
      a.B = B;
      a.H = H;
      a.W = W;
      a.wpart = L.wpart;
      {
        ProfScope ps(s, K_HEAD_WGRAD);
        if ((size_t)2 * B * H * W >= (1ull << 31)) return hipErrorInvalidValue;   // 32-bit indices
        hipLaunchKernelGGL(head_wgrad_kernel, dim3(kHwBlocks), dim3(256), 0, s, a);
      }
      CK(hipGetLastError());
      CK(reduce_partials(L.wpart, kHwBlocks, kHwPart, 73, 0, 0, 73, 72, L.rseg,
                         L.gacc + PL.raw_off[P_HW], L.gacc + PL.raw_off[P_HB], s));
    }
    if (r.grad_x)
      CK(hipMemcpyAsync(r.grad_x + (size_t)g0 * xs, L.gx, (size_t)n * xs * 4, hipMemcpyDeviceToDevice, s));
    if (r.group_done) CK(r.group_done(r.ctx, g0, n, L.gx, s));
    if (sg != sg0) CK(hipEventRecord(evG[gi & 1], sg));
    }
    if (pipe_mode == 4 && sg != s) CK(xwait(s, evG[gi & 1]));
  }
  CK(join_g.join());
  if (r.grad_params) {
    hipLaunchKernelGGL(gacc_to_float_kernel, dim3(256), dim3(256), 0, s, L.gacc, r.grad_params,
                       PL.raw_total);
    CK(hipGetLastError());
  }
#undef CK
  return hipSuccess;
}

}  // namespace aarmvs

namespace aarmvs {
double* bptt_gacc(void* scratch, int B, int H, int W) { return bptt_layout(scratch, B, H, W).gacc; }
}  // namespace aarmvs

// diagnostic (AARMVS_BWD_TRACE, tools/bwd_nondet.py), not part of the ABI: copies the last
// backward's checksum log ([D][32] uint64) to host memory; returns the planes it holds
extern "C" __attribute__((visibility("default"))) int aarmvs_debug_bwd_trace(void* host, size_t bytes) {
  using namespace aarmvs;
  if (!g_trace) return 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const size_t n = std::min(bytes, (size_t)g_trace_planes * kTraceSlots * 8);
  if (hipMemcpy(host, g_trace, n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return g_trace_planes;
}
