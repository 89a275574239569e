// Recurrent regulariser step (UNetConvLSTM, models/drmvsnet.py:119-167) for gfx950.
//
// ConvLSTM cell (models/module.py:76-92) = implicit-GEMM 3x3 conv on the matrix cores
// (split-fp16 v_mfma_f32_32x32x16_f16, below) with the LSTM gate math fused into the
// epilogue:
//   M = 4*hid output channels (gates i,f,o,g), N = pixels, K = 9 taps x Cin.
//   One m-tile = 32 rows = the 4 gates of 8 hidden channels, so every lane holds
//   i,f,o,g of the same (pixel, channel) in its accumulator registers and the
//   c/h update needs no data exchange.
//   A (weights) and the haloed input tile live in LDS.
// Input staging fuses the U-Net glue: 2x2 max-pool (drmvsnet.py:148,152),
// GroupNorm(2,16)+ReLU of the deconv output (module.py:286-287) and the channel
// concatenations (drmvsnet.py:80, 157, 161).
// Layout: every U-Net tensor in the workspace (the cost slice x, h and c of each cell,
// the deconv outputs) is NHWC, [B][H][W][C] fp32.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <type_traits>

#include "device_common.h"

namespace aarmvs {

typedef float floatx16 __attribute__((ext_vector_type(16)));

enum SrcMode : int { SRC_PLAIN = 0, SRC_POOL = 1, SRC_GNRELU = 2 };

struct ChanSrc {
  const float* ptr;     // [B][nch][Hs][Ws]
  int nch;
  int mode;
  const double* stats;  // SRC_GNRELU: 2 statistics (groups of 8 channels)
  const float* gamma;
  const float* beta;
  // SRC_GNRELU from the deconv's per-block partials (when set): every block reduces them as
  // a fixed-order reduce does, block 0 stores the statistics at stats_out
  const double* part;   // [nblk][4]: (sum, sumsq) of groups 0 and 1
  int nblk;
  double* stats_out;
};

// The GroupNorm table (gn[c] = rstd gamma_c, gn[16 + c] = beta_c - mean gn[c]) of a SRC_GNRELU
// part.  From partials: strided sums over 256 lanes and a fixed tree (the reduce kernel these
// replaced: bit-identical statistics), in `red` (>= 8 KB of LDS the staging has not used yet); all
// threads of the block take part in the barriers.
__device__ __forceinline__ void gn_table(const ChanSrc& s, float* gn, double* red, int tid, int H, int W) {
  if (!s.part) {
    if (tid < 16) {
      const GnStat st = stat_read(s.stats + (tid >> 3) * kSlots * 2, 8.0 * H * W);
      const float sc = st.rstd * s.gamma[tid];
      gn[tid] = sc;
      gn[16 + tid] = s.beta[tid] - st.mean * sc;
    }
    return;
  }
  if (tid < 256) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = tid; i < s.nblk; i += 256)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += s.part[4 * i + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) red[j * 256 + tid] = acc[j];
  }
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[j * 256 + tid] += red[j * 256 + tid + o];
    __syncthreads();
  }
  if (tid < 16) {
    const int g = tid >> 3;
    const GnStat st = gn_stat_from(red[2 * g * 256], red[(2 * g + 1) * 256], 8.0 * H * W);
    const float sc = st.rstd * s.gamma[tid];
    gn[tid] = sc;
    gn[16 + tid] = s.beta[tid] - st.mean * sc;
  }
  if (blockIdx.x == 0 && tid < 4) s.stats_out[(tid >> 1) * kSlots * 2 + (tid & 1)] = red[tid * 256];
  __syncthreads();   // the scratch is the staging's buffer
}

struct CellArgs {
  ChanSrc part[3];
  int nparts;
  float* h_new;
  float* c;             // c' out ([B][H][W][HID]); the eval sweep updates c in place (c_in == c)
  const float* c_in;    // c of the previous plane
  float* z_out;         // training record: the gate pre-activations (conv + bias), or null: planar,
                        // [B][HID/4 channel quads][gates i, f, o, g][H*W][4]
  const float* wpk;     // packed A operands [K/2][MT][64]
  const float* bias;    // [4*hid]
  const unsigned* xbound;   // cell 0: float bits of a bound on |x| (fp16 range guard), or null
  int B, H, W;          // cell resolution
  int skew;             // double-buffered kernel: waves with bit skew-1 set stage first (0: none)
};

// Staging scales of the split-fp16 operands.  An fp32 value a is staged as fp16 hi + lo with
// lo = a - hi; lo keeps fp16's 11 significant bits only while it is a normal number
// (|lo| >= 2^-14, i.e. |a| >~ 2^-3): below that its quantum is the subnormal step 2^-24, an
// absolute error that, for the h values of typical magnitude 1e-2, is 10-50x fp32's rounding
// and was the source of the BPTT's excess error in the omega network's gradients.
// So every part is staged at a power-of-two scale that puts its largest possible magnitude
// just under fp16's range, and the accumulators are rescaled (exactly) between parts:
//  * h and pooled h (|h| < 1: sigmoid x tanh): x 2^kHScaleExp;
//  * cell 0's x (the cost slice x = -sum (1 + w) sq / nsrc, bounded by the sweep's ws.xbound)
//    and cells 3 and 4's GroupNorm+ReLU part (deConvGnReLU's output, module.py:286-287,
//    bounded by gn_relu_bound: |xhat| <= sqrt(n - 1) for n values of mean 0 and unit biased
//    variance, Samuelson's inequality): x 2^-e with bound 2^-e in [2^14, 2^15) (fp16's largest
//    finite is 65504), e of either sign.
constexpr int kHScaleExp = 12;

__device__ __forceinline__ int guard_exp_of(float bound) {
  if (!(bound > 0.0f)) return 0;
  const int k = ilogbf(bound);   // 2^k <= bound < 2^(k+1); INT_MAX for inf
  return k >= 134 ? 120 : (k < -100 ? -114 : k - 14);
}
__device__ __forceinline__ int xguard_exp(const unsigned* xb) {
  return xb ? guard_exp_of(__uint_as_float(*xb)) : -kHScaleExp;
}
__device__ __forceinline__ int gguard_exp(const float* gamma, const float* beta, int H, int W) {
  return guard_exp_of(gn_relu_bound(gamma, beta, 8.0 * H * W));
}

constexpr int kMaxParts = 3;

// The five cells of the U-Net (drmvsnet.py:141-161): input parts in concatenation
// order (channels, how they are staged), hidden channels, and the tile shape
// (TH rows of NT x 32 pixels; one wave per row).
template <int KIND>
struct CellDef;
// (A/B builds only: the staging variant of cells 3 and 4; the library uses the defaults)
#ifndef AARMVS_C3DB
#define AARMVS_C3DB 1
#endif
#ifndef AARMVS_C4DB
#define AARMVS_C4DB 0
#endif
#ifndef AARMVS_C3SKEW
#define AARMVS_C3SKEW 3
#endif
#ifndef AARMVS_C4SKEW
#define AARMVS_C4SKEW 0
#endif
#ifndef AARMVS_C4PIPE
#define AARMVS_C4PIPE 0
#endif
template <>
struct CellDef<0> {   // [x, h0] @ H
  static constexpr int NP = 2, CH[kMaxParts] = {32, 16, 0};
  static constexpr int MODE[kMaxParts] = {SRC_PLAIN, SRC_PLAIN, SRC_PLAIN};
  static constexpr int HID = 16;
  static constexpr int H3RW = 1, H3WAVES = 8, H3DB = 1, H3PIPE = 1, H3MS = 1;
  static constexpr int MIN_WAVES = 1;   // amdgpu_waves_per_eu lower bound (register budget)
  static constexpr int SKEW = 3;        // CellArgs::skew of the double-buffered kernel
};
template <>
struct CellDef<1> {   // [maxpool(h0'), h1] @ H/2
  static constexpr int NP = 2, CH[kMaxParts] = {16, 16, 0};
  static constexpr int MODE[kMaxParts] = {SRC_POOL, SRC_PLAIN, SRC_PLAIN};
  static constexpr int HID = 16;
  static constexpr int H3RW = 1, H3WAVES = 8, H3DB = 1, H3PIPE = 1, H3MS = 1;
  static constexpr int MIN_WAVES = 1;
  static constexpr int SKEW = 2;
};
template <>
struct CellDef<2> : CellDef<1> {};   // [maxpool(h1'), h2] @ H/4
template <>
struct CellDef<3> {   // [gnrelu(u0), h1', h3] @ H/2
  static constexpr int NP = 3, CH[kMaxParts] = {16, 16, 16};
  static constexpr int MODE[kMaxParts] = {SRC_GNRELU, SRC_PLAIN, SRC_PLAIN};
  static constexpr int HID = 16;
  static constexpr int H3RW = 1, H3WAVES = 8, H3DB = AARMVS_C3DB, H3PIPE = 1, H3MS = 1;
  static constexpr int MIN_WAVES = 1;
  static constexpr int SKEW = AARMVS_C3SKEW;
};
template <>
struct CellDef<4> {   // [gnrelu(u1), h0', h4] @ H
  static constexpr int NP = 3, CH[kMaxParts] = {16, 16, 8};
  static constexpr int MODE[kMaxParts] = {SRC_GNRELU, SRC_PLAIN, SRC_PLAIN};
  static constexpr int HID = 8;
  static constexpr int H3RW = 1, H3WAVES = 8, H3DB = AARMVS_C4DB, H3PIPE = AARMVS_C4PIPE, H3MS = 1;
  // <= 128 VGPRs: two 512-thread blocks per CU (the sign-balanced accumulator pair took the
  // compiler's choice to 130, one block per CU: 160 -> 202 us per plane at the headline)
  static constexpr int MIN_WAVES = 4;
  static constexpr int SKEW = AARMVS_C4SKEW;
};

// ---------------------------------------------------------------------------
// Split-fp16 ConvLSTM cell ("h3"): the 3x3 conv as an implicit GEMM on
// v_mfma_f32_32x32x16_f16 (M = 4 hid gate rows, N = 32 pixels of a tile row, K = 9 taps x
// Cin) with each fp32 operand split into fp16 hi + lo and three products per k-step,
//   w x = w_hi x_hi + w_hi x_lo + w_lo x_hi   (+ w_lo x_lo, dropped: ~2^-22 relative),
// accumulated in fp32.  The weights carry a power-of-two scale (pack_cell_h3_kernel)
// undone in the epilogue.  Per product the error is ~2^-21 relative, i.e. within a few
// fp32 roundings.
// Rate: 3 x 16 K per 3 x 32 cycles vs 2 K per 64 cycles for the f32 MFMA, 5.3x.
//
// Input channels are processed in 16-channel chunks (one k-group of every tap); a
// chunk of the haloed tile sits in LDS as [pixel][16 ch] fp16 (hi and lo planes, the
// two 16-B halves of a pixel swapped on every other group of 8 pixels: conflict-free
// ds_read_b128 B fragments).  The next chunk (or the next tile's first chunk) is
// prefetched into registers while the MFMAs of the current one run.
// ---------------------------------------------------------------------------
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

// RW: rows (32-pixel n-tiles) per wave -- the A (weight) fragments of a tap are reused
// RW times; WAVES: waves per block.  Defaults per cell in CellDef.
// MS: waves per tile row -- each of a row's MS waves takes MT / MS of the m-tiles (the gates of
// 8 hidden channels per m-tile: the LSTM update of those channels is the wave's own), so a block
// of WAVES waves covers WAVES / MS rows
template <int KIND, int RW_ = CellDef<KIND>::H3RW, int WAVES_ = CellDef<KIND>::H3WAVES, int MS_ = 1>
struct H3Cfg {
  using D = CellDef<KIND>;
  static constexpr int CIN = D::CH[0] + D::CH[1] + D::CH[2];
  static constexpr int NCHK = (CIN + 15) / 16;
  static constexpr int HID = D::HID, MT = HID / 8, COUT = 4 * HID;
  static constexpr int RW = RW_, WAVES = WAVES_, MS = MS_, MTL = MT / MS, RWAVES = WAVES / MS;
  static_assert(MT % MS == 0 && WAVES % MS == 0, "whole m-tiles and rows per wave");
  static constexpr int TH = RW * RWAVES, THREADS = WAVES * 64, TW = 32, W2 = TW + 2, TROWS = TH + 2;
  static constexpr int NPIX = TROWS * W2;
  static constexpr int A_HALVES = NCHK * 9 * MT * 64 * 8;   // per hi / lo
  static constexpr size_t LDS_BYTES = (size_t)A_HALVES * 2 * 2 + (size_t)NPIX * 32 * 2 + 32 * 4;
  static constexpr int c0(int p) { return p == 0 ? 0 : (p == 1 ? D::CH[0] : D::CH[0] + D::CH[1]); }
  static constexpr int chunk_part(int c) {
    return 16 * c < c0(1) ? 0 : (16 * c < c0(2) || D::NP < 3 ? 1 : 2);
  }
  static constexpr int chunk_lc0(int c) { return 16 * c - c0(chunk_part(c)); }
  static constexpr int chunk_nv(int c) {
    return D::CH[chunk_part(c)] - chunk_lc0(c) < 16 ? D::CH[chunk_part(c)] - chunk_lc0(c) : 16;
  }
  // 8 valid channels: two taps per k-step (h3_mfma_chunk), the chunk's second half unused
  static constexpr bool chunk_paired(int c) { return chunk_nv(c) == 8; }
};

// byte offset of (pixel p, 16-B half h) in a chunk plane
__device__ __forceinline__ int h3_pix(int p, int h) { return p * 32 + ((h ^ ((p >> 3) & 1)) << 4); }

// (a, b) -> fp16 hi pair + lo pair (round to nearest even).  Written as vector conversions so
// that the hi pair is one v_cvt_pk_f16_f32 read back by v_cvt_f32_f16 (SDWA for the high
// half): 6 instructions per pair instead of 8 (the scalar form converts hi twice)
typedef float float2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t h3_split2(float a, float b, uint32_t& lo_bits) {
  const half2_t hi = __builtin_convertvector((float2_t){a, b}, half2_t);
  const half2_t lo = __builtin_convertvector((float2_t){a - (float)hi[0], b - (float)hi[1]}, half2_t);
  lo_bits = __builtin_bit_cast(uint32_t, lo);
  return __builtin_bit_cast(uint32_t, hi);
}

// Input staging: item = (half h of the chunk's 16 channels, pixel p of the haloed tile),
// consecutive lanes on consecutive pixels.  The U-Net tensors are NHWC ([B][H][W][C]), so
// an item's 8 channels are 32 contiguous bytes (two 16-B loads; POOL: two per fine pixel
// of the 2x2 window) and a tile row is one contiguous run per part.  An item lands in
// each LDS plane as ONE 16-B store (8 channels as fp16 pairs) at h3_pix(p, h): 2-way bank
// conflicts at most.  Out-of-image pixels and channels past the chunk's valid count load
// zeros through the buffer range check.  NTH: staging threads (default: the block).
template <int KIND, int RW, int WAVES, int NTH = 0, bool PAIRSKIP = false, int MS = 1>
struct H3PixStager {
  using C = H3Cfg<KIND, RW, WAVES, MS>;
  using D = typename C::D;
  static constexpr int TH = NTH ? NTH : C::THREADS;   // staging threads
  static constexpr int NITEM = 2 * C::NPIX;
  static constexpr int NI = (NITEM + TH - 1) / TH;
  static_assert(NI <= 32, "item mask holds 32 items");
  float val[NI][8][4];   // [item][channel][POOL window: fine (2y,2x) (2y,2x+1) (2y+1,2x) (2y+1,2x+1)]
  uint32_t in_mask;      // bit j: item j is an in-image pixel of valid channels
  float xs = 1.0f;       // 2^-e staging scale of part 0: cell 0's x (xguard_exp), cells 3 and
                         // 4's GroupNorm+ReLU part (gguard_exp); h parts: 2^kHScaleExp

  template <int CH>
  __device__ __forceinline__ void load(const CellArgs& a, int b, int y0, int x0, int tid) {
    constexpr int P = C::chunk_part(CH), MODE = D::MODE[P], NCH = D::CH[P];
    constexpr int LC0 = C::chunk_lc0(CH), NV = C::chunk_nv(CH);
    static_assert(NV % 8 == 0, "chunks hold whole 8-channel halves");
    const ChanSrc& s = a.part[P];
    const int H = a.H, W = a.W;
    const int Hs = MODE == SRC_POOL ? 2 * H : H, Ws = MODE == SRC_POOL ? 2 * W : W;
    const uint32_t nbytes = (uint32_t)NCH * (uint32_t)Hs * (uint32_t)Ws * 4u;   // one image
    const __amdgpu_buffer_rsrc_t r = uniform_rsrc(s.ptr + (size_t)b * NCH * Hs * Ws, nbytes);
    in_mask = 0u;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int e = tid + j * TH;
      const int h = e >= C::NPIX ? 1 : 0, p = e - h * C::NPIX;
      // PAIRSKIP: a paired chunk's second half is never read (h3_mfma_chunk): no loads
      if (PAIRSKIP && C::chunk_paired(CH) && h) continue;
      const int row = p / C::W2, col = p - row * C::W2;
      const int gy = y0 - 1 + row, gx = x0 - 1 + col;
      const bool in = e < NITEM && 8 * h < NV && gy >= 0 && gy < H && gx >= 0 && gx < W;
      if (in) in_mask |= 1u << j;
      const uint32_t pix = MODE == SRC_POOL ? (uint32_t)(2 * gy * Ws + 2 * gx) : (uint32_t)(gy * W + gx);
      const uint32_t ob = (pix * (uint32_t)NCH + (uint32_t)(LC0 + 8 * h)) * 4u;
      constexpr int NW = MODE == SRC_POOL ? 4 : 1;   // POOL: the 2x2 fine window
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const uint32_t o = in ? ob + (uint32_t)(((w >> 1) * Ws + (w & 1)) * NCH * 4) : nbytes;
        const float4 q0 = ld4(r, o), q1 = ld4(r, in ? o + 16u : nbytes);
        val[j][0][w] = q0.x;
        val[j][1][w] = q0.y;
        val[j][2][w] = q0.z;
        val[j][3][w] = q0.w;
        val[j][4][w] = q1.x;
        val[j][5][w] = q1.y;
        val[j][6][w] = q1.z;
        val[j][7][w] = q1.w;
      }
    }
  }

  template <int CH>
  __device__ __forceinline__ void store(char* hi_plane, char* lo_plane, const float* gn, int tid,
                                        int x0, int W) const {
    constexpr int MODE = D::MODE[C::chunk_part(CH)];
    constexpr int LC0 = C::chunk_lc0(CH);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int e = tid + j * TH;
      if (e < NITEM) {
        const int h = e >= C::NPIX ? 1 : 0, p = e - h * C::NPIX;
        if (PAIRSKIP && C::chunk_paired(CH) && h) continue;   // (and no stores)
        const bool in = in_mask & (1u << j);
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float x;
          constexpr float HS = (float)(1 << kHScaleExp);
          if (MODE == SRC_POOL) {
            x = fmaxf(fmaxf(val[j][k][0], val[j][k][1]), fmaxf(val[j][k][2], val[j][k][3])) * HS;
          } else if (MODE == SRC_GNRELU) {
            const int lc = LC0 + 8 * h + k;
            x = fmaxf(val[j][k][0] * gn[lc] + gn[16 + lc], 0.0f) * xs;
          } else if constexpr (KIND == 0 && C::chunk_part(CH) == 0) {
            x = val[j][k][0] * xs;
          } else {
            x = val[j][k][0] * HS;
          }
          v[k] = in ? x : 0.0f;
        }
        uint32_t hw[4], lw[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) hw[i] = h3_split2(v[2 * i], v[2 * i + 1], lw[i]);
        const int off = h3_pix(p, h);
        *reinterpret_cast<u32x4*>(hi_plane + off) = u32x4{hw[0], hw[1], hw[2], hw[3]};
        *reinterpret_cast<u32x4*>(lo_plane + off) = u32x4{lw[0], lw[1], lw[2], lw[3]};
      }
    }
  }
};

// Before the MFMAs of chunk CH: bring part 0's partial sums (cell 0's x, cells 3 and 4's
// GroupNorm+ReLU part, staged x 2^-e) to the h parts' scale 2^kHScaleExp (CH is the first chunk
// past part 0); the epilogue undoes 2^kHScaleExp with the weight scale.
template <class C, int KIND, int CH, bool BAL>
__device__ __forceinline__ void xguard_rescale(floatx16 (&acc)[C::MTL][C::RW], floatx16 (&accn)[C::MTL][C::RW],
                                               float xr) {
  if constexpr ((KIND == 0 || C::D::MODE[0] == SRC_GNRELU) && CH > 0 && C::chunk_part(CH) != 0 &&
                C::chunk_part(CH - 1) == 0) {
#pragma unroll
    for (int m = 0; m < C::MTL; ++m)
#pragma unroll
      for (int r = 0; r < C::RW; ++r) {
        acc[m][r] *= xr;
        if constexpr (BAL) accn[m][r] *= xr;
      }
  }
}

// One input chunk's MFMAs: 9 taps x MT m-tiles x RW rows x 3 split products.  PIPE: the
// A/B fragments of tap t+1 are read from LDS into a second register set before tap t's
// MFMAs issue (sched_barrier pins the order); otherwise the compiler's schedule reads
// each tap's fragments just before use and waits on them every 2-3 MFMAs.
// Sign-balanced accumulation: v_mfma_f32_*_f16 does not round its fp32 accumulation to
// nearest -- each MFMA's result errs low by ~0.1 ulp of its largest addend on average
// (tools/microbench/mfma_round.cpp: -0.33 ulp of the result over random inputs), so a long
// chain drifts downwards, a bias that long cancelling gradient sums amplify.
// Taps with (tap + chunk) odd carry negated weights (pack_cell_h3_kernel) and accumulate into
// accn; the result is acc - accn, whose two drifts cancel (tools/microbench/mfma_chain.cpp:
// -0.164 -> +0.001 ulp over 108 MFMAs).  BAL: the training cells only (their record is what
// the BPTT differentiates); the inference cells accumulate every tap into acc with the
// positive fragments (pack_cell_h3_kernel's second copy): 32 fewer accumulator registers.
//
// A chunk of 8 valid channels (cell 4's h4 part) is "paired": its k-step s takes tap 2s in the
// K half of lanes 0-31 and tap 2s+1 in the K half of lanes 32-63 (the weights packed to match,
// pack_cell_h3_kernel), so the chunk costs 5 k-steps instead of 9 with a zero K half each;
// tap 9 of step 4 is a zero weight against tap 8's pixels.
template <class C, int CH, bool PIPE = false, bool BAL = true, int ONCE = 0>
__device__ __forceinline__ void h3_mfma_chunk(floatx16 (&acc)[C::MTL][C::RW], floatx16 (&accn)[C::MTL][C::RW],
                                              const char* wl_hi, const char* wl_lo, const char* in_hi,
                                              const char* in_lo, int wave, int lane, int m0 = 0) {
  // wave: the wave's row group (its rows wave RW ..); m0: its first m-tile (H3Cfg::MS)
  constexpr int MT = C::MT, MTL = C::MTL, RW = C::RW;
  const int col = lane & 31, h = lane >> 5;
  if constexpr (C::chunk_paired(CH)) {
    // (PIPE ignored: the plain fragment schedule.)  The lane's tap offsets are recomputed here
    // rather than hoisted out of the tile loop (5 live VGPRs: the training cell spilled)
    int hv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(hv) : "v"(h));
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int tap = min(2 * s + hv, 8);
      half8 bh[RW], bl[RW];
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int boff = h3_pix((wave * RW + r + tap / 3) * C::W2 + col + tap % 3, 0);
        bh[r] = *reinterpret_cast<const half8*>(in_hi + boff);
        bl[r] = *reinterpret_cast<const half8*>(in_lo + boff);
      }
#pragma unroll
      for (int m = 0; m < MTL; ++m) {
        const int aoff = ((((CH * 9 + s) * MT + m0 + m) * 64) + lane) * 16;
        const half8 ah = *reinterpret_cast<const half8*>(wl_hi + aoff);
        const half8 al = *reinterpret_cast<const half8*>(wl_lo + aoff);
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          floatx16& d = (BAL && ((s + CH) & 1)) ? accn[m][r] : acc[m][r];
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[r], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[r], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[r], d, 0, 0, 0);
        }
      }
    }
  } else if constexpr (PIPE) {
    half8 bh[2][RW], bl[2][RW], ah[2][MTL], al[2][MTL];
    auto fetch = [&](int tap, int s) {
      if ((ONCE & 2) && tap > 0) {   // microbenchmark ablation: B fragments of tap 0 only
#pragma unroll
        for (int r = 0; r < RW; ++r) bh[s][r] = bh[s ^ 1][r], bl[s][r] = bl[s ^ 1][r];
      } else
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int boff = h3_pix((wave * RW + r + tap / 3) * C::W2 + col + tap % 3, h);
        bh[s][r] = *reinterpret_cast<const half8*>(in_hi + boff);
        bl[s][r] = *reinterpret_cast<const half8*>(in_lo + boff);
      }
      if ((ONCE & 1) && tap > 0) {   // microbenchmark ablation: A fragments of tap 0 only
#pragma unroll
        for (int m = 0; m < MTL; ++m) ah[s][m] = ah[s ^ 1][m], al[s][m] = al[s ^ 1][m];
        return;
      }
#pragma unroll
      for (int m = 0; m < MTL; ++m) {
        const int aoff = ((((CH * 9 + tap) * MT + m0 + m) * 64) + lane) * 16;
        ah[s][m] = *reinterpret_cast<const half8*>(wl_hi + aoff);
        al[s][m] = *reinterpret_cast<const half8*>(wl_lo + aoff);
      }
    };
    fetch(0, 0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int s = tap & 1;
      if (tap + 1 < 9) fetch(tap + 1, s ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < MTL; ++m)
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          floatx16& d = (BAL && ((tap + CH) & 1)) ? accn[m][r] : acc[m][r];
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s][m], bh[s][r], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s][m], bl[s][r], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[s][m], bh[s][r], d, 0, 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      half8 bh[RW], bl[RW];
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int p = (wave * RW + r + tap / 3) * C::W2 + col + tap % 3;
        const int boff = h3_pix(p, h);
        bh[r] = *reinterpret_cast<const half8*>(in_hi + boff);
        bl[r] = *reinterpret_cast<const half8*>(in_lo + boff);
      }
#pragma unroll
      for (int m = 0; m < MTL; ++m) {
        const int aoff = ((((CH * 9 + tap) * MT + m0 + m) * 64) + lane) * 16;
        const half8 ah = *reinterpret_cast<const half8*>(wl_hi + aoff);
        const half8 al = *reinterpret_cast<const half8*>(wl_lo + aoff);
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          floatx16& d = (BAL && ((tap + CH) & 1)) ? accn[m][r] : acc[m][r];
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[r], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[r], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[r], d, 0, 0, 0);
        }
      }
    }
  }
}

// Cell state I/O (NHWC [B][H][W][HID]): lane (col, hi) of m-tile m owns channels
// m*8 + 4 hi .. +3 of pixel (y, x): one 16-B load / store per (m, row).
template <class C>
__device__ __forceinline__ void cell_c_load(const CellArgs& a, int b, int yw, int x, int hi,
                                            float (&cst)[C::MTL][C::RW][4], int m0 = 0) {
#pragma unroll
  for (int m = 0; m < C::MTL; ++m)
#pragma unroll
    for (int r = 0; r < C::RW; ++r) {
      const int y = yw + r;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (y < a.H && x < a.W)
        v = *reinterpret_cast<const float4*>(
            a.c_in + (((size_t)b * a.H + y) * a.W + x) * C::HID + (m0 + m) * 8 + 4 * hi);
      cst[m][r][0] = v.x;
      cst[m][r][1] = v.y;
      cst[m][r][2] = v.z;
      cst[m][r][3] = v.w;
    }
}

// gate epilogue (module.py:83-90): undo the weight scale, add the bias, LSTM update
template <class C, int ABL, bool PRECISE>
__device__ __forceinline__ void cell_epilogue(const CellArgs& a, const floatx16 (&acc)[C::MTL][C::RW],
                                              const float (&cst)[C::MTL][C::RW][4], float inv_scale,
                                              int b, int yw, int x, int hi, int m0 = 0) {
  constexpr int HID = C::HID;
#pragma unroll
  for (int r = 0; r < C::RW; ++r) {
    const int y = yw + r;
    if (y < a.H && x < a.W) {
      const size_t pix = ((size_t)b * a.H + y) * a.W + x;
#pragma unroll
      for (int ml = 0; ml < C::MTL; ++ml) {
        const int m = m0 + ml;
        float cn[4], hn[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ch = m * 8 + 4 * hi + q;
          const float gi = fmaf(acc[ml][r][q], inv_scale, a.bias[ch]);
          const float gf = fmaf(acc[ml][r][4 + q], inv_scale, a.bias[HID + ch]);
          const float go = fmaf(acc[ml][r][8 + q], inv_scale, a.bias[2 * HID + ch]);
          const float gg = fmaf(acc[ml][r][12 + q], inv_scale, a.bias[3 * HID + ch]);
          if (ABL & 4) {
            cn[q] = gi + gf;
            hn[q] = go + gg + cst[ml][r][q];
          } else if (PRECISE) {   // the training sweep: unbiased activations (device_common.h)
            cn[q] = precise_sigmoid(gf) * cst[ml][r][q] + precise_sigmoid(gi) * precise_tanh(gg);
            hn[q] = precise_sigmoid(go) * precise_tanh(cn[q]);
          } else {
            cn[q] = fast_sigmoid(gf) * cst[ml][r][q] + fast_sigmoid(gi) * fast_tanh(gg);
            hn[q] = fast_sigmoid(go) * fast_tanh(cn[q]);
          }
        }
        const size_t o = pix * HID + m * 8 + 4 * hi;
        *reinterpret_cast<float4*>(a.c + o) = make_float4(cn[0], cn[1], cn[2], cn[3]);
        *reinterpret_cast<float4*>(a.h_new + o) = make_float4(hn[0], hn[1], hn[2], hn[3]);
        if (a.z_out) {   // gates i, f, o, g of channels m*8 + 4 hi .. +3 (module.py:83)
          // planar record layout [B][HID/4 channel quads][4 gates][H*W][4]: a wave's stores of
          // one gate are contiguous (512 B per half-wave)
          const size_t P = (size_t)a.H * a.W;
          float* zo = a.z_out + (size_t)b * 4 * HID * P + ((size_t)(m * 2 + hi) * 4 * P + (size_t)y * a.W + x) * 4;
#pragma unroll
          for (int gt = 0; gt < 4; ++gt) {
            float zz[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int ch = m * 8 + 4 * hi + q;
              zz[q] = fmaf(acc[ml][r][4 * gt + q], inv_scale, a.bias[gt * HID + ch]);
            }
            *reinterpret_cast<float4*>(zo + gt * P * 4) = make_float4(zz[0], zz[1], zz[2], zz[3]);
          }
        }
      }
    }
  }
}

// Single-buffered kernel.  PIPE: software-pipelined fragment reads (h3_mfma_chunk).  ABL:
// ablation bits for the microbenchmark only (1 no MFMA, 2 no staging loads/stores, 4 no
// gate math, 8 / 16 the A / B fragments read for tap 0 only)
template <int KIND, int RW = CellDef<KIND>::H3RW, int WAVES = CellDef<KIND>::H3WAVES, int ABL = 0,
          int PIPE = CellDef<KIND>::H3PIPE, bool PRECISE = false, int MS = 1>
__global__ void __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(CellDef<KIND>::MIN_WAVES))) lstm_cell_h3_kernel(
    CellArgs a, const float* __restrict__ inv_scale_ptr) {
  using C = H3Cfg<KIND, RW, WAVES, MS>;
  using D = typename C::D;
  constexpr int MT = C::MTL, NCHK = C::NCHK;
  extern __shared__ __attribute__((aligned(16))) char lds_h3[];
  char* wl_hi = lds_h3;
  char* wl_lo = wl_hi + C::A_HALVES * 2;
  char* in_hi = wl_lo + C::A_HALVES * 2;
  char* in_lo = in_hi + C::NPIX * 32;
  float* gn = reinterpret_cast<float*>(in_lo + C::NPIX * 32);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W;
  const float inv_scale = ldexpf(*inv_scale_ptr, -kHScaleExp);   // weight scale and staging scale
  // split-fp16 weights -> LDS once per block
  {
    const float4* s = reinterpret_cast<const float4*>(a.wpk);
    float4* d = reinterpret_cast<float4*>(wl_hi);
    constexpr int N4 = C::A_HALVES * 2 * 2 / 16;
#pragma unroll 8
    for (int i = tid; i < N4; i += C::THREADS) d[i] = s[i];
  }
#pragma unroll
  for (int p = 0; p < D::NP; ++p)
    if (D::MODE[p] == SRC_GNRELU) gn_table(a.part[p], gn, reinterpret_cast<double*>(in_hi), tid, H, W);

  const int tiles_x = (W + C::TW - 1) / C::TW, tiles_y = (H + C::TH - 1) / C::TH;
  const int ntiles = a.B * tiles_x * tiles_y;
  auto coords = [&](int tile, int& b, int& y0, int& x0) {
    b = tile / (tiles_x * tiles_y);
    const int rem = tile % (tiles_x * tiles_y);
    y0 = (rem / tiles_x) * C::TH;
    x0 = (rem % tiles_x) * C::TW;
  };
  // the inference cells skip a paired chunk's unused half; the training cells (PRECISE) keep
  // the uniform staging loop (skipping it costs the 128-VGPR cell 4 spills there)
  H3PixStager<KIND, RW, WAVES, 0, !PRECISE, MS> st;
  const int xe = KIND == 0 ? xguard_exp(a.xbound)
                 : D::MODE[0] == SRC_GNRELU ? gguard_exp(a.part[0].gamma, a.part[0].beta, H, W) : 0;
  st.xs = ldexpf(1.0f, -xe);
  const float xr = ldexpf(1.0f, xe + kHScaleExp);   // part 0's units -> the h parts' 2^kHScaleExp
  int tile = blockIdx.x;
  if (tile < ntiles && !(ABL & 2)) {
    int b, y0, x0;
    coords(tile, b, y0, x0);
    st.template load<0>(a, b, y0, x0, tid);
  }
  const int hi = lane >> 5, col = lane & 31;
  const int rwave = wave % C::RWAVES, m0 = (wave / C::RWAVES) * C::MTL;   // row group, m-tiles
  for (; tile < ntiles; tile += gridDim.x) {
    int b, y0, x0;
    coords(tile, b, y0, x0);
    const int next = tile + (int)gridDim.x;
    int nb = 0, ny0 = 0, nx0 = 0;
    if (next < ntiles) coords(next, nb, ny0, nx0);
    const int yw = y0 + rwave * RW;   // this wave's first row
    floatx16 acc[MT][RW], accn[MT][RW];   // sign-balanced pair (h3_mfma_chunk)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[m][r][j] = accn[m][r][j] = 0.0f;
    float cst[MT][RW][4];
    // chunk loop, fully unrolled so that every chunk's staging mode is compile-time
    auto chunk = [&](auto CHc) {
      constexpr int CH = decltype(CHc)::value;
      __syncthreads();   // previous chunk's B reads done (weights / gn visible the first time)
      if (!(ABL & 2)) st.template store<CH>(in_hi, in_lo, gn, tid, x0, W);
      __syncthreads();
      if (ABL & 2) {
      } else if (CH + 1 < NCHK) {
        st.template load<(CH + 1 < NCHK ? CH + 1 : 0)>(a, b, y0, x0, tid);
      } else if (next < ntiles) {
        st.template load<0>(a, nb, ny0, nx0, tid);
      }
      if (CH == 0) cell_c_load<C>(a, b, yw, x0 + col, hi, cst, m0);
      xguard_rescale<C, KIND, CH, PRECISE>(acc, accn, xr);
      if (!(ABL & 1)) h3_mfma_chunk<C, CH, PIPE != 0, PRECISE, (ABL >> 3) & 3>(acc, accn, wl_hi, wl_lo, in_hi, in_lo, rwave, lane, m0);
    };
    chunk(std::integral_constant<int, 0>{});
    if constexpr (NCHK > 1) chunk(std::integral_constant<int, 1>{});
    if constexpr (NCHK > 2) chunk(std::integral_constant<int, 2>{});
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < RW; ++r)
        if constexpr (PRECISE) acc[m][r] -= accn[m][r];
    cell_epilogue<C, ABL, PRECISE>(a, acc, cst, inv_scale, b, yw, x0 + col, hi, m0);
  }
}

// Double-buffered variant (cells 0 and 3): the haloed input tile has two LDS buffers, so
// a chunk's MFMAs and the staging of the following chunk share one phase (one barrier
// per chunk).  Per step: MFMAs on buffer `par`; store the prefetched following chunk
// (this tile's next, or the next tile's first) into buffer par ^ 1; issue the loads of
// the chunk after that; at a tile's last chunk, the gate epilogue.  Across the two
// waves of a SIMD one wave's staging VALU work fills the other's MFMA issue gaps.
template <int KIND, int RW = CellDef<KIND>::H3RW, int WAVES = CellDef<KIND>::H3WAVES, int ABL = 0,
          int PIPE = CellDef<KIND>::H3PIPE, bool PRECISE = false, int MS = 1>
__global__ void __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(CellDef<KIND>::MIN_WAVES))) lstm_cell_h3db_kernel(
    CellArgs a, const float* __restrict__ inv_scale_ptr) {
  using C = H3Cfg<KIND, RW, WAVES, MS>;
  using D = typename C::D;
  constexpr int MT = C::MTL, NCHK = C::NCHK;
  constexpr int PB = C::NPIX * 32;   // one plane (hi or lo) of one input buffer
  static_assert(NCHK >= 2, "two or more input chunks");
  extern __shared__ __attribute__((aligned(16))) char lds_h3[];
  char* wl_hi = lds_h3;
  char* wl_lo = wl_hi + C::A_HALVES * 2;
  char* inb = wl_lo + C::A_HALVES * 2;   // buffer k: hi plane at 2k PB, lo plane at (2k+1) PB
  float* gn = reinterpret_cast<float*>(inb + 4 * PB);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W;
  const float inv_scale = ldexpf(*inv_scale_ptr, -kHScaleExp);   // weight scale and staging scale
  {
    const float4* s = reinterpret_cast<const float4*>(a.wpk);
    float4* d = reinterpret_cast<float4*>(wl_hi);
    constexpr int N4 = C::A_HALVES * 2 * 2 / 16;
#pragma unroll 8
    for (int i = tid; i < N4; i += C::THREADS) d[i] = s[i];
  }
#pragma unroll
  for (int p = 0; p < D::NP; ++p)
    if (D::MODE[p] == SRC_GNRELU) gn_table(a.part[p], gn, reinterpret_cast<double*>(inb), tid, H, W);
  const int tiles_x = (W + C::TW - 1) / C::TW, tiles_y = (H + C::TH - 1) / C::TH;
  const int ntiles = a.B * tiles_x * tiles_y;
  auto coords = [&](int tile, int& b, int& y0, int& x0) {
    b = tile / (tiles_x * tiles_y);
    const int rem = tile % (tiles_x * tiles_y);
    y0 = (rem / tiles_x) * C::TH;
    x0 = (rem % tiles_x) * C::TW;
  };
  int tile = blockIdx.x;
  if (tile >= ntiles) return;   // whole block
  H3PixStager<KIND, RW, WAVES, 0, false, MS> st;
  const int xe = KIND == 0 ? xguard_exp(a.xbound)
                 : D::MODE[0] == SRC_GNRELU ? gguard_exp(a.part[0].gamma, a.part[0].beta, H, W) : 0;
  st.xs = ldexpf(1.0f, -xe);
  const float xr = ldexpf(1.0f, xe + kHScaleExp);   // part 0's units -> the h parts' 2^kHScaleExp
  int b, y0, x0;
  coords(tile, b, y0, x0);
  if (!(ABL & 2)) st.template load<0>(a, b, y0, x0, tid);
  __syncthreads();   // gn visible to the staging
  if (!(ABL & 2)) {
    st.template store<0>(inb, inb + PB, gn, tid, x0, W);
    st.template load<1>(a, b, y0, x0, tid);
  }
  __syncthreads();
  int par = 0;
  const int hi = lane >> 5, col = lane & 31;
  const int rwave = wave % C::RWAVES, m0 = (wave / C::RWAVES) * C::MTL;   // row group, m-tiles
  const bool early = a.skew > 0 && ((wave >> (a.skew - 1)) & 1) != 0;
  for (; tile < ntiles; tile += gridDim.x) {
    coords(tile, b, y0, x0);
    const int next = tile + (int)gridDim.x;
    int nb = 0, ny0 = 0, nx0 = 0;
    if (next < ntiles) coords(next, nb, ny0, nx0);
    const int yw = y0 + rwave * RW;   // this wave's first row
    const int x = x0 + col;
    floatx16 acc[MT][RW], accn[MT][RW];   // sign-balanced pair (h3_mfma_chunk)
    float cst[MT][RW][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[m][r][j] = accn[m][r][j] = 0.0f;
    cell_c_load<C>(a, b, yw, x, hi, cst, m0);
    auto step = [&](auto CHc) {
      constexpr int CH = decltype(CHc)::value;
      constexpr bool F_NEXT = CH + 1 >= NCHK;   // following chunk: the next tile's first
      constexpr int F = F_NEXT ? 0 : CH + 1;
      constexpr bool A_NEXT = CH + 2 >= NCHK;   // the chunk after it
      constexpr int AC = A_NEXT ? CH + 2 - NCHK : CH + 2;
      const char* cur = inb + 2 * par * PB;
      char* oth = inb + 2 * (par ^ 1) * PB;
      auto stage = [&] {
        if (!(ABL & 2)) {
          if (!F_NEXT || next < ntiles) st.template store<F>(oth, oth + PB, gn, tid, 0, W);
          if (!A_NEXT)
            st.template load<AC>(a, b, y0, x0, tid);
          else if (next < ntiles)
            st.template load<AC>(a, nb, ny0, nx0, tid);
        }
      };
      // The step's barrier aligns every wave's phases, so a SIMD's two waves would stage (VALU)
      // and run their MFMAs at the same times.  With a.skew = k > 0 the waves with bit k-1 of
      // their index set (half of them) stage before their MFMAs and the others after, so that
      // staging overlaps MFMAs on a SIMD shared by one wave of each half (which bit pairs the
      // waves that way is measured per cell: CellDef::SKEW).  Buffer `oth` is free from the
      // start of the step (last read by the previous step's MFMAs, before its barrier), so
      // either order is safe and the results are the same.
      if (early) stage();
      xguard_rescale<C, KIND, CH, PRECISE>(acc, accn, xr);
      if (!(ABL & 1)) h3_mfma_chunk<C, CH, PIPE != 0, PRECISE, (ABL >> 3) & 3>(acc, accn, wl_hi, wl_lo, cur, cur + PB, rwave, lane, m0);
      if (!early) stage();
      if constexpr (CH == NCHK - 1) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int r = 0; r < RW; ++r)
            if constexpr (PRECISE) acc[m][r] -= accn[m][r];
        cell_epilogue<C, ABL, PRECISE>(a, acc, cst, inv_scale, b, yw, x, hi, m0);
      }
      __syncthreads();   // buffer `oth` staged; buffer `cur` free for the step after next
      par ^= 1;
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    if constexpr (NCHK > 2) step(std::integral_constant<int, 2>{});
  }
}

// DB: 1 double-buffered kernel, 0 single-buffered; PIPE: pipelined fragment reads.  Per
// cell in CellDef, from tools/microbench/cell_bench.cpp at the headline geometry (ms,
// DB0/PIPE0 DB0/PIPE1 DB1/PIPE0 DB1/PIPE1): cell0 .405 .379 .352 .324, cell1 .097 .090
// .091 .086, cell3 .087 .082 .083 .082, cell4 .155 .170 .208 .193 (cell 4's second
// buffer or second fragment set costs it a block per CU).  A warp-specialised form (4
// staging waves beside the 8 MFMA waves) measured slower (cell 0 0.43 vs 0.40 ms).  Round 5:
// with the double-buffered kernel's wave halves skewed (CellDef::SKEW) cell 3 is faster
// double-buffered too (95.0 -> 90.8 us per plane in the sweep), cell 4 still is not (161 -> 200).
template <int KIND, int RW = CellDef<KIND>::H3RW, int WAVES = CellDef<KIND>::H3WAVES, int ABL = 0,
          int DB = CellDef<KIND>::H3DB, int PIPE = CellDef<KIND>::H3PIPE, bool PRECISE = false,
          int MS = CellDef<KIND>::H3MS>
static hipError_t run_cell_h3_(const CellArgs& a, const float* inv_scale, int cu, int kid,
                               hipStream_t s) {
  using C = H3Cfg<KIND, RW, WAVES, MS>;
  constexpr size_t lds = C::LDS_BYTES + (DB ? (size_t)C::NPIX * 32 * 2 : 0);
  static_assert(lds <= 160 * 1024, "h3 cell tile exceeds LDS");
  const void* fn = DB ? (const void*)lstm_cell_h3db_kernel<KIND, RW, WAVES, ABL, PIPE, PRECISE, MS>
                      : (const void*)lstm_cell_h3_kernel<KIND, RW, WAVES, ABL, PIPE, PRECISE, MS>;
  static bool attr_set[kMaxDevices] = {};
  if (hipError_t e = ensure_dyn_lds(fn, (int)lds, attr_set); e != hipSuccess) return e;
  const int ntiles = a.B * ((a.W + C::TW - 1) / C::TW) * ((a.H + C::TH - 1) / C::TH);
  const int per_cu = std::max(1, (int)((160 * 1024) / lds));
  const int grid = std::max(1, std::min(ntiles, cu * per_cu));
  // the staging order of the double-buffered kernel's wave halves (lstm_cell_h3db_kernel): per
  // cell the wave bit measured fastest at the headline (tools/gpu_envsets_ab.sh over
  // AARMVS_CELL_SKEW = 0..3: cell 0 311 -> 296 us with bit 2, cell 1 100.5 -> 91.3 with bit 1,
  // cell 2 29.3 -> 28.5; bit-identical); AARMVS_CELL_SKEW overrides it for every cell
  const char* skew_s = std::getenv("AARMVS_CELL_SKEW");   // read per launch (tests switch it)
  const int skew_env = (skew_s && *skew_s) ? std::atoi(skew_s) : -1;
  CellArgs ak = a;
  ak.skew = skew_env >= 0 ? skew_env : CellDef<KIND>::SKEW;
  ProfScope ps(s, kid);
  if (DB)
    hipLaunchKernelGGL((lstm_cell_h3db_kernel<KIND, RW, WAVES, ABL, PIPE, PRECISE, MS>), dim3(grid),
                       dim3(C::THREADS), lds, s, ak, inv_scale);
  else
    hipLaunchKernelGGL((lstm_cell_h3_kernel<KIND, RW, WAVES, ABL, PIPE, PRECISE, MS>), dim3(grid),
                       dim3(C::THREADS), lds, s, ak, inv_scale);
  return hipGetLastError();
}
// The training sweep (a.z_out set: the record for the BPTT) runs the unbiased gate activations
// (PRECISE, device_common.h); the inference sweep the fast ones.
template <int KIND, int RW = CellDef<KIND>::H3RW, int WAVES = CellDef<KIND>::H3WAVES, int ABL = 0,
          int DB = CellDef<KIND>::H3DB, int PIPE = CellDef<KIND>::H3PIPE, int MS = CellDef<KIND>::H3MS>
static hipError_t run_cell_h3(const CellArgs& a, const float* inv_scale, int cu, int kid,
                              hipStream_t s) {
  return a.z_out ? run_cell_h3_<KIND, RW, WAVES, ABL, DB, PIPE, true, MS>(a, inv_scale, cu, kid, s)
                 : run_cell_h3_<KIND, RW, WAVES, ABL, DB, PIPE, false, MS>(a, inv_scale, cu, kid, s);
}

// Tile shape of the cells with two or more m-tiles (round 6, second session; every shape is
// bit-identical, tests/test_gpu_parity.py::test_cell_tile_shapes_are_bit_identical):
//   0: the CellDef configuration (8 waves, one per 32-pixel row, all m-tiles: 8-row tiles);
//   1: 8 waves, two per row (H3Cfg MS = 2, each half the m-tiles): 4-row tiles, twice the blocks;
//   2: 16 waves, two per row: 8-row tiles at four waves per SIMD instead of two.
// In isolation (tools/microbench/cell_bench.cpp CB_SMALL, profiles/r06s6_cell_shapes.txt) shapes
// 1 and 2 beat 0 on small grids and on cell 0 at the headline (128x160 cell 0 12 -> 9 us, 1600x1184
// cell 0 384 -> 314 us).  In the multi-stream sweep they do not (profiles/r06s7_cell_shapes_ab.txt:
// headline cell 0 300 -> 296 us, cells 1 and 2 1 us slower, config 1 0.353 -> 0.341 G hyp/s --
// twice the LDS-bound blocks crowd out the units of the other streams, config 2 +1.5%, the
// training step unchanged), so shape 0 stays the default.  AARMVS_CELL_MS (read per launch)
// selects a shape for every such cell.
template <int KIND>
static int cell_shape(const CellArgs&, int) {
  const char* e = std::getenv("AARMVS_CELL_MS");
  return (e && *e) ? std::max(0, std::min(2, std::atoi(e))) : 0;
}
template <int KIND>
static hipError_t run_cell(const CellArgs& a, const float* inv_scale, int cu, int kid, hipStream_t s) {
  using D = CellDef<KIND>;
  if constexpr (D::HID >= 16) {
    const int sh = cell_shape<KIND>(a, cu);
    if (sh == 1) return run_cell_h3<KIND, 1, 8, 0, D::H3DB, D::H3PIPE, 2>(a, inv_scale, cu, kid, s);
    if (sh == 2) return run_cell_h3<KIND, 1, 16, 0, D::H3DB, D::H3PIPE, 2>(a, inv_scale, cu, kid, s);
  }
  return run_cell_h3<KIND>(a, inv_scale, cu, kid, s);
}

// ---------------------------------------------------------------------------
// deConvGnReLU's transposed conv (module.py:281): ConvTranspose2d(16,16,3,s2,p1,op1), plus
// GroupNorm(2,16) partial sums (the GN+ReLU itself is fused into the consuming cell's input
// staging).
// ---------------------------------------------------------------------------
// deconv_px: one thread per input pixel of an 8 x 32 tile (its 2 x 2 output quad, uniform
// weight taps) and all batch elements in one launch.  The tile and its bottom / right neighbours (9 x 33 px, 19
// KB) are staged once in LDS channel-major; each thread accumulates its 2 x 2 output quad's
// 64 values and stores the quad straight to NHWC (each thread's two 128-B output row runs are
// completed by its own eight 16-B stores).  The round-1 form staged 2 input rows and 2
// output rows of a 256-pixel segment in 76 KB of LDS (2 blocks per CU, 3 barriers per
// segment, a partial last segment per row): 84 / 47 us per plane at the headline geometry
// against 71 / 37 us here (profiles/r02_*).
constexpr int kDpTH = 8, kDpTW = 32;
// One block per 8 x 32 input tile: the tile and its bottom / right neighbours (9 x 33 px)
// staged once in LDS channel-major, the 16 x 9 x 16 weights in LDS (broadcast reads).  A
// thread takes two input pixels (rows ty and ty + 4) and one half of the output channels
// (8), accumulates the 2 x 2 output quads of both pixels (deconv_px2: every weight read
// feeds two pixels' FMAs; 67 vs 74 us at H/2 -> H for one pixel x 16 channels per thread,
// bit-identical outputs), and stores the quads straight to NHWC.  The VALU reference for
// deconv_mfma_kernel (the library's; tools/microbench/cell_bench A/Bs the two).
// ABL: ablation bits for tools/microbench/cell_bench only (the library instantiates 0):
// 1 no output stores, 2 no channel loop, 4 no input staging loads
template <int ABL = 0>
__global__ void __launch_bounds__(256) deconv_px2_kernel(const float* __restrict__ in,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias, int Hi,
                                                         int Wi, float* __restrict__ out,
                                                         double* __restrict__ gn_part) {
  constexpr int SH = kDpTH + 1, SW = kDpTW + 1;
  __shared__ float tin[16][SH][SW];
  __shared__ float4 wsh[16 * 9 * 4];   // [ci][tap][co / 4]
  __shared__ float red[4 * 4];
  const int b = blockIdx.z, tid = threadIdx.x;
  const int y0 = blockIdx.y * kDpTH, x0 = blockIdx.x * kDpTW;
  const int hc = tid >> 7, r = tid & 127;   // output channels 8 hc .. 8 hc + 7
  const int tx = r & 31, tyb = r >> 5;      // pixels (tyb, tx) and (tyb + 4, tx)
  const int ix = x0 + tx;
  const int Wo = 2 * Wi;
  const float* ib = in + (size_t)b * 16 * Hi * Wi;
  for (int i = tid; i < SH * SW * 4; i += 256) {
    const int c4 = i & 3, px = i >> 2, yy = px / SW, xx = px - yy * SW;
    const int gy = y0 + yy, gx = x0 + xx;
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!(ABL & 4) && gy < Hi && gx < Wi)
      q = *reinterpret_cast<const float4*>(ib + ((size_t)gy * Wi + gx) * 16 + 4 * c4);
    tin[4 * c4 + 0][yy][xx] = q.x;
    tin[4 * c4 + 1][yy][xx] = q.y;
    tin[4 * c4 + 2][yy][xx] = q.z;
    tin[4 * c4 + 3][yy][xx] = q.w;
  }
  for (int i = tid; i < 16 * 9 * 4; i += 256) wsh[i] = reinterpret_cast<const float4*>(w)[i];
  __syncthreads();
  float o[2][4][8];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int c = 0; c < 8; ++c) o[p][q][c] = 0.f;
#pragma unroll 1
  for (int ci = 0; ci < ((ABL & 2) ? 1 : 16); ++ci) {
    float v[2][4];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ty = tyb + 4 * p;
      v[p][0] = tin[ci][ty][tx];
      v[p][1] = tin[ci][ty][tx + 1];
      v[p][2] = tin[ci][ty + 1][tx];
      v[p][3] = tin[ci][ty + 1][tx + 1];
    }
    const float4* wc = wsh + ci * 9 * 4 + 2 * hc;
#pragma unroll
    for (int c4 = 0; c4 < 2; ++c4) {
      float4 kt[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) kt[t] = wc[t * 4 + c4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = 4 * c4 + u;
        auto k = [&](int tap) {
          const float4 q = kt[tap];
          return u == 0 ? q.x : u == 1 ? q.y : u == 2 ? q.z : q.w;
        };
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const float v00 = v[p][0], v01 = v[p][1], v10 = v[p][2], v11 = v[p][3];
          o[p][0][c] = fmaf(v00, k(4), o[p][0][c]);
          o[p][1][c] = fmaf(v00, k(5), fmaf(v01, k(3), o[p][1][c]));
          o[p][2][c] = fmaf(v00, k(7), fmaf(v10, k(1), o[p][2][c]));
          o[p][3][c] = fmaf(v00, k(8), fmaf(v01, k(6), fmaf(v10, k(2), fmaf(v11, k(0), o[p][3][c]))));
        }
      }
    }
  }
  float part[4] = {0.f, 0.f, 0.f, 0.f};
  float* ob = out + (size_t)b * 16 * 4 * Hi * Wi;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int iy = y0 + tyb + 4 * p;
    if (iy < Hi && ix < Wi) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4* d = reinterpret_cast<float4*>(ob + ((size_t)(2 * iy + (q >> 1)) * Wo + 2 * ix + (q & 1)) * 16 + 8 * hc);
#pragma unroll
        for (int c4 = 0; c4 < 2; ++c4) {
          float rr[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            rr[u] = o[p][q][4 * c4 + u] + bias[8 * hc + 4 * c4 + u];
            part[2 * hc] += rr[u];
            part[2 * hc + 1] += rr[u] * rr[u];
          }
          if (!(ABL & 1) || rr[0] == 1234.5f) d[c4] = make_float4(rr[0], rr[1], rr[2], rr[3]);
        }
      }
    }
  }
  block_sum<4>(part, red);
  if (tid == 0) {
    double* pp = gn_part + 4 * (((size_t)b * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
#pragma unroll
    for (int j = 0; j < 4; ++j) pp[j] = part[j];
  }
}

// deconv_mfma: the same transposed conv on the matrix cores.  Per 32 input pixels of a row
// (one wave) and input neighbour set (v00, v01, v10, v11: the pixel, its right, lower and
// lower-right neighbour), D[slot * 16 + co][px] += W_pair x V with the six tap pairs of
// pack_deconv_mfma_kernel: acc01 holds output pixels (2y, 2x) | (2y, 2x + 1), acc23
// (2y + 1, 2x) | (2y + 1, 2x + 1).  Each fp32 product as three split-fp16 products (w_hi
// v_hi + w_hi v_lo + w_lo v_hi); V is staged x 2^14 (|h| < 1: tanh outputs),
// the weights carry 2^e, both undone in the epilogue.  B fragments straight from the NHWC
// input (lane: pixel l & 31, channels 8 (l >> 5) .. +7, 32 contiguous bytes).  Block: 4
// waves x 2 rows = the 8 x 32 input tile of deconv_px2 (same GN partial grid).
typedef _Float16 dhalf8 __attribute__((ext_vector_type(8)));
// The 12 A fragments sit in LDS (12 KB per block, read per use) rather than in 48 VGPRs per
// lane, and a wave issues the loads of its two rows' three input rows (the middle one shared:
// 6 pixel loads instead of 8) before any MFMA, keeping them fp32 and splitting each just
// before use: 4 waves per SIMD instead of 3, 40 vs 48.6 us (deconv_1) and 16 vs 17.6 us
// (deconv_0) per plane at the headline against the round-4 form (A fragments in registers,
// each row's loads just before its MFMAs), bit-identical.
template <int ABL = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) deconv_mfma_kernel(const float* __restrict__ in,
                                                           const float* __restrict__ wfrag,
                                                           const float* __restrict__ bias, int Hi,
                                                           int Wi, float* __restrict__ out,
                                                           double* __restrict__ gn_part) {
  __shared__ dhalf8 afs[12 * 64];
  __shared__ double red[4 * 4];
  const int b = blockIdx.z, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int x0 = blockIdx.x * kDpTW;
  const int n = lane & 31, hh = lane >> 5;   // B/D column (pixel), channel half
  const int Wo = 2 * Wi;
  const float* ib = in + (size_t)b * 16 * Hi * Wi;
  const dhalf8* af = reinterpret_cast<const dhalf8*>(wfrag);
  for (int i = tid; i < 12 * 64; i += 256) afs[i] = af[i];
  const float inv = wfrag[6 * 2 * 64 * 8 / 2] * (1.0f / 16384.0f);
  const int iy0 = blockIdx.y * kDpTH + wave * 2, ix = x0 + n;
  float4 raw[3][2][2];   // [input row iy0 + r][column ix + c][channel quad]
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float4 q0 = make_float4(0.f, 0.f, 0.f, 0.f), q1 = q0;
      if (!(ABL & 4) && iy0 + r < Hi && ix + c < Wi) {
        const float4* sp = reinterpret_cast<const float4*>(ib + ((size_t)(iy0 + r) * Wi + ix + c) * 16 + 8 * hh);
        q0 = sp[0];
        q1 = sp[1];
      }
      raw[r][c][0] = q0;
      raw[r][c][1] = q1;
    }
  __syncthreads();   // A fragments in LDS
  // B fragment of one input pixel: channels 8 hh .. +7, x 2^14, split
  auto split = [&](const float4 (&q)[2], dhalf8& bh, dhalf8& bl) {
    const float v[8] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w};
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      uint32_t lo;
      const half2_t hi = __builtin_bit_cast(half2_t, h3_split2(v[j] * 16384.0f, v[j + 1] * 16384.0f, lo));
      const half2_t lw = __builtin_bit_cast(half2_t, lo);
      bh[j] = hi[0];
      bh[j + 1] = hi[1];
      bl[j] = lw[0];
      bl[j + 1] = lw[1];
    }
  };
  double part[4] = {0.0, 0.0, 0.0, 0.0};   // fp64 GroupNorm partials (E[x^2] - E[x]^2 cancels)
  typedef float fx16 __attribute__((ext_vector_type(16)));
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    const int iy = iy0 + rr;
    if (iy < Hi) {
      dhalf8 b00h, b00l, b01h, b01l, b10h, b10l, b11h, b11l;
      split(raw[rr][0], b00h, b00l);
      split(raw[rr][1], b01h, b01l);
      split(raw[rr + 1][0], b10h, b10l);
      split(raw[rr + 1][1], b11h, b11l);
      fx16 a01, a23;
#pragma unroll
      for (int r = 0; r < 16; ++r) a01[r] = a23[r] = 0.f;
      if (!(ABL & 2)) {
        auto mm = [&](fx16 acc, int p, dhalf8 bh, dhalf8 bl) {
          const dhalf8 ah = afs[(p * 2 + 0) * 64 + lane], al = afs[(p * 2 + 1) * 64 + lane];
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
          return acc;
        };
        a01 = mm(a01, 0, b00h, b00l);
        a01 = mm(a01, 1, b01h, b01l);
        a23 = mm(a23, 2, b00h, b00l);
        a23 = mm(a23, 3, b01h, b01l);
        a23 = mm(a23, 4, b10h, b10l);
        a23 = mm(a23, 5, b11h, b11l);
      }
      if (ix < Wi) {
        float* ob = out + (size_t)b * 16 * 4 * Hi * Wi;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int slot = g >> 1, c0 = 4 * hh + 8 * (g & 1), grp = g & 1;
#pragma unroll
          for (int acc_i = 0; acc_i < 2; ++acc_i) {
            const fx16& A = acc_i ? a23 : a01;
            const int oy = 2 * iy + acc_i, ox = 2 * ix + slot;
            float v4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              v4[u] = fmaf(A[4 * g + u], inv, bias[c0 + u]);
              part[2 * grp] += (double)v4[u];
              part[2 * grp + 1] += (double)v4[u] * v4[u];
            }
            float4* d = reinterpret_cast<float4*>(ob + ((size_t)oy * Wo + ox) * 16 + c0);
            if (!(ABL & 1) || v4[0] == 1234.5f) *d = make_float4(v4[0], v4[1], v4[2], v4[3]);
          }
        }
      }
    }
  }
  block_sum_d_store<4>(part, red, gn_part + 4 * (((size_t)b * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x));
}

// ---------------------------------------------------------------------------
// conv_0 head (drmvsnet.py:117,165: Conv2d(8,1,3,pad 1)) fused with the online
// winner-take-all update (drmvsnet.py:324-334) and the optional cost-volume store.
// ---------------------------------------------------------------------------
constexpr int kHeadTH = 8, kHeadTW = 32;

// drmvsnet.py:324-334 for one pixel: p = exp(cost) (no max-subtraction), strict-< flag,
// the arithmetic select of max_prob and depth, exp_sum += p -- op for op (contract off)
__device__ __forceinline__ void wta_select(float cost, float dv, float& max_prob, float& depth,
                                           float& exp_sum) {
#pragma clang fp contract(off)
  const float pr = expf(cost);
  const float mp = max_prob;
  const float f = (mp < pr) ? 1.0f : 0.0f;
  max_prob = __fadd_rn(__fmul_rn(f, pr), __fmul_rn(1.0f - f, mp));
  depth = __fadd_rn(__fmul_rn(f, dv), __fmul_rn(1.0f - f, depth));
  exp_sum = __fadd_rn(exp_sum, pr);
}

// aarmvs_wta_update: the online WTA of one plane on a caller-given cost slice [B,HW]
__global__ void __launch_bounds__(256) wta_update_kernel(const float* __restrict__ cost,
                                                         const float* __restrict__ depth_d,
                                                         float* __restrict__ max_prob,
                                                         float* __restrict__ depth,
                                                         float* __restrict__ exp_sum, int HW) {
  const int b = blockIdx.y;
  const float dv = depth_d[b];
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    const size_t q = (size_t)b * HW + p;
    float mp = max_prob[q], dp = depth[q], es = exp_sum[q];
    wta_select(cost[q], dv, mp, dp, es);
    max_prob[q] = mp;
    depth[q] = dp;
    exp_sum[q] = es;
  }
}

hipError_t launch_wta_update(const float* cost, const float* depth_d, float* max_prob,
                             float* depth, float* exp_sum, int B, int HW, hipStream_t s) {
  const int blocks = std::max(1, std::min((HW + 255) / 256, 4096));
  ProfScope ps(s, K_HEAD_WTA);
  hipLaunchKernelGGL(wta_update_kernel, dim3(blocks, B), dim3(256), 0, s, cost, depth_d, max_prob,
                     depth, exp_sum, HW);
  return hipGetLastError();
}

// The haloed h4 tile sits in LDS pixel-major (32 B per pixel, the NHWC layout): a pixel's 9
// taps are 18 ds_read_b128 (the fma order stays channel-major, tap-minor), the staging 2 16-B
// stores per pixel (27.8 vs 28.8 us per plane at the headline against a channel-major tile
// read by 72 scalar LDS loads; bit-identical).
__global__ void __launch_bounds__(256) head_wta_kernel(const float* __restrict__ h4,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias, int H,
                                                        int W, const float* __restrict__ dvals,
                                                        int d, int D, float* __restrict__ cost_out,
                                                        int wta, float* __restrict__ max_prob,
                                                        float* __restrict__ exp_sum,
                                                        float* __restrict__ depth,
                                                        double* __restrict__ zero_stats,
                                                        int zero_n) {
#pragma clang fp contract(off)
  constexpr int TW2 = kHeadTW + 2, NPX = (kHeadTH + 2) * TW2;
  __shared__ float4 t[NPX][2];
  if (zero_stats && blockIdx.x == 0 && blockIdx.y == 0)
    for (int i = threadIdx.x; i < zero_n; i += blockDim.x) zero_stats[i] = 0.0;
  const int b = blockIdx.y, HW = H * W;
  const int tiles_x = (W + kHeadTW - 1) / kHeadTW;
  const int y0 = (blockIdx.x / tiles_x) * kHeadTH, x0 = (blockIdx.x % tiles_x) * kHeadTW;
  const float* hb = h4 + (size_t)b * 8 * HW;
  // this thread's pixel and its WTA state, loaded with the tile (one memory round trip, not a
  // second one after the conv)
  const int ty = threadIdx.x / kHeadTW, tx = threadIdx.x % kHeadTW;
  const int y = y0 + ty, x = x0 + tx;
  const bool own = y < H && x < W;
  const int p = own ? y * W + x : 0;
  const size_t q = (size_t)b * HW + p;
  float mp = 0.f, dp = 0.f, es = 0.f;
  if (wta && own) {
    mp = max_prob[q];
    dp = depth[q];
    es = exp_sum[q];
  }
  for (int rem = threadIdx.x; rem < NPX; rem += 256) {
    const int yy = y0 - 1 + rem / TW2, xx = x0 - 1 + rem % TW2;
    float4 q0 = make_float4(0.f, 0.f, 0.f, 0.f), q1 = q0;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
      const float4* src = reinterpret_cast<const float4*>(hb + ((size_t)yy * W + xx) * 8);
      q0 = src[0];
      q1 = src[1];
    }
    t[rem][0] = q0;
    t[rem][1] = q1;
  }
  __syncthreads();
  if (!own) return;
  float v[9][8];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int qt = (ty + tap / 3) * TW2 + tx + tap % 3;
    const float4 a0 = t[qt][0], a1 = t[qt][1];
    v[tap][0] = a0.x; v[tap][1] = a0.y; v[tap][2] = a0.z; v[tap][3] = a0.w;
    v[tap][4] = a1.x; v[tap][5] = a1.y; v[tap][6] = a1.z; v[tap][7] = a1.w;
  }
  float acc = 0.f;
#pragma unroll
  for (int ci = 0; ci < 8; ++ci)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) acc = fmaf(v[tap][ci], w[ci * 9 + tap], acc);
  const float cost = acc + bias[0];
  if (cost_out) cost_out[((size_t)b * D + d) * HW + p] = cost;
  if (wta) {
    wta_select(cost, dvals[b * D + d], mp, dp, es);
    max_prob[q] = mp;
    depth[q] = dp;
    exp_sum[q] = es;
  }
}

__global__ void finalize_kernel(const float* __restrict__ max_prob, const float* __restrict__ exp_sum,
                                const float* __restrict__ depth, size_t n, float* depth_out,
                                float* conf_out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    if (depth_out) depth_out[i] = depth[i];
    if (conf_out) conf_out[i] = __fdiv_rn(max_prob[i], exp_sum[i]);
  }
}

// softmax over D (dim=1 of [B,D,H,W], drmvsnet.py:291/:342); one thread per (b, pixel),
// coalesced over pixels.  Two passes over D instead of three: the running max and the
// rescaled running sum in one (online softmax, one exp per element: e = exp(-|v - m|)
// serves both the rescale of the sum when v raises the max and the new term otherwise),
// then exp(v - m) / sum.  Four planes' loads in flight per iteration.
__global__ void __launch_bounds__(256) softmax_depth_kernel(const float* __restrict__ cost,
                                                            float* __restrict__ prob, int D,
                                                            int HW) {
  const int b = blockIdx.y;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x) {
    const float* c = cost + (size_t)b * D * HW + p;
    float* o = prob + (size_t)b * D * HW + p;
    float m = -INFINITY, s = 0.f;
    auto add = [&](float v) {
      const float dv = v - m;
      const float e = expf(-fabsf(dv));
      if (dv > 0.f) {
        s = s * e + 1.0f;
        m = v;
      } else {
        s += e;
      }
    };
    int d = 0;
    for (; d + 4 <= D; d += 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = c[(size_t)(d + u) * HW];
#pragma unroll
      for (int u = 0; u < 4; ++u) add(v[u]);
    }
    for (; d < D; ++d) add(c[(size_t)d * HW]);
    const float inv = 1.0f / s;
    for (d = 0; d + 4 <= D; d += 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = c[(size_t)(d + u) * HW];
#pragma unroll
      for (int u = 0; u < 4; ++u) o[(size_t)(d + u) * HW] = expf(v[u] - m) * inv;
    }
    for (; d < D; ++d) o[(size_t)d * HW] = expf(c[(size_t)d * HW] - m) * inv;
  }
}

// NCHW <-> NHWC for the API edges (aarmvs_unet_step's input slice, the debug slice copy):
// one thread per (b, pixel), all channels.
__global__ void __launch_bounds__(256) layout_kernel(const float* __restrict__ in,
                                                     float* __restrict__ out, int C, int HW,
                                                     int to_nhwc, unsigned* __restrict__ xmax) {
  const int b = blockIdx.y;
  const float* ib = in + (size_t)b * C * HW;
  float* ob = out + (size_t)b * C * HW;
  float mx = 0.f;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < HW; p += gridDim.x * blockDim.x)
    for (int c = 0; c < C; ++c) {
      if (to_nhwc) {
        const float v = ib[(size_t)c * HW + p];
        ob[(size_t)p * C + c] = v;
        const float av = fabsf(v);
        mx = (av > mx || av != av) ? av : mx;
      } else {
        ob[(size_t)c * HW + p] = ib[(size_t)p * C + c];
      }
    }
  if (xmax) {   // |x| bound for cell 0's fp16 range guard (one atomic per wave)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float q = __shfl_xor(mx, o, 64);
      mx = (q > mx || q != q) ? q : mx;
    }
    const unsigned bits = __float_as_uint(mx != mx ? INFINITY : mx);
    if ((threadIdx.x & 63) == 0 &&
        bits > __hip_atomic_load(xmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(xmax, bits);
  }
}

hipError_t launch_layout(const float* in, float* out, int B, int C, int HW, bool to_nhwc,
                         hipStream_t s, unsigned* xmax) {
  const int blocks = std::max(1, std::min((HW + 255) / 256, 4096));
  hipLaunchKernelGGL(layout_kernel, dim3(blocks, B), dim3(256), 0, s, in, out, C, HW,
                     to_nhwc ? 1 : 0, to_nhwc ? xmax : nullptr);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
TrainLayout train_layout(int B, int H, int W) {
  TrainLayout T{};
  auto al = [](size_t n) { return (n + 63) / 64 * 64; };
  const size_t HW = (size_t)H * W;
  const size_t px[5] = {HW, HW / 4, HW / 16, HW / 4, HW};
  for (int k = 0; k < 5; ++k) T.cell_px[k] = (size_t)B * px[k];
  T.x_plane = (size_t)B * HW * kC;
  size_t o = 0;
  for (int k = 0; k < 5; ++k) {
    T.h_off[k] = o;
    o += al(T.cell_px[k] * kCellHid[k]);
    T.c_off[k] = o;
    o += al(T.cell_px[k] * kCellHid[k]);
  }
  T.state_slab = o;
  o = 0;
  for (int k = 0; k < 5; ++k) {
    T.z_off[k] = o;
    o += al(T.cell_px[k] * 4 * kCellHid[k]);
  }
  T.z_slab = o;
  T.u0_off = 0;
  T.u1_off = al((size_t)B * (HW / 4) * 16);
  T.u_slab = T.u1_off + al((size_t)B * HW * 16);
  T.stats_slab = (size_t)B * 4 * kSlots * 2;
  return T;
}

UnetIO unet_io_ws(const Workspace& ws, int d) {
  UnetIO io{};
  for (int k = 0; k < 5; ++k) {
    io.h_prev[k] = ws.h[k][h_slot(k, d)];
    io.h_new[k] = ws.h[k][h_slot(k, d + 1)];
    io.c_prev[k] = ws.c[k];
    io.c_new[k] = ws.c[k];
    io.z[k] = nullptr;
  }
  io.u0 = ws.u0;
  io.u1 = ws.u1;
  io.reg_stats = ws.reg_stats;
  io.clear_stats = true;
  return io;
}

UnetIO unet_io_record(const TrainLayout& T, const aarmvs_train_record& r, int d) {
  UnetIO io{};
  const float* s0 = r.state + (size_t)d * T.state_slab;
  float* s1 = r.state + (size_t)(d + 1) * T.state_slab;
  float* z = r.z + (size_t)d * T.z_slab;
  for (int k = 0; k < 5; ++k) {
    io.h_prev[k] = s0 + T.h_off[k];
    io.c_prev[k] = s0 + T.c_off[k];
    io.h_new[k] = s1 + T.h_off[k];
    io.c_new[k] = s1 + T.c_off[k];
    io.z[k] = z + T.z_off[k];
  }
  float* u = r.u + (size_t)d * T.u_slab;
  io.u0 = u + T.u0_off;
  io.u1 = u + T.u1_off;
  io.reg_stats = r.stats + (size_t)d * T.stats_slab;
  io.clear_stats = false;
  return io;
}

hipError_t launch_unet_step(const float* x, const float* params, const SweepGeom& g,
                            const Workspace& ws, const UnetIO& io, hipStream_t s, int stages) {
  const ParamLayout& L = param_layout();
  const int H = g.H, W = g.W, B = g.B, cu = g.cu_count;
  hipError_t e;
  auto cell = [&](int k, std::initializer_list<ChanSrc> parts, int scale) {
    CellArgs a{};
    int i = 0;
    for (const ChanSrc& p : parts) a.part[i++] = p;
    a.nparts = i;
    a.h_new = io.h_new[k];
    a.c = io.c_new[k];
    a.c_in = io.c_prev[k];
    a.z_out = io.z[k];
    // split-fp16 A fragments: sign-balanced (odd taps negated) for the training cells,
    // positive for the inference cells
    a.wpk = params + (io.z[k] ? L.h3_off[k] : L.h3p_off[k]);
    a.bias = params + L.pk_off[P_C0B + 2 * k];
    a.B = B;
    a.H = H / scale;
    a.W = W / scale;
    return a;
  };
  // per-batch-element views of a cell's outputs (cells 3 and 4 are launched per element)
  auto per_b = [](CellArgs& a, int b, size_t px, int hid) {
    a.B = 1;
    a.h_new += b * hid * px;
    a.c += b * hid * px;
    a.c_in += b * hid * px;
    if (a.z_out) a.z_out += b * 4 * hid * px;
  };
  if (stages & 1) {
  // cell 0: [x, h0] @ H
  CellArgs a0 = cell(0, {{x, 32, SRC_PLAIN, nullptr, nullptr, nullptr},
                         {io.h_prev[0], 16, SRC_PLAIN, nullptr, nullptr, nullptr}}, 1);
  a0.xbound = ws.xbound;
  if ((e = run_cell<0>(a0, params + L.h3_scale_off + 0, cu, K_CELL0, s)) != hipSuccess) return e;
  }
  if (stages & 2) {
  // cell 1: [maxpool(h0'), h1] @ H/2
  CellArgs a1 = cell(1, {{io.h_new[0], 16, SRC_POOL, nullptr, nullptr, nullptr},
                         {io.h_prev[1], 16, SRC_PLAIN, nullptr, nullptr, nullptr}}, 2);
  if ((e = run_cell<1>(a1, params + L.h3_scale_off + 1, cu, K_CELL1, s)) != hipSuccess) return e;
  }
  if (stages & 4) {
  // cell 2: [maxpool(h1'), h2] @ H/4
  CellArgs a2 = cell(2, {{io.h_new[1], 16, SRC_POOL, nullptr, nullptr, nullptr},
                         {io.h_prev[2], 16, SRC_PLAIN, nullptr, nullptr, nullptr}}, 4);
  if ((e = run_cell<2>(a2, params + L.h3_scale_off + 2, cu, K_CELL2, s)) != hipSuccess) return e;
  }
  // GroupNorm statistics are per batch element, so the two cells that consume the deconvs'
  // normalised outputs are launched per batch element; each reduces its element's deconv
  // partials itself (gn_table) and block 0 stores the statistics.
  if (stages & 8) {
  // deconv_0: h2' (H/4) -> u0 (H/2) + GN stats
  int nblk0 = 0;
  {
    const int Hi = H / 4, Wi = W / 4;
    const dim3 grid((Wi + kDpTW - 1) / kDpTW, (Hi + kDpTH - 1) / kDpTH, B);
    {
      ProfScope ps(s, K_DECONV0);
      hipLaunchKernelGGL(deconv_mfma_kernel<0>, grid, dim3(256), 0, s, io.h_new[2], params + L.dcm_off[0],
                         params + L.pk_off[P_D0B], Hi, Wi, io.u0, ws.reg_part0);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    nblk0 = (int)(grid.x * grid.y);
  }
  // cell 3: [gnrelu(u0), h1', h3] @ H/2
  for (int b = 0; b < B; ++b) {
    const double* st = io.reg_stats + reg_stat_index(b, 0, 0);
    const size_t hq = (size_t)(H / 2) * (W / 2);
    CellArgs a3 = cell(3, {{io.u0 + b * 16 * hq, 16, SRC_GNRELU, st, params + L.pk_off[P_D0GW],
                            params + L.pk_off[P_D0GB], ws.reg_part0 + (size_t)b * nblk0 * 4, nblk0,
                            io.reg_stats + reg_stat_index(b, 0, 0)},
                           {io.h_new[1] + b * 16 * hq, 16, SRC_PLAIN, nullptr, nullptr, nullptr},
                           {io.h_prev[3] + b * 16 * hq, 16, SRC_PLAIN, nullptr, nullptr, nullptr}},
                       2);
    per_b(a3, b, hq, 16);
    if ((e = run_cell<3>(a3, params + L.h3_scale_off + 3, cu, K_CELL3, s)) != hipSuccess) return e;
  }
  }
  if (!(stages & 16)) return hipSuccess;
  // deconv_1: h3' (H/2) -> u1 (H) + GN stats
  int nblk1 = 0;
  {
    const int Hi = H / 2, Wi = W / 2;
    const dim3 grid((Wi + kDpTW - 1) / kDpTW, (Hi + kDpTH - 1) / kDpTH, B);
    {
      ProfScope ps(s, K_DECONV1);
      hipLaunchKernelGGL(deconv_mfma_kernel<0>, grid, dim3(256), 0, s, io.h_new[3], params + L.dcm_off[1],
                         params + L.pk_off[P_D1B], Hi, Wi, io.u1, ws.reg_part);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    nblk1 = (int)(grid.x * grid.y);
  }
  // cell 4: [gnrelu(u1), h0', h4] @ H
  for (int b = 0; b < B; ++b) {
    const double* st = io.reg_stats + reg_stat_index(b, 1, 0);
    const size_t hw = (size_t)H * W;
    CellArgs a4 = cell(4, {{io.u1 + b * 16 * hw, 16, SRC_GNRELU, st, params + L.pk_off[P_D1GW],
                            params + L.pk_off[P_D1GB], ws.reg_part + (size_t)b * nblk1 * 4, nblk1,
                            io.reg_stats + reg_stat_index(b, 1, 0)},
                           {io.h_new[0] + b * 16 * hw, 16, SRC_PLAIN, nullptr, nullptr, nullptr},
                           {io.h_prev[4] + b * 8 * hw, 8, SRC_PLAIN, nullptr, nullptr, nullptr}},
                       1);
    per_b(a4, b, hw, 8);
    if ((e = run_cell<4>(a4, params + L.h3_scale_off + 4, cu, K_CELL4, s)) != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_head_wta(const float* params, const SweepGeom& g, const UnetIO& io,
                           const Workspace& ws, const float* depth_values, int d,
                           float* cost_out, bool wta, hipStream_t s) {
  const ParamLayout& L = param_layout();
  const int blocks = ((g.W + kHeadTW - 1) / kHeadTW) * ((g.H + kHeadTH - 1) / kHeadTH);
  ProfScope ps(s, K_HEAD_WTA);
  hipLaunchKernelGGL(head_wta_kernel, dim3(blocks, g.B), dim3(256), 0, s, io.h_new[4],
                     params + L.pk_off[P_HW], params + L.pk_off[P_HB], g.H, g.W, depth_values, d,
                     g.D, cost_out, wta ? 1 : 0, ws.max_prob, ws.exp_sum, ws.depth,
                     io.clear_stats ? io.reg_stats : nullptr,
                     (int)(ws.reg_stats_bytes / sizeof(double)));
  return hipGetLastError();
}

hipError_t launch_finalize(const SweepGeom& g, const Workspace& ws, float* depth_out,
                           float* conf_out, hipStream_t s) {
  const size_t n = (size_t)g.B * g.H * g.W;
  const int blocks = (int)std::min<size_t>((n + 255) / 256, 4096);
  ProfScope ps(s, K_FINALIZE);
  hipLaunchKernelGGL(finalize_kernel, dim3(blocks), dim3(256), 0, s, ws.max_prob, ws.exp_sum,
                     ws.depth, n, depth_out, conf_out);
  return hipGetLastError();
}

hipError_t launch_softmax_depth(const float* cost, float* prob, int B, int D, int HW,
                                hipStream_t s) {
  const int blocks = std::max(1, std::min((HW + 255) / 256, 4096));
  ProfScope ps(s, K_SOFTMAX);
  hipLaunchKernelGGL(softmax_depth_kernel, dim3(blocks, B), dim3(256), 0, s, cost, prob, D, HW);
  return hipGetLastError();
}

}  // namespace aarmvs
