// C-ABI entry points of libaarmvs (include/aarmvs.h): argument validation, the
// parameter packing kernel, the workspace carve and the per-plane sweep schedule.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "aarmvs_internal.h"

namespace aarmvs {

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

static int hip_fail(hipError_t e, const char* where) {
  return fail(AARMVS_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

const ParamLayout& param_layout() {
  static ParamLayout L = [] {
    ParamLayout l{};
    size_t raw = 0, pk = 0;
    for (int i = 0; i < P_COUNT; ++i) {
      l.raw_off[i] = raw;
      l.pk_off[i] = pk;
      raw += kParamSize[i];
      pk += ((size_t)kParamSize[i] + 63) / 64 * 64;
    }
    for (int k = 0; k < 5; ++k) {
      l.h3_off[k] = pk;
      pk += ((size_t)cell_a_halves(k) + 63) / 64 * 64;   // 2 x halves = halves floats
    }
    for (int k = 0; k < 5; ++k) {
      l.h3p_off[k] = pk;
      pk += ((size_t)cell_a_halves(k) + 63) / 64 * 64;
    }
    l.h3_scale_off = pk;
    pk += 64;
    l.ow0t_off = pk;
    pk += 4 * 32 * 9;
    l.owb_scale_off = pk;
    pk += 64;
    l.owm_off = pk;
    pk += 4 * 3 * 64 * 8 / 2;   // halves -> floats
    for (int k = 0; k < 2; ++k) {
      l.dct_off[k] = pk;
      pk += 16 * 9 * 16;
    }
    for (int k = 0; k < 2; ++k) {
      l.dcm_off[k] = pk;
      pk += 6 * 2 * 64 * 8 / 2 + 64;   // halves -> floats, then the scale (64-float aligned)
    }
    for (int k = 0; k < 5; ++k) {
      l.dg_off[k] = pk;
      pk += ((size_t)dg_mtiles(k) * dg_mt_halves(k) / 2 + 63) / 64 * 64;
    }
    l.dg_scale_off = pk;
    pk += 64;
    l.raw_total = raw;
    l.pk_total = pk;
    return l;
  }();
  return L;
}

// ---------------------------------------------------------------------------
// Opt-in kernel timer (aarmvs_profile_*).  Events come from a pool that grows to
// the largest profiling window and is reused after aarmvs_profile_reset.
// ---------------------------------------------------------------------------
bool g_prof_on = false;
static std::mutex g_prof_mu;
static std::vector<hipEvent_t> g_prof_pool;
static size_t g_prof_used = 0;
struct ProfRec {
  int id;
  hipEvent_t a, b;
};
static std::vector<ProfRec> g_prof_recs;
static hipEvent_t g_prof_open[K_COUNT];
static double g_prof_ms[K_COUNT];
static long long g_prof_n[K_COUNT];

static const char* kKernelNames[K_COUNT] = {
    "cost_x", "omega_conv", "fusion", "omega_stats1", "omega_stats2",
    "lstm_cell0", "lstm_cell1", "lstm_cell2", "lstm_cell3", "lstm_cell4",
    "deconv0", "deconv1", "head_wta", "finalize", "softmax_depth", "homo_warp", "to_c8",
    "omega_stat_reduce", "gn_reduce", "evidential",
    "gate_bwd0", "gate_bwd1", "gate_bwd2", "gate_bwd3", "gate_bwd4",
    "dgrad0", "dgrad1", "dgrad2", "dgrad3", "dgrad4",
    "wgrad0", "wgrad1", "wgrad2", "wgrad3", "wgrad4",
    "gnb_partial", "deconv_bwd", "bwd_small", "cbw_chain", "cbw_feat", "cbw_small",
    "deconv_wgrad", "head_wgrad", "deform_sample"};

static hipEvent_t prof_event() {
  if (g_prof_used == g_prof_pool.size()) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    g_prof_pool.push_back(e);
  }
  return g_prof_pool[g_prof_used++];
}

void prof_mark(hipStream_t s, int id, bool begin) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  hipEvent_t e = prof_event();
  if (!e) return;
  (void)hipEventRecord(e, s);
  if (begin) {
    g_prof_open[id] = e;
  } else if (g_prof_open[id]) {
    g_prof_recs.push_back({id, g_prof_open[id], e});
    g_prof_open[id] = nullptr;
  }
}

static void prof_fold() {
  for (const ProfRec& r : g_prof_recs) {
    float ms = 0.f;
    if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      g_prof_ms[r.id] += ms;
      g_prof_n[r.id] += 1;
    }
  }
  g_prof_recs.clear();
  g_prof_used = 0;
}

int cu_count() {
  static int cu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      return 256;
    return n;
  }();
  return cu;
}

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

Workspace carve_workspace(void* base, int B, int H, int W, int nsrc) {
  Workspace ws{};
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = p ? p + off : nullptr;
    off = align_up(off + bytes, 256);
    return r;
  };
  const size_t HW = (size_t)H * W, HW2 = HW / 4, HW4 = HW / 16;
  ws.omega_stats_bytes = (size_t)B * nsrc * 3 * kSlots * 2 * sizeof(double);
  ws.reg_stats_bytes = (size_t)B * 4 * kSlots * 2 * sizeof(double);
  const size_t stats_begin = off;
  ws.omega_stats = reinterpret_cast<double*>(take(kPlaneGroup * ws.omega_stats_bytes));
  ws.reg_stats = reinterpret_cast<double*>(take(ws.reg_stats_bytes));
  ws.xbound = reinterpret_cast<unsigned*>(take(sizeof(unsigned)));
  ws.stats_bytes = off - stats_begin;
  const size_t wta_begin = off;
  ws.max_prob = reinterpret_cast<float*>(take(B * HW * 4));
  ws.exp_sum = reinterpret_cast<float*>(take(B * HW * 4));
  ws.depth = reinterpret_cast<float*>(take(B * HW * 4));
  ws.wta_bytes = off - wta_begin;
  ws.x_plane = (size_t)B * kC * HW;
  ws.t1_plane = (size_t)B * nsrc * HW;
  ws.xg[0] = reinterpret_cast<float*>(take(kPlaneGroup * ws.x_plane * 4));
  ws.xg[1] = reinterpret_cast<float*>(take(kPlaneGroup * ws.x_plane * 4));
  ws.x = ws.xg[0];
  for (int v = 0; v <= nsrc; ++v) ws.feat8[v] = reinterpret_cast<float*>(take(B * kC * HW * 4));
  ws.t1 = reinterpret_cast<float*>(take(kPlaneGroup * ws.t1_plane * 16));
  // one partial per omega block (haloed 16 x TW tiles, 14 x (TW - 2) outputs, TW >= 16; the
  // VALU variant's 16 x 32 output tiles are fewer) or statistics block (<= one per 1024 px)
  ws.omega_part_n = (int)std::max(((size_t)(W + 13) / 14) * ((size_t)(H + 13) / 14), (HW + 1023) / 1024);
  ws.omega_part = reinterpret_cast<double*>(
      take((size_t)kPlaneGroup * B * nsrc * ws.omega_part_n * 2 * sizeof(double)));
  // deconv_1's blocks (8 x 32 tiles of its H/2 x W/2 input) outnumber deconv_0's
  ws.reg_part = reinterpret_cast<double*>(
      take((size_t)B * ((W / 2 + 31) / 32) * ((H / 2 + 7) / 8) * 4 * sizeof(double)));
  ws.reg_part0 = reinterpret_cast<double*>(
      take((size_t)B * ((W / 4 + 31) / 32) * ((H / 4 + 7) / 8) * 4 * sizeof(double)));
  ws.u0 = reinterpret_cast<float*>(take(B * 16 * HW2 * 4));
  ws.u1 = reinterpret_cast<float*>(take(B * 16 * HW * 4));
  const size_t state_begin = off;
  ws.state_begin = p ? p + off : nullptr;
  const size_t cell_px[5] = {HW, HW2, HW4, HW2, HW};
  for (int k = 0; k < 5; ++k) {
    const size_t n = (size_t)B * kCellHid[k] * cell_px[k] * 4;
    for (int r = 0; r < kHRingMax; ++r) ws.h[k][r] = r < kHRing[k] ? reinterpret_cast<float*>(take(n)) : nullptr;
    ws.c[k] = reinterpret_cast<float*>(take(n));
  }
  ws.state_bytes = off - state_begin;
  ws.bytes = off;
  return ws;
}

// ---------------------------------------------------------------------------
// Parameter packing: cell weights [4*hid][cin][3][3] -> MFMA A operands
// [K/2][MT][64] with k = tap*cin + ci and m-tile row r -> cout (r>>3)*hid + 8*mt + (r&7).
// Everything else is copied (64-float aligned sections).
// ---------------------------------------------------------------------------
__global__ void pack_params_kernel(const float* __restrict__ raw, float* __restrict__ pk,
                                   ParamLayout L) {
  const int id = blockIdx.y;
  const int n = kParamSize[id];
  const float* src = raw + L.raw_off[id];
  float* dst = pk + L.pk_off[id];
  const bool is_cell_w = id >= P_C0W && id <= P_C4W && ((id - P_C0W) % 2 == 0);
  const int k = (id - P_C0W) / 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (!is_cell_w) {
      dst[i] = src[i];
      continue;
    }
    const int hid = kCellHid[k], cin = kCellCX[k] + hid, mt_n = hid / 8;
    const int l = i % 64, mt = (i / 64) % mt_n, s = i / (64 * mt_n);
    const int kk = 2 * s + (l >> 5);
    const int tap = kk / cin, ci = kk % cin;
    const int r = l & 31;
    const int cout = (r >> 3) * hid + 8 * mt + (r & 7);
    dst[i] = src[(cout * cin + ci) * 9 + tap];
  }
}

// Split-fp16 cell weights: w * 2^e = hi + lo (both fp16, hi = fp16(w 2^e),
// lo = fp16(w 2^e - hi)), e chosen per cell so that max|w| 2^e <= 2^14 (lo stays in
// fp16's normal range for all but tiny weights).  One block per cell.
__global__ void __launch_bounds__(256) pack_cell_h3_kernel(const float* __restrict__ raw,
                                                           float* __restrict__ pk, ParamLayout L) {
  __shared__ float red[4];
  const int k = blockIdx.x;
  const int hid = kCellHid[k], cin = cell_cin(k), cout = 4 * hid, mt_n = hid / 8;
  const float* w = raw + L.raw_off[P_C0W + 2 * k];   // [cout][cin][3][3]
  const int n = cout * cin * 9;
  float mx = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) mx = fmaxf(mx, fabsf(w[i]));
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int e = 0;
  if (mx > 0.f) {
    e = (int)floorf(log2f(16384.0f / mx));
    e = e < -20 ? -20 : (e > 20 ? 20 : e);
  }
  const float sc = ldexpf(1.0f, e);
  if (threadIdx.x == 0) pk[L.h3_scale_off + k] = ldexpf(1.0f, -e);
  const int halves = cell_a_halves(k);
  _Float16* hi = reinterpret_cast<_Float16*>(pk + L.h3_off[k]);
  _Float16* lo = hi + halves;
  _Float16* hip = reinterpret_cast<_Float16*>(pk + L.h3p_off[k]);
  _Float16* lop = hip + halves;
  for (int i = threadIdx.x; i < halves; i += blockDim.x) {
    const int j = i & 7, l = (i >> 3) & 63, rest = i >> 9;   // [chunk][tap][mt][lane][j]
    const int mt = rest % mt_n, tap = (rest / mt_n) % 9, c = rest / (mt_n * 9);
    const int r = l & 31, h = l >> 5;
    const int co = (r >> 3) * hid + 8 * mt + (r & 7);
    // a chunk of 8 valid channels is paired (convlstm.hip h3_mfma_chunk): its slot s < 5 holds
    // tap 2s (K half 0) and tap 2s+1 (K half 1) of those channels; slots 5..8 stay zero
    const bool paired = cin - 16 * c == 8;
    const int tp = paired ? 2 * tap + h : tap;
    const int ci = paired ? 16 * c + j : 16 * c + 8 * h + j;
    // slots with (slot + chunk) odd negated: the cells' sign-balanced accumulation (convlstm.hip)
    const bool neg = ((tap + c) & 1) != 0;
    const float v = ci < cin && tp < 9 ? w[(co * cin + ci) * 9 + tp] * sc : 0.f;
    const _Float16 vh = (_Float16)v, vl = (_Float16)(v - (float)vh);
    hip[i] = vh;
    lop[i] = vl;
    hi[i] = neg ? -vh : vh;   // (fp16 negation is exact: the balanced copy is the same split)
    lo[i] = neg ? -vl : vl;
  }
}

// omega conv3x3 32->4 weights [co][ci][tap] -> [tap][ci][co]: the 16 weights of one
// (tap, 4-channel group) are contiguous (scalar loads in the VALU form of the conv)
// and -> split-fp16 B fragments of v_mfma_f32_16x16x32_f16 for omega_conv's MFMA conv
// (the eight off-centre taps): per 8-channel chunk c and N tile k, column n = 4 u + co
// (tap slot u = 4 k + n / 4: taps 0..3, 5..8), k8 group g = lane / 16 against the A
// groups [sq hi | sq lo | sq hi | sq lo]: W hi for g < 2, W lo for g >= 2.  Lane l of
// fragment (c, k) holds B[8 g .. 8 g + 7][n = l % 16].  A power-of-two scale keeps the
// weights in fp16's normal range (undone in the kernel's epilogue).
__global__ void pack_omega_conv_kernel(const float* __restrict__ raw, float* __restrict__ pk,
                                       ParamLayout L) {
  __shared__ float red[4];
  const float* w = raw + L.raw_off[P_OW0];
  float* d = pk + L.ow0t_off;
  float mx = 0.f;
  for (int i = threadIdx.x; i < 4 * 32 * 9; i += blockDim.x) {
    const int co = i % 4, ci = (i / 4) % 32, tap = i / 128;
    d[i] = w[(co * 32 + ci) * 9 + tap];
    mx = fmaxf(mx, fabsf(d[i]));
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int e = 0;
  if (mx > 0.f) {
    e = (int)floorf(log2f(16384.0f / mx));
    e = e < -20 ? -20 : (e > 20 ? 20 : e);
  }
  const float sc = ldexpf(1.0f, e);
  if (threadIdx.x == 0) pk[L.owb_scale_off] = ldexpf(1.0f, -e);
  // omega_mfma's v_mfma_f32_32x32x16_f16 B fragments: per chunk c and kind k against
  // A = [sq hi | sq lo]: 0: [W_hi; W_hi], 1: [W_lo; 0], 2: [W_lo2; W_lo] with W = W_hi + W_lo +
  // W_lo2 (three fp16 terms: the weights exact to ~2^-33, so the conv carries no systematic
  // per-weight error; the dropped terms are sq_lo W_lo2 and sq_lo's own rounding, ~2^-22 random
  // per product); lane l holds B[8 (l >> 5) + j][n = l & 31] with column n = 4 u + co.  The
  // kernel passes them as the A operand (the product transposed: rows n, columns pixels), so
  // that slot u of row group g = u >> 1 lands in accumulator registers 4 g .. 4 g + 3 of lanes
  // 0-31 (u even) or 32-63 (u odd); tap slots u -> taps 0, 6, 1, 7, 2, 8, 3, 5 pair the taps of
  // one dx in one register group (omega_item's row sums)
  _Float16* bm = reinterpret_cast<_Float16*>(pk + L.owm_off);
  for (int i = threadIdx.x; i < 4 * 3 * 64 * 8; i += blockDim.x) {
    const int j = i & 7, lane = (i >> 3) & 63, k = (i >> 9) % 3, c = (i >> 9) / 3;
    const int n = lane & 31, u = n >> 2, g = u >> 1, co = n & 3;
    const int tap = (u & 1) ? (g < 3 ? 6 + g : 5) : g;
    const float x = w[(co * 32 + 8 * c + j) * 9 + tap] * sc;
    const _Float16 xh = (_Float16)x;
    const float r1 = x - (float)xh;
    const _Float16 xl = (_Float16)r1;
    const _Float16 xl2 = (_Float16)(r1 - (float)xl);
    const bool top = (lane >> 5) == 0;   // K rows 0-7: against sq hi
    bm[i] = k == 0 ? xh : k == 1 ? (top ? xl : (_Float16)0.0f) : (top ? xl2 : xl);
  }
}

// deconv weights [ci][co][ky][kx] (ConvTranspose2d) -> [ci][tap][co]: the 16 output
// channels of one (ci, tap) are contiguous, so the deconv's packed FMAs pair adjacent
// scalar registers
__global__ void pack_deconv_kernel(const float* __restrict__ raw, float* __restrict__ pk,
                                   ParamLayout L) {
  const int k = blockIdx.x;
  const float* w = raw + L.raw_off[k ? P_D1W : P_D0W];
  float* d = pk + L.dct_off[k];
  for (int i = threadIdx.x; i < 16 * 9 * 16; i += blockDim.x) {
    const int co = i % 16, tap = (i / 16) % 9, ci = i / 144;
    d[i] = w[(ci * 16 + co) * 9 + tap];
  }
}

// deconv_0/1 as split-fp16 MFMA A fragments (deconv_mfma_kernel): six tap pairs, rows
// m = slot * 16 + co (slot 0 / 1: the two output pixels of a pair), k = ci; lane l holds row
// l & 31, input channels 8 (l >> 5) .. +7.  Pairs (tap of slot 0 | slot 1, input pixel):
// (4 | 5, v00), (- | 3, v01), (7 | 8, v00), (- | 6, v01), (1 | 2, v10), (- | 0, v11) -- the
// ConvTranspose2d(k3, s2, p1, op1) taps feeding output (2y + a, 2x + b) from input (y, x)
// and its right / lower neighbours.  Values are scaled by 2^e (max |w| 2^e < 2^15).
__global__ void pack_deconv_mfma_kernel(const float* __restrict__ raw, float* __restrict__ pk,
                                        ParamLayout L) {
  __shared__ float red[4];
  const int k = blockIdx.x;
  const float* w = raw + L.raw_off[k ? P_D1W : P_D0W];   // [ci][co][3][3]
  float mx = 0.f;
  for (int i = threadIdx.x; i < 16 * 16 * 9; i += blockDim.x) mx = fmaxf(mx, fabsf(w[i]));
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int e = mx > 0.f ? 14 - ilogbf(mx) : 0;
  const float sc = ldexpf(1.0f, e);
  constexpr int kTap[6][2] = {{4, 5}, {-1, 3}, {7, 8}, {-1, 6}, {1, 2}, {-1, 0}};
  _Float16* f = reinterpret_cast<_Float16*>(pk + L.dcm_off[k]);
  for (int i = threadIdx.x; i < 6 * 64 * 8; i += blockDim.x) {
    const int j = i & 7, lane = (i >> 3) & 63, pair = i >> 9;
    const int m = lane & 31, slot = m >> 4, co = m & 15, ci = 8 * (lane >> 5) + j;
    const int tap = kTap[pair][slot];
    const float v = tap < 0 ? 0.f : w[(ci * 16 + co) * 9 + tap] * sc;
    const _Float16 hi = (_Float16)v;
    f[((pair * 2 + 0) * 64 + lane) * 8 + j] = hi;
    f[((pair * 2 + 1) * 64 + lane) * 8 + j] = (_Float16)(v - (float)hi);
  }
  if (threadIdx.x == 0) pk[L.dcm_off[k] + 6 * 2 * 64 * 8 / 2] = ldexpf(1.0f, -e);
}

// BPTT input-gradient conv of each cell: dL/d[input] = conv3x3(dL/dz) with the forward
// weight W[cz][ci][tap] (cz: gate channel, ci: input channel) transposed and flipped,
// A[ci][cz, tap] = W[cz][ci][8 - tap].  Fragments [m-tile][chunk][tap][hi, lo][lane][8]: lane l
// holds row ci = 32 mt + (l & 31), gate channels 16 chunk + 8 (l >> 5) .. +7; rows past cin are
// zero.  Power-of-two scale per cell as for the forward fragments.  One block per cell.
__global__ void __launch_bounds__(256) pack_dgrad_kernel(const float* __restrict__ raw,
                                                         float* __restrict__ pk, ParamLayout L) {
  __shared__ float red[4];
  const int k = blockIdx.x;
  const int hid = kCellHid[k], cin = cell_cin(k), cz = 4 * hid;
  const float* w = raw + L.raw_off[P_C0W + 2 * k];   // [cz][cin][3][3]
  const int n = cz * cin * 9;
  float mx = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) mx = fmaxf(mx, fabsf(w[i]));
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int e = 0;
  if (mx > 0.f) {
    e = (int)floorf(log2f(16384.0f / mx));
    e = e < -20 ? -20 : (e > 20 ? 20 : e);
  }
  const float sc = ldexpf(1.0f, e);
  if (threadIdx.x == 0) pk[L.dg_scale_off + k] = ldexpf(1.0f, -e);
  const int nch = dg_chunks(k), mtn = dg_mtiles(k);
  _Float16* f = reinterpret_cast<_Float16*>(pk + L.dg_off[k]);
  const int total = mtn * dg_mt_halves(k);
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const int j = i & 7, l = (i >> 3) & 63, hl = (i >> 9) & 1, rest = i >> 10;
    const int tap = rest % 9, c = (rest / 9) % nch, mt = rest / (9 * nch);
    const int ci = 32 * mt + (l & 31), z = 16 * c + 8 * (l >> 5) + j;
    // taps with (tap + chunk) odd negated: dgrad's sign-balanced accumulation (bptt.hip)
    const float sg = ((tap + c) & 1) ? -1.0f : 1.0f;
    const float v = ci < cin ? w[(z * cin + ci) * 9 + (8 - tap)] * sc * sg : 0.f;
    const _Float16 vh = (_Float16)v;
    f[i] = hl == 0 ? vh : (_Float16)(v - (float)vh);
  }
}

hipError_t launch_pack_params(const float* raw, float* packed, hipStream_t s) {
  const ParamLayout& L = param_layout();
  hipError_t e = hipMemsetAsync(packed, 0, L.pk_total * sizeof(float), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pack_params_kernel, dim3(32, P_COUNT), dim3(256), 0, s, raw, packed, L);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(pack_cell_h3_kernel, dim3(5), dim3(256), 0, s, raw, packed, L);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(pack_omega_conv_kernel, dim3(1), dim3(256), 0, s, raw, packed, L);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(pack_deconv_kernel, dim3(2), dim3(256), 0, s, raw, packed, L);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(pack_deconv_mfma_kernel, dim3(2), dim3(256), 0, s, raw, packed, L);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(pack_dgrad_kernel, dim3(5), dim3(256), 0, s, raw, packed, L);
  return hipGetLastError();
}

}  // namespace aarmvs

using namespace aarmvs;

extern "C" {

const char* aarmvs_last_error(void) { return g_err.c_str(); }

void aarmvs_profile_enable(int on) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof_on = on != 0;
}

void aarmvs_profile_reset(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  prof_fold();
  for (int i = 0; i < K_COUNT; ++i) {
    g_prof_ms[i] = 0.0;
    g_prof_n[i] = 0;
    g_prof_open[i] = nullptr;
  }
}

int aarmvs_profile_kernel_count(void) { return K_COUNT; }

const char* aarmvs_profile_kernel_name(int id) {
  return (id >= 0 && id < K_COUNT) ? kKernelNames[id] : nullptr;
}

int aarmvs_profile_read(int id, long long* launches, double* total_ms) {
  if (id < 0 || id >= K_COUNT || !launches || !total_ms)
    return fail(AARMVS_ERR_INVALID, "profile_read: bad arguments");
  std::lock_guard<std::mutex> lk(g_prof_mu);
  prof_fold();
  *launches = g_prof_n[id];
  *total_ms = g_prof_ms[id];
  return AARMVS_OK;
}
const char* aarmvs_version(void) { return "aarmvs-mi355x 0.1 (gfx950)"; }

size_t aarmvs_param_count(void) { return param_layout().raw_total; }
size_t aarmvs_packed_param_bytes(void) { return param_layout().pk_total * sizeof(float); }

int aarmvs_pack_params(const float* raw_params, void* packed, hipStream_t stream) {
  if (!raw_params || !packed) return fail(AARMVS_ERR_INVALID, "pack_params: null pointer");
  hipError_t e = launch_pack_params(raw_params, static_cast<float*>(packed), stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "pack_params");
}

int aarmvs_homo_warp(const float* src_fea, const float* rel_proj, const float* depth, int B,
                     int C, int H, int W, float* out, hipStream_t stream) {
  if (!src_fea || !rel_proj || !depth || !out) return fail(AARMVS_ERR_INVALID, "homo_warp: null pointer");
  if (B < 1 || C < 1 || H < 2 || W < 2)
    return fail(AARMVS_ERR_INVALID, "homo_warp: need B>=1, C>=1, H>=2, W>=2");
  hipError_t e = launch_homo_warp(src_fea, rel_proj, depth, B, C, H, W, out, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "homo_warp");
}

size_t aarmvs_homo_warp_backward_workspace_bytes(int B, int C, int H, int W) {
  if (B < 1 || C < 1 || H < 2 || W < 2) return 0;
  return homo_warp_bwd_workspace_bytes(B, C, H, W);
}

int aarmvs_homo_warp_backward(const float* grad_out, const float* rel_proj, const float* depth,
                              int B, int C, int H, int W, float* grad_src, void* workspace,
                              hipStream_t stream) {
  if (!grad_out || !rel_proj || !depth || !grad_src || !workspace)
    return fail(AARMVS_ERR_INVALID, "homo_warp_backward: null pointer");
  if (B < 1 || C < 1 || H < 2 || W < 2)
    return fail(AARMVS_ERR_INVALID, "homo_warp_backward: need B>=1, C>=1, H>=2, W>=2");
  hipError_t e = launch_homo_warp_bwd(grad_out, rel_proj, depth, B, C, H, W, grad_src, workspace, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "homo_warp_backward");
}

static int check_geom(int B, int H, int W, int nsrc) {
  if (B < 1) return fail(AARMVS_ERR_INVALID, "B must be >= 1");
  if (H < 4 || W < 4 || H % 4 || W % 4)
    return fail(AARMVS_ERR_INVALID,
                "H and W must be positive multiples of 4 (two 2x2 pools + two stride-2 deconvs)");
  if (nsrc < 1 || nsrc > AARMVS_MAX_SRC)
    return fail(AARMVS_ERR_INVALID, "nsrc must be in [1, AARMVS_MAX_SRC]");
  // the pipeline kernels address one view's 32-channel image with 32-bit byte offsets and
  // the per-view maps with 32-bit element indices
  const long long hw = (long long)H * W;
  if (hw * 128 >= (1ll << 32) || (long long)B * (nsrc + 1) * hw >= (1ll << 31))
    return fail(AARMVS_ERR_INVALID, "H x W (x B x views) too large for 32-bit image offsets");
  return AARMVS_OK;
}

size_t aarmvs_sweep_workspace_bytes(int B, int H, int W, int nsrc) {
  if (check_geom(B, H, W, nsrc) != AARMVS_OK) return 0;
  return carve_workspace(nullptr, B, H, W, nsrc).bytes;
}

size_t aarmvs_train_record_bytes(int B, int H, int W, int which) {
  if (check_geom(B, H, W, 1) != AARMVS_OK) return 0;
  const TrainLayout T = train_layout(B, H, W);
  switch (which) {
    case 0: return T.x_plane * sizeof(float);
    case 1: return T.state_slab * sizeof(float);
    case 2: return T.z_slab * sizeof(float);
    case 3: return T.u_slab * sizeof(float);
    case 4: return T.stats_slab * sizeof(double);
    case 5: return (size_t)B * H * W * 16;                        // t1 of one view
    case 6: return (size_t)B * 3 * kSlots * 2 * sizeof(double);   // omega statistics of one view
    default: return 0;
  }
}

int aarmvs_aux_stream(hipStream_t* out) {
  if (!out) return fail(AARMVS_ERR_INVALID, "aux_stream: null out");
  int dev = 0;
  hipError_t e = current_device(dev);
  if (e == hipSuccess) e = library_stream(dev, kLibStreams, *out);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "aux_stream");
}

float* aarmvs_state_ptr(void* workspace, int B, int H, int W, int nsrc, int planes,
                        int cell, int which) {
  if (!workspace || cell < 0 || cell > 4 || planes < 0 || check_geom(B, H, W, nsrc) != AARMVS_OK)
    return nullptr;
  Workspace ws = carve_workspace(workspace, B, H, W, nsrc);
  return which == 0 ? ws.h[cell][h_slot(cell, planes)] : ws.c[cell];
}

}  // extern "C"

// Multi-stream regulariser.  The U-Net step is five units run in order (U0 cell 0, U1 cell 1,
// U2 cell 2, U3 deconv_0 + cell 3, U4 deconv_1 + cell 4 and the head); a unit of plane d needs
// the earlier units of plane d and its own state only, so the units of neighbouring planes can
// run at once on different streams (stream 0 the caller's, the others library-owned).  Per unit
// and plane an event (a ring of kRegEvRing per unit):
//   data: a unit waits for the previous unit of its plane when that ran on another stream;
//   slots: unit k < 4 overwrites h_k's slot of plane d - kHRing[k]; it waits for that plane's
//   last reader of h_k when that ran on another stream (h0: U4, h1: U3, h2: U3, h3: U4; h4 is
//   read by U4's own head).  The other readers of the slot finished before the last one (the
//   data waits chain a plane's units).  c_k, u0, u1, the deconv partials and the WTA images
//   each have one unit as their only reader and writer.
// Bit-identical to one stream (the same kernels on the same inputs).
// How many streams: a process gets GPU_MAX_HW_QUEUES = 4 hardware queues here, and streams
// beyond that share them (a stream waiting on an event then blocks the other's work), so a
// sweep uses at most four: with an aux stream (the caller asks for concurrency), the cost stage
// on it and the units on three (the caller's + two library streams: cells 0-1 | cell 2,
// deconv_0, cell 3 | deconv_1, cell 4, head).  Small frames (B*H*W <= kSmallFramePx) instead
// put the cost stage on the caller's stream beside cells 0-1 and the other units on the aux
// stream and two library streams (cell 2 | deconv_0, cell 3 | deconv_1, cell 4, head), still
// four streams (the library's are shared with the backward, library_stream): their kernels are a few
// microseconds of one or two tiles per block, so the chain's latency, not the cost stage, is
// what overlapping hides (config 1: 0.279 -> 0.334 G hyp/s, profiles/r06o_small_frames.txt).
// Overrides (A/B runs): AARMVS_REG_STREAMS=1..5 the unit stream count (AARMVS_REG_STREAMS_REC for
// a training forward), AARMVS_REG_MAP five digits unit -> stream (unit 0 on stream 0),
// AARMVS_SMALL_PX the small-frame threshold.
constexpr int kRegMaxStreams = 5, kRegEvRing = 8;
static_assert(kRegMaxStreams - 1 <= kLibStreams, "the unit streams beyond the caller's are library streams");
static_assert(kRegEvRing > kHRingMax, "a unit's event is re-recorded only after its waiters are enqueued");
constexpr int kHLastReader[4] = {4, 3, 3, 4};
constexpr long kSmallFramePx = 65536;
static bool small_frame(long px) {
  const char* s = std::getenv("AARMVS_SMALL_PX");
  return px <= ((s && *s) ? std::atol(s) : kSmallFramePx);
}
static int reg_streams(bool aux, bool rec, bool small) {
  const char* s = std::getenv(rec ? "AARMVS_REG_STREAMS_REC" : "AARMVS_REG_STREAMS");
  const int n = (s && *s) ? std::atoi(s) : (!aux ? 1 : small ? 4 : 3);
  return std::max(1, std::min(kRegMaxStreams, n));
}
// the stream of each unit for n streams; returns the number of streams used
static int reg_unit_streams(int n, int (&us)[kUnetUnits]) {
  static const int map[kRegMaxStreams][kUnetUnits] = {
      {0, 0, 0, 0, 0}, {0, 0, 0, 1, 1}, {0, 0, 1, 1, 2}, {0, 0, 1, 2, 3}, {0, 1, 2, 3, 4}};
  for (int i = 0; i < kUnetUnits; ++i) us[i] = map[n - 1][i];
  const char* m = n > 1 ? std::getenv("AARMVS_REG_MAP") : nullptr;
  if (m && std::strlen(m) == kUnetUnits && m[0] == '0') {
    int top = 0;
    bool ok = true;
    for (int i = 0; i < kUnetUnits; ++i) {
      ok = ok && m[i] >= '0' && m[i] < '0' + kRegMaxStreams;
      top = std::max(top, m[i] - '0');
    }
    if (ok) {
      for (int i = 0; i < kUnetUnits; ++i) us[i] = m[i] - '0';
      return top + 1;
    }
  }
  return n;
}

// planes per cost-stage group: kPlaneGroup, or AARMVS_NPL=n (1 <= n <= kPlaneGroup; A/B runs)
static int plane_group() {
  const char* s = std::getenv("AARMVS_NPL");
  const int n = (s && *s) ? std::atoi(s) : kPlaneGroup;
  return std::max(1, std::min(kPlaneGroup, n));
}

hipError_t aarmvs::library_stream(int dev, int i, hipStream_t& out) {
  static std::mutex mu;
  static hipStream_t pool[kMaxDevices][kLibStreams + 1] = {};
  if (dev < 0 || dev >= kMaxDevices || i < 1 || i > kLibStreams) return hipErrorInvalidValue;
  std::lock_guard<std::mutex> lk(mu);
  if (!pool[dev][i]) {
    hipError_t e = hipStreamCreateWithFlags(&pool[dev][i], hipStreamNonBlocking);
    if (e != hipSuccess) {
      pool[dev][i] = nullptr;
      return e;
    }
  }
  out = pool[dev][i];
  return hipSuccess;
}

extern "C" {

int aarmvs_sweep(const aarmvs_sweep_args* a, hipStream_t stream) {
  if (!a) return fail(AARMVS_ERR_INVALID, "sweep: null args");
  int rc = check_geom(a->B, a->H, a->W, a->nsrc);
  if (rc) return rc;
  if (a->C != kC) return fail(AARMVS_ERR_INVALID, "sweep: feature channels C must be 32");
  if (a->D < 1 || a->d_begin < 0 || a->d_end > a->D || a->d_begin >= a->d_end)
    return fail(AARMVS_ERR_INVALID, "sweep: need 0 <= d_begin < d_end <= D");
  if (!a->ref_fea || !a->rel_proj || !a->depth_values || !a->packed_params || !a->workspace)
    return fail(AARMVS_ERR_INVALID, "sweep: null pointer argument");
  for (int v = 0; v < a->nsrc; ++v)
    if (!a->src_fea[v]) return fail(AARMVS_ERR_INVALID, "sweep: null src_fea pointer");
  const aarmvs_train_record* rec = a->record;
  if (rec && (!rec->x || !rec->state || !rec->z || !rec->u || !rec->stats || !rec->t1 || !rec->ostats))
    return fail(AARMVS_ERR_INVALID, "sweep: training record with a null buffer");
  const TrainLayout T = train_layout(a->B, a->H, a->W);

  SweepGeom g{a->B, a->H, a->W, a->nsrc, a->D, cu_count()};
  Workspace ws = carve_workspace(a->workspace, a->B, a->H, a->W, a->nsrc);
  const float* params = static_cast<const float*>(a->packed_params);
  hipError_t e;
  CostArgs ca{};
  ca.ref = a->ref_fea;
  for (int v = 0; v < a->nsrc; ++v) ca.src[v] = a->src_fea[v];
  ca.rel = a->rel_proj;
  ca.depth_values = a->depth_values;
  ca.params = params;
  // Planes are processed in groups of up to kPlaneGroup (AARMVS_NPL=n for A/B runs).  The
  // cost slices do not depend on the recurrence, so a group's whole cost-slice stage
  // (omega conv, statistics, cost_x: one launch each over the group's planes) runs ahead of
  // its regulariser steps.  Two-stream schedule (a->aux_stream): the cost stage runs on the
  // aux stream, group i's beside group i-1's regulariser steps on the main stream; per
  // group parity two events: ev_cost[p] "group's slices ready" (aux -> main) and
  // ev_used[p] "group's slices consumed" (main -> aux, before group i+2 reuses the slots).
  hipStream_t aux = (a->aux_stream && a->aux_stream != stream) ? a->aux_stream : nullptr;
  // (a training forward, with its record: AARMVS_REG_STREAMS_REC; 3 streams by default too,
  // config-4 training step 251.4 -> 243.3 ms, profiles/r06m_train_streams.txt)
  // under stream capture (a caller recording the sweep into a graph) everything stays on
  // `stream`: the captured graph is the one-stream order, bit-identical to every schedule
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if ((e = hipStreamIsCapturing(stream, &cap)) != hipSuccess) return hip_fail(e, "sweep: capture status");
  if (cap != hipStreamCaptureStatusNone) aux = nullptr;
  const bool small = aux && small_frame((long)a->B * a->H * a->W);
  int ustream[kUnetUnits];
  const int nreg = cap != hipStreamCaptureStatusNone
                       ? reg_unit_streams(1, ustream)
                       : reg_unit_streams(reg_streams(aux != nullptr, rec != nullptr, small), ustream);
  // small frames: the cost stage on the caller's stream, the aux stream one of the units' streams
  hipStream_t unit_aux = nullptr;
  if (small && nreg > 3) {
    unit_aux = aux;
    aux = nullptr;
  }
  const int G = plane_group();
  // ev_cost[2], ev_used[2], fork/join, and the regulariser's part events, fork/join events and
  // streams: a per-thread, per-device set reused across calls (a sweep split into d_range
  // pieces makes one call per piece).  Events are only recorded/waited on the caller's streams and the set's
  // own, and a record overwrites the previous one, so reuse is safe.
  struct EventSet {
    int dev = -1;
    hipEvent_t ev[5 + kUnetUnits * kRegEvRing + kRegMaxStreams] = {};
  };
  static thread_local EventSet evs_dev[kMaxDevices];   // one set per device
  auto sweep_fail = [&](hipError_t err, const char* where) { return hip_fail(err, where); };
  int dev = 0;
  if ((e = current_device(dev)) != hipSuccess) return sweep_fail(e, "sweep: get device");
  EventSet& evs = evs_dev[dev];
  hipEvent_t* ev = evs.ev;
  if ((aux || unit_aux || nreg > 1) && evs.dev != dev) {
    for (hipEvent_t& x : evs.ev)
      if ((e = hipEventCreateWithFlags(&x, hipEventDisableTiming)) != hipSuccess)
        return sweep_fail(e, "sweep: event create");
    evs.dev = dev;
  }
  hipEvent_t* ev_cost = ev;
  hipEvent_t* ev_used = ev + 2;
  hipEvent_t(*ev_part)[kRegEvRing] = reinterpret_cast<hipEvent_t(*)[kRegEvRing]>(ev + 5);
  hipEvent_t* ev_regjoin = ev + 5 + kUnetUnits * kRegEvRing;
  hipStream_t rs[kRegMaxStreams] = {stream};
  for (int i = 1, li = 1; i < nreg; ++i) {
    if (i == 1 && unit_aux) {
      rs[1] = unit_aux;
      continue;
    }
    if ((e = library_stream(dev, li++, rs[i])) != hipSuccess) return sweep_fail(e, "sweep: stream create");
  }
  hipStream_t cs = aux ? aux : stream;   // the cost stage's stream

  if (a->d_begin == 0) {
    // UNetConvLSTM._init_hidden (drmvsnet.py:133-134, 202-206) and the WTA images
    // (drmvsnet.py:302-304)
    if ((e = hipMemsetAsync(ws.state_begin, 0, ws.state_bytes, stream)) != hipSuccess)
      return sweep_fail(e, "sweep: state init");
    if ((e = hipMemsetAsync(ws.max_prob, 0, ws.wta_bytes, stream)) != hipSuccess)
      return sweep_fail(e, "sweep: wta init");
    if ((e = hipMemsetAsync(ws.omega_stats, 0, ws.stats_bytes, stream)) != hipSuccess)
      return sweep_fail(e, "sweep: stats init");
    if (rec && (e = hipMemsetAsync(rec->state, 0, T.state_slab * sizeof(float), stream)) != hipSuccess)
      return sweep_fail(e, "sweep: record state init");
    // c8 copies of the features for the cost stage
    const int HW = a->H * a->W;
    // (each copy also folds 8 max|feature|^2 into ws.xbound: cell 0's fp16 range guard)
    if ((e = launch_to_c8(a->ref_fea, ws.feat8[0], a->B, HW, stream, ws.xbound)) != hipSuccess)
      return sweep_fail(e, "sweep: c8 copy");
    for (int v = 0; v < a->nsrc; ++v)
      if ((e = launch_to_c8(a->src_fea[v], ws.feat8[1 + v], a->B, HW, stream, ws.xbound)) !=
          hipSuccess)
        return sweep_fail(e, "sweep: c8 copy");
  }
  // a record's statistics slabs accumulate from zero (block 0 of cells 3 and 4 fills slot 0 of each)
  if (rec && (e = hipMemsetAsync(rec->stats + (size_t)a->d_begin * T.stats_slab, 0,
                                 (size_t)(a->d_end - a->d_begin) * T.stats_slab * sizeof(double),
                                 stream)) != hipSuccess)
    return sweep_fail(e, "sweep: record stats init");
  if (aux) {   // fork: the aux stream starts after everything enqueued on `stream` so far
    if ((e = hipEventRecord(ev[4], stream)) != hipSuccess ||
        (e = hipStreamWaitEvent(aux, ev[4], 0)) != hipSuccess)
      return sweep_fail(e, "sweep: fork");
  }
  // fork: the regulariser's own streams start after `stream`'s work so far
  for (int i = 1; i < nreg; ++i)
    if ((e = hipEventRecord(ev_regjoin[i], stream)) != hipSuccess ||
        (e = hipStreamWaitEvent(rs[i], ev_regjoin[i], 0)) != hipSuccess)
      return sweep_fail(e, "sweep: fork");
  // every return from here on (errors included) leaves the aux and regulariser streams' work
  // ordered on `stream`
  StreamJoin join{stream, aux, ev[4]};
  StreamJoin join_r[kRegMaxStreams] = {{stream, nullptr, nullptr},
                                       {stream, rs[1], ev_regjoin[1]},
                                       {stream, rs[2], ev_regjoin[2]},
                                       {stream, rs[3], ev_regjoin[3]},
                                       {stream, rs[4], ev_regjoin[4]}};
  // the WTA images are maintained on every plane, whether or not this call returns depth:
  // a sweep split into d_range calls gives the same depth/confidence however its earlier
  // pieces were requested (24 B/px per plane, <0.5% of a plane's time)
  const bool wta = true;
  const int d_last = a->d_end - 1;
  int gi = 0;
  for (int g0 = a->d_begin; g0 < a->d_end; g0 += G, ++gi) {
    const int n = std::min(G, a->d_end - g0);
    // the group's cost slices: two alternating workspace slots, or the record's planes
    float* const xs = rec ? rec->x + (size_t)g0 * T.x_plane : ws.xg[gi & 1];
    // cost stage: its slots were last read by group gi - 2's regulariser steps
    if (aux && gi >= 2 && (e = hipStreamWaitEvent(aux, ev_used[gi & 1], 0)) != hipSuccess)
      return sweep_fail(e, "sweep: event wait");
    // training: the group's omega conv output and statistics go straight to the record (the
    // backward reads them instead of recomputing the omega conv; the record's per-plane layout
    // is the workspace slots')
    Workspace wsg = ws;
    if (rec) {
      wsg.t1 = rec->t1 + (size_t)g0 * ws.t1_plane * 4;
      wsg.omega_stats = rec->ostats + (size_t)g0 * (ws.omega_stats_bytes / 8);
    }
    if ((e = launch_omega_group(ca, g, wsg, g0, n, cs, rec != nullptr)) != hipSuccess)
      return sweep_fail(e, "sweep: omega stage");
    const int ok = d_last < g0 + n ? d_last - g0 : -1;
    if ((e = launch_cost_x_group(ca, g, wsg, g0, n, xs, ok >= 0 ? a->omega_out : nullptr, ok, cs)) !=
        hipSuccess)
      return sweep_fail(e, "sweep: cost slices");
    if (aux && ((e = hipEventRecord(ev_cost[gi & 1], aux)) != hipSuccess ||
                (e = hipStreamWaitEvent(stream, ev_cost[gi & 1], 0)) != hipSuccess))
      return sweep_fail(e, "sweep: event");
    // regulariser steps and WTA of the group's planes
    for (int k = 0; k < n; ++k) {
      const int d = g0 + k;
      const float* xd = xs + (size_t)k * ws.x_plane;
      const UnetIO io = rec ? unet_io_record(T, *rec, d) : unet_io_ws(ws, d);
      if (d == d_last && a->slice_out) {
        e = launch_layout(xd, a->slice_out, a->B, kC, a->H * a->W, false, stream);
        if (e != hipSuccess) return sweep_fail(e, "sweep: slice copy");
      }
      if (nreg > 1) {
        // wait for unit q of plane e on another stream (planes before this call: joined)
        auto wait_unit = [&](int u, int q, int e) -> hipError_t {
          if (e < a->d_begin || ustream[q] == ustream[u]) return hipSuccess;
          return hipStreamWaitEvent(rs[ustream[u]], ev_part[q][e % kRegEvRing], 0);
        };
        UnetIO iom = io;
        iom.clear_stats = false;   // the statistics are stored, never accumulated (one writer each)
        for (int u = 0; u < kUnetUnits; ++u) {
          hipStream_t su = rs[ustream[u]];
          if (u > 0 && (e = wait_unit(u, u - 1, d)) != hipSuccess) return sweep_fail(e, "sweep: event wait");
          // the hidden-state slot this unit overwrites, last read kHRing planes back
          if (u < 4 && (e = wait_unit(u, kHLastReader[u], d - kHRing[u])) != hipSuccess)
            return sweep_fail(e, "sweep: event wait");
          if ((e = launch_unet_step(xd, params, g, ws, iom, su, 1 << u)) != hipSuccess)
            return sweep_fail(e, "sweep: regulariser step");
          if (u == kUnetUnits - 1 &&
              (e = launch_head_wta(params, g, iom, ws, a->depth_values, d, a->cost_out, wta, su)) != hipSuccess)
            return sweep_fail(e, "sweep: head/wta");
          if ((e = hipEventRecord(ev_part[u][d % kRegEvRing], su)) != hipSuccess)
            return sweep_fail(e, "sweep: event record");
        }
        continue;
      }
      if ((e = launch_unet_step(xd, params, g, ws, io, stream)) != hipSuccess)
        return sweep_fail(e, "sweep: regulariser step");
      if ((e = launch_head_wta(params, g, io, ws, a->depth_values, d, a->cost_out, wta,
                               stream)) != hipSuccess)
        return sweep_fail(e, "sweep: head/wta");
    }
    if (aux && (e = hipEventRecord(ev_used[gi & 1], stream)) != hipSuccess)
      return sweep_fail(e, "sweep: event record");
  }
  if (aux) {   // join: everything the call enqueued is ordered on `stream` at return
    join.aux = nullptr;
    if ((e = hipEventRecord(ev[4], aux)) != hipSuccess ||
        (e = hipStreamWaitEvent(stream, ev[4], 0)) != hipSuccess)
      return sweep_fail(e, "sweep: join");
  }
  for (int i = 1; i < nreg; ++i)
    if ((e = join_r[i].join()) != hipSuccess) return sweep_fail(e, "sweep: join");
  if ((a->depth_out || a->conf_out) && a->d_end == a->D) {
    if ((e = launch_finalize(g, ws, a->depth_out, a->conf_out, stream)) != hipSuccess)
      return sweep_fail(e, "sweep: finalize");
  }
  return AARMVS_OK;
}

size_t aarmvs_backward_scratch_bytes(int B, int H, int W, int nsrc) {
  if (check_geom(B, H, W, nsrc) != AARMVS_OK) return 0;
  return bptt_scratch_bytes(B, H, W) + cost_bwd_scratch_bytes(B, H, W, nsrc);
}

int aarmvs_sweep_backward(const aarmvs_backward_args* a, hipStream_t stream) {
  if (!a) return fail(AARMVS_ERR_INVALID, "sweep_backward: null args");
  int rc = check_geom(a->B, a->H, a->W, a->nsrc);
  if (rc) return rc;
  if (a->C != kC) return fail(AARMVS_ERR_INVALID, "sweep_backward: feature channels C must be 32");
  if (a->D < 1 || !a->ref_fea || !a->rel_proj || !a->depth_values || !a->packed_params ||
      !a->record || !a->grad_cost || !a->workspace || !a->scratch)
    return fail(AARMVS_ERR_INVALID, "sweep_backward: null pointer argument or D < 1");
  const aarmvs_train_record* rec = a->record;
  if (!rec->x || !rec->state || !rec->z || !rec->u || !rec->stats || !rec->t1 || !rec->ostats)
    return fail(AARMVS_ERR_INVALID, "sweep_backward: training record with a null buffer");
  for (int v = 0; v < a->nsrc; ++v)
    if (!a->src_fea[v]) return fail(AARMVS_ERR_INVALID, "sweep_backward: null src_fea pointer");
  if (!a->regulariser_only && !a->grad_ref)
    return fail(AARMVS_ERR_INVALID, "sweep_backward: grad_ref is required (the cost-slice part)");
  Workspace ws = carve_workspace(a->workspace, a->B, a->H, a->W, a->nsrc);
  hipError_t e;
  // the c8 feature copies and the fp16 guard bound of the forward, recomputed (the workspace
  // may have served another sweep since)
  const int HW = a->H * a->W;
  if ((e = hipMemsetAsync(ws.xbound, 0, sizeof(unsigned), stream)) != hipSuccess)
    return hip_fail(e, "sweep_backward: bound init");
  if ((e = launch_to_c8(a->ref_fea, ws.feat8[0], a->B, HW, stream, ws.xbound)) != hipSuccess)
    return hip_fail(e, "sweep_backward: c8 copy");
  for (int v = 0; v < a->nsrc; ++v)
    if ((e = launch_to_c8(a->src_fea[v], ws.feat8[1 + v], a->B, HW, stream, ws.xbound)) != hipSuccess)
      return hip_fail(e, "sweep_backward: c8 copy");
  char* scratch = static_cast<char*>(a->scratch);
  const size_t breg = bptt_scratch_bytes(a->B, a->H, a->W);
  CostBwdCtx cctx{};
  cctx.a = a;
  cctx.ws = ws;
  cctx.scratch = scratch + breg;
  cctx.gacc = bptt_gacc(scratch, a->B, a->H, a->W);
  if (!a->regulariser_only && (e = cost_bwd_begin(cctx, stream)) != hipSuccess)
    return hip_fail(e, "sweep_backward: cost-slice init");
  BpttRun r{};
  r.B = a->B;
  r.H = a->H;
  r.W = a->W;
  r.D = a->D;
  r.packed = static_cast<const float*>(a->packed_params);
  r.rec = rec;
  r.grad_cost = a->grad_cost;
  r.xbound = ws.xbound;
  r.scratch = scratch;
  r.grad_x = a->grad_x;
  r.grad_params = a->grad_params;
  r.group_done = a->regulariser_only ? nullptr : cost_bwd_group;
  r.ctx = &cctx;
  if ((e = bptt_regulariser(r, stream)) != hipSuccess) return hip_fail(e, "sweep_backward");
  if (!a->regulariser_only && (e = cost_bwd_end(cctx, stream)) != hipSuccess)
    return hip_fail(e, "sweep_backward: cost-slice gradients");
  return AARMVS_OK;
}

int aarmvs_cost_slice(const float* ref_fea, const float* const* src_fea, const float* rel_proj,
                      const float* depth_d, const void* packed_params, int B, int C, int H, int W,
                      int nsrc, void* workspace, float* slice_out, float* omega_out,
                      hipStream_t stream) {
  int rc = check_geom(B, H, W, nsrc);
  if (rc) return rc;
  if (C != kC) return fail(AARMVS_ERR_INVALID, "cost_slice: feature channels C must be 32");
  if (!ref_fea || !src_fea || !rel_proj || !depth_d || !packed_params || !workspace || !slice_out)
    return fail(AARMVS_ERR_INVALID, "cost_slice: null pointer argument");
  for (int v = 0; v < nsrc; ++v)
    if (!src_fea[v]) return fail(AARMVS_ERR_INVALID, "cost_slice: null src_fea pointer");
  // one plane of the sweep's cost-slice pipeline (D = 1, depth_values = depth_d [B,1])
  SweepGeom g{B, H, W, nsrc, 1, cu_count()};
  Workspace ws = carve_workspace(workspace, B, H, W, nsrc);
  CostArgs ca{};
  ca.ref = ref_fea;
  for (int v = 0; v < nsrc; ++v) ca.src[v] = src_fea[v];
  ca.rel = rel_proj;
  ca.depth_values = depth_d;
  ca.params = static_cast<const float*>(packed_params);
  hipError_t e;
  const int HW = H * W;
  if ((e = hipMemsetAsync(ws.xbound, 0, sizeof(unsigned), stream)) != hipSuccess)
    return hip_fail(e, "cost_slice: bound init");
  if ((e = launch_to_c8(ref_fea, ws.feat8[0], B, HW, stream, ws.xbound)) != hipSuccess)
    return hip_fail(e, "cost_slice: c8 copy");
  for (int v = 0; v < nsrc; ++v)
    if ((e = launch_to_c8(src_fea[v], ws.feat8[1 + v], B, HW, stream, ws.xbound)) != hipSuccess)
      return hip_fail(e, "cost_slice: c8 copy");
  if ((e = launch_omega_group(ca, g, ws, 0, 1, stream)) != hipSuccess)
    return hip_fail(e, "cost_slice: omega stage");
  if ((e = launch_cost_x_group(ca, g, ws, 0, 1, ws.x, omega_out, 0, stream)) != hipSuccess)
    return hip_fail(e, "cost_slice: cost slice");
  if ((e = launch_layout(ws.x, slice_out, B, kC, HW, false, stream)) != hipSuccess)
    return hip_fail(e, "cost_slice: slice copy");
  return AARMVS_OK;
}

int aarmvs_wta_update(const float* cost, const float* depth_d, float* max_prob, float* depth_map,
                      float* exp_sum, int B, int HW, hipStream_t stream) {
  if (!cost || !depth_d || !max_prob || !depth_map || !exp_sum || B < 1 || HW < 1)
    return fail(AARMVS_ERR_INVALID, "wta_update: bad arguments");
  hipError_t e = launch_wta_update(cost, depth_d, max_prob, depth_map, exp_sum, B, HW, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "wta_update");
}

int aarmvs_unet_step(const float* x, int B, int H, int W, int nsrc, int step,
                     const void* packed_params, void* workspace, float* cost_out,
                     hipStream_t stream) {
  int rc = check_geom(B, H, W, nsrc);
  if (rc) return rc;
  if (!x || !packed_params || !workspace || !cost_out || step < 0)
    return fail(AARMVS_ERR_INVALID, "unet_step: null pointer or negative step");
  SweepGeom g{B, H, W, nsrc, 1, cu_count()};
  Workspace ws = carve_workspace(workspace, B, H, W, nsrc);
  const float* params = static_cast<const float*>(packed_params);
  hipError_t e;
  if (step == 0 && (e = hipMemsetAsync(ws.state_begin, 0, ws.state_bytes, stream)) != hipSuccess)
    return hip_fail(e, "unet_step: state init");
  if ((e = hipMemsetAsync(ws.reg_stats, 0, ws.reg_stats_bytes, stream)) != hipSuccess)
    return hip_fail(e, "unet_step: stats reset");
  // the workspace's slice buffer holds x as NHWC, like the sweep's cost slice; max|x| goes
  // to ws.xbound (cell 0's fp16 range guard)
  if ((e = hipMemsetAsync(ws.xbound, 0, sizeof(unsigned), stream)) != hipSuccess)
    return hip_fail(e, "unet_step: bound reset");
  if ((e = launch_layout(x, ws.x, B, kC, H * W, true, stream, ws.xbound)) != hipSuccess)
    return hip_fail(e, "unet_step: x layout");
  const UnetIO io = unet_io_ws(ws, step);
  if ((e = launch_unet_step(ws.x, params, g, ws, io, stream)) != hipSuccess)
    return hip_fail(e, "unet_step");
  // head conv only (no WTA): cost_out is [B,1,H,W] == [B,D=1,H,W] at plane 0
  if ((e = launch_head_wta(params, g, io, ws, nullptr, 0, cost_out, false, stream)) !=
      hipSuccess)
    return hip_fail(e, "unet_step: head");
  return AARMVS_OK;
}

int aarmvs_fusion_filter(const aarmvs_fusion_args* a, hipStream_t stream) {
  if (!a) return fail(AARMVS_ERR_INVALID, "fusion_filter: null args");
  if (a->H < 1 || a->W < 1 || a->nsrc < 1 || a->nsrc > AARMVS_MAX_FUSION_SRC)
    return fail(AARMVS_ERR_INVALID, "fusion_filter: need H, W >= 1 and 1 <= nsrc <= 10");
  if (!a->ref_depth || !a->confidence || !a->cams || !a->photo_mask || !a->geo_mask ||
      !a->final_mask || !a->depth_avg)
    return fail(AARMVS_ERR_INVALID, "fusion_filter: null pointer argument");
  for (int v = 0; v < a->nsrc; ++v)
    if (!a->src_depth[v]) return fail(AARMVS_ERR_INVALID, "fusion_filter: null src_depth pointer");
  hipError_t e = launch_fusion_filter(a, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "fusion_filter");
}

size_t aarmvs_group_norm_scratch_bytes(int B, int C, int HW) {
  return (B < 1 || C < 1 || HW < 1) ? 0 : gn_scratch_bytes(B, C, HW);
}

int aarmvs_group_norm_forward(const float* x, const float* gamma, const float* beta, int B, int C,
                              int HW, int G, float eps, float* y, float* mean_rstd, void* scratch,
                              hipStream_t stream) {
  if (!x || !y || !mean_rstd || !scratch || B < 1 || C < 1 || HW < 1 || G < 1 || C % G != 0 ||
      B > 65535 || C > 65535)
    return fail(AARMVS_ERR_INVALID, "group_norm_forward: bad arguments (need G | C)");
  hipError_t e = launch_group_norm_fwd(x, gamma, beta, B, C, HW, G, eps, y, mean_rstd, scratch, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "group_norm_forward");
}

int aarmvs_group_norm_backward(const float* dy, const float* x, const float* gamma,
                               const float* mean_rstd, int B, int C, int HW, int G, float* dx,
                               float* s1, float* s2, void* scratch, hipStream_t stream) {
  if (!dy || !x || !mean_rstd || !dx || !s1 || !s2 || !scratch || B < 1 || C < 1 || HW < 1 ||
      G < 1 || C % G != 0 || B > 65535 || C > 65535)
    return fail(AARMVS_ERR_INVALID, "group_norm_backward: bad arguments (need G | C)");
  hipError_t e = launch_group_norm_bwd(dy, x, gamma, mean_rstd, B, C, HW, G, dx, s1, s2, scratch, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "group_norm_backward");
}

int aarmvs_lstm_gates_forward(const float* z, const float* c_prev, int B, int hid, int HW, float* h,
                              float* c, hipStream_t stream) {
  if (!z || !c_prev || !h || !c || B < 1 || hid < 1 || HW < 1)
    return fail(AARMVS_ERR_INVALID, "lstm_gates_forward: bad arguments");
  hipError_t e = launch_lstm_gates_fwd(z, c_prev, B, hid, HW, h, c, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "lstm_gates_forward");
}

int aarmvs_lstm_gates_backward(const float* z, const float* c_prev, const float* dh, const float* dc,
                               int B, int hid, int HW, float* dz, float* dc_prev, hipStream_t stream) {
  if (!z || !c_prev || !dz || !dc_prev || B < 1 || hid < 1 || HW < 1)
    return fail(AARMVS_ERR_INVALID, "lstm_gates_backward: bad arguments");
  hipError_t e = launch_lstm_gates_bwd(z, c_prev, dh, dc, B, hid, HW, dz, dc_prev, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "lstm_gates_backward");
}

int aarmvs_softmax_depth(const float* cost, float* prob, int B, int D, int HW, hipStream_t stream) {
  if (!cost || !prob || B < 1 || D < 1 || HW < 1)
    return fail(AARMVS_ERR_INVALID, "softmax_depth: bad arguments");
  hipError_t e = launch_softmax_depth(cost, prob, B, D, HW, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "softmax_depth");
}

int aarmvs_evidential_epilogue(const float* const head[3], const float* depth_values, int D, int HW,
                               float* evidential, float* prob_combine, hipStream_t stream) {
  if (!head || !head[0] || !head[1] || !head[2] || !depth_values || !evidential || !prob_combine ||
      HW < 1)
    return fail(AARMVS_ERR_INVALID, "evidential_epilogue: null pointer or HW < 1");
  if (D != AARMVS_EVIDENTIAL_D)
    return fail(AARMVS_ERR_INVALID, "evidential_epilogue: D must be 32 (the head's maxdisp)");
  hipError_t e = launch_evidential(head, depth_values, D, HW, evidential, prob_combine, nullptr,
                                   nullptr, nullptr, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "evidential_epilogue");
}

int aarmvs_evidential_epilogue_backward(const float* const head[3], const float* depth_values, int D,
                                        int HW, const float* grad_evidential,
                                        const float* grad_prob_combine, float* const grad_head[3],
                                        hipStream_t stream) {
  if (!head || !head[0] || !head[1] || !head[2] || !depth_values || !grad_head || !grad_head[0] ||
      !grad_head[1] || !grad_head[2] || HW < 1)
    return fail(AARMVS_ERR_INVALID, "evidential_epilogue_backward: null pointer or HW < 1");
  if (D != AARMVS_EVIDENTIAL_D)
    return fail(AARMVS_ERR_INVALID, "evidential_epilogue_backward: D must be 32 (the head's maxdisp)");
  hipError_t e = launch_evidential(head, depth_values, D, HW, nullptr, nullptr, grad_evidential,
                                   grad_prob_combine, grad_head, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "evidential_epilogue_backward");
}

static int deform_check(const char* who, const float* x, const float* offset, int B, int C, int H,
                        int W, int h, int w, int stride, int pad) {
  if (!x || !offset) return fail(AARMVS_ERR_INVALID, std::string(who) + ": null pointer");
  if (C != AARMVS_DEFORM_C)
    return fail(AARMVS_ERR_INVALID, std::string(who) + ": C must be 32 (FeatNet's deformable convs)");
  if (B < 1 || H < 1 || W < 1 || h < 1 || w < 1 || stride < 1 || pad < 0)
    return fail(AARMVS_ERR_INVALID, std::string(who) + ": bad geometry");
  return AARMVS_OK;
}

static DfArgs deform_args(const float* x, const float* offset, const float* mask, int B, int H,
                          int W, int h, int w, int stride, int pad) {
  DfArgs a{};
  a.x = x;
  a.off = offset;
  a.m = mask;
  a.B = B;
  a.H = H;
  a.W = W;
  a.h = h;
  a.w = w;
  a.stride = stride;
  a.pad = pad;
  return a;
}

int aarmvs_deform_sample(const float* x_nhwc, const float* offset, const float* mask, int B, int C,
                         int H, int W, int h, int w, int stride, int pad, float* val,
                         hipStream_t stream) {
  if (int rc = deform_check("deform_sample", x_nhwc, offset, B, C, H, W, h, w, stride, pad)) return rc;
  if (!val) return fail(AARMVS_ERR_INVALID, "deform_sample: null pointer");
  DfArgs a = deform_args(x_nhwc, offset, mask, B, H, W, h, w, stride, pad);
  a.val = val;
  hipError_t e = launch_deform_sample(a, false, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "deform_sample");
}

int aarmvs_deform_sample_backward(const float* x_nhwc, const float* offset, const float* mask, int B,
                                  int C, int H, int W, int h, int w, int stride, int pad,
                                  const float* grad_val, float* grad_x_nhwc, float* grad_offset,
                                  float* grad_mask, hipStream_t stream) {
  if (int rc = deform_check("deform_sample_backward", x_nhwc, offset, B, C, H, W, h, w, stride, pad))
    return rc;
  if (!grad_val || !grad_x_nhwc || !grad_offset || (mask && !grad_mask))
    return fail(AARMVS_ERR_INVALID, "deform_sample_backward: null pointer");
  DfArgs a = deform_args(x_nhwc, offset, mask, B, H, W, h, w, stride, pad);
  a.gval = grad_val;
  a.gx = grad_x_nhwc;
  a.goff = grad_offset;
  a.gm = mask ? grad_mask : nullptr;
  hipError_t e = launch_deform_sample(a, true, stream);
  return e == hipSuccess ? AARMVS_OK : hip_fail(e, "deform_sample_backward");
}

}  // extern "C"
