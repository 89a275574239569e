// Internal declarations shared by the HIP translation units of libaarmvs.
// Layouts of the packed parameter buffer and of the sweep workspace live here.
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

#include "../../include/aarmvs.h"

namespace aarmvs {

constexpr int kC = 32;          // feature channels (FeatNet output)
constexpr int kSlots = 32;      // fp64 atomic slots per GroupNorm statistic
constexpr float kGnEps = 1e-5f; // nn.GroupNorm default eps
// The sweep computes cost slices in groups of up to kPlaneGroup planes: one launch of each
// cost-slice kernel covers the group, so the neighbouring planes' bilinear footprints (and
// the reference tile) are fetched from HBM once and re-read from L2.
constexpr int kPlaneGroup = 16;

// ---------------------------------------------------------------------------
// Parameter tensors, in raw-blob order (aarmvs.h).
// ---------------------------------------------------------------------------
enum ParamId : int {
  P_OW0, P_OB0, P_OG0W, P_OG0B, P_OW1, P_OB1, P_OG1W, P_OG1B, P_OW2, P_OB2, P_OG2W, P_OG2B,
  P_OWO, P_OBO,
  P_C0W, P_C0B, P_C1W, P_C1B, P_C2W, P_C2B, P_C3W, P_C3B, P_C4W, P_C4B,
  P_D0W, P_D0B, P_D0GW, P_D0GB, P_D1W, P_D1B, P_D1GW, P_D1GB,
  P_HW, P_HB,
  P_COUNT
};

constexpr int kParamSize[P_COUNT] = {
    4 * 32 * 9, 4, 4, 4, 16, 4, 4, 4, 16, 4, 4, 4, 4, 1,
    64 * 48 * 9, 64, 64 * 32 * 9, 64, 64 * 32 * 9, 64, 64 * 48 * 9, 64, 32 * 40 * 9, 32,
    16 * 16 * 9, 16, 16, 16, 16 * 16 * 9, 16, 16, 16,
    8 * 9, 1};

// LSTM cell geometry (drmvsnet.py:241-244): input x-channels, hidden channels, scale.
constexpr int kCellCX[5] = {32, 16, 16, 32, 32};
constexpr int kCellHid[5] = {16, 16, 16, 16, 8};
constexpr int kCellScale[5] = {1, 2, 4, 2, 1};

// Split-fp16 MFMA operands of a cell's conv weights (see convlstm.hip): input channels
// padded to a multiple of 16 (one 16-channel chunk per k-group), A fragments ordered
// [chunk][tap][m-tile][lane][8 halves], hi then lo.
__host__ __device__ constexpr int cell_cin(int k) { return kCellCX[k] + kCellHid[k]; }
__host__ __device__ constexpr int cell_chunks(int k) { return (cell_cin(k) + 15) / 16; }
__host__ __device__ constexpr int cell_a_halves(int k) {   // per hi / lo
  return cell_chunks(k) * 9 * (kCellHid[k] / 8) * 64 * 8;
}
// BPTT input-gradient conv of cell k: K = 4 hid gate channels (16-channel chunks), M = cin
// rows in 32-row m-tiles; halves per m-tile (hi and lo)
__host__ __device__ constexpr int dg_chunks(int k) { return 4 * kCellHid[k] / 16; }
__host__ __device__ constexpr int dg_mtiles(int k) { return (cell_cin(k) + 31) / 32; }
__host__ __device__ constexpr int dg_mt_halves(int k) { return dg_chunks(k) * 9 * 2 * 64 * 8; }

struct ParamLayout {
  size_t raw_off[P_COUNT];
  size_t pk_off[P_COUNT];   // packed offsets (floats), 64-float aligned
  size_t h3_off[5];         // split-fp16 cell weights (hi then lo halves), in floats; taps with
                            // (tap + chunk) odd negated (the training cells' sign balance)
  size_t h3p_off[5];        // the same, every tap positive (the inference cells)
  size_t h3_scale_off;      // 5 floats: 1 / (power-of-two weight scale) per cell
  size_t ow0t_off;          // omega conv3x3 weights as [tap][ci][co] (1,152 floats)
  size_t owb_scale_off;     // 1 float: 1 / (power-of-two scale of the omega conv fragments)
  size_t owm_off;           // omega conv3x3 off-centre taps as split-fp16 v_mfma_f32_32x32x16_f16
                            // B fragments [chunk][2][64 lanes][8] (omega_mfma; same scale)
  size_t dct_off[2];        // deconv_0/1 weights as [ci][tap][co] (2,304 floats each)
  size_t dcm_off[2];        // deconv_0/1 as split-fp16 v_mfma_f32_32x32x16_f16 A fragments
                            // [6 tap pairs][hi, lo][64 lanes][8 halves], then 1 float: 2^-e
                            // (the fragments carry the power-of-two weight scale 2^e)
  size_t dg_off[5];         // BPTT: each cell's input-gradient conv (the forward conv
                            // transposed: taps flipped, in/out channels swapped) as split-fp16
                            // A fragments [m-tile][chunk][tap][hi, lo][64 lanes][8 halves]
  size_t dg_scale_off;      // 5 floats: 1 / (power-of-two scale) of those fragments
  size_t raw_total;
  size_t pk_total;
};
const ParamLayout& param_layout();

// ---------------------------------------------------------------------------
// Workspace layout.
// ---------------------------------------------------------------------------
// hidden-state ring lengths: h_k of plane e is overwritten by plane e + kHRing[k], so the
// multi-stream regulariser's unit writing h_k may run up to kHRing[k] - 1 planes ahead of the
// last unit that reads it (h0: cell 4, four units on; h1: cell 3; h2: deconv_0; h3: deconv_1)
constexpr int kHRingMax = 6;
constexpr int kHRing[5] = {6, 4, 3, 3, 2};
inline int h_slot(int k, int e) { return e % kHRing[k]; }

struct Workspace {
  double* omega_stats;    // [kPlaneGroup][B][nsrc][3][kSlots][2] omega GN statistics per group plane
  double* omega_part;     // [kPlaneGroup][B][nsrc][omega_part_n][2] per-block GN partial sums
  int omega_part_n;       // partials per (plane, b, view): >= omega tiles, >= statistics blocks
  double* reg_stats;      // [B][2 deconvs][2 groups][kSlots][2] U-Net GN statistics
  double* reg_part;       // [B][deconv_1 blocks][4] deconv_1's per-block GN partials
  double* reg_part0;      // [B][deconv_0 blocks][4] deconv_0's (its own region: the two deconvs
                          // of neighbouring planes may run at once on the regulariser's streams)
  unsigned* xbound;       // float bits of an upper bound on |x| (cost slice) for this sweep:
                          // 8 max|feature|^2 (to_c8) or max|x| (unet_step); cell 0's fp16 range
  float* max_prob;        // [B,HW]
  float* exp_sum;         // [B,HW]
  float* depth;           // [B,HW]
  float* xg[2];           // per group parity: [kPlaneGroup][B][H][W][32] cost slices (NHWC)
  float* x;               // = xg[0]: the single-slice buffer of aarmvs_unet_step / cost_slice
  float* feat8[AARMVS_MAX_SRC + 1]; // [B][4][H][W][8] "c8" copies of ref (0) and source views
  float* t1;              // [kPlaneGroup][B][nsrc][HW][4] omega conv3x3 output per group plane
  float* u0;              // [B,16,H/2,W/2] deconv_0 output (pre-GN)
  float* u1;              // [B,16,H,W]     deconv_1 output (pre-GN)
  float* h[5][kHRingMax]; // hidden states: a ring of kHRing[k] slots (plane d reads slot d % r
                          // and writes slot (d + 1) % r)
  float* c[5];            // cell states (updated in place)
  size_t bytes;
  size_t omega_stats_bytes;  // one plane
  size_t reg_stats_bytes;
  size_t stats_bytes;        // omega + reg statistics and xbound (contiguous, for the initial clear)
  size_t state_bytes;        // h[*][*], c[*] region (contiguous) for zero-init
  void* state_begin;
  size_t wta_bytes;          // max_prob/exp_sum/depth region
  size_t x_plane;            // floats per plane in xg
  size_t t1_plane;           // float4s per plane in t1
};
Workspace carve_workspace(void* base, int B, int H, int W, int nsrc);
// U-Net statistic (deconv j, group g) of batch element b within reg_stats
__host__ __device__ inline size_t reg_stat_index(int b, int j, int g) {
  return ((size_t)(b * 2 + j) * 2 + g) * kSlots * 2;
}

// ---------------------------------------------------------------------------
// Kernel launchers (defined in the .hip units).
// ---------------------------------------------------------------------------
struct SweepGeom {
  int B, H, W, nsrc, D;
  int cu_count;
};

hipError_t launch_pack_params(const float* raw, float* packed, hipStream_t s);
hipError_t launch_homo_warp(const float* src, const float* rel, const float* depth, int B, int C,
                            int H, int W, float* out, hipStream_t s);
size_t homo_warp_bwd_workspace_bytes(int B, int C, int H, int W);
hipError_t launch_homo_warp_bwd(const float* gout, const float* rel, const float* depth, int B, int C, int H,
                                int W, float* gsrc, void* workspace, hipStream_t s);

struct CostArgs {
  const float* ref;
  const float* src[AARMVS_MAX_SRC];
  const float* rel;       // [nsrc][B][12]
  const float* depth_values;  // [B,D]
  const float* params;    // packed
};
// The cost-slice stage (warp_cost.hip) for the planes d0 .. d0 + n - 1 (n <= kPlaneGroup):
// omega_group clears the group's statistics, then writes t1 and the three GroupNorm
// statistics of every plane (omega conv + omega_stats<1> + <2>); cost_x_group then writes
// each plane's cost slice to x0 + k ws.x_plane (and, for plane omega_k, the omega weights
// to omega_out).  Both use the t1 / statistics slots of the workspace: one group at a time.
// NCHW <-> NHWC copy of a [B][C][HW] / [B][HW][C] fp32 tensor (API edges only)
// depth-map fusion core (fusion.hip)
hipError_t launch_fusion_filter(const aarmvs_fusion_args* a, hipStream_t s);
// xmax (optional, to_nhwc only): atomic max of |in| as float bits
hipError_t launch_layout(const float* in, float* out, int B, int C, int HW, bool to_nhwc,
                         hipStream_t s, unsigned* xmax = nullptr);
// xbound (optional): atomic max of 8 max|src|^2 as float bits, an upper bound on the cost
// slice's |x| (|warp - ref| <= 2 max|feature|, (1 + w) <= 2)
hipError_t launch_to_c8(const float* src, float* dst, int B, int HW, hipStream_t s,
                        unsigned* xbound = nullptr);
hipError_t launch_omega_group(const CostArgs& a, const SweepGeom& g, const Workspace& ws, int d0,
                              int n, hipStream_t s,
                              bool balanced = false);
hipError_t launch_cost_x_group(const CostArgs& a, const SweepGeom& g, const Workspace& ws, int d0,
                               int n, float* x0, float* omega_out, int omega_k, hipStream_t s);

// Where one regulariser step reads and writes its tensors (all NHWC): the eval sweep's
// workspace ping-pong (c updated in place) or a training record's per-plane slabs
// (unet_io_ws / unet_io_record).
struct UnetIO {
  const float* h_prev[5];
  float* h_new[5];
  const float* c_prev[5];
  float* c_new[5];
  float* z[5];          // gate pre-activations [B][Hk][Wk][4 hid], or null (eval)
  float* u0;            // deconv_0 output [B][H/2][W/2][16] (pre-GN)
  float* u1;            // deconv_1 output [B][H][W][16]
  double* reg_stats;    // the two deconvs' GroupNorm statistics (reg_stat_index layout)
  bool clear_stats;     // the head kernel zeroes reg_stats after use (eval: one shared set)
};

// Training record (aarmvs_train_record, include/aarmvs.h): per-plane slabs, in floats
// (stats in doubles).  A state slab holds h then c of every cell; slab 0 is the zero initial
// state (drmvsnet.py:133-134), slab d + 1 the state after plane d.
struct TrainLayout {
  size_t x_plane;
  size_t state_slab, h_off[5], c_off[5];
  size_t z_slab, z_off[5];
  size_t u_slab, u0_off, u1_off;
  size_t stats_slab;   // doubles
  size_t cell_px[5];   // B * pixels of cell k
};
TrainLayout train_layout(int B, int H, int W);
UnetIO unet_io_ws(const Workspace& ws, int d);   // plane d (absolute index in the sweep)
UnetIO unet_io_record(const TrainLayout& T, const aarmvs_train_record& r, int d);

// stages: the step's five units (bit u = unit u, run in that order: cell 0 | cell 1 | cell 2 |
// deconv_0 + cell 3 | deconv_1 + cell 4); a unit of plane d reads only the earlier units'
// outputs of plane d and its own state, so the units of neighbouring planes may run at once on
// different streams (the sweep's multi-stream regulariser)
constexpr int kUnetUnits = 5, kUnetAll = (1 << kUnetUnits) - 1;
hipError_t launch_unet_step(const float* x, const float* params, const SweepGeom& g,
                            const Workspace& ws, const UnetIO& io, hipStream_t s,
                            int stages = kUnetAll);
hipError_t launch_head_wta(const float* params, const SweepGeom& g, const UnetIO& io,
                           const Workspace& ws, const float* depth_values, int d,
                           float* cost_out, bool wta, hipStream_t s);
hipError_t launch_wta_update(const float* cost, const float* depth_d, float* max_prob,
                             float* depth, float* exp_sum, int B, int HW, hipStream_t s);
hipError_t launch_finalize(const SweepGeom& g, const Workspace& ws, float* depth_out,
                           float* conf_out, hipStream_t s);
hipError_t launch_softmax_depth(const float* cost, float* prob, int B, int D, int HW,
                                hipStream_t s);
// the evidential head's epilogue (evidential.hip): forward when g_head is null (ev [4][HW],
// pc [D][HW]), else the backward from g_ev / g_pc (either may be null) into g_head
hipError_t launch_evidential(const float* const head[3], const float* dv, int D, int HW, float* ev,
                             float* pc, const float* g_ev, const float* g_pc, float* const g_head[3],
                             hipStream_t s);
// the sampling half of FeatNet's deformable conv (deform.hip): val from x (forward), or dL/dx,
// dL/d offset, dL/d m from dL/d val (backward)
struct DfArgs {
  const float* x;        // [B][H][W][C]
  const float* off;      // [B][18][h][w]
  const float* m;        // [B][9][h][w] or null (no modulation)
  int B, H, W, h, w, stride, pad;
  float* val;            // [B][h w][9][C]
  const float* gval;     // backward: dL/d val
  float* gx;             // backward: dL/d x, NHWC, accumulated
  float* goff;           // backward: dL/d offset
  float* gm;             // backward: dL/d m (null if m is null)
};
hipError_t launch_deform_sample(const DfArgs& a, bool bwd, hipStream_t s);
// GroupNorm of NCHW [B][C][HW] fp32 (group_norm.hip): mean_rstd [B][G][2]; gamma / beta may
// be null (1 / 0); scratch of gn_scratch_bytes(B, C, HW); bwd also writes s1 = sum dy xhat and
// s2 = sum dy per (b, c) (the per-sample dgamma / dbeta terms)
size_t gn_scratch_bytes(int B, int C, int HW);
hipError_t launch_group_norm_fwd(const float* x, const float* gamma, const float* beta, int B,
                                 int C, int HW, int G, float eps, float* y, float* mean_rstd,
                                 void* scratch, hipStream_t s);
// ConvLSTMCell gate math (lstm_train.hip): z [B][4 hid][HW] -> h, c [B][hid][HW]; backward
// from dh, dc (either may be null: zero) to dz and dc_prev
hipError_t launch_lstm_gates_fwd(const float* z, const float* c_prev, int B, int hid, int HW,
                                 float* h, float* c, hipStream_t s);
hipError_t launch_lstm_gates_bwd(const float* z, const float* c_prev, const float* dh,
                                 const float* dc, int B, int hid, int HW, float* dz, float* dc_prev,
                                 hipStream_t s);
hipError_t launch_group_norm_bwd(const float* dy, const float* x, const float* gamma,
                                 const float* mean_rstd, int B, int C, int HW, int G, float* dx,
                                 float* s1, float* s2, void* scratch, hipStream_t s);

int cu_count();

// Per-device host state (func attributes, aux streams and events) is kept in arrays indexed by
// the current device, so that one process driving several devices (nn.DataParallel) gets each
// device its own.
constexpr int kMaxDevices = 64;
inline hipError_t current_device(int& dev) {
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess && (dev < 0 || dev >= kMaxDevices)) e = hipErrorInvalidDevice;
  return e;
}
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per device for a kernel
inline hipError_t ensure_dyn_lds(const void* fn, int bytes, bool (&done)[kMaxDevices]) {
  int dev = 0;
  hipError_t e = current_device(dev);
  if (e != hipSuccess || done[dev]) return e;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done[dev] = true;
  return e;
}
// The library's own streams (i = 1 .. kLibStreams), created on first use per device and shared
// by every call of the process, from any host thread (sweeps: the regulariser's unit streams;
// backward: the plane pipeline's and the group stage's).  A process gets GPU_MAX_HW_QUEUES = 4
// hardware queues here and every stream it creates holds one, so streams beyond four share a
// queue, where one stream's event wait stalls the other's work: the library keeps the process's
// total (the caller's stream and aux stream included) at four.  Calls on different host threads
// that share a stream are only ordered, never mixed: each call's events are its thread's own.
constexpr int kLibStreams = 4;   // 1-3: unit / backward streams; 4: aarmvs_aux_stream
hipError_t library_stream(int dev, int i, hipStream_t& out);
// Joins an auxiliary stream back into the caller's stream when it goes out of scope: on every
// return after a fork (errors included), nothing the call enqueued on the aux stream is left
// unordered with the caller's stream, whose buffers the caller may free on an error.
struct StreamJoin {
  hipStream_t main, aux;
  hipEvent_t ev;
  hipError_t join() {   // order the aux stream's work so far on main (once)
    hipError_t e = hipSuccess;
    if (aux && aux != main && ev) {
      e = hipEventRecord(ev, aux);
      if (e == hipSuccess) e = hipStreamWaitEvent(main, ev, 0);
    }
    aux = nullptr;
    return e;
  }
  ~StreamJoin() { (void)join(); }
};

// Backward of the regulariser (bptt.hip) over every plane of a training record: the
// parameter gradients of the cells / deconvs / head into the fp64 accumulators of its scratch
// (written to grad_params as float at the end, the cost-slice part included if group_done
// adds to them), and per group of planes dL/dx handed to group_done (planes g0 .. g0 + n - 1,
// gx [n][B][H][W][32]) and copied to grad_x if set.
struct BpttRun {
  int B, H, W, D;
  const float* packed;
  const aarmvs_train_record* rec;
  const float* grad_cost;      // [B][D][H][W]
  const unsigned* xbound;      // float bits of a bound on |x| (the forward's fp16 guard bound)
  void* scratch;               // bptt_scratch_bytes
  float* grad_x;               // optional [D][B][H][W][32]
  float* grad_params;          // optional [raw count]
  hipError_t (*group_done)(void* ctx, int g0, int n, const float* gx, hipStream_t s);
  void* ctx;
};
size_t bptt_scratch_bytes(int B, int H, int W);
hipError_t bptt_regulariser(const BpttRun& r, hipStream_t s);
// the fp64 parameter-gradient accumulators inside a bptt scratch buffer
double* bptt_gacc(void* scratch, int B, int H, int W);

// Backward of the cost-slice stage (cost_bwd.hip): per group of planes, from dL/dx to the
// omega.* parameter gradients (into gacc) and dL/d features (accumulated, written out by
// cost_bwd_end).
struct CostBwdCtx {
  const aarmvs_backward_args* a;
  Workspace ws;
  void* scratch;      // cost_bwd_scratch_bytes
  double* gacc;       // the regulariser's fp64 accumulators (raw layout)
};
size_t cost_bwd_scratch_bytes(int B, int H, int W, int nsrc);
hipError_t cost_bwd_begin(CostBwdCtx& c, hipStream_t s);
hipError_t cost_bwd_group(void* ctx, int g0, int n, const float* gx, hipStream_t s);
hipError_t cost_bwd_end(CostBwdCtx& c, hipStream_t s);

// ---------------------------------------------------------------------------
// Opt-in per-kernel timing (aarmvs_profile_*): hipEvents recorded on the launch
// stream around each kernel.  Off by default; costs nothing when off.
// ---------------------------------------------------------------------------
enum KernelId : int {
  K_COST_X, K_OMEGA_CONV, K_FUSION, K_OMEGA1, K_OMEGA2,
  K_CELL0, K_CELL1, K_CELL2, K_CELL3, K_CELL4,
  K_DECONV0, K_DECONV1, K_HEAD_WTA, K_FINALIZE, K_SOFTMAX, K_WARP, K_TO_C8, K_STAT_REDUCE,
  K_GN_REDUCE, K_EVIDENTIAL,
  // the training backward (bptt.hip, the cbw_* kernels of warp_cost.hip)
  K_GATE_BWD0, K_GATE_BWD1, K_GATE_BWD2, K_GATE_BWD3, K_GATE_BWD4,
  K_DGRAD0, K_DGRAD1, K_DGRAD2, K_DGRAD3, K_DGRAD4,
  K_WGRAD0, K_WGRAD1, K_WGRAD2, K_WGRAD3, K_WGRAD4,
  K_GNB_PARTIAL, K_DECONV_BWD, K_BWD_SMALL, K_CBW_CHAIN, K_CBW_FEAT, K_CBW_SMALL,
  K_DECONV_WGRAD, K_HEAD_WGRAD, K_DEFORM,
  K_COUNT
};
extern bool g_prof_on;
void prof_mark(hipStream_t s, int id, bool begin);
struct ProfScope {
  hipStream_t s;
  int id;
  ProfScope(hipStream_t s_, int id_) : s(s_), id(id_) {
    if (g_prof_on) prof_mark(s, id, true);
  }
  ~ProfScope() {
    if (g_prof_on) prof_mark(s, id, false);
  }
};

}  // namespace aarmvs
