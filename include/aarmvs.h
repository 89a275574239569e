/*
 * aarmvs.h — C ABI of the MI355X (gfx950) depth-sweep library (libaarmvs.so).
 *
 * This is the drop-in boundary beneath the reference's Python API
 * (BuTTerK3ks/AA-RMVSNet, models/drmvsnet.py).  The reference has no native
 * layer: every entry point below replaces a block of PyTorch ops inside
 * EMVSNet.forward's depth loop (models/drmvsnet.py:255-345).  The Python mirror
 * in aa-rmvsnet_amd/models binds these with ctypes.
 *
 * Conventions
 *   - All tensors are fp32, contiguous, NCHW, resident in device memory and owned
 *     by the caller; the library never allocates device memory and keeps no
 *     pointer across calls.
 *   - Every launch goes to the caller's stream; no host synchronisation happens
 *     inside any entry point (graph-capturable).
 *   - Return 0 on success, a nonzero aarmvs_status otherwise; the message is in
 *     aarmvs_last_error() (thread-local).  Shapes are validated before launch.
 *   - Constraints (from the reference's own shape rules): C == 32 feature
 *     channels, H % 4 == 0 and W % 4 == 0 (two 2x2 max-pools and two stride-2
 *     deconvs must round-trip, drmvsnet.py:148-161), 1 <= nsrc <= AARMVS_MAX_SRC.
 */
#ifndef AARMVS_H_
#define AARMVS_H_

#include <stddef.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AARMVS_MAX_SRC 16
#define AARMVS_FEAT_C 32

typedef enum aarmvs_status {
  AARMVS_OK = 0,
  AARMVS_ERR_INVALID = 1,   /* bad shape / null pointer / unsupported argument */
  AARMVS_ERR_HIP = 2        /* a HIP runtime call or kernel launch failed     */
} aarmvs_status;

const char* aarmvs_last_error(void);
const char* aarmvs_version(void);

/* ---------------------------------------------------------------------------
 * Parameters.
 * The raw blob is the sweep's checkpoint tensors (the 48 omega.* and
 * cost_regularization.* keys of the reference state_dict, drmvsnet.py:66-117 and
 * :27-38) flattened and concatenated in this order:
 *   omega.reweight_network.0.0.weight [4,32,3,3], .0.0.bias [4], .0.1.weight [4],
 *   .0.1.bias [4], .1.stem.0.0.weight [4,4,1,1], .1.stem.0.0.bias [4],
 *   .1.stem.0.1.weight [4], .1.stem.0.1.bias [4], .1.stem.1.weight [4,4,1,1],
 *   .1.stem.1.bias [4], .1.stem.2.weight [4], .1.stem.2.bias [4],
 *   .2.weight [1,4,1,1], .2.bias [1],
 *   cost_regularization.cell_list.{0..4}.conv.{weight,bias}
 *     ([64,48,3,3],[64],[64,32,3,3],[64],[64,32,3,3],[64],[64,48,3,3],[64],[32,40,3,3],[32]),
 *   cost_regularization.deconv_{0,1}.{conv.weight [16,16,3,3], conv.bias [16],
 *     gn.weight [16], gn.bias [16]},
 *   cost_regularization.conv_0.weight [1,8,3,3], cost_regularization.conv_0.bias [1].
 * aarmvs_pack_params rearranges it (on the device) into the kernels' layout.
 * ------------------------------------------------------------------------- */
size_t aarmvs_param_count(void);            /* floats in the raw blob            */
size_t aarmvs_packed_param_bytes(void);     /* bytes of the packed device buffer */
int aarmvs_pack_params(const float* raw_params, void* packed, hipStream_t stream);

/* ---------------------------------------------------------------------------
 * homo_warping_depthwise (models/module.py:6-38): bilinear warp of src_fea
 * [B,C,H,W] into the reference view at one depth per batch element.
 * rel_proj [B,12] = rows 0..2 of src_proj @ inverse(ref_proj) (module.py:16-18),
 * depth [B].  grid_sample semantics: bilinear, zero padding, align_corners=False
 * applied to the align_corners=True-normalised grid.
 * ------------------------------------------------------------------------- */
int aarmvs_homo_warp(const float* src_fea, const float* rel_proj, const float* depth,
                     int B, int C, int H, int W, float* out, hipStream_t stream);

/* Backward of aarmvs_homo_warp w.r.t. src_fea (the grid carries no gradient,
 * module.py:15; grid_sample's backward at module.py:36): grad_src += bilinear
 * scatter of grad_out.  grad_src must be initialised by the caller (zeros for the
 * plain gradient).  The scatter sums are formed in 64-bit fixed point (exponent from
 * max |grad_out|), so the result is bit-reproducible whatever the order the GPU
 * serves the contributions in; a batch element whose grad_out holds a NaN or an
 * infinity is scattered with fp32 atomics instead (the NaN/inf reaches the source
 * pixels grid_sample's backward sends it to, the others stay finite).  Batch
 * elements are processed 64 at a time.  workspace:
 * aarmvs_homo_warp_backward_workspace_bytes = 256 + min(B,64)*C*H*W*8 bytes
 * (caller-owned, device memory). */
size_t aarmvs_homo_warp_backward_workspace_bytes(int B, int C, int H, int W);
int aarmvs_homo_warp_backward(const float* grad_out, const float* rel_proj, const float* depth,
                              int B, int C, int H, int W, float* grad_src, void* workspace,
                              hipStream_t stream);

/* ---------------------------------------------------------------------------
 * Whole depth sweep (drmvsnet.py:273-291 train / :306-342 eval).
 * Replaces, per plane d: homo_warping_depthwise x nsrc, (warp-ref)^2, omega
 * re-weighting, weighted accumulation, UNetConvLSTM.forward and the online WTA.
 * ------------------------------------------------------------------------- */
/* Training record of a sweep (the BPTT's saved tensors; see aarmvs_sweep_backward):
 * when aarmvs_sweep_args.record is set, the sweep keeps every plane's regulariser
 * tensors in these caller-owned device buffers instead of overwriting its workspace copies.
 * Per-plane slab sizes in bytes: aarmvs_train_record_bytes(B, H, W, which) with which =
 *   0 x      [B,H,W,32] cost slice of the plane (NHWC);                 D slabs
 *   1 state  h, c of the five cells (NHWC); slab 0 is the zero initial state
 *            (drmvsnet.py:133-134), slab d+1 the state after plane d;  D+1 slabs
 *   2 z      the five cells' gate pre-activations (conv + bias), per cell planar
 *            [B][hid/4 channel quads][gates i,f,o,g][H*W][4];           D slabs
 *   3 u      the two deconvs' outputs before GroupNorm;                  D slabs
 *   4 stats  the two deconvs' GroupNorm statistics (fp64);               D slabs
 *   5 t1     the omega conv output (4 ch) of ONE source view;        D x nsrc slabs
 *   6 ostats the omega chain's GroupNorm statistics of ONE view (fp64); D x nsrc slabs
 *   (5 and 6 let the backward skip recomputing the omega conv of every plane)
 * ~1 KB per pixel and plane at B = 1 (63 GB for 640x512, D = 192). */
typedef struct aarmvs_train_record {
  float* x;
  float* state;
  float* z;
  float* u;
  double* stats;
  float* t1;
  double* ostats;
} aarmvs_train_record;
size_t aarmvs_train_record_bytes(int B, int H, int W, int which);

typedef struct aarmvs_sweep_args {
  int B, C, H, W;                         /* C must be 32                         */
  int nsrc;                               /* N-1 source views                     */
  int D;                                  /* depth hypotheses (depth_values.shape[1]) */
  int d_begin, d_end;                     /* plane range; d_begin == 0 resets state */
  const float* ref_fea;                   /* [B,C,H,W]                             */
  const float* src_fea[AARMVS_MAX_SRC];   /* nsrc x [B,C,H,W]                      */
  const float* rel_proj;                  /* [nsrc][B][12]                         */
  const float* depth_values;              /* [B,D]                                 */
  const void* packed_params;              /* from aarmvs_pack_params               */
  void* workspace;                        /* aarmvs_sweep_workspace_bytes() bytes  */
  float* depth_out;                       /* [B,H,W] WTA depth, or NULL            */
  float* conf_out;                        /* [B,H,W] max_prob / exp_sum, or NULL   */
  float* cost_out;                        /* [B,D,H,W] regulariser output, or NULL */
  float* slice_out;                       /* debug: [B,32,H,W] last plane's cost slice, or NULL */
  float* omega_out;                       /* debug: [nsrc,B,H,W] last plane's omega weights, or NULL */
  hipStream_t aux_stream;                 /* optional second stream, or NULL: the cost slices
                                             are computed in groups of up to 16 planes, and
                                             the next group's (omega conv, GroupNorm
                                             statistics, cost_x) run on it beside the current
                                             group's regulariser steps (events per group); a
                                             sweep with it also spreads each plane's U-Net
                                             step (five units: cell 0 | cell 1 | cell 2 |
                                             deconv_0, cell 3 | deconv_1, cell 4, head) over
                                             `stream` and library-owned streams, so that the
                                             units of neighbouring planes run at once (events
                                             per unit and plane; at most four streams in all,
                                             and for small frames, B*H*W <= 65536, the cost
                                             stage moves to `stream` so that the units get
                                             four).  At return all work is ordered on
                                             `stream`; results are bit-identical either way */
  const aarmvs_train_record* record;      /* training record, or NULL (eval): the cost
                                             slices and regulariser tensors of the planes
                                             d_begin..d_end-1 go to its slabs           */
} aarmvs_sweep_args;

size_t aarmvs_sweep_workspace_bytes(int B, int H, int W, int nsrc);
int aarmvs_sweep(const aarmvs_sweep_args* args, hipStream_t stream);
/* A stream for aux_stream owned by the library (one per device, created on first use, never
 * destroyed): a process gets four hardware queues and streams beyond four share them, so a
 * caller without streams of its own passes this one rather than creating a fifth (the library's
 * other streams are its two to three unit / backward streams).  *out: the current device's. */
int aarmvs_aux_stream(hipStream_t* out);

/* ---------------------------------------------------------------------------
 * Backward of a training sweep (the BPTT through drmvsnet.py:273-291): given the record
 * of a forward over all D planes (aarmvs_sweep with `record`, d_begin = 0, d_end = D) and
 * dL/dcost [B,D,H,W] (the sweep's cost volume, before the softmax), the gradients w.r.t.
 * the sweep's parameters (raw-blob layout, aarmvs_param_count() floats: the omega.* and
 * cost_regularization.* tensors), the reference features and the source features.
 * Replaces autograd through homo_warping_depthwise, the omega network, the weighted
 * accumulation and UNetConvLSTM.forward (module.py:6-38, 76-92, 252-287; drmvsnet.py:27-38,
 * 119-167); no gradient flows to the projections or depths (module.py:15).
 * Planes are processed last to first in groups of 16.  Parameter gradients are fixed-order
 * fp64 sums (deterministic); grad_ref / grad_src are overwritten (NCHW [B,32,H,W]).
 * grad_x (debug, or NULL): [D][B][H][W][32] dL/dx per plane (the cost slices, NHWC).
 * regulariser_only (debug): skip the cost-slice part (grad_ref / grad_src untouched, the
 * omega.* entries of grad_params zero).  `workspace` is the sweep workspace
 * (aarmvs_sweep_workspace_bytes), `scratch` aarmvs_backward_scratch_bytes bytes.
 * ------------------------------------------------------------------------- */
typedef struct aarmvs_backward_args {
  int B, C, H, W, nsrc, D;
  const float* ref_fea;                   /* [B,C,H,W]                          */
  const float* src_fea[AARMVS_MAX_SRC];   /* nsrc x [B,C,H,W]                   */
  const float* rel_proj;                  /* [nsrc][B][12]                      */
  const float* depth_values;              /* [B,D]                              */
  const void* packed_params;
  const aarmvs_train_record* record;
  const float* grad_cost;                 /* [B,D,H,W]                          */
  float* grad_ref;                        /* [B,C,H,W] out, or NULL             */
  float* grad_src[AARMVS_MAX_SRC];        /* nsrc x [B,C,H,W] out, or NULL      */
  float* grad_params;                     /* [aarmvs_param_count()] out, or NULL */
  float* grad_x;                          /* debug out, or NULL                 */
  void* workspace;
  void* scratch;
  int regulariser_only;
} aarmvs_backward_args;
size_t aarmvs_backward_scratch_bytes(int B, int H, int W, int nsrc);
int aarmvs_sweep_backward(const aarmvs_backward_args* args, hipStream_t stream);

/* Hidden state of the regulariser inside the workspace, for inspection/BPTT:
 * cell k in 0..4, which = 0 for h, 1 for c, planes = the number of planes (or
 * aarmvs_unet_step steps) processed so far: the state they left (h lives in a ring of
 * 3 slots for cell 0 and 2 for the others, indexed by plane).  Valid after an
 * aarmvs_sweep call; returns a device pointer to [B,H_k,W_k,hid_k] (NHWC: the workspace
 * keeps the U-Net tensors channel-innermost) or NULL. */
float* aarmvs_state_ptr(void* workspace, int B, int H, int W, int nsrc, int planes,
                        int cell, int which);

/* ---------------------------------------------------------------------------
 * One UNetConvLSTM step (drmvsnet.py:119-167) on a given cost slice x [B,32,H,W]
 * using the hidden state held in `workspace` (same layout as aarmvs_sweep).
 * step == 0 zero-initialises the state (drmvsnet.py:133-134).  cost_out [B,1,H,W].
 * ------------------------------------------------------------------------- */
int aarmvs_unet_step(const float* x, int B, int H, int W, int nsrc, int step,
                     const void* packed_params, void* workspace, float* cost_out,
                     hipStream_t stream);

/* ---------------------------------------------------------------------------
 * One plane's cost slice (SURVEY §8b aarmvs_cost_slice): replaces, for one depth
 * hypothesis per batch element, drmvsnet.py:307-319 -- homo_warping_depthwise x nsrc
 * (module.py:6-38), (warp - ref)^2, InterViewAAModule (drmvsnet.py:27-38) and the
 * weighted accumulation -- giving x = -(sum_v (1 + w_v) sq_v) / nsrc.
 * src_fea is a HOST array of nsrc device pointers [B,C,H,W]; rel_proj [nsrc][B][12]
 * (as for aarmvs_sweep); depth_d [B].  slice_out [B,32,H,W]; omega_out [nsrc,B,H,W]
 * (the omega weights w_v) or NULL.  `workspace` is an aarmvs_sweep_workspace_bytes
 * buffer used as scratch: a sweep in progress in the same workspace is invalidated.
 * ------------------------------------------------------------------------- */
int aarmvs_cost_slice(const float* ref_fea, const float* const* src_fea, const float* rel_proj,
                      const float* depth_d, const void* packed_params, int B, int C, int H, int W,
                      int nsrc, void* workspace, float* slice_out, float* omega_out,
                      hipStream_t stream);

/* Online winner-take-all update of one plane (SURVEY §8b aarmvs_wta_update;
 * drmvsnet.py:324-334): p = exp(cost) without max-subtraction, flag = max_prob < p
 * (strict: the first plane wins ties), max_prob/depth_map updated by the reference's
 * arithmetic select, exp_sum += p.  cost, max_prob, depth_map, exp_sum [B,HW];
 * depth_d [B].  Start from max_prob = depth_map = exp_sum = 0 (drmvsnet.py:301-304);
 * the confidence is max_prob / exp_sum after the last plane (:339). */
int aarmvs_wta_update(const float* cost, const float* depth_d, float* max_prob, float* depth_map,
                      float* exp_sum, int B, int HW, hipStream_t stream);

/* softmax over the depth axis of cost [B,D,H,W] (drmvsnet.py:291/:342). */
int aarmvs_softmax_depth(const float* cost, float* prob, int B, int D, int HW,
                         hipStream_t stream);

/* GroupNorm (nn.GroupNorm, module.py:98-103, 245-287; FeatNet and the BPTT recompute of
 * the omega chain and the U-Net deconvs) on NCHW fp32 x [B,C,HW] with G groups (G | C).
 * gamma / beta [C] may be NULL (weight 1, bias 0).  mean_rstd: [B,G,2] out (forward) / in
 * (backward).  scratch: aarmvs_group_norm_scratch_bytes(B,C,HW) bytes of device memory.
 * Backward writes dx [B,C,HW] and, per (b,c), s1 = sum_hw dy*xhat and s2 = sum_hw dy
 * (dgamma = sum_b s1, dbeta = sum_b s2).  Statistics are fixed-order fp64 reductions. */
/* ConvLSTMCell gate math (module.py:76-92) for the BPTT recompute: from the conv output z
 * [B,4*hid,HW] (gates i, f, o, g in channel blocks) and c_prev [B,hid,HW] to h, c
 * [B,hid,HW]; backward from dh, dc (either may be NULL: zero) to dz [B,4*hid,HW] and
 * dc_prev [B,hid,HW], recomputing the gates from z. */
int aarmvs_lstm_gates_forward(const float* z, const float* c_prev, int B, int hid, int HW, float* h,
                              float* c, hipStream_t stream);
int aarmvs_lstm_gates_backward(const float* z, const float* c_prev, const float* dh, const float* dc,
                               int B, int hid, int HW, float* dz, float* dc_prev, hipStream_t stream);

size_t aarmvs_group_norm_scratch_bytes(int B, int C, int HW);
int aarmvs_group_norm_forward(const float* x, const float* gamma, const float* beta, int B, int C,
                              int HW, int G, float eps, float* y, float* mean_rstd, void* scratch,
                              hipStream_t stream);
int aarmvs_group_norm_backward(const float* dy, const float* x, const float* gamma,
                               const float* mean_rstd, int B, int C, int HW, int G, float* dx,
                               float* s1, float* s2, void* scratch, hipStream_t stream);

/* ---------------------------------------------------------------------------
 * Depth-map fusion core of one reference view (fusion.py:71-220, the per-view part of
 * filter_depth after file I/O): for every reference pixel the geometric consistency
 * against each source view's depth map (reproject_with_depth, check_geometric_consistency)
 * and filter_depth's photometric mask, per-threshold votes, geometric mask and averaged
 * depth.  Depth maps and confidence are device [H,W] float32 (all views the same size);
 * `cams` is HOST memory, AARMVS_FUSION_CAM_FLOATS(nsrc) float32 values as numpy forms
 * them in the reference (float32 inverses and products): inv(K_ref) 3x3, K_ref 3x3, then
 * per source view K 3x3, inv(K) 3x3, (E_src inv(E_ref))[:3] 3x4, (E_ref inv(E_src))[:3]
 * 3x4, row-major (aarmvs/fusion.py packs them).  Outputs (device): three [H,W] uint8
 * masks (photo, geo, final) and the [H,W] float64 averaged depth.  1 <= nsrc <=
 * AARMVS_MAX_FUSION_SRC (the reference indexes its mask list up to 10 source views).
 * ------------------------------------------------------------------------- */
#define AARMVS_MAX_FUSION_SRC 10
#define AARMVS_FUSION_CAM_FLOATS(nsrc) (18 + 42 * (nsrc))
typedef struct aarmvs_fusion_args {
  int H, W, nsrc;
  const float* ref_depth;                          /* [H,W]                 */
  const float* confidence;                         /* [H,W]                 */
  const float* src_depth[AARMVS_MAX_FUSION_SRC];   /* nsrc x [H,W]          */
  const float* cams;                               /* host, see above       */
  float photo_threshold;                           /* 0.35 DTU, 0.2 T&T     */
  unsigned char* photo_mask;                       /* [H,W] out             */
  unsigned char* geo_mask;                         /* [H,W] out             */
  unsigned char* final_mask;                       /* [H,W] out             */
  double* depth_avg;                               /* [H,W] out             */
} aarmvs_fusion_args;
int aarmvs_fusion_filter(const aarmvs_fusion_args* args, hipStream_t stream);

/* ---------------------------------------------------------------------------
 * Epilogue of the evidential head (evidential/models.py:385-459): from the three
 * classifier outputs head[i] = classif_i(...) [1][4][D][H][W] (channels: cost, log nu, log
 * alpha, log beta; at the head's full [maxdisp, H, W] resolution, where get_pred / get_logits'
 * align_corners=True trilinear resampling is the identity) and depth_values [D]:
 *   prob_i = softmax_D(cost_i) (:421), pred_i = sum_d prob_i depth_values (disparity_regression,
 *   :40-45), nu_i / alpha_i / beta_i = softplus(sum_d prob_i logit_i) (+1 for alpha; :426-430,
 *   :281-285), the NIG mixture moe_nig(moe_nig(e0, e1), e2) (:287-304) -> evidential [4][H*W]
 *   = (gamma, nu, alpha, beta), and prob_combine [D][H*W] = the mean of the three prob_i
 *   (:457-458).  B == 1 and D == AARMVS_EVIDENTIAL_D only, the reference head's limits
 *   (SURVEY F2).  HW = H * W.  The backward (for the training losses through the head,
 *   :517-558) takes dL/d evidential and dL/d prob_combine (either may be NULL: zero) and
 *   overwrites grad_head[i] [1][4][D][H][W]; no gradient flows to depth_values.
 * ------------------------------------------------------------------------- */
#define AARMVS_EVIDENTIAL_D 32
int aarmvs_evidential_epilogue(const float* const head[3], const float* depth_values, int D, int HW,
                               float* evidential, float* prob_combine, hipStream_t stream);
int aarmvs_evidential_epilogue_backward(const float* const head[3], const float* depth_values, int D,
                                        int HW, const float* grad_evidential,
                                        const float* grad_prob_combine, float* const grad_head[3],
                                        hipStream_t stream);

/* ---------------------------------------------------------------------------
 * The sampling half of FeatNet's modulated deformable convolution (models/module.py:105-236,
 * DeformConv2d.forward; used by IntraViewAAModule, drmvsnet.py:7-24): for output pixel (i, j)
 * and tap n of the 3x3 kernel, the bilinear sample of the zero-padded input at
 * (i*stride + 1 + n/3 - 1 + offset[n], j*stride + 1 + n%3 - 1 + offset[9 + n]) with the
 * reference's clamping and corner weights (:160-214), times mask[n] (the sigmoid of m_conv,
 * :216-219; NULL: no modulation).  x_nhwc [B][H][W][C] (C == 32), offset [B][18][h][w], mask
 * [B][9][h][w], val [B][h*w][9][C]: the A operand of the conv over (tap, channel) (:230-234),
 * which the caller multiplies by the weights [9*C][outc].  The forward's val equals the
 * reference's sampled tensor op for op in fp32.  The backward takes dL/d val and ADDS dL/dx
 * into grad_x_nhwc (atomically: zero it first), and writes dL/d offset [B][18][h][w] and
 * dL/d mask [B][9][h][w] (NULL when mask is NULL); like the reference's gather backward, dL/dx's
 * summation order is not fixed.
 * ------------------------------------------------------------------------- */
#define AARMVS_DEFORM_C 32
int aarmvs_deform_sample(const float* x_nhwc, const float* offset, const float* mask, int B, int C,
                         int H, int W, int h, int w, int stride, int pad, float* val,
                         hipStream_t stream);
int aarmvs_deform_sample_backward(const float* x_nhwc, const float* offset, const float* mask, int B,
                                  int C, int H, int W, int h, int w, int stride, int pad,
                                  const float* grad_val, float* grad_x_nhwc, float* grad_offset,
                                  float* grad_mask, hipStream_t stream);

/* ---------------------------------------------------------------------------
 * Opt-in per-kernel timing (a diagnostic, not part of the reference interface).
 * When enabled, every launch made by the entry points above is bracketed by
 * hipEvents on its stream; aarmvs_profile_read synchronises on the recorded
 * events and returns the launch count and summed device time of one kernel.
 * ------------------------------------------------------------------------- */
void aarmvs_profile_enable(int on);
void aarmvs_profile_reset(void);
int aarmvs_profile_kernel_count(void);
const char* aarmvs_profile_kernel_name(int id);
int aarmvs_profile_read(int id, long long* launches, double* total_ms);

#ifdef __cplusplus
}
#endif
#endif /* AARMVS_H_ */
