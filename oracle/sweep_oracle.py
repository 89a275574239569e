"""CPU oracle for the AA-RMVSNet depth-sweep hot path (TEST INFRASTRUCTURE ONLY).

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The shipped path (``aa-rmvsnet_amd``) never imports it and has no CPU fallback.

It restates, in plain fp32 PyTorch-CPU tensor arithmetic, the algorithm of the
reference's per-plane sweep (``/root/reference`` = BuTTerK3ks/AA-RMVSNet):

* homography grid          models/module.py:15-33
* bilinear sampling        models/module.py:36-37 -> F.grid_sample(bilinear, zeros,
                           align_corners=False default on torch>=1.3).
                           Restated here as an explicit 4-tap gather following the
                           ATen CPU kernel's compiled arithmetic (fma-contracted
                           unnormalise (g+1)*W/2-0.5 and tap accumulation).
* squared difference       models/drmvsnet.py:311
* inter-view AA (omega)    models/drmvsnet.py:27-38, module.py:98-103, 252-267
* weighted accumulation    models/drmvsnet.py:313-319
* UNetConvLSTM step        models/drmvsnet.py:119-167, ConvLSTMCell module.py:76-92,
                           deConvGnReLU module.py:269-287
* online WTA / confidence  models/drmvsnet.py:301-304, 324-339
* softmax over depth       models/drmvsnet.py:289-291, 341-342

Parity is pinned by the golden fixtures in ``tests/golden`` that were produced by
importing and running the reference itself in the build container
(``tests/golden/make_golden.py``); ``tests/test_oracle.py`` checks this module
against them.

Parameters are passed as a dict keyed by the reference's own ``state_dict`` names
(``omega.reweight_network.0.0.weight`` ...), i.e. the checkpoint layout.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

GN_EPS = 1e-5  # nn.GroupNorm default, module.py:101,258,284


# ----------------------------------------------------------------------------------
# homography + bilinear warp  (module.py:6-38)
# ----------------------------------------------------------------------------------
def relative_projection(src_proj: torch.Tensor, ref_proj: torch.Tensor) -> torch.Tensor:
    """P = src_proj @ inv(ref_proj) -> rows 0..2 ([B,3,4]), module.py:16-18."""
    proj = torch.matmul(src_proj.float(), torch.inverse(ref_proj.float()))
    return proj[:, :3, :4].contiguous()


def homography_grid(rel: torch.Tensor, depth: torch.Tensor, H: int, W: int):
    """Normalised sampling grid of module.py:20-33.  rel [B,3,4], depth [B]."""
    B = rel.shape[0]
    rot, trans = rel[:, :, :3], rel[:, :, 3:4]
    y, x = torch.meshgrid(torch.arange(H, dtype=torch.float32),
                          torch.arange(W, dtype=torch.float32), indexing="ij")
    xyz = torch.stack((x.reshape(-1), y.reshape(-1), torch.ones(H * W)))       # [3,HW]
    rot_xyz = torch.matmul(rot, xyz.unsqueeze(0).expand(B, 3, H * W))          # [B,3,HW]
    p = rot_xyz * depth.view(B, 1, 1).float() + trans                           # :27-28
    z = p[:, 2]
    z = torch.where(z == 0, z + 1e-4, z)                                        # :29
    px, py = p[:, 0] / z, p[:, 1] / z                                           # :30
    gx = px / ((W - 1) / 2) - 1                                                 # :31
    gy = py / ((H - 1) / 2) - 1                                                 # :32
    return gx.view(B, H, W), gy.view(B, H, W)


def _fma(a: torch.Tensor, b, c: torch.Tensor) -> torch.Tensor:
    """fp32 fused multiply-add, emulated exactly enough in fp64 (product is exact)."""
    return (a.double() * (b.double() if torch.is_tensor(b) else b) + c.double()).float()


def bilinear_zeros(src: torch.Tensor, gx: torch.Tensor, gy: torch.Tensor) -> torch.Tensor:
    """grid_sample(bilinear, padding zeros, align_corners=False) as a 4-tap gather.

    Arithmetic follows ATen's CPU kernel as compiled (GridSamplerKernel.cpp with
    GCC's default FP contraction): ix = fma(gx + 1, W/2, -0.5) and the four taps
    accumulated as an fma chain nw -> ne -> sw -> se.  Verified bit-exact against the
    reference on the warp fixture.
    """
    B, C, Hs, Ws = src.shape
    ix = _fma(gx + 1, Ws / 2, torch.full_like(gx, -0.5))
    iy = _fma(gy + 1, Hs / 2, torch.full_like(gy, -0.5))
    x0, y0 = torch.floor(ix), torch.floor(iy)
    wx, wy = ix - x0, iy - y0
    ex, sy = 1 - wx, 1 - wy
    flat = src.reshape(B, C, Hs * Ws)
    acc = None
    for dy, dx, wgt in ((0, 0, sy * ex), (0, 1, sy * wx), (1, 0, wy * ex), (1, 1, wy * wx)):
        xi, yi = x0 + dx, y0 + dy
        ok = (xi > -1) & (xi < Ws) & (yi > -1) & (yi < Hs)
        xi_c = torch.where(ok, xi, torch.zeros_like(xi)).long()
        yi_c = torch.where(ok, yi, torch.zeros_like(yi)).long()
        idx = (yi_c * Ws + xi_c).view(B, 1, -1).expand(B, C, -1)
        val = torch.gather(flat, 2, idx).view(B, C, *gx.shape[1:])
        val = torch.where(ok.unsqueeze(1), val, torch.zeros_like(val))
        w = wgt.unsqueeze(1)
        acc = val * w if acc is None else _fma(val, w, acc)
    return acc


def homo_warp(src_fea: torch.Tensor, rel: torch.Tensor, depth: torch.Tensor,
              fast: bool = False) -> torch.Tensor:
    """homo_warping_depthwise (module.py:6-38) for a precomputed rel = src@inv(ref).

    ``fast`` samples with ``F.grid_sample`` itself (the reference's own call,
    module.py:36-37, align_corners=False as torch>=1.3 defaults) instead of the explicit
    gather: the same ATen kernel the reference runs, used by the CPU timing baseline
    (bench.py) so that it costs what the reference costs.  With ``fast`` a
    float64 ``src_fea`` is sampled in float64 (on the reference's fp32 grid): the fp64
    anchor of the gradient tests.
    """
    H, W = src_fea.shape[2:]
    gx, gy = homography_grid(rel, depth, H, W)
    if fast:
        grid = torch.stack((gx, gy), dim=3)
        src = src_fea if src_fea.dtype == torch.float64 else src_fea.float()
        return F.grid_sample(src, grid.to(src.dtype), mode="bilinear", padding_mode="zeros",
                             align_corners=False)
    return bilinear_zeros(src_fea.float(), gx, gy)


# ----------------------------------------------------------------------------------
# normalisation helpers
# ----------------------------------------------------------------------------------
def group_norm(x: torch.Tensor, groups: int, gamma: torch.Tensor, beta: torch.Tensor,
               eps: float = GN_EPS, fast: bool = False) -> torch.Tensor:
    """GroupNorm with biased variance over (C/G, H, W) per sample and group.  ``fast`` calls
    F.group_norm, the ATen kernel nn.GroupNorm (the reference) runs."""
    if fast:
        return F.group_norm(x, groups, gamma, beta, eps)
    B, C, H, W = x.shape
    xg = x.reshape(B, groups, -1)
    mean = xg.mean(dim=2, keepdim=True)
    var = ((xg - mean) ** 2).mean(dim=2, keepdim=True)
    y = ((xg - mean) / torch.sqrt(var + eps)).reshape(B, C, H, W)
    return y * gamma.view(1, C, 1, 1) + beta.view(1, C, 1, 1)


# ----------------------------------------------------------------------------------
# inter-view adaptive aggregation (omega)   drmvsnet.py:27-38
# ----------------------------------------------------------------------------------
def omega_weight(sq: torch.Tensor, P: dict, fast: bool = False) -> torch.Tensor:
    k = "omega.reweight_network."
    a = F.conv2d(sq, P[k + "0.0.weight"], P[k + "0.0.bias"], padding=1)
    a = F.relu(group_norm(a, 1, P[k + "0.1.weight"], P[k + "0.1.bias"], fast=fast))
    t = F.conv2d(a, P[k + "1.stem.0.0.weight"], P[k + "1.stem.0.0.bias"])
    t = F.relu(group_norm(t, 1, P[k + "1.stem.0.1.weight"], P[k + "1.stem.0.1.bias"], fast=fast))
    t = F.conv2d(t, P[k + "1.stem.1.weight"], P[k + "1.stem.1.bias"])
    t = group_norm(t, 1, P[k + "1.stem.2.weight"], P[k + "1.stem.2.bias"], fast=fast)
    r = F.relu(t + a)                                                # ResnetBlockGn :262-263
    z = F.conv2d(r, P[k + "2.weight"], P[k + "2.bias"])
    if LOGIT_HOOK is not None:   # tests: the pre-sigmoid logits (their gradients are the bias's terms)
        LOGIT_HOOK(z)
    return torch.sigmoid(z)


# test hook: called with every omega logit tensor (the input of the final sigmoid) if set
LOGIT_HOOK = None


def cost_slice(ref_fea, src_feas, rels, depth, P, fast: bool = False) -> torch.Tensor:
    """-(sum_v (1+w_v)(warp_v-ref)^2)/(N-1), drmvsnet.py:307-319 (sign folded in)."""
    acc = None
    for src, rel in zip(src_feas, rels):
        sq = (homo_warp(src, rel, depth, fast) - ref_fea).pow(2)
        w = omega_weight(sq, P, fast)
        term = (w + 1) * sq
        acc = term if acc is None else acc + term
    return -1 * (acc / len(src_feas))


# ----------------------------------------------------------------------------------
# recurrent regulariser   drmvsnet.py:66-167
# ----------------------------------------------------------------------------------
CELL_HID = (16, 16, 16, 16, 8)


def lstm_cell(x, h, c, w, b):
    z = F.conv2d(torch.cat([x, h], 1), w, b, padding=1)
    i, f, o, g = torch.split(z, h.shape[1], dim=1)
    c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
    h2 = torch.sigmoid(o) * torch.tanh(c2)
    return h2, c2


def deconv_gn_relu(x, P, name, fast=False):
    k = "cost_regularization." + name + "."
    y = F.conv_transpose2d(x, P[k + "conv.weight"], P[k + "conv.bias"], stride=2,
                           padding=1, output_padding=1)
    return F.relu(group_norm(y, 2, P[k + "gn.weight"], P[k + "gn.bias"], fast=fast))


def init_state(B, H, W):
    shapes = [(16, H, W), (16, H // 2, W // 2), (16, H // 4, W // 4), (16, H // 2, W // 2), (8, H, W)]
    return [(torch.zeros(B, *s), torch.zeros(B, *s)) for s in shapes]


def unet_step(x, state, P, fast=False):
    """One depth step of UNetConvLSTM (process_sq branch), returns cost [B,1,H,W]."""
    cw = lambda i: (P[f"cost_regularization.cell_list.{i}.conv.weight"],
                    P[f"cost_regularization.cell_list.{i}.conv.bias"])
    h0, c0 = lstm_cell(x, *state[0], *cw(0))
    h1, c1 = lstm_cell(F.max_pool2d(h0, 2, 2), *state[1], *cw(1))
    h2, c2 = lstm_cell(F.max_pool2d(h1, 2, 2), *state[2], *cw(2))
    h3, c3 = lstm_cell(torch.cat([deconv_gn_relu(h2, P, "deconv_0", fast), h1], 1), *state[3], *cw(3))
    h4, c4 = lstm_cell(torch.cat([deconv_gn_relu(h3, P, "deconv_1", fast), h0], 1), *state[4], *cw(4))
    cost = F.conv2d(h4, P["cost_regularization.conv_0.weight"],
                    P["cost_regularization.conv_0.bias"], padding=1)
    return cost, [(h0, c0), (h1, c1), (h2, c2), (h3, c3), (h4, c4)]


# ----------------------------------------------------------------------------------
# full sweep
# ----------------------------------------------------------------------------------
@torch.no_grad()
def sweep(ref_fea, src_feas, ref_proj, src_projs, depth_values, P, planes=None,
          want_volume=True, fast=False, plane_times=None):
    """EMVSNet.forward's depth loop on precomputed features.

    Returns dict(depth [B,H,W], conf [B,H,W], cost [B,D,H,W] or None,
    prob [B,D,H,W] or None).  ``planes`` limits the loop (CPU-baseline sampling);
    ``fast`` warps with F.grid_sample (see homo_warp); ``plane_times``, if a list,
    receives each plane's wall seconds.
    """
    import time
    P = {k: v.float() for k, v in P.items()}
    B, C, H, W = ref_fea.shape
    rels = [relative_projection(sp, ref_proj) for sp in src_projs]
    D = depth_values.shape[1] if planes is None else planes
    state = init_state(B, H, W)
    depth_img = torch.zeros(B, H, W)
    max_prob = torch.zeros(B, H, W)
    exp_sum = torch.zeros(B, H, W)
    costs = []
    for d in range(D):
        t0 = time.perf_counter()
        dv = depth_values[:, d].float()
        x = cost_slice(ref_fea.float(), [s.float() for s in src_feas], rels, dv, P, fast)
        cost, state = unet_step(x, state, P, fast)
        if want_volume:
            costs.append(cost)
        prob = torch.exp(cost.squeeze(1))                       # :324 (no max-subtraction)
        flag = (max_prob < prob).float()                        # :327 strict: first plane wins ties
        max_prob = flag * prob + (1 - flag) * max_prob          # :328 arithmetic select (NaN-faithful)
        depth_img = flag * dv.view(B, 1, 1).expand(B, H, W) + (1 - flag) * depth_img
        exp_sum = exp_sum + prob                                # :334
        if plane_times is not None:
            plane_times.append(time.perf_counter() - t0)
    out = {"depth": depth_img, "conf": max_prob / exp_sum, "cost": None, "prob": None}
    if want_volume:
        vol = torch.stack(costs, 1).squeeze(2)
        out["cost"] = vol
        out["prob"] = F.softmax(vol, dim=1)
    return out


# ----------------------------------------------------------------------------------
# training step through the sweep (train.py:297-306)
# ----------------------------------------------------------------------------------
def cls_loss(prob_volume, depth_gt, mask, depth_value):
    """mvsnet_cls_loss (drmvsnet.py:347-372): masked cross entropy of the one-hot nearest
    hypothesis (argmin |d - gt|, :357; index 0 where the mask is 0, :359-360) against
    log(prob), summed per sample over valid pixels / (count + 1e-6), mean over the batch."""
    B, D, H, W = prob_volume.shape
    dvm = depth_value.to(prob_volume.dtype).view(B, D, 1, 1).expand(B, D, H, W)
    idx = torch.argmin((dvm - depth_gt.to(prob_volume.dtype).unsqueeze(1)).abs(), dim=1)
    idx = torch.round(mask.to(prob_volume.dtype) * idx.to(prob_volume.dtype)).long().unsqueeze(1)
    onehot = torch.zeros_like(prob_volume).scatter_(1, idx, 1)
    ce = -(onehot * torch.log(prob_volume)).sum(dim=1)
    m = mask.to(prob_volume.dtype)
    return ((m * ce).sum(dim=[1, 2]) / (m.sum(dim=[1, 2]) + 1e-6)).mean()


def train_grads(features, proj, depth_values, P, depth_gt, mask, dtype=torch.float32):
    """The training step's gradients through the sweep by CPU autograd in ``dtype``:
    EMVSNet.forward train branch (drmvsnet.py:272-291, features as the leaves: identity
    FeatNet) -> softmax -> cls_loss -> backward.  float32 is the reference's arithmetic,
    float64 the anchor.  features [N,B,32,H,W], proj [B,N,4,4].
    Returns (loss, prob, dL/dfeatures [N,B,32,H,W], {param: dL/dparam})."""
    N, B, C, H, W = features.shape
    fc = features.to(dtype).clone().requires_grad_(True)
    Pp = {k: v.detach().to(dtype).clone().requires_grad_(True) for k, v in P.items()}
    rels = [relative_projection(proj[:, v], proj[:, 0]) for v in range(1, N)]
    state = [(h.to(dtype), c.to(dtype)) for h, c in init_state(B, H, W)]
    costs = []
    for d in range(depth_values.shape[1]):
        x = cost_slice(fc[0], [fc[v] for v in range(1, N)], rels, depth_values[:, d], Pp, fast=True)
        cost, state = unet_step(x, state, Pp)
        costs.append(cost)
    prob = F.softmax(torch.stack(costs, 1).squeeze(2), dim=1)
    loss = cls_loss(prob, depth_gt, mask, depth_values)
    loss.backward()
    return loss.detach(), prob.detach(), fc.grad, {k: v.grad for k, v in Pp.items()}
