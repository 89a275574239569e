"""Drop-in ``models.drmvsnet`` (BuTTerK3ks/AA-RMVSNet, models/drmvsnet.py) whose depth
sweep runs on the MI355X HIP library.

Same public names, constructor/forward signatures, return values and submodule names
(so the reference checkpoints' ``feature.*``, ``omega.*`` and ``cost_regularization.*``
keys load unchanged) as the reference:

* ``EMVSNet(disparity_level, image_scale=0.25, max_h=960, max_w=480, return_depth=False)``
  (drmvsnet.py:234-253) and ``forward(imgs, proj_matrices, depth_values)``
  (drmvsnet.py:255-345);
* ``mvsnet_cls_loss`` (drmvsnet.py:347-381);
* ``FeatNet``, ``IntraViewAAModule``, ``InterViewAAModule``, ``UNetConvLSTM`` and the
  blocks of ``models.module``.

What runs where:
* FeatNet (2D CNN) stays PyTorch (north_star).
* The D-loop (warp x (N-1), squared difference, omega re-weighting, accumulation,
  ConvLSTM U-Net step, online WTA, softmax over D) runs in libaarmvs.so
  (``aarmvs.ops.DepthSweep``).  There is no CPU fallback: CPU tensors raise.
* Training (autograd through the sweep): the forward is one HIP sweep call that keeps a
  training record (~1 KB/px/plane instead of the reference's ~2.3 KB/px/plane of autograd
  activations); the backward (BPTT through every plane, the omega/warp backward and all
  parameter gradients) is the library's aarmvs_sweep_backward.
* The evidential head (evidential/models.py) is this package's PyTorch
  restatement ``evidential.models.EvidentialModule``, attached by default with the
  reference's 221 ``evidential.*`` keys (311 keys in all, as the reference: its shipped
  90-key checkpoints do not load strictly; ``evidential=False`` drops the head).
  It runs on the softmax of the HIP cost volume.  The reference head only works at B == 1
  and D == 32 and raises elsewhere; here ``EMVSNet.forward`` returns None for
  its outputs at other shapes (``evidential="strict"`` raises EvidentialShapeError, like
  the reference), so the sweep's outputs stay usable at every BASELINE config.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from aarmvs import ops as _ops
from aarmvs._lib import AarmvsError
from evidential.models import EvidentialModule, EvidentialShapeError
from evidential.models import *  # noqa: F401,F403  (the reference: drmvsnet.py:5)

from .module import *  # noqa: F401,F403  (reference re-exports models.module names)
from .module import (ConvLSTMCell, convgnrelu, deConvGnReLU, deformconvgnrelu,
                     homo_warping_depthwise, resnet_block_gn)

__all__ = [
    "IntraViewAAModule", "InterViewAAModule", "FeatNet", "UNetConvLSTM", "EMVSNet",
    "mvsnet_cls_loss", "EvidentialUnavailable", "EvidentialModule", "EvidentialShapeError",
    "loss_der", "loss_emvsnet", "criterion_uncertainty",
    "homo_warping_depthwise", "ConvLSTMCell", "convgnrelu", "DeformConv2d", "deformconvgnrelu",
    "ResnetBlockGn", "resnet_block_gn", "deConvGnReLU",
]
from .module import DeformConv2d, ResnetBlockGn  # noqa: E402,F401
from evidential.models import criterion_uncertainty, loss_der, loss_emvsnet  # noqa: E402,F401


# ----------------------------------------------------------------------------------
# 2D feature network (PyTorch, out of the HIP scope)   drmvsnet.py:7-63
# ----------------------------------------------------------------------------------
class IntraViewAAModule(nn.Module):
    """drmvsnet.py:7-24: three deformable branches at 1, 1/2, 1/4 resolution, fused."""

    def __init__(self):
        super().__init__()
        bf = 8
        self.deformconv0 = deformconvgnrelu(bf * 4, bf * 4, kernel_size=3, stride=1, dilation=1)
        self.conv0 = convgnrelu(bf * 4, bf * 2, kernel_size=1, stride=1, dilation=1)
        self.deformconv1 = deformconvgnrelu(bf * 4, bf * 4, kernel_size=3, stride=1, dilation=1)
        self.conv1 = convgnrelu(bf * 4, bf * 1, kernel_size=1, stride=1, dilation=1)
        self.deformconv2 = deformconvgnrelu(bf * 4, bf * 4, kernel_size=3, stride=1, dilation=1)
        self.conv2 = convgnrelu(bf * 4, bf * 1, kernel_size=1, stride=1, dilation=1)

    def forward(self, x0, x1, x2):
        m0 = self.conv0(self.deformconv0(x0))
        m1 = F.interpolate(self.conv1(self.deformconv1(x1)), scale_factor=2, mode="bilinear",
                           align_corners=True)
        m2 = F.interpolate(self.conv2(self.deformconv2(x2)), scale_factor=4, mode="bilinear",
                           align_corners=True)
        return torch.cat([m0, m1, m2], 1)


class InterViewAAModule(nn.Module):
    """drmvsnet.py:27-38: per-view saliency weight from the squared-difference volume."""

    def __init__(self, in_channels=32, bias=True):
        super().__init__()
        self.reweight_network = nn.Sequential(
            convgnrelu(in_channels, 4, kernel_size=3, stride=1, dilation=1, bias=bias),
            resnet_block_gn(4, kernel_size=1),
            nn.Conv2d(4, 1, kernel_size=1, padding=0),
            nn.Sigmoid(),
        )

    def forward(self, x):
        return self.reweight_network(x)


class FeatNet(nn.Module):
    """drmvsnet.py:41-63: 32-channel features at input resolution."""

    def __init__(self):
        super().__init__()
        bf = 8
        self.init_conv = nn.Sequential(
            convgnrelu(3, bf, kernel_size=3, stride=1, dilation=1),
            convgnrelu(bf, bf * 2, kernel_size=3, stride=1, dilation=1),
        )
        self.conv0 = convgnrelu(bf * 2, bf * 4, kernel_size=3, stride=1, dilation=1)
        self.conv1 = convgnrelu(bf * 4, bf * 4, kernel_size=3, stride=2, dilation=1)
        self.conv2 = convgnrelu(bf * 4, bf * 4, kernel_size=3, stride=2, dilation=1)
        self.intraAA = IntraViewAAModule()

    def forward(self, x):
        x0 = self.conv0(self.init_conv(x))
        x1 = self.conv1(x0)
        x2 = self.conv2(x1)
        return self.intraAA(x0, x1, x2)


# ----------------------------------------------------------------------------------
# recurrent regulariser   drmvsnet.py:66-218
# ----------------------------------------------------------------------------------
class UNetConvLSTM(nn.Module):
    """drmvsnet.py:66-218 (process_sq branch).  ``forward`` is the PyTorch step used by the
    training recompute; EMVSNet's sweep runs the same step in libaarmvs."""

    def __init__(self, input_size, input_dim, hidden_dim, kernel_size, num_layers, bias=True):
        super().__init__()
        if not (isinstance(kernel_size, tuple) or
                (isinstance(kernel_size, list) and all(isinstance(k, tuple) for k in kernel_size))):
            raise ValueError("`kernel_size` must be tuple or list of tuples")
        kernel_size = kernel_size if isinstance(kernel_size, list) else [kernel_size] * num_layers
        hidden_dim = hidden_dim if isinstance(hidden_dim, list) else [hidden_dim] * num_layers
        if not len(kernel_size) == len(hidden_dim) == num_layers:
            raise ValueError("Inconsistent list length.")
        self.height, self.width = input_size
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.kernel_size = kernel_size
        self.num_layers = num_layers
        self.bias = bias
        self.down_num = (num_layers + 1) / 2
        cells = []
        for i in range(num_layers):
            scale = 2 ** i if i < self.down_num else 2 ** (num_layers - i - 1)
            cells.append(ConvLSTMCell(input_size=(int(self.height / scale), int(self.width / scale)),
                                      input_dim=input_dim[i], hidden_dim=hidden_dim[i],
                                      kernel_size=kernel_size[i], bias=bias))
        self.cell_list = nn.ModuleList(cells)
        self.deconv_0 = deConvGnReLU(16, 16, kernel_size=3, stride=2, padding=1, bias=bias,
                                     output_padding=1)
        self.deconv_1 = deConvGnReLU(16, 16, kernel_size=3, stride=2, padding=1, bias=bias,
                                     output_padding=1)
        self.conv_0 = nn.Conv2d(8, 1, 3, 1, padding=1)

    def _init_hidden(self, batch_size, device=None):
        return [list(c.init_hidden(batch_size, device)) for c in self.cell_list]

    def forward(self, input_tensor, hidden_state=None, idx=0, process_sq=True):
        if not process_sq:
            # drmvsnet.py:168-200 is dead code in the reference (nn.Tanh(cost) raises)
            raise NotImplementedError("UNetConvLSTM: only the process_sq=True step exists")
        if idx == 0:
            hidden_state = self._init_hidden(input_tensor.size(0), input_tensor.device)
        cl = self.cell_list
        h0, c0 = cl[0](input_tensor, hidden_state[0])
        h1, c1 = cl[1](F.max_pool2d(h0, 2, 2), hidden_state[1])
        h2, c2 = cl[2](F.max_pool2d(h1, 2, 2), hidden_state[2])
        h3, c3 = cl[3](torch.cat([self.deconv_0(h2), h1], 1), hidden_state[3])
        h4, c4 = cl[4](torch.cat([self.deconv_1(h3), h0], 1), hidden_state[4])
        hidden_state[0], hidden_state[1], hidden_state[2] = [h0, c0], [h1, c1], [h2, c2]
        hidden_state[3], hidden_state[4] = [h3, c3], [h4, c4]
        return self.conv_0(h4), hidden_state


class EvidentialUnavailable(nn.Module):
    """No evidential head (``EMVSNet(..., evidential=False)``): outputs are None."""

    def __init__(self, depth=None):
        super().__init__()
        self.depth = depth

    def forward(self, prob_volume, depth_values):
        return None, None


# sweep parameters in the library's raw-blob order (include/aarmvs.h).  Looked up by
# walking attributes, not named_parameters(): nn.DataParallel replicas (train.py:173,
# eval.py:77) hold their parameter copies as plain attributes and expose none.
def _sweep_params(model: "EMVSNet"):
    out = []
    for key in _ops.SWEEP_KEYS:
        obj = model
        for part in key.split("."):
            obj = getattr(obj, part)
        out.append(obj)
    return out


class _SweepTrain(torch.autograd.Function):
    """cost volume [B,D,H,W] of the sweep with its backward (BPTT) on the HIP library.

    The forward is ONE aarmvs_sweep call over all D planes with a training record (the cost
    slices, every plane's regulariser state, gate pre-activations and deconv outputs: ~1 KB
    per pixel and plane, instead of the reference's ~2.3 KB of autograd activations); the
    backward is aarmvs_sweep_backward on that record (the recurrence's reverse sweep, the
    cost-slice / omega / warp backward and every parameter gradient, drmvsnet.py:273-291
    differentiated).  The record is saved with save_for_backward, so autograd frees it after
    the backward and a second backward through a freed graph raises autograd's own error."""

    @staticmethod
    def forward(ctx, model, sweep, ref_proj, src_projs, depth_values, ref, *rest):
        nsrc = len(src_projs)
        srcs, params = list(rest[:nsrc]), rest[nsrc:]
        B, C, H, W = ref.shape
        D = depth_values.shape[1]
        cost = torch.empty(B, D, H, W, device=ref.device)
        rel = sweep.relative(ref_proj, src_projs, B)
        rec = sweep.record_buffers(B, H, W, D, ref.device, nsrc=nsrc)
        sweep(ref, srcs, ref_proj, src_projs, depth_values, want_depth=False, cost_out=cost,
              rel=rel, record=rec)
        ctx.sweep = sweep
        ctx.nsrc = nsrc
        ctx.nparams = len(params)
        ctx.save_for_backward(ref, *srcs, rel, depth_values, *(rec[k] for k in _ops.DepthSweep.RECORD_KEYS))
        return cost

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad_cost):
        saved = ctx.saved_tensors
        nsrc = ctx.nsrc
        ref, srcs = saved[0], list(saved[1:1 + nsrc])
        rel, dv = saved[1 + nsrc], saved[2 + nsrc]
        rec = dict(zip(_ops.DepthSweep.RECORD_KEYS, saved[3 + nsrc:]))
        g_ref, g_srcs, g_par, _ = ctx.sweep.backward(ref, srcs, rel, dv, rec, grad_cost)
        g_params = [g_par[k] for k in _ops.SWEEP_KEYS]
        return (None, None, None, None, None, g_ref, *g_srcs, *g_params)


class _SoftmaxDepth(torch.autograd.Function):
    """softmax over dim 1 of [B,D,H,W] (drmvsnet.py:291/:342) on the HIP kernel."""

    @staticmethod
    def forward(ctx, cost):
        p = _ops.softmax_depth(cost)
        ctx.save_for_backward(p)
        return p

    @staticmethod
    def backward(ctx, g):
        (p,) = ctx.saved_tensors
        return p * (g - (g * p).sum(dim=1, keepdim=True))


class EMVSNet(nn.Module):
    """drmvsnet.py:234-345 with the depth loop on libaarmvs (gfx950)."""

    BACKWARD_PATH = ("aarmvs_sweep_backward (HIP): one recorded forward sweep, the BPTT "
                     "(gate / input-gradient / GroupNorm / deconv kernels per plane, weight "
                     "gradients per 16-plane group) and the cost-slice backward (omega chain, "
                     "warp gather/scatter) on gfx950")

    def __init__(self, disparity_level, image_scale=0.25, max_h=960, max_w=480, return_depth=False,
                 evidential=True):
        super().__init__()
        self.feature = FeatNet()
        input_size = (int(max_h * image_scale), int(max_w * image_scale))
        num_layers = 5
        self.cost_regularization = UNetConvLSTM(input_size, [32, 16, 16, 32, 32],
                                                [16, 16, 16, 16, 8],
                                                [(3, 3) for _ in range(num_layers)], num_layers,
                                                bias=True)
        self.omega = InterViewAAModule(32)
        if evidential:
            self.evidential = EvidentialModule(depth=disparity_level)
        else:
            self.evidential = EvidentialUnavailable(depth=disparity_level)
        self.evidential_strict = evidential == "strict"
        self.return_depth = return_depth
        self._sweep_cache = None

    # -- HIP sweep object, repacked whenever a sweep parameter changed ---------------
    def _sweep(self, device) -> _ops.DepthSweep:
        params = _sweep_params(self)
        key = (str(device), tuple((p.data_ptr(), p._version) for p in params))
        if self._sweep_cache is None or self._sweep_cache[0] != key:
            sw = _ops.DepthSweep({k: p.detach() for k, p in zip(_ops.SWEEP_KEYS, params)}, device)
            self._sweep_cache = (key, sw)
        return self._sweep_cache[1]

    def _check_geometry(self, H, W):
        reg = self.cost_regularization
        if (H, W) != (reg.height, reg.width):
            raise ValueError(f"EMVSNet: feature size {H}x{W} differs from the hidden-state size "
                             f"{reg.height}x{reg.width} fixed by (max_h, max_w) * image_scale "
                             "(drmvsnet.py:239, module.py:95)")

    def forward(self, imgs, proj_matrices, depth_values):
        imgs = torch.unbind(imgs, 1)
        projs = torch.unbind(proj_matrices, 1)
        assert len(imgs) == len(projs), "Different number of images and projection matrices"
        if not imgs[0].is_cuda:
            raise AarmvsError("EMVSNet: the depth sweep runs on libaarmvs (ROCm device tensors "
                              "required; there is no CPU fallback)")
        features = [self.feature(img) for img in imgs]
        ref, srcs = features[0], features[1:]
        ref_proj, src_projs = projs[0], list(projs[1:])
        B, C, H, W = ref.shape
        self._check_geometry(H, W)
        sweep = self._sweep(ref.device)
        dv = depth_values.float()
        # the reference head runs at B == 1, D == 32 only
        evidential_on = not isinstance(self.evidential, EvidentialUnavailable) and (
            self.evidential_strict or (B == 1 and depth_values.shape[1] == 32))

        if not self.return_depth:
            params = _sweep_params(self)
            need_grad = torch.is_grad_enabled() and (
                ref.requires_grad or any(s.requires_grad for s in srcs) or
                any(p.requires_grad for p in params))
            if need_grad:
                cost = _SweepTrain.apply(self, sweep, ref_proj, src_projs, dv, ref, *srcs, *params)
            else:
                cost = sweep(ref, srcs, ref_proj, src_projs, dv, want_depth=False,
                             want_cost=True)["cost"]
            prob = _SoftmaxDepth.apply(cost)
            evidential, prob_combine = None, None
            if evidential_on:
                evidential, prob_combine = self.evidential(prob, depth_values)
            return prob, evidential, prob_combine

        out = sweep(ref, srcs, ref_proj, src_projs, dv, want_depth=True, want_cost=evidential_on)
        evidential = None
        if evidential_on:
            evidential, _ = self.evidential(_ops.softmax_depth(out["cost"]), depth_values)
        return {"depth": out["depth"], "photometric_confidence": out["conf"],
                "evidential_prediction": evidential}


def mvsnet_cls_loss(prob_volume, depth_gt, mask, depth_value, return_prob_map=False):
    """drmvsnet.py:347-381: masked cross entropy against the one-hot nearest hypothesis.

    Returns (loss, wta_depth[, max-prob confidence]).
    """
    B, H, W = depth_gt.shape
    D = depth_value.shape[-1]
    valid = mask.sum(dim=[1, 2]) + 1e-6
    dv_map = depth_value.view(B, D, 1, 1).expand(B, D, H, W)
    gt_idx = torch.argmin((dv_map - depth_gt.unsqueeze(1)).abs(), dim=1)
    gt_idx = torch.round(mask * gt_idx.float()).long().unsqueeze(1)
    onehot = torch.zeros(B, D, H, W, dtype=mask.dtype, device=mask.device).scatter_(1, gt_idx, 1)
    ce = -(onehot * torch.log(prob_volume)).sum(dim=1)
    loss = ((mask * ce).sum(dim=[1, 2]) / valid).mean()
    wta_idx = torch.argmax(prob_volume, dim=1, keepdim=True)
    wta = torch.gather(dv_map, 1, wta_idx).squeeze(1)
    if return_prob_map:
        return loss, wta, prob_volume.max(dim=1)[0]
    return loss, wta
