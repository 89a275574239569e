"""Building blocks of the reference's ``models.module`` (BuTTerK3ks/AA-RMVSNet,
models/module.py), re-exported by ``models.drmvsnet``.

* ``homo_warping_depthwise`` runs on the HIP library (``aarmvs_homo_warp`` forward,
  ``aarmvs_homo_warp_backward`` bilinear scatter for d/d src_fea).  It needs ROCm
  device tensors; there is no CPU fallback.
* The nn.Module blocks keep the reference's constructor signatures and submodule
  names, so ``state_dict`` keys match the reference checkpoints.  Their
  forwards are the plain PyTorch definitions of each block: they are what the 2D
  feature network (out of the HIP scope, north_star) is made of, and what the
  training backward recomputes per depth plane.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from aarmvs import ops as _ops

__all__ = [
    "homo_warping_depthwise", "ConvLSTMCell", "convgnrelu", "DeformConv2d", "deformconvgnrelu",
    "ResnetBlockGn", "resnet_block_gn", "deConvGnReLU",
]


class _HomoWarp(torch.autograd.Function):
    """Bilinear homography warp; gradient flows to src_fea only (module.py:15 no_grad grid)."""

    @staticmethod
    def forward(ctx, src_fea, rel, depth):
        out = _ops.homo_warp(src_fea, rel, depth)
        ctx.save_for_backward(rel, depth)
        ctx.shape = src_fea.shape
        return out

    @staticmethod
    def backward(ctx, grad_out):
        rel, depth = ctx.saved_tensors
        grad_src = None
        if ctx.needs_input_grad[0]:
            grad_src = _ops.homo_warp_backward(grad_out, rel, depth, ctx.shape)
        return grad_src, None, None


def homo_warping_depthwise(src_fea, src_proj, ref_proj, depth_value):
    """models/module.py:6-38.  src_fea [B,C,H,W], src_proj/ref_proj [B,4,4], depth_value [B].

    Returns the source features bilinearly sampled (zero padding, grid_sample's
    align_corners=False convention applied to the align_corners=True-normalised
    grid) at the reference pixels' projections at depth_value.
    """
    rel = _ops.relative_projection(src_proj, ref_proj)
    return _HomoWarp.apply(src_fea, rel, depth_value.detach().reshape(-1))


class ConvLSTMCell(nn.Module):
    """models/module.py:40-96: conv3x3([x, h]) -> gates i, f, o, g."""

    def __init__(self, input_size, input_dim, hidden_dim, kernel_size, bias=True):
        super().__init__()
        self.height, self.width = input_size
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.kernel_size = kernel_size
        self.padding = kernel_size[0] // 2, kernel_size[1] // 2
        self.bias = bias
        self.conv = nn.Conv2d(input_dim + hidden_dim, 4 * hidden_dim, kernel_size=kernel_size,
                              padding=self.padding, bias=bias)

    def forward(self, input_tensor, cur_state):
        h, c = cur_state
        z = self.conv(torch.cat([input_tensor, h], dim=1))
        if z.is_cuda and z.dtype == torch.float32:
            # the gate math of :83-90 in one HIP kernel each way (the BPTT recompute)
            return _ops.lstm_gates(z, c)
        zi, zf, zo, zg = torch.split(z, self.hidden_dim, dim=1)
        c_next = torch.sigmoid(zf) * c + torch.sigmoid(zi) * torch.tanh(zg)
        return torch.sigmoid(zo) * torch.tanh(c_next), c_next

    def init_hidden(self, batch_size, device=None):
        dev = device if device is not None else self.conv.weight.device
        z = torch.zeros(batch_size, self.hidden_dim, self.height, self.width, device=dev)
        return z, z.clone()


def _groups(channels: int, group_channel: int) -> int:
    return int(max(1, channels / group_channel))


class GroupNorm(nn.GroupNorm):
    """nn.GroupNorm (same parameters and state_dict keys) whose GPU forward and backward
    run on the library's HIP GroupNorm kernels (aarmvs_group_norm_forward/_backward).

    ATen's ROCm group_norm reduces each (sample, group) row in ONE thread block
    (RowwiseMomentsCUDAKernel): at B=1 with one or two groups over a full-resolution plane
    that is one or two busy CUs -- 0.9 ms per call at 640x512, over half of a training
    step's GPU time in the BPTT recompute (rocprofv3).  The HIP kernels take
    the statistics as grid-wide fixed-order fp64 reductions and return ATen's output form
    y = x * (rstd * gamma) + (beta - mean * rstd * gamma).  On the CPU the reference's
    F.group_norm runs unchanged."""

    def forward(self, x):
        if not x.is_cuda or x.dtype != torch.float32:
            # CPU, and the dtypes the HIP kernels do not take (autocast, gradcheck in fp64)
            return super().forward(x)
        return _ops.group_norm(x, self.num_groups, self.weight if self.affine else None,
                               self.bias if self.affine else None, self.eps)


def convgnrelu(in_channels, out_channels, kernel_size=3, stride=1, dilation=1, bias=True,
               group_channel=8):
    """models/module.py:98-103."""
    return nn.Sequential(
        nn.Conv2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                  dilation=dilation, padding=((kernel_size - 1) // 2) * dilation, bias=bias),
        GroupNorm(_groups(out_channels, group_channel), out_channels),
        nn.ReLU(inplace=True),
    )


class DeformConv2d(nn.Module):
    """Modulated deformable convolution of models/module.py:105-236 (used by FeatNet).

    Semantics restated: for output pixel (i, j) and kernel tap n = 3*a + b the sampling
    point in the zero-padded input is (row, col) = (i*s + a + off_row, j*s + b + off_col)
    (p_0 starts at 1 = the padding), both coordinates clamped to the padded image; the
    four corner taps are also clamped, each corner weight is the product of
    (1 -/+ (corner - p)) factors, and the sample is scaled by the modulation mask.
    The output is sum_{c,n} W[o,c,n] * sample[c,n] (+ bias).
    """

    def __init__(self, inc, outc, kernel_size=3, padding=1, stride=1, bias=None, modulation=True):
        super().__init__()
        self.kernel_size = kernel_size
        self.padding = padding
        self.stride = stride
        self.zero_padding = nn.ZeroPad2d(padding)
        self.conv = nn.Conv2d(inc, outc, kernel_size=kernel_size, stride=kernel_size, bias=bias)
        self.p_conv = nn.Conv2d(inc, 2 * kernel_size * kernel_size, kernel_size=3, padding=1,
                                stride=stride)
        nn.init.constant_(self.p_conv.weight, 0)
        self.modulation = modulation
        if modulation:
            self.m_conv = nn.Conv2d(inc, kernel_size * kernel_size, kernel_size=3, padding=1,
                                    stride=stride)
            nn.init.constant_(self.m_conv.weight, 0)

    def forward(self, x):
        # the HIP sampler takes float32 only: under autocast p_conv / m_conv return float16
        # offsets, so autocast (like any non-float32 input) takes the PyTorch expression
        if (x.is_cuda and self.kernel_size == 3 and x.shape[1] == 32 and x.dtype == torch.float32
                and not torch.is_autocast_enabled()):
            return self._forward_hip(x)
        ks = self.kernel_size
        n_taps = ks * ks
        offset = self.p_conv(x)                                   # [B, 2n, h, w]
        B, _, h, w = offset.shape
        xp = self.zero_padding(x) if self.padding else x
        Hp, Wp = xp.shape[2], xp.shape[3]
        dt, dev = offset.dtype, offset.device
        a = torch.arange(n_taps, device=dev) // ks - (ks - 1) // 2   # tap row offset
        b = torch.arange(n_taps, device=dev) % ks - (ks - 1) // 2    # tap col offset
        rows = torch.arange(1, h * self.stride + 1, self.stride, device=dev)
        cols = torch.arange(1, w * self.stride + 1, self.stride, device=dev)
        pr = (rows.view(1, 1, h, 1) + a.view(1, n_taps, 1, 1)).to(dt) + offset[:, :n_taps]
        pc = (cols.view(1, 1, 1, w) + b.view(1, n_taps, 1, 1)).to(dt) + offset[:, n_taps:]
        pr, pc = pr.permute(0, 2, 3, 1), pc.permute(0, 2, 3, 1)    # [B, h, w, n]
        r0, c0 = pr.detach().floor(), pc.detach().floor()
        r0c, r1c = r0.clamp(0, Hp - 1), (r0 + 1).clamp(0, Hp - 1)
        c0c, c1c = c0.clamp(0, Wp - 1), (c0 + 1).clamp(0, Wp - 1)
        pr, pc = pr.clamp(0, Hp - 1), pc.clamp(0, Wp - 1)
        C = xp.shape[1]
        # channels-last rows: one gather of the four corners' 32-channel rows (the backward
        # is one scatter-add of contiguous rows, not 4 x C strided planes)
        rows_cl = xp.permute(0, 2, 3, 1).reshape(B, Hp * Wp, C)
        idx = torch.stack([r0c * Wp + c0c, r1c * Wp + c1c, r0c * Wp + c1c, r1c * Wp + c0c], 1)
        idx = idx.long().reshape(B, -1, 1).expand(-1, -1, C)              # [B, 4 h w n, C]
        taps = rows_cl.gather(1, idx).view(B, 4, h * w * n_taps, C)

        # corner weights: (lt) (1+(r0-p))(1+(c0-p)), (rb) (1-(r1-p))(1-(c1-p)),
        # (lb) rows r0 / cols c1, (rt) rows r1 / cols c0
        g_lt = (1 + (r0c - pr)) * (1 + (c0c - pc))
        g_rb = (1 - (r1c - pr)) * (1 - (c1c - pc))
        g_lb = (1 + (r0c - pr)) * (1 - (c1c - pc))
        g_rt = (1 - (r1c - pr)) * (1 + (c0c - pc))
        g = torch.stack([g_lt, g_rb, g_lb, g_rt], 1).reshape(B, 4, h * w * n_taps, 1)
        val = g[:, 0] * taps[:, 0] + g[:, 1] * taps[:, 1] + g[:, 2] * taps[:, 2] + g[:, 3] * taps[:, 3]
        if self.modulation:
            m = torch.sigmoid(self.m_conv(x)).permute(0, 2, 3, 1).reshape(B, h * w * n_taps, 1)
            val = val * m
        # sum_{c,n} W[o,c,n] val[c,n] as one GEMM over (n, c)
        wgt = self.conv.weight.reshape(self.conv.out_channels, C, n_taps).permute(2, 1, 0)
        out = val.view(B, h * w, n_taps * C) @ wgt.reshape(n_taps * C, -1)   # [B, h w, O]
        out = out.view(B, h, w, -1).permute(0, 3, 1, 2)
        if self.conv.bias is not None:
            out = out + self.conv.bias.view(1, -1, 1, 1)
        return out.contiguous()


    def _forward_hip(self, x):
        """The same operator on the GPU: the sampling (with modulation) as one HIP kernel
        (aarmvs_deform_sample, forward and backward), the contraction with the weights as one
        GEMM over (tap, channel)."""
        from aarmvs import ops
        offset = self.p_conv(x)
        B, C, _, _ = x.shape
        h, w = offset.shape[2:]
        m = torch.sigmoid(self.m_conv(x)) if self.modulation else None
        val = ops.deform_sample(x.permute(0, 2, 3, 1).contiguous(), offset, m, self.stride, self.padding)
        wgt = self.conv.weight.reshape(self.conv.out_channels, C, 9).permute(2, 1, 0)
        out = val @ wgt.reshape(9 * C, -1)                                     # [B, h w, O]
        out = out.view(B, h, w, -1).permute(0, 3, 1, 2)
        if self.conv.bias is not None:
            out = out + self.conv.bias.view(1, -1, 1, 1)
        return out.contiguous()


def deformconvgnrelu(in_channels, out_channels, kernel_size=3, stride=1, dilation=1, bias=True,
                     group_channel=8):
    """models/module.py:238-243."""
    return nn.Sequential(
        DeformConv2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride, bias=bias),
        GroupNorm(_groups(out_channels, group_channel), out_channels),
        nn.ReLU(inplace=True),
    )


class ResnetBlockGn(nn.Module):
    """models/module.py:245-259: relu(stem(x) + x)."""

    def __init__(self, in_channels, kernel_size, dilation, bias, group_channel=8):
        super().__init__()
        self.stem = nn.Sequential(
            convgnrelu(in_channels, in_channels, kernel_size=kernel_size, stride=1,
                       dilation=dilation[0], bias=bias, group_channel=group_channel),
            nn.Conv2d(in_channels, in_channels, kernel_size=kernel_size, stride=1,
                      dilation=dilation[1], padding=((kernel_size - 1) // 2) * dilation[1],
                      bias=bias),
            GroupNorm(_groups(in_channels, group_channel), in_channels),
        )
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.relu(self.stem(x) + x)


def resnet_block_gn(in_channels, kernel_size=3, dilation=(1, 1), bias=True, group_channel=8):
    """models/module.py:261-262."""
    return ResnetBlockGn(in_channels, kernel_size, list(dilation), bias=bias,
                         group_channel=group_channel)


class deConvGnReLU(nn.Module):  # noqa: N801  (reference name)
    """models/module.py:264-287: ConvTranspose2d -> GroupNorm -> ReLU."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=2, padding=1, bias=True,
                 output_padding=1, group_channel=8):
        super().__init__()
        self.conv = nn.ConvTranspose2d(in_channels, out_channels, kernel_size=kernel_size,
                                       padding=padding, output_padding=output_padding,
                                       stride=stride, bias=bias)
        self.group_channel = group_channel
        self.gn = GroupNorm(_groups(out_channels, group_channel), out_channels)

    def forward(self, x):
        return F.relu(self.gn(self.conv(x)), inplace=True)
