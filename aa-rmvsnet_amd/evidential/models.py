"""Drop-in ``evidential.models`` (BuTTerK3ks/AA-RMVSNet, evidential/models.py): the
ELFNet-style evidential head that EMVSNet runs after the depth sweep, and its losses.

PyTorch-ROCm restatement (after the sweep, off the HIP hot path).  Names,
signatures, submodule attribute names (the 221 ``evidential.*`` state_dict keys) and
results follow the reference, including its shape limits, which are raised
here as explicit errors instead of failing deep inside a conv:

* the volume is read as ``input.unsqueeze(0)`` (evidential/models.py:380), so the batch
  becomes the channel axis of a 1-channel Conv3d: only B == 1 works;
* ``disparity_regression`` views depth_values as [1, D, 1, 1] against a probability
  volume resampled to ``maxdisp`` = 32 planes (:44-45, :245): only D == 32 works.

Reference quirks kept on purpose: the third pyramid level's softmax runs over the
size-1 channel axis (dim=1, :393), so that volume is all ones; BatchNorm layers use the
caller's train/eval mode.  Pinned by tests/golden/evidential.npz and e2e.npz (made by
running the reference, tests/golden/make_golden.py: gen_evidential, gen_e2e).
"""
from __future__ import annotations

# The drivers star-import this module (train.py:21) and so receive its module-level names,
# including these imports (no __all__, as in the reference)
import math  # noqa: F401

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.optim as optim  # noqa: F401
from torch import Tensor  # noqa: F401


class EvidentialShapeError(ValueError):
    """The reference head only runs at B == 1 and D == 32."""


def FMish(x):
    """mish(x) = x * tanh(softplus(x))  (evidential/models.py:26-37)."""
    return x * torch.tanh(F.softplus(x))


class Mish(nn.Module):
    """Module form of FMish (evidential/models.py:16-23)."""

    def forward(self, x):
        return FMish(x)


def convbn_3d(in_channels, out_channels, kernel_size, stride, pad):
    """Conv3d (no bias) + BatchNorm3d as a two-entry Sequential (keys ``.0`` / ``.1``),
    evidential/models.py:10-13."""
    conv = nn.Conv3d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                     padding=pad, bias=False)
    return nn.Sequential(conv, nn.BatchNorm3d(out_channels))


def _up(cin, cout):
    """ConvTranspose3d(k3, s2, p1, op1, no bias) + BatchNorm3d: doubles D, H and W."""
    return nn.Sequential(nn.ConvTranspose3d(cin, cout, 3, stride=2, padding=1, output_padding=1,
                                            bias=False),
                         nn.BatchNorm3d(cout))


def _cbm(cin, cout, stride=1):
    """convbn_3d(3x3x3, pad 1) followed by Mish."""
    return nn.Sequential(convbn_3d(cin, cout, 3, stride, 1), Mish())


def disparity_regression(x, depth_values, max_d=60):
    """sum_d prob_d * depth_d over dim 1 (evidential/models.py:40-45); depth_values [1, D]
    must hold as many hypotheses as x has planes."""
    if x.dim() != 4:
        raise EvidentialShapeError("disparity_regression expects a [B, D, H, W] volume")
    D = depth_values.shape[1]
    if x.shape[1] != D:
        raise EvidentialShapeError(
            f"evidential head: the probability volume is resampled to {x.shape[1]} planes but "
            f"depth_values holds {D} (the reference head works only for D == 32, SURVEY F2)")
    return (x * depth_values.reshape(1, D, 1, 1)).sum(dim=1)


def disparity_classification(x, depth_values):
    """WTA form (evidential/models.py:48-52): depth_values.take(argmax over dim 1)."""
    if x.dim() != 4:
        raise EvidentialShapeError("disparity_classification expects a [B, D, H, W] volume")
    return torch.take(depth_values, torch.argmax(x, dim=1))


class HourGlassUp(nn.Module):
    """Two-level encoder taking the coarser pyramid volumes as side inputs, then a two-step
    transposed-conv decoder with redirect skips (evidential/models.py:55-125)."""

    def __init__(self, in_channels):
        super().__init__()
        c = in_channels
        self.conv1 = nn.Conv3d(c, 2 * c, kernel_size=3, stride=2, padding=1, bias=False)
        self.conv2 = _cbm(2 * c, 2 * c)
        self.conv3 = nn.Conv3d(2 * c, 4 * c, kernel_size=3, stride=2, padding=1, bias=False)
        self.conv4 = _cbm(4 * c, 4 * c)
        self.conv8 = _up(4 * c, 2 * c)
        self.conv9 = _up(2 * c, c)
        self.combine1 = _cbm(3 * c, 2 * c)
        self.combine2 = _cbm(5 * c, 4 * c)
        self.redir1 = convbn_3d(c, c, kernel_size=1, stride=1, pad=0)
        self.redir2 = convbn_3d(2 * c, 2 * c, kernel_size=1, stride=1, pad=0)
        self.redir3 = convbn_3d(4 * c, 4 * c, kernel_size=1, stride=1, pad=0)

    def forward(self, x, feature4, feature5):
        half = self.conv2(self.combine1(torch.cat((self.conv1(x), feature4), dim=1)))      # 1/2
        quarter = self.conv4(self.combine2(torch.cat((self.conv3(half), feature5), dim=1)))  # 1/4
        y = FMish(self.redir3(quarter))
        y = FMish(self.conv8(y) + self.redir2(half))
        return FMish(self.conv9(y) + self.redir1(x))


class HourGlass(nn.Module):
    """Stacked-hourglass block: two stride-2 stages down, two transposed convs up with
    redirect skips (evidential/models.py:128-169)."""

    def __init__(self, in_channels):
        super().__init__()
        c = in_channels
        self.conv1 = _cbm(c, 2 * c, stride=2)
        self.conv2 = _cbm(2 * c, 2 * c)
        self.conv3 = _cbm(2 * c, 4 * c, stride=2)
        self.conv4 = _cbm(4 * c, 4 * c)
        self.conv5 = _up(4 * c, 2 * c)
        self.conv6 = _up(2 * c, c)
        self.redir1 = convbn_3d(c, c, kernel_size=1, stride=1, pad=0)
        self.redir2 = convbn_3d(2 * c, 2 * c, kernel_size=1, stride=1, pad=0)

    def forward(self, x):
        half = self.conv2(self.conv1(x))
        quarter = self.conv4(self.conv3(half))
        y = FMish(self.conv5(quarter) + self.redir2(half))
        return FMish(self.conv6(y) + self.redir1(x))


def _head(c):
    """convbn + Mish + Conv3d(c -> 4): per-plane logits of (cost, log nu, log alpha, log beta)."""
    return nn.Sequential(convbn_3d(c, c, 3, 1, 1), Mish(),
                         nn.Conv3d(c, 4, kernel_size=3, padding=1, stride=1, bias=False))


class EvidentialModule(nn.Module):
    """Evidential depth head (evidential/models.py:183-459).

    forward(prob_volume [1, D, H, W], depth_values [1, D]) -> (evidential [4, H, W] =
    (gamma, nu, alpha, beta) of the NIG mixture, prob_combine [1, 32, H, W]).
    """

    def __init__(self, depth):
        super().__init__()
        self.maxdisp = 32
        c = 32
        self.dres0 = nn.Sequential(convbn_3d(1, c, 3, 1, 1), Mish(), convbn_3d(c, c, 3, 1, 1), Mish())
        self.dres1 = nn.Sequential(convbn_3d(c, c, 3, 1, 1), Mish(), convbn_3d(c, c, 3, 1, 1), Mish())
        self.conv_vol2 = nn.Sequential(convbn_3d(1, c, 3, 1, 1), Mish(), convbn_3d(c, c, 3, 1, 1))
        self.conv_vol3 = nn.Sequential(convbn_3d(1, c, 3, 1, 1), Mish(), convbn_3d(c, c, 3, 1, 1))
        self.combine1 = HourGlassUp(c)
        self.dres2 = HourGlass(c)
        self.dres3 = HourGlass(c)
        self.classif0 = _head(c)
        self.classif1 = _head(c)
        self.classif2 = _head(c)

    # evidence and the normal-inverse-gamma mixture (evidential/models.py:281-307)
    def evidence(self, x):
        return F.softplus(x)

    def get_uncertainty(self, logv, logalpha, logbeta):
        return self.evidence(logv), self.evidence(logalpha) + 1, self.evidence(logbeta)

    def moe_nig(self, u1, la1, alpha1, beta1, u2, la2, alpha2, beta2):
        la = la1 + la2
        u = (la1 * u1 + u2 * la2) / la
        alpha = alpha1 + alpha2 + 0.5
        beta = beta1 + beta2 + 0.5 * (la1 * (u1 - u) ** 2 + la2 * (u2 - u) ** 2)
        return u, la, alpha, beta

    def combine_uncertainty(self, ests):
        acc = tuple(ests[0])
        for e in ests[1:]:
            acc = self.moe_nig(*acc, *e)
        return acc

    def _pyramid(self, x, D, H, W, dim):
        v = F.interpolate(x, [D, H, W], mode="trilinear", align_corners=True)
        return F.softmax(v, dim=dim)

    def forward(self, input, depth_value):
        if input.dim() != 4 or input.shape[0] != 1:
            raise EvidentialShapeError(
                f"evidential head: needs a [1, D, H, W] probability volume, got "
                f"{tuple(input.shape)} (the reference reads the batch as Conv3d channels, "
                "evidential/models.py:380: B == 1 only, SURVEY F2)")
        if depth_value.dim() != 2 or depth_value.shape[1] != self.maxdisp:
            raise EvidentialShapeError(
                f"evidential head: depth_values must be [1, {self.maxdisp}], got "
                f"{tuple(depth_value.shape)} (disparity_regression against maxdisp = 32 planes, "
                "evidential/models.py:44-45, 245: D == 32 only, SURVEY F2)")
        H, W = input.shape[2], input.shape[3]
        x = input.unsqueeze(0)                     # [1, B=1, D, H, W]
        md = self.maxdisp
        vol1 = self._pyramid(x, md, H, W, dim=2)
        vol2 = self._pyramid(x, md // 2, H // 2, W // 2, dim=2)
        vol3 = self._pyramid(x, md // 4, H // 4, W // 4, dim=1)   # reference: dim=1 (size 1)

        cost0 = self.dres0(vol1)
        cost0 = self.dres1(cost0) + cost0
        mid = self.combine1(cost0, self.conv_vol2(vol2), self.conv_vol3(vol3))
        out1 = self.dres2(mid)
        out2 = self.dres3(out1)

        outs = [head(feat) for head, feat in ((self.classif0, cost0), (self.classif1, out1),
                                              (self.classif2, out2))]
        if input.is_cuda:
            # the epilogue (softmax, disparity_regression, softplus evidence, moe_nig, mean) as
            # one HIP kernel (aarmvs_evidential_epilogue); the heads are at [md, H, W] already,
            # where get_pred / get_logits' align_corners=True resampling is the identity
            if any(tuple(o.shape[2:]) != (md, H, W) for o in outs):
                raise EvidentialShapeError(f"evidential head: classifier outputs "
                                           f"{[tuple(o.shape) for o in outs]} are not at [{md}, {H}, {W}]")
            from aarmvs import ops as _ops
            return _ops.evidential_epilogue(*outs, depth_value)

        def upsample(t):
            return F.interpolate(t, [md, H, W], mode="trilinear", align_corners=True).squeeze(1)

        ests, probs = [], []
        for o in outs:
            cost, logla, logalpha, logbeta = torch.split(o, 1, dim=1)
            prob = F.softmax(upsample(cost), dim=1)
            pred = disparity_regression(prob, depth_value)
            # logits of the evidential parameters, weighted by this level's probabilities
            la, alpha, beta = self.get_uncertainty(*((upsample(t) * prob).sum(dim=1)
                                                     for t in (logla, logalpha, logbeta)))
            ests.append((pred, la, alpha, beta))
            probs.append(prob)
        u, la, alpha, beta = self.combine_uncertainty(ests)
        evidential = torch.cat((u, la, alpha, beta))
        prob_combine = torch.stack(probs).mean(dim=0)
        return evidential, prob_combine


class EvidentialWrapper(nn.Module):
    """evidential/models.py:172-180: the head on a random [1, 32] depth vector (an export
    helper of the reference's analysis scripts)."""

    def __init__(self):
        super().__init__()
        self.original_model = EvidentialModule(depth=32)

    def forward(self, x):
        dv = torch.randn(1, 32, device=x.device)
        return self.original_model(x, dv)


def criterion_uncertainty(u, la, alpha, beta, y, mask, weight_reg=0.1):
    """NIG negative log-likelihood + evidence regulariser over masked pixels
    (evidential/models.py:462-477)."""
    m = mask.bool()
    n = m.sum()
    om = 2 * beta * (1 + la)
    nll = (0.5 * torch.log(np.pi / la) - alpha * torch.log(om)
           + (alpha + 0.5) * torch.log(la * (u - y) ** 2 + om)
           + torch.lgamma(alpha) - torch.lgamma(alpha + 0.5))
    reg = torch.abs(u - y) * (2 * la + alpha)
    return nll[m].sum() / n + weight_reg * reg[m].sum() / n


def loss_emvsnet(u, la, alpha, beta, y, mask, weight_reg=0.1):
    """log(var) + (1 + weight_reg nu) err^2 / var with var = beta / nu, masked mean
    (evidential/models.py:496-504)."""
    m = mask.bool()
    var = beta / la
    per_px = torch.log(var) + (1.0 + weight_reg * la) * (u - y) ** 2 / var
    return per_px[m].sum() / m.sum()


def compute_uncertainty(self, u, la, alpha, beta):
    """(aleatoric, epistemic) = (beta / (alpha - 1), beta / (alpha - 1) / nu); module-level
    with a leading ``self`` exactly as the reference defines it (:511-514)."""
    aleatoric = beta / (alpha - 1)
    return aleatoric, aleatoric / la


def loss_der(outputs, depth_gt, mask, depth_value, coeff=0.01):
    """The loss train.py:304 calls (the second definition of evidential/models.py, :517-558,
    which shadows the first): loss_emvsnet on the head's (gamma, nu, alpha, beta), plus the
    uncertainty maps.  Returns (loss, gamma [1, H, W], dict of [1, H, W] maps)."""
    ev = outputs["evidential_prediction"]
    if ev is None:
        raise EvidentialShapeError("loss_der: the model produced no evidential prediction")
    gamma, nu, alpha, beta = (ev[i].unsqueeze(0) for i in range(4))
    loss = loss_emvsnet(gamma, nu, alpha, beta, depth_gt, mask, weight_reg=0.1)
    aleatoric_2 = beta / (alpha - 1)
    evidential = {
        "gamma": gamma,
        "nu": nu,
        "alpha": alpha,
        "beta": beta,
        "aleatoric_1": torch.sqrt(beta * (nu + 1) / nu / alpha),   # "unreasonably effective DER"
        "epistemic_1": 1.0 / torch.sqrt(nu),
        "aleatoric_2": aleatoric_2,                                 # classic NIG moments
        "epistemic_2": beta / (alpha - 1) / nu,
        "total": aleatoric_2,
    }
    return loss, gamma, evidential

