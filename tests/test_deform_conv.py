"""DeformConv2d (models/module.py, the reference's models/module.py:105-236): the channels-last
one-gather formulation against the per-corner, per-channel-plane restatement it replaced
(round 4's, which test_models_api.py::test_featnet_matches_reference pinned to the reference's
features) -- forward and every gradient (input, offsets' conv, modulation conv, weights, bias),
in float64 on the CPU, with offsets large enough to push taps off the padded image."""
import pytest
import torch

from models.module import DeformConv2d


def planar_val(x, offset, mask, stride, padding, ks=3):
    """The previous formulation's samples: four gathers of [B, C, h*w*n] planes of the
    zero-padded x at the offset positions, times the modulation mask (None: none) ->
    [B, C, h, w, n]."""
    n_taps = ks * ks
    B, _, h, w = offset.shape
    xp = torch.nn.functional.pad(x, (padding,) * 4) if padding else x
    Hp, Wp = xp.shape[2], xp.shape[3]
    dt, dev = offset.dtype, offset.device
    a = torch.arange(n_taps, device=dev) // ks - (ks - 1) // 2
    b = torch.arange(n_taps, device=dev) % ks - (ks - 1) // 2
    rows = torch.arange(1, h * stride + 1, stride, device=dev)
    cols = torch.arange(1, w * stride + 1, stride, device=dev)
    pr = (rows.view(1, 1, h, 1) + a.view(1, n_taps, 1, 1)).to(dt) + offset[:, :n_taps]
    pc = (cols.view(1, 1, 1, w) + b.view(1, n_taps, 1, 1)).to(dt) + offset[:, n_taps:]
    pr, pc = pr.permute(0, 2, 3, 1), pc.permute(0, 2, 3, 1)
    r0, c0 = pr.detach().floor(), pc.detach().floor()
    r0c, r1c = r0.clamp(0, Hp - 1), (r0 + 1).clamp(0, Hp - 1)
    c0c, c1c = c0.clamp(0, Wp - 1), (c0 + 1).clamp(0, Wp - 1)
    pr, pc = pr.clamp(0, Hp - 1), pc.clamp(0, Wp - 1)
    flat = xp.reshape(B, xp.shape[1], Hp * Wp)

    def tap(ri, ci):
        idx = (ri.long() * Wp + ci.long()).reshape(B, 1, -1).expand(-1, flat.shape[1], -1)
        return flat.gather(2, idx).view(B, flat.shape[1], h, w, n_taps)

    g_lt = (1 + (r0c - pr)) * (1 + (c0c - pc))
    g_rb = (1 - (r1c - pr)) * (1 - (c1c - pc))
    g_lb = (1 + (r0c - pr)) * (1 - (c1c - pc))
    g_rt = (1 - (r1c - pr)) * (1 + (c0c - pc))
    val = (g_lt.unsqueeze(1) * tap(r0c, c0c) + g_rb.unsqueeze(1) * tap(r1c, c1c)
           + g_lb.unsqueeze(1) * tap(r0c, c1c) + g_rt.unsqueeze(1) * tap(r1c, c0c))
    if mask is not None:
        val = val * mask.permute(0, 2, 3, 1).unsqueeze(1)
    return val


def planar_forward(mod, x, want_val=False):
    """The previous DeformConv2d formulation: planar_val, then einsum over (c, n).
    want_val: also return the modulated samples [B, C, h, w, n]."""
    offset = mod.p_conv(x)
    mask = torch.sigmoid(mod.m_conv(x)) if mod.modulation else None
    val = planar_val(x, offset, mask, mod.stride, mod.padding, mod.kernel_size)
    wgt = mod.conv.weight.reshape(mod.conv.out_channels, -1, mod.kernel_size ** 2)
    out = torch.einsum("bchwn,ocn->bohw", val, wgt)
    if mod.conv.bias is not None:
        out = out + mod.conv.bias.view(1, -1, 1, 1)
    return (out, val) if want_val else out


def random_deform(C, stride, scale, dtype=torch.float64, seed=0):
    """A DeformConv2d with every weight random (the reference zero-inits the offset and
    modulation convs; trained ones are not), offsets of size ~scale pixels."""
    torch.manual_seed(seed)
    mod = DeformConv2d(C, C, kernel_size=3, padding=1, stride=stride, bias=True).to(dtype)
    with torch.no_grad():
        for p in mod.parameters():
            p.copy_(torch.randn_like(p) * (scale if p is mod.p_conv.weight else 0.3))
    return mod


@pytest.mark.parametrize("B,C,H,W,stride,scale", [(2, 8, 9, 11, 1, 0.5), (1, 32, 12, 10, 1, 3.0),
                                                 (1, 4, 13, 9, 2, 1.5)])
def test_deform_conv_matches_planar_restatement(B, C, H, W, stride, scale):
    mod = random_deform(C, stride, scale)
    x = torch.randn(B, C, H, W, dtype=torch.float64)
    outs, grads = [], []
    for f in (lambda xx: mod(xx), lambda xx: planar_forward(mod, xx)):
        xx = x.clone().requires_grad_(True)
        mod.zero_grad()
        y = f(xx)
        gy = torch.linspace(-1, 1, y.numel(), dtype=torch.float64).view_as(y)
        (y * gy).sum().backward()
        outs.append(y.detach())
        grads.append([xx.grad.clone()] + [p.grad.clone() for p in mod.parameters()])
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-12, atol=1e-12)
    for g0, g1 in zip(*grads):
        torch.testing.assert_close(g0, g1, rtol=1e-10, atol=1e-10)
