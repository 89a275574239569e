"""FeatNet's deformable convolution on the GPU (aarmvs_deform_sample, the reference's
models/module.py:105-236): the HIP sampling kernel's output equals the PyTorch expression of the
same samples bit for bit (fp32, every operation one rounding in the reference's order); the
whole DeformConv2d forward and every gradient (input, offset conv, modulation conv, weights,
bias) match float64 autograd of that expression on the CPU within max(2e-5, 3x float32 CPU
autograd's error); the kernel is what runs."""
import copy

import pytest
import torch

from test_deform_conv import planar_forward, planar_val, random_deform

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [(2, 9, 11, 1, 0.5), (1, 12, 10, 1, 3.0), (1, 13, 9, 2, 1.5), (1, 64, 80, 1, 2.0)]


@pytest.mark.parametrize("B,H,W,stride,scale", CASES)
def test_samples_bit_equal_to_the_pytorch_expression(B, H, W, stride, scale):
    """val from the same x, offsets and mask: bit-identical to planar_val on the CPU."""
    from aarmvs import ops
    torch.manual_seed(1)
    x = torch.randn(B, 32, H, W)
    h, w = (H - 1) // stride + 1, (W - 1) // stride + 1
    off = torch.randn(B, 18, h, w) * scale
    off[:, :, 0, 0] = 0.0                        # integer positions (corner weights 1 / 0)
    off[:, :, -1, -1] = float(max(H, W))         # far outside: clamped to the border
    m = torch.rand(B, 9, h, w)
    ref = planar_val(x, off, m, stride, 1)        # [B, C, h, w, n]
    with torch.no_grad():
        val = ops.deform_sample(x.to(DEV).permute(0, 2, 3, 1).contiguous(), off.to(DEV), m.to(DEV),
                                stride, 1)
    got = val.cpu().view(B, h, w, 9, 32).permute(0, 4, 1, 2, 3)
    assert torch.equal(got, ref)
    ref_u = planar_val(x, off, None, stride, 1)
    with torch.no_grad():
        val_u = ops.deform_sample(x.to(DEV).permute(0, 2, 3, 1).contiguous(), off.to(DEV), None,
                                  stride, 1)
    assert torch.equal(val_u.cpu().view(B, h, w, 9, 32).permute(0, 4, 1, 2, 3), ref_u)


@pytest.mark.parametrize("B,H,W,stride,scale", CASES)
def test_deform_conv_forward_backward_match_float64(B, H, W, stride, scale):
    from aarmvs import ops
    mod = random_deform(32, stride, scale, dtype=torch.float32)
    x = torch.randn(B, 32, H, W)
    gy = None
    res = {}
    for name, dev, dt in (("ref", "cpu", torch.float64), ("f32", "cpu", torch.float32),
                          ("hip", DEV, torch.float32)):
        md = copy.deepcopy(mod).to(dev, dt)
        xx = x.detach().to(dev, dt).clone().requires_grad_(True)
        if name == "hip":
            ops.profile_enable(True)
            ops.profile_reset()
        try:
            y = planar_forward(md, xx) if name != "hip" else md(xx)
            if gy is None:
                gy = torch.linspace(-1, 1, y.numel(), dtype=torch.float64).view_as(y)
            (y * gy.to(dev, dt)).sum().backward()
            if name == "hip":
                torch.cuda.synchronize()
                assert ops.profile_read()["deform_sample"][0] == 2   # forward + backward kernels
        finally:
            if name == "hip":
                ops.profile_enable(False)
        res[name] = [y.detach()] + [xx.grad] + [p.grad for p in md.parameters()]
    # bound: relative L2 error <= max(2e-5, 3 x float32 CPU autograd's own error): the weight
    # gradient is a cancelling sum over the pixels (gy spans -1..1), whose float32 error the
    # summation order sets
    names = ["out", "x"] + [n for n, _ in mod.named_parameters()]
    for nm, r, f, g in zip(names, res["ref"], res["f32"], res["hip"]):
        rel = lambda t: float((t.double().cpu() - r).norm() / r.norm().clamp_min(1e-30))  # noqa: E731
        err, e32 = rel(g), rel(f)
        assert err <= max(2e-5, 3 * e32), f"{nm}: relative L2 error {err:.3g} (float32 CPU {e32:.3g})"
