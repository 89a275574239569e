"""HIP GroupNorm (aarmvs_group_norm_forward/_backward, behind models.module.GroupNorm on the
GPU) against torch's F.group_norm autograd in fp32 on the same device: outputs, input and
parameter gradients, ragged and full-resolution planes, affine and not, and run-to-run
bit identity (fixed-order reductions)."""
import pytest
import torch
import torch.nn.functional as F

from aarmvs import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("B,C,H,W,G,affine", [
    (2, 16, 37, 53, 2, True),      # deConvGnReLU's GroupNorm(2, 16), ragged plane
    (1, 4, 512, 640, 1, True),     # omega's GroupNorm(1, 4) at config 4's frame
    (1, 32, 100, 120, 4, True),    # FeatNet's GroupNorm(4, 32)
    (3, 8, 9, 11, 1, False),
])
def test_group_norm_matches_torch(B, C, H, W, G, affine):
    g = torch.Generator(device="cpu").manual_seed(B * 1000 + C)
    x = (torch.randn(B, C, H, W, generator=g) * 3 + 0.5).to(DEV)
    w = (torch.randn(C, generator=g) * 0.5 + 1).to(DEV) if affine else None
    b = (torch.randn(C, generator=g) * 0.1).to(DEV) if affine else None
    gy = torch.randn(B, C, H, W, generator=g).to(DEV)
    leaves = [t.clone().requires_grad_(True) if t is not None else None for t in (x, w, b)]
    ref = F.group_norm(leaves[0], G, leaves[1], leaves[2], 1e-5)
    ref.backward(gy)
    hl = [t.clone().requires_grad_(True) if t is not None else None for t in (x, w, b)]
    out = ops.group_norm(hl[0], G, hl[1], hl[2], 1e-5)
    out.backward(gy)
    torch.cuda.synchronize()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(hl[0].grad, leaves[0].grad, rtol=1e-4, atol=1e-4)
    if affine:
        for a, r in zip(hl[1:], leaves[1:]):
            assert float((a.grad - r.grad).norm() / r.grad.norm()) < 1e-4
    # fixed-order reductions: bit-identical on a second run
    x2 = x.clone().requires_grad_(True)
    out2 = ops.group_norm(x2, G, w, b, 1e-5)
    out2.backward(gy)
    assert torch.equal(out2, out.detach()) and torch.equal(x2.grad, hl[0].grad)


def test_module_uses_the_hip_kernels_on_the_gpu():
    from models.module import GroupNorm
    m = GroupNorm(2, 16).to(DEV)
    x = torch.randn(1, 16, 24, 32, device=DEV, requires_grad=True)
    y = m(x)
    assert y.grad_fn is not None and "GroupNormHip" in type(y.grad_fn).__name__
    torch.testing.assert_close(y, F.group_norm(x, 2, m.weight, m.bias, m.eps), rtol=1e-5, atol=2e-5)
