"""HIP ConvLSTMCell gate math (aarmvs_lstm_gates_forward/_backward, behind
models.module.ConvLSTMCell on the GPU: the BPTT recompute) against the module.py:83-90
formula under torch autograd in fp32 on the same device."""
import pytest
import torch

from aarmvs import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _torch_gates(z, c, hid):
    zi, zf, zo, zg = torch.split(z, hid, dim=1)
    cn = torch.sigmoid(zf) * c + torch.sigmoid(zi) * torch.tanh(zg)
    return torch.sigmoid(zo) * torch.tanh(cn), cn


@pytest.mark.parametrize("B,hid,H,W", [(1, 16, 64, 80), (2, 8, 37, 53)])
def test_lstm_gates_match_torch(B, hid, H, W):
    g = torch.Generator(device="cpu").manual_seed(hid * 100 + B)
    z = (torch.randn(B, 4 * hid, H, W, generator=g) * 2).to(DEV)
    c = torch.randn(B, hid, H, W, generator=g).to(DEV)
    dh = torch.randn(B, hid, H, W, generator=g).to(DEV)
    dc = torch.randn(B, hid, H, W, generator=g).to(DEV)
    zr, cr = z.clone().requires_grad_(True), c.clone().requires_grad_(True)
    hr, cnr = _torch_gates(zr, cr, hid)
    torch.autograd.backward([hr, cnr], [dh, dc])
    zh, ch = z.clone().requires_grad_(True), c.clone().requires_grad_(True)
    h, cn = ops.lstm_gates(zh, ch)
    torch.autograd.backward([h, cn], [dh, dc])
    torch.cuda.synchronize()
    for a, b in ((h, hr), (cn, cnr), (zh.grad, zr.grad), (ch.grad, cr.grad)):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # h alone (no gradient into c): the dc = None path
    zh2 = z.clone().requires_grad_(True)
    h2, _ = ops.lstm_gates(zh2, c)
    h2.backward(dh)
    zr2 = z.clone().requires_grad_(True)
    _torch_gates(zr2, c, hid)[0].backward(dh)
    torch.testing.assert_close(zh2.grad, zr2.grad, rtol=1e-5, atol=1e-6)


def test_cell_module_uses_the_hip_gates():
    from models.module import ConvLSTMCell
    cell = ConvLSTMCell((24, 32), 16, 8, (3, 3), True).to(DEV)
    x = torch.randn(1, 16, 24, 32, device=DEV)
    h0 = torch.randn(1, 8, 24, 32, device=DEV)
    c0 = torch.randn(1, 8, 24, 32, device=DEV)
    h, c = cell(x, (h0, c0))
    assert "LstmGatesHip" in type(h.grad_fn).__name__
    z = cell.conv(torch.cat([x, h0], 1))
    hr, cr = _torch_gates(z, c0, 8)
    torch.testing.assert_close(h, hr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(c, cr, rtol=1e-5, atol=1e-6)
