"""The evidential head's epilogue on HIP (SURVEY §8f-3 "then fuse its softmax, regression, and
NIG combine"; aarmvs_evidential_epilogue, csrc/evidential.hip): softmax over each classifier's
plane axis, disparity_regression, the softplus evidence and moe_nig (evidential/models.py:40-45,
281-304, 385-459) in one kernel, forward and backward.

* the whole head on the GPU (the convs in PyTorch/MIOpen, the epilogue on HIP) against the
  reference's outputs in evidential.npz (eval and train mode), at test_evidential.py's
  tolerance (1e-4 of each output's scale);
* the kernel alone against a float64 restatement of the reference's expressions (forward) and
  its float64 autograd (backward), on random classifier outputs with logits past softplus's
  threshold (20) and costs spread over +-30: 2e-6 of each output's scale (fp32 exp / log1p and
  D = 32 term sums);
* the kernel is the path that runs (profiling counter), and loss_der's gradients through the
  head match CPU autograd of the PyTorch head.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN
from aarmvs import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def close(a, b, rel):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    np.testing.assert_allclose(a, b, atol=rel * max(np.abs(b).max(), 1e-30), rtol=0)


def _head(wseed):
    from models import EMVSNet
    m = EMVSNet(32, image_scale=1.0, max_h=32, max_w=40)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    wts = syn.init_weights(shapes, seed=wseed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in wts.items()}, strict=True)
    return m.evidential


def test_head_on_gpu_matches_reference():
    from aarmvs import ops
    g = np.load(os.path.join(GOLDEN, "evidential.npz"), allow_pickle=False)
    h = _head(int(g["wseed"])).to(DEV)
    prob = torch.softmax(torch.from_numpy(g["logits"]), dim=1).to(DEV)
    dv = torch.from_numpy(g["depth_values"]).to(DEV)
    ops.profile_enable(True)
    ops.profile_reset()
    try:
        with torch.no_grad():
            h.eval()
            ev, comb = h(prob, dv)
            close(ev.cpu(), g["ev_eval"], 1e-4)
            close(comb.cpu(), g["comb_eval"], 1e-4)
            h.train()
            ev, comb = h(prob, dv)
            close(ev.cpu(), g["ev_train"], 1e-4)
            close(comb.cpu(), g["comb_train"], 1e-4)
        torch.cuda.synchronize()
        assert ops.profile_read()["evidential"][0] == 2
    finally:
        ops.profile_enable(False)


def _epilogue64(heads, dv):
    """float64 restatement of evidential/models.py:421-459 on [1,4,D,H,W] classifier outputs."""
    ests, probs = [], []
    sp = lambda x: F.softplus(x)   # noqa: E731
    for o in heads:
        cost, la, al, be = (o[:, i] for i in range(4))
        p = F.softmax(cost, dim=1)
        pred = (p * dv.view(1, -1, 1, 1)).sum(1)
        ests.append((pred, sp((la * p).sum(1)), sp((al * p).sum(1)) + 1, sp((be * p).sum(1))))
        probs.append(p)

    def moe(a, b):
        u1, la1, al1, be1 = a
        u2, la2, al2, be2 = b
        la = la1 + la2
        u = (la1 * u1 + u2 * la2) / la
        return u, la, al1 + al2 + 0.5, be1 + be2 + 0.5 * (la1 * (u1 - u) ** 2 + la2 * (u2 - u) ** 2)
    r = moe(moe(ests[0], ests[1]), ests[2])
    return torch.cat(r), torch.stack(probs).mean(0)


def _random_heads(H, W, seed):
    g = torch.Generator().manual_seed(seed)
    hs = []
    for i in range(3):
        t = torch.randn(1, 4, 32, H, W, generator=g, dtype=torch.float64)
        t[:, 0] *= 10.0                       # costs spread over ~+-30
        t[:, 1:] *= 4.0
        t[:, 1:, :, :4] += 25.0               # a band of logits past softplus's threshold (20)
        hs.append(t)
    return hs


def test_epilogue_kernel_forward_and_backward_match_float64():
    from aarmvs import ops
    H, W = 37, 53                             # HW not a multiple of the block
    hs64 = _random_heads(H, W, 7)
    dv64 = torch.from_numpy(syn.depth_hypotheses(32)).double()
    hs = [h.float().to(DEV).requires_grad_(True) for h in hs64]
    ev, pc = ops.evidential_epilogue(*hs, dv64.float().to(DEV))
    hr = [h.clone().requires_grad_(True) for h in hs64]
    ev64, pc64 = _epilogue64(hr, dv64)
    for i in range(4):
        close(ev[i].detach().cpu(), ev64[i].detach(), 2e-6)
    close(pc.detach().cpu(), pc64.detach(), 2e-6)
    gen = torch.Generator().manual_seed(3)
    g_ev = torch.randn(4, H, W, generator=gen, dtype=torch.float64)
    g_pc = torch.randn(1, 32, H, W, generator=gen, dtype=torch.float64)
    torch.autograd.backward([ev, pc], [g_ev.float().to(DEV), g_pc.float().to(DEV)])
    torch.autograd.backward([ev64, pc64], [g_ev, g_pc])
    for a, b in zip(hs, hr):
        for c in range(4):   # per channel: the cost channel carries the softmax backward
            close(a.grad[:, c].cpu(), b.grad[:, c], 2e-5)
    # only one of the two outputs used: the other's gradient is zero
    for h in hs:
        h.grad = None
    ev, pc = ops.evidential_epilogue(*hs, dv64.float().to(DEV))
    ev.sum().backward()
    hr = [h.clone().requires_grad_(True) for h in hs64]
    ev64, _ = _epilogue64(hr, dv64)
    ev64.sum().backward()
    for a, b in zip(hs, hr):
        close(a.grad.cpu(), b.grad, 2e-5)


def test_loss_der_gradients_through_the_head_match_cpu():
    """train.py's evidential loss (loss_der, :517-558) backpropagated through the head: GPU
    (HIP epilogue) against CPU autograd of the PyTorch head, every head parameter and the
    probability volume."""
    from evidential.models import loss_der
    g = np.load(os.path.join(GOLDEN, "evidential.npz"), allow_pickle=False)
    res = {}
    for dev in ("cpu", DEV):
        h = _head(int(g["wseed"])).to(dev).train()
        logits = torch.from_numpy(g["logits"]).to(dev).requires_grad_(True)
        prob = torch.softmax(logits, dim=1)
        dv = torch.from_numpy(g["depth_values"]).to(dev)
        ev, _ = h(prob, dv)
        loss, _, _ = loss_der({"probability_volume": prob, "evidential_prediction": ev},
                              torch.from_numpy(g["depth_gt"]).to(dev), torch.from_numpy(g["mask"]).to(dev), dv)
        loss.backward()
        res[dev] = (float(loss), logits.grad.cpu().double(),
                    {k: p.grad.cpu().double() for k, p in h.named_parameters() if p.grad is not None})
    assert abs(res[DEV][0] - res["cpu"][0]) <= 1e-5 * abs(res["cpu"][0])
    close(res[DEV][1], res["cpu"][1], 1e-3)
    assert res[DEV][2].keys() == res["cpu"][2].keys() and len(res["cpu"][2]) > 0
    for k in res["cpu"][2]:
        close(res[DEV][2][k], res["cpu"][2][k], 1e-3)
