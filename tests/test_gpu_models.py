"""GPU tests of the drop-in ``models`` API (EMVSNet / homo_warping_depthwise) on libaarmvs:
end-to-end against fixtures made by running the reference, the reference's real
checkpoint weights, and the training backward against CPU autograd of the oracle.

Tolerances: depth <= 1e-3 relative L1 (north_star), confidences/probabilities 1e-4/1e-5
abs, gradients 1e-4 relative to the gradient's max magnitude (fp32 atomics and
reassociation in the backward).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import GOLDEN
from aarmvs import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda"


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def close(a, b, rel=1e-4):
    """within rel x the reference output's largest magnitude (the 3D hourglass in fp32)"""
    np.testing.assert_allclose(a, b, atol=rel * max(np.abs(b).max(), 1e-30), rtol=0)


def rel_l1(a, b):
    return float(np.abs(a - b).sum() / max(np.abs(b).sum(), 1e-30))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")


def _model(D, H, W, wseed, return_depth, identity_feature=True):
    from models import EMVSNet
    m = EMVSNet(disparity_level=D, image_scale=1.0, max_h=H, max_w=W, return_depth=return_depth)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    wts = syn.init_weights(shapes, seed=wseed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in wts.items()}, strict=True)
    if identity_feature:
        m.feature = nn.Identity()
    return m.to(DEV)


def test_emvsnet_end_to_end_with_featnet():
    """Full EMVSNet.forward (FeatNet in PyTorch + HIP sweep) vs the reference (e2e.npz)."""
    g = load("e2e.npz")
    B, N, H, W, D = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]), images=True)
    m = _model(D, H, W, int(g["wseed"]), True, identity_feature=False).eval()
    imgs = torch.from_numpy(sc["imgs"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"]).to(DEV)
    dv = torch.from_numpy(sc["depth_values"]).to(DEV)
    with torch.no_grad():
        out = m(imgs, proj, dv)
        assert rel_l1(out["depth"].cpu().numpy(), g["depth"]) <= 1e-3
        np.testing.assert_allclose(out["photometric_confidence"].cpu().numpy(), g["conf"], atol=1e-4)
        # the evidential head on the softmax of the HIP cost volume
        close(out["evidential_prediction"].cpu().numpy(), g["evidential_eval"])
        m.return_depth = False
        prob, ev, comb = m(imgs, proj, dv)
        np.testing.assert_allclose(prob.cpu().numpy(), g["prob"], atol=1e-4)
        close(ev.cpu().numpy(), g["evidential"])
        close(comb.cpu().numpy(), g["prob_combine"])
        m.train()   # BatchNorm batch statistics, as the reference's training step
        prob_t, ev_t, _ = m(imgs, proj, dv)
    np.testing.assert_allclose(prob_t.cpu().numpy(), g["prob_train"], atol=1e-4)
    close(ev_t.cpu().numpy(), g["evidential_train"])
    # loss_der (train.py:297-304) runs on the drop-in's outputs
    from evidential.models import loss_der
    loss, gamma, evd = loss_der({"probability_volume": prob_t, "evidential_prediction": ev_t},
                                torch.from_numpy(g["depth_gt"]).to(DEV),
                                torch.from_numpy(g["mask"]).to(DEV), dv)
    assert torch.isfinite(loss) and gamma.shape == (1, H, W)


def test_emvsnet_real_checkpoint_weights():
    """Eval + train-mode sweep with the reference's model_dtu_v2 weights (real_weights_sweep.npz)."""
    g = load("real_weights_sweep.npz")
    B, N, H, W, D = (int(x) for x in g["shape"])
    from models import EMVSNet
    m = EMVSNet(disparity_level=D, image_scale=1.0, max_h=H, max_w=W, return_depth=True)
    sd = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w:")}
    missing = m.load_state_dict(sd, strict=False).missing_keys
    assert all(k.startswith(("feature.", "evidential.")) for k in missing)
    m.feature = nn.Identity()
    m = m.to(DEV).eval()
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]))
    assert syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]) == str(g["digest"])
    imgs = torch.from_numpy(np.moveaxis(sc["features"], 0, 1).copy()).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"]).to(DEV)
    dv = torch.from_numpy(sc["depth_values"]).to(DEV)
    with torch.no_grad():
        out = m(imgs, proj, dv)
        m.return_depth = False
        prob, _, _ = m(imgs, proj, dv)
    assert rel_l1(out["depth"].cpu().numpy(), g["depth"]) <= 1e-3
    np.testing.assert_allclose(out["photometric_confidence"].cpu().numpy(), g["conf"], atol=1e-4)
    np.testing.assert_allclose(prob.cpu().numpy()[:, :, ::4, ::4], g["prob_sub"], atol=1e-5)


def test_homo_warping_depthwise_forward_backward():
    """models.homo_warping_depthwise (HIP) vs the warp fixture and CPU autograd of the oracle."""
    from models import homo_warping_depthwise
    from oracle import sweep_oracle as orc
    g = load("warp.npz")
    B, N, H, W, C = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D=4, seed=int(g["seed"]), C=C)
    proj = torch.from_numpy(sc["proj_matrices"])
    src = torch.from_numpy(sc["features"][1]).to(DEV).requires_grad_(True)
    dep = torch.from_numpy(g["depths"][:, 1])
    out = homo_warping_depthwise(src, proj[:, 1].to(DEV), proj[:, 0].to(DEV), dep.to(DEV))
    np.testing.assert_allclose(out.detach().cpu().numpy(), g["out"][0, 1], atol=1e-4)
    gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(0))
    out.backward(gout.to(DEV))
    src_c = torch.from_numpy(sc["features"][1]).requires_grad_(True)
    rel = orc.relative_projection(proj[:, 1], proj[:, 0])
    orc.homo_warp(src_c, rel, dep).backward(gout)
    ref_g = src_c.grad.numpy()
    np.testing.assert_allclose(src.grad.cpu().numpy(), ref_g, atol=1e-4 * np.abs(ref_g).max())
    # the scatter is summed in fixed point: a second backward is bit-identical
    g1 = src.grad.detach().clone()
    src.grad = None
    out2 = homo_warping_depthwise(src, proj[:, 1].to(DEV), proj[:, 0].to(DEV), dep.to(DEV))
    out2.backward(gout.to(DEV))
    assert torch.equal(src.grad, g1)


def test_homo_warp_backward_nonfinite_and_large_batch():
    """a NaN / inf in grad_out reaches exactly the source pixels grid_sample's
    backward sends it to, every other pixel keeps its finite gradient, and the other batch
    elements keep the bit-reproducible fixed-point sums; B > 64 is processed in chunks."""
    from aarmvs import ops
    from oracle import sweep_oracle as orc
    g = load("warp.npz")
    _, N, H, W, C = (int(x) for x in g["shape"])
    B = 3
    sc = syn.scene(B, N, H, W, D=4, seed=int(g["seed"]), C=C)
    proj = torch.from_numpy(sc["proj_matrices"])
    rel = orc.relative_projection(proj[:, 1], proj[:, 0])
    dep = torch.from_numpy(sc["depth_values"][:, 1].copy())   # both bad pixels sample in-image
    gout = torch.randn(B, C, H, W, generator=torch.Generator().manual_seed(3))
    gout[1, 3, H // 2, W // 2] = float("nan")
    gout[1, 5, 1, 2] = float("inf")
    src_c = torch.from_numpy(sc["features"][1]).requires_grad_(True)
    orc.homo_warp(src_c, rel, dep, fast=True).backward(gout)   # grid_sample's own backward
    ref = src_c.grad.numpy()
    got = ops.homo_warp_backward(gout.to(DEV), rel.to(DEV), dep.to(DEV), (B, C, H, W)).cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(np.isinf(got), np.isinf(ref))
    fin = np.isfinite(ref)
    assert 0 < (~fin[1]).sum() <= 8 and fin[[0, 2]].all()   # only the bad pixels' taps
    np.testing.assert_allclose(got[fin], ref[fin], atol=1e-4 * np.abs(ref[fin]).max())
    # the finite batch elements are the fixed-point sums of a finite-only call, bit for bit
    clean = gout.clone()
    clean[1] = 0.0
    got_c = ops.homo_warp_backward(clean.to(DEV), rel.to(DEV), dep.to(DEV), (B, C, H, W)).cpu().numpy()
    assert np.array_equal(got[[0, 2]], got_c[[0, 2]])
    # B = 66 > 64: two chunks of batch elements, each element equal to its own single call
    Bl = 66
    rel_l = rel[:1].expand(Bl, 3, 4).contiguous()
    dep_l = torch.from_numpy(np.linspace(500.0, 700.0, Bl).astype(np.float32))
    g_l = torch.randn(Bl, 4, 8, 12, generator=torch.Generator().manual_seed(4))
    big = ops.homo_warp_backward(g_l.to(DEV), rel_l.to(DEV), dep_l.to(DEV), (Bl, 4, 8, 12)).cpu()
    for b in (0, 63, 64, 65):
        one = ops.homo_warp_backward(g_l[b:b + 1].to(DEV), rel_l[b:b + 1].to(DEV), dep_l[b:b + 1].to(DEV),
                                     (1, 4, 8, 12)).cpu()
        assert torch.equal(big[b:b + 1], one)


def test_training_backward_matches_cpu_autograd():
    """BPTT through the sweep (HIP forward + per-plane recompute) vs CPU autograd."""
    from oracle import sweep_oracle as orc
    B, N, H, W, D = 1, 3, 16, 24, 4
    sc = syn.scene(B, N, H, W, D, seed=51)
    m = _model(D, H, W, 4, False)
    P_cpu = {k: v.detach().cpu().clone().requires_grad_(True)
             for k, v in m.named_parameters() if k in syn.SWEEP_SHAPES}
    feats = torch.from_numpy(sc["features"])                       # [N,B,C,H,W]
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(1))

    # CPU reference: autograd through the oracle's fp32 restatement
    fc = feats.clone().requires_grad_(True)
    rels = [orc.relative_projection(proj[:, v], proj[:, 0]) for v in range(1, N)]
    state = orc.init_state(B, H, W)
    costs = []
    for d in range(D):
        x = orc.cost_slice(fc[0], [fc[v] for v in range(1, N)], rels, dv[:, d], P_cpu)
        cost, state = orc.unet_step(x, state, P_cpu)
        costs.append(cost)
    prob_c = torch.softmax(torch.stack(costs, 1).squeeze(2), dim=1)
    (prob_c * R).sum().backward()

    imgs = torch.from_numpy(np.moveaxis(sc["features"], 0, 1).copy()).to(DEV).requires_grad_(True)
    prob, _, _ = m(imgs, proj.to(DEV), dv.to(DEV))
    np.testing.assert_allclose(prob.detach().cpu().numpy(), prob_c.detach().numpy(), atol=1e-5)
    (prob * R.to(DEV)).sum().backward()
    gi = imgs.grad.cpu().numpy()
    gref = np.moveaxis(fc.grad.numpy(), 0, 1)
    np.testing.assert_allclose(gi, gref, atol=1e-4 * np.abs(gref).max())
    # conv_0.bias's true gradient is exactly 0 (softmax over D sums the cost gradients to
    # zero): both sides hold only fp32 cancellation noise, so it is checked for smallness;
    # every other parameter at 1e-4 of max(its own scale, 1e-3 x the largest)
    gmax = max(float(p.grad.abs().max()) for p in P_cpu.values())
    for k, p in m.named_parameters():
        if k not in P_cpu:
            continue
        gr = P_cpu[k].grad.numpy()
        if k == "cost_regularization.conv_0.bias":
            assert abs(float(p.grad)) < 1e-4 * gmax and abs(float(gr.item())) < 1e-4 * gmax
            continue
        tol = 1e-4 * max(np.abs(gr).max(), 1e-3 * gmax)
        np.testing.assert_allclose(p.grad.cpu().numpy(), gr, atol=tol, err_msg=k)

