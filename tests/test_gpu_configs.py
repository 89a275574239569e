"""GPU parity at BASELINE.json's full frames (configs 2, 3 and 5) against the CPU oracle,
the fp16 range guards (cell 0's cost slice, cells 3 and 4's GroupNorm+ReLU part), and the
standalone §8b entries (aarmvs_cost_slice,
aarmvs_wta_update).

The oracle runs the first k planes of each full-frame workload (its F.grid_sample form,
pinned to the warp fixture and to the real-weight sweep fixture in test_oracle.py); the
HIP sweep runs the same planes, and the full D in two d_range pieces against one call.
Tolerances as in test_gpu_parity.py: cost 1e-4, depth 1e-3 relative L1 (north_star).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from aarmvs import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_l1(a, b):
    return float(np.abs(a - b).sum() / max(np.abs(b).sum(), 1e-30))


def real_P():
    g = np.load(os.path.join(GOLDEN, "real_weights_sweep.npz"), allow_pickle=False)
    return {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w:")}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    torch.set_num_threads(min(16, os.cpu_count() or 1))


def _views(feats, proj):
    N = feats.shape[0]
    return feats[0], [feats[v] for v in range(1, N)], proj[:, 0], [proj[:, v] for v in range(1, N)]


@pytest.mark.parametrize("cfg,k", [
    ((1, 5, 600, 800, 256), 3),      # configs[1]: DTU eval 800x600, N=5, D=256
    ((1, 7, 1184, 1600, 512), 2),    # configs[2]: the headline, 1600x1184, N=7, D=512
    ((1, 11, 1056, 1920, 898), 2),   # configs[4]: Tanks&Temples 1920x1056, N=11 (nsrc=10), D=898
])
def test_full_frame_config_matches_oracle(cfg, k):
    from oracle import sweep_oracle as orc
    from aarmvs import ops
    B, N, H, W, D = cfg
    sc = syn.scene(B, N, H, W, D, seed=N * 100 + D)
    P = real_P()
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    ref = orc.sweep(*_views(feats, proj), dv[:, :k].contiguous(), P, fast=True)
    sw = ops.DepthSweep({n: v.to(DEV) for n, v in P.items()}, DEV)
    fd = feats.to(DEV)
    args = _views(fd, proj)
    part = sw(*args, dv[:, :k].contiguous(), want_cost=True)
    torch.cuda.synchronize()
    np.testing.assert_allclose(part["cost"].cpu().numpy(), ref["cost"].numpy(), atol=1e-4, rtol=1e-4)
    assert rel_l1(part["depth"].cpu().numpy(), ref["depth"].numpy()) <= 1e-3
    np.testing.assert_allclose(part["conf"].cpu().numpy(), ref["conf"].numpy(), atol=1e-4)
    # the whole D: one call against a continued d_range, bit for bit; its first k planes are
    # the planes just checked
    full = sw(*args, dv, want_cost=True)
    cost = torch.empty(B, D, H, W, device=DEV)
    cut = D // 3
    sw(*args, dv, d_range=(0, cut), cost_out=cost, want_depth=False)
    cont = sw(*args, dv, d_range=(cut, D), cost_out=cost)
    assert torch.equal(full["cost"], cost)
    assert torch.equal(full["depth"], cont["depth"]) and torch.equal(full["conf"], cont["conf"])
    assert torch.equal(full["cost"][:, :k], part["cost"])
    assert torch.isfinite(full["cost"]).all()
    hyp = torch.cat([torch.zeros(B, 1), dv], 1).to(DEV).view(B, D + 1, 1, 1)
    assert (full["depth"].unsqueeze(1) == hyp).any(dim=1).all()


def test_cell0_fp16_range_guard_with_large_features():
    """Features x100: the cost slice reaches |x| > 65504 (fp16's largest finite), which the
    split-fp16 cells would turn into inf without the guard (convlstm.hip xguard_exp)."""
    from oracle import sweep_oracle as orc
    from aarmvs import ops
    B, N, H, W, D = 1, 4, 64, 96, 4
    sc = syn.scene(B, N, H, W, D, seed=300)
    feats = torch.from_numpy(sc["features"]) * 100.0
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    P = real_P()
    views = _views(feats, proj)
    rels = [orc.relative_projection(sp, views[2]) for sp in views[3]]
    x0 = orc.cost_slice(views[0], views[1], rels, dv[:, 0], P)
    assert float(x0.abs().max()) > 65504.0
    ref = orc.sweep(*views, dv, P)
    sw = ops.DepthSweep({n: v.to(DEV) for n, v in P.items()}, DEV)
    out = sw(*_views(feats.to(DEV), proj), dv, want_cost=True)
    cost = out["cost"].cpu().numpy()
    assert np.isfinite(cost).all()
    np.testing.assert_allclose(cost, ref["cost"].numpy(), atol=1e-4, rtol=1e-4)
    assert rel_l1(out["depth"].cpu().numpy(), ref["depth"].numpy()) <= 1e-3
    # the standalone step (aarmvs_unet_step) takes max|x| itself
    state = orc.init_state(B, H, W)
    c_ref, _ = orc.unet_step(x0, state, P)
    c_gpu = sw.unet_step(x0.to(DEV), 0)
    np.testing.assert_allclose(c_gpu.cpu().numpy(), c_ref.numpy(), atol=1e-4, rtol=1e-4)


def test_gn_relu_fp16_range_guard_with_large_gamma():
    """deConvGnReLU's GroupNorm affine x100000: relu(GN(u)) feeding cells 3 and 4 exceeds 65504
    (fp16's largest finite; checked in the oracle), which their split-fp16 staging would turn
    into inf without the guard (convlstm.hip gguard_exp: bound |gamma| sqrt(n - 1) + |beta|).
    The sweep matches the oracle; the training backward (the weight gradients' GroupNorm+ReLU
    chunks use the same bound) stays finite."""
    from oracle import sweep_oracle as orc
    from aarmvs import ops
    B, N, H, W, D = 1, 3, 48, 64, 4
    sc = syn.scene(B, N, H, W, D, seed=301)
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    P = real_P()
    for j in (0, 1):
        for t in ("weight", "bias"):
            P[f"cost_regularization.deconv_{j}.gn.{t}"] = P[f"cost_regularization.deconv_{j}.gn.{t}"] * 1e5
    views = _views(feats, proj)
    rels = [orc.relative_projection(sp, views[2]) for sp in views[3]]
    x0 = orc.cost_slice(views[0], views[1], rels, dv[:, 0], P)
    st = orc.init_state(B, H, W)
    cw = lambda i: (P[f"cost_regularization.cell_list.{i}.conv.weight"],   # noqa: E731
                    P[f"cost_regularization.cell_list.{i}.conv.bias"])
    h0, _ = orc.lstm_cell(x0, *st[0], *cw(0))
    h1, _ = orc.lstm_cell(torch.nn.functional.max_pool2d(h0, 2, 2), *st[1], *cw(1))
    h2, _ = orc.lstm_cell(torch.nn.functional.max_pool2d(h1, 2, 2), *st[2], *cw(2))
    assert float(orc.deconv_gn_relu(h2, P, "deconv_0").max()) > 65504.0
    ref = orc.sweep(*views, dv, P)
    sw = ops.DepthSweep({n: v.to(DEV) for n, v in P.items()}, DEV)
    args = _views(feats.to(DEV), proj)
    out = sw(*args, dv, want_cost=True)
    cost = out["cost"].cpu().numpy()
    assert np.isfinite(cost).all()
    np.testing.assert_allclose(cost, ref["cost"].numpy(), atol=1e-3, rtol=1e-3)
    assert rel_l1(out["depth"].cpu().numpy(), ref["depth"].numpy()) <= 1e-3
    # the BPTT on the same weights
    rec = sw.record_buffers(B, H, W, D, DEV, nsrc=N - 1)
    rel = sw.relative(args[2], args[3], B)
    cvol = torch.empty(B, D, H, W, device=DEV)
    sw(*args, dv, want_depth=False, cost_out=cvol, rel=rel, record=rec)
    g_ref, g_srcs, g_par, _ = sw.backward(args[0], args[1], rel, dv, rec, torch.ones_like(cvol))
    torch.cuda.synchronize()
    assert torch.isfinite(g_ref).all() and all(torch.isfinite(g).all() for g in g_srcs)
    assert all(torch.isfinite(g).all() for g in g_par.values())


def test_standalone_cost_slice_matches_reference_fixture():
    """aarmvs_cost_slice against cost_slice.npz (made by running the reference)."""
    from aarmvs import ops
    g = np.load(os.path.join(GOLDEN, "cost_slice.npz"), allow_pickle=False)
    B, N, H, W, D = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]))
    P = {k: torch.from_numpy(v).to(DEV) for k, v in syn.sweep_weights(int(g["wseed"])).items()}
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    d = int(g["plane"])
    sw = ops.DepthSweep(P, DEV)
    x, om = sw.cost_slice(*_views(feats, proj), torch.from_numpy(sc["depth_values"][:, d].copy()),
                          want_omega=True)
    np.testing.assert_allclose(om.cpu().numpy(), g["omega"].reshape(N - 1, B, H, W), atol=1e-5)
    np.testing.assert_allclose(x.cpu().numpy(), g["slice"], atol=1e-4, rtol=1e-5)


def test_standalone_wta_update_matches_sweep_and_reference_rule():
    """aarmvs_wta_update over a cost volume equals the sweep's fused WTA bit for bit, and the
    reference's select rule (strict <, exp without max-subtraction) on hand-made ties."""
    from aarmvs import ops
    B, N, H, W, D = 2, 3, 32, 48, 6
    sc = syn.scene(B, N, H, W, D, seed=12)
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    sw = ops.DepthSweep({k: torch.from_numpy(v).to(DEV) for k, v in syn.sweep_weights(2).items()}, DEV)
    out = sw(*_views(feats, proj), dv, want_cost=True)
    mp, dm, es = (torch.zeros(B, H, W, device=DEV) for _ in range(3))
    for d in range(D):
        ops.wta_update(out["cost"][:, d].contiguous(), dv[:, d], mp, dm, es)
    assert torch.equal(dm, out["depth"])
    assert torch.equal(mp / es, out["conf"])
    # ties: equal costs keep the first plane's depth (drmvsnet.py:327 strict <)
    c = torch.zeros(1, 2, 2, device=DEV)
    mp, dm, es = (torch.zeros(1, 2, 2, device=DEV) for _ in range(3))
    ops.wta_update(c, torch.tensor([5.0]), mp, dm, es)
    ops.wta_update(c, torch.tensor([7.0]), mp, dm, es)
    assert torch.equal(dm, torch.full_like(dm, 5.0)) and torch.equal(es, torch.full_like(es, 2.0))


def test_softmax_depth_matches_torch():
    """aarmvs_softmax_depth (online two-pass softmax over D) vs torch.softmax(dim=1), D not
    a multiple of the kernel's 4-plane unroll, costs spanning +-80 (exp over/underflow
    handled by the max subtraction)."""
    import torch
    from aarmvs import ops
    g = torch.Generator().manual_seed(9)
    for B, D, H, W in [(2, 37, 24, 40), (1, 192, 16, 20), (1, 1, 8, 8)]:
        cost = (torch.rand(B, D, H, W, generator=g) * 160.0 - 80.0)
        ref = torch.softmax(cost.double(), dim=1).float()
        got = ops.softmax_depth(cost.cuda()).cpu()
        np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-5, atol=1e-7)


def test_sweep_is_bit_reproducible_across_runs_and_plane_groupings(monkeypatch):
    """The cost-slice stage runs in plane groups on a second stream beside the regulariser;
    every GroupNorm statistic is a fixed-order reduction of per-block partials, so the sweep
    is bit-identical run to run (whatever the two streams' interleaving) and for any plane
    group size (AARMVS_NPL), at config 2's full frame over several groups."""
    from aarmvs import ops
    B, N, H, W, D = 1, 5, 600, 800, 40
    sc = syn.scene(B, N, H, W, D, seed=11)
    P = real_P()
    fd = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    args = _views(fd, proj)
    sw = ops.DepthSweep({n: v.to(DEV) for n, v in P.items()}, DEV)   # two streams
    a = sw(*args, dv, want_cost=True)
    b = sw(*args, dv, want_cost=True)
    monkeypatch.setenv("AARMVS_NPL", "3")
    c = sw(*args, dv, want_cost=True)
    torch.cuda.synchronize()
    for k in ("cost", "depth", "conf"):
        assert torch.equal(a[k], b[k]), k
        assert torch.equal(a[k], c[k]), k
