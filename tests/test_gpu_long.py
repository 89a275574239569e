"""The whole recurrence at BASELINE's view and depth counts against the reference itself.

long_n5_d256 / long_n7_d512 / long_n11_d898 (tests/golden/make_golden.py gen_long) were made
by running the reference's EMVSNet eval forward (drmvsnet.py:300-345) with the shipped
model_dtu_v2 core weights at 96x128 over configs 2, 3 and 5's N and D.  The HIP sweep runs
the full D here and must match: depth rel-L1 <= 1e-3 (north_star), confidence 1e-4, the
per-plane cost (every 8th pixel) 1e-4 and the softmax at those pixels 1e-5, the per-plane
mean softmax probability 1e-6.

wta_overflow (gen_overflow) drives exp(cost) past fp32 overflow (drmvsnet.py:324-333):
the NaN positions of the confidence must be the reference's.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from aarmvs import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda"


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def rel_l1(a, b):
    return float(np.abs(a - b).sum() / max(np.abs(b).sum(), 1e-30))


def real_P():
    g = load("real_weights_sweep.npz")
    return {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w:")}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    from aarmvs import ops  # noqa: F401  (loads libaarmvs.so, raises if missing)


def _run(g, P, **kw):
    from aarmvs import ops
    B, N, H, W, D = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]))
    assert syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]) == str(g["digest"])
    fd = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    sw = ops.DepthSweep({k: v.to(DEV) for k, v in P.items()}, DEV)
    return sw(fd[0], [fd[v] for v in range(1, N)], proj[:, 0], [proj[:, v] for v in range(1, N)],
              torch.from_numpy(sc["depth_values"]), **kw)


@pytest.mark.parametrize("name", ["long_n5_d256.npz", "long_n7_d512.npz", "long_n11_d898.npz"])
def test_full_depth_sweep_matches_reference(name):
    from aarmvs import ops
    g = load(name)
    out = _run(g, real_P(), want_cost=True)
    depth, conf = out["depth"].cpu().numpy(), out["conf"].cpu().numpy()
    cost = out["cost"]
    assert rel_l1(depth, g["depth"]) <= 1e-3
    np.testing.assert_allclose(conf, g["conf"], atol=1e-4)
    np.testing.assert_allclose(cost[:, :, ::8, ::8].cpu().numpy(), g["cost_sub"], atol=1e-4, rtol=1e-5)
    prob = ops.softmax_depth(cost)
    ref_sub = torch.softmax(torch.from_numpy(g["cost_sub"]).double(), dim=1).numpy()
    np.testing.assert_allclose(prob[:, :, ::8, ::8].cpu().numpy(), ref_sub, atol=1e-5)
    np.testing.assert_allclose(prob.mean(dim=(2, 3)).cpu().numpy(), g["prob_plane_mean"], atol=1e-6)


def test_wta_exp_overflow_matches_reference():
    """conv_0 scaled so that exp(cost) overflows on ~5% of (pixel, plane)s: inf max_prob, NaN
    after a second overflow (0 * inf in the select), inf exp_sum.  The confidence's NaN
    positions, its finite values and the depth must be the reference's (pixels whose cost
    comes within 1e-3 of ln(FLT_MAX) on some plane are left out: <1% of the image)."""
    g = load("wta_overflow.npz")
    s, b = (float(x) for x in g["head_scale"])
    P = real_P()
    P["cost_regularization.conv_0.weight"] = P["cost_regularization.conv_0.weight"] * s
    P["cost_regularization.conv_0.bias"] = P["cost_regularization.conv_0.bias"] * s + b
    out = _run(g, P)
    conf, depth = out["conf"].cpu().numpy(), out["depth"].cpu().numpy()
    n = g["n_overflow"]
    ok = g["margin"] > 1e-3
    assert ok.mean() > 0.99 and (n[ok] >= 1).any() and (n[ok] == 0).any()
    np.testing.assert_array_equal(np.isnan(conf)[ok], np.isnan(g["conf"])[ok])
    fin = ok & ~np.isnan(g["conf"])
    np.testing.assert_allclose(conf[fin], g["conf"][fin], atol=1e-4)
    assert rel_l1(depth[ok], g["depth"][ok]) <= 1e-3
