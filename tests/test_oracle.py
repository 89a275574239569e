"""Pin the CPU oracle against the golden fixtures produced by running the reference.

CPU-only (``-m "not gpu"``).  Tolerances: per-op <=1e-5 abs, end-to-end
depth <=1e-3 relative L1 (BASELINE.json north_star).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from aarmvs import synthetic as syn
from oracle import sweep_oracle as orc


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def P_of(wseed):
    return {k: torch.from_numpy(v) for k, v in syn.sweep_weights(wseed).items()}


def rel_l1(a, b):
    return float(np.abs(a - b).sum() / max(np.abs(b).sum(), 1e-30))


def test_inputs_regenerate_bit_identically():
    g = load("warp.npz")
    B, N, H, W, C = g["shape"]
    sc = syn.scene(B, N, H, W, D=4, seed=int(g["seed"]), C=C)
    assert syn.array_digest(sc["features"], sc["proj_matrices"]) == str(g["digest"])


def test_warp_matches_reference():
    g = load("warp.npz")
    B, N, H, W, C = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D=4, seed=int(g["seed"]), C=C)
    proj = torch.from_numpy(sc["proj_matrices"])
    feats = torch.from_numpy(sc["features"])
    for v in range(1, N):
        rel = orc.relative_projection(proj[:, v], proj[:, 0])
        for d in range(4):
            out = orc.homo_warp(feats[v], rel, torch.from_numpy(g["depths"][:, d])).numpy()
            np.testing.assert_allclose(out, g["out"][v - 1, d], atol=1e-5, rtol=0)


def test_omega_and_cost_slice_match_reference():
    g = load("cost_slice.npz")
    B, N, H, W, D = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]))
    P = P_of(int(g["wseed"]))
    proj = torch.from_numpy(sc["proj_matrices"])
    feats = torch.from_numpy(sc["features"])
    d = int(g["plane"])
    dv = torch.from_numpy(sc["depth_values"][:, d])
    rels = [orc.relative_projection(proj[:, v], proj[:, 0]) for v in range(1, N)]
    for v in range(1, N):
        sq = (orc.homo_warp(feats[v], rels[v - 1], dv) - feats[0]).pow(2)
        np.testing.assert_allclose(orc.omega_weight(sq, P).numpy(), g["omega"][v - 1], atol=1e-5)
    x = orc.cost_slice(feats[0], [feats[v] for v in range(1, N)], rels, dv, P).numpy()
    np.testing.assert_allclose(x, g["slice"], atol=1e-4, rtol=1e-5)


def test_unet_steps_match_reference():
    g = load("unet.npz")
    B, H, W, steps = (int(x) for x in g["shape"])
    P = P_of(int(g["wseed"]))
    xs = np.random.default_rng(int(g["seed"])).standard_normal((steps, B, 32, H, W), dtype=np.float32)
    state = orc.init_state(B, H, W)
    for s in range(steps):
        cost, state = orc.unet_step(torch.from_numpy(xs[s]), state, P)
        np.testing.assert_allclose(cost.numpy(), g["cost"][s], atol=1e-5)
    for i in range(5):
        np.testing.assert_allclose(state[i][0].numpy(), g[f"h{i}"], atol=1e-5)
        np.testing.assert_allclose(state[i][1].numpy(), g[f"c{i}"], atol=1e-5)


def _sweep(g, want_volume):
    B, N, H, W, D = (int(x) for x in g["shape"])
    desc = bool(g["descending"]) if "descending" in g.files else False
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]), descending=desc)
    assert syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]) == str(g["digest"])
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    return orc.sweep(feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
                     [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]),
                     P_of(int(g["wseed"])), want_volume=want_volume)


@pytest.mark.parametrize("name", ["sweep_eval.npz", "sweep_eval_desc.npz"])
def test_eval_sweep_matches_reference(name):
    g = load(name)
    out = _sweep(g, want_volume=False)
    assert rel_l1(out["depth"].numpy(), g["depth"]) <= 1e-3
    np.testing.assert_allclose(out["conf"].numpy(), g["conf"], atol=1e-4)


def test_train_sweep_prob_volume_matches_reference():
    g = load("sweep_train.npz")
    out = _sweep(g, want_volume=True)
    np.testing.assert_allclose(out["prob"].numpy(), g["prob"], atol=1e-5)


def test_config1_matches_reference():
    g = load("config1.npz")
    out = _sweep(g, want_volume=True)
    assert rel_l1(out["depth"].numpy(), g["depth"]) <= 1e-3
    np.testing.assert_allclose(out["conf"].numpy(), g["conf"], atol=1e-4)
    p = out["prob"].numpy()
    np.testing.assert_allclose(p[:, :, ::8, ::8], g["prob_sub"], atol=1e-5)
    np.testing.assert_allclose(p.mean(axis=(2, 3)), g["prob_plane_mean"], atol=1e-6)


def test_fast_warp_matches_reference_and_gather():
    """The timing restatement's warp (F.grid_sample, the reference's own call) against the
    warp fixture, and bit-for-bit against the oracle's explicit gather."""
    g = load("warp.npz")
    B, N, H, W, C = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D=4, seed=int(g["seed"]), C=C)
    proj = torch.from_numpy(sc["proj_matrices"])
    feats = torch.from_numpy(sc["features"])
    for v in range(1, N):
        rel = orc.relative_projection(proj[:, v], proj[:, 0])
        for d in range(4):
            dep = torch.from_numpy(g["depths"][:, d])
            fast = orc.homo_warp(feats[v], rel, dep, fast=True)
            np.testing.assert_allclose(fast.numpy(), g["out"][v - 1, d], atol=1e-5, rtol=0)
            np.testing.assert_allclose(fast.numpy(), orc.homo_warp(feats[v], rel, dep).numpy(),
                                       atol=1e-6, rtol=0)


def test_fast_sweep_matches_real_weight_fixture():
    """The fast sweep with the reference's real model_dtu_v2 weights (real_weights_sweep.npz)."""
    g = load("real_weights_sweep.npz")
    B, N, H, W, D = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]))
    assert syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]) == str(g["digest"])
    P = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w:")}
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    times = []
    out = orc.sweep(feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
                    [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]), P,
                    fast=True, plane_times=times)
    assert len(times) == D
    assert rel_l1(out["depth"].numpy(), g["depth"]) <= 1e-3
    np.testing.assert_allclose(out["conf"].numpy(), g["conf"], atol=1e-4)
    np.testing.assert_allclose(out["prob"].numpy()[:, :, ::4, ::4], g["prob_sub"], atol=1e-5)


def _real_P():
    g = load("real_weights_sweep.npz")
    return {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w:")}


def _long_inputs(g):
    B, N, H, W, D = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]))
    assert syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]) == str(g["digest"])
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    return (feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
            [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]))


def test_fast_sweep_matches_long_d256_fixture():
    """The whole recurrence over config 2's N=5, D=256 (long_n5_d256.npz, made by running the
    reference with the model_dtu_v2 weights at 96x128).  The N=7/D=512 and N=11/D=898
    fixtures are checked against the HIP sweep in tests/test_gpu_long.py."""
    g = load("long_n5_d256.npz")
    out = orc.sweep(*_long_inputs(g), _real_P(), fast=True)
    assert rel_l1(out["depth"].numpy(), g["depth"]) <= 1e-3
    np.testing.assert_allclose(out["conf"].numpy(), g["conf"], atol=1e-4)
    np.testing.assert_allclose(out["cost"].numpy()[:, :, ::8, ::8], g["cost_sub"], atol=1e-4, rtol=1e-5)
    np.testing.assert_allclose(out["prob"].numpy().mean(axis=(2, 3)), g["prob_plane_mean"], atol=1e-6)


def overflow_params():
    """The real weights with the head conv_0 scaled as in make_golden.gen_overflow."""
    g = load("wta_overflow.npz")
    s, b = (float(x) for x in g["head_scale"])
    P = _real_P()
    P["cost_regularization.conv_0.weight"] = P["cost_regularization.conv_0.weight"] * s
    P["cost_regularization.conv_0.bias"] = P["cost_regularization.conv_0.bias"] * s + b
    return P


def test_wta_overflow_semantics_match_reference():
    """exp(cost) without max-subtraction (drmvsnet.py:324) past fp32 overflow: inf max_prob,
    then NaN from 0 * inf in the arithmetic select (:328), inf exp_sum -> NaN/0 confidence.
    The fixture has pixels that never overflow, overflow once and overflow repeatedly."""
    g = load("wta_overflow.npz")
    n = g["n_overflow"]
    assert (n == 0).any() and (n == 1).any() and (n >= 2).any()
    out = orc.sweep(*_long_inputs(g), overflow_params(), want_volume=False)
    conf = out["conf"].numpy()
    ok = g["margin"] > 1e-3          # pixels whose costs all stay clear of ln(FLT_MAX)
    assert ok.mean() > 0.99
    np.testing.assert_array_equal(np.isnan(conf)[ok], np.isnan(g["conf"])[ok])
    assert np.isnan(g["conf"][n >= 1]).all()
    fin = ok & ~np.isnan(g["conf"])
    np.testing.assert_allclose(conf[fin], g["conf"][fin], atol=1e-4)
    assert rel_l1(out["depth"].numpy()[ok], g["depth"][ok]) <= 1e-3


@pytest.mark.parametrize("name", ["train_grads_n3_d192.npz", "train_grads_n5_d48.npz"])
def test_train_grads_match_reference(name):
    """The oracle's training step (orc.train_grads: forward, softmax, cls_loss, autograd)
    against the reference's own float32 gradients (make_golden.gen_train_grads, real weights,
    D=192 at 32x48 N=3 and D=48 at 48x64 N=5): in float32 the oracle repeats the reference's
    arithmetic to rounding (<=1e-5 relative L2 per tensor; measured <=1.3e-6), and the
    reference's float32 error against the oracle's float64 is the oracle's own float32 error
    (within 1.5x + 1e-6): the float64 oracle is the anchor the GPU backward is measured
    against (tests/test_gpu_train_fixtures.py)."""
    import train_fixture as tf
    c = tf.load_case(name)
    fix = c["fixture"]
    l32, f32, p32 = tf.oracle_grads(name, "float32")
    l64, f64, p64 = tf.oracle_grads(name, "float64")
    assert abs(l32 - fix["loss"]) <= 1e-6 * abs(fix["loss"])
    assert abs(l64 - fix["loss"]) <= 1e-5 * abs(fix["loss"])
    checks = [("features", fix["features"], f32, f64)]
    checks += [(k, fix["params"][k], p32[k], p64[k]) for k in fix["params"] if k != tf.ZERO_GRAD]
    assert len(checks) == len(syn.SWEEP_SHAPES)
    bad = []
    for k, g_ref, g32, g64 in checks:
        e_same, e_ref, e_o32 = tf.rel_l2(g32, g_ref), tf.rel_l2(g_ref, g64), tf.rel_l2(g32, g64)
        if not (e_same <= 1e-5 and e_ref <= 1.5 * e_o32 + 1e-6):
            bad.append((k, e_same, e_ref, e_o32))
    assert not bad, bad
    # the zero-gradient bias: a float32 residue only, in the reference as in the oracle
    scale = float(np.abs(fix["params"]["cost_regularization.conv_0.weight"]).max())
    assert abs(float(np.asarray(fix["params"][tf.ZERO_GRAD]).reshape(-1)[0])) <= 1e-3 * scale
