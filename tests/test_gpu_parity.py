"""GPU parity tests: the HIP path (through the C ABI) against the golden fixtures
made by running the reference, and against the CPU oracle at larger sizes.

Tolerances: per-op <= 1e-5 abs where the reference computes a single op, cost
slices/states 1e-4 (fp32 reassociation in conv sums), depth maps <= 1e-3
relative L1 (BASELINE.json north_star).
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


def P_of(wseed, device=DEV):
    return {k: torch.from_numpy(v).to(device) for k, v in syn.sweep_weights(wseed).items()}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    from aarmvs import ops  # noqa: F401  (loads libaarmvs.so, raises if missing)


def test_homo_warp_matches_reference():
    from aarmvs import ops
    g = load("warp.npz")
    B, N, H, W, C = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D=4, seed=int(g["seed"]), C=C)
    proj = torch.from_numpy(sc["proj_matrices"])
    feats = torch.from_numpy(sc["features"]).to(DEV)
    for v in range(1, N):
        rel = ops.relative_projection(proj[:, v], proj[:, 0])
        for d in range(4):
            out = ops.homo_warp(feats[v], rel, torch.from_numpy(g["depths"][:, d]))
            np.testing.assert_allclose(out.cpu().numpy(), g["out"][v - 1, d], atol=1e-5, rtol=0)


def _sweep_obj(wseed):
    from aarmvs import ops
    return ops.DepthSweep(P_of(wseed), DEV)


def test_cost_slice_and_omega_match_reference():
    g = load("cost_slice.npz")
    B, N, H, W, D = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]))
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    d = int(g["plane"])
    sw = _sweep_obj(int(g["wseed"]))
    out = sw(feats[0], [feats[v] for v in range(1, N)], proj[:, 0], [proj[:, v] for v in range(1, N)],
             torch.from_numpy(sc["depth_values"][:, d:d + 1].copy()), want_depth=False, debug=True)
    np.testing.assert_allclose(out["omega"].cpu().numpy(), g["omega"].reshape(N - 1, B, H, W),
                               atol=1e-5)
    np.testing.assert_allclose(out["slice"].cpu().numpy(), g["slice"], atol=1e-4, rtol=1e-5)


def test_unet_steps_match_reference():
    g = load("unet.npz")
    B, H, W, steps = (int(x) for x in g["shape"])
    xs = np.random.default_rng(int(g["seed"])).standard_normal((steps, B, 32, H, W), dtype=np.float32)
    sw = _sweep_obj(int(g["wseed"]))
    for s in range(steps):
        cost = sw.unet_step(torch.from_numpy(xs[s]).to(DEV), s)
        np.testing.assert_allclose(cost.cpu().numpy(), g["cost"][s], atol=1e-5, rtol=1e-5)
    for i in range(5):
        h = sw.state(B, H, W, 1, steps, i, 0).cpu().numpy()
        c = sw.state(B, H, W, 1, steps, i, 1).cpu().numpy()
        np.testing.assert_allclose(h, g[f"h{i}"], atol=1e-5)
        np.testing.assert_allclose(c, g[f"c{i}"], atol=1e-5)


def _run(g, **kw):
    B, N, H, W, D = (int(x) for x in g["shape"])
    desc = bool(g["descending"]) if "descending" in g.files else False
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]), descending=desc)
    assert syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]) == str(g["digest"])
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    sw = _sweep_obj(int(g["wseed"]))
    return sw(feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
              [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]), **kw)


@pytest.mark.parametrize("name", ["sweep_eval.npz", "sweep_eval_desc.npz"])
def test_eval_sweep_matches_reference(name):
    g = load(name)
    out = _run(g)
    assert rel_l1(out["depth"].cpu().numpy(), g["depth"]) <= 1e-3
    np.testing.assert_allclose(out["conf"].cpu().numpy(), g["conf"], atol=1e-4)


def test_train_sweep_prob_volume_matches_reference():
    from aarmvs import ops
    g = load("sweep_train.npz")
    out = _run(g, want_depth=False, want_cost=True)
    prob = ops.softmax_depth(out["cost"])
    np.testing.assert_allclose(prob.cpu().numpy(), g["prob"], atol=1e-5)


def test_config1_matches_reference():
    from aarmvs import ops
    g = load("config1.npz")
    out = _run(g, want_cost=True)
    assert rel_l1(out["depth"].cpu().numpy(), g["depth"]) <= 1e-3
    np.testing.assert_allclose(out["conf"].cpu().numpy(), g["conf"], atol=1e-4)
    p = ops.softmax_depth(out["cost"]).cpu().numpy()
    np.testing.assert_allclose(p[:, :, ::8, ::8], g["prob_sub"], atol=1e-5)
    np.testing.assert_allclose(p.mean(axis=(2, 3)), g["prob_plane_mean"], atol=1e-6)


def test_larger_views_and_batch_match_oracle():
    """N=6 views, B=2, 96x200 (W not a multiple of 32): HIP vs the CPU oracle."""
    from oracle import sweep_oracle as orc
    B, N, H, W, D = 2, 6, 96, 200, 5
    sc = syn.scene(B, N, H, W, D, seed=41)
    P = {k: torch.from_numpy(v) for k, v in syn.sweep_weights(3).items()}
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    ref = orc.sweep(feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
                    [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]), P)
    from aarmvs import ops
    sw = ops.DepthSweep({k: v.to(DEV) for k, v in P.items()}, DEV)
    fd = feats.to(DEV)
    out = sw(fd[0], [fd[v] for v in range(1, N)], proj[:, 0], [proj[:, v] for v in range(1, N)],
             torch.from_numpy(sc["depth_values"]), want_cost=True)
    np.testing.assert_allclose(out["cost"].cpu().numpy(), ref["cost"].numpy(), atol=1e-4, rtol=1e-4)
    assert rel_l1(out["depth"].cpu().numpy(), ref["depth"].numpy()) <= 1e-3


@pytest.mark.parametrize("shape", [(1, 3, 52, 84, 3), (1, 2, 4, 4, 2), (1, 3, 4, 132, 3)])
def test_ragged_and_minimum_sizes_match_oracle(shape):
    """H, W multiples of 4 (the U-Net's two 2x pools, drmvsnet.py:148-150) but not of the
    16x32 pixel tile: partial tiles, the 4x4 minimum (level-2 maps are 1x1), a 4-row strip."""
    from oracle import sweep_oracle as orc
    B, N, H, W, D = shape
    sc = syn.scene(B, N, H, W, D, seed=H * 1000 + W)
    P = {k: torch.from_numpy(v) for k, v in syn.sweep_weights(7).items()}
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    ref = orc.sweep(feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
                    [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]), P)
    from aarmvs import ops
    sw = ops.DepthSweep({k: v.to(DEV) for k, v in P.items()}, DEV)
    fd = feats.to(DEV)
    out = sw(fd[0], [fd[v] for v in range(1, N)], proj[:, 0], [proj[:, v] for v in range(1, N)],
             torch.from_numpy(sc["depth_values"]), want_cost=True)
    np.testing.assert_allclose(out["cost"].cpu().numpy(), ref["cost"].numpy(), atol=1e-4, rtol=1e-4)
    assert rel_l1(out["depth"].cpu().numpy(), ref["depth"].numpy()) <= 1e-3


def test_rejects_cpu_tensors_and_bad_shapes():
    from aarmvs import ops
    from aarmvs._lib import AarmvsError
    sw = _sweep_obj(1)
    x = torch.zeros(1, 32, 16, 16)
    proj = torch.eye(4).expand(1, 4, 4)
    with pytest.raises(AarmvsError):
        sw(x, [x], proj, [proj], torch.ones(1, 2))
    y = torch.zeros(1, 32, 18, 16, device=DEV)
    with pytest.raises(AarmvsError):
        sw(y, [y], proj, [proj], torch.ones(1, 2))



@pytest.mark.parametrize("cap", ["4", "96"])
def test_pipeline_box_fallbacks_are_bit_identical(monkeypatch, cap):
    """AARMVS_PIPE_BOX_CAP shrinks omega_conv's LDS source boxes, sending (tile, view)
    blocks to the global-gather path.  The arithmetic is the same, so the sweep must be
    bit-identical."""
    B, N, H, W, D = 1, 4, 64, 96, 4
    sc = syn.scene(B, N, H, W, D, seed=5)
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    sw = _sweep_obj(2)
    args = (feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
            [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]))
    a = sw(*args, want_cost=True, debug=True)
    monkeypatch.setenv("AARMVS_PIPE_BOX_CAP", cap)
    b = sw(*args, want_cost=True, debug=True)
    for k in ("cost", "slice", "omega", "depth", "conf"):
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("ipb", ["1", "3", "8"])
def test_omega_items_per_block_are_bit_identical(monkeypatch, ipb):
    """AARMVS_OMEGA_IPB sets how many consecutive (plane) items of one (tile, view) an
    omega_conv block walks (default: 8, fewer on small grids).  The items' arithmetic is
    unchanged, so the sweep must be bit-identical; D = 6 leaves a ragged last block."""
    B, N, H, W, D = 2, 3, 64, 96, 6
    sc = syn.scene(B, N, H, W, D, seed=11)
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    sw = _sweep_obj(2)
    args = (feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
            [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]))
    a = sw(*args, want_cost=True, debug=True)
    monkeypatch.setenv("AARMVS_OMEGA_IPB", ipb)
    b = sw(*args, want_cost=True, debug=True)
    for k in ("cost", "slice", "omega", "depth", "conf"):
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("skew", ["0", "1", "2", "3"])
def test_cell_wave_skew_is_bit_identical(monkeypatch, skew):
    """AARMVS_CELL_SKEW picks which half of the double-buffered cells' waves stages before its
    MFMAs (default: per cell, CellDef::SKEW).  Only the order of independent work changes, so
    the sweep must be bit-identical to the default for every setting."""
    B, N, H, W, D = 1, 3, 72, 100, 3
    sc = syn.scene(B, N, H, W, D, seed=13)
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    sw = _sweep_obj(3)
    args = (feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
            [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]))
    a = sw(*args, want_cost=True)
    monkeypatch.setenv("AARMVS_CELL_SKEW", skew)
    b = sw(*args, want_cost=True)
    for k in ("cost", "depth", "conf"):
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("ms", ["0", "1", "2"])
@pytest.mark.parametrize("B,N,H,W,D", [(1, 3, 68, 100, 3), (2, 3, 128, 160, 2)])
def test_cell_tile_shapes_are_bit_identical(monkeypatch, B, N, H, W, D, ms):
    """AARMVS_CELL_MS forces the cells' tile shape (convlstm.hip cell_shape: 0 one wave per
    32-px row with every m-tile, the default; 1 two waves per row each with half the m-tiles;
    2 the same at 16 waves per block).  Every m-tile's MFMAs and
    gate update are the same instructions in the same order, so the sweep must be bit-identical
    to the default for every shape (68 rows: a ragged last 8-row tile)."""
    sc = syn.scene(B, N, H, W, D, seed=17)
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    sw = _sweep_obj(3)
    args = (feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
            [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]))
    a = sw(*args, want_cost=True)
    monkeypatch.setenv("AARMVS_CELL_MS", ms)
    b = sw(*args, want_cost=True)
    for k in ("cost", "depth", "conf"):
        assert torch.equal(a[k], b[k]), k


def test_two_stream_schedule_is_bit_identical():
    """The omega pipeline of plane d+1 on a second stream (the default) against the
    single-stream schedule: same kernels, same inputs, so bit-identical outputs; a
    continued range (d_range) must also match a full sweep."""
    from aarmvs import ops
    B, N, H, W, D = 1, 4, 64, 96, 6
    sc = syn.scene(B, N, H, W, D, seed=9)
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    args = (feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
            [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]))
    P = P_of(4)
    a = ops.DepthSweep(P, DEV, overlap=True)(*args, want_cost=True)
    b = ops.DepthSweep(P, DEV, overlap=False)(*args, want_cost=True)
    sw = ops.DepthSweep(P, DEV, overlap=True)
    cost = torch.empty(B, D, H, W, device=DEV)
    sw(*args, d_range=(0, 2), cost_out=cost)
    c = sw(*args, d_range=(2, D), cost_out=cost)
    for k in ("cost", "depth", "conf"):
        assert torch.equal(a[k], b[k]), k
    assert torch.equal(a["cost"], cost)
    assert torch.equal(a["depth"], c["depth"]) and torch.equal(a["conf"], c["conf"])


@pytest.mark.parametrize("nreg", ["default", "2", "3", "4", "5", "5:02121"])
@pytest.mark.parametrize("B,N,H,W,D", [(1, 3, 128, 160, 37), (2, 4, 64, 96, 5), (1, 3, 256, 320, 20)])
def test_multi_stream_regulariser_is_bit_identical(monkeypatch, B, N, H, W, D, nreg):
    """The U-Net step's five units (cell 0 | cell 1 | cell 2 | deconv_0, cell 3 | deconv_1,
    cell 4, head) of neighbouring planes on the library's streams (AARMVS_REG_STREAMS=2: cells
    0-2 | the rest; 3: cells 0-1 | cell 2, deconv_0, cell 3 | deconv_1, cell 4, head; 4: cell 1
    and cell 2 share a stream; 5: one unit per stream; "5:02121" an assignment out of unit order,
    AARMVS_REG_MAP) against the one-stream order: bit-identical cost volume, depth and
    confidence, also over continued d_ranges whose boundaries fall inside and at the end of
    plane groups, with and without the cost-stage stream (config 1's 160x128 at D=37 crosses
    three plane groups).  "default": the library's choice: for the small frames (B*H*W <= 65536)
    the cost stage on the caller's stream and the units over four streams, at 256x320 the cost
    stage on the aux stream and the units over three."""
    nreg, _, umap = nreg.partition(":")
    if umap:
        monkeypatch.setenv("AARMVS_REG_MAP", umap)
    from aarmvs import ops
    sc = syn.scene(B, N, H, W, D, seed=21)
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    args = (feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
            [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]))
    P = P_of(6)
    monkeypatch.setenv("AARMVS_REG_STREAMS", "1")
    ref = ops.DepthSweep(P, DEV, overlap=True)(*args, want_cost=True)
    if nreg == "default":
        monkeypatch.delenv("AARMVS_REG_STREAMS")
    else:
        monkeypatch.setenv("AARMVS_REG_STREAMS", nreg)
    for overlap in (True, False):
        got = ops.DepthSweep(P, DEV, overlap=overlap)(*args, want_cost=True)
        for k in ("cost", "depth", "conf"):
            assert torch.equal(got[k], ref[k]), (overlap, k)
    sw = ops.DepthSweep(P, DEV, overlap=True)
    cost = torch.empty(B, D, H, W, device=DEV)
    cuts = [0, 1, min(16, D - 1), D] if D > 17 else [0, 2, D]
    for d0, d1 in zip(cuts[:-1], cuts[1:]):
        c = sw(*args, d_range=(d0, d1), cost_out=cost)
    assert torch.equal(cost, ref["cost"])
    assert torch.equal(c["depth"], ref["depth"]) and torch.equal(c["conf"], ref["conf"])


def test_full_size_properties():
    """BASELINE's full frame (1600x1184, N=7) at D=3, where the oracle is too slow: the
    two-stream and single-stream schedules and a continued d_range must agree bit for bit,
    and the WTA depth must be one of the hypotheses (drmvsnet.py:324-339)."""
    from aarmvs import ops
    B, N, H, W, D = 1, 7, 1184, 1600, 3
    sc = syn.scene(B, N, H, W, D, seed=77)
    feats = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    args = (feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
            [proj[:, v] for v in range(1, N)], dv)
    P = P_of(5)
    a = ops.DepthSweep(P, DEV, overlap=True)(*args, want_cost=True)
    b = ops.DepthSweep(P, DEV, overlap=False)(*args, want_cost=True)
    sw = ops.DepthSweep(P, DEV, overlap=True)
    cost = torch.empty(B, D, H, W, device=DEV)
    sw(*args, d_range=(0, 1), cost_out=cost)
    c = sw(*args, d_range=(1, D), cost_out=cost)
    for k in ("cost", "depth", "conf"):
        assert torch.equal(a[k], b[k]), k
    assert torch.equal(a["cost"], cost)
    assert torch.equal(a["depth"], c["depth"]) and torch.equal(a["conf"], c["conf"])
    assert torch.isfinite(a["cost"]).all()
    depth = a["depth"].cpu()
    # 0 is the initial depth map (drmvsnet.py:301), kept where every exp(cost) underflows
    hyp = torch.cat([torch.zeros(B, 1), dv.to(depth.dtype)], 1).view(B, D + 1, 1, 1)
    assert (depth.unsqueeze(1) == hyp).any(dim=1).all()


def test_sweep_with_points_behind_a_source_camera_matches_oracle():
    """A source projection whose z row is mixed with its x row (z' = z - x / (W/2) in
    pixel units): z' changes sign across the image, so omega_conv sees tiles with every
    corner in front (the corner-box path), tiles straddling z' = 0 and tiles wholly
    behind (both on the per-pixel box path), and positions far outside the image."""
    from oracle import sweep_oracle as orc
    from aarmvs import ops
    B, N, H, W, D = 1, 3, 64, 160, 4
    sc = syn.scene(B, N, H, W, D, seed=23)
    proj = torch.from_numpy(sc["proj_matrices"]).clone()
    M = torch.eye(4)
    M[2, 0] = -1.0 / (W / 2)
    proj[:, 2] = M @ proj[:, 2]
    rel = ops.relative_projection(proj[:, 2], proj[:, 0])[0].numpy()
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)
    zs = [(rel[2, 0] * xs + rel[2, 1] * ys + rel[2, 2]) * d + rel[2, 3]
          for d in sc["depth_values"][0]]
    neg = float(np.mean(np.stack(zs) <= 0))
    assert 0.1 < neg < 0.9, neg
    P = {k: torch.from_numpy(v) for k, v in syn.sweep_weights(6).items()}
    feats = torch.from_numpy(sc["features"])
    ref = orc.sweep(feats[0], [feats[v] for v in range(1, N)], proj[:, 0],
                    [proj[:, v] for v in range(1, N)], torch.from_numpy(sc["depth_values"]), P)
    sw = ops.DepthSweep({k: v.to(DEV) for k, v in P.items()}, DEV)
    fd = feats.to(DEV)
    out = sw(fd[0], [fd[v] for v in range(1, N)], proj[:, 0], [proj[:, v] for v in range(1, N)],
             torch.from_numpy(sc["depth_values"]), want_cost=True)
    np.testing.assert_allclose(out["cost"].cpu().numpy(), ref["cost"].numpy(), atol=1e-4, rtol=1e-4)
    assert rel_l1(out["depth"].cpu().numpy(), ref["depth"].numpy()) <= 1e-3


@pytest.mark.parametrize("B,N,H,W,D", [(1, 3, 128, 160, 20), (1, 3, 256, 320, 20)])
def test_sweep_graph_capture_replays_bit_identical(B, N, H, W, D):
    """A caller may record the sweep into a HIP graph (torch.cuda.CUDAGraph): under stream
    capture the library keeps everything on the capturing stream (api.hip: the multi-stream
    schedules are not captured), and the replay's cost volume and depth equal the eager sweep's
    bit for bit, for a small-frame and a large-frame schedule."""
    from aarmvs import ops
    sc = syn.scene(B, N, H, W, D, seed=5)
    P = P_of(6)
    sw = ops.DepthSweep(P, DEV, overlap=True)
    f = torch.from_numpy(sc["features"]).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"]).to(DEV).float().contiguous()
    ref, srcs = f[0].contiguous(), [f[v].contiguous() for v in range(1, N)]
    rel = sw.relative(proj[:, 0], [proj[:, v] for v in range(1, N)], B)
    cost = torch.empty(B, D, H, W, device=DEV)

    def run():
        return sw(ref, srcs, None, [None] * (N - 1), dv, want_depth=True, cost_out=cost, rel=rel)

    out = run()
    torch.cuda.synchronize()
    eager_cost, eager_depth = cost.clone(), out["depth"].clone()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    cost.zero_()
    with torch.cuda.graph(g):
        gout = run()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(cost, eager_cost) and torch.equal(gout["depth"], eager_depth)
