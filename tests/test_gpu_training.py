"""GPU tests of the training path (configs[3]: DTU training 640x512, N=3, D=192, DDP):
BPTT through the HIP sweep at the full 640x512 frame over a truncated D against CPU
autograd of the oracle, nn.DataParallel replicas (train.py:173, eval.py:77), and a
world-2 DDP step (gloo, two processes on the one device) whose gradients must equal the
hand-averaged per-rank gradients.

Gradient tolerance: 1e-4 of max(the gradient's own scale, 1e-3 x the largest), as in
test_gpu_models.py (fp32 atomics and reassociation in the backward).
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import ROOT
from aarmvs import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    torch.set_num_threads(min(16, os.cpu_count() or 1))


F32_THREADS = (4, 8, 16)   # reduction orders of the float32 reference (full frame: >= 4 threads)


def _model(D, H, W, wseed):
    from models import EMVSNet
    m = EMVSNet(disparity_level=D, image_scale=1.0, max_h=H, max_w=W, return_depth=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    wts = syn.init_weights(shapes, seed=wseed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in wts.items()}, strict=True)
    m.feature = nn.Identity()
    return m.to(DEV)


def _oracle_grads(feats, proj, dv, P_cpu, R, dtype=torch.float32):
    """CPU autograd of the oracle's restatement (F.grid_sample warp) in `dtype`: float32 is the
    reference's own arithmetic, float64 the anchor both are measured against."""
    from oracle import sweep_oracle as orc
    N, B, C, H, W = feats.shape
    fc = feats.to(dtype).clone().requires_grad_(True)
    P = {k: v.detach().to(dtype).clone().requires_grad_(True) for k, v in P_cpu.items()}
    rels = [orc.relative_projection(proj[:, v], proj[:, 0]) for v in range(1, N)]
    state = [(h.to(dtype), c.to(dtype)) for h, c in orc.init_state(B, H, W)]
    costs = []
    for d in range(dv.shape[1]):
        x = orc.cost_slice(fc[0], [fc[v] for v in range(1, N)], rels, dv[:, d], P, fast=True)
        cost, state = orc.unet_step(x, state, P)
        costs.append(cost)
    prob = torch.softmax(torch.stack(costs, 1).squeeze(2), dim=1)
    (prob * R.to(dtype)).sum().backward()
    return prob.detach(), fc.grad, {k: v.grad for k, v in P.items()}


def _rel_err(a, ref):
    a, ref = np.asarray(a, np.float64).ravel(), np.asarray(ref, np.float64).ravel()
    return float(np.linalg.norm(a - ref) / max(np.linalg.norm(ref), 1e-300))


def test_config4_full_frame_training_backward_matches_cpu_autograd():
    """640x512, N=3 (configs[3]) over the first 4 of D=192's hypotheses, every gradient
    anchored to float64 CPU autograd of the oracle: per tensor, the GPU's relative L2 error
    against float64 must be at most twice the float32 CPU autograd's (the reference's own
    arithmetic) error against float64 -- the max over the reduction orders ATen uses at
    F32_THREADS threads -- plus 1e-6 for tensors where float32 is exact to round-off (the
    split-fp16 products' ~2^-22)."""
    B, N, H, W, D = 1, 3, 512, 640, 4
    sc = syn.scene(B, N, H, W, 192, seed=404)
    dv = torch.from_numpy(sc["depth_values"][:, :D].copy())
    m = _model(D, H, W, 8)
    P_cpu = {k: v.detach().cpu().clone() for k, v in m.named_parameters() if k in syn.SWEEP_SHAPES}
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(3))
    prob64, gf64, gp64 = _oracle_grads(feats, proj, dv, P_cpu, R, torch.float64)
    # float32's error depends on ATen's reduction order, i.e. its thread count: the reference
    # error is the max over F32_THREADS (a fixed function of the inputs, not of the host)
    e32, gb32 = {}, 0.0
    prev = torch.get_num_threads()
    try:
        for n in F32_THREADS:
            torch.set_num_threads(n)
            _, gf32, gp32 = _oracle_grads(feats, proj, dv, P_cpu, R, torch.float32)
            cand = {"features": _rel_err(np.moveaxis(gf32.numpy(), 0, 1), np.moveaxis(gf64.numpy(), 0, 1))}
            cand.update({k: _rel_err(gp32[k].numpy(), gp64[k].numpy()) for k in gp64})
            for k, v in cand.items():
                e32[k] = max(e32.get(k, 0.0), v)
            gb32 = max(gb32, gp32["cost_regularization.conv_0.bias"].abs().max().item())
    finally:
        torch.set_num_threads(prev)

    imgs = torch.from_numpy(np.moveaxis(sc["features"], 0, 1).copy()).to(DEV).requires_grad_(True)
    prob, _, _ = m(imgs, proj.to(DEV), dv.to(DEV))
    np.testing.assert_allclose(prob.detach().cpu().numpy(), prob64.numpy(), atol=1e-5)
    (prob * R.to(DEV)).sum().backward()
    report = {}
    checks = [("features", imgs.grad.cpu().numpy(), np.moveaxis(gf64.numpy(), 0, 1))]
    for k, p in m.named_parameters():
        if k in P_cpu and k != "cost_regularization.conv_0.bias":   # true gradient 0 (softmax)
            checks.append((k, p.grad.cpu().numpy(), gp64[k].numpy()))
    bad = []
    for k, g_gpu, g64 in checks:
        e_gpu, e_cpu = _rel_err(g_gpu, g64), e32[k]
        report[k] = (e_gpu, e_cpu)
        lim = 2.0 * e_cpu + 1e-6
        if not e_gpu <= lim:
            bad.append((k, e_gpu, e_cpu))
    print("\nrelative L2 error vs float64 (gpu, cpu fp32):")
    for k, (a, b) in report.items():
        print(f"  {k:48s} {a:.3e} {b:.3e}")
    assert not bad, bad
    # the conv_0 bias: its float64 gradient is ~0; the GPU's must be as small as float32's
    gb = m.cost_regularization.conv_0.bias.grad.abs().max().item()
    assert gb <= 2.0 * gb32 + 1e-6


def test_second_backward_through_freed_graph_raises():
    """The saved plane states are freed by the first backward (save_for_backward), so a second
    backward raises autograd's own error; with retain_graph=True it runs and repeats."""
    B, N, H, W, D = 1, 3, 16, 24, 3
    sc = syn.scene(B, N, H, W, D, seed=5)
    m = _model(D, H, W, 2)
    imgs = torch.from_numpy(np.moveaxis(sc["features"], 0, 1).copy()).to(DEV).requires_grad_(True)
    proj = torch.from_numpy(sc["proj_matrices"]).to(DEV)
    dv = torch.from_numpy(sc["depth_values"]).to(DEV)
    prob, _, _ = m(imgs, proj, dv)
    loss = (prob * torch.arange(D, device=DEV).view(1, D, 1, 1)).sum()
    loss.backward(retain_graph=True)
    g1 = imgs.grad.clone()
    imgs.grad = None
    loss.backward()
    # every sum of the backward has a fixed order (dL/dsrc in 64-bit fixed point): bit-equal
    assert torch.equal(imgs.grad, g1)
    with pytest.raises(RuntimeError):
        loss.backward()


def test_dataparallel_replica_runs_the_hip_sweep():
    """nn.DataParallel's replicas hold parameters as plain attributes (named_parameters() is
    empty): the sweep finds them by attribute, forward and backward."""
    from torch.nn.parallel import replicate
    B, N, H, W, D = 1, 3, 32, 48, 4
    sc = syn.scene(B, N, H, W, D, seed=31)
    m = _model(D, H, W, 3)
    imgs = torch.from_numpy(np.moveaxis(sc["features"], 0, 1).copy()).to(DEV)
    proj = torch.from_numpy(sc["proj_matrices"]).to(DEV)
    dv = torch.from_numpy(sc["depth_values"]).to(DEV)
    rep = replicate(m, [0])[0]
    assert len(list(rep.named_parameters())) == 0
    prob_r, _, _ = rep(imgs, proj, dv)
    prob_m, _, _ = m(imgs, proj, dv)
    assert torch.equal(prob_r, prob_m)
    prob_r.sum().backward()   # gradients flow back to the original parameters
    assert m.cost_regularization.cell_list[0].conv.weight.grad is not None
    m.return_depth = True
    rep = replicate(m, [0])[0]
    with torch.no_grad():
        assert torch.equal(rep(imgs, proj, dv)["depth"], m(imgs, proj, dv)["depth"])


def test_ddp_world2_gradients_equal_hand_averaged():
    """Two processes on the one device, gloo (RCCL refuses two ranks on one GPU): DDP over
    EMVSNet's HIP training path (_SweepTrain) averages the gradients of the two ranks."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = os.path.join(ROOT, "tests", "ddp_worker.py")
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
        assert p.returncode == 0, out[-3000:]
    for out in outs:
        assert "DDP_OK" in out, out[-3000:]


def test_ddp_rccl_one_rank_gradients_equal_local():
    """The RCCL (`nccl` backend) process group with DDP over the HIP training path: one rank
    (RCCL refuses two ranks on one GPU), DDP's gradient all-reduce over RCCL leaves the
    gradients bit-identical to a plain backward of the same sample."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), DDP_BACKEND="nccl")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ddp_worker.py")], env=env,
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "DDP_OK" in r.stdout, r.stdout[-3000:]


def _train_args(tmp_path, numdepth, extra=()):
    from aarmvs import train_ddp
    mini = os.path.join(ROOT, "tests", "golden", "dtu_mini")
    return train_ddp.parse_args([
        "--trainpath", mini, "--trainlist", os.path.join(mini, "scans.txt"), "--numdepth", str(numdepth),
        "--max_h", "64", "--max_w", "80", "--image_scale", "0.25", "--epochs", "2", "--max_steps", "2",
        "--logdir", str(tmp_path / "ckpt"), "--summary_freq", "1", "--train_light_idx", "3", *extra])


@pytest.mark.parametrize("numdepth", [8, 32])
def test_train_driver_steps_and_checkpoints(tmp_path, numdepth):
    """aarmvs.train_ddp (train.py's loop) on the tiny DTU tree: finite losses, one checkpoint
    per epoch in train.py's format, reloadable into a fresh model, and --resume continues
    from the last epoch (D=32: the evidential head and loss_der run, as in train.py)."""
    from aarmvs import train_ddp
    from models import EMVSNet
    out = train_ddp.train(_train_args(tmp_path, numdepth), 0, 1, DEV, log=lambda *a: None)
    assert len(out["losses"]) == 4 and all(np.isfinite(out["losses"]))
    assert [os.path.basename(p) for p in out["checkpoints"]] == ["model_000000.ckpt", "model_000001.ckpt"]
    st = torch.load(out["checkpoints"][-1], map_location="cpu", weights_only=True)
    assert set(st) == {"epoch", "model", "optimizer"} and st["epoch"] == 1
    EMVSNet(disparity_level=numdepth, image_scale=0.25, max_h=64, max_w=80).load_state_dict(st["model"], strict=True)
    args = _train_args(tmp_path, numdepth, ["--resume"])
    args.epochs = 3
    out2 = train_ddp.train(args, 0, 1, DEV, log=lambda *a: None)
    assert [os.path.basename(p) for p in out2["checkpoints"]] == ["model_000002.ckpt"]


def test_train_driver_two_ranks_share_the_samples(tmp_path):
    """Two ranks of aarmvs.train_ddp (shared-GPU rehearsal: both on cuda:0, gloo): DDP over
    the HIP training path, each rank on its half of the samples, rank 0 checkpoints."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mini = os.path.join(ROOT, "tests", "golden", "dtu_mini")
    cmd = [sys.executable, "-m", "aarmvs.train_ddp", "--trainpath", mini, "--trainlist",
           os.path.join(mini, "scans.txt"), "--numdepth", "8", "--max_h", "64", "--max_w", "80",
           "--epochs", "1", "--max_steps", "2", "--logdir", str(tmp_path / "ck"), "--train_light_idx", "3"]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), AARMVS_SHARED_GPU="1",
                   PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "aa-rmvsnet_amd"), ROOT,
                                               os.environ.get("PYTHONPATH", "")]))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
        assert p.returncode == 0, out[-3000:]
    assert "rank 0/2: 2 steps" in outs[0] and "rank 1/2: 2 steps" in outs[1], outs
    assert os.path.exists(tmp_path / "ck" / "model_000000.ckpt")
