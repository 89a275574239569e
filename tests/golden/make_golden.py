"""Generate the golden fixtures by importing and RUNNING the reference on the CPU.

Runs only in the build container, where the reference is mounted read-only at
/root/reference.  Nothing from the reference is copied: the fixtures hold seeds,
input digests and reference OUTPUTS.  Inputs and weights are regenerated
bit-identically from ``aarmvs.synthetic`` (numpy PCG64) wherever they are needed.

In-process patches needed to run the reference on a CPU:
  * ``sys.path.append`` (not insert: the reference's top-level statistics.py would
    shadow the stdlib module);
  * ``torch.Tensor.cuda`` / ``nn.Module.cuda`` -> identity (module.py:95-96,
    drmvsnet.py:302-304);
  * ``model.evidential`` stubbed where the head cannot run (D != 32 or B > 1,
    SURVEY F2), and ``model.feature`` replaced by identity where a case feeds
    precomputed features instead of images.

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "aa-rmvsnet_amd"))
from aarmvs import synthetic as syn  # noqa: E402

REF = "/root/reference"


def import_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    # our drop-in package is also called ``models``: keep it off the path here
    sys.path[:] = [p for p in sys.path if os.path.abspath(p) != os.path.join(REPO, "aa-rmvsnet_amd")]
    for name in [m for m in sys.modules if m == "models" or m.startswith("models.")]:
        del sys.modules[name]
    if REF not in sys.path:
        sys.path.append(REF)
    torch.Tensor.cuda = lambda self, *a, **k: self
    nn.Module.cuda = lambda self, *a, **k: self
    import models.drmvsnet as drm  # noqa
    import models.module as mod  # noqa
    return drm, mod


class _NoEvidential(nn.Module):
    def forward(self, prob, depth_values):
        B, D, H, W = prob.shape
        return torch.zeros(4, H, W), torch.zeros(1, 32, H, W)


def make_model(drm, D, H, W, return_depth, seed, identity_feature=True, evidential=False):
    model = drm.EMVSNet(disparity_level=D, image_scale=1.0, max_h=H, max_w=W,
                        return_depth=return_depth)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    wts = syn.init_weights(shapes, seed=seed)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in wts.items()}, strict=True)
    if identity_feature:
        model.feature = nn.Identity()
    if not evidential:
        model.evidential = _NoEvidential()
    return model, wts


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def gen_warp(drm, mod, out):
    """homo_warping_depthwise (module.py:6-38) incl. far-out-of-bounds depths."""
    B, N, H, W, C = 2, 3, 24, 40, 8
    sc = syn.scene(B, N, H, W, D=4, seed=11, C=C)
    feats = sc["features"]
    proj = sc["proj_matrices"]
    depths = np.array([[40.0, 425.0, 935.0, 5000.0], [935.0, 30.0, 600.0, 425.0]], np.float32)
    res = np.zeros((N - 1, 4, B, C, H, W), np.float32)
    for v in range(1, N):
        for d in range(4):
            r = mod.homo_warping_depthwise(t(feats[v]), t(proj[:, v]), t(proj[:, 0]), t(depths[:, d]))
            res[v - 1, d] = r.numpy()
    np.savez_compressed(os.path.join(HERE, "warp.npz"), out=res, depths=depths,
                        seed=11, shape=np.array([B, N, H, W, C]),
                        digest=syn.array_digest(feats, proj))
    out.append("warp.npz")


def gen_slice_omega(drm, mod, out):
    """omega (drmvsnet.py:27-38) and one cost slice (drmvsnet.py:307-319)."""
    B, N, H, W, D = 2, 3, 24, 40, 4
    sc = syn.scene(B, N, H, W, D, seed=12)
    model, _ = make_model(drm, D, H, W, True, seed=5)
    feats, proj, dv = sc["features"], sc["proj_matrices"], sc["depth_values"]
    with torch.no_grad():
        d = 1
        acc = None
        ws = []
        for v in range(1, N):
            wv = mod.homo_warping_depthwise(t(feats[v]), t(proj[:, v]), t(proj[:, 0]), t(dv[:, d]))
            sq = (wv - t(feats[0])).pow_(2)
            rw = model.omega(sq)
            ws.append(rw.numpy())
            acc = (rw + 1) * sq if acc is None else acc + (rw + 1) * sq
        x = -1 * (acc / (N - 1))
    np.savez_compressed(os.path.join(HERE, "cost_slice.npz"), omega=np.stack(ws), slice=x.numpy(),
                        plane=d, seed=12, wseed=5, shape=np.array([B, N, H, W, D]),
                        digest=syn.array_digest(feats, proj, dv))
    out.append("cost_slice.npz")


def gen_unet(drm, mod, out):
    """UNetConvLSTM.forward (drmvsnet.py:119-167), three recurrent steps."""
    B, H, W, steps = 2, 24, 40, 3
    model, _ = make_model(drm, 4, H, W, True, seed=6)
    rng = np.random.default_rng(13)
    xs = rng.standard_normal((steps, B, 32, H, W), dtype=np.float32)
    costs = []
    hidden = None
    with torch.no_grad():
        for s in range(steps):
            c, hidden = model.cost_regularization(t(xs[s]), hidden, s)
            costs.append(c.numpy())
    st = {f"h{i}": hidden[i][0].numpy() for i in range(5)}
    st.update({f"c{i}": hidden[i][1].numpy() for i in range(5)})
    np.savez_compressed(os.path.join(HERE, "unet.npz"), cost=np.stack(costs), seed=13, wseed=6,
                        shape=np.array([B, H, W, steps]), digest=syn.array_digest(xs), **st)
    out.append("unet.npz")


def run_sweep(drm, B, N, H, W, D, seed, wseed, return_depth, descending=False):
    sc = syn.scene(B, N, H, W, D, seed=seed, descending=descending)
    model, _ = make_model(drm, D, H, W, return_depth, seed=wseed)
    model.eval()
    imgs = t(np.moveaxis(sc["features"], 0, 1))        # features fed through identity FeatNet
    with torch.no_grad():
        res = model(imgs, t(sc["proj_matrices"]), t(sc["depth_values"]))
    return sc, res


def gen_sweeps(drm, mod, out):
    # eval-mode sweep (online WTA), ascending and descending hypotheses
    for name, desc in (("sweep_eval.npz", False), ("sweep_eval_desc.npz", True)):
        B, N, H, W, D = 2, 3, 48, 64, 16
        sc, res = run_sweep(drm, B, N, H, W, D, seed=21, wseed=7, return_depth=True, descending=desc)
        np.savez_compressed(os.path.join(HERE, name), depth=res["depth"].numpy(),
                            conf=res["photometric_confidence"].numpy(), seed=21, wseed=7,
                            descending=desc, shape=np.array([B, N, H, W, D]),
                            digest=syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]))
        out.append(name)
    # train-mode sweep: softmax probability volume (drmvsnet.py:289-291), N=4 views
    B, N, H, W, D = 1, 4, 32, 48, 12
    sc, res = run_sweep(drm, B, N, H, W, D, seed=22, wseed=8, return_depth=False)
    np.savez_compressed(os.path.join(HERE, "sweep_train.npz"), prob=res[0].numpy(), seed=22, wseed=8,
                        shape=np.array([B, N, H, W, D]),
                        digest=syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]))
    out.append("sweep_train.npz")


def gen_config1(drm, mod, out):
    """BASELINE config 1: 3-view 160x128, D=48 (features fed directly)."""
    B, N, H, W, D = 1, 3, 128, 160, 48
    sc = syn.scene(B, N, H, W, D, seed=0)
    model, _ = make_model(drm, D, H, W, return_depth=False, seed=1)
    model.eval()
    imgs = t(np.moveaxis(sc["features"], 0, 1))
    with torch.no_grad():
        prob, _, _ = model(imgs, t(sc["proj_matrices"]), t(sc["depth_values"]))
    model.return_depth = True
    with torch.no_grad():
        res = model(imgs, t(sc["proj_matrices"]), t(sc["depth_values"]))
    p = prob.numpy()
    np.savez_compressed(os.path.join(HERE, "config1.npz"), depth=res["depth"].numpy(),
                        conf=res["photometric_confidence"].numpy(),
                        prob_sub=p[:, :, ::8, ::8].copy(), prob_plane_mean=p.mean(axis=(2, 3)),
                        seed=0, wseed=1, shape=np.array([B, N, H, W, D]),
                        digest=syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]))
    out.append("config1.npz")


def gen_e2e(drm, mod, out):
    """Full EMVSNet incl. FeatNet and the evidential head (B=1, D=32 only: SURVEY F2)."""
    B, N, H, W, D = 1, 3, 32, 40, 32
    sc = syn.scene(B, N, H, W, D, seed=31, images=True)
    model, _ = make_model(drm, D, H, W, return_depth=True, seed=9, identity_feature=False,
                          evidential=True)
    model.eval()
    imgs, proj, dv = t(sc["imgs"]), t(sc["proj_matrices"]), t(sc["depth_values"])
    with torch.no_grad():
        feat = model.feature(imgs[:, 0]).numpy()
        ev = model(imgs, proj, dv)
        model.return_depth = False
        prob, evid, comb = model(imgs, proj, dv)
    # train-mode (BatchNorm batch statistics) evidential output
    model.train()
    with torch.no_grad():
        prob_t, evid_t, comb_t = model(imgs, proj, dv)
    # mvsnet_cls_loss (drmvsnet.py:347-381) on the eval probability volume
    rng = np.random.default_rng(32)
    depth_gt = rng.uniform(400, 960, (B, H, W)).astype(np.float32)
    mask = (rng.uniform(0, 1, (B, H, W)) > 0.3).astype(np.float32)
    loss, wta, conf = drm.mvsnet_cls_loss(prob, t(depth_gt), t(mask), dv, return_prob_map=True)
    np.savez_compressed(os.path.join(HERE, "e2e.npz"), feature0=feat, depth=ev["depth"].numpy(),
                        conf=ev["photometric_confidence"].numpy(),
                        evidential_eval=ev["evidential_prediction"].numpy(), prob=prob.numpy(),
                        evidential=evid.numpy(), prob_combine=comb.numpy(),
                        prob_train=prob_t.numpy(), evidential_train=evid_t.numpy(),
                        depth_gt=depth_gt, mask=mask, loss=loss.numpy(), wta=wta.numpy(),
                        loss_conf=conf.numpy(), seed=31, wseed=9, shape=np.array([B, N, H, W, D]),
                        digest=syn.array_digest(sc["imgs"], sc["proj_matrices"], sc["depth_values"]))
    out.append("e2e.npz")


def gen_ckpt(drm, mod, out):
    """Checkpoint contract: the shipped core checkpoint's key layout, and an
    eval sweep run by the reference with its real (model_dtu_v2) omega/regulariser weights.
    The checkpoint is read with torch.load(weights_only=True)."""
    import json
    ck = torch.load(os.path.join(REF, "checkpoints", "model_dtu_v2.ckpt"), map_location="cpu",
                    weights_only=True)
    sd = ck["model"]
    layout = {k: list(v.shape) for k, v in sd.items()}
    with open(os.path.join(HERE, "ckpt_layout.json"), "w") as f:
        json.dump({"source": "checkpoints/model_dtu_v2.ckpt", "epoch": int(ck["epoch"]),
                   "keys": layout}, f, indent=0, sort_keys=True)
    out.append("ckpt_layout.json")
    B, N, H, W, D = 1, 4, 64, 80, 24
    sc = syn.scene(B, N, H, W, D, seed=41)
    model = drm.EMVSNet(disparity_level=D, image_scale=1.0, max_h=H, max_w=W, return_depth=True)
    model.load_state_dict(sd, strict=False)
    model.feature = nn.Identity()
    model.evidential = _NoEvidential()
    model.eval()
    imgs = t(np.moveaxis(sc["features"], 0, 1))
    with torch.no_grad():
        res = model(imgs, t(sc["proj_matrices"]), t(sc["depth_values"]))
        model.return_depth = False
        prob, _, _ = model(imgs, t(sc["proj_matrices"]), t(sc["depth_values"]))
    sweep_w = {k: sd[k].numpy() for k in syn.SWEEP_SHAPES}
    np.savez_compressed(os.path.join(HERE, "real_weights_sweep.npz"), depth=res["depth"].numpy(),
                        conf=res["photometric_confidence"].numpy(), prob_sub=prob.numpy()[:, :, ::4, ::4],
                        seed=41, shape=np.array([B, N, H, W, D]),
                        digest=syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]),
                        **{"w:" + k: v for k, v in sweep_w.items()})
    out.append("real_weights_sweep.npz")


def _real_core_weights():
    """The shipped model_dtu_v2 core, read with weights_only=True."""
    ck = torch.load(os.path.join(REF, "checkpoints", "model_dtu_v2.ckpt"), map_location="cpu",
                    weights_only=True)
    return ck["model"]


class _CostRecorder(nn.Module):
    """Wraps the reference's UNetConvLSTM and keeps every plane's cost_reg (the tensors the
    reference stacks at drmvsnet.py:320/341); the call itself is passed through unchanged."""

    def __init__(self, inner):
        super().__init__()
        self.inner = inner
        self.costs = []

    def forward(self, x, hidden, d):
        cost, hidden = self.inner(x, hidden, d)
        self.costs.append(cost.detach().clone())
        return cost, hidden


def _real_eval_sweep(drm, sd, B, N, H, W, D, seed, head_scale=None):
    """Eval-mode EMVSNet.forward (drmvsnet.py:300-345) with the real core weights on
    identity-FeatNet features; returns the scene, the outputs, the recorded cost volume and
    F.softmax over it (exactly drmvsnet.py:341-342 on the same tensors)."""
    sc = syn.scene(B, N, H, W, D, seed=seed)
    model = drm.EMVSNet(disparity_level=D, image_scale=1.0, max_h=H, max_w=W, return_depth=True)
    sd = dict(sd)
    if head_scale is not None:
        sc_w, sc_b = head_scale
        sd["cost_regularization.conv_0.weight"] = sd["cost_regularization.conv_0.weight"] * sc_w
        sd["cost_regularization.conv_0.bias"] = sd["cost_regularization.conv_0.bias"] * sc_w + sc_b
    model.load_state_dict(sd, strict=False)
    model.feature = nn.Identity()
    model.evidential = _NoEvidential()
    rec = _CostRecorder(model.cost_regularization)
    model.cost_regularization = rec
    model.eval()
    imgs = t(np.moveaxis(sc["features"], 0, 1))
    with torch.no_grad():
        res = model(imgs, t(sc["proj_matrices"]), t(sc["depth_values"]))
    cost = torch.stack(rec.costs, dim=1).squeeze(2)
    prob = torch.softmax(cost, dim=1)
    return sc, res, cost.numpy(), prob.numpy()


# Long-D cases at BASELINE's view counts and depth counts (configs 2, 3, 5), on a small frame
# so the reference finishes on the CPU; the real model_dtu_v2 core weights.
LONG_CASES = {"long_n5_d256.npz": (5, 256, 51), "long_n7_d512.npz": (7, 512, 52),
              "long_n11_d898.npz": (11, 898, 53)}
LONG_HW = (96, 128)


def gen_long(drm, mod, out):
    """The whole recurrence over BASELINE's depth counts: N=5/D=256, N=7/D=512 and
    N=11/D=898 (nsrc=10) at 96x128, run by the reference with the real weights.  Stored:
    depth and confidence (the eval outputs), the per-plane cost subsampled every 8 px (the
    softmax at those pixels follows from it) and the per-plane mean softmax probability."""
    sd = _real_core_weights()
    H, W = LONG_HW
    for name, (N, D, seed) in LONG_CASES.items():
        sc, res, cost, prob = _real_eval_sweep(drm, sd, 1, N, H, W, D, seed)
        np.savez_compressed(os.path.join(HERE, name), depth=res["depth"].numpy(),
                            conf=res["photometric_confidence"].numpy(),
                            cost_sub=cost[:, :, ::8, ::8].copy(),
                            prob_plane_mean=prob.mean(axis=(2, 3)), seed=seed,
                            shape=np.array([1, N, H, W, D]),
                            digest=syn.array_digest(sc["features"], sc["proj_matrices"],
                                                    sc["depth_values"]))
        out.append(name)


# conv_0 (the head, drmvsnet.py:117) scaled so that exp(cost) overflows fp32 on part of the
# planes and pixels: cost' = OVF_SCALE * cost + OVF_SHIFT.
OVF_SCALE, OVF_SHIFT = 4.0, 221.0


def gen_overflow(drm, mod, out):
    """The WTA's exp(cost) without max-subtraction (drmvsnet.py:324-339) driven past fp32
    overflow: where exp(cost) = inf the arithmetic select gives max_prob = inf, then NaN
    (0 * inf) at the next overflowing plane; exp_sum = inf; conf = NaN or 0.  Stored: depth,
    conf (NaN kept), per pixel the number of planes whose exp(cost) overflows and the
    smallest |cost - ln(FLT_MAX)| over the planes (to tell borderline pixels); real weights,
    N=3, 48x64, D=32."""
    sd = _real_core_weights()
    B, N, H, W, D = 1, 3, 48, 64, 32
    sc, res, cost, prob = _real_eval_sweep(drm, sd, B, N, H, W, D, 61,
                                           head_scale=(OVF_SCALE, OVF_SHIFT))
    conf = res["photometric_confidence"].numpy()
    ovf = np.isinf(np.exp(cost.astype(np.float32)))
    margin = np.abs(cost.astype(np.float64) - np.log(np.finfo(np.float32).max)).min(axis=1)
    np.savez_compressed(os.path.join(HERE, "wta_overflow.npz"), depth=res["depth"].numpy(),
                        conf=conf, n_overflow=ovf.sum(axis=1).astype(np.uint8),
                        margin=margin.astype(np.float32), seed=61, shape=np.array([B, N, H, W, D]),
                        head_scale=np.array([OVF_SCALE, OVF_SHIFT], np.float32),
                        digest=syn.array_digest(sc["features"], sc["proj_matrices"],
                                                sc["depth_values"]))
    out.append("wta_overflow.npz")


# Training-gradient cases (the BPTT's fixtures): (N, D, H, W, seed), B = 1, real weights.
# D = 192 is configs[3]'s depth count; the frame is small so the reference's CPU autograd
# finishes in seconds.
TRAIN_CASES = {"train_grads_n3_d192.npz": (3, 192, 32, 48, 71),
               "train_grads_n5_d48.npz": (5, 48, 48, 64, 72)}


def gen_train_grads(drm, mod, out):
    """The reference's training step through the sweep (train.py:297-306): train-mode
    EMVSNet.forward (drmvsnet.py:272-295: the depth loop with autograd, F.softmax) ->
    mvsnet_cls_loss (:347-381) -> backward(), identity FeatNet (the features are the leaves),
    evidential head stubbed, the real model_dtu_v2 core weights.  Stored: the loss, the
    gradient of every omega.* / cost_regularization.* parameter and dL/d features
    [N,B,32,H,W], all in the reference's float32."""
    sd = _real_core_weights()
    for name, (N, D, H, W, seed) in TRAIN_CASES.items():
        sc = syn.scene(1, N, H, W, D, seed=seed)
        model = drm.EMVSNet(disparity_level=D, image_scale=1.0, max_h=H, max_w=W, return_depth=False)
        model.load_state_dict(sd, strict=False)
        model.feature = nn.Identity()
        model.evidential = _NoEvidential()
        model.train()
        imgs = t(np.moveaxis(sc["features"], 0, 1)).requires_grad_(True)
        dv = t(sc["depth_values"])
        depth_gt, mask = syn.depth_targets(sc["depth_values"], H, W, seed)
        prob, _, _ = model(imgs, t(sc["proj_matrices"]), dv)
        loss, wta = drm.mvsnet_cls_loss(prob, t(depth_gt), t(mask), dv)
        loss.backward()
        grads = {"g:" + k: p.grad.numpy().copy() for k, p in model.named_parameters()
                 if k in syn.SWEEP_SHAPES}
        assert len(grads) == len(syn.SWEEP_SHAPES), sorted(set(syn.SWEEP_SHAPES) - set(grads))
        np.savez_compressed(os.path.join(HERE, name), loss=loss.detach().numpy(),
                            grad_features=np.moveaxis(imgs.grad.numpy(), 1, 0).copy(),
                            wta=wta.numpy(), prob_plane_mean=prob.detach().numpy().mean(axis=(2, 3)),
                            seed=seed, shape=np.array([1, N, H, W, D]),
                            digest=syn.array_digest(sc["features"], sc["proj_matrices"],
                                                    sc["depth_values"]), **grads)
        out.append(name)


def gen_evidential(drm, mod, out):
    """The evidential head (evidential/models.py:183-459) and loss_der (:517-558), which the
    reference's drivers consume (train.py:297-304, eval.py:151-153): the full EMVSNet
    state_dict layout, the head's outputs in eval and train mode on a softmax volume at its
    only working shape (B=1, D=32), and loss_der / loss_emvsnet /
    criterion_uncertainty on the train-mode output."""
    import json
    import evidential.models as evm
    model, _ = make_model(drm, 32, 32, 40, return_depth=False, seed=9, identity_feature=False,
                          evidential=True)
    layout = {k: list(v.shape) for k, v in model.state_dict().items()}
    with open(os.path.join(HERE, "emvsnet_layout.json"), "w") as f:
        json.dump({"keys": layout}, f, indent=0, sort_keys=True)
    out.append("emvsnet_layout.json")
    head = model.evidential
    rng = np.random.default_rng(77)
    logits = rng.standard_normal((1, 32, 32, 40)).astype(np.float32) * 2.0
    dv = syn.depth_hypotheses(32)[None]
    prob = torch.softmax(t(logits), dim=1)
    with torch.no_grad():
        head.eval()
        ev_e, comb_e = head(prob, t(dv))
        head.train()
        ev_t, comb_t = head(prob, t(dv))
    depth_gt = rng.uniform(400, 960, (1, 32, 40)).astype(np.float32)
    mask = (rng.uniform(0, 1, (1, 32, 40)) > 0.3).astype(np.float32)
    outputs = {"probability_volume": prob, "evidential_prediction": ev_t}
    loss, gamma, evd = evm.loss_der(outputs, t(depth_gt), t(mask), t(dv))
    u, la, al, be = (ev_t[i:i + 1] for i in range(4))
    crit = evm.criterion_uncertainty(u, la, al, be, t(depth_gt), t(mask))
    lem = evm.loss_emvsnet(u, la, al, be, t(depth_gt), t(mask))
    np.savez_compressed(os.path.join(HERE, "evidential.npz"), logits=logits, depth_values=dv,
                        ev_eval=ev_e.numpy(), comb_eval=comb_e.numpy(), ev_train=ev_t.numpy(),
                        comb_train=comb_t.numpy(), depth_gt=depth_gt, mask=mask,
                        loss_der=loss.numpy(), gamma=gamma.numpy(),
                        criterion_uncertainty=crit.numpy(), loss_emvsnet=lem.numpy(),
                        wseed=9, **{"der:" + k: v.numpy() for k, v in evd.items()})
    out.append("evidential.npz")


def _reference_datasets():
    """The reference's ``datasets`` package, loaded by path (the name is also taken by an
    installed library)."""
    import importlib.util
    for name in [m for m in sys.modules if m == "datasets" or m.startswith("datasets.")]:
        del sys.modules[name]
    spec = importlib.util.spec_from_file_location(
        "datasets", os.path.join(REF, "datasets", "__init__.py"),
        submodule_search_locations=[os.path.join(REF, "datasets")])
    pkg = importlib.util.module_from_spec(spec)
    sys.modules["datasets"] = pkg
    spec.loader.exec_module(pkg)
    import datasets.dtu_yao as dy  # noqa
    return dy


def gen_datasets(drm, mod, out):
    """The training loader (datasets/dtu_yao.py) run by the reference on the committed tiny
    DTU-format tree tests/golden/dtu_mini (synthetic cameras, 64x80 PNGs, 16x20 PFMs):
    samples with ascending and flipped hypotheses, linear and inverse spacing, fixed range.
    (The eval loaders import OpenCV, absent here: their camera/hypothesis recipes are
    checked against known answers in tests/test_datasets.py.)"""
    dy = _reference_datasets()
    root = os.path.join(HERE, "dtu_mini")
    res = {}
    for tag, kw, idxs in (("lin", {}, (0, 1, 5)),
                          ("inv", {"inverse_depth": True, "fix_range": True}, (2, 7))):
        ds = dy.MVSDataset(root, os.path.join(root, "scans.txt"), "train", 3, ndepths=48,
                           light_idx=3, image_scale=0.25, **kw)
        res[f"{tag}:n"] = np.array(len(ds))
        for i in idxs:
            smp = ds[i]
            for k, v in smp.items():
                if k == "name":
                    v = os.path.relpath(v, root)
                res[f"{tag}:{i}:{k}"] = np.asarray(v)
    np.savez_compressed(os.path.join(HERE, "datasets.npz"), **res)
    out.append("datasets.npz")


GENERATORS = (gen_warp, gen_slice_omega, gen_unet, gen_sweeps, gen_config1, gen_e2e, gen_ckpt,
              gen_evidential, gen_datasets, gen_long, gen_overflow, gen_train_grads)


def main():
    """``make_golden.py [gen_name ...]`` regenerates only the named fixtures (default all);
    MANIFEST.txt lists every generator's output."""
    torch.manual_seed(0)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    drm, mod = import_reference()
    only = set(sys.argv[1:])
    out = []
    for fn in GENERATORS:
        if only and fn.__name__ not in only:
            continue
        fn(drm, mod, out)
        print("wrote", out[-1], flush=True)
    manifest = os.path.join(HERE, "MANIFEST.txt")
    names = [ln.strip() for ln in open(manifest) if ln.strip() and not ln.startswith("#")] \
        if only and os.path.exists(manifest) else []
    names += [n for n in out if n not in names]
    with open(manifest, "w") as f:
        f.write("# generated by tests/golden/make_golden.py from the reference run on CPU\n")
        f.write(f"# torch {torch.__version__}, numpy {np.__version__}\n")
        for name in names:
            f.write(name + "\n")


if __name__ == "__main__":
    main()
