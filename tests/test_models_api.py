"""CPU checks of the drop-in ``models`` package (the reference's Python API).

* state_dict layout == the shipped checkpoint's 90 core keys (ckpt_layout.json);
* FeatNet (PyTorch, incl. the DeformConv2d restatement) == the reference's features;
* mvsnet_cls_loss == the reference's loss / WTA depth / confidence;
* UNetConvLSTM's PyTorch step (used by the training recompute) == the reference;
* the sweep refuses CPU tensors (no CPU fallback in the product path).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from aarmvs import synthetic as syn


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def test_state_dict_matches_checkpoint_layout():
    """Without the head: the shipped checkpoints' 90 core keys (load strictly).  With it (the
    default): the reference EMVSNet's full 311-key layout (emvsnet_layout.json)."""
    from models import EMVSNet
    with open(os.path.join(GOLDEN, "ckpt_layout.json")) as f:
        layout = json.load(f)["keys"]
    m = EMVSNet(disparity_level=48, evidential=False)
    sd = {k: list(v.shape) for k, v in m.state_dict().items()}
    assert sd == layout
    assert sum(int(np.prod(s)) for s in sd.values()) == 187203
    with open(os.path.join(GOLDEN, "emvsnet_layout.json")) as f:
        full = json.load(f)["keys"]
    sd = {k: list(v.shape) for k, v in EMVSNet(disparity_level=48).state_dict().items()}
    assert sd == full and len(sd) == 311
    assert len([k for k in sd if k.startswith("evidential.")]) == 221
    n = sum(int(np.prod(s)) for k, s in sd.items() if not k.endswith("num_batches_tracked"))
    assert n - sum(int(np.prod(s)) for k, s in sd.items() if "running_" in k) == 4494115


def _model_with_weights(D, H, W, wseed, return_depth):
    from models import EMVSNet
    m = EMVSNet(disparity_level=D, image_scale=1.0, max_h=H, max_w=W, return_depth=return_depth)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    wts = syn.init_weights(shapes, seed=wseed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in wts.items()}, strict=True)
    return m


def test_featnet_matches_reference():
    g = load("e2e.npz")
    B, N, H, W, D = (int(x) for x in g["shape"])
    # the reference model held 311 keys (with its evidential head); the core keys
    # draw from the same per-name seeds, so the FeatNet weights are identical
    m = _model_with_weights(D, H, W, int(g["wseed"]), True)
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]), images=True)
    with torch.no_grad():
        f0 = m.feature(torch.from_numpy(sc["imgs"][:, 0])).numpy()
    np.testing.assert_allclose(f0, g["feature0"], atol=2e-5, rtol=1e-5)


def test_mvsnet_cls_loss_matches_reference():
    from models import mvsnet_cls_loss
    g = load("e2e.npz")
    B, N, H, W, D = (int(x) for x in g["shape"])
    sc = syn.scene(B, N, H, W, D, seed=int(g["seed"]), images=True)
    loss, wta, conf = mvsnet_cls_loss(torch.from_numpy(g["prob"]), torch.from_numpy(g["depth_gt"]),
                                      torch.from_numpy(g["mask"]),
                                      torch.from_numpy(sc["depth_values"]), return_prob_map=True)
    np.testing.assert_allclose(loss.numpy(), g["loss"], rtol=1e-6)
    np.testing.assert_array_equal(wta.numpy(), g["wta"])
    np.testing.assert_array_equal(conf.numpy(), g["loss_conf"])
    l2, w2 = mvsnet_cls_loss(torch.from_numpy(g["prob"]), torch.from_numpy(g["depth_gt"]),
                             torch.from_numpy(g["mask"]), torch.from_numpy(sc["depth_values"]))
    assert float(l2) == float(loss)


def test_unet_torch_step_matches_reference():
    from models.drmvsnet import UNetConvLSTM
    g = load("unet.npz")
    B, H, W, steps = (int(x) for x in g["shape"])
    reg = UNetConvLSTM((H, W), [32, 16, 16, 32, 32], [16, 16, 16, 16, 8],
                       [(3, 3)] * 5, 5)
    P = syn.sweep_weights(int(g["wseed"]))
    sd = {k[len("cost_regularization."):]: torch.from_numpy(v) for k, v in P.items()
          if k.startswith("cost_regularization.")}
    reg.load_state_dict(sd, strict=True)
    xs = np.random.default_rng(int(g["seed"])).standard_normal((steps, B, 32, H, W), dtype=np.float32)
    hidden = None
    with torch.no_grad():
        for s in range(steps):
            cost, hidden = reg(torch.from_numpy(xs[s]), hidden, s)
            np.testing.assert_allclose(cost.numpy(), g["cost"][s], atol=1e-5)
    for i in range(5):
        np.testing.assert_allclose(hidden[i][0].numpy(), g[f"h{i}"], atol=1e-5)
        np.testing.assert_allclose(hidden[i][1].numpy(), g[f"c{i}"], atol=1e-5)


def test_sweep_refuses_cpu_tensors():
    from aarmvs._lib import AarmvsError
    from models import EMVSNet
    m = EMVSNet(disparity_level=4, image_scale=1.0, max_h=16, max_w=16, return_depth=True)
    with pytest.raises(AarmvsError):
        m(torch.zeros(1, 2, 3, 16, 16), torch.eye(4).expand(1, 2, 4, 4), torch.ones(1, 4))


def test_sweep_params_found_on_dataparallel_style_replicas():
    """nn.DataParallel replicas (train.py:173) hold parameters as plain attributes, with an
    empty named_parameters(): the sweep's parameter lookup walks attributes instead."""
    from models.drmvsnet import EMVSNet, _sweep_params
    from aarmvs.ops import SWEEP_KEYS
    m = EMVSNet(8, image_scale=1.0, max_h=16, max_w=16)
    rep = m._replicate_for_data_parallel()
    mods = dict(m.named_modules())
    reps = {"": rep}
    for name, mod in m.named_modules():          # mimic torch.nn.parallel.replicate
        if name:
            parent, _, leaf = name.rpartition(".")
            r = mod._replicate_for_data_parallel()
            reps[name] = r
            reps[parent]._modules[leaf] = r
    copies = {}
    for name, mod in mods.items():
        for pn, p in mod._parameters.items():
            if p is None:
                continue
            t = p.detach().clone() * 1.0
            copies[(name + "." + pn).lstrip(".")] = t
            setattr(reps[name], pn, t)
    assert len(list(rep.named_parameters())) == 0
    got = _sweep_params(rep)
    assert [t is copies[k] for k, t in zip(SWEEP_KEYS, got)] == [True] * len(SWEEP_KEYS)
    assert [a is b for a, b in zip(_sweep_params(m), [dict(m.named_parameters())[k] for k in SWEEP_KEYS])] \
        == [True] * len(SWEEP_KEYS)
