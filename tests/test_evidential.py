"""The evidential head and its losses (evidential/models.py:183-459,
:462-558) against evidential.npz and e2e.npz, made by running the reference
(tests/golden/make_golden.py gen_evidential / gen_e2e).  CPU: the head is PyTorch.

Tolerances: 1e-4 relative to each output's scale (a 3D hourglass of ~4.3 M weights in
fp32, summation order differs with thread count), losses 1e-5 relative.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from aarmvs import synthetic as syn


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def close(a, b, rel=1e-4):
    a, b = np.asarray(a), np.asarray(b)
    np.testing.assert_allclose(a, b, atol=rel * max(np.abs(b).max(), 1e-30), rtol=0)


def head(wseed):
    from models import EMVSNet
    m = EMVSNet(32, image_scale=1.0, max_h=32, max_w=40)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    wts = syn.init_weights(shapes, seed=wseed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in wts.items()}, strict=True)
    return m.evidential


def test_head_matches_reference_eval_and_train_mode():
    g = load("evidential.npz")
    h = head(int(g["wseed"]))
    prob = torch.softmax(torch.from_numpy(g["logits"]), dim=1)
    dv = torch.from_numpy(g["depth_values"])
    with torch.no_grad():
        h.eval()
        ev, comb = h(prob, dv)
        close(ev.numpy(), g["ev_eval"])
        close(comb.numpy(), g["comb_eval"])
        h.train()
        ev, comb = h(prob, dv)
        close(ev.numpy(), g["ev_train"])
        close(comb.numpy(), g["comb_train"])


def test_losses_match_reference():
    from evidential.models import criterion_uncertainty, loss_der, loss_emvsnet
    g = load("evidential.npz")
    ev = torch.from_numpy(g["ev_train"])
    y, mask = torch.from_numpy(g["depth_gt"]), torch.from_numpy(g["mask"])
    dv = torch.from_numpy(g["depth_values"])
    prob = torch.softmax(torch.from_numpy(g["logits"]), dim=1)
    loss, gamma, evd = loss_der({"probability_volume": prob, "evidential_prediction": ev}, y, mask, dv)
    close(loss.numpy(), g["loss_der"], 1e-5)
    np.testing.assert_array_equal(gamma.numpy(), g["gamma"])
    keys = [k[4:] for k in g.files if k.startswith("der:")]
    assert sorted(keys) == sorted(evd)
    for k in keys:
        np.testing.assert_allclose(evd[k].numpy(), g["der:" + k], rtol=1e-6, atol=0)
    u, la, al, be = (ev[i:i + 1] for i in range(4))
    close(criterion_uncertainty(u, la, al, be, y, mask).numpy(), g["criterion_uncertainty"], 1e-5)
    close(loss_emvsnet(u, la, al, be, y, mask).numpy(), g["loss_emvsnet"], 1e-5)


def test_shape_limits_are_explicit_errors():
    """B != 1 or D != 32 fail in the reference deep inside a conv; here they
    raise EvidentialShapeError up front."""
    from evidential.models import EvidentialModule, EvidentialShapeError
    h = EvidentialModule(depth=32)
    with pytest.raises(EvidentialShapeError):
        h(torch.rand(2, 32, 16, 16), torch.rand(2, 32))
    with pytest.raises(EvidentialShapeError):
        h(torch.rand(1, 48, 16, 16), torch.rand(1, 48))


def test_drop_in_names_and_star_exports():
    """train.py star-imports evidential.models (train.py:21) and models (train.py:14)."""
    import models
    ns = {}
    exec("from evidential.models import *", ns)
    for n in ("EvidentialModule", "loss_der", "loss_emvsnet", "criterion_uncertainty", "HourGlass",
              "HourGlassUp", "Mish", "FMish", "convbn_3d", "disparity_regression", "np", "torch", "F"):
        assert n in ns, n
    assert models.loss_der is ns["loss_der"]
