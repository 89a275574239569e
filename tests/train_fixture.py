"""Shared by tests/test_oracle.py (CPU) and tests/test_gpu_train_fixtures.py (GPU): the
reference-made training-gradient fixtures (tests/golden/make_golden.py gen_train_grads: the
reference's train-mode EMVSNet.forward -> F.softmax -> mvsnet_cls_loss -> backward with the
model_dtu_v2 weights, drmvsnet.py:272-295, 347-381, train.py:297-306), their regenerated
inputs, and float64 / float32 CPU autograd of the oracle on the same inputs."""
import functools
import os

import numpy as np
import torch

from conftest import GOLDEN
from aarmvs import synthetic as syn
from oracle import sweep_oracle as orc

CASES = ("train_grads_n3_d192.npz", "train_grads_n5_d48.npz")


def rel_l2(a, ref):
    a = np.asarray(a, np.float64).ravel()
    ref = np.asarray(ref, np.float64).ravel()
    return float(np.linalg.norm(a - ref) / max(np.linalg.norm(ref), 1e-300))


@functools.lru_cache(maxsize=None)
def load_case(name):
    g = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    B, N, H, W, D = (int(x) for x in g["shape"])
    seed = int(g["seed"])
    sc = syn.scene(B, N, H, W, D, seed=seed)
    assert syn.array_digest(sc["features"], sc["proj_matrices"], sc["depth_values"]) == str(g["digest"])
    depth_gt, mask = syn.depth_targets(sc["depth_values"], H, W, seed)
    rw = np.load(os.path.join(GOLDEN, "real_weights_sweep.npz"), allow_pickle=False)
    P = {k[2:]: torch.from_numpy(rw[k]) for k in rw.files if k.startswith("w:")}
    fix = {"loss": float(g["loss"]), "features": g["grad_features"],
           "params": {k[2:]: g[k] for k in g.files if k.startswith("g:")}}
    return dict(shape=(B, N, H, W, D), features=torch.from_numpy(sc["features"]),
                proj=torch.from_numpy(sc["proj_matrices"]), dv=torch.from_numpy(sc["depth_values"]),
                depth_gt=torch.from_numpy(depth_gt), mask=torch.from_numpy(mask), P=P, fixture=fix)


@functools.lru_cache(maxsize=None)
def oracle_grads(name, dtype_name):
    """(loss, dL/dfeatures [N,B,32,H,W], {param: grad}) of the oracle in float32/float64."""
    c = load_case(name)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    loss, _, gf, gp = orc.train_grads(c["features"], c["proj"], c["dv"], c["P"], c["depth_gt"],
                                      c["mask"], dtype=getattr(torch, dtype_name))
    return float(loss), gf.double().numpy(), {k: v.double().numpy() for k, v in gp.items()}


# conv_0.bias: its true gradient is 0 (a constant shift of every plane's cost cancels in the
# softmax over D); float32 leaves a rounding residue, checked for size separately
ZERO_GRAD = "cost_regularization.conv_0.bias"
