"""How well-conditioned is omega.reweight_network.2.bias's gradient (one scalar: a cancelling sum
over every pixel, view and plane)?  At test_gpu_bptt's shape (2, 4, 24, 40, 5), CPU only:
  1. float32 autograd's error against float64 per torch thread count (reduction order only);
  2. float64 autograd with sq staged as the HIP omega conv stages it (two fp16 terms at a
     power-of-two scale, forward values only) -- the staging's share of the GPU's error.
usage: python tests/diag_omega_bias.py   (a diagnostic, not collected by pytest)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_bptt as T  # noqa: E402
from aarmvs import synthetic as syn  # noqa: E402
from oracle import sweep_oracle as orc  # noqa: E402

KEY = "omega.reweight_network.2.bias"
B, N, H, W, D = (2, 4, 24, 40, 5)


def split_sq(sq):
    """sq -> fp16 hi + lo of sq 2^-e (e: the tensor's max near fp16's top), straight-through."""
    m = float(sq.detach().abs().max())
    e = int(np.floor(np.log2(m))) - 15 if m > 0 else 0
    s = sq.detach() * 2.0 ** -e
    hi = s.to(torch.float16).to(sq.dtype)
    lo = (s - hi).to(torch.float16).to(sq.dtype)
    return sq + ((hi + lo) * 2.0 ** e - sq.detach())


def main():
    sc = syn.scene(B, N, H, W, D, seed=11 + D)
    P = {k: torch.from_numpy(v) for k, v in syn.sweep_weights(6).items()}
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(5))
    _, _, g64, _ = T._oracle_grads(feats, proj, dv, P, R, torch.float64)
    print(f"{KEY}: float64 value {float(g64[KEY]):.9e}")
    for nt in (1, 2, 4, 8):
        torch.set_num_threads(nt)
        _, _, g32, _ = T._oracle_grads(feats, proj, dv, P, R, torch.float32)
        print(f"  float32, {nt} threads: rel err {T.rel_l2(g32[KEY].numpy(), g64[KEY].numpy()):.3e}", flush=True)
    orig = orc.omega_weight
    orc.omega_weight = lambda sq, Pd, fast=False: orig(split_sq(sq), Pd, fast)
    try:
        _, _, g64e, _ = T._oracle_grads(feats, proj, dv, P, R, torch.float64)
    finally:
        orc.omega_weight = orig
    print(f"  float64 with sq staged as two fp16 terms: rel err {T.rel_l2(g64e[KEY].numpy(), g64[KEY].numpy()):.3e}")


if __name__ == "__main__":
    main()
