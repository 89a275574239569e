"""Signed error of the omega logits' bias gradient (omega.reweight_network.2.bias) over seeds
(round 6): per seed the GPU's and float32 CPU autograd's (1 and 8 threads)
error against float64 autograd of the oracle, in units of u * sum|dL/dlogit| (u = 2^-24).
A systematic (single-signed) GPU error would point at a biased accumulation.
usage: python tests/diag_omega_bias_seeds.py [NSEEDS] [B N H W D]"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
import conftest  # noqa: E402,F401  (import paths)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_bptt as T  # noqa: E402

KB = "omega.reweight_network.2.bias"


def one(seed, shape):
    from oracle import sweep_oracle as orc
    B, N, H, W, D = shape
    sc, P, feats, proj, dv, sw, args = T._setup(B, N, H, W, D, seed, 6)
    cost, rec, rel = T._record_forward(sw, args, B, H, W, D)
    R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(seed + 1))
    tsum = [0.0]
    orc.LOGIT_HOOK = lambda z: z.register_hook(lambda g: tsum.__setitem__(0, tsum[0] + float(g.abs().sum())))
    try:
        _, _, gp64, _ = T._oracle_grads(feats, proj, dv, P, R, torch.float64)
    finally:
        orc.LOGIT_HOOK = None
    gcost = None
    # dL/dcost of (prob * R).sum() with prob = softmax over D of the recorded cost (as the test)
    c = cost.detach().clone().requires_grad_(True)
    (torch.softmax(c, 1) * R.to(c.device)).sum().backward()
    gcost = c.grad
    _, _, gp, _ = sw.backward(args[0], args[1], rel, dv, rec, gcost)
    ref = float(gp64[KB])
    unit = 2.0 ** -24 * tsum[0]
    out = {"gpu": (float(gp[KB]) - ref) / unit}
    prev = torch.get_num_threads()
    for n in (1, 8):
        torch.set_num_threads(n)
        _, _, gp32, _ = T._oracle_grads(feats, proj, dv, P, R, torch.float32)
        out[f"f32x{n}"] = (float(gp32[KB]) - ref) / unit
    torch.set_num_threads(prev)
    return out, ref, tsum[0]


def main():
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    shape = tuple(int(x) for x in sys.argv[2:7]) if len(sys.argv) >= 7 else (1, 3, 32, 48, 6)
    signs = []
    for s in range(ns):
        o, ref, ts = one(100 + s, shape)
        signs.append(np.sign(o["gpu"]))
        print(f"seed {100 + s}: bias {ref:+.6e}, sum|terms| {ts:.4e}; error / (u sum|terms|): "
              + ", ".join(f"{k} {v:+.4f}" for k, v in o.items()), flush=True)
    print(f"GPU error signs: {signs}")


if __name__ == "__main__":
    main()
