"""Diagnostic: split the backward's error between the regulariser (dL/dx) and the cost-slice
part.  float64 CPU autograd of the oracle's cost slice is driven by (a) float64 dL/dx and (b)
the GPU's dL/dx; the GPU's cost-slice parameter gradients are compared with both."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import sweep_oracle as orc  # noqa: E402
import test_gpu_bptt as T  # noqa: E402

B, N, H, W, D = [int(v) for v in os.environ.get("SHAPE", "1,3,32,48,6").split(",")]
if os.environ.get("ROUND_W"):
    # experiment: cell and deconv weights made exactly representable by the kernels' two fp16
    # terms (after their power-of-two scales), in the GPU and the CPU runs alike
    from aarmvs import ops, synthetic as syn

    def rounded(w, dec):
        mx = float(w.abs().max())
        e = (14 - int(np.floor(np.log2(mx)))) if dec else int(np.floor(np.log2(16384.0 / mx)))
        v = w.double() * 2.0 ** e
        hi = v.half().double()
        lo = (v - hi).float().half().double()
        return ((hi + lo) * 2.0 ** -e).float()

    orig = T._setup

    def _setup(*a, **k):
        sc, P, feats, proj, dv, sw, args = orig(*a, **k)
        for key in list(P):
            if (".cell_list." in key or ".deconv_" in key and ".conv." in key) and key.endswith("weight"):
                P[key] = rounded(P[key], ".deconv_" in key)
        sw = ops.DepthSweep({k2: v.to("cuda") for k2, v in P.items()}, "cuda")
        return sc, P, feats, proj, dv, sw, args
    T._setup = _setup
sc, P, feats, proj, dv, sw, args = T._setup(B, N, H, W, D, 11 + D, 6)
cost, rec, rel = T._record_forward(sw, args, B, H, W, D)
R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(5))
prob64, gf64, gp64, gx64 = T._oracle_grads(feats, proj, dv, P, R, torch.float64)
prob = torch.softmax(cost, dim=1)
Rd = R.to("cuda")
gcost = prob * (Rd - (Rd * prob).sum(dim=1, keepdim=True))
_, _, gp_r, gx = sw.backward(args[0], args[1], rel, dv, rec, gcost, regulariser_only=True, want_grad_x=True)
g_ref, g_src, gp, _ = sw.backward(args[0], args[1], rel, dv, rec, gcost)
gx_gpu = gx.permute(0, 1, 4, 2, 3).double().cpu()


def cost_slice_grads(gxs, dtype):
    fc = feats.to(dtype).clone().requires_grad_(True)
    Pp = {k: v.detach().to(dtype).clone().requires_grad_(True) for k, v in P.items()}
    rels = [orc.relative_projection(proj[:, v], proj[:, 0]) for v in range(1, N)]
    tot = 0
    for d in range(D):
        x = orc.cost_slice(fc[0], [fc[v] for v in range(1, N)], rels, dv[:, d], Pp, fast=True)
        tot = tot + (x * gxs[d].to(dtype)).sum()
    tot.backward()
    return fc.grad, {k: v.grad for k, v in Pp.items() if k.startswith("omega.")}


_, pa = cost_slice_grads([g for g in gx64], torch.float64)
_, pb = cost_slice_grads([g for g in gx_gpu], torch.float64)
_, pc = cost_slice_grads([g.float() for g in gx64], torch.float32)
for k in pa:
    a, b, c, g = pa[k].numpy(), pb[k].numpy(), pc[k].double().numpy(), gp[k].double().cpu().numpy()
    print(f"{k:44s} gpu-vs-a {T.rel_l2(g, a):.3e} gpu-vs-b {T.rel_l2(g, b):.3e} "
          f"b-vs-a {T.rel_l2(b, a):.3e} cpu32(a)-vs-a {T.rel_l2(c, a):.3e}  |a| {np.abs(a).max():.3e}")

# per plane: relative L2 and relative mean error of dL/dx (GPU and float32 CPU autograd vs float64)
_, _, _, gx32 = T._oracle_grads(feats, proj, dv, P, R, torch.float32)
for d in range(D):
    a = gx64[d].numpy()
    g = gx_gpu[d].numpy()
    c = gx32[d].double().numpy()
    print(f"plane {d}: l2 gpu {T.rel_l2(g, a):.3e} cpu32 {T.rel_l2(c, a):.3e} | mean a {a.mean():+.4e} "
          f"gpu-a {(g - a).mean():+.3e} cpu32-a {(c - a).mean():+.3e} | per-channel mean err gpu "
          f"{np.abs((g - a).mean(axis=(0, 2, 3))).max():.2e} cpu {np.abs((c - a).mean(axis=(0, 2, 3))).max():.2e}")
