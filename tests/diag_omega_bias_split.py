"""Where the GPU's error on omega.reweight_network.2.bias comes from (round 6).
The bias gradient is linear in dL/dx: g_b = sum_d <dL/dx_d, dx_d/db>.  Per seed:
  g64  float64 autograd of the oracle (the reference's arithmetic, exact);
  ghyb float64 autograd of the oracle's cost slice with the GPU's dL/dx fed in plane by plane
       (the regulariser backward's error, projected on the bias);
  ggpu the GPU's value.
ghyb - g64 is the BPTT's share (dL/dx), ggpu - ghyb the cost-slice backward's own (its fp32
omega chain on the recorded t1, the fp32 dot dL/dx . sq, the fixed-order fp64 sums).  In units
of u * sum|dL/dlogit| (u = 2^-24), as test_gpu_bptt's bound.
usage: python tests/diag_omega_bias_split.py SEED [SEED ...]"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
import conftest  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_bptt as T  # noqa: E402

KB = "omega.reweight_network.2.bias"


def run(seed, shape=(1, 3, 32, 48, 6), f32=False, where=False):
    from oracle import sweep_oracle as orc
    B, N, H, W, D = shape
    sc, P, feats, proj, dv, sw, args = T._setup(B, N, H, W, D, seed, 6)
    cost, rec, rel = T._record_forward(sw, args, B, H, W, D)
    R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(seed + 1))
    tsum = [0.0]
    orc.LOGIT_HOOK = lambda z: z.register_hook(lambda g: tsum.__setitem__(0, tsum[0] + float(g.abs().sum())))
    try:
        _, _, gp64, gx64 = T._oracle_grads(feats, proj, dv, P, R, torch.float64)
    finally:
        orc.LOGIT_HOOK = None
    c = cost.detach().clone().requires_grad_(True)
    (torch.softmax(c, 1) * R.to(c.device)).sum().backward()
    _, _, gp, gx = sw.backward(args[0], args[1], rel, dv, rec, c.grad, want_grad_x=True)
    gx = gx.permute(0, 1, 4, 2, 3).double().cpu()            # [D,B,32,H,W]
    # hybrid: float64 cost-slice autograd per plane, fed the GPU's dL/dx
    f64 = feats.double()
    P64 = {k: v.double().clone().requires_grad_(True) for k, v in P.items()}
    rels = [orc.relative_projection(proj[:, v], proj[:, 0]) for v in range(1, N)]
    for d in range(D):
        x = orc.cost_slice(f64[0], [f64[v] for v in range(1, N)], rels, dv[:, d], P64, fast=True)
        x.backward(gx[d])
    unit = 2.0 ** -24 * tsum[0]
    g64, ghyb, ggpu = float(gp64[KB]), float(P64[KB].grad), float(gp[KB])
    gxe = float(torch.linalg.norm(gx - torch.stack(gx64).double()) / torch.linalg.norm(torch.stack(gx64).double()))
    e32 = ""
    if f32:
        prev = torch.get_num_threads()
        errs = []
        for nt in T.F32_THREADS:
            torch.set_num_threads(nt)
            _, _, gp32, _ = T._oracle_grads(feats, proj, dv, P, R, torch.float32)
            errs.append((float(gp32[KB]) - g64) / unit)
        torch.set_num_threads(prev)
        e32 = "; float32 (threads " + ",".join(map(str, T.F32_THREADS)) + "): " + " ".join(f"{e:+.4f}" for e in errs)
    print(f"{shape} seed {seed}: bias {g64:+.6e}; (ggpu - g64) / u sum|t| = {(ggpu - g64) / unit:+.4f} = "
          f"dL/dx share {(ghyb - g64) / unit:+.4f} + cost-slice backward {(ggpu - ghyb) / unit:+.4f}; "
          f"dL/dx rel L2 {gxe:.2e}{e32}", flush=True)
    if where:   # where the dL/dx error sits: per plane, and the largest element
        g64x = torch.stack(gx64).double()
        err = (gx - g64x).abs()
        per = [f"{float(torch.linalg.norm(gx[d] - g64x[d]) / torch.linalg.norm(g64x[d])):.1e}" for d in range(D)]
        i = int(err.argmax())
        idx = np.unravel_index(i, tuple(err.shape))
        print(f"   dL/dx rel L2 per plane {per}; largest |error| {float(err.max()):.3e} at "
              f"[d,b,c,y,x] = {tuple(int(t) for t in idx)} (|ref| max {float(g64x.abs().max()):.3e}); "
              f"elements with |error| > 1e-3 max: {int((err > 1e-3 * float(g64x.abs().max())).sum())}", flush=True)


if __name__ == "__main__":
    # args: SEED[:B,N,H,W,D] ...; env F32=1 adds float32's errors, WHERE=1 the dL/dx error map
    for a in sys.argv[1:]:
        seed, _, shp = a.partition(":")
        shape = tuple(int(x) for x in shp.split(",")) if shp else (1, 3, 32, 48, 6)
        run(int(seed), shape, f32=os.environ.get("F32") == "1", where=os.environ.get("WHERE") == "1")
