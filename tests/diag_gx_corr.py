"""CPU half of the dL/dx error bisection (no GPU): the omega gradient g_theta = sum_d <dL/dx_d,
dx_d/dtheta> is linear in dL/dx, so an error e_d in dL/dx changes it by sum_d <e_d, K_d> with
K_d = dx_d/dtheta (forward-mode AD of the oracle's cost slice in float64).  Splits that change
by plane, channel, batch element and pixel position for the HIP dL/dx (gpurun_out/<dump>.npz
from tests/diag_gx_dump.py) and for float32 CPU autograd, both against float64.
usage: python tests/diag_gx_corr.py gpurun_out/gx_dump_r04c.npz [param]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from aarmvs import synthetic as syn  # noqa: E402
from oracle import sweep_oracle as orc  # noqa: E402
import test_gpu_bptt as T  # noqa: E402

torch.set_num_threads(8)
dump = np.load(sys.argv[1])
pname = sys.argv[2] if len(sys.argv) > 2 else "omega.reweight_network.2.bias"
shapes = [(1, 3, 32, 48, 6), (2, 4, 24, 40, 5)]
for i, (B, N, H, W, D) in enumerate(shapes):
    sc = syn.scene(B, N, H, W, D, seed=11 + D)
    P = {k: torch.from_numpy(v) for k, v in syn.sweep_weights(6).items()}
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(5))
    _, _, gp64, gx64 = T._oracle_grads(feats, proj, dv, P, R, torch.float64)
    _, _, gp32, gx32 = T._oracle_grads(feats, proj, dv, P, R, torch.float32)
    gx64 = np.stack([g.numpy() for g in gx64])
    gx32 = np.stack([g.double().numpy() for g in gx32])
    gxg = dump[f"gx{i}"].astype(np.float64)
    rels = [orc.relative_projection(proj[:, v], proj[:, 0]) for v in range(1, N)]
    P64 = {k: v.double() for k, v in P.items()}
    fd = feats.double()
    K = []
    for d in range(D):
        def f(b):
            Q = dict(P64)
            Q[pname] = b
            return orc.cost_slice(fd[0], [fd[v] for v in range(1, N)], rels, dv[:, d], Q, fast=True)
        _, t = torch.func.jvp(f, (P64[pname],), (torch.ones_like(P64[pname]),))
        K.append(t.numpy())
    K = np.stack(K)   # [D,B,32,H,W] (for a vector parameter: along the all-ones direction)
    g_true = float((gx64 * K).sum())
    print(f"shape {i} {(B, N, H, W, D)}: <dL/dx, K> float64 {g_true:.6e}  sum|.| {np.abs(gx64 * K).sum():.3e}")
    for tag, g in (("gpu", gxg), ("cpu32", gx32)):
        e = (g - gx64) * K
        print(f"  {tag:5s} total {e.sum() / abs(g_true):+.3e} rel | L2(e_gx) {np.linalg.norm(g - gx64) / np.linalg.norm(gx64):.3e}")
        print("     per plane  ", " ".join(f"{e[d].sum() / abs(g_true):+.2e}" for d in range(D)))
        print("     per batch  ", " ".join(f"{e[:, b].sum() / abs(g_true):+.2e}" for b in range(B)))
        pc = e.sum(axis=(0, 1, 3, 4)) / abs(g_true)
        print("     channels top", " ".join(f"{c}:{pc[c]:+.1e}" for c in np.argsort(-np.abs(pc))[:6]))
        sp = e.sum(axis=(0, 1, 2)) / abs(g_true)
        border = np.zeros((H, W), bool)
        border[:2] = border[-2:] = True
        border[:, :2] = border[:, -2:] = True
        print(f"     border px {sp[border].sum():+.2e} interior {sp[~border].sum():+.2e}")
        cols = sp.sum(axis=0)
        rows = sp.sum(axis=1)
        print("     cols top", " ".join(f"{c}:{cols[c]:+.1e}" for c in np.argsort(-np.abs(cols))[:6]))
        print("     rows top", " ".join(f"{r}:{rows[r]:+.1e}" for r in np.argsort(-np.abs(rows))[:6]))
        # correlation of the error with dL/dx itself and with x-like quantities
        ee = (g - gx64).ravel()
        print(f"     corr(e_gx, gx64) {np.corrcoef(ee, gx64.ravel())[0, 1]:+.3f}   corr(e_gx, K) {np.corrcoef(ee, K.ravel())[0, 1]:+.3f}")
