"""Where two omega_conv variants differ (debug tooling): one cost slice with each variant
(AARMVS_OMEGA values, read at every launch), the omega weights compared per pixel and the
differing pixels binned by their position in the 14x30 output tile of omega_mfma.

  python tools/omega_diff.py mfma mfmadb
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import bench  # noqa: E402
from aarmvs import ops, synthetic as syn  # noqa: E402


def main():
    a, b = sys.argv[1:3]
    H, W, N = 296, 400, 4
    dev = torch.device("cuda", 0)
    P = {k: torch.from_numpy(v).to(dev) for k, v in bench.real_weights().items()}
    sc = syn.scene(1, N, H, W, 8, seed=0)
    feats = torch.from_numpy(sc["features"]).to(dev)
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    sw = ops.DepthSweep(P, dev)
    outs = {}
    for var in (a, b):
        os.environ["AARMVS_OMEGA"] = var
        x, om = sw.cost_slice(feats[0], list(feats[1:]), proj[:, 0], list(proj[:, 1:].unbind(1)),
                              dv[:, 3], want_omega=True)
        torch.cuda.synchronize()
        outs[var] = (x.cpu().numpy(), om.cpu().numpy())
    dx = np.abs(outs[a][0] - outs[b][0]).max()
    do = np.abs(outs[a][1] - outs[b][1])   # [nsrc, B, H, W]
    print("x max diff", dx, "omega max diff", do.max())
    bad = do.max(axis=(0, 1)) > 1e-6
    ys, xs = np.nonzero(bad)
    print("differing pixels", len(ys), "of", H * W)
    if len(ys):
        print("row-in-tile hist", np.bincount(ys % 14, minlength=14).tolist())
        print("col-in-tile hist", np.bincount(xs % 30, minlength=30).tolist())
        print("per view", [(int((do[v] > 1e-6).sum())) for v in range(do.shape[0])])
        print("first", list(zip(ys[:10].tolist(), xs[:10].tolist())))


if __name__ == "__main__":
    main()
