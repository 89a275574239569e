"""Diagnostic: full sweep vs the same sweep split into two d_range calls (test_gpu_configs'
continuation check) -- first differing plane and the size of the differences."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd"), os.path.join(ROOT, "tests")]
from aarmvs import ops, synthetic as syn  # noqa: E402
from test_gpu_configs import real_P, _views  # noqa: E402

B, N, H, W, D = 1, 5, 600, 800, int(os.environ.get("DBG_D", "256"))
sc = syn.scene(B, N, H, W, D, seed=N * 100 + 256)
P = real_P()
fd = torch.from_numpy(sc["features"]).cuda()
proj = torch.from_numpy(sc["proj_matrices"])
dv = torch.from_numpy(sc["depth_values"])
args = _views(fd, proj)
for overlap in (True, False):
    sw = ops.DepthSweep({n: v.cuda() for n, v in P.items()}, "cuda", overlap=overlap)
    full = sw(*args, dv, want_cost=True)["cost"]
    full2 = sw(*args, dv, want_cost=True)["cost"]
    cost = torch.empty(B, D, H, W, device="cuda")
    cut = D // 3
    sw(*args, dv, d_range=(0, cut), cost_out=cost, want_depth=False)
    sw(*args, dv, d_range=(cut, D), cost_out=cost)
    torch.cuda.synchronize()
    for name, other in (("rerun", full2), ("split", cost)):
        d = (full - other).abs().amax(dim=(0, 2, 3)).cpu().numpy()
        bad = np.nonzero(d)[0]
        print(f"overlap={overlap} {name}: {len(bad)} differing planes"
              + (f", first {bad[0]}, max {d.max():.3e}, planes {bad[:12].tolist()}" if len(bad) else ""),
              flush=True)
