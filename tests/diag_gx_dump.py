"""GPU half of the dL/dx error bisection: runs test_gpu_bptt's backward at one shape and saves
the HIP dL/dx per plane ([D,B,32,H,W]) and the recorded cost volume, dL/dcost and the record's cost slices and states, for the CPU-side analysis
in tests/diag_gx_corr.py (which needs no GPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_bptt as T  # noqa: E402

shapes = [(1, 3, 32, 48, 6), (2, 4, 24, 40, 5)]
out = {}
for i, (B, N, H, W, D) in enumerate(shapes):
    sc, P, feats, proj, dv, sw, args = T._setup(B, N, H, W, D, 11 + D, 6)
    cost, rec, rel = T._record_forward(sw, args, B, H, W, D)
    R = torch.randn(B, D, H, W, generator=torch.Generator().manual_seed(5))
    prob = torch.softmax(cost, dim=1)
    Rd = R.to("cuda")
    gcost = prob * (Rd - (Rd * prob).sum(dim=1, keepdim=True))
    _, _, _, gx = sw.backward(args[0], args[1], rel, dv, rec, gcost, regulariser_only=True, want_grad_x=True)
    out[f"gx{i}"] = gx.permute(0, 1, 4, 2, 3).cpu().numpy()
    out[f"cost{i}"] = cost.cpu().numpy()
    out[f"gcost{i}"] = gcost.cpu().numpy()
    out[f"rec_x{i}"] = rec["x"].view(torch.float32).cpu().numpy()
    out[f"rec_state{i}"] = rec["state"].view(torch.float32).cpu().numpy()
np.savez_compressed(os.path.join(ROOT, "gpurun_out", sys.argv[1] if len(sys.argv) > 1 else "gx_dump.npz"), **out)
print("saved")
