"""Helper of tests/test_gpu_bptt.py::test_backward_schedules_are_bit_identical: one recorded
training sweep and its backward (aarmvs_sweep_backward) at a small geometry spanning two plane
groups (D = 36: 16 + 16 + 4, odd and even planes, both group buffer sets), printing a SHA-256 of every gradient's bytes and saving the
source-feature gradients to argv[1] (.npy) and dL/dref to argv[2].  BWD_DIGEST_REPS repeats the
backward in the process (one digest block per repetition).  Run once per stream schedule
(AARMVS_BWD_PIPE: 0 one stream, 3 the two-stream plane pipeline, 1 with the group stage on a
third stream)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from aarmvs import ops, synthetic as syn  # noqa: E402

B, N, H, W, D = 1, 3, 96, 128, 36
sc = syn.scene(B, N, H, W, D, seed=3)
P = {k: torch.from_numpy(v).cuda() for k, v in syn.sweep_weights(5).items()}
sw = ops.DepthSweep(P, "cuda")
f = torch.from_numpy(sc["features"]).cuda()
proj = torch.from_numpy(sc["proj_matrices"])
dv = torch.from_numpy(sc["depth_values"])
ref, srcs = f[0], [f[v] for v in range(1, N)]
rec = sw.record_buffers(B, H, W, D, "cuda", nsrc=N - 1)
rel = sw.relative(proj[:, 0], [proj[:, v] for v in range(1, N)], B)
cost = torch.empty(B, D, H, W, device="cuda")
sw(ref, srcs, proj[:, 0], [proj[:, v] for v in range(1, N)], dv, want_depth=False, cost_out=cost,
   rel=rel, record=rec)
torch.cuda.synchronize()
print("DIGEST cost", hashlib.sha256(cost.cpu().numpy().tobytes()).hexdigest(), flush=True)
torch.manual_seed(0)
g = torch.randn_like(cost)
want_x = os.environ.get("BWD_DIGEST_NOX") != "1"
reps = int(os.environ.get("BWD_DIGEST_REPS", "1"))
for rep in range(reps):   # the same backward again: every repetition must print the same digests
    g_ref, g_src, g_par, g_x = sw.backward(ref, srcs, rel, dv, rec, g, want_grad_x=want_x)
    if g_x is None:
        g_x = torch.zeros(1)
    torch.cuda.synchronize()
    for name, ts in (("ref", [g_ref]), ("src", g_src), ("params", [g_par[k] for k in sorted(g_par)]),
                     ("x", [g_x])):
        h = hashlib.sha256()
        for t in ts:
            h.update(t.detach().cpu().contiguous().numpy().tobytes())
        print("DIGEST", name, h.hexdigest(), flush=True)
np.save(sys.argv[1], torch.stack(g_src).cpu().numpy())
if len(sys.argv) > 2:
    np.save(sys.argv[2], g_ref.cpu().numpy())
