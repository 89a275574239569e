"""Digest of an eval sweep's outputs at 640x512, N=3, PROBE_D planes (default 48): run under
different environment switches (AARMVS_OMEGA_IPB, AARMVS_NPL, ...) to confirm a schedule
change is bit-identical."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import ops, synthetic as syn  # noqa: E402

B, N, H, W, D = 1, 3, 512, 640, int(os.environ.get("PROBE_D", "48"))
sc = syn.scene(B, N, H, W, D, seed=0)
P = {k: torch.from_numpy(v).cuda() for k, v in syn.sweep_weights(1).items()}
sw = ops.DepthSweep(P, "cuda")
f = torch.from_numpy(sc["features"]).cuda()
proj = torch.from_numpy(sc["proj_matrices"])
dv = torch.from_numpy(sc["depth_values"])
cost = torch.empty(B, D, H, W, device="cuda")
out = sw(f[0], [f[v] for v in range(1, N)], proj[:, 0], [proj[:, v] for v in range(1, N)], dv,
         want_depth=True, cost_out=cost)
torch.cuda.synchronize()
ts = [cost] + [out[k] for k in sorted(out) if torch.is_tensor(out[k])]
dig = hashlib.sha256(b"".join(t.detach().cpu().contiguous().numpy().tobytes() for t in ts)).hexdigest()
env = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("AARMVS_"))
print(f"[{env}] sweep digest {dig[:16]}", flush=True)
