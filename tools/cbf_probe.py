"""Backward timing at 640x512, N=3: the whole aarmvs_sweep_backward per call over PROBE_D planes
(default 16, one plane group) taken from the first planes of a PROBE_OF-plane sweep (default
192: config 4's plane spacing), with CUDA events; run once per library build (AARMVS_LIB) to
compare variants."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import ops, synthetic as syn  # noqa: E402

B, N, H, W, D = 1, 3, 512, 640, int(os.environ.get("PROBE_D", "16"))
sc = syn.scene(B, N, H, W, int(os.environ.get("PROBE_OF", "192")), seed=0)
sc["depth_values"] = sc["depth_values"][:, :D].copy()
P = {k: torch.from_numpy(v).cuda() for k, v in syn.sweep_weights(1).items()}
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
torch.manual_seed(0)
g = torch.randn_like(cost)
out = sw.backward(ref, srcs, rel, dv, rec, g)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    sw.backward(ref, srcs, rel, dv, rec, g)
e1.record()
torch.cuda.synchronize()
chk = float(out[0].double().abs().sum()) + sum(float(x.double().abs().sum()) for x in out[1])
import hashlib  # noqa: E402
dig = hashlib.sha256(b"".join(t.detach().cpu().contiguous().numpy().tobytes()
                              for t in [out[0], *out[1], *[out[2][k] for k in sorted(out[2])]])).hexdigest()[:12]
print(f"{os.environ.get('AARMVS_LIB', 'in-tree')}: backward {e0.elapsed_time(e1) / 3:8.2f} ms "
      f"({D} planes) |g_feat| {chk:.6e} digest {dig}", flush=True)
