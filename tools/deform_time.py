"""Times the deformable-conv sampling kernels (aarmvs_deform_sample forward and backward) at
FeatNet's full resolution for config 4 (640x512, 32 channels), for the in-tree library or
AARMVS_LIB.  usage: python tools/deform_time.py [H W]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import ops  # noqa: E402

H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (512, 640)
torch.manual_seed(0)
x = torch.randn(1, H, W, 32, device="cuda", requires_grad=True)
off = (torch.randn(1, 18, H, W, device="cuda") * 1.5).requires_grad_(True)
m = torch.rand(1, 9, H, W, device="cuda").requires_grad_(True)
gv = torch.randn(1, H * W, 288, device="cuda")
for _ in range(2):
    v = ops.deform_sample(x, off, m, 1, 1)
    v.backward(gv)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
R = 10
e[0].record()
for _ in range(R):
    v = ops.deform_sample(x, off, m, 1, 1)
e[1].record()
for _ in range(R):
    x.grad = None
    torch.autograd.grad(v, (x, off, m), gv, retain_graph=True)
e[2].record()
torch.cuda.synchronize()
g = torch.autograd.grad(v, (x, off, m), gv, retain_graph=True)
print(f"{os.environ.get('AARMVS_LIB', 'in-tree')}: {H}x{W} forward {e[0].elapsed_time(e[1]) / R:.3f} ms, "
      f"backward {e[1].elapsed_time(e[2]) / R:.3f} ms; |gx| {float(g[0].double().abs().sum()):.6e} "
      f"|goff| {float(g[1].double().abs().sum()):.6e} |gm| {float(g[2].double().abs().sum()):.6e}", flush=True)
