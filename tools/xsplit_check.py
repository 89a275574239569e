"""The inference sweep with cost_x's pre-staged x (AARMVS_XSPLIT=1, default) against fp32 x
staged by cell 0 itself (AARMVS_XSPLIT=0): the cost volume, depth and confidence must be
bit-identical (same operand bits, same kernels otherwise).  usage: python tools/xsplit_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import ops, synthetic as syn  # noqa: E402


def run(flag, B, N, H, W, D):
    os.environ["AARMVS_XSPLIT"] = flag
    sc = syn.scene(B, N, H, W, D, seed=5)
    P = {k: torch.from_numpy(v).cuda() for k, v in syn.sweep_weights(2).items()}
    sw = ops.DepthSweep(P, "cuda")
    f = torch.from_numpy(sc["features"]).cuda()
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    out = sw(f[0], [f[v] for v in range(1, N)], proj[:, 0], [proj[:, v] for v in range(1, N)], dv,
             want_depth=True, want_cost=True)
    torch.cuda.synchronize()
    return [out["cost"].cpu(), out["depth"].cpu(), out["conf"].cpu()]


ok = True
for shape in [(1, 3, 96, 128, 40), (2, 5, 120, 200, 20), (1, 7, 264, 352, 36)]:
    a, b = run("1", *shape), run("0", *shape)
    eq = [torch.equal(x, y) for x, y in zip(a, b)]
    print(f"{shape}: cost/depth/conf bit-equal {eq}, max|dcost| {float((a[0] - b[0]).abs().max()):.3g}",
          flush=True)
    ok = ok and all(eq)
print("XSPLIT parity", "OK" if ok else "FAILED")
sys.exit(0 if ok else 1)
