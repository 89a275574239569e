"""Debug aid: omega weights of one plane from the VALU and MFMA omega kernels at a given
size (aarmvs_cost_slice), run twice each; prints repeatability and where they differ
(positions modulo the MFMA kernel's 14 x 30 output tile)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(H, W, N, out):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
    import torch
    import bench
    from aarmvs import ops, synthetic as syn
    dev = torch.device("cuda", 0)
    P = {k: torch.from_numpy(v).to(dev) for k, v in bench.real_weights().items()}
    sc = syn.scene(1, N, H, W, 4, seed=0)
    f = torch.from_numpy(sc["features"]).to(dev)
    proj = torch.from_numpy(sc["proj_matrices"])
    sw = ops.DepthSweep(P, dev)
    res = []
    ops.profile_enable(True)
    ops.profile_reset()
    for _ in range(2):
        x, om = sw.cost_slice(f[0], list(f[1:]), proj[:, 0], list(proj[:, 1:].unbind(1)),
                              torch.from_numpy(sc["depth_values"][:, 1].copy()), want_omega=True)
        torch.cuda.synchronize()
        res.append(om.cpu().numpy())
    prof = ops.profile_read()
    print("TIMING", {k: round(ms / n * 1e3, 1) for k, (n, ms) in prof.items()}, flush=True)
    np.save(out, np.stack(res))


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
        sys.exit(0)
    H, W, N = (int(v) for v in sys.argv[1:4])
    outs = {}
    for var, extra in (("valu", {}), ("mfma", {}), ("mfma_global", {"AARMVS_PIPE_BOX_CAP": "4"})):
        env = dict(os.environ, AARMVS_OMEGA=var.split("_")[0], **extra)
        p = f"/tmp/dbg_{var}.npy"
        r = subprocess.run([sys.executable, __file__, "--child", str(H), str(W), str(N), p], env=env,
                           check=True, timeout=300, capture_output=True, text=True)
        print(var, [ln for ln in r.stdout.splitlines() if ln.startswith("TIMING")])
        outs[var] = np.load(p)
    for var, a in outs.items():
        print(var, "repeatable:", bool(np.array_equal(a[0], a[1])),
              "max run-to-run diff", float(np.abs(a[0] - a[1]).max()))
    dg = np.abs(outs["valu"][0] - outs["mfma_global"][0])
    print("max |valu - mfma_global|", float(dg.max()), "count > 1e-4:", int((dg > 1e-4).sum()))
    d = np.abs(outs["valu"][0] - outs["mfma"][0])   # [nsrc,1,H,W]
    print("max |valu - mfma|", float(d.max()), "mean", float(d.mean()))
    bad = np.argwhere(d > 1e-4)
    print("count > 1e-4:", len(bad), "of", d.size)
    if len(bad):
        v, _, y, x = bad.T
        print("per view:", np.bincount(v, minlength=N - 1).tolist())
        print("y mod 14 hist:", np.bincount(y % 14, minlength=14).tolist())
        print("x mod 30 hist:", np.bincount(x % 30, minlength=30).tolist())
        print("first:", bad[:12].tolist())
    d2 = np.abs(outs["mfma"][0] - outs["mfma"][1])
    badr = np.argwhere(d2 > 0)
    if len(badr):
        v, _, y, x = badr.T
        print("nondeterministic px:", len(badr), "y mod 14:", np.bincount(y % 14, minlength=14).tolist(),
              "x mod 30:", np.bincount(x % 30, minlength=30).tolist())
