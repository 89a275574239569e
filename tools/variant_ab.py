"""A/B of kernel variants selected by environment variables (measurement tooling).

Runs the headline sweep (1600x1184, N=7, model_dtu_v2 weights) over the first P planes once
per variant in child processes, and prints per-kernel average times (hipEvents per launch,
serialised) and the whole-sweep ms per plane (two streams, no events), plus the max
difference of each variant's cost volume from the first variant's.

  python tools/variant_ab.py --planes 24 AARMVS_OMEGA=valu AARMVS_OMEGA=mfma
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(planes, N, H, W, B):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
    import time
    import numpy as np
    import torch
    import bench
    from aarmvs import ops, synthetic as syn
    dev = torch.device("cuda", 0)
    P = {k: torch.from_numpy(v).to(dev) for k, v in bench.real_weights().items()}
    sc = syn.scene(B, N, H, W, planes, seed=0)
    feats = torch.from_numpy(sc["features"]).to(dev)
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])
    sw = ops.DepthSweep(P, dev, overlap=os.environ.get("AB_OVERLAP", "1") == "1")
    args = (feats[0], list(feats[1:]), proj[:, 0], list(proj[:, 1:].unbind(1)), dv)
    out = sw(*args, want_cost=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        sw(*args, want_cost=False)
    torch.cuda.synchronize()
    ms_plane = (time.perf_counter() - t0) / 3 / planes * 1e3
    sw.overlap = False
    ops.profile_enable(True)
    ops.profile_reset()
    sw(*args, want_cost=False)
    torch.cuda.synchronize()
    prof = ops.profile_read()
    ops.profile_enable(False)
    np.save(os.environ["AB_OUT"], out["cost"].cpu().numpy())
    print(json.dumps({"ms_per_plane": ms_plane,
                      "kernels_us": {k: round(ms / n * 1e3, 2) for k, (n, ms) in prof.items()}}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--planes", type=int, default=24)
    ap.add_argument("--config", default="1184x1600x7")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    H, W, N = (int(x) for x in a.config.split("x"))
    if a.child:
        child(a.planes, N, H, W, a.batch)
        return
    import numpy as np
    base = None
    for i, var in enumerate(a.variants or ["default"]):
        env = dict(os.environ)
        for kv in var.split(","):
            if "=" in kv:
                k, v = kv.split("=", 1)
                env[k] = v
        env["AB_OUT"] = f"/tmp/ab_{i}.npy"
        r = subprocess.run([sys.executable, __file__, "--child", "--planes", str(a.planes),
                            "--config", a.config, "--batch", str(a.batch)],
                           env=env, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(var, "FAILED", r.stdout[-2000:], r.stderr[-3000:], flush=True)
            sys.exit(1)
        res = json.loads(r.stdout.strip().splitlines()[-1])
        cost = np.load(env["AB_OUT"])
        if base is None:
            base = cost
        res["cost_max_diff_vs_first"] = float(np.abs(cost - base).max())
        res["finite"] = bool(np.isfinite(cost).all())
        print(var, json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
