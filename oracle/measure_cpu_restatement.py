"""Time the CPU restatement (oracle/sweep_oracle.py, fast=True: the form bench.py's
cpu_baseline runs) beside the imported reference itself (EMVSNet's eval depth loop,
models/drmvsnet.py:300-345) on the same inputs at the headline size: SURVEY §8d asks the
timed restatement to run within +-20% of the reference's per-plane time.

TEST/MEASUREMENT INFRASTRUCTURE: runs only in the build container (imports the reference
from /root/reference with the same in-process patches as tests/golden/make_golden.py).
Per-plane time = (t(D = 1 + K) - t(D = 1)) / K for the reference (its forward runs whole
sweeps), and the mean of planes 1..K for the restatement (plane 0 is its warm-up).

  python oracle/measure_cpu_restatement.py [K]   -> profiles/r02_cpu_restatement_vs_reference.json
"""
from __future__ import annotations

import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    threads = min(8, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    import make_golden as mg          # reference import helpers (build container only)
    sys.path.insert(0, os.path.join(REPO, "aa-rmvsnet_amd"))
    from aarmvs import synthetic as syn
    from oracle import sweep_oracle as orc
    drm, _ = mg.import_reference()
    B, N, H, W = 1, 7, 1184, 1600
    g = np.load(os.path.join(REPO, "tests", "golden", "real_weights_sweep.npz"), allow_pickle=False)
    P = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w:")}
    sc = syn.scene(B, N, H, W, 1 + K, seed=0)
    feats = torch.from_numpy(sc["features"])
    proj = torch.from_numpy(sc["proj_matrices"])
    dv = torch.from_numpy(sc["depth_values"])

    model = drm.EMVSNet(disparity_level=1 + K, image_scale=1.0, max_h=H, max_w=W, return_depth=True)
    model.load_state_dict(P, strict=False)
    model.feature = nn.Identity()
    model.evidential = mg._NoEvidential()
    model.eval()
    imgs = feats.permute(1, 0, 2, 3, 4).contiguous()
    ref_t = {}
    with torch.no_grad():
        for D in (1, 1 + K):
            t0 = time.perf_counter()
            model(imgs, proj, dv[:, :D].contiguous())
            ref_t[D] = time.perf_counter() - t0
    ref_plane = (ref_t[1 + K] - ref_t[1]) / K

    times = []
    orc.sweep(feats[0], list(feats[1:]), proj[:, 0], list(proj[:, 1:].unbind(1)), dv, P,
              want_volume=True, fast=True, plane_times=times)
    port_plane = float(np.mean(times[1:]))
    res = {
        "workload": "dtu_eval_1600x1184_n7_d512 (B=1), model_dtu_v2 weights, features ~N(0,1)",
        "cpu": platform.processor() or "unknown",
        "threads": threads,
        "timed_planes": K,
        "reference_s_per_plane": round(ref_plane, 3),
        "reference_runs_s": {f"D={d}": round(t, 3) for d, t in ref_t.items()},
        "restatement_s_per_plane": round(port_plane, 3),
        "restatement_plane_times_s": [round(t, 3) for t in times],
        "ratio_restatement_over_reference": round(port_plane / ref_plane, 3),
        "torch": torch.__version__,
    }
    try:
        with open("/proc/cpuinfo") as f:
            res["cpu"] = next(ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    out = os.path.join(REPO, "profiles", "r02_cpu_restatement_vs_reference.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
