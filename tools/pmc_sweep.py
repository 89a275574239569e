"""Short sweep at a bench geometry for rocprofv3 PMC passes (per-launch HBM traffic).

usage (on the GPU box, one counter set per pass, see MI355X_MICROARCH.md):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
      python tools/pmc_sweep.py --config dtu_eval_1600x1184_n7_d512 --planes 6
  rocprofv3 --pmc WRITE_SIZE ... (same)
then python tools/pmc_summarize.py gpurun_out/pmc_fetch gpurun_out/pmc_write
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from aarmvs import ops, synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=bench.DEFAULT_CONFIG, choices=sorted(bench.CONFIGS))
    ap.add_argument("--planes", type=int, default=6)
    args = ap.parse_args()
    cfg = dict(bench.CONFIGS[args.config])
    cfg["D"] = args.planes
    dev = torch.device("cuda", 0)
    P = {k: torch.from_numpy(v).to(dev) for k, v in syn.sweep_weights(1).items()}
    _, proj, dv, feats = bench.make_inputs(cfg, 1, 0, dev)
    sw = ops.DepthSweep(P, dev)
    sw(feats[0], list(feats[1:]), proj[:, 0], list(proj[:, 1:].unbind(1)), dv, want_depth=True)
    torch.cuda.synchronize()
    print("pmc sweep done", args.config, args.planes)


if __name__ == "__main__":
    main()
