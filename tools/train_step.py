"""Config-4 training step alone (bench.py's train_bench), for rocprofv3 traces:
python tools/train_step.py [--planes D] [--steps K]."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--planes", type=int, default=192)
ap.add_argument("--steps", type=int, default=2)
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
print(json.dumps(bench.train_bench(dev, D=args.planes, reps=args.steps)), flush=True)
