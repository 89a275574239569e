"""Training-step profile aid: one config-4 training step (640x512, N=3, D=16) after a warm-up,
for rocprofv3 --kernel-trace --stats (GPU busy time vs wall time of the step)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import bench  # noqa: E402

r = bench.train_bench(torch.device("cuda:0"), planes=(8, 16), reps=1)
print(r, flush=True)
