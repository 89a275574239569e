"""Driver for rocprofv3 counter passes over the depth-fusion core (fusion_filter_kernel,
csrc/fusion.hip; fusion.py:71-220): bench.py's fusion workload (1600x1184, 10 source views,
aarmvs.synthetic.fusion_views) run `reps` times after one warm-up."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

from aarmvs import fusion, synthetic as syn  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
H, W, nsrc = 1184, 1600, 10
depths, cams, conf = syn.fusion_views(H, W, nsrc, seed=7)
t = [torch.from_numpy(d).cuda() for d in depths]
c = torch.from_numpy(conf).cuda()
for _ in range(1 + args.reps):
    fusion.filter_depth_core(t[0], c, cams[0], t[1:], cams[1:], 0.35)
torch.cuda.synchronize()
print("fusion passes done")
