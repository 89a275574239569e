"""Times the fusion core (bench.py's fusion_bench) at the headline geometry, optionally for an
alternative library build (AARMVS_LIB).  usage: python tools/fusion_time.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
r = bench.fusion_bench(1184, 1600, 10, torch.device("cuda", 0), False, reps=reps)
print(f"{os.environ.get('AARMVS_LIB', 'in-tree')}: fusion {r['ms_per_view']:.4f} ms per view, "
      f"{r['frac']:.4f} of HBM", flush=True)
