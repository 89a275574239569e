"""Count GPU-vs-oracle fusion mask mismatches per case (measurement tooling)."""
import sys
import numpy as np
import torch
sys.path[:0] = [".", "aa-rmvsnet_amd"]
from oracle import fusion_oracle as fo
from aarmvs import fusion, synthetic as syn

for (H, W, nsrc, seed) in [(96, 128, 10, 0), (75, 101, 4, 1), (40, 52, 1, 2), (300, 400, 10, 3)]:
    depths, cams, conf = syn.fusion_views(H, W, nsrc, seed=seed)
    photo, geo, final, avg = fo.filter_depth_core(depths[0], conf, cams[0], depths[1:], cams[1:], 0.35)
    t = [torch.from_numpy(d).cuda() for d in depths]
    g = fusion.filter_depth_core(t[0], torch.from_numpy(conf).cuda(), cams[0], t[1:], cams[1:], 0.35)
    gp, gg, gf, ga = (x.cpu().numpy() for x in g)
    bad = np.argwhere(gg != geo)
    print(H, W, nsrc, "geo mismatches", len(bad), "final", int((gf != final).sum()),
          "avg max diff on same", float(np.abs(ga - avg)[gg == geo].max()), bad[:5].tolist(), flush=True)
