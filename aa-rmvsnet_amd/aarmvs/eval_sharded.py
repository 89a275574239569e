"""Multi-GPU depth-map inference: the reference's eval.py ``save_depth`` (eval.py:57-170)
with its (scan, ref_view) samples sharded across ranks.

One process per GPU (``torch.distributed.run``; RANK / LOCAL_RANK / WORLD_SIZE from the
environment).  Rank r takes the contiguous slice ``shard_range(len(dataset), r, world)`` of
the eval dataset, runs the drop-in ``EMVSNet(return_depth=True)`` on it (the depth sweep on
libaarmvs) and writes that slice's maps.  There is no collective: the ranks share nothing
but the output directory.

Outputs per sample, as eval.py names them (``filename.format(kind, ext)``):
  depth_est_0/<ref>.pfm     the evidential head's gamma where the head runs (B = 1, D = 32,
                            as eval.py saves it), otherwise the sweep's winner-take-all depth
                            (eval.py writes nothing there: its head raises for D != 32)
  confidence_0/<ref>.pfm    photometric confidence (max prob / exp sum)
  epistemic_0/, aleatoric_0/  where the head runs: 1/sqrt(nu), sqrt(beta (nu+1) / (nu alpha))
eval.py's PNG previews are not written (data_io.save_png is broken on numpy >= 1.24,
SURVEY §8f-4).

usage: python -m torch.distributed.run --nproc-per-node N -m aarmvs.eval_sharded \\
           --testpath DTU --testlist lists/test.txt --loadckpt model.ckpt --outdir out
"""
from __future__ import annotations

import argparse
import ast
import os
import sys
from collections import OrderedDict

import numpy as np
import torch
from torch.utils.data import DataLoader, Subset

from .dist import env, local_device_index, shard_range
from .fusion import save_pfm


def parse_args(argv=None):
    """eval.py's arguments (eval.py:19-46)."""
    ap = argparse.ArgumentParser(description="Predict depth (sharded over ranks)")
    ap.add_argument("--inverse_depth", type=ast.literal_eval, default=False)
    ap.add_argument("--return_depth", type=ast.literal_eval, default=True)
    ap.add_argument("--max_h", type=int, default=512)
    ap.add_argument("--max_w", type=int, default=960)
    ap.add_argument("--image_scale", type=float, default=1.0)
    ap.add_argument("--light_idx", type=int, default=3)
    ap.add_argument("--view_num", type=int, default=7)
    ap.add_argument("--dataset", default="data_eval_transform")
    ap.add_argument("--testpath")
    ap.add_argument("--testlist")
    ap.add_argument("--batch_size", type=int, default=1)
    ap.add_argument("--numdepth", type=int, default=256)
    ap.add_argument("--interval_scale", type=float, default=1.0)
    ap.add_argument("--loadckpt", default=None)
    ap.add_argument("--outdir", default="./outputs")
    return ap.parse_args(argv)


def load_checkpoint(model, path):
    """eval.py:103-113: the checkpoint's 'model' dict with any 'module.' prefix removed,
    loaded strictly.  Tensors only (weights_only=True): nothing in the file is executed."""
    state = torch.load(path, map_location="cpu", weights_only=True)["model"]
    fixed = OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in state.items())
    model.load_state_dict(fixed, strict=True)


def save_dir_for(args) -> str:
    """outdir/<ckpt dir>_<ckpt file> as eval.py:48-52 (outdir alone without a checkpoint)."""
    if not args.loadckpt:
        return args.outdir
    parts = args.loadckpt.split("/")
    return os.path.join(args.outdir, parts[-2] + "_" + parts[-1])


def save_depth(args, rank: int = 0, world: int = 1, device=None, model=None) -> list:
    """Run rank's shard of the eval set; returns the reference-view filenames it wrote."""
    from datasets import find_dataset_def
    from models import EMVSNet
    device = torch.device(device or f"cuda:{local_device_index(env()[1])}")
    if device.type == "cuda":
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        # libaarmvs launches on the current device's stream: make it this rank's GPU
        torch.cuda.set_device(device)
    ds = find_dataset_def(args.dataset)(args.testpath, args.testlist, "test", args.view_num,
                                        args.numdepth, args.interval_scale,
                                        inverse_depth=args.inverse_depth, adaptive_scaling=True,
                                        max_h=args.max_h, max_w=args.max_w, sample_scale=1,
                                        base_image_size=8)
    shard = list(shard_range(len(ds), rank, world))
    loader = DataLoader(Subset(ds, shard), args.batch_size, shuffle=False, num_workers=0,
                        drop_last=False)
    if model is None:
        model = EMVSNet(disparity_level=32, image_scale=args.image_scale, max_h=args.max_h,
                        max_w=args.max_w, return_depth=True)
        if args.loadckpt:
            load_checkpoint(model, args.loadckpt)
    model = model.to(device).eval()
    save_dir = save_dir_for(args)
    written = []
    with torch.no_grad():
        for sample in loader:
            out = model(sample["imgs"].to(device), sample["proj_matrices"].to(device),
                        sample["depth_values"].to(device))
            depth = out["depth"].cpu().numpy()
            conf = out["photometric_confidence"].cpu().numpy()
            ev = out["evidential_prediction"]
            ev = None if ev is None else ev.cpu().numpy()
            for b, filename in enumerate(sample["filename"]):
                path = lambda kind: os.path.join(save_dir, filename.format(kind + "_0", ".pfm"))
                for kind in ("depth_est", "confidence") + (("epistemic", "aleatoric") if ev is not None else ()):
                    os.makedirs(os.path.dirname(path(kind)), exist_ok=True)
                if ev is not None:   # eval.py:143-160 (B == 1)
                    gamma, nu, alpha, beta = ev[0], ev[1], ev[2], ev[3]
                    save_pfm(path("depth_est"), np.ascontiguousarray(gamma, np.float32))
                    save_pfm(path("epistemic"), (1.0 / np.sqrt(nu)).astype(np.float32))
                    save_pfm(path("aleatoric"), np.sqrt(beta * (nu + 1) / nu / alpha).astype(np.float32))
                else:
                    save_pfm(path("depth_est"), np.ascontiguousarray(depth[b], np.float32))
                save_pfm(path("confidence"), np.ascontiguousarray(conf[b], np.float32))
                written.append(filename)
    return written


def main(argv=None) -> int:
    args = parse_args(argv)
    rank, _, world = env()
    written = save_depth(args, rank, world)
    print(f"rank {rank}/{world}: {len(written)} reference views written", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
