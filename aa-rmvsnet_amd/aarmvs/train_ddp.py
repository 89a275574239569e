"""Multi-GPU training driver: the reference's train.py loop (train.py:147-262) as one
process per GPU with DistributedDataParallel.

Each rank takes its shard of the training set (DistributedSampler, one or more samples per
GPU), runs the drop-in ``EMVSNet`` train forward (FeatNet + the HIP sweep), the loss, and the
backward; DDP's gradient all-reduce (``nccl`` = RCCL over xGMI; ``gloo`` in the shared-GPU
rehearsal, ``aarmvs.dist.shared_gpu``) is the only exchange.  As in train.py: Adam at
``--lr``, CosineAnnealingLR(T_max=epochs, eta_min=2e-6) stepped per epoch, checkpoints
``{'epoch', 'model', 'optimizer'}`` as ``logdir/model_{epoch:0>6}.ckpt`` (rank 0; the
wrapped model's keys, ``module.``-prefixed under DDP as under train.py's DataParallel), and
``--resume`` from the latest of them.

Loss: ``loss_der`` on the evidential outputs where the head runs (B = 1, D = 32: train.py:297-
304), otherwise the core ``mvsnet_cls_loss`` (the head cannot train at D = 192).
tensorboard summaries and the per-epoch test pass of train.py are not reproduced.

usage: python -m torch.distributed.run --nproc-per-node 8 -m aarmvs.train_ddp \\
           --trainpath DTU --trainlist lists/train.txt --numdepth 192 --logdir ckpt
"""
from __future__ import annotations

import argparse
import ast
import os
import sys
import time
from collections import OrderedDict

import torch
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

from .dist import env, init_process_group, local_device_index


def parse_args(argv=None):
    """train.py's arguments (train.py:28-68) that the loop uses, plus --max_steps."""
    ap = argparse.ArgumentParser(description="AA-RMVSNet training (DDP, one process per GPU)")
    ap.add_argument("--inverse_depth", type=ast.literal_eval, default=False)
    ap.add_argument("--origin_size", type=ast.literal_eval, default=False)
    ap.add_argument("--max_h", type=int, default=512)
    ap.add_argument("--max_w", type=int, default=640)
    ap.add_argument("--view_num", type=int, default=3)
    ap.add_argument("--image_scale", type=float, default=0.25)
    ap.add_argument("--dataset", default="dtu_yao")
    ap.add_argument("--trainpath")
    ap.add_argument("--trainlist")
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--lr", type=float, default=0.001)
    ap.add_argument("--batch_size", type=int, default=1, help="samples per GPU per step")
    ap.add_argument("--numdepth", type=int, default=192)
    ap.add_argument("--interval_scale", type=float, default=1.06)
    ap.add_argument("--loadckpt", default=None)
    ap.add_argument("--logdir", default="./checkpoints/debug")
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--summary_freq", type=int, default=20)
    ap.add_argument("--save_freq_checkpoint", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max_steps", type=int, default=0, help="stop each epoch after this many steps (0: all)")
    ap.add_argument("--train_light_idx", type=int, default=-1,
                    help="light index of the training images (train.py: -1, all seven)")
    return ap.parse_args(argv)


def _strip_module(state):
    return OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in state.items())


def train(args, rank: int = 0, world: int = 1, device=None, log=print) -> dict:
    """Runs train.py's epochs on this rank's shard; returns {'losses', 'checkpoints'}."""
    from datasets import find_dataset_def
    from evidential.models import loss_der
    from models import EMVSNet, mvsnet_cls_loss
    device = torch.device(device or f"cuda:{local_device_index(env()[1])}")
    if device.type == "cuda":
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        # libaarmvs launches on the current device's stream: make it this rank's GPU
        torch.cuda.set_device(device)
    torch.manual_seed(args.seed)
    init_process_group(device)
    ds = find_dataset_def(args.dataset)(args.trainpath, args.trainlist, "train", args.view_num,
                                        args.numdepth, args.interval_scale, args.inverse_depth,
                                        args.origin_size, args.train_light_idx, args.image_scale)
    sampler = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=args.seed,
                                 drop_last=True)
    loader = DataLoader(ds, args.batch_size, sampler=sampler, num_workers=0, drop_last=True)
    model = EMVSNet(disparity_level=args.numdepth, image_scale=args.image_scale,
                    max_h=args.max_h, max_w=args.max_w)
    if args.loadckpt:   # train.py:150-170: tensors only, any 'module.' prefix removed
        state = torch.load(args.loadckpt, map_location="cpu", weights_only=True)["model"]
        model.load_state_dict(_strip_module(state), strict=True)
    model = model.to(device)
    head_runs = args.batch_size == 1 and args.numdepth == 32
    if world > 1:
        # the evidential head's parameters get no gradient where it does not run
        model = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[device.index] if torch.distributed.get_backend() == "nccl" else None,
            find_unused_parameters=not head_runs)
    optimizer = torch.optim.Adam(model.parameters(), lr=args.lr)
    start_epoch = 0
    if args.resume:   # train.py:186-197
        saved = sorted((f for f in os.listdir(args.logdir) if f.endswith(".ckpt")),
                       key=lambda f: int(f.split("_")[-1].split(".")[0]))
        state = torch.load(os.path.join(args.logdir, saved[-1]), map_location="cpu", weights_only=True)
        # a checkpoint saved at another world size has (or lacks) DDP's 'module.' prefix
        core = model.module if isinstance(model, torch.nn.parallel.DistributedDataParallel) else model
        core.load_state_dict(_strip_module(state["model"]))
        optimizer.load_state_dict(state["optimizer"])
        start_epoch = state["epoch"] + 1
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=args.epochs, eta_min=2e-06)
    for _ in range(start_epoch):
        sched.step()
    if rank == 0:
        os.makedirs(args.logdir, exist_ok=True)
    losses, ckpts = [], []
    for epoch in range(start_epoch, args.epochs):
        sampler.set_epoch(epoch)
        for step, sample in enumerate(loader):
            if args.max_steps and step >= args.max_steps:
                break
            t0 = time.time()
            model.train()
            optimizer.zero_grad()
            s = {k: v.to(device) if torch.is_tensor(v) else v for k, v in sample.items()}
            prob, evidential, _ = model(s["imgs"], s["proj_matrices"], s["depth_values"])
            if evidential is not None:   # train.py:297-304
                loss = loss_der({"probability_volume": prob, "evidential_prediction": evidential},
                                s["depth"], s["mask"], s["depth_values"])[0]
            else:
                loss = mvsnet_cls_loss(prob, s["depth"], s["mask"], s["depth_values"])[0]
            loss.backward()
            optimizer.step()
            losses.append(float(loss))
            if rank == 0 and step % args.summary_freq == 0:
                log("Epoch {}/{}, Iter {}/{}, LR {}, train loss = {:.3f}, time = {:.3f}".format(
                    epoch, args.epochs, step, len(loader), optimizer.param_groups[0]["lr"],
                    losses[-1], time.time() - t0))
        sched.step()
        if rank == 0 and (epoch + 1) % args.save_freq_checkpoint == 0:   # train.py:232-237
            path = "{}/model_{:0>6}.ckpt".format(args.logdir, epoch)
            torch.save({"epoch": epoch, "model": model.state_dict(),
                        "optimizer": optimizer.state_dict()}, path)
            ckpts.append(path)
    return {"losses": losses, "checkpoints": ckpts}


def main(argv=None) -> int:
    args = parse_args(argv)
    rank, _, world = env()
    out = train(args, rank, world)
    print(f"rank {rank}/{world}: {len(out['losses'])} steps, last loss "
          f"{out['losses'][-1] if out['losses'] else float('nan'):.4f}", file=sys.stderr)
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
