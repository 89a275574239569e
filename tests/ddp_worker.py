"""One rank of tests/test_gpu_training.py::test_ddp_world2_gradients_equal_hand_averaged.

Reads RANK / WORLD_SIZE / MASTER_* from the environment (set by the test), runs one DDP
training step of EMVSNet (HIP sweep forward, _SweepTrain backward) on cuda:0 with the gloo
backend (DDP_BACKEND=nccl: RCCL, one rank -- RCCL refuses two ranks on one GPU), then
recomputes every rank's local gradients without DDP and checks that the DDP gradients equal
their average (bit for bit with one rank: the backward is deterministic).  Prints DDP_OK.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "aa-rmvsnet_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402

from aarmvs import synthetic as syn  # noqa: E402


def model(D, H, W):
    from models import EMVSNet
    m = EMVSNet(disparity_level=D, image_scale=1.0, max_h=H, max_w=W, return_depth=False)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    wts = syn.init_weights(shapes, seed=6)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in wts.items()}, strict=True)
    m.feature = nn.Identity()
    return m.cuda()


def sample(rank, B, N, H, W, D):
    sc = syn.scene(B, N, H, W, D, seed=1000 + rank)
    imgs = torch.from_numpy(np.moveaxis(sc["features"], 0, 1).copy()).cuda()
    return imgs, torch.from_numpy(sc["proj_matrices"]).cuda(), torch.from_numpy(sc["depth_values"]).cuda()


def loss_of(prob, D):
    return (prob * torch.linspace(-1.0, 1.0, D, device=prob.device).view(1, D, 1, 1)).sum()


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    backend = os.environ.get("DDP_BACKEND", "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    B, N, H, W, D = 1, 3, 32, 48, 4
    m = model(D, H, W)
    ddp = nn.parallel.DistributedDataParallel(m, device_ids=[0], find_unused_parameters=True)
    imgs, proj, dv = sample(rank, B, N, H, W, D)
    prob, _, _ = ddp(imgs, proj, dv)
    loss_of(prob, D).backward()
    got = {k: p.grad.detach().clone() for k, p in m.named_parameters()
           if k in syn.SWEEP_SHAPES and p.grad is not None}
    local = []
    for r in range(world):
        ref = model(D, H, W)
        i2, p2, d2 = sample(r, B, N, H, W, D)
        pr, _, _ = ref(i2, p2, d2)
        loss_of(pr, D).backward()
        local.append({k: p.grad for k, p in ref.named_parameters() if k in got})
    assert len(got) == len(syn.SWEEP_SHAPES), sorted(set(syn.SWEEP_SHAPES) - set(got))
    expects = {k: sum(lg[k] for lg in local) / world for k in got}
    gmax = max(float(e.abs().max()) for e in expects.values())
    for k, g in got.items():
        if world == 1:
            assert torch.equal(g, expects[k]), k
            continue
        # 1e-5 of max(own scale, 1e-3 x the largest): the average of two ranks' gradients is
        # summed in another order than DDP's all-reduce; conv_0.bias's true gradient is 0
        # (softmax over D), so it holds cancellation noise only
        scale = max(float(expects[k].abs().max()), 1e-3 * gmax)
        err = float((g - expects[k]).abs().max())
        assert err <= 1e-5 * scale, (k, err, scale)
    dist.destroy_process_group()
    print("DDP_OK", rank, flush=True)


if __name__ == "__main__":
    main()
