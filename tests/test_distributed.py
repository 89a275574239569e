"""Multi-process CPU tests (gloo, world_size 2) of the N>1 paths: reference-view
sharding + max-over-ranks timing (inference, no data-path collective) and DDP gradient
averaging of the regulariser (training, the one all-reduce per step)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aarmvs.dist import max_over_ranks, shard_range


def test_shard_range_covers_every_item_once():
    for n in (0, 1, 7, 8, 9, 100):
        for world in (1, 2, 3, 8):
            items = [i for r in range(world) for i in shard_range(n, r, world)]
            assert items == list(range(n))
            sizes = [len(shard_range(n, r, world)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # inference: every rank times its own shard; the reported time is the max
        t = max_over_ranks(1.0 + rank)
        # training: DDP over the regulariser (pure PyTorch step on CPU) averages grads
        from models.drmvsnet import UNetConvLSTM
        torch.manual_seed(0)
        reg = UNetConvLSTM((8, 8), [32, 16, 16, 32, 32], [16, 16, 16, 16, 8], [(3, 3)] * 5, 5)
        ddp = torch.nn.parallel.DistributedDataParallel(reg)
        x = torch.randn(1, 32, 8, 8, generator=torch.Generator().manual_seed(100 + rank))
        cost, _ = ddp(x, None, 0)
        cost.sum().backward()
        g = reg.cell_list[0].conv.weight.grad.clone()
        # local grads of each rank, recomputed without DDP, averaged by hand
        local = []
        for r in range(world):
            ref = UNetConvLSTM((8, 8), [32, 16, 16, 32, 32], [16, 16, 16, 16, 8], [(3, 3)] * 5, 5)
            ref.load_state_dict(reg.state_dict())
            xr = torch.randn(1, 32, 8, 8, generator=torch.Generator().manual_seed(100 + r))
            c, _ = ref(xr, None, 0)
            c.sum().backward()
            local.append(ref.cell_list[0].conv.weight.grad)
        expect = sum(local) / world
        q.put((rank, t, float((g - expect).abs().max()), list(shard_range(5, rank, world))))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_timing_and_ddp():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [2.0, 2.0]
    assert all(r[2] < 1e-6 for r in res)
    assert res[0][3] + res[1][3] == list(range(5))
