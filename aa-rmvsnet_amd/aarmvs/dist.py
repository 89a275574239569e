"""Multi-GPU helpers: one process per GPU (torchrun), reference views sharded across
ranks with no data-path collective; RCCL (``nccl`` backend) only for the
training gradient all-reduce (DDP) and the benchmark's timing reductions."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (1 process default)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard_range(n_items: int, rank: int, world: int) -> range:
    """Contiguous, balanced slice of ``n_items`` (scan, ref-view) samples for ``rank``.

    The first ``n_items % world`` ranks take one extra item; every item is owned by
    exactly one rank.
    """
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def shared_gpu() -> bool:
    """AARMVS_SHARED_GPU=1: a rehearsal of the multi-rank path with every rank on the one
    visible GPU (gloo, since RCCL refuses two ranks on one device); never set in production."""
    return os.environ.get("AARMVS_SHARED_GPU", "0") == "1"


def local_device_index(local_rank: int) -> int:
    """The GPU a rank drives: its local rank (one process per GPU), or the one visible GPU
    in a shared-GPU rehearsal."""
    return local_rank % max(1, torch.cuda.device_count()) if shared_gpu() else local_rank


def max_over_ranks(value: float, device=None) -> float:
    """Max of a host float over all ranks (identity without a process group)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = None
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def init_process_group(device: torch.device | None = None) -> None:
    """nccl (= RCCL on ROCm) on GPUs, gloo on CPU; no-op for a single process."""
    _, _, world = env()
    if world == 1 or dist.is_initialized():
        return
    if device is not None and device.type == "cuda" and not shared_gpu():
        dist.init_process_group("nccl", device_id=device)
    else:
        dist.init_process_group("gloo")
