"""One process per GPU: chunk partitioning with no data-path collective.

Chunks encode and decode independently (the validator processes them one by one with no
cross-chunk state, /root/reference/storb/validator/validator.py:1352-1431), so a multi-GPU
job splits the chunk list into contiguous ranges balanced by bytes and each rank runs its
range on its own device.  The only collectives are the measurement's barrier and the
max-over-ranks of the elapsed time (``torch.distributed``: RCCL on GPUs, gloo on CPU).
"""

from __future__ import annotations

import os

import numpy as np


def rank_env() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (defaults: single process)."""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world


def partition(sizes, world: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) chunk ranges, one per rank, balanced by total bytes.

    Boundary r is the first chunk whose prefix sum reaches r/world of the total; every chunk
    lands in exactly one range and ranges are in rank order.
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    sizes = np.asarray(sizes, dtype=np.float64)
    n = len(sizes)
    if n == 0:
        return [(0, 0)] * world
    prefix = np.concatenate([[0.0], np.cumsum(sizes)])
    total = prefix[-1]
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        b = int(np.searchsorted(prefix, target, side="left"))
        bounds.append(min(max(b, bounds[-1]), n))
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def init(backend: str | None = None):
    """Initialise torch.distributed when launched under torchrun; returns the module or None."""
    import torch.distributed as dist

    _, _, world = rank_env()
    if world <= 1:
        return None
    if not dist.is_initialized():
        if backend is None:
            import torch
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend)
    return dist


def barrier(dist_mod, device=None) -> None:
    if dist_mod is None:
        return
    if device is not None and dist_mod.get_backend() == "nccl":
        dist_mod.barrier(device_ids=[device])
    else:
        dist_mod.barrier()


def max_over_ranks(dist_mod, value: float, device=None) -> float:
    if dist_mod is None:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64,
                     device=f"cuda:{device}" if (device is not None and dist_mod.get_backend() == "nccl") else "cpu")
    dist_mod.all_reduce(t, op=dist_mod.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist_mod, value: float, device=None) -> float:
    if dist_mod is None:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64,
                     device=f"cuda:{device}" if (device is not None and dist_mod.get_backend() == "nccl") else "cpu")
    dist_mod.all_reduce(t, op=dist_mod.ReduceOp.SUM)
    return float(t.item())


def gather_counts(dist_mod, count: int, rank: int, world: int, device=None) -> list[int]:
    """Every rank's `count`, in rank order (one all-reduce of a one-hot vector)."""
    if dist_mod is None:
        return [int(count)]
    import torch

    t = torch.zeros(world, dtype=torch.float64,
                    device=f"cuda:{device}" if (device is not None and dist_mod.get_backend() == "nccl") else "cpu")
    t[rank] = float(count)
    dist_mod.all_reduce(t, op=dist_mod.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]
