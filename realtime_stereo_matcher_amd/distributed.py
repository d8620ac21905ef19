"""Data-parallel plumbing: one process per GPU, stereo pairs sharded by batch, per-pair
disparities gathered to rank 0 over RCCL (torch.distributed backend "nccl" on ROCm).

The reference's only parallelism is ``torch.nn.DataParallel`` (train_stereo.py:139,
evaluate_stereo.py:300, test_stereo.py:62): one process that scatters the batch, replicates
the model and gathers outputs.  Here pairs are independent, so each rank owns a contiguous
slice of the global batch and builds its volumes locally; the ONLY collective is the gather
of the (B_r, 1, H, W) disparity maps -- volumes never cross devices.  ``dist.gather`` lets
rank 0 receive from every peer over its own xGMI link instead of a ring all-gather.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank():
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard_range(global_batch: int, rank: int, world: int):
    """Contiguous [start, stop) slice of the global batch owned by ``rank`` (remainder to the
    lowest ranks, so shard sizes differ by at most one)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard(batch: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    s, e = shard_range(batch.shape[0], rank, world)
    return batch[s:e]


def gather_disparities(disp: torch.Tensor, global_batch: int, dst: int = 0):
    """Gather every rank's (B_r, ...) disparity shard to ``dst``; returns the (global_batch, ...)
    tensor on ``dst`` and None elsewhere.  Shards may be ragged (uneven split)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return disp
    world, rank = dist.get_world_size(), dist.get_rank()
    sizes = [shard_range(global_batch, r, world) for r in range(world)]
    maxb = max(e - s for s, e in sizes)
    tail = tuple(disp.shape[1:])
    if disp.shape[0] != maxb:  # pad ragged shards to a common shape for the collective
        pad = disp.new_zeros((maxb - disp.shape[0],) + tail)
        send = torch.cat([disp, pad], 0)
    else:
        send = disp.contiguous()
    if rank == dst:
        bufs = [torch.empty((maxb,) + tail, dtype=disp.dtype, device=disp.device) for _ in range(world)]
        dist.gather(send, gather_list=bufs, dst=dst)
        return torch.cat([b[: e - s] for b, (s, e) in zip(bufs, sizes)], 0)
    dist.gather(send, dst=dst)
    return None
