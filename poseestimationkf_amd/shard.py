"""Data-parallel sharding of the independent-filter batch over ranks.

Filters are independent (no state shared between KalmanFilter instances,
ExtendedKalmanFilter.py:6-80) and the time axis is a strict recurrence, so the only
parallel axis is the batch: rank r owns the contiguous filter range
[r*B_local, (r+1)*B_local) and runs it with no communication at all.  The single
collective is one gather of the final quaternions to rank 0 (RCCL over xGMI when the
process group is "nccl"; gloo in the CPU tests).
"""
from __future__ import annotations


def shard_range(global_batch, rank, world):
    """(first_filter, count) of rank's contiguous shard; shards are equal-sized."""
    if global_batch % world:
        raise ValueError("global batch %d must divide evenly over %d ranks" % (global_batch, world))
    per = global_batch // world
    return rank * per, per


def gather_quaternions(x_local, rank, world, dst=0, force_collective=False):
    """Gather every rank's (B_local, 4) float64 quaternion tensor to `dst`.

    Returns the (world*B_local, 4) tensor on dst (rows ordered by filter id) and None elsewhere.
    One torch.distributed.gather call -- a single RCCL collective on the "nccl" backend.
    """
    import torch
    import torch.distributed as dist

    if world == 1 and not force_collective:
        return x_local
    bufs = [torch.empty_like(x_local) for _ in range(world)] if rank == dst else None
    dist.gather(x_local, gather_list=bufs, dst=dst)
    return torch.cat(bufs, dim=0) if rank == dst else None
