"""Multi-GPU sharding for the packet stage.

Packets are independent at this stage, so ranks never exchange packet data: rank r filters its
own contiguous shard of the frame stream on its own GPU (weak scaling). The only collective is
the reduction of per-rank totals and timings, once, outside the timed region — SURVEY §8e's
`allreduce(sum)` of {packets, accepted, forwarded, delivered} plus a max of the per-rank times.
The same functions run over RCCL ("nccl") on GPUs and over gloo in the CPU tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    start: int  # index of the rank's first frame in the global stream
    count: int  # frames per rank (weak scaling: fixed per rank)


def env_rank() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(frames_per_rank: int, rank: int, world: int) -> Shard:
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return Shard(rank, world, rank * frames_per_rank, frames_per_rank)


def reduce_totals(totals, times):
    """Sum the per-rank totals (int64 tensor) and take the max of the per-rank times (float64
    tensor) over all ranks, in place; a no-op on one rank. Returns (totals, times)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        host = dist.get_backend() == "gloo" and totals.is_cuda  # gloo reduces host tensors
        t, m = (totals.cpu(), times.cpu()) if host else (totals, times)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        if host:
            totals.copy_(t)
            times.copy_(m)
    return totals, times


def aggregate_mpps(frames_per_rank: int, world: int, steps: int, max_wall_s: float) -> float:
    """Whole-job throughput: every rank's frames over the slowest rank's time."""
    return frames_per_rank * world * steps / max_wall_s / 1e6
