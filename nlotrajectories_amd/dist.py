"""Multi-GPU plumbing for the batched solve (DESIGN.md §0 row e).

Instances are independent, so the data path has no collective: each rank samples its own seeded shard
(`sampling.sample_start_goal(..., rank=r)`), solves it on its own GPU, and only the solutions are
gathered afterwards (RCCL all_gather over xGMI for `nccl`, or gloo on CPU in the tests).  Timing is the
max over ranks, counts are summed.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def rank_world():
    """(rank, local_rank, world_size) from the torch.distributed.run environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def gather_solutions(r: dict, keys=("X", "U", "S", "cost", "status", "iters")) -> dict:
    """All-gather every rank's per-instance outputs (equal shard sizes), concatenated in rank order."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return {k: r[k] for k in keys}
    out = {}
    for k in keys:
        parts = [torch.empty_like(r[k]) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, r[k].contiguous())
        out[k] = torch.cat(parts, 0)
    return out


def max_over_ranks(x: float, device) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(n: int, device) -> int:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return n
    t = torch.tensor([n], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
