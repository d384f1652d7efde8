"""Multi-GPU plumbing for the batched solve (DESIGN.md §0 row e).

Instances are independent, so the data path has no collective: each rank samples its own seeded shard
(`sampling.sample_start_goal(..., rank=r)`), solves it on its own GPU, and only the solutions are
gathered to rank 0 afterwards (RCCL gather over xGMI for `nccl`, or gloo on CPU in the tests).  Timing is the
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


def gather_solutions(r: dict, keys=("X", "U", "S", "cost", "status", "iters"), dst: int = 0) -> dict:
    """Gather every rank's per-instance outputs (equal shard sizes) to rank `dst`, concatenated in rank
    order (RCCL gather over xGMI under `nccl`).  Other ranks get None per key: only the destination
    needs the solutions, so nothing is broadcast back."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return {k: r[k] for k in keys}
    world, me = dist.get_world_size(), dist.get_rank()
    host = dist.get_backend() == "gloo"  # gloo gathers host tensors (the CPU tests and the 1-GPU rehearsal)
    out = {}
    for k in keys:
        t = r[k].contiguous()
        if host:
            t = t.cpu()
        parts = [torch.empty_like(t) for _ in range(world)] if me == dst else None
        dist.gather(t, parts, dst=dst)
        out[k] = torch.cat(parts, 0) if me == dst else None
    return out


def _coll_device(device):
    return "cpu" if dist.get_backend() == "gloo" else device


def max_over_ranks(x: float, device) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(n: int, device) -> int:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return n
    t = torch.tensor([n], dtype=torch.int64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def gather_rank_rows(row, device):
    """Every rank's small float vector (the same length on all ranks) as a [world, len] list on every rank
    (one all_gather): per-rank status counts and iteration tails, so straggler imbalance is visible."""
    row = [float(v) for v in row]
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [row]
    t = torch.tensor(row, dtype=torch.float64, device=_coll_device(device))
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [p.cpu().tolist() for p in parts]
