"""Scenario sharding and the end-of-batch gather.

Scenarios are independent, so a node runs one process per GPU, each owning a
contiguous range of GLOBAL scenario ids; the inputs are generated from the
global id (counter-based), so any sharding reproduces the single-GPU batch
bit for bit.  The only collective is the gather of the per-step outputs at
the end of the batch (RCCL over xGMI with the "nccl" backend; gloo on CPU):
``gather_scenarios`` leaves the whole batch on every rank (all-gather),
``gather_to_root`` only on one rank (each rank's block crosses xGMI once, into
the root, instead of into every rank: 1/(world-1) of the all-gather traffic).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """[first, first+count) of the global ids owned by ``rank`` (balanced, contiguous)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, rem = divmod(total, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def gather_scenarios(t: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """All-gather a (..., B_rank) scenario-minor tensor into (..., total).

    Ranks may hold different B_rank (uneven split): every rank pads to the
    largest share, one all_gather_into_tensor moves the data, and the padding
    is dropped.  Returns the global tensor on every rank (scenario order =
    global id order)."""
    world = dist.get_world_size(group)
    if world == 1:
        return t
    shares = [shard_range(total, world, r)[1] for r in range(world)]
    bmax = max(shares)
    lead = t.shape[:-1]
    pad = torch.zeros(*lead, bmax, dtype=t.dtype, device=t.device)
    pad[..., :t.shape[-1]] = t
    flat = pad.reshape(-1, bmax).t().contiguous()                  # (bmax, E): scenario-major rows
    out = torch.empty(world * bmax, flat.shape[1], dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, flat, group=group)
    parts = [out[r * bmax:r * bmax + shares[r]] for r in range(world)]
    return torch.cat(parts, 0).t().reshape(*lead, total).contiguous()


def gather_to_root(t: torch.Tensor, total: int, root: int = 0, group=None):
    """Gather a (..., B_rank) scenario-minor tensor into (..., total) on ``root``
    only (None on the other ranks); ranks may hold uneven shares (shard_range).
    One ``dist.gather`` of each rank's scenario-major block (RCCL point-to-point
    sends into the root over xGMI)."""
    world = dist.get_world_size(group)
    if world == 1:
        return t
    rank = dist.get_rank(group)
    shares = [shard_range(total, world, r)[1] for r in range(world)]
    bmax = max(shares)
    lead = t.shape[:-1]
    pad = torch.zeros(*lead, bmax, dtype=t.dtype, device=t.device)
    pad[..., :t.shape[-1]] = t
    flat = pad.reshape(-1, bmax).t().contiguous()                  # (bmax, E)
    bufs = [torch.empty_like(flat) for _ in range(world)] if rank == root else None
    dist.gather(flat, gather_list=bufs, dst=root, group=group)
    if rank != root:
        return None
    parts = [bufs[r][:shares[r]] for r in range(world)]
    return torch.cat(parts, 0).t().reshape(*lead, total).contiguous()
