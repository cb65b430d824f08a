"""Scenario sharding and the end-of-batch gather.

Scenarios are independent, so a node runs one process per GPU, each owning a
contiguous range of GLOBAL scenario ids; the inputs are generated from the
global id (counter-based), so any sharding reproduces the single-GPU batch
bit for bit, provided every rank runs the build one GPU would run for the
whole batch (``pin_layout``: the library picks the N = 20 build by batch size,
and the two builds agree to the parity tolerances, not bit for bit).  The only
collective is the gather of the per-step outputs at
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


def pin_layout(ctl, total: int, cfg=None) -> str:
    """Pin ``ctl`` (an ntm_mpc.NtmMpc) to the step build a single GPU would take
    for the whole ``total``-scenario batch, and return it ("lds" or "far").

    The library chooses the N = 20 build from each call's batch size
    (ntm_ctx_set_small_batch; all-LDS up to 8 scenarios per CU, the far
    workspace above), so without this a far-build total sharded over many GPUs
    would run its shards on the all-LDS build and lose bitwise agreement with
    the one-GPU run.  Horizons with one build are unaffected."""
    layout = ctl.step_layout(int(total), cfg)
    ctl.set_small_batch((1 << 62) if layout == "lds" else 0)
    return layout


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
    ``root`` is a rank of ``group`` (group-relative, like the shares), converted
    to the global rank ``dist.gather`` expects.  One ``dist.gather`` of each
    rank's scenario-major block (RCCL point-to-point sends into the root over
    xGMI)."""
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
    dst = root if group is None else dist.get_global_rank(group, root)
    dist.gather(flat, gather_list=bufs, dst=dst, group=group)
    if rank != root:
        return None
    parts = [bufs[r][:shares[r]] for r in range(world)]
    return torch.cat(parts, 0).t().reshape(*lead, total).contiguous()
