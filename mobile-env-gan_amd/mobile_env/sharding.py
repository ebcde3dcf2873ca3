"""Env sharding across GPUs (one process per GPU, torch.distributed; backend "nccl" = RCCL).

Envs are independent (no cross-env term anywhere in MComCore.step, reference base.py:230-296),
so the batch is partitioned, never exchanged: rank r owns the global envs
[r*E, (r+1)*E) (weak scaling, E envs per GPU) and seeds them with base + global index. The
only collective is one all-gather of the final (reward, done) batch to every rank; the obs
batch (E x U x 4 floats per rank) is gathered only on request, after timing, because a
per-step obs all-gather would move ~ E*U*16 bytes per rank per step over xGMI.
"""
from __future__ import annotations

import numpy as np


def shard_envs(envs_per_rank: int, rank: int):
    """Global env index range [start, stop) of `rank`."""
    return rank * envs_per_rank, (rank + 1) * envs_per_rank


def shard_seeds(base_seed: int, envs_per_rank: int, rank: int) -> np.ndarray:
    """Config seeds of the envs of `rank` (movement stream = seed + 4, base.py:156-168)."""
    start, stop = shard_envs(envs_per_rank, rank)
    return base_seed + np.arange(start, stop, dtype=np.int64)


def gather_final(reward, done, group=None):
    """All-gather the final (reward, done) batch of every rank -> [world, 2, E] float32 on
    every rank (the run's single collective)."""
    import torch
    import torch.distributed as dist

    rd = torch.stack([reward.float(), done.float()])
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":  # CPU rehearsal backend
        rd = rd.cpu()
        parts = [torch.empty_like(rd) for _ in range(world)]
        dist.all_gather(parts, rd, group=group)
        return torch.stack(parts)
    # RCCL: one collective straight into the [world, 2, E] result (no per-rank list + stack)
    out = torch.empty((world,) + tuple(rd.shape), dtype=rd.dtype, device=rd.device)
    dist.all_gather_into_tensor(out, rd, group=group)
    return out


def gather_obs(obs, group=None):
    """All-gather the obs batch (end of run only): [world, E, U, 4]."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":
        obs = obs.cpu()
        parts = [torch.empty_like(obs) for _ in range(world)]
        dist.all_gather(parts, obs.contiguous(), group=group)
        return torch.stack(parts)
    out = torch.empty((world,) + tuple(obs.shape), dtype=obs.dtype, device=obs.device)
    dist.all_gather_into_tensor(out, obs.contiguous(), group=group)
    return out
