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


def pack_final(reward, done, out=None):
    """One rank's final (reward float32 [E], done u8 [E]) batch as 5 E bytes (reward bytes, then
    done bytes) -- the payload of the run's single all-gather (5 B per env instead of 8 as two
    float32 rows). ``out``: a preallocated uint8 [5 E] buffer on the same device."""
    import torch
    E = reward.numel()
    if out is None:
        out = torch.empty(5 * E, dtype=torch.uint8, device=reward.device)
    out[:4 * E].view(torch.float32).copy_(reward.reshape(-1))
    out[4 * E:].copy_(done.reshape(-1))
    return out


def unpack_final(packed):
    """[world, 5 E] uint8 (gather_final's result) -> [world, 2, E] float32 {reward, done}."""
    import torch
    world, n = packed.shape
    E = n // 5
    rew = packed[:, :4 * E].contiguous().view(torch.float32)
    dn = packed[:, 4 * E:].float()
    return torch.stack([rew, dn], dim=1)


def gather_final(reward, done, group=None, packed=False, buf=None):
    """All-gather the final (reward, done) batch of every rank (the run's single collective):
    [world, 2, E] float32 on every rank, or with ``packed`` the raw [world, 5 E] uint8 result
    (unpack_final; keeps the unpacking out of a timed region). ``buf``: preallocated
    (send [5 E], receive [world, 5 E]) uint8 buffers."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    send, recv = buf if buf is not None else (None, None)
    send = pack_final(reward, done, send)
    if dist.get_backend(group) == "gloo":  # CPU rehearsal backend
        send = send.cpu()
        parts = [torch.empty_like(send) for _ in range(world)]
        dist.all_gather(parts, send, group=group)
        out = torch.stack(parts)
    else:  # RCCL: one collective straight into the [world, 5 E] result
        out = recv if recv is not None else torch.empty((world, send.numel()), dtype=torch.uint8,
                                                         device=send.device)
        dist.all_gather_into_tensor(out, send, group=group)
    return out if packed else unpack_final(out)


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
