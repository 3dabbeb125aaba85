"""Multi-GPU sharding: one process per GPU, each owning a contiguous env range.

Envs are independent (nothing in WalkerBaseBulletEnv._step couples two envs;
the reference's scene only ever holds one robot, scene_bases.py:54-55), so the step
itself needs no communication: rank r steps envs [offset_r, offset_r + n_r) with its
own handle.  The reset RNG is keyed by the *global* env id, so every env's trajectory
is the same whatever the number of GPUs.  The only collective is the optional
all-gather of observations/rewards/dones for a learner that wants one flat batch
(RCCL over xGMI with the "nccl" backend; gloo on CPU tests).
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def shard_range(num_global: int, rank: int, world: int) -> Tuple[int, int]:
    """(offset, count) of rank's contiguous share; the first num_global % world ranks get one more."""
    base, extra = divmod(num_global, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def gather_flat(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather equal-size per-rank tensors [n_local, ...] into [world * n_local, ...]
    in rank order (= global env order for equal shards)."""
    world = dist.get_world_size(group)
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out


class ShardedVecEnv:
    """This rank's share of a global batch of envs, plus the optional flat gather."""

    def __init__(self, env_id: str, num_global: int, rank: int, world: int, device, seed: int = 0,
                 autoreset: bool = True):
        from .vec_env import VecEnv
        self.offset, self.count = shard_range(num_global, rank, world)
        self.env = VecEnv(env_id, self.count, device=device, seed=seed, env_offset=self.offset, autoreset=autoreset)

    def reset(self, **kw):
        return self.env.reset(**kw)

    def step(self, actions):
        return self.env.step(actions)

    def gather(self):
        """(obs, reward, done) of every env of every rank, flat, on every rank."""
        e = self.env
        return gather_flat(e.obs), gather_flat(e.reward), gather_flat(e.done)
