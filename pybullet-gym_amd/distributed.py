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

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(num_global: int, rank: int, world: int) -> Tuple[int, int]:
    """(offset, count) of rank's contiguous share; the first num_global % world ranks get one more."""
    base, extra = divmod(num_global, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def gather_flat(local: torch.Tensor, num_global: Optional[int] = None, group=None) -> torch.Tensor:
    """All-gather per-rank tensors [n_rank, ...] into [num_global, ...] in rank order (= global
    env order).  Shards may differ by one row (shard_range): every rank pads its share to
    ceil(num_global / world) rows, one all_gather_into_tensor moves the padded blocks, and the
    pad rows are dropped.  num_global=None assumes equal shards (world * n_local)."""
    world = dist.get_world_size(group)
    if local.is_cuda and dist.get_backend(group) == "gloo":
        # gloo moves host memory: stage the device shard through the host and hand the flat
        # batch back on the shard's device (RCCL, the "nccl" backend, gathers in HBM directly)
        return gather_flat(local.cpu(), num_global, group).to(local.device)
    n_local = local.shape[0]
    if num_global is None:
        num_global = world * n_local
    rows = -(-num_global // world)
    rank = dist.get_rank(group)
    off, cnt = shard_range(num_global, rank, world)
    if cnt != n_local:
        raise ValueError(f"rank {rank} holds {n_local} rows, shard_range says {cnt} of {num_global}")
    tail = tuple(local.shape[1:])
    if n_local == rows:
        send = local.contiguous()
    else:
        send = torch.zeros((rows,) + tail, dtype=local.dtype, device=local.device)
        send[:n_local] = local
    out = torch.empty((world * rows,) + tail, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, send, group=group)
    if num_global == world * rows:
        return out
    keep = torch.cat([torch.arange(r * rows, r * rows + shard_range(num_global, r, world)[1], device=out.device)
                      for r in range(world)])
    return out.index_select(0, keep)


def gather_step(obs: torch.Tensor, reward: torch.Tensor, done: torch.Tensor, num_global: Optional[int] = None,
                group=None):
    """(obs, reward, done) of every rank, flat in global env order, with ONE collective: each
    rank packs its rows as float32 [n_rank, obs_dim + 2] = (obs | reward | done) -- done is 0/1,
    exact in float32 -- one gather_flat moves the packed block (one ring pass over xGMI
    instead of three latency-bound small ones), and the columns are split back."""
    D = obs.shape[1]
    packed = torch.empty((obs.shape[0], D + 2), dtype=torch.float32, device=obs.device)
    packed[:, :D] = obs
    packed[:, D] = reward.to(torch.float32)
    packed[:, D + 1] = done.to(torch.float32)
    flat = gather_flat(packed, num_global, group)
    return flat[:, :D], flat[:, D].contiguous(), flat[:, D + 1].to(done.dtype)


class ShardedVecEnv:
    """This rank's share of a global batch of envs, plus the optional flat gather.

    env_factory(env_id, count, device, seed, env_offset, autoreset) builds the per-rank env
    (default: the HIP VecEnv at ``precision`` -- 64, the reference's double, unless 32 is asked
    for); anything with ``obs`` / ``reward`` / ``done`` tensors and ``reset`` / ``step`` works (the
    CPU tests drive the oracle through it)."""

    def __init__(self, env_id: str, num_global: int, rank: int, world: int, device, seed: int = 0,
                 autoreset: bool = True, env_factory: Optional[Callable] = None, precision: int = 64):
        self.num_global = num_global
        self.offset, self.count = shard_range(num_global, rank, world)
        if env_factory is None:
            from .vec_env import VecEnv

            def env_factory(env_id, count, device, seed, env_offset, autoreset):
                return VecEnv(env_id, count, device=device, seed=seed, env_offset=env_offset, autoreset=autoreset,
                              precision=precision)
        self.env = env_factory(env_id, self.count, device, seed, self.offset, autoreset)

    def reset(self, **kw):
        return self.env.reset(**kw)

    def step(self, actions):
        return self.env.step(actions)

    def gather(self):
        """(obs, reward, done) of every env of every rank, flat in global env order, on every rank."""
        e = self.env
        return gather_step(e.obs, e.reward, e.done, self.num_global)
