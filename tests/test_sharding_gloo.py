"""Multi-process sharding on CPU (gloo, world_size 2): each rank steps its contiguous env
range with reset noise keyed by global env id, and the product's flat all-gather
(pybulletgym_amd.distributed.ShardedVecEnv.gather -> gather_flat, padded for uneven shards)
reproduces a single-process run over all envs bit-for-bit -- obs float32, reward float32 and
the uint8 done flags.  The per-rank env is the CPU oracle behind VecEnv's buffer interface
(the HIP path needs a GPU); shard arithmetic, env factory and gather are the product's."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pybulletgym_amd  # noqa: F401
from pybulletgym_amd import distributed as pd, rng

ENV = "AntPyBulletEnv-v0"
N_GLOBAL, STEPS, SEED = 7, 4, 11  # 7 envs: uneven shards on 2 and 3 ranks


class OracleShard:
    """VecEnv-shaped CPU stand-in (obs / reward / done tensors, reset / step) over the oracle,
    for the gloo tests only."""

    def __init__(self, env_id, count, device, seed, env_offset, autoreset):
        import oracle
        self.e = oracle.OracleEnvs(env_id, count)
        self.ids = np.arange(env_offset, env_offset + count)
        self.seed = seed
        self.obs = torch.zeros((count, self.e.info.OBS), dtype=torch.float32)
        self.reward = torch.zeros(count, dtype=torch.float32)
        self.done = torch.zeros(count, dtype=torch.uint8)

    def reset(self):
        q = rng.reset_noise(self.seed, self.ids, 0, self.e.info.NR).astype(np.float64)
        self.obs[:] = torch.from_numpy(self.e.reset(q))
        return self.obs

    def step(self, actions):
        o, r, d, _ = self.e.step(np.asarray(actions))
        self.obs[:] = torch.from_numpy(o)
        self.reward[:] = torch.from_numpy(r.astype(np.float32))
        self.done[:] = torch.from_numpy(d.astype(np.uint8))
        return self.obs


def actions_for(global_ids, step, na):
    return rng.sample_actions(na, global_ids, [step], seed=SEED)[0]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env = pd.ShardedVecEnv(ENV, N_GLOBAL, rank, world, device="cpu", seed=SEED, env_factory=OracleShard)
    env.reset()
    for t in range(STEPS):
        env.step(actions_for(np.arange(env.offset, env.offset + env.count), t, 8))
    obs, rew, done = env.gather()
    if rank == 0:
        q.put((env.count, obs.numpy(), rew.numpy(), done.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_covers_all():
    for n in (1, 7, 16384, 65536, 65537):
        for w in (1, 2, 3, 8):
            spans = [pd.shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and sum(c for _, c in spans) == n
            for (o1, c1), (o2, _) in zip(spans, spans[1:]):
                assert o1 + c1 == o2


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_vecenv_gather_matches_single_process(world):
    """Uneven shards (7 envs over 2 ranks: 4 + 3; over 3 ranks: 3 + 2 + 2) gather back to
    the single-process trajectory bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    count0, flat_obs, flat_rew, flat_done = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert count0 == pd.shard_range(N_GLOBAL, 0, world)[1]
    assert flat_obs.shape == (N_GLOBAL, 28) and flat_done.dtype == np.uint8
    ref = OracleShard(ENV, N_GLOBAL, "cpu", SEED, 0, True)
    ref.reset()
    for t in range(STEPS):
        ref.step(actions_for(np.arange(N_GLOBAL), t, 8))
    np.testing.assert_array_equal(flat_obs, ref.obs.numpy())
    np.testing.assert_array_equal(flat_rew, ref.reward.numpy())
    np.testing.assert_array_equal(flat_done, ref.done.numpy())
