"""Multi-process sharding with the real HIP VecEnv: two processes on
cuda:0 each own a contiguous, uneven shard of one global batch through
pybulletgym_amd.distributed.ShardedVecEnv (env_offset = the shard's first global env id, reset
noise and actions keyed by the global id), step it with auto-reset, and gather
(obs | reward | done) over gloo with the product's gather_step.  The flat result must equal a
one-process VecEnv over all envs bit for bit.  (One GPU per rank over RCCL is the bench's
N > 1 path; two ranks cannot share a device under RCCL, so this test uses gloo.)"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pybulletgym_amd  # noqa: F401

pytestmark = pytest.mark.gpu

N_GLOBAL, STEPS, SEED = 1001, 40, 23  # 1001 envs over 2 ranks: 501 + 500


def _run(env_id, vec, offset, count):
    from pybulletgym_amd.vec_env import sample_actions
    na = vec.info.action_dim
    acts = sample_actions(na, count, STEPS, seed=SEED, env_offset=offset)
    vec.reset()
    # age the episodes by global env id so that TimeLimit auto-resets fall inside the window
    phys, aux = vec.get_state()
    gid = torch.arange(offset, offset + count, device=aux.device, dtype=torch.float64)
    aux[:, 2] = 975.0 + torch.remainder(gid, 30.0)
    vec.set_state(phys, aux)
    dones = 0
    for t in range(STEPS):
        vec.step(acts[t])
        dones += int(vec.done.sum())
    return dones


def _worker(rank, world, port, env_id, q, precision=32):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pybulletgym_amd import distributed as pd
    env = pd.ShardedVecEnv(env_id, N_GLOBAL, rank, world, device="cuda:0", seed=SEED, autoreset=True,
                           precision=precision)
    _run(env_id, env.env, env.offset, env.count)
    obs, rew, done = env.gather()
    assert obs.is_cuda and obs.shape[0] == N_GLOBAL
    if rank == 0:
        q.put((env.count, obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("env_id,precision", [("AntPyBulletEnv-v0", 32), ("HumanoidPyBulletEnv-v0", 32),
                                              ("AntPyBulletEnv-v0", 64), ("HumanoidPyBulletEnv-v0", 64)])
def test_two_process_shards_gather_bitwise_equal_single_process(env_id, precision):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pybulletgym_amd import distributed as pd
    from pybulletgym_amd.vec_env import VecEnv
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, env_id, q, precision)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        count0, obs, rew, done = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert count0 == pd.shard_range(N_GLOBAL, 0, world)[1] == 501
    ref = VecEnv(env_id, N_GLOBAL, seed=SEED, autoreset=True, precision=precision)
    dones = _run(env_id, ref, 0, N_GLOBAL)
    assert dones > 0  # auto-resets happened inside the compared window
    np.testing.assert_array_equal(obs.view(np.uint32), ref.obs.cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(rew.view(np.uint32), ref.reward.cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(done, ref.done.cpu().numpy())
    ref.close()
