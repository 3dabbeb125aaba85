"""BASELINE.json configs C4 and C5 at their WHOLE-JOB sizes on one GPU.

  C4  HalfCheetahPyBulletEnv-v0, 65,536 envs (8 x 8,192 per GPU) + the all-gather of obs
  C5  HumanoidPyBulletEnv-v0, 32,768 envs (8 x 4,096 per GPU)

(a) ``test_full_batch_teacher_forced``: one VecEnv holding the whole batch (launch geometry,
    LDS capacity and envs per CU of the full size), 200 teacher-forced steps with auto-reset
    against the float64 oracle on 384 envs spread evenly over the batch (every workgroup
    position).  Float32 handles go through the class A/B/C bounds and outlier explanation of the
    per-GPU config tests (tests/test_gpu.py SplitStats); float64 handles (the reference's
    precision and the facade's default) through tests/test_f64.py's bounds --
    every same-contact-set step's state within 1e-9 of the oracle.  Every step's
    (obs | reward | done) of all envs is digested (sha256) for (b).
(b) ``test_full_batch_eight_shards_bitwise``: the product's multi-GPU path on one device -- 8
    processes on cuda:0, each a ``ShardedVecEnv`` owning 1/8 of the batch (env_offset = its first
    global env id, Philox reset noise and actions keyed by the global id), stepping with
    auto-reset and gathering (obs | reward | done) with ``gather_step`` over gloo every
    GATHER_EVERY steps.  The gathered flat batch must be bitwise equal to (a)'s whole-batch
    trajectory at every gathered step (auto-resets happen inside the window: asserted).  RCCL
    cannot put two ranks on one device, so the collective is gloo here; the RCCL branch of
    gather_flat runs in the driver's multi-GPU bench (bench.py --gpus N).

Reference: /root/reference/pybulletgym/envs/__init__.py:59-64,80-84 (the env ids),
scene_bases.py:47-51 (one scene per env: envs are independent, so sharding is exact).
"""
import hashlib
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pybulletgym_amd  # noqa: F401

pytestmark = pytest.mark.gpu

FULL = [("HalfCheetahPyBulletEnv-v0", 65536), ("HumanoidPyBulletEnv-v0", 32768)]
FULLP = [(e, n, p) for p in (32, 64) for e, n in FULL]
STEPS, SEED, SAMPLE, WORLD, GATHER_EVERY = 200, 29, 384, 8, 4
_DIGESTS = {}  # (env_id, precision) -> per-step sha256 of the whole batch (filled by (a), reused by (b))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _digest(obs, rew, done):
    """sha256 over the float32 obs bytes, the float32 reward bytes and the done bytes."""
    h = hashlib.sha256()
    h.update(obs.detach().contiguous().cpu().numpy().tobytes())
    h.update(rew.detach().to(torch.float32).contiguous().cpu().numpy().tobytes())
    h.update(done.detach().to(torch.uint8).contiguous().cpu().numpy().tobytes())
    return h.hexdigest()


def _single_process_digests(env_id, n, precision):
    """(a)'s GPU trajectory without the oracle (when (b) runs alone): the same handle, actions and
    seed -- teacher forcing only reads the device state, it never writes it."""
    from pybulletgym_amd.vec_env import VecEnv, sample_actions
    env = VecEnv(env_id, n, seed=SEED, autoreset=True, precision=precision)
    env.reset()
    acts = sample_actions(env.info.action_dim, n, STEPS, seed=SEED)
    out, dones = [], 0
    for t in range(STEPS):
        env.step(acts[t])
        dones += int(env.done.sum())
        out.append(_digest(env.obs, env.reward, env.done))
    env.close()
    return out, dones


@pytest.mark.timeout(900)
@pytest.mark.parametrize("env_id,n,precision", FULLP)
def test_full_batch_teacher_forced(env_id, n, precision):
    digests, dones = [], [0]

    def on_step(t, env):
        assert env.precision == precision
        dones[0] += int(env.done.sum())
        digests.append(_digest(env.obs, env.reward, env.done))

    if precision == 64:
        from test_f64 import _teacher_forced64
        rec = _teacher_forced64(env_id, n, STEPS, sample=SAMPLE, seed=SEED,
                                name=f"f64_full_batch[{env_id},{n}x{STEPS}]", on_step=on_step)
    else:
        from test_gpu import _teacher_forced
        rec = _teacher_forced(env_id, n, STEPS, sample=SAMPLE, seed=SEED, name=f"full_batch[{env_id},{n}x{STEPS}]",
                              on_step=on_step)
    assert len(digests) == STEPS
    assert dones[0] > 0, "no auto-reset inside the window"
    _DIGESTS[(env_id, precision)] = (digests, dones[0])
    assert rec["env_steps"] == SAMPLE * STEPS


def _worker(rank, world, port, env_id, n, precision, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pybulletgym_amd import distributed as pd
    from pybulletgym_amd.vec_env import sample_actions
    env = pd.ShardedVecEnv(env_id, n, rank, world, device="cuda:0", seed=SEED, autoreset=True, precision=precision)
    assert env.env.precision == precision
    acts = sample_actions(env.env.info.action_dim, env.count, STEPS, seed=SEED, env_offset=env.offset)
    env.reset()
    out, dones = {}, 0
    t0 = time.time()
    for t in range(STEPS):
        env.step(acts[t])
        dones += int(env.env.done.sum())
        if t % GATHER_EVERY == GATHER_EVERY - 1 or t == STEPS - 1:
            obs, rew, done = env.gather()
            assert obs.is_cuda and obs.shape[0] == n
            if rank == 0:
                out[t] = _digest(obs, rew, done)
        if rank == 0 and t % 50 == 0:
            print(f"  shards[{env_id}]: step {t}/{STEPS} {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    tot = torch.tensor([dones], dtype=torch.int64)
    dist.all_reduce(tot)
    if rank == 0:
        q.put((out, int(tot.item()), env.count))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
@pytest.mark.parametrize("env_id,n,precision", FULLP)
def test_full_batch_eight_shards_bitwise(env_id, n, precision):
    from pybulletgym_amd import distributed as pd
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, env_id, n, precision, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        shard_digests, shard_dones, count0 = q.get(timeout=500)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert count0 == pd.shard_range(n, 0, WORLD)[1] == n // WORLD
    ref, ref_dones = _DIGESTS.get((env_id, precision)) or _single_process_digests(env_id, n, precision)
    assert shard_dones == ref_dones > 0  # the same auto-resets, inside the compared window
    assert len(shard_digests) >= STEPS // GATHER_EVERY
    bad = [t for t, d in sorted(shard_digests.items()) if d != ref[t]]
    assert not bad, f"gathered batch differs from the single-process batch at steps {bad[:10]}"
