"""Pretrained-policy behavioural regression -- test helper.

The reference's roboschool-weights policies (examples/roboschool-weights/enjoy_TF_*.py,
``SmallReactivePolicy.act`` at :25-31 of each file; weights extracted by
tests/golden/make_policies.py into tests/golden/policy_*.npz) were trained on pybullet.
Run on a simulator whose physics differs materially from pybullet's (friction, contact
stiffness, joint limits, motor gains, mass/inertia import), they fall or stall; on a faithful
one they score in a band far above a random policy.  This is a loose behavioural check of
the unpinned physics, not a numeric pin (SURVEY.md section 8c "Known-answer tests").

``episode_returns_oracle`` rolls the policy through the CPU oracle (float64 physics);
``episode_returns_device`` through the HIP step (libpbg_amd.so) -- the same episodes,
since the reset draws come from the same host RNG.

  python tests/policies.py [oracle|gpu|gpu32] [env_id ...]   # prints the score table
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
POLICY_FILES = {
    "InvertedPendulumPyBulletEnv-v0": "policy_invertedpendulum.npz",
    "InvertedPendulumSwingupPyBulletEnv-v0": "policy_invertedpendulumswingup.npz",
    "InvertedDoublePendulumPyBulletEnv-v0": "policy_inverteddoublependulum.npz",
    "HopperPyBulletEnv-v0": "policy_hopper.npz",
    "Walker2DPyBulletEnv-v0": "policy_walker2d.npz",
    "HalfCheetahPyBulletEnv-v0": "policy_halfcheetah.npz",
    "AntPyBulletEnv-v0": "policy_ant.npz",
    "HumanoidPyBulletEnv-v0": "policy_humanoid.npz",
    "HumanoidFlagrunPyBulletEnv-v0": "policy_humanoidflagrun.npz",
    "HumanoidFlagrunHarderPyBulletEnv-v0": "policy_humanoidflagrunharder.npz",
    "AtlasPyBulletEnv-v0": "policy_atlas.npz",
}
MAX_STEPS = 1000  # TimeLimit (envs/__init__.py max_episode_steps)


class Policy:
    """relu(x W1 + b1) -> relu(. W2 + b2) -> . W3 + b3 (enjoy_TF_*.py:25-31), float32."""

    def __init__(self, env_id: str):
        z = np.load(os.path.join(GOLDEN, POLICY_FILES[env_id]))
        self.w = [z[f"weights_{k}"] for k in ("dense1_w", "dense1_b", "dense2_w", "dense2_b", "final_w", "final_b")]

    def act(self, obs: np.ndarray) -> np.ndarray:
        w1, b1, w2, b2, w3, b3 = self.w
        x = np.maximum(obs.astype(np.float32) @ w1 + b1, 0)
        x = np.maximum(x @ w2 + b2, 0)
        return (x @ w3 + b3).astype(np.float32)

    def torch_act(self, obs):
        import torch
        if not hasattr(self, "_tw"):
            self._tw = [torch.from_numpy(a).to(obs.device) for a in self.w]
        w1, b1, w2, b2, w3, b3 = self._tw
        x = torch.relu(obs @ w1 + b1)
        x = torch.relu(x @ w2 + b2)
        return x @ w3 + b3


def reset_draws(n: int, nr: int, seed: int) -> np.ndarray:
    return np.random.default_rng(seed).uniform(-0.1, 0.1, (n, nr))


def episode_returns_oracle(env_id: str, n: int, seed: int = 0, steps: int = MAX_STEPS, nthreads: int = 8,
                           precision: int = 64):
    """One episode per env (until done or `steps`) through the CPU oracle (precision 64: float64
    physics; 32: the same algorithm in IEEE float32, the kernels' formulation).
    Returns (returns[n] float64, lengths[n] int)."""
    import oracle
    pi = Policy(env_id)
    e = oracle.OracleEnvs(env_id, n, nthreads=nthreads, precision=precision)
    obs = e.reset(reset_draws(n, e.info.NR, seed))
    ret = np.zeros(n)
    length = np.zeros(n, dtype=np.int64)
    alive = np.ones(n, dtype=bool)
    for _ in range(steps):
        obs, r, d, _ = e.step(pi.act(obs))
        ret += np.where(alive, r, 0.0)
        length += alive
        alive &= ~d
        if not alive.any():
            break
    return ret, length


def episode_returns_device(env_id: str, n: int, seed: int = 0, steps: int = MAX_STEPS, precision: int = 64):
    """Same episodes through the HIP step kernel (libpbg_amd.so), reset draws passed in; precision
    64: the float64 handle (the reference's btScalar), 32: the float32 fast mode."""
    import torch
    from pybulletgym_amd.vec_env import VecEnv
    pi = Policy(env_id)
    env = VecEnv(env_id, n, device="cuda:0", seed=seed, autoreset=False, precision=precision)
    assert env.precision == precision
    obs = env.reset(init_q=torch.from_numpy(reset_draws(n, env.info.reset_dofs, seed).astype(np.float32)))
    ret = torch.zeros(n, dtype=torch.float64, device=env.device)
    length = torch.zeros(n, dtype=torch.int64, device=env.device)
    alive = torch.ones(n, dtype=torch.bool, device=env.device)
    for _ in range(steps):
        r = env.step(pi.torch_act(obs), want_reward64=True)
        ret += torch.where(alive, env.reward64, torch.zeros_like(env.reward64))
        length += alive
        alive &= r.done == 0
        obs = r.obs
    out = ret.cpu().numpy(), length.cpu().numpy()
    env.close()
    return out


def random_returns_oracle(env_id: str, n: int, seed: int = 0, steps: int = MAX_STEPS, nthreads: int = 8):
    """U(-1, 1) actions (gym's action_space.sample()) for comparison."""
    import oracle
    e = oracle.OracleEnvs(env_id, n, nthreads=nthreads)
    e.reset(reset_draws(n, e.info.NR, seed))
    rng = np.random.default_rng(seed + 1)
    ret = np.zeros(n)
    alive = np.ones(n, dtype=bool)
    for _ in range(steps):
        _, r, d, _ = e.step(rng.uniform(-1, 1, (n, e.info.NA)).astype(np.float32))
        ret += np.where(alive, r, 0.0)
        alive &= ~d
        if not alive.any():
            break
    return ret


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    mode = sys.argv[1] if len(sys.argv) > 1 else "oracle"
    ids = sys.argv[2:] or list(POLICY_FILES)
    for env_id in ids:
        n = 16
        if mode in ("gpu", "gpu32"):
            import pybulletgym_amd  # noqa: F401
            ret, ln = episode_returns_device(env_id, n, precision=32 if mode == "gpu32" else 64)
        else:
            ret, ln = episode_returns_oracle(env_id, n)
        rr = random_returns_oracle(env_id, n) if mode == "oracle" else np.zeros(1)
        print(f"{env_id:40s} policy return mean {ret.mean():9.1f} min {ret.min():9.1f} max {ret.max():9.1f}  "
              f"len mean {ln.mean():6.1f} min {ln.min():4d}   random mean {rr.mean():8.1f}", flush=True)
